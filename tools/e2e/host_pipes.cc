// host_pipes.cc -- the host side of P concurrent parse pipelines, no GPU
// (the host-DRAM budget of 8 GPUs' pipelines).
//
// Each pipeline is one process, as on an 8-GPU node (one rank per GPU).  It
// reads part k of P of the input with the product's TextSplit (8 MiB
// InputSplit chunks into a batch buffer, its pool of pread threads), and a
// second thread stands in for the link: per filled batch it streams the
// batch once (what the H2D copy reads from host memory) and writes
// csr_ratio x the batch's bytes into an output buffer (what the D2H copy of
// the CSR writes).  Two batch buffers, as the engine double-buffers.
//   host_pipes <uri> <P> [passes=3] [batch_mib=32] [csr_ratio=0.55] [link_threads=4]
// HOST_PIPES_MAPPED=1: the engine's mapped form (round 6, TextSplit::FillPieces):
// no reader copy -- the link threads stream the batch's pieces straight from
// the page cache (what the DMA reads from the registered mappings).
// Prints one JSON line: total input bytes over all P pipelines, wall seconds
// (first start to last end), aggregate GB/s of input, and the host-DRAM
// bytes per input byte this model moves.
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "text_split.h"

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

struct Slot {
  std::vector<char> buf;
  std::vector<dmlc_amd::TextPiece> pieces;  // mapped form
  size_t bytes = 0;
  bool full = false, end = false;
};

// one pipeline: returns input bytes moved
uint64_t run_pipe(const std::string &uri, unsigned part, unsigned nparts, int passes, size_t batch,
                  double csr_ratio, int link_threads, bool mapped) {
  Slot slot[2];
  for (auto &s : slot) {
    s.buf.resize(batch + (16u << 20));
    std::memset(s.buf.data(), 0, s.buf.size());  // resident before timing, as pinned memory is
  }
  std::vector<char> out((size_t)(batch * csr_ratio) + 4096);
  std::memset(out.data(), 0, out.size());
  std::mutex mu;
  std::condition_variable cv;
  std::atomic<uint64_t> total{0};
  volatile uint64_t sink = 0;
  std::thread link([&] {
    for (int k = 0;; k ^= 1) {
      Slot &s = slot[k];
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return s.full; });
      }
      // the H2D copy's host reads (stream the batch once) and the D2H copy's
      // host writes (the CSR arrays), split over link_threads threads: the
      // DMA engines / copy kernels move them at link rate, far above what
      // one core streams
      const size_t ob = std::min(out.size(), (size_t)(s.bytes * csr_ratio));
      std::vector<std::thread> lt;
      std::atomic<uint64_t> accs{0};
      for (int t = 0; t < link_threads; ++t)
        lt.emplace_back([&, t] {
          uint64_t acc = 0;
          auto stream = [&](const char *base, size_t bytes) {
            const size_t words = bytes / 64 * 8;  // whole 64 B lines
            const size_t lo = words * t / link_threads / 8 * 8, hi = words * (t + 1) / link_threads / 8 * 8;
            uint64_t w0, w4;
            for (size_t i = lo; i < hi; i += 8) {  // two words per 64 B line (unaligned in a mapping)
              std::memcpy(&w0, base + i * 8, 8);
              std::memcpy(&w4, base + i * 8 + 32, 8);
              acc += w0 ^ w4;
            }
          };
          if (mapped) {
            for (const dmlc_amd::TextPiece &pc : s.pieces)
              if (pc.src) stream(pc.src, pc.len);
          } else {
            stream(s.buf.data(), s.bytes);
          }
          accs += acc;
          const size_t olo = ob * t / link_threads, ohi = ob * (t + 1) / link_threads;
          std::memset(out.data() + olo, (int)(acc & 0x7f), ohi - olo);
        });
      for (auto &th : lt) th.join();
      sink = sink + accs.load();
      total += s.bytes;
      const bool end = s.end;
      {
        std::lock_guard<std::mutex> lk(mu);
        s.full = false;
      }
      cv.notify_all();
      if (end) return;
    }
  });
  dmlc_amd::TextSplit split(uri, part, nparts);
  if (mapped && !split.Mapped()) {
    std::fprintf(stderr, "the split did not map its files\n");
    std::exit(1);
  }
  std::vector<uint64_t> ends;
  int k = 0;
  for (int pass = 0; pass < passes; ++pass) {
    if (pass) split.BeforeFirst();
    for (;;) {
      Slot &s = slot[k];
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return !s.full; });
      }
      ends.clear();
      const dmlc_amd::TextSplit::Fill f = mapped ? split.FillPieces(batch, &ends, &s.pieces)
                                                 : split.FillChunks(s.buf.data(), s.buf.size(), batch, &ends);
      if (f.need) {
        std::fprintf(stderr, "record longer than the batch buffer\n");
        std::exit(1);
      }
      s.bytes = ends.empty() ? 0 : ends.back();
      s.end = f.end && pass + 1 == passes;
      {
        std::lock_guard<std::mutex> lk(mu);
        s.full = true;
      }
      cv.notify_all();
      k ^= 1;
      if (f.end) break;
    }
  }
  link.join();
  return total.load();
}
}  // namespace

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: host_pipes <uri> <P> [passes] [batch_mib] [csr_ratio]\n");
    return 2;
  }
  const std::string uri = argv[1];
  const unsigned P = (unsigned)std::atoi(argv[2]);
  const int passes = argc > 3 ? std::atoi(argv[3]) : 3;
  const size_t batch = (size_t)(argc > 4 ? std::atoi(argv[4]) : 32) << 20;
  const double ratio = argc > 5 ? std::atof(argv[5]) : 0.55;
  const int link_threads = argc > 6 ? std::atoi(argv[6]) : 4;
  const char *mm = std::getenv("HOST_PIPES_MAPPED");
  const bool mapped = mm && mm[0] == '1';
  int fds[64][2];
  if (P < 1 || P > 64) return 2;
  const double t0 = now_s();
  std::vector<pid_t> kids;
  for (unsigned r = 0; r < P; ++r) {
    if (pipe(fds[r]) != 0) return 1;
    const pid_t pid = fork();
    if (pid == 0) {
      close(fds[r][0]);
      const uint64_t b = run_pipe(uri, r, P, passes, batch, ratio, link_threads, mapped);
      const double t1 = now_s();
      char msg[64];
      const int n = std::snprintf(msg, sizeof(msg), "%llu %.6f", (unsigned long long)b, t1);
      if (write(fds[r][1], msg, (size_t)n) != n) _exit(1);
      _exit(0);
    }
    close(fds[r][1]);
    kids.push_back(pid);
  }
  uint64_t bytes = 0;
  double last = t0;
  int bad = 0;
  for (unsigned r = 0; r < P; ++r) {
    char msg[64] = {0};
    const ssize_t n = read(fds[r][0], msg, sizeof(msg) - 1);
    int st = 0;
    waitpid(kids[r], &st, 0);
    if (n <= 0 || !WIFEXITED(st) || WEXITSTATUS(st)) {
      ++bad;
      continue;
    }
    unsigned long long b = 0;
    double t1 = 0;
    std::sscanf(msg, "%llu %lf", &b, &t1);
    bytes += b;
    last = t1 > last ? t1 : last;
  }
  const double s = last - t0;
  // host DRAM bytes per input byte in this model: page cache read + batch
  // write (the reader), the H2D copy's read, the CSR write; mapped: the
  // H2D read from the page cache and the CSR write
  const double dram = (mapped ? 1.0 : 3.0) + ratio;
  std::printf("{\"case\": \"host_pipes\", \"pipelines\": %u, \"read_threads_each\": \"%s\", \"passes\": %d, "
              "\"batch_mib\": %zu, \"csr_ratio\": %.2f, \"link_threads\": %d, \"input_bytes\": %llu, \"s\": %.4f, \"GBps_in\": %.2f, "
              "\"dram_bytes_per_input_byte\": %.2f, \"GBps_dram\": %.1f, \"mapped\": %d, \"failed\": %d}\n",
              P, std::getenv("DMLC_AMD_READ_THREADS") ? std::getenv("DMLC_AMD_READ_THREADS") : "8", passes,
              batch >> 20, ratio, link_threads, (unsigned long long)bytes, s, bytes / s / 1e9, dram, bytes * dram / s / 1e9,
              mapped ? 1 : 0, bad);
  return bad ? 1 : 0;
}
