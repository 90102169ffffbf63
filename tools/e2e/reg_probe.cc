// Registered page-cache probe: can the
// text go from the page cache to HBM by DMA without the pinned copy?  A file
// of S bytes in the page cache is mmap'd; per chunk of C bytes the probe times
//   reg:   hipHostRegister of the mapped range (pins its page-cache pages)
//   copy:  hipMemcpyAsync of the range to HBM (DMA reads the page cache)
//   unreg: hipHostUnregister
// against the engine's path today: pread into a pinned block + DMA of it.
// Prints one JSON line per chunk size.  usage: reg_probe <file> [MiB ...]
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e_ = (x);                                                   \
    if (e_ != hipSuccess) {                                                \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));         \
      std::exit(1);                                                        \
    }                                                                      \
  } while (0)

int main(int argc, char **argv) {
  if (argc < 2) return 2;
  const int fd = open(argv[1], O_RDONLY);
  struct stat st;
  if (fd < 0 || fstat(fd, &st) != 0) return 3;
  const size_t S = (size_t)st.st_size & ~(size_t)4095;
  char *m = (char *)mmap(nullptr, S, PROT_READ, MAP_SHARED, fd, 0);
  if (m == MAP_FAILED) return 4;
  volatile uint64_t sink = 0;
  for (size_t i = 0; i < S; i += 4096) sink += (unsigned char)m[i];  // resident
  std::vector<size_t> sizes;
  for (int i = 2; i < argc; ++i) sizes.push_back((size_t)std::atol(argv[i]) << 20);
  if (sizes.empty()) sizes = {32u << 20, 256u << 20, 2048u << 20};
  void *d = nullptr;
  CK(hipMalloc(&d, S));
  hipStream_t s;
  CK(hipStreamCreate(&s));
  for (size_t C : sizes) {
    if (C > S) C = S;
    double treg = 0, tcopy = 0, tun = 0;
    for (size_t off = 0; off + C <= S; off += C) {
      double t0 = now();
      CK(hipHostRegister(m + off, C, hipHostRegisterDefault | hipHostRegisterReadOnly));
      double t1 = now();
      CK(hipMemcpyAsync((char *)d + off, m + off, C, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      double t2 = now();
      CK(hipHostUnregister(m + off));
      double t3 = now();
      treg += t1 - t0;
      tcopy += t2 - t1;
      tun += t3 - t2;
    }
    const size_t moved = (S / C) * C;
    // today's path: pread into a pinned block, then DMA it
    void *pin = nullptr;
    CK(hipHostMalloc(&pin, C, hipHostMallocDefault));
    double tread = 0, tdma = 0;
    for (size_t off = 0; off + C <= S; off += C) {
      double t0 = now();
      size_t got = 0;
      while (got < C) {
        ssize_t r = pread(fd, (char *)pin + got, C - got, (off_t)(off + got));
        if (r <= 0) return 5;
        got += (size_t)r;
      }
      double t1 = now();
      CK(hipMemcpyAsync((char *)d + off, pin, C, hipMemcpyHostToDevice, s));
      CK(hipStreamSynchronize(s));
      tdma += now() - t1;
      tread += t1 - t0;
    }
    CK(hipHostFree(pin));
    const double g = moved / 1e9;
    std::printf("{\"chunk_mib\": %zu, \"bytes\": %zu, \"register_GBps\": %.2f, \"copy_from_registered_GBps\": %.2f, "
                "\"unregister_GBps\": %.2f, \"registered_path_GBps\": %.2f, \"pread_pinned_GBps\": %.2f, "
                "\"dma_from_pinned_GBps\": %.2f, \"pinned_path_GBps\": %.2f}\n",
                C >> 20, moved, g / treg, g / tcopy, g / tun, g / (treg + tcopy + tun), g / tread, g / tdma,
                g / (tread + tdma));
    std::fflush(stdout);
  }
  (void)sink;
  return 0;
}
