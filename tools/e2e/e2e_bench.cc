// e2e_bench.cc -- end-to-end rate of the drop-in API: file -> host InputSplit
// (8 MiB chunks, prefetch thread) -> pinned staging -> H2D -> MI355X parse ->
// D2H into pinned RowBlock storage -> the caller's Next()/Value() loop, i.e.
// what dmlc::Parser<uint32_t, float>::Create(uri, 0, 1, type) costs a caller.
//   e2e_bench <uri> <libsvm|csv> [passes] [epochs]
// Prints one JSON line: input bytes, wall seconds of the best pass, GB/s,
// rows and nnz seen (the checksum of a full iteration).  epochs > 0: then one
// Parser reads the input `epochs` times (BeforeFirst between, as a training
// loop does) and a second line gives the first and the best later epoch.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "dmlc/data.h"

int main(int argc, char **argv) {
  if (argc < 3) {
    std::fprintf(stderr, "usage: e2e_bench <uri> <libsvm|csv> [passes]\n");
    return 2;
  }
  const int passes = argc > 3 ? std::atoi(argv[3]) : 3;
  double best = 1e30, first = 0, best_create = 0, best_first_block = 0, best_delete = 0;
  size_t bytes = 0, rows = 0, nnz = 0, blocks = 0;
  using clk = std::chrono::steady_clock;
  auto sec = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double>(b - a).count(); };
  for (int pass = 0; pass < passes; ++pass) {
    const auto t0 = clk::now();
    dmlc::Parser<uint32_t, float> *p = dmlc::Parser<uint32_t, float>::Create(argv[1], 0, 1, argv[2]);
    const auto t1 = clk::now();
    clk::time_point tb = t1;
    rows = nnz = blocks = 0;
    while (p->Next()) {
      if (!blocks) tb = clk::now();
      const dmlc::RowBlock<uint32_t, float> &b = p->Value();
      rows += b.size;
      nnz += b.offset[b.size] - b.offset[0];
      ++blocks;
    }
    bytes = p->BytesRead();
    const auto t2 = clk::now();
    delete p;
    const auto t3 = clk::now();
    const double s = sec(t0, t3);
    if (pass == 0) first = s;
    if (s < best) {
      best = s;
      best_create = sec(t0, t1);
      best_first_block = sec(t1, tb);
      best_delete = sec(t2, t3);
    }
  }
  // create_s: Parser construction (threads, pinned batch buffers); first_block_s:
  // from there to the first RowBlock (the first batch's read, copy, parse and
  // copy-out); delete_s: teardown; GBps_stream: input bytes over the best
  // pass's time without construction and teardown
  std::printf("{\"uri\": \"%s\", \"type\": \"%s\", \"bytes\": %zu, \"rows\": %zu, \"nnz\": %zu, "
              "\"blocks\": %zu, \"best_s\": %.4f, \"first_s\": %.4f, \"GBps\": %.3f, \"create_s\": %.4f, "
              "\"first_block_s\": %.4f, \"delete_s\": %.4f, \"GBps_stream\": %.3f}\n",
              argv[1], argv[2], bytes, rows, nnz, blocks, best, first, bytes / best / 1e9, best_create,
              best_first_block, best_delete, bytes / (best - best_create - best_delete) / 1e9);
  const int epochs = argc > 4 ? std::atoi(argv[4]) : 0;
  if (epochs > 0) {
    dmlc::Parser<uint32_t, float> *p = dmlc::Parser<uint32_t, float>::Create(argv[1], 0, 1, argv[2]);
    double e_first = 0, e_best = 1e30;
    size_t erows = 0;
    for (int e = 0; e < epochs; ++e) {
      const auto t0 = clk::now();
      if (e) p->BeforeFirst();
      erows = 0;
      while (p->Next()) erows += p->Value().size;
      const double s = sec(t0, clk::now());
      if (e == 0) e_first = s;
      else if (s < e_best) e_best = s;
    }
    delete p;
    std::printf("{\"uri\": \"%s\", \"type\": \"%s\", \"mode\": \"epochs\", \"epochs\": %d, \"bytes\": %zu, "
                "\"rows\": %zu, \"first_epoch_s\": %.4f, \"best_later_epoch_s\": %.4f, \"GBps_first_epoch\": %.3f, "
                "\"GBps_later_epochs\": %.3f}\n",
                argv[1], argv[2], epochs, bytes, erows, e_first, e_best, bytes / e_first / 1e9,
                epochs > 1 ? bytes / e_best / 1e9 : 0.0);
  }
  return 0;
}
