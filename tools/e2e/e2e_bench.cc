// e2e_bench.cc -- end-to-end rate of the drop-in API: file -> host InputSplit
// (8 MiB chunks, prefetch thread) -> pinned staging -> H2D -> MI355X parse ->
// D2H into pinned RowBlock storage -> the caller's Next()/Value() loop, i.e.
// what dmlc::Parser<uint32_t, float>::Create(uri, 0, 1, type) costs a caller.
//   e2e_bench <uri> <libsvm|csv> [passes]
// Prints one JSON line: input bytes, wall seconds of the best pass, GB/s,
// rows and nnz seen (the checksum of a full iteration).
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
  double best = 1e30, first = 0;
  size_t bytes = 0, rows = 0, nnz = 0, blocks = 0;
  for (int pass = 0; pass < passes; ++pass) {
    const auto t0 = std::chrono::steady_clock::now();
    dmlc::Parser<uint32_t, float> *p = dmlc::Parser<uint32_t, float>::Create(argv[1], 0, 1, argv[2]);
    rows = nnz = blocks = 0;
    while (p->Next()) {
      const dmlc::RowBlock<uint32_t, float> &b = p->Value();
      rows += b.size;
      nnz += b.offset[b.size] - b.offset[0];
      ++blocks;
    }
    bytes = p->BytesRead();
    delete p;
    const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    if (pass == 0) first = s;
    if (s < best) best = s;
  }
  std::printf("{\"uri\": \"%s\", \"type\": \"%s\", \"bytes\": %zu, \"rows\": %zu, \"nnz\": %zu, "
              "\"blocks\": %zu, \"best_s\": %.4f, \"first_s\": %.4f, \"GBps\": %.3f}\n",
              argv[1], argv[2], bytes, rows, nnz, blocks, best, first, bytes / best / 1e9);
  return 0;
}
