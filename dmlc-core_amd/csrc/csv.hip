// csv.hip -- MI355X kernels for CSVParser<I,D>::ParseBlock (csv_parser.h:71-149);
// the tile body lives in csv_core.h.
#include "block.h"
#include "csv_core.h"
#include "dmlc_amd_kernels.h"
#include "scan.h"

namespace dmlc_amd {
namespace {

template <int MODE>
__global__ void __launch_bounds__(kThreads) csv_tile(CsvArgs a) {
  __shared__ __attribute__((aligned(16))) csv::Shared sh;
  __shared__ uint64_t scratch[kBlockScratchU64];
  DevBlock bk{scratch};
  csv::tile<MODE>(a, sh, bk, blockIdx.x);
}

// fill phase after a count phase: the count phase's finalize turned "no error"
// (~0) into 0; reopen it so the write pass can record the first error, and
// store the closing offset (the reference's final push, libsvm_parser.h:157-159)
// the size query could not (it had no output buffers)
__global__ void reopen_kernel(uint64_t *res, uint64_t *offset, uint64_t cap_rows) {
  if (res[8] == 0) res[8] = ~0ull;
  if (offset && res[0] < cap_rows + 1) offset[res[0]] = res[1];
}

__global__ void finalize_kernel(uint64_t *res) {
  if (res[8] == ~0ull) res[8] = 0;
  res[9] = 1;  // dmlc_amd_result.path: exact tile kernels
}

}  // namespace

hipError_t launch_csv(const CsvArgs &a, uint64_t *res, int phase, hipStream_t s) {
  hipError_t e;
  if (phase != kPhaseFill) {
    if ((e = hipMemsetAsync(res, 0, 16 * sizeof(uint64_t), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(res + 8, 0xFF, sizeof(uint64_t), s)) != hipSuccess) return e;
  } else {
    reopen_kernel<<<1, 1, 0, s>>>(res, a.offset, a.cap[C_ROWS]);
  }
  if (!a.ntiles && phase != kPhaseCount && a.offset && (e = hipMemsetAsync(a.offset, 0, 8, s)) != hipSuccess)
    return e;  // empty input: offset = {0}
  if (a.ntiles) {
    if (phase != kPhaseFill) {
      csv_tile<1><<<a.ntiles, kThreads, 0, s>>>(a);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], nullptr);
    }
    if (phase != kPhaseCount) {
      prof_mark(0, s, "csv_tile<2>");
      csv_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
      prof_mark(1, s, "csv_tile<2>");
    }
  }
  finalize_kernel<<<1, 1, 0, s>>>(res);
  return hipGetLastError();
}

}  // namespace dmlc_amd
