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

__global__ void finalize_kernel(uint64_t *res) {
  if (res[8] == ~0ull) res[8] = 0;
}

}  // namespace

hipError_t launch_csv(const CsvArgs &a, uint64_t *res, bool count_only, hipStream_t s) {
  hipError_t e;
  if ((e = hipMemsetAsync(res, 0, 16 * sizeof(uint64_t), s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(res + 8, 0xFF, sizeof(uint64_t), s)) != hipSuccess) return e;
  if (!a.ntiles && !count_only && a.offset && (e = hipMemsetAsync(a.offset, 0, 8, s)) != hipSuccess)
    return e;  // empty input: offset = {0}
  if (a.ntiles) {
    csv_tile<1><<<a.ntiles, kThreads, 0, s>>>(a);
    tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                            res, count_only ? nullptr : a.offset, a.cap[C_ROWS]);
    if (!count_only) csv_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
  }
  finalize_kernel<<<1, 1, 0, s>>>(res);
  return hipGetLastError();
}

}  // namespace dmlc_amd
