// libsvm.hip -- MI355X kernels for LibSVMParser::ParseBlock (libsvm_parser.h:85-172);
// the tile body lives in libsvm_core.h.
#include "block.h"
#include "dmlc_amd_kernels.h"
#include "libsvm_core.h"
#include "scan.h"

namespace dmlc_amd {
namespace {

template <int MODE>
__global__ void __launch_bounds__(kThreads) libsvm_tile(LibsvmArgs a) {
  __shared__ __attribute__((aligned(16))) svm::Shared sh;
  __shared__ uint64_t scratch[kBlockScratchU64];
  DevBlock bk{scratch};
  svm::tile<MODE>(a, sh, bk, blockIdx.x);
}

__global__ void finalize_kernel(uint64_t *res) {
  if (res[8] == ~0ull) res[8] = 0;  // no error raised
}

}  // namespace

hipError_t launch_libsvm(const LibsvmArgs &a, uint64_t *res, bool count_only, hipStream_t s) {
  hipError_t e;
  if ((e = hipMemsetAsync(res, 0, 16 * sizeof(uint64_t), s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(res + 8, 0xFF, sizeof(uint64_t), s)) != hipSuccess) return e;
  if (a.indexing_mode < 0 &&
      (e = hipMemsetAsync(a.chunk_min, 0xFF, (size_t)a.nchunk * sizeof(uint64_t), s)) != hipSuccess)
    return e;
  if (!a.ntiles && !count_only && a.offset && (e = hipMemsetAsync(a.offset, 0, 8, s)) != hipSuccess)
    return e;  // empty input: offset = {0}
  if (a.ntiles) {
    libsvm_tile<1><<<a.ntiles, kThreads, 0, s>>>(a);
    tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                            res, count_only ? nullptr : a.offset, a.cap[C_ROWS]);
    if (!count_only) libsvm_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
  }
  finalize_kernel<<<1, 1, 0, s>>>(res);
  return hipGetLastError();
}

}  // namespace dmlc_amd
