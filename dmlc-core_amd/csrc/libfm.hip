// libfm.hip -- MI355X kernels for LibFMParser<I>::ParseBlock (libfm_parser.h:67-144);
// the tile body lives in libfm_core.h.  Exact count -> scan -> write only:
// libfm files are rare next to libsvm/CSV, and the exact path is the one
// every quirk of ParseTriple goes through.
#include "block.h"
#include "dmlc_amd_kernels.h"
#include "libfm_core.h"
#include "scan.h"

namespace dmlc_amd {
namespace {

template <int MODE>
__global__ void __launch_bounds__(kThreads) libfm_tile(LibfmArgs a) {
  __shared__ __attribute__((aligned(16))) svm::Shared sh;
  __shared__ uint64_t scratch[kBlockScratchU64];
  DevBlock bk{scratch};
  fm::tile<MODE>(a, sh, bk, blockIdx.x);
}

// fill phase after a count phase: reopen the first-error word (the count
// phase's finish turned "no error" into 0) and store the closing offset
__global__ void fm_reopen_kernel(uint64_t *res, uint64_t *offset, uint64_t cap_rows) {
  if (res[8] == 0) res[8] = ~0ull;
  if (offset && res[0] < cap_rows + 1) offset[res[0]] = res[1];
}

__global__ void fm_finish_kernel(uint64_t *res) {
  if (res[8] == ~0ull) res[8] = 0;
  res[9] = 1;  // dmlc_amd_result.path: the exact tile kernels
}

}  // namespace

hipError_t launch_libfm(const LibfmArgs &a, uint64_t *res, int phase, hipStream_t s) {
  hipError_t e;
  if (phase != kPhaseFill) {
    if ((e = hipMemsetAsync(res, 0, 16 * sizeof(uint64_t), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(res + 8, 0xFF, sizeof(uint64_t), s)) != hipSuccess) return e;
    if (a.indexing_mode < 0 &&
        (e = hipMemsetAsync(a.chunk_min, 0xFF, (size_t)a.nchunk * sizeof(uint64_t), s)) != hipSuccess)
      return e;
  } else {
    fm_reopen_kernel<<<1, 1, 0, s>>>(res, a.offset, a.cap[C_ROWS]);
  }
  if (phase != kPhaseCount && a.chunk_tab &&
      (e = hipMemsetAsync(a.chunk_tab, 0xFF, (size_t)a.nchunk * 8 * sizeof(uint64_t), s)) != hipSuccess)
    return e;  // rows no tile writes are filled by chunk_fixup_kernel
  if (!a.ntiles && phase != kPhaseCount && a.offset && (e = hipMemsetAsync(a.offset, 0, 8, s)) != hipSuccess)
    return e;  // empty input: offset = {0}
  if (a.ntiles) {
    if (phase != kPhaseFill) {
      libfm_tile<1><<<a.ntiles, kThreads, 0, s>>>(a);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], nullptr);
    }
    if (phase != kPhaseCount) {
      prof_mark(0, s, "libfm_tile<2>");
      libfm_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
      prof_mark(1, s, "libfm_tile<2>");
    }
  }
  fm_finish_kernel<<<1, 1, 0, s>>>(res);
  if (phase != kPhaseCount && a.chunk_tab && a.nchunk > 0) chunk_fixup_kernel<<<1, 1, 0, s>>>(a.chunk_tab, a.nchunk, res);
  return hipGetLastError();
}

}  // namespace dmlc_amd
