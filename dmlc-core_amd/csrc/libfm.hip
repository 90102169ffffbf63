// libfm.hip -- MI355X kernels for LibFMParser<I>::ParseBlock (libfm_parser.h:67-144).
//   fm_fast_tile  single-pass uniform-grammar kernel (svm_fast.h with the
//                 libfm roles): the normal path; sets the gate word when the
//                 input leaves the grammar
//   libfm_tile    exact count / write tile kernels (libfm_core.h), run only
//                 when the gate is set (or indexing_mode < 0)
#include "block.h"
#include "dmlc_amd_kernels.h"
#include "libfm_core.h"
#include "scan.h"
#include "svm_fast.h"

namespace dmlc_amd {
namespace {

template <int MODE>
#ifndef FEX_MINW
#define FEX_MINW 4  // waves per SIMD the exact tile kernels are register-budgeted for (round 4: 1 -> 4, libfm 1M x 64 exact 22.4 -> 19.7 ms)
#endif
__global__ void __launch_bounds__(kThreads, FEX_MINW) libfm_tile(LibfmArgs a) {
  __shared__ __attribute__((aligned(16))) svm::Shared sh;
  __shared__ uint64_t scratch[kBlockScratchU64];
  DevBlock bk{scratch};
  fm::tile<MODE>(a, sh, bk, blockIdx.x);
}

static_assert(sizeof(fsvm::Shared) + kSmallScratchU64 * 8 <= fast::kLdsBudget,
              "fm_fast_tile LDS above the 6-workgroup budget (fast_common.h kLdsBudget)");

#ifndef FFM_MINW
#define FFM_MINW (fast::kFWaves == 1 ? 5 : 6)
#endif
template <int MODE>
__global__ void __launch_bounds__(fast::kFThreads, FFM_MINW) fm_fast_tile(FastSvmArgs a) {
  __shared__ __attribute__((aligned(16))) fsvm::Shared sh;
  __shared__ uint64_t scratch[kSmallScratchU64];
  DevBlockS bk{scratch};
  fsvm::tile<MODE, true>(a, sh, bk, blockIdx.x);
}

// fill phase after a count phase that fell back to the exact kernels: reopen
// the first-error word and store the closing offset the size query could not
__global__ void fm_reopen_kernel(uint64_t *res, uint64_t *offset, uint64_t cap_rows, const uint32_t *gate) {
  if (*gate == 0) return;
  if (res[8] == 0) res[8] = ~0ull;
  if (offset && res[0] < cap_rows + 1) offset[res[0]] = res[1];
}

// the error of whichever path produced the result
__global__ void fm_select_kernel(uint64_t *res, const uint32_t *gate, const unsigned long long *ferr) {
  if (*gate == 0) res[8] = *ferr;
  if (res[8] == ~0ull) res[8] = 0;
  res[9] = *gate;  // dmlc_amd_result.path
}

}  // namespace

hipError_t launch_libfm(const LibfmArgs &a, const FastSvmArgs &f, bool use_fast, uint64_t *res, int phase,
                        hipStream_t s) {
  hipError_t e;
  uint32_t *gate = f.gate;
  if (phase != kPhaseFill) {
    if ((e = hipMemsetAsync(res, 0, 16 * sizeof(uint64_t), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(res + 8, 0xFF, sizeof(uint64_t), s)) != hipSuccess) return e;
    if ((e = hipMemsetD32Async(reinterpret_cast<hipDeviceptr_t>(gate), use_fast ? 0 : 1, 1, s)) !=
        hipSuccess)
      return e;
  }
  if (phase != kPhaseCount && a.chunk_tab &&
      (e = hipMemsetAsync(a.chunk_tab, 0xFF, (size_t)a.nchunk * 8 * sizeof(uint64_t), s)) != hipSuccess)
    return e;  // rows no tile writes are filled by chunk_fixup_kernel
  if (use_fast) {
    if ((e = hipMemsetAsync(f.err, 0xFF, sizeof(uint64_t), s)) != hipSuccess) return e;
    if ((e = hipMemsetAsync(f.lb, 0, (size_t)f.ntiles * fast::kLbWords * sizeof(uint64_t), s)) != hipSuccess) return e;
    if (phase == kPhaseCount) {
      fm_fast_tile<1><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
    } else {
      if (f.indexing_mode < 0 &&
          (e = hipMemsetAsync(f.umin, 0xFF, (size_t)f.nchunk * sizeof(uint64_t), s)) != hipSuccess)
        return e;
      prof_mark(0, s, "fm_fast_tile<2>");
      fm_fast_tile<2><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      prof_mark(1, s, "fm_fast_tile<2>");
    }
  } else if ((e = hipMemsetAsync(f.err, 0xFF, sizeof(uint64_t), s)) != hipSuccess) {
    return e;
  }
  // ---- exact path, gated on the device flag (early exit when the fast path stood)
  if (phase != kPhaseFill) {
    if (a.indexing_mode < 0 &&
        (e = hipMemsetAsync(a.chunk_min, 0xFF, (size_t)a.nchunk * sizeof(uint64_t), s)) != hipSuccess)
      return e;
  } else {
    fm_reopen_kernel<<<1, 1, 0, s>>>(res, a.offset, a.cap[C_ROWS], gate);
  }
  if (!a.ntiles && phase != kPhaseCount && a.offset && (e = hipMemsetAsync(a.offset, 0, 8, s)) != hipSuccess)
    return e;  // empty input: offset = {0}
  if (a.ntiles) {
    if (phase != kPhaseFill) {
      libfm_tile<1><<<a.ntiles, kThreads, 0, s>>>(a);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], gate);
      if (phase == kPhaseCount) note_gate_kernel<<<1, 1, 0, s>>>(gate);
    } else {
      // the count phase stood on the single-pass kernel but its write pass
      // handed over: count on the exact path first (scan.h recount_flag_kernel)
      recount_flag_kernel<<<1, 1, 0, s>>>(gate);
      auto ra = a;
      ra.gate = gate + 2;
      libfm_tile<1><<<a.ntiles, kThreads, 0, s>>>(ra);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], gate + 2);
    }
    if (phase != kPhaseCount) {
      if (use_fast && a.chunk_tab && f.nchunk > 0)
        tab_reset_kernel<<<(f.nchunk * 8 + 255) / 256, 256, 0, s>>>(a.chunk_tab, (uint64_t)f.nchunk * 8, gate);
      if (!use_fast) prof_mark(0, s, "libfm_tile<2>");
      libfm_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
      if (!use_fast) prof_mark(1, s, "libfm_tile<2>");
    }
  }
  fm_select_kernel<<<1, 1, 0, s>>>(res, gate, f.err);
  if (phase != kPhaseCount && a.chunk_tab && a.nchunk > 0) chunk_fixup_kernel<<<1, 256, 0, s>>>(a.chunk_tab, a.nchunk, res);
  if (use_fast && phase != kPhaseCount && f.indexing_mode < 0 &&
      (e = launch_umin_fix(f.index, f.field, f.wide, f.chunk_tab, f.nchunk, f.umin, res, gate, f.cap[C_INDEX], f.cap[C_FIELD], s)) !=
          hipSuccess)
    return e;
  return hipGetLastError();
}

}  // namespace dmlc_amd
