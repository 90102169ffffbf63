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
#define FEX_MINW 5  // waves per SIMD the exact tile kernels are register-budgeted for (round 4: 1 -> 4, libfm 1M x 64 exact 22.4 -> 19.7 ms; round 6, with the role masks and records: 4 / 5 / 6 -> 7.15 / 6.74 / 7.76 ms, profiles/r6_ab/ab_exact_minw.txt)
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


}  // namespace

hipError_t launch_libfm(const LibfmArgs &a, const FastSvmArgs &f, bool use_fast, uint64_t *res, int phase,
                        hipStream_t s) {
  hipError_t e;
  uint32_t *gate = f.gate;
  // ---- set-up, one launch (libsvm.hip launch_libsvm)
  FillList fl{};
  if (phase != kPhaseFill) {
    fill_result(fl, res);
    fl.gate = gate;
    fl.gate_v = use_fast ? 0u : 1u;
  }
  if (phase != kPhaseCount) fl.add(a.chunk_tab, (uint64_t)a.nchunk * 8, ~0ull);  // rows no tile writes: finish kernel
  fl.add(reinterpret_cast<uint64_t *>(f.err), 1, ~0ull);
  if (use_fast) {
    fl.add(f.lb, (uint64_t)f.ntiles * fast::kLbWords, 0);
    if (phase != kPhaseCount && f.indexing_mode < 0) fl.add(f.umin, (uint64_t)f.nchunk, ~0ull);
  }
  if (phase != kPhaseFill && a.indexing_mode < 0) fl.add(a.chunk_min, (uint64_t)a.nchunk, ~0ull);
  if (!a.ntiles && phase != kPhaseCount) fl.add(a.offset, 1, 0);  // empty input: offset = {0}
  if ((e = launch_prologue(fl, s)) != hipSuccess) return e;
  if (use_fast) {
    if (phase == kPhaseCount) {
      fm_fast_tile<1><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
    } else {
      prof_mark(0, s, "fm_fast_tile<2>");
      fm_fast_tile<2><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      prof_mark(1, s, "fm_fast_tile<2>");
    }
  }
  // ---- exact path, gated on the device flag (early exit when the fast path stood)
  if (phase == kPhaseFill) fm_reopen_kernel<<<1, 1, 0, s>>>(res, a.offset, a.cap[C_ROWS], gate);
  const bool reset_tab = use_fast && phase != kPhaseCount && a.chunk_tab && f.nchunk > 0;
  uint64_t *rtab = reset_tab ? a.chunk_tab : nullptr;
  const uint64_t ntab = reset_tab ? (uint64_t)f.nchunk * 8 : 0;
  if (a.ntiles) {
    if (phase != kPhaseFill) {
      libfm_tile<1><<<a.ntiles, kThreads, 0, s>>>(a);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], gate, rtab, ntab, gate);
      if (phase == kPhaseCount) note_gate_kernel<<<1, 1, 0, s>>>(gate);
    } else {
      // the count phase stood on the single-pass kernel but its write pass
      // handed over: count on the exact path first (scan.h recount_flag_kernel)
      recount_flag_kernel<<<1, 1, 0, s>>>(gate);
      auto ra = a;
      ra.gate = gate + 2;
      libfm_tile<1><<<a.ntiles, kThreads, 0, s>>>(ra);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], gate + 2, rtab, ntab, gate);
    }
    if (phase != kPhaseCount) {
      if (!use_fast) prof_mark(0, s, "libfm_tile<2>");
      libfm_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
      if (!use_fast) prof_mark(1, s, "libfm_tile<2>");
    }
  }
  finish_kernel<<<1, 256, 0, s>>>(res, gate, f.err, phase != kPhaseCount ? a.chunk_tab : nullptr, a.nchunk);
  if (use_fast && phase != kPhaseCount && f.indexing_mode < 0 &&
      (e = launch_umin_fix(f.index, f.field, f.wide, f.chunk_tab, f.nchunk, f.umin, res, gate, f.cap[C_INDEX], f.cap[C_FIELD], s)) !=
          hipSuccess)
    return e;
  return hipGetLastError();
}

}  // namespace dmlc_amd
