// libsvm.hip -- MI355X kernels for LibSVMParser::ParseBlock (libsvm_parser.h:85-172).
//
//   svm_fast_tile   single-pass uniform-grammar kernel (svm_fast.h): the
//                   normal path; sets the gate word when the input leaves
//                   the grammar
//   libsvm_tile     exact count / write tile kernels (libsvm_core.h), run
//                   only when the gate is set (or indexing_mode < 0)
#include <atomic>

#include "block.h"
#include "dmlc_amd_kernels.h"
#include "libsvm_core.h"
#include "scan.h"
#include "svm_fast.h"
#include "svm_lean.h"

namespace dmlc_amd {
namespace {

template <int MODE>
#ifndef FEX_MINW
#define FEX_MINW 5  // waves per SIMD the exact tile kernels are register-budgeted for (round 4: 1 -> 4 -> 5, config 2 exact 13.2 -> 11.9 -> 10.9 ms)
#endif
#ifndef FEX_MINW1
#define FEX_MINW1 FEX_MINW  // the count pass's own budget
#endif
__global__ void __launch_bounds__(kThreads, MODE == 1 ? FEX_MINW1 : FEX_MINW) libsvm_tile(LibsvmArgs a) {
  __shared__ __attribute__((aligned(16))) svm::Shared sh;
  __shared__ uint64_t scratch[kBlockScratchU64];
  DevBlock bk{scratch};
  if (MODE == 1 && a.qsum && *a.gate == 0) {  // block-uniform
    // the single pass stood; its qid runs stand only when every row has one
    // (svm_fast.h qid_decide): a mix of rows with and without a qid hands the
    // input over here, a clean qid input is finished by finish_kernel
    if (a.qsum[1] == 0) return;  // no tile held a qid run
    __shared__ int mix;
    if (threadIdx.x < kWave) {
      uint64_t t = a.qsum[threadIdx.x * 8];
      for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d, kWave);
      if (threadIdx.x == 0) mix = t != a.qres[C_ROWS];
    }
    __syncthreads();
    if (!mix) return;
    if (threadIdx.x == 0) atomic_or_u32(const_cast<uint32_t *>(a.gate), 1u);
    a.gate = nullptr;
  }
  svm::tile<MODE>(a, sh, bk, blockIdx.x);
}

static_assert(sizeof(fsvm::Shared) + kSmallScratchU64 * 8 <= fast::kLdsBudget,
              "svm_fast_tile LDS above the 6-workgroup budget (fast_common.h kLdsBudget)");

template <int MODE>
#ifndef FSVM_MINW
#define FSVM_MINW (fast::kFWaves == 1 ? 5 : 6)  // waves per SIMD the fill kernel is register-budgeted for
#endif
#ifndef FSVM_PERSIST
#define FSVM_PERSIST 0  // workgroups loop over tiles (svm_fast.h tile_p)
#endif
__global__ void __launch_bounds__(fast::kFThreads, FSVM_MINW) svm_fast_tile(FastSvmArgs a) {
  __shared__ __attribute__((aligned(16))) fsvm::Shared sh;
  __shared__ uint64_t scratch[kSmallScratchU64];
#ifdef FSVM_ABL_PAD_LDS  // occupancy experiment only: pad the workgroup's LDS
  __shared__ uint32_t pad[FSVM_ABL_PAD_LDS / 4];
  if (a.n == 1) pad[threadIdx.x] = 1, a.res[15] = pad[(threadIdx.x + 1) % fast::kFThreads];
#endif
  DevBlockS bk{scratch};
#if FSVM_PERSIST
  // persistent: the first tile is the workgroup's index (dispatch order makes
  // every lower one resident first), later ones come from the ticket
  if (a.skip_if_gated && *a.gate) return;  // fill phase after an exact-path count: block-uniform
  fsvm::init_tables(sh, bk);
  fast::StageRegs sr;
  uint32_t k = blockIdx.x;
  fast::stage_issue(a.text, a.n, (uint64_t)k * fast::kTile, sr, bk);
  while (k < a.ntiles) {
    k = fsvm::tile_p<MODE, false, true>(a, sh, bk, k, sr);
    bk.sync();  // every thread is done with the tile's LDS
  }
#else
  fsvm::tile<MODE>(a, sh, bk, blockIdx.x);
#endif
}

// The lean single-pass kernel (svm_lean.h), ahead of svm_fast_tile<2> in a
// full call: budgeted for 8 workgroups per CU (64 VGPRs).
#ifndef LSVM_MINW
#define LSVM_MINW 6
#endif
static_assert(sizeof(lsvm::Shared) <= 160 * 1024 / LSVM_MINW, "svm_lean_tile LDS above its occupancy budget");
__global__ void __launch_bounds__(fast::kFThreads, LSVM_MINW) svm_lean_tile(FastSvmArgs a) {
  __shared__ __attribute__((aligned(16))) lsvm::Shared sh;
  DevBlockS bk{nullptr};
  lsvm::tile(a, sh, bk, blockIdx.x);
}
// DMLC_AMD_LEAN=0 / 1 turns the lean kernel off / on (A/B timing; off, the
// full kernel takes every tile, as before round 6); LSVM_DEFAULT the default
#ifndef LSVM_DEFAULT
#define LSVM_DEFAULT 0
#endif
bool lean_enabled() {
  static const int on = [] {
    const char *e = getenv("DMLC_AMD_LEAN");
    return e && e[0] ? (e[0] == '0' ? 0 : 1) : LSVM_DEFAULT;
  }();
  return on != 0;
}

// workgroups of a persistent single-pass launch: what the device holds at
// once (the occupancy calculator, capped at the 6 per CU the LDS budget
// allows), never more than the tiles.  The per-device answer is cached in
// atomics: the engine's workers launch from several host threads.  (The
// persistent form -- FSVM_PERSIST, off by default -- takes later tiles from a
// ticket, so it never deadlocks; when other streams' kernels share the device
// and part of the grid is not resident, the look-back's kSpinLimit valve is
// what bounds a wait on a tile that is not yet running.)
template <class K>
uint32_t persistent_grid(K kernel, uint32_t ntiles) {
  static std::atomic<int> cache_n[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return ntiles;
  int n = cache_n[dev].load(std::memory_order_relaxed);
  if (n == 0) {
    int cus = 0, per = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        hipOccupancyMaxActiveBlocksPerMultiprocessor(&per, kernel, fast::kFThreads, 0) != hipSuccess || cus < 1 || per < 1)
      return ntiles;
    const int cap = 6 * kWaves / fast::kFWaves;
    n = cus * (per < cap ? per : cap);
    cache_n[dev].store(n, std::memory_order_relaxed);
  }
  return (uint32_t)n < ntiles ? (uint32_t)n : ntiles;
}

// fill phase after a count phase that fell back to the exact kernels: the
// count phase's select turned "no error" (~0) into 0; reopen it so the write
// pass can record the first error, and store the closing offset (the
// reference's final push, libsvm_parser.h:157-159) the size query could not
__global__ void reopen_kernel(uint64_t *res, uint64_t *offset, uint64_t cap_rows, const uint32_t *gate) {
  if (*gate == 0) return;
  if (res[8] == 0) res[8] = ~0ull;
  if (offset && res[0] < cap_rows + 1) offset[res[0]] = res[1];
}

// after the single-pass kernel: the tiles' qid run counts against the rows
// (svm_fast.h qid_decide); when every row has a qid, each chunk row's qid
// count is its row count
__global__ void __launch_bounds__(256) qid_fix_kernel(const uint64_t *qsum, uint64_t *res, uint32_t *gate,
                                                      uint64_t *chunk_tab, int nchunk) {
  __shared__ int fix_tab;
  if (threadIdx.x == 0) {
    uint64_t total = 0;
    for (int i = 0; i < kLabShards; ++i) total += qsum[i * 8];
    fix_tab = fsvm::qid_decide(total, res, gate) && chunk_tab;
  }
  __syncthreads();
  if (fix_tab)
    for (int i = threadIdx.x; i < nchunk; i += 256) {
      uint64_t *row = chunk_tab + (uint64_t)i * 8;
      if (row[C_ROWS] != ~0ull) row[C_QID] = row[C_ROWS];
    }
}


}  // namespace

hipError_t launch_libsvm(const LibsvmArgs &a, const FastSvmArgs &f, bool use_fast, uint64_t *res,
                         int phase, hipStream_t s) {
  hipError_t e;
  uint32_t *gate = f.gate;
  // ---- set-up, one launch: result block and gate (gate = 0: the single
  // pass decides; 1: exact path only), chunk rows no tile writes (~0, filled
  // by the finish kernel), the single pass's first error, look-back words,
  // qid shards and unit minima, the exact path's unit minima
  FillList fl{};
  if (phase != kPhaseFill) {
    fill_result(fl, res);
    fl.gate = gate;
    fl.gate_v = use_fast ? 0u : 1u;
  }
  if (phase != kPhaseCount) fl.add(f.chunk_tab, (uint64_t)f.nchunk * 8, ~0ull);
  fl.add(reinterpret_cast<uint64_t *>(f.err), 1, ~0ull);
  // the lean kernel first on a full call (indexing_mode < 0 and the count /
  // fill phases stay on svm_fast_tile alone)
  const bool lean = use_fast && phase == kPhaseFull && f.indexing_mode >= 0 && f.lean_lb && lean_enabled();
  if (lean) fl.add(f.lean_lb, (uint64_t)f.ntiles * fast::kLbWords + 1, 0);  // + the poison word
  if (use_fast) {
    fl.add(f.lb, (uint64_t)f.ntiles * fast::kLbWords + 1, 0);  // + the ticket word
    fl.add(f.qsum, kLabShards * 8, 0);
    if (phase != kPhaseCount && f.indexing_mode < 0) fl.add(f.umin, (uint64_t)f.nchunk, ~0ull);
  }
  if (phase != kPhaseFill && a.indexing_mode < 0) fl.add(a.chunk_min, (uint64_t)a.nchunk, ~0ull);
  if (!a.ntiles && phase != kPhaseCount) fl.add(a.offset, 1, 0);  // empty input: offset = {0}
  if ((e = launch_prologue(fl, s)) != hipSuccess) return e;
  FastSvmArgs fa = f;  // the full kernel on its own (no lean launch ahead of it)
  fa.lean_lb = fa.lean_poison = nullptr;
  if (use_fast) {
    if (phase == kPhaseCount) {
      prof_mark(0, s, "svm_fast_tile<1>");
      svm_fast_tile<1><<<FSVM_PERSIST ? persistent_grid(svm_fast_tile<1>, f.ntiles) : f.ntiles, fast::kFThreads, 0, s>>>(fa);
      prof_mark(1, s, "svm_fast_tile<1>");
    } else if (lean) {
      // the full kernel resumes at the first tile the lean one poisoned (all
      // of its workgroups exit at once when none did)
      prof_mark(0, s, "svm_lean_tile");
      svm_lean_tile<<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      prof_mark(1, s, "svm_lean_tile");
      svm_fast_tile<2><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
    } else {
      prof_mark(0, s, "svm_fast_tile<2>");
      svm_fast_tile<2><<<FSVM_PERSIST ? persistent_grid(svm_fast_tile<2>, f.ntiles) : f.ntiles, fast::kFThreads, 0, s>>>(fa);
      prof_mark(1, s, "svm_fast_tile<2>");
    }
    // the qid decision (qid_fix_kernel) is folded into the exact count
    // kernel (a mix hands over) and the finish kernel (every row has a qid);
    // the fill phase keeps the kernel
    if (phase == kPhaseFill) qid_fix_kernel<<<1, 256, 0, s>>>(f.qsum, res, gate, f.chunk_tab, f.nchunk);
  }
  LibsvmArgs ac = a;  // the exact count pass of a full / count phase: the qid check
  if (use_fast && phase != kPhaseFill) {
    ac.qsum = f.qsum;
    ac.qres = res;
  }
  // ---- exact path, gated on the device flag (early exit when the fast path stood)
  if (phase == kPhaseFill) reopen_kernel<<<1, 1, 0, s>>>(res, a.offset, a.cap[C_ROWS], gate);
  // the chunk rows the single pass wrote are reset when it handed over
  const bool reset_tab = use_fast && phase != kPhaseCount && f.chunk_tab && f.nchunk > 0;
  uint64_t *rtab = reset_tab ? f.chunk_tab : nullptr;
  const uint64_t ntab = reset_tab ? (uint64_t)f.nchunk * 8 : 0;
  if (a.ntiles) {
    if (phase != kPhaseFill) {
      libsvm_tile<1><<<a.ntiles, kThreads, 0, s>>>(ac);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], gate, rtab, ntab, gate);
      if (phase == kPhaseCount) note_gate_kernel<<<1, 1, 0, s>>>(gate);
    } else {
      // the count phase stood on the single-pass kernel but its write pass
      // handed over: count on the exact path first (scan.h recount_flag_kernel)
      recount_flag_kernel<<<1, 1, 0, s>>>(gate);
      auto ra = a;
      ra.gate = gate + 2;
      libsvm_tile<1><<<a.ntiles, kThreads, 0, s>>>(ra);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], gate + 2, rtab, ntab, gate);
    }
    if (phase != kPhaseCount) {
      if (!use_fast) prof_mark(0, s, "libsvm_tile<2>");
      libsvm_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
      if (!use_fast) prof_mark(1, s, "libsvm_tile<2>");
    }
  }
  finish_kernel<<<1, 256, 0, s>>>(res, gate, f.err, phase != kPhaseCount ? f.chunk_tab : nullptr, f.nchunk,
                                  use_fast && phase != kPhaseFill ? f.qsum : nullptr);
  if (use_fast && phase != kPhaseCount && f.indexing_mode < 0 &&
      (e = launch_umin_fix(f.index, nullptr, f.wide, f.chunk_tab, f.nchunk, f.umin, res, gate, f.cap[C_INDEX], 0, s)) !=
          hipSuccess)
    return e;
  return hipGetLastError();
}

}  // namespace dmlc_amd

#if defined(DMLC_AMD_STAMPS)
// diagnostic build: copy the phase stamps of the last launch to the host
extern "C" int dmlc_amd_debug_stamps(void *dst, size_t bytes) {
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(dmlc_amd::fast::g_stamps), bytes, 0,
                             hipMemcpyDeviceToHost) == hipSuccess ? 0 : 33;
}
#endif
