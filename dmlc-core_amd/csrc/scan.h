// scan.h -- exclusive scan of per-tile counter vectors (single workgroup) and
// pipeline finalisation.  Included by each kernel translation unit (no RDC).
#pragma once
#include "block.h"

namespace dmlc_amd {
namespace {  // one private copy per kernel translation unit (no RDC)

struct Cnt64 {
  uint64_t c[8];
};
struct Cnt64Add {
  DA_HD Cnt64 operator()(const Cnt64 &a, const Cnt64 &b) const {
    Cnt64 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.c[i] = a.c[i] + b.c[i];
    return r;
  }
};

// tile_base[k] = sum_{j<k} tile_cnt[j]; res[0..C_N) = totals;
// offset[total_rows] = total index count (the reference's final offset push).
__global__ void __launch_bounds__(kThreads)
tile_scan_kernel(const uint64_t *tile_cnt, uint64_t *tile_base, uint32_t ntiles, uint64_t *res,
                 uint64_t *offset, uint64_t cap_rows, const uint32_t *gate, uint64_t *tab = nullptr,
                 uint64_t ntab = 0, const uint32_t *tab_gate = nullptr) {
  // before the exact write pass of a call whose single pass handed over:
  // forget the chunk-table rows it wrote (units the exact kernels never visit
  // -- no line in them -- then take the next unit's counts in the finish
  // kernel instead of stale single-pass ones)
  if (tab && *tab_gate)
    for (uint64_t i = threadIdx.x; i < ntab; i += blockDim.x) tab[i] = ~0ull;
  if (gate && *gate == 0) return;
  __shared__ uint64_t scratch[kBlockScratchU64];
  DevBlock bk{scratch};
  const uint32_t per = (ntiles + kThreads - 1) / kThreads;
  const uint32_t t0 = threadIdx.x * per, t1 = min(t0 + per, ntiles);
  Cnt64 mine, zero;
#pragma unroll
  for (int i = 0; i < 8; ++i) mine.c[i] = zero.c[i] = 0;
  for (uint32_t k = t0; k < t1; ++k)
    for (int i = 0; i < C_N; ++i) mine.c[i] += tile_cnt[(uint64_t)k * C_N + i];
  Cnt64 total;
  Cnt64 run = bk.exclusive(mine, zero, Cnt64Add(), &total);
  for (uint32_t k = t0; k < t1; ++k)
    for (int i = 0; i < C_N; ++i) {
      tile_base[(uint64_t)k * C_N + i] = run.c[i];
      run.c[i] += tile_cnt[(uint64_t)k * C_N + i];
    }
  if (threadIdx.x == 0) {
    for (int i = 0; i < C_N; ++i) res[i] = total.c[i];
    if (offset && total.c[C_ROWS] < cap_rows + 1) offset[total.c[C_ROWS]] = total.c[C_INDEX];
  }
}

// Chunk rows no tile wrote (chunks holding no line: all newlines, empty, or
// starting at the end of the text) -- the launchers pre-fill the table with
// ~0 -- take the exclusive counts of the next chunk, or the totals.
// One block: each unwritten row first notes its source (the next written
// row, or nchunk for the totals) in the unused eighth slot, then copies from
// it -- sources are never copied into, so the two phases do not race.  (A
// single thread walking the rows backwards took ~160 us on ~500 rows: one
// dependent global round trip per row.)
__device__ __forceinline__ void chunk_fixup_body(uint64_t *chunk_tab, int nchunk, const uint64_t *res) {
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    uint64_t *row = chunk_tab + (uint64_t)c * 8;
    if (row[0] != ~0ull) continue;
    int j = c + 1;
    while (j < nchunk && chunk_tab[(uint64_t)j * 8] == ~0ull) ++j;
    row[7] = (uint64_t)j;
  }
  __syncthreads();
  for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
    uint64_t *row = chunk_tab + (uint64_t)c * 8;
    if (row[0] == ~0ull) {
      const uint64_t j = row[7];
      const uint64_t *nx = j < (uint64_t)nchunk ? chunk_tab + j * 8 : res;
      for (int i = 0; i < 7; ++i) row[i] = nx[i];
    }
    row[7] = 0;  // the unused eighth slot
  }
}

// The fill phase of a COUNT_ONLY -> FILL_ONLY pair reuses the tile bases of
// the count phase.  When that count ran on the single-pass kernel (gate 0)
// but the single-pass write kernel then hands over (the kSpinLimit valve sets
// gate bit 1), no exact-path tile bases exist yet: the fill phase must count
// first.  gate[1] = the gate as the count phase left it; gate[2] = "recount".
__global__ void note_gate_kernel(uint32_t *gate) { gate[1] = gate[0]; }
__global__ void recount_flag_kernel(uint32_t *gate) { gate[2] = (gate[0] != 0 && gate[1] == 0) ? 1u : 0u; }

// ---- per-call set-up and finish, one launch each (every kernel boundary on
// the stream costs a few microseconds: the set-up used to be six memsets and
// the finish two kernels).  Prologue: fill up to kFillRegions word ranges and
// set the gate word.
// (launch_libsvm's largest list is 10: indexing_mode < 0 on empty input.)
// A region past kFillRegions is never dropped silently: add() notes the
// overflow and launch_prologue refuses the call.
constexpr int kFillRegions = 12;
struct FillList {
  uint64_t *p[kFillRegions];
  uint64_t n[kFillRegions];
  uint64_t v[kFillRegions];
  uint32_t *gate;  // set to gate_v when non-null
  uint32_t gate_v;
  int count;
  int overflow;
  DA_HD void add(uint64_t *ptr, uint64_t words, uint64_t value) {
    if (!ptr || !words) return;
    if (count >= kFillRegions) {
      overflow = 1;
      return;
    }
    p[count] = ptr;
    n[count] = words;
    v[count] = value;
    ++count;
  }
};
__global__ void __launch_bounds__(256) prologue_kernel(FillList f) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  if (t == 0 && f.gate) *f.gate = f.gate_v;
  for (int r = 0; r < f.count; ++r)
    for (uint64_t i = t; i < f.n[r]; i += stride) f.p[r][i] = f.v[r];
}
inline hipError_t launch_prologue(const FillList &f, hipStream_t s) {
  if (f.overflow) return hipErrorInvalidValue;  // a buffer would stay unset
  uint64_t most = 1;
  for (int r = 0; r < f.count; ++r) most = f.n[r] > most ? f.n[r] : most;
  uint64_t blocks = (most + 1023) / 1024;  // four words per thread on the largest range
  blocks = blocks < 1 ? 1 : (blocks > 1024 ? 1024 : blocks);
  prologue_kernel<<<(unsigned)blocks, 256, 0, s>>>(f);
  return hipGetLastError();
}
// The result block of a call's first phase: counts 0, first error "none" (~0).
inline void fill_result(FillList &f, uint64_t *res) {
  f.add(res, 8, 0);
  f.add(res + 8, 1, ~0ull);
  f.add(res + 9, 7, 0);
}

// Finish: the error of whichever path produced the result (res[8]) and the
// path (res[9]), then the chunk rows no tile wrote (chunk_fixup_body), one block of 256.
// With qsum (libsvm after its single pass, full and count phases): first the
// qid decision when the single pass stood (svm_fast.h qid_decide; a mix was
// handed over by the exact count kernel): every row has a qid, so the qid
// count is the row count, in the result and in each written chunk row.
__global__ void __launch_bounds__(256) finish_kernel(uint64_t *res, const uint32_t *gate,
                                                     const unsigned long long *ferr, uint64_t *chunk_tab, int nchunk,
                                                     const uint64_t *qsum = nullptr) {
  __shared__ int qid_rows;
  if (threadIdx.x < kWave) {
    uint64_t t = qsum && *gate == 0 && qsum[1] ? qsum[threadIdx.x * 8] : 0;
    for (int d = 32; d >= 1; d >>= 1) t += __shfl_xor(t, d, kWave);
    if (threadIdx.x == 0) {
      qid_rows = t != 0 && t == res[C_ROWS];
      if (qid_rows) res[C_QID] = t;
      if (*gate == 0) res[8] = *ferr;
      if (res[8] == ~0ull) res[8] = 0;
      res[9] = *gate;  // dmlc_amd_result.path
    }
  }
  __syncthreads();
  if (!chunk_tab || nchunk <= 0) return;
  if (qid_rows) {
    for (int c = threadIdx.x; c < nchunk; c += blockDim.x) {
      uint64_t *row = chunk_tab + (uint64_t)c * 8;
      if (row[C_ROWS] != ~0ull) row[C_QID] = row[C_ROWS];
    }
    __syncthreads();
  }
  chunk_fixup_body(chunk_tab, nchunk, res);
}

}  // namespace
}  // namespace dmlc_amd
