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
                 uint64_t *offset, uint64_t cap_rows, const uint32_t *gate) {
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
__global__ void __launch_bounds__(256) chunk_fixup_kernel(uint64_t *chunk_tab, int nchunk, const uint64_t *res) {
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

// Before the exact write pass: when the gate handed the input over, forget the
// chunk-table rows the single-pass kernel wrote (units the exact kernels never
// visit -- no line in them -- then take the next unit's counts in
// chunk_fixup_kernel instead of stale single-pass ones).
__global__ void tab_reset_kernel(uint64_t *tab, uint64_t n, const uint32_t *gate) {
  if (*gate == 0) return;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    tab[i] = ~0ull;
}

// The fill phase of a COUNT_ONLY -> FILL_ONLY pair reuses the tile bases of
// the count phase.  When that count ran on the single-pass kernel (gate 0)
// but the single-pass write kernel then hands over (the kSpinLimit valve sets
// gate bit 1), no exact-path tile bases exist yet: the fill phase must count
// first.  gate[1] = the gate as the count phase left it; gate[2] = "recount".
__global__ void note_gate_kernel(uint32_t *gate) { gate[1] = gate[0]; }
__global__ void recount_flag_kernel(uint32_t *gate) { gate[2] = (gate[0] != 0 && gate[1] == 0) ? 1u : 0u; }

}  // namespace
}  // namespace dmlc_amd
