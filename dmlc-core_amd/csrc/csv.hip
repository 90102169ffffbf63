// csv.hip -- MI355X kernels for CSVParser<I,D>::ParseBlock (csv_parser.h:71-149);
// the tile body lives in csv_core.h.
#include "block.h"
#include "csv_core.h"
#include "csv_fast.h"
#include "dmlc_amd_kernels.h"
#include "scan.h"

namespace dmlc_amd {
namespace {

template <int MODE>
#ifndef FEX_MINW
#define FEX_MINW 4  // waves per SIMD the exact tile kernels are register-budgeted for (round 4: 1 -> 4, config 3 exact 15.0 -> 13.6 ms; 5 waves spill more and lose: 14.9 ms)
#endif
__global__ void __launch_bounds__(kThreads, FEX_MINW) csv_tile(CsvArgs a) {
  __shared__ __attribute__((aligned(16))) csv::Shared sh;
  __shared__ uint64_t scratch[kBlockScratchU64];
  DevBlock bk{scratch};
  csv::tile<MODE>(a, sh, bk, blockIdx.x);
}

static_assert(sizeof(fcsv::Shared) + kSmallScratchU64 * 8 <= fast::kLdsBudget,
              "csv_fast_tile LDS above the 6-workgroup budget (fast_common.h kLdsBudget)");

#ifndef FCSV_MINW
#define FCSV_MINW 6
#endif
template <int MODE>
__global__ void __launch_bounds__(fast::kFThreads, FCSV_MINW) csv_fast_tile(FastCsvArgs a) {
  __shared__ __attribute__((aligned(16))) fcsv::Shared sh;
  __shared__ uint64_t scratch[kSmallScratchU64];
  DevBlockS bk{scratch};
  fcsv::tile<MODE, false, 0>(a, sh, bk, blockIdx.x);
}
// integer DTypes (strtoll)
template <int MODE>
__global__ void __launch_bounds__(fast::kFThreads, FCSV_MINW) csv_fast_tile_int(FastCsvArgs a) {
  __shared__ __attribute__((aligned(16))) fcsv::Shared sh;
  __shared__ uint64_t scratch[kSmallScratchU64];
  DevBlockS bk{scratch};
  fcsv::tile<MODE, false, 1>(a, sh, bk, blockIdx.x);
}
// with a label and / or weight column
template <int MODE>
__global__ void __launch_bounds__(fast::kFThreads, FCSV_MINW) csv_fast_tile_sp(FastCsvArgs a) {
  __shared__ __attribute__((aligned(16))) fcsv::Shared sh;
  __shared__ uint64_t scratch[kSmallScratchU64];
  DevBlockS bk{scratch};
  fcsv::tile<MODE, true, 0>(a, sh, bk, blockIdx.x);
}

// fill phase after a count phase that fell back to the exact kernels: reopen
// the first-error word so the write pass can record it, and store the closing
// offset (the reference's final push) the size query could not
__global__ void reopen_kernel(uint64_t *res, uint64_t *offset, uint64_t cap_rows, const uint32_t *gate) {
  if (*gate == 0) return;
  if (res[8] == 0) res[8] = ~0ull;
  if (offset && res[0] < cap_rows + 1) offset[res[0]] = res[1];
}

// label column: the single pass assumed one non-empty label field per row
// (and, for column 0, a delimiter in every row); a nonzero check sum hands the
// input to the exact kernels
__global__ void label_check_kernel(const uint64_t *labsum, uint32_t *gate) {
  const uint32_t i = threadIdx.x;  // kLabShards threads, one wave
  uint64_t a = labsum[i * 8], b = labsum[i * 8 + 1], c = labsum[i * 8 + 2];
  for (int d = 32; d >= 1; d >>= 1) {
    a += __shfl_xor(a, d, kWave);
    b += __shfl_xor(b, d, kWave);
    c += __shfl_xor(c, d, kWave);
  }
  if (i == 0 && (a != 0 || b != 0 || c != 0)) *gate |= 1u;
}


}  // namespace

hipError_t launch_csv(const CsvArgs &a, const FastCsvArgs &f, bool use_fast, uint64_t *res, int phase,
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
  if (phase != kPhaseCount) fl.add(f.chunk_tab, (uint64_t)f.nchunk * 8, ~0ull);  // rows no tile writes: finish kernel
  fl.add(reinterpret_cast<uint64_t *>(f.err), 1, ~0ull);
  const bool sp = f.label_col >= 0 || f.weight_col >= 0;
  if (use_fast) {
    fl.add(f.lb, (uint64_t)f.ntiles * kCsvLbWords, 0);
    if (sp) fl.add(f.labsum, kLabShards * 8, 0);
  }
  if (!a.ntiles && phase != kPhaseCount) fl.add(reinterpret_cast<uint64_t *>(a.offset), 1, 0);  // empty input: offset = {0}
  if ((e = launch_prologue(fl, s)) != hipSuccess) return e;
  if (use_fast) {
    const bool iv = f.vtype != 0;
    if (phase == kPhaseCount) {
      prof_mark(0, s, iv ? "csv_fast_tile_int<1>" : "csv_fast_tile<1>");
      if (iv) csv_fast_tile_int<1><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      else if (sp) csv_fast_tile_sp<1><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      else csv_fast_tile<1><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      prof_mark(1, s, "csv_fast_tile<1>");
    } else {
      prof_mark(0, s, iv ? "csv_fast_tile_int<2>" : "csv_fast_tile<2>");
      if (iv) csv_fast_tile_int<2><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      else if (sp) csv_fast_tile_sp<2><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      else csv_fast_tile<2><<<f.ntiles, fast::kFThreads, 0, s>>>(f);
      prof_mark(1, s, "csv_fast_tile<2>");
    }
    if (sp) label_check_kernel<<<1, kLabShards, 0, s>>>(f.labsum, gate);
  }
  // ---- exact path, gated on the device flag (early exit when the fast path stood)
  if (phase == kPhaseFill) reopen_kernel<<<1, 1, 0, s>>>(res, a.offset, a.cap[C_ROWS], gate);
  const bool reset_tab = use_fast && phase != kPhaseCount && f.chunk_tab && f.nchunk > 0;
  uint64_t *rtab = reset_tab ? f.chunk_tab : nullptr;
  const uint64_t ntab = reset_tab ? (uint64_t)f.nchunk * 8 : 0;
  if (a.ntiles) {
    if (phase != kPhaseFill) {
      csv_tile<1><<<a.ntiles, kThreads, 0, s>>>(a);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], gate, rtab, ntab, gate);
      if (phase == kPhaseCount) note_gate_kernel<<<1, 1, 0, s>>>(gate);
    } else {
      // the count phase stood on the single-pass kernel but its write pass
      // handed over: count on the exact path first (scan.h recount_flag_kernel)
      recount_flag_kernel<<<1, 1, 0, s>>>(gate);
      auto ra = a;
      ra.gate = gate + 2;
      csv_tile<1><<<a.ntiles, kThreads, 0, s>>>(ra);
      tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                              res, a.offset, a.cap[C_ROWS], gate + 2, rtab, ntab, gate);
    }
    if (phase != kPhaseCount) {
      if (!use_fast) prof_mark(0, s, "csv_tile<2>");
      csv_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
      if (!use_fast) prof_mark(1, s, "csv_tile<2>");
    }
  }
  finish_kernel<<<1, 256, 0, s>>>(res, gate, f.err, phase != kPhaseCount ? f.chunk_tab : nullptr, f.nchunk);
  return hipGetLastError();
}

}  // namespace dmlc_amd
