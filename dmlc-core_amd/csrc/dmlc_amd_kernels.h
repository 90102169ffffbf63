// dmlc_amd_kernels.h -- argument blocks and launchers shared between the
// C-ABI (capi.cpp) and the per-format kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "args.h"

namespace dmlc_amd {

// Pipeline phases: full = count -> scan -> write; count = count -> scan (the
// size query; tile bases stay in the workspace); fill = write only, reusing
// the tile bases a count phase left in the same workspace.
enum { kPhaseFull = 0, kPhaseCount = 1, kPhaseFill = 2 };

// Kernel timing hook (capi.cpp): launchers bracket their dominant kernel with
// prof_mark(0, ...) / prof_mark(1, ...); a no-op unless dmlc_amd_profile_begin
// was called on this thread.
void prof_mark(int end, hipStream_t s, const char *kernel);

// Launch the phase on `s`.  `res` is the device result block (dmlc_amd_result layout).
// libsvm: the uniform-grammar kernel (f) runs first when use_fast; the exact
// kernels (a) run when it sets the gate word (f.gate), or always when !use_fast.
hipError_t launch_libsvm(const LibsvmArgs &a, const FastSvmArgs &f, bool use_fast, uint64_t *res,
                         int phase, hipStream_t s);
hipError_t launch_libfm(const LibfmArgs &a, const FastSvmArgs &f, bool use_fast, uint64_t *res, int phase,
                        hipStream_t s);
// units[c * nthread + t] = start of FillData range t of chunk c
// (text_parser.h:116-155); units[nchunk * nthread] = n.
hipError_t launch_ranges(const uint8_t *text, const uint64_t *cs, int nchunk, int nthread, uint64_t n,
                         uint64_t *units, hipStream_t s);
// *out = max(arr[0 .. min(*count, cap))) (0 when empty); arr is u32, or u64 when wide
hipError_t launch_max(const void *arr, int wide, const uint64_t *count, uint64_t cap, uint64_t *out,
                      hipStream_t s);
hipError_t launch_csv(const CsvArgs &a, const FastCsvArgs &f, bool use_fast, uint64_t *res, int phase,
                      hipStream_t s);

}  // namespace dmlc_amd
