// dmlc_amd_kernels.h -- argument blocks and launchers shared between the
// C-ABI (capi.cpp) and the per-format kernel translation units.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "args.h"

namespace dmlc_amd {

// Launch count -> scan -> write on `s`.  `res` is the device result block
// (dmlc_amd_result layout).  count_only skips the write pass.
hipError_t launch_libsvm(const LibsvmArgs &a, uint64_t *res, bool count_only, hipStream_t s);
hipError_t launch_csv(const CsvArgs &a, uint64_t *res, bool count_only, hipStream_t s);

}  // namespace dmlc_amd
