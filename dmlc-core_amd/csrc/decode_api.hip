// decode_api.hip -- batch entry point over the exact decoders (decode.h):
// dmlc::strtof semantics (strtonum.h:279-281) for many NUL-delimited strings.
#include "decode.h"
#include "dmlc_amd.h"

namespace dmlc_amd {
namespace {
__global__ void strtof_batch_kernel(const uint8_t *text, const uint64_t *off, uint64_t n, float *out,
                                    uint32_t *consumed, uint32_t *nan_err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  Src at;
  at.g = text;
  at.lim = off[i + 1];
  at.lds = nullptr;
  at.wbase = at.wend = 0;
  uint64_t e;
  bool bad = false;
  out[i] = parse_float(at, off[i], &e, &bad);
  if (consumed) consumed[i] = (uint32_t)(e - off[i]);
  if (nan_err) nan_err[i] = bad;
}
}  // namespace
}  // namespace dmlc_amd

extern "C" int dmlc_amd_strtof_batch(const void *d_text, const uint64_t *d_offsets, uint64_t n,
                                     float *d_out, uint32_t *d_consumed, uint32_t *d_nan_error,
                                     void *stream) {
  if (n == 0) return DMLC_AMD_OK;
  if (!d_text || !d_offsets || !d_out) return DMLC_AMD_ERR_ARG;
  const unsigned blocks = (unsigned)((n + 255) / 256);
  dmlc_amd::strtof_batch_kernel<<<blocks, 256, 0, reinterpret_cast<hipStream_t>(stream)>>>(
      reinterpret_cast<const uint8_t *>(d_text), d_offsets, n, d_out, d_consumed, d_nan_error);
  return hipGetLastError() == hipSuccess ? DMLC_AMD_OK : DMLC_AMD_ERR_HIP;
}
