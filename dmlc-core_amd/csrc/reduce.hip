// reduce.hip -- maxima of the written index / field arrays
// (DMLC_AMD_FLAG_MAX_INDEX): RowBlockContainer::Push tracks max_index /
// max_field over every pushed entry (src/data/row_block.h:126-168) and
// BasicRowIter::NumCol returns max_index + 1 (basic_row_iter.h:46-48).  The
// element count is read on the device (the result block), so the reduction
// needs no host round trip; one 64-bit atomicMax per workgroup.
#include "common.h"
#include "dmlc_amd_kernels.h"

namespace dmlc_amd {
namespace {

template <typename T>
__global__ void __launch_bounds__(256) max_kernel(const T *a, const uint64_t *count, uint64_t cap,
                                                  unsigned long long *out) {
  const uint64_t n = *count < cap ? *count : cap;
  uint64_t m = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (uint64_t)gridDim.x * 256) {
    const uint64_t v = (uint64_t)a[i];
    m = v > m ? v : m;
  }
  for (int d = 32; d >= 1; d >>= 1) {
    const uint64_t o = __shfl_xor(m, d, kWave);
    m = o > m ? o : m;
  }
  __shared__ uint64_t w[4];
  if ((threadIdx.x & 63u) == 0) w[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t r = w[0];
    for (int i = 1; i < 4; ++i) r = w[i] > r ? w[i] : r;
    if (r) atomicMax(out, (unsigned long long)r);
  }
}

}  // namespace

hipError_t launch_max(const void *arr, int wide, const uint64_t *count, uint64_t cap, uint64_t *out,
                      hipStream_t s) {
  hipError_t e = hipMemsetAsync(out, 0, sizeof(uint64_t), s);
  if (e != hipSuccess || !arr || cap == 0) return e;
  unsigned long long *o = reinterpret_cast<unsigned long long *>(out);
  if (wide) max_kernel<uint64_t><<<1024, 256, 0, s>>>(static_cast<const uint64_t *>(arr), count, cap, o);
  else max_kernel<uint32_t><<<1024, 256, 0, s>>>(static_cast<const uint32_t *>(arr), count, cap, o);
  return hipGetLastError();
}

}  // namespace dmlc_amd
