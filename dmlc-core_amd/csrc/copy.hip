// copy.hip -- stream copies between page-locked host memory and HBM by a
// kernel (the engine's H2D of text batches and D2H of CSR arrays).  One SDMA
// engine moved ~20 GB/s per copy on the MI355X box; wavefronts reading or
// writing the host buffer directly keep enough PCIe requests in flight to
// run the pipeline ~1.3x faster end to end.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "dmlc_amd.h"

namespace dmlc_amd {
namespace {
constexpr int kCopyThreads = 256, kCopyUnroll = 4;  // 16-byte units per thread per round
constexpr unsigned kCopyMaxBlocks = 2048;

__global__ void __launch_bounds__(kCopyThreads) copy16_kernel(uint4 *__restrict__ dst, const uint4 *__restrict__ src,
                                                             uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * kCopyThreads * kCopyUnroll;
  for (uint64_t i = (uint64_t)blockIdx.x * kCopyThreads * kCopyUnroll + threadIdx.x; i < n16; i += stride) {
    uint4 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {  // every load of the round in flight before any store
      const uint64_t j = i + (uint64_t)u * kCopyThreads;
      if (j < n16) v[u] = src[j];
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint64_t j = i + (uint64_t)u * kCopyThreads;
      if (j < n16) dst[j] = v[u];
    }
  }
}

__global__ void copy_tail_kernel(uint8_t *dst, const uint8_t *src, uint32_t n) {
  if (threadIdx.x < n) dst[threadIdx.x] = src[threadIdx.x];
}

// Several copies in one launch (dmlc_amd_copy_n: the CSR arrays of a batch):
// copy i owns blocks [first[i], first[i+1]) and walks its 16-byte units with
// that stride; its last block also copies the tail bytes.
constexpr int kCopyN = DMLC_AMD_COPY_MAX;
struct CopyList {
  uint4 *dst[kCopyN];
  const uint4 *src[kCopyN];
  uint64_t bytes[kCopyN];
  uint32_t first[kCopyN + 1];
  int n;
};
__global__ void __launch_bounds__(kCopyThreads) copy_n_kernel(CopyList L) {
  int i = 0;
  while (i + 1 < L.n && blockIdx.x >= L.first[i + 1]) ++i;  // block-uniform
  const uint32_t b = blockIdx.x - L.first[i], nb = L.first[i + 1] - L.first[i];
  uint4 *__restrict__ dst = L.dst[i];
  const uint4 *__restrict__ src = L.src[i];
  const uint64_t n16 = L.bytes[i] >> 4;
  const uint64_t stride = (uint64_t)nb * kCopyThreads * kCopyUnroll;
  for (uint64_t j0 = (uint64_t)b * kCopyThreads * kCopyUnroll + threadIdx.x; j0 < n16; j0 += stride) {
    uint4 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint64_t j = j0 + (uint64_t)u * kCopyThreads;
      if (j < n16) v[u] = src[j];
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint64_t j = j0 + (uint64_t)u * kCopyThreads;
      if (j < n16) dst[j] = v[u];
    }
  }
  const uint32_t tail = (uint32_t)(L.bytes[i] & 15u);
  if (b + 1 == nb && threadIdx.x < tail)
    reinterpret_cast<uint8_t *>(dst + n16)[threadIdx.x] = reinterpret_cast<const uint8_t *>(src + n16)[threadIdx.x];
}

// Device-sized form: copy i's byte count comes from d_counts when the kernel
// runs (its blocks were laid out for max_bytes; the ones past the count idle)
struct CopyListDev {
  uint4 *dst[kCopyN];
  const uint4 *src[kCopyN];
  uint64_t scale[kCopyN], add[kCopyN], maxb[kCopyN];
  int slot[kCopyN];
  uint32_t first[kCopyN + 1];
  int n;
};
__global__ void __launch_bounds__(kCopyThreads) copy_n_dev_kernel(CopyListDev L, const uint64_t *d_counts) {
  int i = 0;
  while (i + 1 < L.n && blockIdx.x >= L.first[i + 1]) ++i;  // block-uniform
  const uint32_t b = blockIdx.x - L.first[i], nb = L.first[i + 1] - L.first[i];
  uint64_t bytes = L.slot[i] >= 0 ? d_counts[L.slot[i]] * L.scale[i] + L.add[i] : L.add[i];
  bytes = bytes < L.maxb[i] ? bytes : L.maxb[i];
  uint4 *__restrict__ dst = L.dst[i];
  const uint4 *__restrict__ src = L.src[i];
  const uint64_t n16 = bytes >> 4;
  const uint64_t stride = (uint64_t)nb * kCopyThreads * kCopyUnroll;
  for (uint64_t j0 = (uint64_t)b * kCopyThreads * kCopyUnroll + threadIdx.x; j0 < n16; j0 += stride) {
    uint4 v[kCopyUnroll];
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint64_t j = j0 + (uint64_t)u * kCopyThreads;
      if (j < n16) v[u] = src[j];
    }
#pragma unroll
    for (int u = 0; u < kCopyUnroll; ++u) {
      const uint64_t j = j0 + (uint64_t)u * kCopyThreads;
      if (j < n16) dst[j] = v[u];
    }
  }
  const uint32_t tail = (uint32_t)(bytes & 15u);
  if (b == 0 && threadIdx.x < tail)
    reinterpret_cast<uint8_t *>(dst + n16)[threadIdx.x] = reinterpret_cast<const uint8_t *>(src + n16)[threadIdx.x];
}
}  // namespace
}  // namespace dmlc_amd

extern "C" int dmlc_amd_copy_n_dev(void *const *dst, const void *const *src, const uint64_t *d_counts,
                                   const int *slot, const uint64_t *scale, const uint64_t *add,
                                   const uint64_t *max_bytes, int n, void *stream) {
  if (n < 0 || n > DMLC_AMD_COPY_MAX || (n && (!dst || !src || !slot || !scale || !add || !max_bytes)))
    return DMLC_AMD_ERR_ARG;
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dmlc_amd::CopyListDev L;
  L.n = 0;
  uint32_t blocks = 0;
  const uint64_t per_block = (uint64_t)dmlc_amd::kCopyThreads * dmlc_amd::kCopyUnroll;
  for (int i = 0; i < n; ++i) {
    if (max_bytes[i] == 0) continue;
    if (!dst[i] || !src[i] || slot[i] >= DMLC_AMD_COPY_SLOTS || (slot[i] >= 0 && !d_counts)) return DMLC_AMD_ERR_ARG;
    if (((reinterpret_cast<uintptr_t>(dst[i]) | reinterpret_cast<uintptr_t>(src[i])) & 15u) != 0)
      return DMLC_AMD_ERR_ARG;
    const uint64_t nb =
        std::max<uint64_t>(1, std::min<uint64_t>(((max_bytes[i] >> 4) + per_block - 1) / per_block, 1024));
    L.dst[L.n] = static_cast<uint4 *>(dst[i]);
    L.src[L.n] = static_cast<const uint4 *>(src[i]);
    L.slot[L.n] = slot[i];
    L.scale[L.n] = scale[i];
    L.add[L.n] = add[i];
    L.maxb[L.n] = max_bytes[i];
    L.first[L.n] = blocks;
    blocks += (uint32_t)nb;
    ++L.n;
  }
  if (L.n == 0) return DMLC_AMD_OK;
  L.first[L.n] = blocks;
  dmlc_amd::copy_n_dev_kernel<<<blocks, dmlc_amd::kCopyThreads, 0, s>>>(L, d_counts);
  return hipGetLastError() == hipSuccess ? DMLC_AMD_OK : DMLC_AMD_ERR_HIP;
}

extern "C" int dmlc_amd_copy_n(void *const *dst, const void *const *src, const uint64_t *bytes, int n,
                               void *stream) {
  if (n < 0 || n > DMLC_AMD_COPY_MAX || (n && (!dst || !src || !bytes))) return DMLC_AMD_ERR_ARG;
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  dmlc_amd::CopyList L;
  L.n = 0;
  uint32_t blocks = 0;
  const uint64_t per_block = (uint64_t)dmlc_amd::kCopyThreads * dmlc_amd::kCopyUnroll;
  for (int i = 0; i < n; ++i) {
    if (bytes[i] == 0) continue;
    if (!dst[i] || !src[i]) return DMLC_AMD_ERR_ARG;
    if (((reinterpret_cast<uintptr_t>(dst[i]) | reinterpret_cast<uintptr_t>(src[i])) & 15u) != 0) {
      const int rc = dmlc_amd_copy(dst[i], src[i], bytes[i], stream);  // unaligned: on its own
      if (rc != DMLC_AMD_OK) return rc;
      continue;
    }
    const uint64_t nb = std::max<uint64_t>(1, std::min<uint64_t>(((bytes[i] >> 4) + per_block - 1) / per_block, 1024));
    L.dst[L.n] = static_cast<uint4 *>(dst[i]);
    L.src[L.n] = static_cast<const uint4 *>(src[i]);
    L.bytes[L.n] = bytes[i];
    L.first[L.n] = blocks;
    blocks += (uint32_t)nb;
    ++L.n;
  }
  if (L.n == 0) return DMLC_AMD_OK;
  L.first[L.n] = blocks;
  dmlc_amd::copy_n_kernel<<<blocks, dmlc_amd::kCopyThreads, 0, s>>>(L);
  return hipGetLastError() == hipSuccess ? DMLC_AMD_OK : DMLC_AMD_ERR_HIP;
}

extern "C" int dmlc_amd_copy(void *dst, const void *src, uint64_t bytes, void *stream) {
  if (bytes == 0) return DMLC_AMD_OK;
  if (!dst || !src) return DMLC_AMD_ERR_ARG;
  const hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  if (((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15u) != 0)
    return hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, s) == hipSuccess ? DMLC_AMD_OK : DMLC_AMD_ERR_HIP;
  const uint64_t n16 = bytes >> 4;
  if (n16) {
    const uint64_t per_block = (uint64_t)dmlc_amd::kCopyThreads * dmlc_amd::kCopyUnroll;
    const unsigned blocks = (unsigned)std::min<uint64_t>((n16 + per_block - 1) / per_block, dmlc_amd::kCopyMaxBlocks);
    dmlc_amd::copy16_kernel<<<blocks, dmlc_amd::kCopyThreads, 0, s>>>(
        static_cast<uint4 *>(dst), static_cast<const uint4 *>(src), n16);
  }
  const uint32_t tail = (uint32_t)(bytes & 15u);
  if (tail)
    dmlc_amd::copy_tail_kernel<<<1, 64, 0, s>>>(static_cast<uint8_t *>(dst) + (n16 << 4),
                                                static_cast<const uint8_t *>(src) + (n16 << 4), tail);
  return hipGetLastError() == hipSuccess ? DMLC_AMD_OK : DMLC_AMD_ERR_HIP;
}
