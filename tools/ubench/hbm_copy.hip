// HBM copy-rate probe (bench.py hbm_copy context): device-to-device copies of
// 4 GiB by 16-byte lanes, over grid shapes and unroll depths, plain or
// non-temporal; (read + write bytes) / time, best of 5 per shape.
//   hipcc --offload-arch=gfx950 -O3 -o hbm_copy hbm_copy.hip && ./hbm_copy
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

typedef unsigned v4u __attribute__((ext_vector_type(4)));

template <int U, bool NT>
__global__ void __launch_bounds__(256) copy_gs(uint4 *__restrict__ dst, const uint4 *__restrict__ src, uint64_t n16) {
  const uint64_t stride = (uint64_t)gridDim.x * 256 * U;
  for (uint64_t i = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; i < n16; i += stride) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = i + (uint64_t)u * 256;
      if (j < n16) {
        if (NT) {
          const v4u x = __builtin_nontemporal_load(reinterpret_cast<const v4u *>(src + j));
          v[u] = make_uint4(x.x, x.y, x.z, x.w);
        } else {
          v[u] = src[j];
        }
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = i + (uint64_t)u * 256;
      if (j < n16) {
        if (NT) __builtin_nontemporal_store(v4u{v[u].x, v[u].y, v[u].z, v[u].w}, reinterpret_cast<v4u *>(dst + j));
        else dst[j] = v[u];
      }
    }
  }
}

#define CK(x)                                                                 \
  do {                                                                        \
    hipError_t e_ = (x);                                                      \
    if (e_ != hipSuccess) {                                                   \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));            \
      return 1;                                                               \
    }                                                                         \
  } while (0)

template <int U, bool NT>
int run(uint4 *d, const uint4 *s, uint64_t n16, unsigned blocks, hipEvent_t e0, hipEvent_t e1) {
  const uint64_t need = (n16 + 256ull * U - 1) / (256ull * U);
  const unsigned g = blocks ? blocks : (unsigned)need;
  float best = 1e30f;
  for (int r = 0; r < 6; ++r) {
    CK(hipEventRecord(e0, 0));
    copy_gs<U, NT><<<g, 256>>>(d, s, n16);
    CK(hipEventRecord(e1, 0));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    if (r && ms < best) best = ms;
  }
  std::printf("{\"case\": \"hbm_copy\", \"unroll\": %d, \"nt\": %d, \"blocks\": %u, \"GBps\": %.1f}\n", U, NT ? 1 : 0,
              g, 2.0 * n16 * 16 / (best * 1e-3) / 1e9);
  return 0;
}

int main() {
  const uint64_t bytes = 4ull << 30, n16 = bytes / 16;
  uint4 *a, *b;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMemset(a, 1, bytes));
  CK(hipMemset(b, 0, bytes));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const unsigned grids[] = {2048, 4096, 8192, 16384, 0};
  for (unsigned g : grids) {
    if (run<4, false>(b, a, n16, g, e0, e1)) return 1;
    if (run<8, false>(b, a, n16, g, e0, e1)) return 1;
    if (run<4, true>(b, a, n16, g, e0, e1)) return 1;
    if (run<2, false>(b, a, n16, g, e0, e1)) return 1;
  }
  CK(hipFree(a));
  CK(hipFree(b));
  return 0;
}
