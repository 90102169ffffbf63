// hd.h -- portability layer so the tile bodies compile both as HIP device code
// (the product) and as plain C++ for the test-only CPU emulator (tests/emu/).
#pragma once
#include <stdint.h>
#include <string.h>
#if defined(__HIPCC__)
#include <hip/hip_runtime.h>
#define DA_HD __host__ __device__ __forceinline__
#define DA_HDF __host__ __device__ __forceinline__
#else
#include <cstring>
#define DA_HD inline
#define DA_HDF
#endif

namespace dmlc_amd {

DA_HD float u2f(uint32_t u) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __uint_as_float(u);
#else
  float f;
  memcpy(&f, &u, 4);
  return f;
#endif
}

DA_HD void atomic_or_u32(uint32_t *p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(p, v);
#else
  __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
#endif
}

DA_HD void atomic_min_u64(unsigned long long *p, unsigned long long v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicMin(p, v);
#else
  unsigned long long cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (v < cur && !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
#endif
}

template <typename T>
DA_HD T mn(T a, T b) { return a < b ? a : b; }
template <typename T>
DA_HD T mx(T a, T b) { return a < b ? b : a; }

DA_HD int ctz32(uint32_t x) { return __builtin_ctz(x); }
DA_HD int clz32(uint32_t x) { return __builtin_clz(x); }
DA_HD int popc32(uint32_t x) { return __builtin_popcount(x); }

}  // namespace dmlc_amd
