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

DA_HD uint32_t f2u(float f) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __float_as_uint(f);
#else
  uint32_t u;
  memcpy(&u, &f, 4);
  return u;
#endif
}

DA_HD void atomic_or_u32(uint32_t *p, uint32_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr(p, v);
#else
  __atomic_fetch_or(p, v, __ATOMIC_RELAXED);
#endif
}

DA_HD void atomic_or_u64(uint64_t *p, uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicOr((unsigned long long *)p, (unsigned long long)v);
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

DA_HD void atomic_max_u64(unsigned long long *p, unsigned long long v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicMax(p, v);
#else
  unsigned long long cur = __atomic_load_n(p, __ATOMIC_RELAXED);
  while (v > cur && !__atomic_compare_exchange_n(p, &cur, v, true, __ATOMIC_RELAXED, __ATOMIC_RELAXED)) {
  }
#endif
}

// atomic min, skipped when a plain read already shows a value <= v: minima
// of many tiles on one word (a ParseBlock unit's) mostly do not improve it,
// and same-address device atomics serialise (a stale read only costs an
// atomic: the word only ever decreases)
DA_HD void atomic_min_u64_if_lower(unsigned long long *p, unsigned long long v) {
#if defined(__HIP_DEVICE_COMPILE__)
  const unsigned long long cur = *(volatile unsigned long long *)p;
#else
  const unsigned long long cur = __atomic_load_n(p, __ATOMIC_RELAXED);
#endif
  if (v < cur) atomic_min_u64(p, v);
}

// a text byte from global memory, typed as such: a read that may come from
// LDS or global memory (the fast kernels' at()) would otherwise become one
// flat load of a selected pointer, which waits on both counters
DA_HD uint32_t gbyte(const uint8_t *t, uint64_t p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return *((const __attribute__((address_space(1))) uint8_t *)t + p);
#else
  return t[p];
#endif
}

// a plain store other threads may race with on the same value (a flag);
// relaxed-atomic on the host so the emulator's threads do not race
DA_HD void store_flag_u64(uint64_t *p, uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  *p = v;
#else
  __atomic_store_n(p, v, __ATOMIC_RELAXED);
#endif
}

DA_HD uint32_t gridDim_x() {  // workgroups of the launch (0 on the host)
#if defined(__HIP_DEVICE_COMPILE__)
  return gridDim.x;
#else
  return 0;
#endif
}

DA_HD uint32_t atomic_add_u32(uint32_t *p, uint32_t v) {  // returns the old value
#if defined(__HIP_DEVICE_COMPILE__)
  return atomicAdd(p, v);
#else
  return __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
#endif
}

DA_HD void atomic_add_u64(uint64_t *p, uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  atomicAdd((unsigned long long *)p, (unsigned long long)v);
#else
  __atomic_fetch_add(p, v, __ATOMIC_RELAXED);
#endif
}

// Look-back words: one 8-byte {status, value} word per counter, stored and
// polled whole by agent-scope relaxed atomics (sc1: no L1, no tearing), so no
// fence or separate flag is needed (MI355X_MICROARCH.md, visibility: R2 form).
DA_HD void store_agent_u64(uint64_t *p, uint64_t v) {
#if defined(__HIP_DEVICE_COMPILE__)
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  __atomic_store_n(p, v, __ATOMIC_RELEASE);
#endif
}
DA_HD uint64_t load_agent_u64(uint64_t *p) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
#else
  return __atomic_load_n(p, __ATOMIC_ACQUIRE);
#endif
}
DA_HD void spin_pause() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_sleep(2);
#endif
}

// Wave priority (s_setprio): a tile on the look-back chain's critical path
// (its serial per-line walk) raised above the tiles that wait for it.
DA_HD void prio_high() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_setprio(3);
#endif
}
DA_HD void prio_normal() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_s_setprio(0);
#endif
}

// v_perm_b32: byte i of the result = byte sel[i] (0..7) of {s0:s1} (s1 = bytes 0-3).
// Callers only pass selectors 0..7.
DA_HD uint32_t perm_b32(uint32_t s0, uint32_t s1, uint32_t sel) {
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_perm(s0, s1, sel);
#else
  // V_PERM_B32: selector byte 0-7 picks a byte of {s0:s1}; 8-11 replicate
  // the sign bit of bytes 1, 3 of s1 and 1, 3 of s0; 12 gives 0x00, 13+ 0xFF
  const uint64_t src = ((uint64_t)s0 << 32) | s1;
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t k = (sel >> (8 * i)) & 0xFFu;
    uint32_t b;
    if (k < 8) b = (uint32_t)(src >> (8 * k)) & 0xFFu;
    else if (k < 12) b = ((src >> (16 * (k - 8) + 15)) & 1u) ? 0xFFu : 0u;
    else b = k == 12 ? 0u : 0xFFu;
    r |= b << (8 * i);
  }
  return r;
#endif
}

// compiler scheduling barrier (device): no instruction moves across it
DA_HD void sched_fence() {
#if defined(__HIP_DEVICE_COMPILE__)
  __builtin_amdgcn_sched_barrier(0);
#endif
}

DA_HD int popc64(uint64_t x) { return __builtin_popcountll(x); }
DA_HD int ctz64(uint64_t x) { return __builtin_ctzll(x); }
DA_HD int clz64(uint64_t x) { return __builtin_clzll(x); }
// x + y + cin, returning the carry out of bit 63
DA_HD uint64_t add_carry(uint64_t x, uint64_t y, uint32_t cin, uint32_t *cout) {
  const uint64_t s = x + y;
  const uint64_t r = s + cin;
  *cout = (uint32_t)((s < x) | (r < s));
  return r;
}

template <typename T>
DA_HD T mn(T a, T b) { return a < b ? a : b; }
template <typename T>
DA_HD T mx(T a, T b) { return a < b ? b : a; }

DA_HD int ctz32(uint32_t x) { return __builtin_ctz(x); }
DA_HD int clz32(uint32_t x) { return __builtin_clz(x); }
DA_HD int popc32(uint32_t x) { return __builtin_popcount(x); }

}  // namespace dmlc_amd
