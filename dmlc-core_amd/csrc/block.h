// block.h -- the GPU block policy for the tile bodies: thread id, barrier,
// block-wide min and exclusive scan over wave64 shuffles + LDS.
#pragma once
#include "args.h"
#include "common.h"

namespace dmlc_amd {

// kSlot: bytes per scan slot in the LDS scratch -- the largest scan element
// the kernel uses (64 for the counter vectors of the exact kernels, 8 for the
// single-pass kernels, whose LDS budget is tight: fast_common.h kLdsBudget)
// NW: waves per workgroup (kWaves for the exact kernels; the single-pass
// kernels' kFastThreads / kWave, one by default -- then sync() is a wave-level
// ordering point and the scans stay in registers).
template <int kSlot, int NW = kWaves>
struct DevBlockT {
  static_assert(kSlot % 8 == 0 && kSlot >= 8, "8-byte granular slots");
  static constexpr int kSlotU64 = kSlot / 8;
  // LDS scratch: (NW + 1) slots of kSlot bytes
  uint64_t *scratch;

  __device__ __forceinline__ int tid() const { return threadIdx.x; }
  __device__ __forceinline__ void sync() const {
    if constexpr (NW == 1) {
      wave_sync();  // one wave: its LDS operations complete in order
    } else {
      __syncthreads();
    }
  }
  // wave-level: ballot over the 64 lanes, and an LDS-ordering point for a
  // protocol run by one wave (LDS ops of a wave complete in order; the fence
  // stops the compiler from moving LDS accesses across it)
  __device__ __forceinline__ uint64_t ballot(bool p) const { return __ballot(p); }
  __device__ __forceinline__ void wave_sync() const {
    __builtin_amdgcn_fence(__ATOMIC_ACQ_REL, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }

  // one word per wave (its lane 0's) for the whole block: wave_put, the
  // caller's sync(), then wave_get(w) in any thread (the scan scratch: no scan
  // may run between the put and the last get without a sync in between)
  __device__ __forceinline__ void wave_put(uint32_t v) const {
    if ((threadIdx.x & (kWave - 1)) == 0) scratch[threadIdx.x / kWave] = v;
  }
  __device__ __forceinline__ uint32_t wave_get(int w) const { return (uint32_t)scratch[w]; }

  // v of lane `src` of the calling wave (all lanes active)
  template <typename T>
  __device__ __forceinline__ static T shfl(T v, int src) {
    static_assert(sizeof(T) % 4 == 0, "4-byte granular");
    T o;
    const int *s = reinterpret_cast<const int *>(&v);
    int *d = reinterpret_cast<int *>(&o);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) d[k] = __shfl(s[k], src, kWave);
    return o;
  }

  // sum over the 64 lanes of the calling wave (all lanes active)
  __device__ __forceinline__ uint32_t wave_sum(uint32_t v) const {
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) v += __shfl_xor(v, d, kWave);
    return v;
  }

  template <typename T>
  __device__ __forceinline__ static T shfl_up(T v, int d) {
    static_assert(sizeof(T) % 4 == 0, "4-byte granular");
    T o;
    const int *src = reinterpret_cast<const int *>(&v);
    int *dst = reinterpret_cast<int *>(&o);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) dst[k] = __shfl_up(src[k], d, kWave);
    return o;
  }

  __device__ __forceinline__ uint64_t min_u64(uint64_t v) const {
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const uint64_t o = __shfl_xor(v, d, kWave);
      v = o < v ? o : v;
    }
    if (lane == 0) scratch[wid * kSlotU64] = v;
    __syncthreads();
    uint64_t r = scratch[0];
#pragma unroll
    for (int w = 1; w < NW; ++w) r = scratch[w * kSlotU64] < r ? scratch[w * kSlotU64] : r;
    __syncthreads();
    return r;
  }

  // inclusive prefix sum of 32-bit lanes over the wave by DPP (GFX9 forms:
  // row_shr inside rows of 16, then row_bcast:15 / row_bcast:31 across rows),
  // six VALU adds instead of six LDS permutes
  __device__ __forceinline__ static uint32_t wave_incl_add(uint32_t x) {
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, false);  // row_shr:1
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, false);  // row_shr:2
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, false);  // row_shr:4
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, false);  // row_shr:8
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);  // row_bcast:15
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);  // row_bcast:31
    return x;
  }
  // Exclusive prefix sum and block total of packed counters whose fields
  // never carry across bit 31 (the tiles' 16-bit role counts): two 32-bit
  // DPP wave scans, one LDS round for the wave totals.
  __device__ __forceinline__ uint64_t exclusive_add(uint64_t v, uint64_t *total) const {
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    const uint64_t inc = wave_incl_add((uint32_t)v) | ((uint64_t)wave_incl_add((uint32_t)(v >> 32)) << 32);
    if constexpr (NW == 1) {
      *total = shfl(inc, kWave - 1);
      (void)lane;
      (void)wid;
      return inc - v;
    }
    if (lane == kWave - 1) scratch[wid] = inc;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint64_t t = scratch[w];
      pre += w < wid ? t : 0;
      tot += t;
    }
    *total = tot;
    __syncthreads();
    return pre + inc - v;
  }

  // Exclusive prefix sum of packed counters (fields never carry across bit
  // 31) with one barrier, and the OR of a flag over the block: each wave's
  // total and flag go to wtot / wbad (caller's LDS, never rewritten before
  // the workgroup ends), every thread then reads all of them.
  // *wpre: the exclusive prefix at the wave's first lane.
  __device__ __forceinline__ uint64_t exclusive_add1(uint64_t v, bool flag, uint64_t *wtot, uint32_t *wbad,
                                                     uint64_t *total, uint64_t *wpre) const {
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    const uint64_t inc = wave_incl_add((uint32_t)v) | ((uint64_t)wave_incl_add((uint32_t)(v >> 32)) << 32);
    const uint64_t fm = __ballot(flag);
    if (lane == kWave - 1) {
      wtot[wid] = inc;
      wbad[wid] = fm != 0 ? 1u : 0u;
    }
    __syncthreads();
    uint64_t pre = 0, tot = 0;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const uint64_t t = wtot[w];
      pre += w < wid ? t : 0;
      tot += t;
    }
    *total = tot;
    *wpre = pre;
    return pre + inc - v;
  }

  // The same with one barrier: every wave reads all wave totals itself.  The
  // scratch slots stay read until the caller's next barrier, so a second
  // scan must not follow before one.
  template <typename T, typename Op>
  __device__ __forceinline__ T exclusive1(T v, T identity, Op op, T *total) const {
    static_assert(sizeof(T) <= kSlot, "scan element larger than the scratch slot");
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    T inc = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      T o = shfl_up(inc, d);
      if (lane >= d) inc = op(o, inc);
    }
    const T up = shfl_up(inc, 1);
    if constexpr (NW == 1) {
      *total = shfl(inc, kWave - 1);
      return lane == 0 ? identity : up;
    }
    T *sc = reinterpret_cast<T *>(scratch);
    if (lane == kWave - 1) *reinterpret_cast<T *>(reinterpret_cast<char *>(sc) + kSlot * wid) = inc;
    __syncthreads();
    T pre = identity, tot = identity;
#pragma unroll
    for (int w = 0; w < NW; ++w) {
      const T t = *reinterpret_cast<T *>(reinterpret_cast<char *>(sc) + kSlot * w);
      if (w < wid) pre = op(pre, t);
      tot = op(tot, t);
    }
    *total = tot;
    return lane == 0 ? pre : op(pre, up);
  }

  // Exclusive prefix (identity for thread 0) and the block total.
  template <typename T, typename Op>
  __device__ __forceinline__ T exclusive(T v, T identity, Op op, T *total) const {
    static_assert(sizeof(T) <= kSlot, "scan element larger than the scratch slot");
    T *sc = reinterpret_cast<T *>(scratch);
    const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
    T inc = v;
#pragma unroll
    for (int d = 1; d < kWave; d <<= 1) {
      T o = shfl_up(inc, d);
      if (lane >= d) inc = op(o, inc);
    }
    if constexpr (NW == 1) {  // the wave is the block
      *total = shfl(inc, kWave - 1);
      const T up = shfl_up(inc, 1);
      (void)sc;
      (void)wid;
      return lane == 0 ? identity : up;
    }
    T *slot = reinterpret_cast<T *>(reinterpret_cast<char *>(sc) + kSlot * wid);
    if (lane == kWave - 1) *slot = inc;
    __syncthreads();
    if (threadIdx.x == 0) {
      T acc = *reinterpret_cast<T *>(reinterpret_cast<char *>(sc));
      for (int w = 1; w < NW; ++w) {
        T *sw = reinterpret_cast<T *>(reinterpret_cast<char *>(sc) + kSlot * w);
        T t = *sw;
        *sw = acc;
        acc = op(acc, t);
      }
      *reinterpret_cast<T *>(reinterpret_cast<char *>(sc)) = identity;
      *reinterpret_cast<T *>(reinterpret_cast<char *>(sc) + kSlot * NW) = acc;
    }
    __syncthreads();
    const T up = shfl_up(inc, 1);
    const T wpre = *reinterpret_cast<T *>(reinterpret_cast<char *>(sc) + kSlot * wid);
    const T ex = lane == 0 ? wpre : op(wpre, up);
    *total = *reinterpret_cast<T *>(reinterpret_cast<char *>(sc) + kSlot * NW);
    __syncthreads();
    return ex;
  }
};

using DevBlock = DevBlockT<64>;
// the single-pass kernels: scan elements <= 8 bytes, kFastThreads per block
using DevBlockS = DevBlockT<8, kFastThreads / kWave>;

// LDS words the policies need
constexpr int kBlockScratchU64 = 8 * (kWaves + 1);
constexpr int kSmallScratchU64 = kFastThreads / kWave + 1;

}  // namespace dmlc_amd
