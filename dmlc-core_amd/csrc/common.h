// common.h -- device-side building blocks shared by the libsvm / CSV / libfm
// tile kernels: byte source over (LDS window | HBM), character classes, and
// 256-thread block scans.  gfx950 only (wave64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace dmlc_amd {

constexpr int kWave = 64;
constexpr int kThreads = 256;           // threads per tile workgroup (4 waves)
constexpr int kSeg = 32;                // bytes per thread per window
constexpr int kWin = kThreads * kSeg;   // 8 KiB window staged in LDS per step
constexpr int kWaves = kThreads / kWave;

// Counter slots carried through the tile scan (rows, index, value, weight, qid,
// label, field).  The same layout is used by the C-ABI result struct.
enum { C_ROWS = 0, C_INDEX, C_VALUE, C_WEIGHT, C_QID, C_LABEL, C_FIELD, C_N };

// Error codes (mirror the reference's fatal CHECKs; see include/dmlc_amd.h).
enum {
  E_OK = 0,
  E_NEG_INDEX = 1,      // strtonum.h:416 CHECK_EQ(sign, true)
  E_NAN_LITERAL = 2,    // strtonum.h:163 CHECK_EQ(*p, ')') "Invalid NAN literal"
  E_CSV_DELIM = 3,      // csv_parser.h:128-132 delimiter not found
  E_CAPACITY = 16,      // caller buffers too small (not a reference error)
  E_TIMEOUT = 17,
};

// ---------------------------------------------------------- char classes --
// dmlc::isspace (strtonum.h:27-29)
__host__ __device__ inline bool is_space(uint32_t c) {
  return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f';
}
__host__ __device__ inline bool is_blank(uint32_t c) { return c == ' ' || c == '\t'; }
__host__ __device__ inline bool is_digit(uint32_t c) { return c - '0' < 10u; }
__host__ __device__ inline bool is_alpha(uint32_t c) { return (c | 32u) - 'a' < 26u; }
// dmlc::isdigitchars (strtonum.h:70-72)
__host__ __device__ inline bool is_digitchar(uint32_t c) {
  return is_digit(c) || c == '+' || c == '-' || c == '.' || c == 'e' || c == 'E';
}
__host__ __device__ inline bool is_nl(uint32_t c) { return c == '\n' || c == '\r'; }
// glibc isspace, C locale (strtoll / atoll)
__host__ __device__ inline bool is_cspace(uint32_t c) { return c == ' ' || c - '\t' < 5u; }

// ----------------------------------------------------------- byte source --
// Reads text bytes at absolute positions.  Bytes inside the staged LDS window
// come from LDS, others from HBM (decoders that run past a window, or the
// rare read-ahead of ParseFloat/atoll).  Positions at or beyond `lim` (the end
// of the chunk being parsed) read as NUL, which is what the reference sees
// after a std::string and what the oracle restates.
struct Src {
  const uint8_t *g;
  uint64_t lim;
  const uint8_t *lds;  // LDS bytes for [wbase, wbase + wcap)
  uint64_t wbase, wend;
  __device__ __forceinline__ uint32_t operator()(uint64_t p) const {
    if (p >= lim) return 0u;
    if (p >= wbase && p < wend) return lds[p - wbase];
    return g[p];
  }
};

// ------------------------------------------------------------ block scan --
// Generic inclusive scan over a 256-thread block with a user combine
// (associative, not necessarily commutative).  T must be trivially copyable
// and <= 16 bytes; `scratch` holds kWaves+1 elements.
template <typename T, typename Op>
__device__ __forceinline__ T wave_inclusive(T v, Op op) {
  const int lane = threadIdx.x & (kWave - 1);
#pragma unroll
  for (int d = 1; d < kWave; d <<= 1) {
    T o;
    static_assert(sizeof(T) % 4 == 0, "scan type must be 4-byte granular");
    const int *src = reinterpret_cast<const int *>(&v);
    int *dst = reinterpret_cast<int *>(&o);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) dst[k] = __shfl_up(src[k], d, kWave);
    if (lane >= d) v = op(o, v);
  }
  return v;
}

// Returns the exclusive prefix for this thread (identity for thread 0) and
// the block total in *total.  Two barriers.
template <typename T, typename Op>
__device__ __forceinline__ T block_exclusive(T v, T identity, Op op, T *scratch, T *total) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
  T inc = wave_inclusive(v, op);
  if (lane == kWave - 1) scratch[wid] = inc;
  __syncthreads();
  if (threadIdx.x == 0) {
    T acc = scratch[0];
    for (int w = 1; w < kWaves; ++w) {
      T t = scratch[w];
      scratch[w] = acc;
      acc = op(acc, t);
    }
    scratch[0] = identity;
    scratch[kWaves] = acc;
  }
  __syncthreads();
  // exclusive within wave
  T up;
  {
    const int *src = reinterpret_cast<const int *>(&inc);
    int *dst = reinterpret_cast<int *>(&up);
#pragma unroll
    for (int k = 0; k < (int)(sizeof(T) / 4); ++k) dst[k] = __shfl_up(src[k], 1, kWave);
  }
  T wpre = scratch[wid];
  T ex = lane == 0 ? wpre : op(wpre, up);
  *total = scratch[kWaves];
  __syncthreads();  // scratch reusable after return
  return ex;
}

template <typename T>
__device__ __forceinline__ T block_min(T v, T *scratch) {
  const int lane = threadIdx.x & (kWave - 1), wid = threadIdx.x / kWave;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    T o = __shfl_xor(v, d, kWave);
    v = o < v ? o : v;
  }
  if (lane == 0) scratch[wid] = v;
  __syncthreads();
  T r = scratch[0];
#pragma unroll
  for (int w = 1; w < kWaves; ++w) r = scratch[w] < r ? scratch[w] : r;
  __syncthreads();
  return r;
}

// Counter vector (8 x u32) for per-window scans.
struct Cnt {
  uint32_t c[8];
};
struct CntAdd {
  __device__ Cnt operator()(const Cnt &a, const Cnt &b) const {
    Cnt r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r.c[i] = a.c[i] + b.c[i];
    return r;
  }
};

// Record the first (lowest position) error.
__device__ inline void raise_error(unsigned long long *err, uint32_t code, uint64_t pos) {
  // packed: position (48 bits) | code (16 bits); lower position wins
  unsigned long long v = ((unsigned long long)(pos & 0xFFFFFFFFFFFFull) << 16) | code;
  atomicMin(err, v);
}

// Chunk containing position p (chunk_start is sorted, nchunk+1 entries).
__device__ inline int chunk_of(const uint64_t *cs, int nchunk, uint64_t p) {
  int lo = 0, hi = nchunk;  // invariant cs[lo] <= p < cs[hi]
  while (hi - lo > 1) {
    int mid = (lo + hi) >> 1;
    if (cs[mid] <= p) lo = mid;
    else hi = mid;
  }
  return lo;
}

}  // namespace dmlc_amd
