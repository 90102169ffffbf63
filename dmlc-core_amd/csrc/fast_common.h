// fast_common.h -- pieces shared by the single-pass uniform-grammar kernels
// (svm_fast.h for libsvm, csv_fast.h for CSV): tile geometry, the byte-class
// tables, SWAR number decoders, LDS staging, the chunk list of a tile and the
// decoupled look-back.  Compiles as HIP device code and as plain C++ (test
// emulator, tests/emu).
#pragma once
#include "args.h"
#include "decode.h"

namespace dmlc_amd {
namespace fast {

constexpr int kSegB = 64;                // bytes per thread (one 64-bit mask)
constexpr int kTile = kThreads * kSegB;  // 16 KiB of text per tile
constexpr int kPre = 64;                 // staged bytes before the tile (look-back)
constexpr int kPost = 128;               // staged bytes after it (runs crossing the end)
constexpr int kStage = kPre + kTile + kPost;
constexpr int kMaxCs = 32;               // chunk starts per tile the fast path accepts
constexpr uint64_t kAgg = 1ull << 62, kIncl = 2ull << 62, kValMask = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 26;

// Diagnostic build only (-DDMLC_AMD_STAMPS, libdmlc_amd_stamps.so): thread 0
// of each tile records s_memtime at phase boundaries into g_stamps; the
// product build executes no stamp.
constexpr uint32_t kStampTiles = 1u << 17;
#if defined(DMLC_AMD_STAMPS) && defined(__HIPCC__)
__device__ uint64_t g_stamps[kStampTiles * 8];
#endif
#if defined(DMLC_AMD_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
#define FAST_STAMP(k, i)                                                         \
  do {                                                                           \
    if (tid == 0 && (k) < kStampTiles) {                                         \
      __builtin_amdgcn_sched_barrier(0);                                         \
      g_stamps[(uint64_t)(k) * 8 + (i)] =                                        \
          (i) == 0 ? __builtin_amdgcn_s_memrealtime() : __builtin_amdgcn_s_memtime(); \
      __builtin_amdgcn_sched_barrier(0);                                         \
    }                                                                            \
  } while (0)
#else
#define FAST_STAMP(k, i) \
  do {                   \
  } while (0)
#endif

// Byte classes by two 16-entry nibble tables (v_perm_b32 lookups): cls =
// LO[b & 15] & HI[b >> 4]; bits 0-2 digitchar (strtonum.h:70-72: 0-9, then
// + - ., then e E), bit 3 ':', bit 4 '\n' '\r', bits 5-6 ' ' '\t'
// (strtonum.h:37-39).  A zero class is a byte outside the grammar.
constexpr uint32_t kLoA = 0x01010121u, kLoB = 0x01010501u;  // LO[0..7]
constexpr uint32_t kLoC = 0x02184101u, kLoD = 0x00021200u;  // LO[8..15]
constexpr uint32_t kHiA = 0x09220050u, kHiB = 0x00040004u;  // HI[0..7]

struct Masks {
  uint64_t d, n, c;
  uint32_t bad;
};

DA_HD uint32_t nib_d(uint32_t cls) {  // digitchar byte flags -> 4 bits
  return ((((cls & 0x07070707u) + 0x7F7F7F7Fu) & 0x80808080u) * 0x00204081u) >> 28;
}
DA_HD uint32_t nib_n(uint32_t cls) { return ((cls & 0x10101010u) * 0x01020408u) >> 28; }
DA_HD uint32_t nib_c(uint32_t cls) { return ((cls & 0x08080808u) * 0x02040810u) >> 28; }

DA_HD uint32_t classify4(uint32_t x) {
  const uint32_t lo = x & 0x0F0F0F0Fu, s = lo & 0x07070707u;
  const uint32_t a = perm_b32(kLoB, kLoA, s), b = perm_b32(kLoD, kLoC, s);
  const uint32_t m8 = ((lo >> 3) & 0x01010101u) * 0xFFu;
  const uint32_t lov = (b & m8) | (a & ~m8);
  const uint32_t hv = perm_b32(kHiB, kHiA, (x >> 4) & 0x07070707u);
  return lov & hv;
}

DA_HD void load16(const uint8_t *p, uint32_t w[4]) {
#if defined(__HIP_DEVICE_COMPILE__)
  const uint4 v = *reinterpret_cast<const uint4 *>(p);
  w[0] = v.x;
  w[1] = v.y;
  w[2] = v.z;
  w[3] = v.w;
#else
  memcpy(w, p, 16);
#endif
}

struct Nib {
  uint32_t d, n, c, bad;
};
DA_HD Nib classify_dword(uint32_t x) {  // 4-bit masks of 4 bytes; bad: a byte outside the grammar
  const uint32_t cls = classify4(x);
  Nib r;
  r.d = nib_d(cls);
  r.n = nib_n(cls);
  r.c = nib_c(cls);
  r.bad = ((cls + 0x7F7F7F7Fu) & 0x80808080u) != 0x80808080u || (x & 0x80808080u);
  return r;
}

// Masks of the 64 bytes at p (16-byte aligned).  Bytes past the end of the
// text are staged as blanks, so they are neutral here.
DA_HD Masks classify64(const uint8_t *p) {
  uint32_t dl = 0, dh = 0, nl = 0, nh = 0, cl = 0, ch = 0;
  uint32_t all = 0x80808080u, orv = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t w[4];
    load16(p + 16 * q, w);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * q + j;
      const uint32_t x = w[j];
      const uint32_t cls = classify4(x);
      all &= cls + 0x7F7F7F7Fu;
      orv |= x;
      const int sh = 4 * (i & 7);
      if (i < 8) {
        dl |= nib_d(cls) << sh;
        nl |= nib_n(cls) << sh;
        cl |= nib_c(cls) << sh;
      } else {
        dh |= nib_d(cls) << sh;
        nh |= nib_n(cls) << sh;
        ch |= nib_c(cls) << sh;
      }
    }
  }
  Masks m;
  m.d = dl | ((uint64_t)dh << 32);
  m.n = nl | ((uint64_t)nh << 32);
  m.c = cl | ((uint64_t)ch << 32);
  m.bad = ((all & 0x80808080u) != 0x80808080u) || (orv & 0x80808080u);
  return m;
}

struct AddU64 {
  DA_HD uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
};

// ---- SWAR decoders on the first 16 bytes of a run (read from the staged LDS
// text with five aligned words).  Digits are located with byte-parallel masks
// and converted eight at a time (multiply-shift 8-digit conversion), then
// combined with exactly the reference's arithmetic.

DA_HD uint32_t funnel(uint32_t hi, uint32_t lo, uint32_t sft) {  // ((hi:lo) >> sft), sft < 32
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(hi, lo, sft);
#else
  return (uint32_t)((((uint64_t)hi << 32) | lo) >> sft);
#endif
}

DA_HD uint32_t nondigit8(uint64_t x) {  // bit i: byte i is not '0'..'9' (grammar bytes < 0x80)
  const uint64_t t = x ^ 0x3030303030303030ull;
  const uint64_t h = ((t + 0x7676767676767676ull) & 0x8080808080808080ull) >> 7;
  return (uint32_t)((h * 0x0102040810204080ull) >> 56);
}

DA_HD uint64_t parse8(uint64_t w) {  // 8 ASCII digits, first char in the low byte
  w = ((w & 0x0F0F0F0F0F0F0F0Full) * 2561ull) >> 8;
  w = ((w & 0x00FF00FF00FF00FFull) * 6553601ull) >> 16;
  return ((w & 0x0000FFFF0000FFFFull) * 42949672960001ull) >> 32;
}

struct W16 {
  uint64_t lo, hi;  // window bytes 0..7, 8..15
  DA_HD uint32_t byte(uint32_t p) const {
    return (uint32_t)((p < 8 ? lo >> (8 * p) : hi >> (8 * (p - 8))) & 0xFFu);
  }
  DA_HD uint64_t at(uint32_t a) const {  // bytes a .. a+7 (zero beyond the window)
    if (a == 0) return lo;
    if (a < 8) return (lo >> (8 * a)) | (hi << (64 - 8 * a));
    return a < 16 ? hi >> (8 * (a - 8)) : 0;
  }
  DA_HD uint64_t span8(uint32_t a, uint32_t len) const {  // value of len <= 8 digits at a
    if (len == 0) return 0;
    uint64_t w = at(a) << (8 * (8 - len));
    if (len < 8) w |= 0x3030303030303030ull >> (8 * len);
    return parse8(w);
  }
  DA_HD uint64_t span16(uint32_t a, uint32_t len) const {  // len <= 16
    return len <= 8 ? span8(a, len) : span8(a, len - 8) * 100000000ull + span8(a + len - 8, 8);
  }
  DA_HD uint32_t digits() const { return ~(nondigit8(lo) | (nondigit8(hi) << 8)) & 0xFFFFu; }
};

DA_HD uint32_t run_len(uint32_t dm, uint32_t a) {  // consecutive digits from byte a
  return a >= 16 ? 0 : (uint32_t)ctz32(~(dm >> a));
}

DA_HD double pow10_exact(uint32_t k) {  // 10^k as a double, exact for k <= 22
  double p = 1.0;
  if (k & 1u) p *= 10.0;
  if (k & 2u) p *= 100.0;
  if (k & 4u) p *= 1e4;
  if (k & 8u) p *= 1e8;
  if (k & 16u) p *= 1e16;
  return p;
}

// ParseFloat<float> (strtonum.h:95-264) restated for a run of the uniform
// grammar -- inf / nan / the 'f' suffix need letters outside it -- with the
// reference's operations: u64 integer part, f32 conversion, one f64 division
// of the (<= 19-digit) fraction, f32 add, f32 exponent scaling.
// *ok = false when the number may continue past the window (caller falls back).
DA_HD float wfloat(const W16 &w, bool *ok) {
  const uint32_t dm = w.digits();
  const uint32_t b0 = w.byte(0);
  const bool sign = b0 != '-';
  const uint32_t s = (b0 == '-' || b0 == '+') ? 1u : 0u;
  const uint32_t il = run_len(dm, s);
  uint32_t p = s + il;
  *ok = false;
  if (p >= 16) return 0.f;
  float value = (float)w.span16(s, il);
  uint32_t c = w.byte(p);
  if (c == '.') {
    const uint32_t fs = p + 1;
    const uint32_t fl = run_len(dm, fs);
    p = fs + fl;
    if (p >= 16) return 0.f;
    value += (float)((double)w.span16(fs, fl) / pow10_exact(fl));
    c = w.byte(p);
  }
  if (c == 'e' || c == 'E') {
    bool frac = false;
    float scale = 1.0f;
    if (++p >= 16) return 0.f;
    c = w.byte(p);
    if (c == '-' || c == '+') {
      frac = c == '-';
      if (++p >= 16) return 0.f;
      c = w.byte(p);
    }
    uint32_t expon = 0;
    for (; is_digit(c); c = w.byte(p)) {
      expon = expon * 10u + (c - '0');
      if (++p >= 16) return 0.f;
    }
    if (expon > 38u) expon = 38u;
    const float kMaxSig = (float)3.402823466, kMaxSigNeg = (float)1.175494351;
    if (expon == 38u && ((!frac && value > kMaxSig) || (frac && value < kMaxSigNeg)))
      value = frac ? kMaxSigNeg : kMaxSig;
    while (expon >= 8u) {
      scale *= 1E8f;
      expon -= 8u;
    }
    while (expon > 0u) {
      scale *= 10.0f;
      expon -= 1u;
    }
    value = frac ? (value / scale) : (value * scale);
  }
  *ok = true;
  return sign ? value : -value;
}

// ParseUnsignedInt (strtonum.h:392-428) on a run (no leading blanks there):
// false on a leading '-' (the reference's fatal CHECK).  Up to 16 digits the
// exact value truncated to the index width equals the reference's wrapping
// accumulation.
DA_HD bool wuint(const W16 &w, bool wide, uint64_t *out, bool *ok) {
  const uint32_t b0 = w.byte(0);
  *ok = true;
  if (b0 == '-') return false;
  const uint32_t s = b0 == '+' ? 1u : 0u;
  const uint32_t il = run_len(w.digits(), s);
  if (s + il >= 16) {
    *ok = false;
    return true;
  }
  const uint64_t v = w.span16(s, il);
  *out = wide ? v : (uint64_t)(uint32_t)v;
  return true;
}

// the 16 bytes at absolute position q (staged in LDS at `text`, which holds
// position tlo - kPre at index 0; q < tile end) as a window
DA_HD W16 win_at(const uint8_t *text, uint64_t tlo, uint64_t q) {
  const uint32_t off = (uint32_t)(q - tlo) + kPre;
  const uint32_t *w = reinterpret_cast<const uint32_t *>(text + (off & ~3u));
  const uint32_t sft = (off & 3u) * 8u;
  const uint32_t x0 = w[0], x1 = w[1], x2 = w[2], x3 = w[3], x4 = w[4];
  W16 r;
  r.lo = funnel(x1, x0, sft) | ((uint64_t)funnel(x2, x1, sft) << 32);
  r.hi = funnel(x3, x2, sft) | ((uint64_t)funnel(x4, x3, sft) << 32);
  return r;
}

// ---- per-tile state every fast kernel keeps in LDS
struct TileCommon {
  alignas(16) uint8_t text[kStage];  // position p <-> text[p - tlo + kPre]
  uint64_t csl[kMaxCs + 1];           // chunk starts in [tlo, thi]
  uint64_t cfloor, cnext, base[4];    // last chunk start <= tlo, first beyond the list, output bases
  uint64_t lbw[4 * kWave];            // look-back round: values per lane and counter
  uint32_t ncs, c_first, tile, toomany, bad;
};

// Thread 0: the chunk starts touching [tlo, thi] (binary search once).
DA_HD void chunk_list(const uint64_t *cs, int nchunk, uint64_t tlo, uint64_t thi, TileCommon &c) {
  const int c0 = chunk_of(cs, nchunk, tlo);
  c.cfloor = cs[c0];
  int i = c0;
  if (cs[i] < tlo) ++i;
  c.c_first = (uint32_t)i;
  uint32_t m = 0;
  while (i < nchunk && cs[i] <= thi) {
    if (m < kMaxCs) c.csl[m] = cs[i];
    ++m;
    ++i;
  }
  c.ncs = m < kMaxCs ? m : kMaxCs;
  c.cnext = cs[i];  // cs[nchunk] == n
  c.toomany = m > kMaxCs;
  c.bad = 0;
}

// All threads: stage [tlo - kPre, tlo + kTile + kPost) into LDS with 16-byte
// loads; bytes past the end of the text become blanks (neutral to every
// classifier, never decoded).  The caller synchronises.
template <class BK>
DA_HDF void stage(const uint8_t *text, uint64_t n, uint64_t tlo, TileCommon &c, BK &bk) {
  const uint64_t s0 = tlo >= (uint64_t)kPre ? tlo - kPre : 0;
  const uint64_t s1 = tlo + kTile + kPost;
  uint8_t *dst = c.text + (s0 + kPre - tlo);
  const uint64_t nunits = (s1 - s0) >> 4;
  for (uint64_t u = bk.tid(); u < nunits; u += kThreads) {
    const uint64_t g = s0 + (u << 4);
    uint32_t w[4];
    if (g + 16 <= n) {
      load16(text + g, w);
    } else {
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        uint32_t x = 0;
#pragma unroll
        for (int b = 0; b < 4; ++b) {
          const uint64_t pos = g + 4 * q + b;
          x |= (uint32_t)(pos < n ? text[pos] : (uint8_t)' ') << (8 * b);
        }
        w[q] = x;
      }
    }
    memcpy(dst + (u << 4), w, 16);
  }
}

// Lanes 0..3: publish this tile's aggregate (record words 0-3; the inclusive
// prefix later goes to words 4-7, so a reader never mixes the two).
DA_HD void publish_aggregate(uint64_t *lb, uint32_t k, int lane, uint64_t agg) {
  uint64_t *rec = lb + (uint64_t)k * 8;
  if (k == 0) store_agent_u64(rec + 4 + lane, kIncl | agg);
  else store_agent_u64(rec + lane, kAgg | agg);
}

// Wave 0: decoupled look-back.  Lane i reads predecessor j-1-i's record; a
// round consumes predecessors up to the first inclusive one and stops before
// the first unpublished one.  Lanes 0..3 end with c.base[lane] = exclusive
// prefix of counter `lane` and publish the inclusive prefix (agg = this
// tile's count).  Returns the number of rounds.  The caller synchronises.
template <class BK>
DA_HDF uint32_t look_back(uint64_t *lb, uint32_t k, uint64_t agg, uint32_t *gate, TileCommon &c,
                          BK &bk) {
  const uint32_t lane = bk.tid();
  uint64_t j = k;
  uint32_t spins = 0, rounds = 0;
  uint64_t acc = 0;  // lane c < 4: counter c
  bool done = k == 0;
  while (!done) {
    ++rounds;
    uint64_t v0 = 0, v1 = 0, v2 = 0, v3 = 0;
    uint32_t st = 2;  // before tile 0: an inclusive 0
    if (lane < j) {
      uint64_t *rec = lb + (j - 1 - lane) * 8;
      // all eight words in one round trip
      const uint64_t a0 = load_agent_u64(rec + 0), a1 = load_agent_u64(rec + 1),
                     a2 = load_agent_u64(rec + 2), a3 = load_agent_u64(rec + 3),
                     i0 = load_agent_u64(rec + 4), i1 = load_agent_u64(rec + 5),
                     i2 = load_agent_u64(rec + 6), i3 = load_agent_u64(rec + 7);
      const bool inc = (i0 & i1 & i2 & i3) >> 63;
      v0 = inc ? i0 : a0;
      v1 = inc ? i1 : a1;
      v2 = inc ? i2 : a2;
      v3 = inc ? i3 : a3;
      st = inc ? 2 : ((a0 & a1 & a2 & a3) >> 62 ? 1 : 0);
    }
    const uint64_t zero = bk.ballot(st == 0), incl = bk.ballot(st == 2);
    const uint32_t fz = zero ? (uint32_t)ctz64(zero) : 64u, fi = incl ? (uint32_t)ctz64(incl) : 64u;
    const uint32_t take = fi < fz ? fi + 1 : fz;
    const bool use = lane < take;
    c.lbw[4 * lane + 0] = use ? v0 & kValMask : 0;
    c.lbw[4 * lane + 1] = use ? v1 & kValMask : 0;
    c.lbw[4 * lane + 2] = use ? v2 & kValMask : 0;
    c.lbw[4 * lane + 3] = use ? v3 & kValMask : 0;
    bk.wave_sync();
    if (lane < 4)
      for (uint32_t i = 0; i < take; ++i) acc += c.lbw[4 * i + lane];
    bk.wave_sync();
    j -= take;
    done = fi < fz;
    if (!done && take == 0) {
      if (++spins > kSpinLimit) {  // never expected: hand the input to the exact path
        if (lane == 0) atomic_or_u32(gate, 2u);
        done = true;
      }
      spin_pause();
    }
  }
  if (lane < 4) {
    if (k > 0) store_agent_u64(lb + (uint64_t)k * 8 + 4 + lane, kIncl | (acc + agg));
    c.base[lane] = acc;
  }
  return rounds;
}

}  // namespace fast
}  // namespace dmlc_amd
