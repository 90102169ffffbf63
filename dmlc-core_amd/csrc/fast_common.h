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

// Tile geometry: kFThreads threads (args.h kFastThreads), 64 text bytes each.
constexpr int kFThreads = kFastThreads;
constexpr int kFWaves = kFThreads / kWave;
static_assert(kFThreads % kWave == 0 && (kFWaves == 1 || kFWaves == 2 || kFWaves == 4 || kFWaves == 6 || kFWaves == 8),
              "whole waves: 1, 2, 4, 6 or 8");

// LDS of one single-pass workgroup.  gfx950 allocates LDS in 1280-byte
// granules (160 KiB / 128): at four waves per tile, 6 workgroups per CU fit
// 21 granules each (26,880 bytes), one byte more and the launch dropped to 5
// per CU (+32 bytes took svm_fast_tile from 1.84 to 2.04 ms); a one-wave
// tile gets 6 granules (7,680 bytes: 21 workgroups per CU); six- and eight-wave
// tiles (24 / 32 KiB of text) get 4 and 3 workgroups per CU: 32 and 42 granules.
constexpr int kLdsGranule = 1280;
constexpr int kLdsBudget =
    (kFWaves == 1 ? 6 : kFWaves == 2 ? 11 : kFWaves == 4 ? 21 : kFWaves == 6 ? 32 : 42) * kLdsGranule;

constexpr int kSegB = 64;                 // bytes per thread (one 64-bit mask)
constexpr int kTile = kFThreads * kSegB;  // text per tile (4 KiB at one wave)
constexpr int kPre = 64;                  // staged bytes before the tile (the segment before it)
// (staging 80 bytes before the tile instead -- 16 more for the qid token
// checks -- cost 11 % on the 1M x 128 libsvm launch: those read global memory)
constexpr int kPost = kFWaves == 1 ? 64 : 128;  // staged bytes after it (runs crossing the end)
constexpr int kStage = kPre + kTile + kPost;
constexpr int kMaxCs = kFastMaxCs;       // chunk starts per tile the fast path accepts (args.h)
constexpr uint64_t kAgg = 1ull << 62, kIncl = 2ull << 62, kValMask = (1ull << 62) - 1;
// look-back rounds without progress before a tile gives up and hands the
// input to the exact kernels (never expected: a safety valve that bounds the
// wait should a predecessor tile not be resident, see svm_fast.h tile order)
constexpr uint32_t kSpinLimit = 1u << 22;

// Diagnostic build only (-DDMLC_AMD_STAMPS, libdmlc_amd_stamps.so): thread 0
// of each tile records s_memtime at phase boundaries into g_stamps; the
// product build executes no stamp.
constexpr uint32_t kStampTiles = 1u << 17;
constexpr uint32_t kStampSlots = 20;  // per tile: 0 realtime start, 1.. phase ends, 15 look-back rounds
#if defined(DMLC_AMD_STAMPS) && defined(__HIPCC__)
__device__ uint64_t g_stamps[kStampTiles * kStampSlots];
#endif
#if defined(DMLC_AMD_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
#define FAST_STAMP(k, i)                                                         \
  do {                                                                           \
    if (tid == 0 && (k) < kStampTiles) {                                         \
      __builtin_amdgcn_sched_barrier(0);                                         \
      g_stamps[(uint64_t)(k) * kStampSlots + (i)] =                                        \
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
  uint64_t g;   // table form: byte-1 plane (G digit for libsvm, outside-the-grammar for CSV)
  uint32_t hi;  // table form: a byte >= 0x80 among the 64 (its planes are not the table's)
};

// The class tables hold all 256 byte values (1 KiB of LDS per tile): a byte
// >= 0x80 has its own class (outside the grammar; CSV's junk), so the table
// body needs no per-byte range check.  (Round 4 tried 128 entries -- 512 B
// less LDS -- with the bytes >= 0x80 patched afterwards: the OR of the
// words that finds them cost the libfm kernel 7 spilled VGPRs, and the
// out-of-table reads leaked into neighbouring bytes' planes.)
constexpr int kClsEntries = 256;
DA_HD uint32_t cls_index(uint32_t b) { return b & 0xFFu; }
// bit i: byte i of the 64 at p (16-byte aligned) is >= 0x80 (rare: a slow loop)
DA_HD uint64_t hi_mask64(const uint8_t *p) {
  uint64_t m = 0;
  for (int i = 0; i < 64; ++i) m |= (uint64_t)(p[i] >> 7) << i;
  return m;
}
DA_HD uint32_t hi_nib4(uint32_t x) { return (((x >> 3) & 0x10101010u) * 0x01020408u) >> 28; }  // bytes >= 0x80

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
  uint32_t d, n, c, bad, g, hi;
};
DA_HD Nib classify_dword(uint32_t x) {  // 4-bit masks of 4 bytes; bad: a byte outside the grammar
  const uint32_t cls = classify4(x);
  Nib r;
  r.d = nib_d(cls);
  r.n = nib_n(cls);
  r.c = nib_c(cls);
  r.bad = ((cls + 0x7F7F7F7Fu) & 0x80808080u) != 0x80808080u || (x & 0x80808080u);
  r.g = 0;
  r.hi = hi_nib4(x);
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
  m.g = 0;
  m.hi = (orv & 0x80808080u) != 0u;
  return m;
}

// ---- byte classes by table lookup (the VALU-cheap form on MI355X: one SDWA
// shift + one shift-or per byte, the lookup on the LDS pipe).  Entry planes:
// byte 0 D digitchar, 1 G digit, 2 N newline, 3 C colon; blanks are 0; a byte
// outside the grammar is G without D.  The letters of "qid:" (libsvm only,
// libsvm_parser.h:119-132) are N and C together, which no other byte is:
// svm_fast.h qid_clean turns them into blanks and the token's ':' into a
// qid marker (N and C) or flags them.
DA_HD uint32_t class_of(uint32_t b) {
  if (b - '0' < 10u) return 0x00000101u;
  if (b == '+' || b == '-' || b == '.' || b == 'e' || b == 'E') return 0x00000001u;
  if (b == '\n' || b == '\r') return 0x00010000u;
  if (b == ':') return 0x01000000u;
  if (b == ' ' || b == '\t') return 0u;
  if (b == 'q' || b == 'i' || b == 'd') return 0x01010000u;
  return 0x00000100u;
}

// Masks of the 64 bytes at p (16-byte aligned) through the class table.
DA_HD Masks classify64_lut(const uint8_t *p, const uint32_t *cls) {
  uint32_t acc[8];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t w[4];
    load16(p + 16 * q, w);
#pragma unroll
    for (int j = 0; j < 4; ++j)
#pragma unroll
      for (int b = 0; b < 4; ++b) {
        const int i = 16 * q + 4 * j + b;
        const uint32_t x = cls[cls_index((w[j] >> (8 * b)) & 0xFFu)];
        if ((i & 7) == 0) acc[i >> 3] = x;
        else acc[i >> 3] |= x << (i & 7);
      }
  }
  // byte p of acc[j] = plane p of bytes 8j..8j+7: gather plane bytes
  uint32_t pd[2], pg[2], pn[2], pc[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t t = perm_b32(acc[4 * h + 1], acc[4 * h], 0x05010400u);
    const uint32_t u = perm_b32(acc[4 * h + 3], acc[4 * h + 2], 0x05010400u);
    pd[h] = perm_b32(u, t, 0x05040100u);
    pg[h] = perm_b32(u, t, 0x07060302u);
    const uint32_t t2 = perm_b32(acc[4 * h + 1], acc[4 * h], 0x07030602u);
    const uint32_t u2 = perm_b32(acc[4 * h + 3], acc[4 * h + 2], 0x07030602u);
    pn[h] = perm_b32(u2, t2, 0x05040100u);
    pc[h] = perm_b32(u2, t2, 0x07060302u);
  }
  Masks m;
  m.d = pd[0] | ((uint64_t)pd[1] << 32);
  m.n = pn[0] | ((uint64_t)pn[1] << 32);
  m.c = pc[0] | ((uint64_t)pc[1] << 32);
  const uint64_t g = pg[0] | ((uint64_t)pg[1] << 32);
  m.g = g;
  m.hi = 0u;  // (the table classes bytes >= 0x80 itself)
  m.bad = (g & ~m.d) != 0;
  return m;
}
// ---- The same masks in registers (A/B build FSVM_REGCLS): eight one-bit
// classes from two nibble tables by v_perm (digit, + - ., e E, ':', newline,
// space, tab, and the letters a d i q t y, which qid_clean checks against
// "qid:" as the table's N+C letters), then per plane a flag bit per byte
// gathered four at a time by one multiply and shifted in by v_alignbit.
constexpr uint32_t kRLoA = 0x01018121u, kRLoB = 0x01010581u, kRLoC = 0x0218C101u, kRLoD = 0x00021200u;
constexpr uint32_t kRHiA = 0x09220050u, kRHiB = 0x80840004u;
DA_HD uint32_t rcls4(uint32_t x) {  // one class bit per byte (0: outside the grammar)
  const uint32_t s = x & 0x07070707u;
  const uint32_t a = perm_b32(kRLoB, kRLoA, s), b = perm_b32(kRLoD, kRLoC, s);
  const uint32_t m = perm_b32(0xFFFFFFFFu, 0u, (x >> 1) & 0x04040404u);  // 0xFF where the low nibble >= 8
  const uint32_t hv = perm_b32(kRHiB, kRHiA, (x >> 4) & 0x07070707u);
  return ((b & m) | (a & ~m)) & hv;
}
DA_HD uint32_t gather_in(uint32_t acc, uint32_t f, uint32_t mul) {  // acc << 4 | the 4 flags (one bit per byte)
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_alignbit(acc, f * mul, 28u);
#else
  return (acc << 4) | ((f * mul) >> 28);
#endif
}
DA_HD Masks classify64_reg(const uint8_t *p) {
  uint32_t d[2] = {0, 0}, g[2] = {0, 0}, n[2] = {0, 0}, c[2] = {0, 0};
  uint32_t all = 0x80808080u, orv = 0;
#pragma unroll
  for (int q = 3; q >= 0; --q) {  // last dword first: each gather shifts the earlier ones up
    uint32_t w[4];
    load16(p + 16 * q, w);
#pragma unroll
    for (int j = 3; j >= 0; --j) {
      const int h = q >> 1;
      const uint32_t x = w[j], cls = rcls4(x);
      all &= cls + 0x7F7F7F7Fu;
      orv |= x;
      g[h] = gather_in(g[h], cls & 0x01010101u, 0x10204080u);
      d[h] = gather_in(d[h], ((cls & 0x07070707u) + 0x03030303u) & 0x04040404u, 0x04081020u);
      n[h] = gather_in(n[h], ((cls & 0x90909090u) + 0x70707070u) & 0x80808080u, 0x00204081u);
      c[h] = gather_in(c[h], ((cls & 0x88888888u) + 0x78787878u) & 0x80808080u, 0x00204081u);
    }
  }
  Masks m;
  m.d = d[0] | ((uint64_t)d[1] << 32);
  m.g = g[0] | ((uint64_t)g[1] << 32);
  m.n = n[0] | ((uint64_t)n[1] << 32);
  m.c = c[0] | ((uint64_t)c[1] << 32);
  m.hi = 0u;
  m.bad = ((all & 0x80808080u) != 0x80808080u) || (orv & 0x80808080u);
  return m;
}

// 4 bytes (x) through the table: 4-bit masks (a byte >= 0x80: r.hi, planes
// cleared, bad; its table word is masked to the plane bits so that it cannot
// reach the other bytes' planes)
DA_HD Nib classify_dword_lut(uint32_t x, const uint32_t *cls) {
  uint32_t acc = 0;
#pragma unroll
  for (int b = 0; b < 4; ++b) acc |= (cls[cls_index((x >> (8 * b)) & 0xFFu)] & 0x01010101u) << b;
  const uint32_t h = hi_nib4(x), k = ~h & 0xFu;
  Nib r;
  r.d = acc & k;
  r.n = (acc >> 16) & k;
  r.c = (acc >> 24) & k;
  r.g = (acc >> 8) & k;
  r.bad = (r.g & ~r.d) != 0 || h != 0;
  r.hi = h;
  return r;
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

// ---- 32-bit decoders (MI355X: v_dot4_u32_u8, 32-bit mul and perm are full
// rate; 64-bit multiplies and the f64 divide sequence are not)
struct DecTables {
  double p10[16], i10[16];  // 10^k and RN(10^-k)
  uint64_t hib[9];          // 0x0F in bytes >= k of 8 (k <= 8): the fraction's byte masks
};
// The tables as compile-time constants (constant evaluation divides with
// IEEE round-to-nearest, so i10[k] is the correctly rounded 10^-k); each tile
// copies them to LDS with one load per lane instead of computing them.
constexpr DecTables make_dec_tables() {
  DecTables t{};
  double p = 1.0;
  for (int k = 0; k < 16; ++k) {
    t.p10[k] = p;
    t.i10[k] = 1.0 / p;
    p *= 10.0;
  }
  for (int k = 0; k <= 8; ++k) {
    uint64_t m = 0;
    for (int b = k; b < 8; ++b) m |= 0x0Full << (8 * b);
    t.hib[k] = m;
  }
  return t;
}
constexpr DecTables kDecTables = make_dec_tables();
template <class BK>
DA_HDF void init_dec_tables(DecTables &tb, BK &bk) {
  const int t = bk.tid();
  if (t < 16) {
    tb.p10[t] = kDecTables.p10[t];
    tb.i10[t] = kDecTables.i10[t];
  } else if (t < 25) {
    tb.hib[t - 16] = kDecTables.hib[t - 16];
  }
}
DA_HD uint32_t udot4(uint32_t a, uint32_t b, uint32_t c) {  // sum of the 4 byte products + c
#if defined(__HIP_DEVICE_COMPILE__)
  return __builtin_amdgcn_udot4(a, b, c, false);
#else
  for (int i = 0; i < 4; ++i) c += ((a >> (8 * i)) & 0xFFu) * ((b >> (8 * i)) & 0xFFu);
  return c;
#endif
}
// acc * 10^4 + the 4-digit value of the nibbles d (byte 0 most significant)
DA_HD uint32_t dig4(uint32_t d, uint32_t acc) {
  const uint32_t t = udot4(d, 0x0000010Au, acc * 100u);  // acc*100 + 10 d0 + d1
  return udot4(d, 0x010A0000u, t * 100u);                // t*100 + 10 d2 + d3
}
DA_HD uint32_t nd4(uint32_t x) {  // 4 bits: byte i is not '0'..'9' (bytes < 0x80)
  return udot4((((x ^ 0x30303030u) + 0x76767676u) >> 7) & 0x01010101u, 0x08040201u, 0u);
}
DA_HD uint32_t byte_of(const uint32_t w[4], uint32_t p) {  // window byte p < 16 (one v_perm)
  // (the four words as values: a select between array elements compiled to
  // a dynamically indexed private array, i.e. scratch memory)
  const uint32_t w0 = w[0], w1 = w[1], w2 = w[2], w3 = w[3];
  const bool h = (p & 8u) != 0u;
  return perm_b32(h ? w3 : w1, h ? w2 : w0, (p & 7u) | 0x0C0C0C00u);
}
DA_HD uint64_t low_bytes(uint32_t k) {  // mask of the low k bytes, k <= 8
  return k >= 8 ? ~0ull : ((1ull << (8u * k)) - 1ull);
}
// value of the L <= 8 decimal digits at window bytes s .. s+L-1 (s <= 1): the
// 8 bytes from s shifted up so the digits end at byte 7 -- the bytes after
// them fall off the top, zeros enter below -- then 4 + 4 digits by dot4 (no
// division by 10^(8-L), no table)
DA_HD uint32_t digits_ra(const uint32_t w[4], uint32_t s, uint32_t L) {
  const uint32_t sh = 8u * s;
  const uint64_t x = ((uint64_t)funnel(w[2], w[1], sh) << 32) | funnel(w[1], w[0], sh);
  const uint64_t y = L ? x << (64u - 8u * L) : 0ull;
  return dig4((uint32_t)(y >> 32) & 0x0F0F0F0Fu, dig4((uint32_t)y & 0x0F0F0F0Fu, 0u));
}

// ParseFloat<float> (strtonum.h:95-264) on a run of the uniform grammar,
// 32-bit form: integer part (<= 8 digits) right-aligned by a shift and
// converted by dot4 (digits_ra); the fraction digits [fs, pe) -- the window
// shifted up so byte pe - 1 lands on byte 15, the bytes below the fraction
// cleared -- give val2 exactly (< 10^15), and val2 / 10^fl, the reference's
// (double)val2/(double)pow10, is rounded by a Markstein quotient (one
// multiply, two FMAs, tabulated reciprocal).  The reference's arithmetic is
// kept: integer part -> f32, f64 fraction -> f32, f32 add.  *ok = false:
// exponent, long parts or a number that may continue past the window (caller
// falls back to the byte decoder).
// M: bit i set when window byte i is not '0'..'9' (16 bits)
// Straight-line (no early return: a decoder in a loop of the tile kernels
// must not split the wave's exec mask); the value is meaningless when *ok is
// false.
DA_HD float wfloat32m(const uint32_t w[4], uint32_t M, const DecTables &tb, bool *ok) {
  const uint32_t b0 = w[0] & 0xFFu;
  const bool neg = b0 == '-';
  const uint32_t sg = (neg || b0 == '+') ? 1u : 0u;
  const uint32_t p = (uint32_t)ctz32((M & ~sg) | 0x10000u);  // 0..16
  const uint32_t pc = p & 15u;
  const uint32_t c = byte_of(w, pc);
  const bool dot = c == '.';
  const uint32_t fs = pc + 1u;  // 1..16
  const uint32_t pd = (uint32_t)ctz32((M & ~((2u << pc) - 1u)) | 0x10000u);
  const uint32_t cd = byte_of(w, pd & 15u);
  const uint32_t pe = dot ? pd : pc;
  const uint32_t ce = dot ? cd : c;
  const uint32_t il = p - sg;
  *ok = p < 16u && pe < 16u && (ce | 0x20u) != 'e' && il <= 8u;
  const uint32_t iv = digits_ra(w, sg, il < 8u ? il : 8u);
  // fraction bytes [fs, pe) (empty without a '.', pe < fs): tabulated byte
  // masks of each 8-byte half
  const uint32_t pk = pe < 16u ? pe : 16u;
  const uint32_t fs8 = fs < 8u ? fs : 8u, pe8 = pk < 8u ? pk : 8u;
  const uint32_t fsh = fs > 8u ? fs - 8u : 0u, peh = pk > 8u ? pk - 8u : 0u;
  const uint64_t flo = ((uint64_t)w[1] << 32 | w[0]) & tb.hib[fs8] & ~tb.hib[pe8];
  const uint64_t fhi = ((uint64_t)w[3] << 32 | w[2]) & tb.hib[fsh] & ~tb.hib[peh];
  const uint32_t fh = dig4((uint32_t)(flo >> 32), dig4((uint32_t)flo, 0u));
  const uint32_t fo = dig4((uint32_t)(fhi >> 32), dig4((uint32_t)fhi, 0u));
  const double v = __builtin_fma((double)fh, 1e8, (double)fo);  // exact: < 10^15
  const uint32_t e = 16u - fs;                                  // 0..15
  const double r = tb.i10[e], t = v * r;
  const double q = __builtin_fma(r, __builtin_fma(-t, tb.p10[e], v), t);
  const float value = (float)iv + (float)q;
  return neg ? -value : value;
}
DA_HD float wfloat32(const uint32_t w[4], const DecTables &tb, bool *ok) {
  return wfloat32m(w, nd4(w[0]) | (nd4(w[1]) << 4) | (nd4(w[2]) << 8) | (nd4(w[3]) << 12), tb, ok);
}

// ParseUnsignedInt (strtonum.h:392-428): [+] then up to 8 digits.  Returns
// false on a leading '-' (the reference's fatal CHECK); *ok = false when the
// digits may not fit the form (caller falls back).
// M: bit i set when window byte i is not '0'..'9' (bits 0-11 used)
DA_HD bool wuint32m(const uint32_t w[4], uint32_t M, const DecTables &tb, uint64_t *out, bool *ok) {
  (void)tb;
  const uint32_t b0 = w[0] & 0xFFu;
  const uint32_t s = b0 == '+' ? 1u : 0u;
  M = (M & 0xFFFu) | 0x1000u;
  const uint32_t L = (uint32_t)ctz32(M & ~s) - s;
  *ok = L <= 8u;  // branch-free, as wfloat32m
  *out = digits_ra(w, s, L < 8u ? L : 8u);
  return b0 != '-';
}
DA_HD bool wuint32(const uint32_t w[4], const DecTables &tb, uint64_t *out, bool *ok) {
  return wuint32m(w, nd4(w[0]) | (nd4(w[1]) << 4) | (nd4(w[2]) << 8), tb, out, ok);
}

struct GSrc {  // text bytes; NUL at or beyond the chunk end (as Src), global memory
  const uint8_t *g;
  uint64_t lim;
  DA_HD uint32_t operator()(uint64_t p) const { return p < lim ? (uint32_t)g[p] : 0u; }
};

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

// the same at tile offset o (position tlo + o)
DA_HD W16 win_at_o(const uint8_t *text, uint32_t o) {
#if defined(FSVM_UAWIN) && defined(__HIP_DEVICE_COMPILE__)
  // one ds_read_b128 at the byte offset (gfx950 LDS takes unaligned reads)
  uint4 v;
  __builtin_memcpy(&v, text + o + kPre, 16);
  W16 q;
  q.lo = v.x | ((uint64_t)v.y << 32);
  q.hi = v.z | ((uint64_t)v.w << 32);
  return q;
#endif
#if defined(FSVM_WIN64)
  {  // three 8-byte aligned reads (a wave's windows are ~16 B apart: b32 reads 4-way conflict)
    const uint32_t off = o + kPre;
    // (each address made opaque: merged into ds_read2_b64 the pair costs twice two ds_read_b64)
    uint32_t a0 = off & ~7u, a1 = a0 + 8u, a2 = a0 + 16u;
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(a1));
    asm volatile("" : "+v"(a2));
#endif
    const uint64_t a = *reinterpret_cast<const uint64_t *>(text + a0), b = *reinterpret_cast<const uint64_t *>(text + a1),
                   c = *reinterpret_cast<const uint64_t *>(text + a2);
    const bool s = (off & 4u) != 0u;
    const uint32_t x0 = s ? (uint32_t)(a >> 32) : (uint32_t)a, x1 = s ? (uint32_t)b : (uint32_t)(a >> 32),
                   x2 = s ? (uint32_t)(b >> 32) : (uint32_t)b, x3 = s ? (uint32_t)c : (uint32_t)(b >> 32),
                   x4 = s ? (uint32_t)(c >> 32) : (uint32_t)c;
    const uint32_t sft = (off & 3u) * 8u;
    W16 r;
    r.lo = funnel(x1, x0, sft) | ((uint64_t)funnel(x2, x1, sft) << 32);
    r.hi = funnel(x3, x2, sft) | ((uint64_t)funnel(x4, x3, sft) << 32);
    return r;
  }
#endif
  const uint32_t off = o + kPre;
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
#ifdef FSVM_LB_DRAIN
  uint64_t lbw[4];                    // look-back: the inclusive prefix read by one lane
#endif
  uint32_t ncs, c_first, toomany, bad;
};

// Wave 0 (all 64 lanes): the chunk starts touching [tlo, thi].  The chunk of
// tlo is found by a 64-ary search -- one round of 64 independent loads per
// factor of 64 chunks, instead of a dependent binary-search chain per tile
// (9 loads at 257 chunks, the longest latency of the tile prologue) -- and the
// list comes from one more window load: csl = cs[c_first ..] inside [tlo, thi]
// (excluding cs[nchunk]), cnext = the entry after the list (cs[nchunk] == n).
//
// Split in two so the last load's latency overlaps other prologue work:
// chunk_list_begin runs the search rounds and issues the window load,
// chunk_list_end consumes it (the caller classifies in between).
struct ChunkProbe {
  uint64_t lo, cnt, v;
};
template <class BK>
DA_HDF ChunkProbe chunk_list_begin(const uint64_t *cs, int nchunk, uint64_t tlo, BK &bk) {
  const uint32_t lane = (uint32_t)bk.tid();
  const uint64_t kBig = ~0ull;
  // invariant: cs[lo] <= tlo, the answer (last i < nchunk with cs[i] <= tlo) lies in [lo, lo + cnt)
  uint64_t lo = 0, cnt = (uint64_t)nchunk;
  while (cnt > (uint64_t)kWave) {
    const uint64_t S = (cnt + kWave - 1) / kWave;
    const uint64_t i = lo + lane * S;
    const uint64_t v = (lane * S < cnt) ? cs[i] : kBig;
    const uint64_t m = bk.ballot(v <= tlo);
    const uint64_t j = 63 - clz64(m);  // lane 0 always holds (cs[lo] <= tlo)
    const uint64_t nlo = lo + j * S;
    cnt = mn<uint64_t>(S, lo + cnt - nlo);
    lo = nlo;
  }
  // window cs[lo .. lo + 64) (entries past cs[nchunk] read as "beyond")
  ChunkProbe p;
  p.lo = lo;
  p.cnt = cnt;
  p.v = lo + lane <= (uint64_t)nchunk ? cs[lo + lane] : kBig;
  return p;
}
template <class BK>
DA_HDF void chunk_list_end(const uint64_t *cs, int nchunk, uint64_t tlo, uint64_t thi, const ChunkProbe &p,
                           TileCommon &c, BK &bk) {
  const uint32_t lane = (uint32_t)bk.tid();
  const uint64_t kBig = ~0ull;
  uint64_t lo = p.lo, v = p.v;
  const uint64_t cnt = p.cnt;
  uint64_t m = bk.ballot(lane < cnt && v <= tlo);
  const uint64_t c0 = lo + (63 - clz64(m));
  if (c0 - lo > (uint64_t)(kWave - kMaxCs - 2)) {  // the list may run past the window: reload at c0
    lo = c0;
    v = lo + lane <= (uint64_t)nchunk ? cs[lo + lane] : kBig;
  }
  const uint64_t idx = lo + lane;
  const uint64_t vf = bk.shfl(v, (int)(c0 - lo));  // cs[c0]
  const uint32_t first = (uint32_t)(c0 - lo) + (vf < tlo ? 1u : 0u);  // lane of c_first
  const uint64_t lm = bk.ballot(lane >= first && idx < (uint64_t)nchunk && v <= thi);
  const uint32_t m_all = (uint32_t)popc64(lm);
  const uint32_t ln = first + m_all;                                 // lane of cnext
  const uint64_t vn = bk.shfl(v, (int)(ln < (uint32_t)kWave ? ln : 0u));
  if (lane >= first && lane - first < (uint32_t)kMaxCs && ((lm >> lane) & 1u)) c.csl[lane - first] = v;
  if (lane == 0) {
    c.cfloor = vf;
    c.c_first = (uint32_t)(lo + first);
    const bool over = m_all > (uint32_t)kMaxCs || ln >= (uint32_t)kWave;
    c.ncs = over ? (uint32_t)kMaxCs : m_all;
    c.cnext = ln < (uint32_t)kWave ? vn : kBig;
    c.toomany = over;
    c.bad = 0;
  }
}
template <class BK>
DA_HDF void chunk_list(const uint64_t *cs, int nchunk, uint64_t tlo, uint64_t thi, TileCommon &c,
                       BK &bk) {
  const ChunkProbe p = chunk_list_begin(cs, nchunk, tlo, bk);
  chunk_list_end(cs, nchunk, tlo, thi, p, c, bk);
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
  for (uint64_t u = bk.tid(); u < nunits; u += kFThreads) {
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

// The same staging split in two so every load of the tile is in flight at
// once: stage_issue loads each thread's 16-byte units into registers (all
// kStageRounds loads before any wait), stage_commit writes them to LDS.  The
// caller puts the tile's other prologue work (chunk list, tables) between the
// two, so its latency overlaps the loads'.  (A single loop of load -> LDS
// store waited for each load in turn: 5 HBM round trips per tile, ~14k cycles
// of a ~57k-cycle tile.)  Tiles whose staged range leaves the text take the
// byte-wise path of stage() at commit time.
constexpr int kStageUnits = kStage / 16;
constexpr int kStageRounds = (kStageUnits + kFThreads - 1) / kFThreads;
static_assert(kStage % 16 == 0, "staged range is whole 16-byte units");
struct StageRegs {
  uint32_t w[kStageRounds][4];
  bool interior;
};
#if defined(FSVM_GLDS) && defined(__HIP_DEVICE_COMPILE__)
// LDS-DMA form (global_load_lds_dwordx4): the staged range is contiguous in
// HBM and in LDS, so each wave-instruction moves 1 KiB straight into LDS
// (lane l's 16 bytes at base + 16 l) -- no staging VGPRs, no ds_write; the
// barrier after stage_commit waits for them (vmcnt).  `c` names the LDS.
constexpr int kStagePieces = (kStage + kWave * 16 - 1) / (kWave * 16);
template <class BK>
DA_HDF void stage_issue_lds(const uint8_t *text, uint64_t n, uint64_t tlo, StageRegs &r, TileCommon &c, BK &bk) {
  r.interior = tlo >= (uint64_t)kPre && tlo + kTile + kPost <= n;
  if (!r.interior) return;
  const uint8_t *src = text + (tlo - kPre);
  const int t = bk.tid(), lane = t & (kWave - 1), w = t / kWave;
#pragma unroll
  for (int q = w; q < kStagePieces; q += kFWaves) {
    const int off = q * kWave * 16 + lane * 16;
    if (off < kStage)
      __builtin_amdgcn_global_load_lds((const void *)(src + off),
                                       (__attribute__((address_space(3))) void *)(c.text + q * kWave * 16), 16, 0, 0);
  }
}
#endif
template <class BK>
DA_HDF void stage_issue(const uint8_t *text, uint64_t n, uint64_t tlo, StageRegs &r, BK &bk) {
  r.interior = tlo >= (uint64_t)kPre && tlo + kTile + kPost <= n;
  if (!r.interior) return;
  const uint8_t *src = text + (tlo - kPre);
  const int t = bk.tid();
#pragma unroll
  for (int i = 0; i < kStageRounds; ++i) {
    const int u = t + i * kFThreads;
#if defined(FSVM_NT_STAGE) && defined(__HIP_DEVICE_COMPILE__)  // A/B: streaming (non-temporal) text loads
    if (u < kStageUnits) {
      typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
      const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4 *>(src + 16 * u));
      r.w[i][0] = v.x;
      r.w[i][1] = v.y;
      r.w[i][2] = v.z;
      r.w[i][3] = v.w;
    }
#else
    if (u < kStageUnits) load16(src + 16 * u, r.w[i]);
#endif
  }
}
template <class BK>
DA_HDF void stage_commit(const uint8_t *text, uint64_t n, uint64_t tlo, const StageRegs &r, TileCommon &c,
                         BK &bk) {
  if (!r.interior) {
    stage(text, n, tlo, c, bk);
    return;
  }
#if defined(FSVM_GLDS) && defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // stage_issue_lds's bytes have landed
  return;
#endif
  const int t = bk.tid();
#pragma unroll
  for (int i = 0; i < kStageRounds; ++i) {
    const int u = t + i * kFThreads;
    if (u < kStageUnits) memcpy(c.text + 16 * u, r.w[i], 16);
  }
}

// ---- decoupled look-back records.  Two arrays: st[ntiles], one 8-byte
// status word per tile -- bits 62-63 state (1 aggregate, 2 inclusive) | the
// tile's four counts packed 15 bits each (a 16 KiB tile holds < 2^15 of
// anything) -- and incl[ntiles][4], the inclusive prefix per counter, written
// and drained (vmcnt(0)) before the status turns inclusive.  The status words
// of consecutive tiles share cache lines: one poll instruction of a wave reads
// 64 predecessors' words (512 contiguous bytes, 4 lines), where a record of a
// line per tile cost a line per predecessor.  (kLbPer > 1 polls more
// predecessors per round; measured slower at 4.)
constexpr uint64_t kSAgg = 1ull << 62, kSIncl = 2ull << 62;
#ifndef FSVM_LB_PER
#define FSVM_LB_PER 1
#endif
constexpr int kLbPer = FSVM_LB_PER;  // predecessors polled per lane per round
DA_HD uint64_t pack4(const uint32_t c[4]) {
  return (uint64_t)c[0] | ((uint64_t)c[1] << 15) | ((uint64_t)c[2] << 30) | ((uint64_t)c[3] << 45);
}
DA_HD void drain_stores() {
#if defined(__HIP_DEVICE_COMPILE__)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
}

// Inclusive prefixes are tagged words: incl[k][f] = kMark | value, each an
// untorn 8-byte granule that the launch's memset left 0, so a reader takes
// a tile's inclusive prefix as soon as all four of its words carry the mark
// -- no drain between the prefix and a status flag, and the reader polls a
// predecessor's status word and prefix words in the same round trip.
constexpr uint64_t kMark = 1ull << 63;
#ifndef FSVM_LB_DRAIN

// Lane 0: publish this tile's aggregate (tile 0 publishes its inclusive).
// kf / seed: a launch that resumes at tile kf (svm_lean.h) -- tile kf is the
// first, its exclusive prefix is seed[4] (tagged inclusive words of the
// launch before: the mark is dropped).
DA_HD void publish_aggregate(uint64_t *lb, uint32_t ntiles, uint32_t k, const uint32_t cnt[4], uint32_t kf = 0,
                             const uint64_t *seed = nullptr) {
  uint64_t *st = lb, *incl = lb + ntiles;
  if (k == kf) {
    for (int i = 0; i < 4; ++i) store_agent_u64(incl + (uint64_t)k * 4 + i, kMark | ((seed ? seed[i] & ~kMark : 0) + cnt[i]));
  } else {
    store_agent_u64(st + k, kSAgg | pack4(cnt));
  }
}

// Wave 0: decoupled look-back.  Lane l polls predecessor j-1-l: its status
// word (512 contiguous bytes per wave) and its four prefix words; a round
// consumes predecessors up to the nearest one with a complete inclusive
// prefix and stops before the nearest unpublished one.  cnt = this tile's
// counts (wave uniform).  Ends with c.base[0..3] = exclusive prefixes and
// publishes the inclusive prefix.  Returns the number of rounds.  The caller
// synchronises.
template <class BK>
DA_HDF uint32_t look_back(uint64_t *lb, uint32_t ntiles, uint32_t k, const uint32_t cnt[4], uint32_t *gate,
                          TileCommon &c, BK &bk, uint32_t kf = 0, const uint64_t *seed = nullptr) {
  const uint32_t lane = bk.tid();
  uint64_t *st = lb, *incl = lb + ntiles;
  uint64_t j = k;
  uint32_t spins = 0, rounds = 0;
  uint64_t acc[4] = {0, 0, 0, 0};
  if (k == kf && seed)
    for (int f = 0; f < 4; ++f) acc[f] = seed[f] & ~kMark;
  bool done = k == kf;  // (a resumed launch: tile kf published its inclusive prefix, svm_lean.h)
  while (!done) {
    ++rounds;
    uint64_t s = 0, w[4] = {kMark, kMark, kMark, kMark};  // before tile 0: an inclusive 0
    if (lane < j) {
      const uint64_t p = j - 1 - lane;
      s = load_agent_u64(st + p);
#pragma unroll
      for (int f = 0; f < 4; ++f) w[f] = load_agent_u64(incl + p * 4 + f);
    }
    const bool inc = (w[0] & w[1] & w[2] & w[3] & kMark) != 0;
    const uint64_t mi = bk.ballot(inc), mz = bk.ballot(!inc && (s >> 62) == 0);
    uint64_t D = kWave;  // predecessors that contribute their aggregates
    bool stop_incl = false;
    if (mz | mi) {
      D = (uint64_t)ctz64(mz | mi);
      stop_incl = (mi >> D) & 1u;
    }
    uint32_t part[4] = {0, 0, 0, 0};
    if (lane < D) {
#pragma unroll
      for (int f = 0; f < 4; ++f) part[f] = (uint32_t)((s >> (15 * f)) & 0x7FFFu);
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[f] += bk.wave_sum(part[f]);
    if (stop_incl) {
      done = true;
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[f] += bk.shfl(w[f] & ~kMark, (int)D);
    } else {
      j -= D;
      if (D == 0) {
        if (++spins > kSpinLimit) {  // never expected: hand the input to the exact path
          if (lane == 0) atomic_or_u32(gate, 2u);
          done = true;
        }
        spin_pause();
      }
    }
  }
  if (lane < 4) {
    const uint64_t v = acc[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3];
    c.base[lane] = v;
    if (k > kf) store_agent_u64(incl + (uint64_t)k * 4 + lane, kMark | (v + cnt[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3]));
  }
  return rounds;
}
#else  // A/B build: inclusive prefix drained before an inclusive status word (round 2)
// Lane 0: publish this tile's aggregate (tile 0 publishes its inclusive).
DA_HD void publish_aggregate(uint64_t *lb, uint32_t ntiles, uint32_t k, const uint32_t cnt[4]) {
  uint64_t *st = lb, *incl = lb + ntiles;
  if (k == 0) {
    for (int i = 0; i < 4; ++i) store_agent_u64(incl + i, cnt[i]);
    drain_stores();
    store_agent_u64(st, kSIncl | pack4(cnt));
  } else {
    store_agent_u64(st + k, kSAgg | pack4(cnt));
  }
}

// Wave 0: decoupled look-back.  Poll i of lane l reads the status word of
// predecessor j-1-(64 i + l) (each poll instruction reads 512 contiguous
// bytes); a round consumes predecessors up to the first inclusive one and
// stops before the first unpublished one.  cnt = this tile's counts (wave
// uniform).  Ends with c.base[0..3] = exclusive prefixes, and publishes the
// inclusive prefix.  Returns the number of rounds.  The caller synchronises.
template <class BK>
DA_HDF uint32_t look_back(uint64_t *lb, uint32_t ntiles, uint32_t k, const uint32_t cnt[4], uint32_t *gate,
                          TileCommon &c, BK &bk) {
  const uint32_t lane = bk.tid();
  uint64_t *st = lb, *incl = lb + ntiles;
  uint64_t j = k;
  uint32_t spins = 0, rounds = 0;
  uint64_t acc[4] = {0, 0, 0, 0};
  bool done = k == 0;
  while (!done) {
    ++rounds;
    uint64_t s[kLbPer];
#pragma unroll
    for (int i = 0; i < kLbPer; ++i) {
      const uint64_t d = (uint64_t)i * kWave + lane;  // predecessor j-1-d
      s[i] = d < j ? load_agent_u64(st + (j - 1 - d)) : kSIncl;  // before tile 0: an inclusive 0
    }
    // the nearest stop: the smallest d whose word is unpublished or inclusive
    uint64_t D = (uint64_t)kWave * kLbPer;  // predecessors that contribute their aggregates
    bool stop_incl = false;
#pragma unroll
    for (int i = kLbPer - 1; i >= 0; --i) {
      const uint32_t state = (uint32_t)(s[i] >> 62);
      const uint64_t mz = bk.ballot(state == 0), mi = bk.ballot(state == 2);
      if (mz | mi) {
        const uint32_t f = (uint32_t)ctz64(mz | mi);
        D = (uint64_t)i * kWave + f;
        stop_incl = (mi >> f) & 1u;
      }
    }
    uint32_t part[4] = {0, 0, 0, 0};
#pragma unroll
    for (int i = 0; i < kLbPer; ++i) {
      if ((uint64_t)i * kWave + lane < D) {
#pragma unroll
        for (int f = 0; f < 4; ++f) part[f] += (uint32_t)((s[i] >> (15 * f)) & 0x7FFFu);
      }
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[f] += bk.wave_sum(part[f]);
    if (stop_incl) {
      done = true;
      if (D < j) {  // a real inclusive record (else: the start, 0)
        if (lane < 4) c.lbw[lane] = load_agent_u64(incl + (j - 1 - D) * 4 + lane);
        bk.wave_sync();
#pragma unroll
        for (int f = 0; f < 4; ++f) acc[f] += c.lbw[f];
        bk.wave_sync();
      }
    } else {
      j -= D;
      if (D == 0) {
        if (++spins > kSpinLimit) {  // never expected: hand the input to the exact path
          if (lane == 0) atomic_or_u32(gate, 2u);
          done = true;
        }
        spin_pause();
      }
    }
  }
  if (lane < 4) c.base[lane] = acc[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3];
  if (k > 0) {
    if (lane < 4) {
      const uint64_t v = acc[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3];
      const uint32_t cv = cnt[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3];
      store_agent_u64(incl + (uint64_t)k * 4 + lane, v + cv);
    }
    drain_stores();
    bk.wave_sync();
    if (lane == 0) store_agent_u64(st + k, kSIncl | pack4(cnt));
  }
  return rounds;
}
#endif
// words of look-back state per tile the launch must zero (status + prefix)
constexpr uint64_t kLbWords = kFastLbWords;  // args.h: the launcher sizes the workspace by it

}  // namespace fast
}  // namespace dmlc_amd
