// decode.h -- exact device restatements of the reference's numeric decoders.
//
//   parse_float   <- dmlc::ParseFloat<float,false>      include/dmlc/strtonum.h:95-264
//   parse_uint    <- dmlc::ParseUnsignedInt<T>(p,0,10)  include/dmlc/strtonum.h:392-428
//   c_strtoll     <- glibc strtoll(p, &e, base 10|0)    (csv_parser.h:102,105; atoll at
//                                                         libsvm_parser.h:127)
//
// Bit-exactness notes: u64 digit accumulation wraps exactly as on the host; the
// fraction is ONE IEEE f64 division (double)val2/(double)pow10 followed by a
// f64->f32 rounding and an f32 add; the exponent applies an f32 multiply chain.
// This translation unit is built with -ffp-contract=off and correctly rounded
// f32 division (-fhip-fp32-correctly-rounded-divide-sqrt), so no FMA
// contraction or approximate reciprocal changes a bit.
#pragma once
#include "common.h"

namespace dmlc_amd {

template <typename F>
DA_HD float parse_float(const F &at, uint64_t p, uint64_t *endp, bool *nan_err) {
  while (is_space(at(p))) ++p;
  bool sign = true;
  uint32_t c = at(p);
  if (c == '-') {
    sign = false;
    ++p;
  } else if (c == '+') {
    ++p;
  }
  {
    // case-insensitive "inf" / "infinity" (exactly 3 or 8 letters), then "nan"
    const char kInf[8] = {'i', 'n', 'f', 'i', 'n', 'i', 't', 'y'};
    int i = 0;
    while (i < 8 && ((at(p + i) | 32u) & 0xFFu) == (uint32_t)kInf[i]) ++i;
    if (i == 3 || i == 8) {
      *endp = p + i;
      return sign ? __builtin_huge_valf() : -__builtin_huge_valf();
    }
    const char kNan[3] = {'n', 'a', 'n'};
    i = 0;
    while (i < 3 && ((at(p + i) | 32u) & 0xFFu) == (uint32_t)kNan[i]) ++i;
    if (i == 3) {
      p += 3;
      if (at(p) == '(') {
        ++p;
        for (;;) {
          uint32_t d = at(p);
          if (is_digit(d) || is_alpha(d) || d == '_') ++p;
          else break;
        }
        if (at(p) != ')') *nan_err = true;
        ++p;
      }
      *endp = p;
      return u2f(0x7FC00000u);
    }
  }
  uint64_t predec = 0;
  for (c = at(p); is_digit(c); c = at(++p)) predec = predec * 10ull + (uint64_t)(c - '0');
  float value = (float)predec;
  if (c == '.') {
    uint64_t pow10 = 1, val2 = 0;
    int cnt = 0;
    for (c = at(++p); is_digit(c); c = at(++p)) {
      if (cnt < 19) {  // kStrtofMaxDigits
        val2 = val2 * 10ull + (uint64_t)(c - '0');
        pow10 *= 10ull;
      }
      ++cnt;
    }
    value += (float)((double)val2 / (double)pow10);
  }
  if (c == 'e' || c == 'E') {
    bool frac = false;
    float scale = 1.0f;
    c = at(++p);
    if (c == '-') {
      frac = true;
      c = at(++p);
    } else if (c == '+') {
      c = at(++p);
    }
    uint32_t expon = 0;
    for (; is_digit(c); c = at(++p)) expon = expon * 10u + (c - '0');
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
  if (c == 'f' || c == 'F') ++p;
  *endp = p;
  return sign ? value : -value;
}

// Returns false on a leading '-' (the reference's fatal CHECK).
template <typename F>
DA_HD bool parse_uint(const F &at, uint64_t p, bool wide, uint64_t *out) {
  uint32_t c = at(p);
  while (is_space(c)) c = at(++p);
  if (c == '-') return false;
  if (c == '+') c = at(++p);
  if (wide) {
    uint64_t v = 0;
    for (; is_digit(c); c = at(++p)) v = v * 10ull + (c - '0');
    *out = v;
  } else {
    uint32_t v = 0;
    for (; is_digit(c); c = at(++p)) v = v * 10u + (c - '0');
    *out = v;
  }
  return true;
}

// glibc strtoll, C locale, base 10 or 0 (auto 0x / 0 prefixes), saturating.
// *endp = first unconsumed byte, or `p` itself when no digits were consumed.
template <typename F>
DA_HD int64_t c_strtoll(const F &at, uint64_t p0, int base, uint64_t *endp) {
  uint64_t p = p0;
  uint32_t c = at(p);
  while (is_cspace(c)) c = at(++p);
  bool neg = false;
  if (c == '-') {
    neg = true;
    c = at(++p);
  } else if (c == '+') {
    c = at(++p);
  }
  if (base == 0) {
    base = 10;
    if (c == '0') {
      uint32_t x = at(p + 1), h = at(p + 2);
      bool hexd = is_digit(h) || (h | 32u) - 'a' < 6u;
      if ((x | 32u) == 'x' && hexd) {
        base = 16;
        p += 2;
        c = at(p);
      } else {
        base = 8;
      }
    }
  }
  const uint64_t cutoff = neg ? (1ull << 63) : (1ull << 63) - 1;
  uint64_t acc = 0;
  bool any = false, ovf = false;
  for (;; c = at(++p)) {
    uint32_t d;
    if (is_digit(c)) d = c - '0';
    else if ((c | 32u) - 'a' < 26u) d = (c | 32u) - 'a' + 10;
    else break;
    if (d >= (uint32_t)base) break;
    any = true;
    if (ovf) continue;
    if (acc > (cutoff - d) / (uint64_t)base) {
      ovf = true;
      continue;
    }
    acc = acc * (uint64_t)base + d;
  }
  *endp = any ? p : p0;
  if (ovf) return neg ? (int64_t)(1ull << 63) : (int64_t)((1ull << 63) - 1);
  if (!any) return 0;
  return neg ? (int64_t)(0ull - acc) : (int64_t)acc;
}

}  // namespace dmlc_amd
