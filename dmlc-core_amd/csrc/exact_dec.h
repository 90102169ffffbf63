// exact_dec.h -- the exact tile kernels' number decoding in registers.
//
// The exact kernels (libsvm_core.h, csv_core.h, libfm_core.h) stage the text
// in LDS windows and decode each run with the byte decoders of decode.h
// (ParseFloat / ParseUnsignedInt, strtonum.h:95-264, :392-428).  A run whose
// 16 bytes lie inside the staged window and before its chunk end goes through
// the single-pass kernels' window decoders (fast_common.h wfloat32m /
// wuint32m) instead, which report when a run does not fit their form; the
// byte decoders take those.  tests/emu/dec_check.cpp compares both on
// generated strings of every byte value.
#pragma once
#include "common.h"
#include "decode.h"
#include "fast_common.h"

namespace dmlc_amd {

// The 16 bytes at x from the staged window (two aligned LDS words per output
// word, funnel-shifted), when all of them lie inside the window and before
// the chunk end: the run at x can then be decoded in registers by the
// window decoders of the single-pass kernels (fast_common.h wfloat32 /
// wuint32), which report when the run does not fit their form -- the byte
// decoders of decode.h take those.
DA_HD bool win16(const Src &s, uint64_t x, uint32_t w[4]) {
  if (x < s.wbase || x + 16 > s.wend || x + 16 > s.lim) return false;
  const uint64_t o = x - s.wbase;
  const uint32_t *q = reinterpret_cast<const uint32_t *>(s.lds + (o & ~3ull));
  const uint32_t sh = 8u * (uint32_t)(o & 3u);
  uint32_t v[5];
  for (int i = 0; i < 5; ++i) v[i] = q[i];
  for (int i = 0; i < 4; ++i) w[i] = fast::funnel(v[i + 1], v[i], sh);
  return true;
}
// bit i: window byte i is not '0'..'9' -- any byte value (fast_common.h nd4
// assumes bytes < 0x80, which the single-pass grammar guarantees and the
// text of the exact kernels does not)
DA_HD uint32_t nondigit16(const uint32_t w[4]) {
  uint32_t m = 0;
  for (int i = 0; i < 4; ++i) {
    const uint32_t y = w[i] & 0x7F7F7F7Fu;
    const uint32_t t = ((((y ^ 0x30303030u) + 0x76767676u) | w[i]) >> 7) & 0x01010101u;
    m |= fast::udot4(t, 0x08040201u, 0u) << (4 * i);
  }
  return m;
}
// ParseUnsignedInt of the run at x through the window when it fits (a '-' or
// more than 8 digits: the byte decoder, which also raises the '-' error)
DA_HD bool index_at(const Src &src, uint64_t x, bool wide, const fast::DecTables *dt, uint64_t *v) {
  uint32_t w[4];
  if (dt && win16(src, x, w) && !is_space(w[0] & 0xFFu)) {  // (the byte decoder skips leading blanks)
    bool ok;
    uint64_t t;
    const bool pos = fast::wuint32m(w, nondigit16(w), *dt, &t, &ok);
    if (ok && pos) {
      *v = t;
      return true;
    }
  }
  return parse_uint(src, x, wide, v);
}
// ParseFloat<float> of the text at x through the window when it fits.  Beyond
// the single-pass grammar, a sign followed by inf / nan letters is left to
// the byte decoder (wfloat32 reads it as a signed zero).
DA_HD float value_at(const Src &src, uint64_t x, const fast::DecTables *dt, bool *nan_err) {
  uint32_t w[4];
  if (dt && win16(src, x, w)) {
    const uint32_t b0 = w[0] & 0xFFu, b1 = ((w[0] >> 8) & 0xFFu) | 0x20u, l0 = b0 | 0x20u;
    const bool letter = ((b0 == '-' || b0 == '+') && (b1 == 'i' || b1 == 'n')) || l0 == 'i' || l0 == 'n' ||
                        is_space(b0);  // (inf / nan tokens and leading blanks: the byte decoder)
    bool ok;
    const float f = fast::wfloat32m(w, nondigit16(w), *dt, &ok);
    if (ok && !letter) return f;
  }
  uint64_t e;
  return parse_float(src, x, &e, nan_err);
}

// The same for a CSV field at x (csv_parser.h:102-106): when the window
// decodes it, *end = the byte after the number (the reference's endptr,
// strtonum.h:258-263: a trailing 'f' / 'F' is consumed).  Only a field that
// starts with a digit or with a sign / '.' followed by a digit or '.' is
// taken, so the field is never empty and never inf / nan.
DA_HD bool csv_value_at(const Src &src, uint64_t x, const fast::DecTables *dt, float *v, uint64_t *end) {
  uint32_t w[4];
  if (!dt || !win16(src, x, w)) return false;
  const uint32_t M = nondigit16(w);
  const uint32_t b0 = w[0] & 0xFFu, b1 = (w[0] >> 8) & 0xFFu;
  const bool sgn = b0 == '-' || b0 == '+';
  const bool d0 = !(M & 1u), d1 = !(M & 2u);
  if (!(d0 || ((sgn || b0 == '.') && (d1 || b1 == '.')))) return false;
  bool ok;
  const float f = fast::wfloat32m(w, M, *dt, &ok);
  if (!ok) return false;
  const uint32_t sg = sgn ? 1u : 0u;
  const uint32_t p = (uint32_t)ctz32((M & ~sg) | 0x10000u);
  const uint32_t pc = p & 15u;
  uint32_t pe = pc;
  if (fast::byte_of(w, pc) == '.') pe = (uint32_t)ctz32((M & ~((2u << pc) - 1u)) | 0x10000u) & 15u;
  const uint32_t ce = fast::byte_of(w, pe) | 0x20u;
  *end = x + pe + (ce == 'f' ? 1u : 0u);
  *v = f;
  return true;
}

// Digitchar (strtonum.h:70-72) and newline masks of the len <= 32 staged
// bytes at win + off: nine aligned LDS words funnel-shifted to the segment,
// classified four bytes at a time by the nibble tables (fast_common.h
// classify_dword; bytes >= 0x80 are neither) -- instead of 32 byte reads.
// The window buffer must hold 36 bytes past off.
DA_HD void seg_masks(const uint8_t *win, uint32_t off, int len, uint32_t *dm, uint32_t *nl) {
  const uint32_t *q = reinterpret_cast<const uint32_t *>(win + (off & ~3u));
  const uint32_t sh = 8u * (off & 3u);
  uint32_t v[9];
  for (int i = 0; i < 9; ++i) v[i] = q[i];
  uint32_t d = 0, n = 0;
  for (int i = 0; i < 8; ++i) {
    const fast::Nib b = fast::classify_dword(fast::funnel(v[i + 1], v[i], sh));
    d |= (b.d & ~b.hi) << (4 * i);
    n |= (b.n & ~b.hi) << (4 * i);
  }
  const uint32_t m = len >= 32 ? ~0u : ((1u << len) - 1u);
  *dm = d & m;
  *nl = n & m;
}

DA_HD uint32_t eq_nib(uint32_t x, uint32_t rep) {  // 4 bits: byte i of x == the byte repeated in rep
  const uint32_t t = x ^ rep;
  const uint32_t nz = (((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;  // bit 7: byte nonzero
  return ((((~nz >> 7) & 0x01010101u) * 0x01020408u) >> 24) & 0xFu;
}
// The same plus the ':' , blank (' ' '\t') and '#' masks: what gap_fnb
// (libsvm_core.h) reads byte by byte, for the role walk's gap classes.
DA_HD void seg_masks5(const uint8_t *win, uint32_t off, int len, uint32_t *dm, uint32_t *nl, uint32_t *cm,
                      uint32_t *bm, uint32_t *hm) {
  const uint32_t *q = reinterpret_cast<const uint32_t *>(win + (off & ~3u));
  const uint32_t sh = 8u * (off & 3u);
  uint32_t v[9];
  for (int i = 0; i < 9; ++i) v[i] = q[i];
  uint32_t d = 0, n = 0, c = 0, b = 0, h = 0;
  for (int i = 0; i < 8; ++i) {
    const uint32_t x = fast::funnel(v[i + 1], v[i], sh);
    const uint32_t cls = fast::classify4(x), hi = fast::hi_nib4(x);
    d |= (fast::nib_d(cls) & ~hi) << (4 * i);
    n |= (fast::nib_n(cls) & ~hi) << (4 * i);
    c |= (fast::nib_c(cls) & ~hi) << (4 * i);
    b |= ((((((cls >> 5) | (cls >> 6)) & 0x01010101u) * 0x01020408u) >> 24) & ~hi & 0xFu) << (4 * i);
    h |= eq_nib(x, 0x23232323u) << (4 * i);
  }
  const uint32_t m = len >= 32 ? ~0u : ((1u << len) - 1u);
  *dm = d & m;
  *nl = n & m;
  *cm = c & m;
  *bm = b & m;
  *hm = h & m;
}

// Newline and delimiter masks of the len <= 32 staged bytes at win + off (the
// CSV exact kernels): byte-equality by the carry-free zero-byte test on nine
// aligned LDS words, four bytes at a time.
DA_HD void seg_masks_csv(const uint8_t *win, uint32_t off, int len, uint32_t delim, uint32_t *nl, uint32_t *dl) {
  const uint32_t *q = reinterpret_cast<const uint32_t *>(win + (off & ~3u));
  const uint32_t sh = 8u * (off & 3u);
  const uint32_t rd = (delim & 0xFFu) * 0x01010101u;
  uint32_t v[9];
  for (int i = 0; i < 9; ++i) v[i] = q[i];
  uint32_t n = 0, d = 0;
  for (int i = 0; i < 8; ++i) {
    const uint32_t x = fast::funnel(v[i + 1], v[i], sh);
    n |= (eq_nib(x, 0x0A0A0A0Au) | eq_nib(x, 0x0D0D0D0Du)) << (4 * i);
    d |= eq_nib(x, rd) << (4 * i);
  }
  const uint32_t m = len >= 32 ? ~0u : ((1u << len) - 1u);
  *nl = n & m;
  *dl = d & m;
}

}  // namespace dmlc_amd
