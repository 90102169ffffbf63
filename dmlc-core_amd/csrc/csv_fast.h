// csv_fast.h -- the single-pass CSV tile body for the "uniform CSV grammar":
// every byte is a number character (0-9 + - . e E), the delimiter or a
// newline; no label / weight column; float values.  Inside that grammar
// CSVParser::ParseBlock (src/data/csv_parser.h:71-149) reduces to:
//
//   row     a maximal run of non-newline bytes (leading newlines skipped,
//           empty lines dropped, csv_parser.h:78-80,138-140); one offset each
//   field   starts at a row start or after a delimiter that is not the last
//           byte of the line (no phantom trailing field, :123-134)
//   column  = delimiters between the row start and the field start
//   token   a non-empty field: strtof consumed >= 1 byte, so the reference
//           pushes value = ParseFloat(field), index = column (:112-118);
//           an empty field only advances the column
//
// So the parse is bitmask arithmetic on 64-byte segments plus one segmented
// count: the column of a token needs the delimiters since its row start,
// which may lie in an earlier segment or tile -- a segmented scan inside the
// tile and a segmented counter in the decoupled look-back across tiles.
// Values use the 32-bit window decoder (fast_common.h wfloat32) with the
// exact byte decoder as fallback.  Any byte outside the grammar sets the gate
// word and the exact tile kernels (csv_core.h) produce the result.
//
// Same structure and block policy as svm_fast.h (the CPU emulator runs it).
#pragma once
#include <type_traits>

#include "fast_common.h"

namespace dmlc_amd {
namespace fcsv {
using namespace fast;

// look-back slots: rows, values, the segmented delimiter tail, its row-start flag
enum { Q_ROWS = 0, Q_VALS = 1, Q_TAIL = 2, Q_FLAG = 3 };

struct Planes {  // slot 0: the segment before the tile; slot t+1: segment t
  uint64_t d[kFThreads + 1];  // number characters
  uint64_t n[kFThreads + 1];  // newlines
  uint64_t l[kFThreads + 1];  // delimiters
};
// token list entries (svm_fast.h's run lists for CSV): tile offset (14 bits),
// column since the row start or the tile start (17 bits: at most kTile
// delimiters lie before a token in its tile), bit 31: add the carry the
// look-back brings (the token's row started before the tile)
constexpr int kListCap = (int)(sizeof(Planes) / sizeof(uint32_t));
constexpr uint32_t kPassTokens = (uint32_t)kListCap - kSegB;
constexpr uint32_t kColBits = 17;

struct Shared {  // LDS of one workgroup
  TileCommon c;
  union {
    Planes m;
    uint32_t lst[kListCap];
  } u;
  uint32_t cls[kClsEntries];  // byte classes: byte 0 number char, 1 digit (without 0: outside the grammar),
                              // 2 newline, 3 delimiter
  DecTables dt;
  uint32_t gw[2 * kFThreads + 2];  // digit plane as words: 2t, 2t+1 segment t; 2 kFThreads: the post-halo
  uint64_t segc;      // the tile's segmented carry (delimiters since the last row start before it)
  uint32_t nlab, nfirst;  // label tokens (bits 0-15) and weight tokens (16-31) / first delimiters
                          // of rows in this tile (a tile holds < 2^16 tokens; one word keeps the
                          // LDS footprint -- 16 more bytes cost the plain kernel 8%)
  uint32_t pend[kTile / kPassTokens + 2];  // token counts at the end of each pass
  uint32_t npass;
  uint32_t junk;  // the tile (or its halos) holds junk bytes (csv_junk_byte)
};

// "Junk" (float values, no label / weight column): text a number ends at
// (strtonum.h:95-264) -- a header word, a text column, "3.5kg", bytes >=
// 0x80.  A field that starts with it holds no value (ParseFloat consumed
// nothing: the column advances, csv_parser.h:115-118) -- except where
// ParseFloat does read it: an 'f' / 'F' is the suffix it consumes (a field
// "feature_1" is the value 0, which the window decoder yields), "inf" /
// "infinity" / "nan" (any case, also after a sign) are the values +-inf and
// NaN (csv_inf_nan; decoded by inf_nan_of), and junk after blanks is a 0
// (ParseFloat consumed the blanks).  "nan(" -- ParseFloat's NAN(chars) form
// with its fatal CHECK for the ')' -- is left to the exact kernels.  A UTF-8
// BOM at a row start is skipped (IgnoreUTF8BOM, text_parser.h:83-102,
// csv_parser.h:83): the row's first field starts after it.  Not junk: number
// characters and what ParseFloat skips (isspace; '\f' and '\v' stay outside
// the grammar).
DA_HD bool csv_junk_byte(uint32_t b) { return b != ' ' && b != '\t' && b != '\v' && b != '\f'; }
// Letters of "infinity" matched at p (case-insensitive, at most 8): the
// reference's INF branch stands only for exactly 3 or 8 of them
// (strtonum.h:133-148; "infin" is no number)
DA_HD uint32_t infinity_len(uint64_t lo) {  // lo: the 8 bytes at p, little-endian
  const uint64_t x = (lo | 0x2020202020202020ull) ^ 0x7974696E69666E69ull;  // "infinity"
  return x ? (uint32_t)ctz64(x) >> 3 : 8u;
}
// the bytes at p start ParseFloat's "inf" / "infinity" or "nan":
// 1 inf, 2 nan, 3 "nan(" (its NAN(chars) form), 0 neither.  nv: the bytes
// before the InputSplit chunk end (ParseFloat reads NUL from there on).
DA_HD uint32_t csv_inf_nan(const uint8_t *p, uint64_t nv) {
  uint64_t lo = 0;
  for (int i = 0; i < 8; ++i) lo |= (uint64_t)((uint64_t)i < nv ? p[i] : 0u) << (8 * i);
  const uint32_t k = infinity_len(lo);
  if (k == 3u || k == 8u) return 1u;
  if (((lo | 0x202020u) & 0xFFFFFFu) == 0x6E616Eu) return nv > 3u && p[3] == '(' ? 3u : 2u;
  return 0u;
}
// ParseFloat's INF / NAN branch (strtonum.h:133-175) on a token window whose
// first byte after the optional sign is a letter: +-inf ("inf" and
// "infinity" alike), the quiet NaN (no sign: the reference returns
// quiet_NaN() whatever the sign), else false (the letters are no number:
// the window decoder's 0 stands)
DA_HD bool inf_nan_of(const uint32_t w[4], float *v) {
  const uint32_t b0 = w[0] & 0xFFu;
  const uint32_t sg = (b0 == '-' || b0 == '+') ? 1u : 0u;
  const uint32_t s8 = 8u * sg;  // the 8 bytes after the sign
  const uint64_t lo = (uint64_t)funnel(w[1], w[0], s8) | ((uint64_t)funnel(w[2], w[1], s8) << 32);
  const uint32_t k = infinity_len(lo);
  if (k == 3u || k == 8u) {
    *v = b0 == '-' ? -__builtin_huge_valf() : __builtin_huge_valf();
    return true;
  }
  if (((uint32_t)lo | 0x202020u) == (((uint32_t)lo & 0xFF000000u) | 0x6E616Eu)) {  // "nan"
    *v = u2f(0x7FC00000u);
    return true;
  }
  return false;
}
// junk: with the junk class (digit + newline, a pair no other byte has; the
// classifier splits it off)
DA_HD uint32_t class_of_csv(uint32_t b, uint32_t delim, bool blanks, bool junk = false) {
  if (b == delim) return 0x01000000u;
  if (is_digitchar(b)) return is_digit(b) ? 0x00000101u : 0x00000001u;
  if (b == '\n' || b == '\r') return 0x00010000u;
  if (blanks && (b == ' ' || b == '\t')) return 0u;  // blank: class 0
  if (junk && csv_junk_byte(b)) return 0x00010100u;
  return 0x00000100u;  // outside the grammar: "digit" without "number char"
}

// segmented sum on 32 bits: bit 31 = "a row starts here", bits 0-30 the
// count since (a is the earlier operand)
DA_HD uint32_t seg_combine(uint32_t a, uint32_t b) {
  return (b >> 31) ? b : (a & 0x80000000u) | ((a + b) & 0x7FFFFFFFu);
}
// per-lane scan element: bits 0-15 rows, 16-31 values, 32-62 the segmented
// delimiter count (seg_combine), 63 its flag
struct CsvScanOp {
  DA_HD uint64_t operator()(uint64_t a, uint64_t b) const {
    const uint64_t lo = ((a & 0xFFFFFFFFull) + (b & 0xFFFFFFFFull)) & 0xFFFFFFFFull;
    return lo | ((uint64_t)seg_combine((uint32_t)(a >> 32), (uint32_t)(b >> 32)) << 32);
  }
};

// Look-back with the four slots above: rows and values are sums; the tail is
// segmented (walking back, it stops at the nearest tile holding a row start).
// Record word 0 = status | rows | values << 15 | tail << 30 | flag << 45;
// words 1..3 = inclusive rows, values, and the carry out of the tile
// (delimiters since its last row start, or through it).
template <class BK>
DA_HDF uint32_t csv_look_back(uint64_t *lb, uint32_t k, const uint32_t cnt[4], uint32_t *gate, TileCommon &c,
                              BK &bk, uint64_t *segc) {
  const uint32_t lane = bk.tid();
  uint64_t j = k;
  uint32_t spins = 0, rounds = 0;
  uint64_t rows = 0, vals = 0, tail = 0;
  bool seg_done = false;
  bool done = k == 0;
  while (!done) {
    ++rounds;
    // status word and the three prefix words of predecessor j-1-lane (before
    // tile 0: an inclusive 0); the prefix stands when all three carry kMark
    uint64_t s = 0, w[3] = {kMark, kMark, kMark};
    if (lane < j) {
      const uint64_t *rec = lb + (j - 1 - lane) * kCsvLbWords;
      s = load_agent_u64(const_cast<uint64_t *>(rec));
#pragma unroll
      for (int i = 0; i < 3; ++i) w[i] = load_agent_u64(const_cast<uint64_t *>(rec) + 1 + i);
    }
    const bool inc = (w[0] & w[1] & w[2] & kMark) != 0;
    const uint64_t zero = bk.ballot(!inc && (s >> 62) == 0), incl = bk.ballot(inc);
    const uint32_t fz = zero ? (uint32_t)ctz64(zero) : 64u, fi = incl ? (uint32_t)ctz64(incl) : 64u;
    const uint32_t tagg = fi < fz ? fi : fz;
    const uint64_t mine = lane < tagg ? s : 0ull;
    rows += bk.wave_sum((uint32_t)(mine & 0x7FFFu));
    vals += bk.wave_sum((uint32_t)((mine >> 15) & 0x7FFFu));
    if (!seg_done) {
      const uint64_t flg = bk.ballot(lane < tagg && ((s >> 45) & 1u));
      const uint32_t f = flg ? (uint32_t)ctz64(flg) : 64u;  // nearest tile with a row start
      tail += bk.wave_sum(lane < tagg && lane <= f ? (uint32_t)((s >> 30) & 0x7FFFu) : 0u);
      seg_done = f < 64u;
    }
    done = fi < fz;
    if (done) {
      rows += bk.shfl(w[0] & ~kMark, (int)fi);
      vals += bk.shfl(w[1] & ~kMark, (int)fi);
      const uint64_t t2 = bk.shfl(w[2] & ~kMark, (int)fi);
      if (!seg_done) tail += t2;
    } else {
      j -= tagg;
      if (tagg == 0) {
        if (++spins > kSpinLimit) {
          if (lane == 0) atomic_or_u32(gate, 2u);
          done = true;
        }
        spin_pause();
      }
    }
  }
  if (lane == 0) {
    c.base[Q_ROWS] = rows;
    c.base[Q_VALS] = vals;
    *segc = tail;
  }
  uint64_t *rec = lb + (uint64_t)k * kCsvLbWords;
  if (lane < 3) {
    const uint64_t v = lane == 0 ? rows + cnt[0] : lane == 1 ? vals + cnt[1]
                                                           : (cnt[3] ? (uint64_t)cnt[2] : tail + cnt[2]);
    store_agent_u64(rec + 1 + lane, kMark | v);
  }
  return rounds;
}

struct Tile {
  const FastCsvArgs *a;
  Shared *sh;
  uint64_t tlo, thi;
  DA_HD uint64_t next_cs(uint64_t p) const {  // first chunk start > p
    for (uint32_t i = 0; i < sh->c.ncs; ++i)
      if (sh->c.csl[i] > p) return sh->c.csl[i];
    return sh->c.cnext;
  }
  DA_HD bool is_cs(uint64_t p) const {
    for (uint32_t i = 0; i < sh->c.ncs; ++i)
      if (sh->c.csl[i] == p) return true;
    return p == sh->c.cnext;
  }
};

// strtoll(p, &e, 0) (csv_parser.h:101-105) on a token of the grammar: [sign]
// digits, decimal -- a leading 0 followed by a digit is octal and goes to the
// byte decoder, as do more than 8 digits (saturation); *ok = false then.
// M: bit i set when window byte i is not '0'..'9' (16 bits)
DA_HD int64_t wint64m(const uint32_t w[4], uint32_t M, bool *ok) {
  const uint32_t b0 = w[0] & 0xFFu;
  const bool neg = b0 == '-';
  const uint32_t s = (neg || b0 == '+') ? 1u : 0u;
  const uint32_t L = (uint32_t)ctz32((M & ~s) | 0x10000u) - s;
  const uint32_t d0 = byte_of(w, s);
  *ok = L >= 1u && L <= 8u && !(d0 == '0' && L > 1u);
  if (!*ok) return 0;
  const int64_t v = (int64_t)digits_ra(w, s, L);
  return neg ? -v : v;
}

// MODE 1: count only (size query); MODE 2: parse and write.
// SP: label / weight columns may be set (a separate kernel, so the plain
// form carries none of their code); blanks are outside its grammar.
// VT: 0 float values (ParseFloat), 1 integer values (strtoll base 0, int32 /
// int64 by a.vtype; no label column, the weight column is a plain column for
// integer DTypes, csv_parser.h:111-114).
template <int MODE, bool SP, int VT, class BK>
DA_HDF void tile(const FastCsvArgs &a, Shared &sh, BK &bk, uint32_t k) {
  // Tile k = workgroup k (its blockIdx).  The look-back needs every tile's
  // predecessors to become resident eventually; workgroups are dispatched in
  // index order on every XCD, so the least unstarted tile's XCD only holds
  // lower tiles, which finish.  (A device-wide ticket counter gave the same
  // guarantee for any dispatch order but saturates near 88 grabs/us -- it
  // capped the 131k-tile launch at ~1.5 ms.)  Should a predecessor ever not
  // publish, kSpinLimit bounds the wait and the exact kernels take over.
  const int tid = bk.tid();
  constexpr bool JK = VT == 0 && !SP;  // junk fields in the grammar (csv_junk_byte)
  if (a.skip_if_gated && *a.gate) return;  // fill phase after an exact-path count: block-uniform
  FAST_STAMP(k, 0);
  FAST_STAMP(k, 1);
  Tile t;
  t.a = &a;
  t.sh = &sh;
  t.tlo = (uint64_t)k * kTile;
  t.thi = mn<uint64_t>(t.tlo + kTile, a.n);
  StageRegs sr;
#if defined(FSVM_GLDS) && defined(__HIP_DEVICE_COMPILE__)
  stage_issue_lds(a.text, a.n, t.tlo, sr, sh.c, bk);  // text loads first: the chunk search overlaps them
#else
  stage_issue(a.text, a.n, t.tlo, sr, bk);  // text loads first: the chunk search overlaps them
#endif
  ChunkProbe cp;  // wave 0: the window load stays in flight through classification
  if (tid < kWave) cp = chunk_list_begin(a.cs, a.nchunk, t.tlo, bk);
  if (tid == 0) {
    sh.u.m.d[0] = sh.u.m.n[0] = sh.u.m.l[0] = 0;
    sh.nlab = sh.nfirst = 0;
    sh.junk = 0;
  }
  for (int i = tid; i < kClsEntries; i += kFThreads) sh.cls[i] = class_of_csv((uint32_t)i, a.delim, !SP, JK);
  init_dec_tables(sh.dt, bk);
  stage_commit(a.text, a.n, t.tlo, sr, sh.c, bk);
  bk.sync();
  // ---- classify: segment tid -> slot tid+1; lanes 0..15 also one dword
  // each of the 64 bytes before the tile -> slot 0
  uint32_t bad = 0;
  uint64_t J = 0;  // junk bytes of my segment (JK)
  {
    Masks m = classify64_lut(sh.c.text + kPre + tid * kSegB, sh.cls);
    if (JK) {  // split the junk class (digit + newline) off the planes
      J = m.g & m.n;
      m.g &= ~J;
      m.n &= ~J;
      if (J) sh.junk = 1;
    }
    sh.gw[2 * tid] = (uint32_t)m.g;
    sh.gw[2 * tid + 1] = (uint32_t)(m.g >> 32);
    if (tid == (kFWaves > 1 ? kWave : kFThreads - 1)) {  // digits of the 16 bytes after the tile (windows of my last values)
      uint32_t g = 0;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        uint32_t x;
        memcpy(&x, sh.c.text + kPre + kTile + 4 * i, 4);
        const Nib b = classify_dword_lut(x, sh.cls);  // (bytes >= 0x80: no digit)
        g |= (JK ? b.g & ~b.n : b.g) << (4 * i);
        if (JK && ((b.g & b.n) | b.hi)) sh.junk = 1;
      }
      sh.gw[2 * kFThreads] = g;
    }
    sh.u.m.d[tid + 1] = m.d;
    sh.u.m.n[tid + 1] = m.n;
    sh.u.m.l[tid + 1] = m.c;
    // bytes past the end of the text are staged as blanks: judge valid bytes only
    const uint64_t P0 = t.tlo + (uint64_t)tid * kSegB;
    const uint64_t vmask = P0 >= a.n ? 0ull : (a.n - P0 >= 64 ? ~0ull : ((1ull << (a.n - P0)) - 1));
    bad = (m.g & ~m.d & vmask) != 0;
    if (tid < 16 && t.tlo > 0) {
      uint32_t x;
      memcpy(&x, sh.c.text + (kPre - kSegB) + 4 * tid, 4);
      const Nib b = classify_dword_lut(x, sh.cls);  // (bytes >= 0x80: planes clear -- junk for JK)
      const uint32_t jb = JK ? b.g & b.n : 0u;
      if (jb | (JK ? b.hi : 0u)) sh.junk = 1;
      if (b.hi && a.delim >= 0x80u) bad = 1;  // (a delimiter >= 0x80 in the pre-halo: exact kernels)
      atomic_or_u64(&sh.u.m.d[0], (uint64_t)b.d << (4 * tid));
      atomic_or_u64(&sh.u.m.n[0], (uint64_t)(b.n & ~jb) << (4 * tid));
      atomic_or_u64(&sh.u.m.l[0], (uint64_t)b.c << (4 * tid));
    }
  }
  if (tid < kWave) chunk_list_end(a.cs, a.nchunk, t.tlo, t.thi, cp, sh.c, bk);
  bk.sync();
  if (tid == 0) bad |= sh.c.toomany;
  // ---- rows, fields, tokens of my segment
  const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
  uint64_t RS = 0, T = 0, L = 0;
  if (P < a.n) {
    const int nv = (int)mn<uint64_t>(64, a.n - P);
    const uint64_t valid = nv == 64 ? ~0ull : ((1ull << nv) - 1);
    const uint64_t N = sh.u.m.n[tid + 1], D = sh.u.m.d[tid + 1];
    L = sh.u.m.l[tid + 1] & valid;
    uint64_t S = 0;  // chunk starts: a "newline before" for the row rule, a field barrier
    for (uint32_t i = 0; i < sh.c.ncs; ++i) {
      const uint64_t x = sh.c.csl[i];
      if (x >= P && x < P + (uint64_t)nv) S |= 1ull << (x - P);
    }
    const uint64_t n1 = sh.u.m.n[tid], l1 = sh.u.m.l[tid];
    RS = ~N & valid & ((N << 1) | (n1 >> 63) | S);
    const uint64_t FSd = ((L << 1) | (l1 >> 63)) & ~N & ~S & valid;
    uint64_t F = RS | FSd;  // field starts
    if (JK && sh.junk) {  // block-uniform
      // a UTF-8 BOM at a row start (IgnoreUTF8BOM, text_parser.h:83-102):
      // the row's first field starts after it -- in this segment, or in the
      // next one for a BOM in the last three bytes (that segment sees it
      // below).  A BOM whose next byte is a newline (the reference's line end
      // search then starts past it), lies beyond the text, or that holds or
      // ends at a chunk start goes to the exact kernels.
      const uint8_t *seg = sh.c.text + kPre + tid * kSegB;
      auto is_bom = [&](int i) {  // staged bytes seg[i..i+2]
        return seg[i] == 0xEFu && seg[i + 1] == 0xBBu && seg[i + 2] == 0xBFu;
      };
      for (uint64_t m = RS & J; m; m &= m - 1) {
        const uint32_t i = (uint32_t)ctz64(m);
        if (!is_bom((int)i)) continue;
        const uint64_t bit = m & (0 - m);
        F &= ~bit;
        if (i <= 60u) {
          if ((((N | ~valid | S) >> (i + 1u)) & 7u) != 0u) bad = 1;
          else F |= bit << 3;
        }
      }
      // a BOM that began at a row start in the last three bytes before P
      for (int i = -3; i < 0; ++i) {
        const uint64_t x = P + (uint64_t)(int64_t)i;
        if (P < 3 || !is_bom(i)) continue;
        // chunk starts before the tile are known only as cfloor (the last one
        // <= tlo): one inside [x, tlo] leaves the question to the exact kernels
        if (x < t.tlo && sh.c.cfloor >= x) {
          bad = 1;
          continue;
        }
        const uint32_t pb = seg[i - 1];
        const bool cs_x = x == sh.c.cfloor || t.is_cs(x);
        if (!(cs_x || pb == '\n' || pb == '\r')) continue;  // not a row start: junk
        const uint32_t j = (uint32_t)(i + 3);  // the field start in this segment (0..2)
        bool cs_in = (S & ((2ull << j) - 1)) != 0;  // a chunk start inside the BOM or right after it
        for (uint64_t y = x + 1; y < P; ++y) cs_in = cs_in || y == sh.c.cfloor || t.is_cs(y);
        if (cs_in || (((N | ~valid) >> j) & 1u)) bad = 1;
        else F |= 1ull << j;
      }
    }
    if constexpr (SP) {
      T = F & D;
    } else {
      // Blanks (' ', '\t', class 0): ParseFloat / strtoll skip them at a field
      // start (strtonum.h:95-264), so a field's token is the first non-blank
      // byte after its start -- found by a carry through the blank run that
      // begins at a blank field start (a field start always begins its run).
      // The run carried in from the segment before when that one ends in
      // blanks which follow a delimiter, a newline or a chunk start.
      // A chunk start ends a blank run (the decoder would read past the
      // chunk: bad) and, when blank, starts a run of its own (X).
      const uint64_t B = ~(D | N | L | J) & valid, Bs = B & ~S, X = F & B & S;
      uint32_t cin = 0;
      if (P > 0 && !(S & 1u)) {
        uint64_t nb1 = sh.u.m.d[tid] | n1 | l1;  // non-blank bytes of the segment before
        if (JK && !(nb1 >> 63) && sh.junk) {
          // its junk bytes are not in the planes: its trailing blanks from its bytes
          const uint8_t *prev = sh.c.text + kPre + (tid - 1) * kSegB;
          int j = 63;
          while (j >= 0 && (prev[j] == ' ' || prev[j] == '\t')) --j;
          if (j >= 0) nb1 |= 1ull << j;
        }
        if (!(nb1 >> 63)) {
          if (!nb1) {
            bad = 1;  // 64 blanks in a row: beyond this carry, the exact kernels take it
          } else {
            const uint32_t j = 63u - (uint32_t)clz64(nb1);
            const uint64_t x0 = P - 64u + j + 1u;  // the trailing run's first byte
            bool cs = x0 <= sh.c.cfloor && sh.c.cfloor < P;  // a chunk (and row) starts inside the run
            for (uint32_t i = 0; i < sh.c.ncs; ++i) cs = cs || (x0 <= sh.c.csl[i] && sh.c.csl[i] < P);
            cin = (((n1 | l1) >> j) & 1u) || cs ? 1u : 0u;
            if (JK && !cin && j >= 2u && sh.junk) {
              // a UTF-8 BOM at a row start right before the run: the row's
              // first field starts the run (IgnoreUTF8BOM, csv_parser.h:83)
              const uint8_t *prev = sh.c.text + kPre + (tid - 1) * kSegB;
              const uint64_t xb = P - 64u + j - 2u;  // the BOM's first byte
              if (prev[j - 2] == 0xEFu && prev[j - 1] == 0xBBu && prev[j] == 0xBFu) {
                const uint32_t pb = xb > 0 ? (uint32_t)gbyte(a.text, xb - 1) : (uint32_t)'\n';
                if (pb == '\n' || pb == '\r' || xb == sh.c.cfloor || t.is_cs(xb)) cin = 1u;
              }
            }
          }
        }
      }
      uint32_t c1, c2;
      const uint64_t land = (add_carry(Bs, F & Bs, cin, &c1) | add_carry(Bs, X << 1, 0u, &c2)) & ~Bs;
      // the run reaches a newline, a chunk start or the text end: ParseFloat /
      // strtoll would skip on into the next line (csv_parser.h:99-105)
      if (land & (N | S | ~valid)) bad = 1;
      const uint32_t cout = c1 | c2 | (uint32_t)(X >> 63);
      if (cout && (P + 64 >= a.n || t.is_cs(P + 64))) bad = 1;
      if constexpr (VT == 0) {
        // a blank field ending at a delimiter is ParseFloat's 0 (it consumed
        // the blanks), and so is one whose blanks run into junk (or into
        // "inf" / "nan": their value)
        T = (F & D) | (land & (D | L | J));
        if (JK && sh.junk) {  // block-uniform
          // junk field starts: no value, unless ParseFloat reads one there --
          // the 'f' suffix (the value 0: a token), inf / nan (their values,
          // inf_nan_of; also after a sign: "-inf" is a number-char token),
          // "nan(chars)" (NaN; dec_float checks the literal -- round 6: it
          // no longer sends the input to the exact kernels)
          const uint8_t *seg = sh.c.text + kPre + tid * kSegB;
          auto nv = [&](uint64_t i) { return t.next_cs(P + i) - (P + i); };  // bytes to the chunk end
          for (uint64_t m = F & J; m; m &= m - 1) {
            const uint32_t i = (uint32_t)ctz64(m), k = csv_inf_nan(seg + i, nv(i));
            if (k != 0u || (seg[i] | 0x20u) == 'f') T |= m & (0 - m);
          }
        }
      } else {
        // strtoll consumed nothing unless a digit follows the optional sign:
        // the field is then a missing value (csv_parser.h:115-118)
        const uint64_t C = (F & D) | (land & D);
        const uint64_t G = (uint64_t)sh.gw[2 * tid] | ((uint64_t)sh.gw[2 * tid + 1] << 32);
        // next byte a digit of the same chunk (strtoll stops at the chunk end)
        const uint64_t Gn = ((G >> 1) | ((uint64_t)(sh.gw[2 * tid + 2] & 1u) << 63)) & ~(S >> 1) &
                            ~((uint64_t)t.is_cs(P + 64) << 63);
        T = C & G;
        for (uint64_t m = C & ~G & Gn; m; m &= m - 1) {
          const uint32_t b = sh.c.text[kPre + tid * kSegB + ctz64(m)];
          if (b == '-' || b == '+') T |= m & (0 - m);
        }
      }
    }
  }
  if (bad) atomic_or_u32(&sh.c.bad, 1u);
  // segmented delimiter count of my segment: since my last row start, or all
  const uint32_t has_rs = RS != 0;
  const uint32_t lastr = has_rs ? 63u - (uint32_t)clz64(RS) : 0u;
  const uint32_t tailc = (uint32_t)popc64(has_rs ? (L & (~0ull << lastr)) : L);
  const uint64_t mine = (uint64_t)popc64(RS) | ((uint64_t)popc64(T) << 16) | ((uint64_t)tailc << 32) |
                        ((uint64_t)has_rs << 63);
  uint64_t totp;
  const uint64_t ex = bk.exclusive(mine, (uint64_t)0, CsvScanOp(), &totp);
  const uint32_t nR = (uint32_t)(totp & 0xFFFF), nT = (uint32_t)((totp >> 16) & 0xFFFF);
  const uint32_t cnt4[4] = {nR, nT, (uint32_t)((totp >> 32) & 0x7FFFFFFF), (uint32_t)(totp >> 63)};
  if (tid == 0) {
    uint64_t *rec = a.lb + (uint64_t)k * kCsvLbWords;
    const uint64_t packed = (uint64_t)cnt4[0] | ((uint64_t)cnt4[1] << 15) | ((uint64_t)cnt4[2] << 30) |
                            ((uint64_t)cnt4[3] << 45);
    if (k == 0) {
      store_agent_u64(rec + 1, kMark | cnt4[0]);
      store_agent_u64(rec + 2, kMark | cnt4[1]);
      store_agent_u64(rec + 3, kMark | cnt4[2]);
    } else {
      store_agent_u64(rec, kSAgg | packed);
    }
    if (sh.c.bad) atomic_or_u32(a.gate, 1u);
  }
  const bool one_chunk = sh.c.ncs == 0;
  const bool junk_tile = JK && sh.junk != 0;  // inf / nan tokens possible (block-uniform)
  // the value of the token at q: float (VT 0) or the strtoll result (VT 1)
  using Val = typename std::conditional<VT == 0, float, int64_t>::type;
  auto dec_float = [&](uint64_t q) -> Val {
    const uint32_t o = (uint32_t)(q - t.tlo);  // non-digit flags of the window from the digit plane
    const uint32_t M = ~funnel(sh.gw[(o >> 5) + 1], sh.gw[o >> 5], o & 31u);
    const uint64_t lim = one_chunk ? sh.c.cnext : t.next_cs(q);
    bool ok = false;
    Val v = 0;
    if (q + 16 <= lim) {
      const W16 wq = win_at(sh.c.text, t.tlo, q);
      const uint32_t w4[4] = {(uint32_t)wq.lo, (uint32_t)(wq.lo >> 32), (uint32_t)wq.hi, (uint32_t)(wq.hi >> 32)};
      if constexpr (VT == 0) {
        v = wfloat32m(w4, M, sh.dt, &ok);
        if (junk_tile) {  // inf / nan letters after the optional sign (rare: a branch, not a select)
          const uint32_t b0 = w4[0] & 0xFFu, sg = (b0 == '-' || b0 == '+') ? 1u : 0u, l = (w4[0] >> (8 * sg)) & 0xFFu;
          float x;
          if (((l | 0x20u) == 'i' || (l | 0x20u) == 'n') && inf_nan_of(w4, &x)) v = x;
          // "nan(chars)": the byte decoder checks the literal (strtonum.h:157-165)
          if ((l | 0x20u) == 'n' && byte_of(w4, sg + 3u) == '(') ok = false;
        }
      } else {
        v = wint64m(w4, M, &ok);
      }
    }
    if (!ok) {
      GSrc src{a.text, lim};
      uint64_t e;
      if constexpr (VT == 0) {
        bool nan_err = false;
        v = parse_float(src, q, &e, &nan_err);
        if (MODE == 2 && nan_err) {  // "Invalid NAN literal", at the field's start (csv_core.h csv_line_seq)
          uint64_t f = q;
          for (uint32_t b; f > 0 && (b = gbyte(a.text, f - 1)) != a.delim && !is_nl(b) && is_space(b);) --f;
          raise_error(a.err, E_NAN_LITERAL, f);
        }
      } else {
        v = c_strtoll(src, q, 0, &e);
      }
    }
    return v;
  };
  // the value array: DType float, or int32 / int64 (a.vtype 1 / 2)
  auto put_val = [&](uint64_t g, Val v) {
    if constexpr (VT == 0) {
      reinterpret_cast<float *>(a.value)[g] = v;
    } else {
      if (a.vtype == 1) reinterpret_cast<int32_t *>(a.value)[g] = (int32_t)v;
      else reinterpret_cast<int64_t *>(a.value)[g] = v;
    }
  };
#ifndef FCSV_KB
#define FCSV_KB 4
#endif
  constexpr int kB = FCSV_KB;  // tokens decoded before the look-back
  Val vb[kB > 0 ? kB : 1];
  uint64_t mT = T;
  const bool has_lab = SP && a.label_col >= 0, has_w = SP && a.weight_col >= 0;
  const bool has_sp = has_lab || has_w;  // special columns: tokens stored per token, not listed
  const uint64_t nsp = (has_lab ? 1u : 0u) + (has_w ? 1u : 0u);
  // Without a label column the tokens go to an LDS list in output order
  // (svm_fast.h's run lists): each wave decodes ceil(tokens / 256) values per
  // thread and consecutive lanes store consecutive values and column ids.  The
  // list reuses the planes' LDS (the block scan's barriers ordered their last
  // reads); a tile with more tokens than fit is done in passes.
  const uint32_t exT = (uint32_t)((ex >> 16) & 0xFFFF);
  const uint64_t sexl = ex >> 32;  // segmented exclusive delimiter count (flag in bit 31)
  uint32_t np = 1, mypass = 0, pe0 = nT;
  auto build = [&](uint32_t s0, uint32_t e0) {  // my tokens into the list of the pass [s0, e0)
    uint32_t x = exT - s0;
    const uint32_t o0 = (uint32_t)tid * kSegB;
    for (uint64_t m = T; m; m &= m - 1) {
      const uint32_t b = (uint32_t)ctz64(m);
      const uint64_t below = (1ull << b) - 1, r = RS & (below | (1ull << b));
      uint32_t col, carried = 0;
      if (r) {
        col = (uint32_t)popc64(L & below & (~0ull << (63 - clz64(r))));
      } else {
        col = (uint32_t)(sexl & 0x7FFFFFFFu) + (uint32_t)popc64(L & below);
        carried = (sexl >> 31) ? 0u : 1u;
      }
      sh.u.lst[x++] = (o0 + b) | ((col & ((1u << kColBits) - 1)) << 14) | (carried << 31);
    }
    (void)e0;
  };
  if (MODE == 2 && !has_sp) {
    if (nT > kPassTokens) {  // block-uniform: several passes
      const uint32_t own = (uint32_t)popc64(T);
      mypass = exT / kPassTokens;
      if (tid == kFThreads - 1 || (exT + own) / kPassTokens != mypass) sh.pend[mypass] = exT + own;
      if (tid == kFThreads - 1) sh.npass = mypass + 1;
      bk.sync();
      np = sh.npass;
      pe0 = sh.pend[0];
    }
    if (mypass == 0) build(0, pe0);
    bk.sync();
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const uint32_t j = (uint32_t)tid + (uint32_t)u * kFThreads;
      vb[u] = 0;
      if (j < pe0) vb[u] = dec_float(t.tlo + (sh.u.lst[j] & 0x3FFFu));
    }
  } else if (MODE == 2) {
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      vb[u] = 0;
      if (mT) {
        vb[u] = dec_float(P + ctz64(mT));
        mT &= mT - 1;
      }
    }
  }
  // ---- decoupled look-back by wave 0
  if (tid < kWave) csv_look_back(a.lb, k, cnt4, a.gate, sh.c, bk, &sh.segc);
#ifdef DMLC_AMD_VALVE_TEST  // test-only build (lib/variants): the write pass of tile 1 hands over
  if (MODE == 2 && k == 1 && tid == 0) atomic_or_u32(a.gate, 2u);
#endif
  bk.sync();
  const uint64_t bRows = sh.c.base[Q_ROWS], bVal = sh.c.base[Q_VALS], tcarry = sh.segc;
  // With a label column (csv_parser.h:111-112) the field at column label_col
  // of every row is its label and the other fields keep their column minus one
  // past it.  The single pass assumes every row holds exactly one non-empty
  // label field (then labels = rows and a token's value rank is its token rank
  // minus the labels before it) and checks that assumption: the tiles sum
  // (label tokens - rows) and, for label_col 0 (where a row without a
  // delimiter is the reference's fatal "Delimiter not found",
  // csv_parser.h:128-132), (first delimiters - rows) into labsum; a nonzero
  // sum sets the gate after this kernel and the exact kernels redo the input.
  const uint64_t Lc = has_lab ? (uint64_t)a.label_col : ~0ull;
  const uint64_t Wc = has_w ? (uint64_t)a.weight_col : ~0ull;  // weight_column likewise (:113-114)
  const uint64_t eR = bRows + (ex & 0xFFFF), eT = bVal + ((ex >> 16) & 0xFFFF);
  const uint64_t sex = ex >> 32;  // segmented exclusive (flag in bit 31)
  const uint64_t carry = (sex >> 31) ? (sex & 0x7FFFFFFFull) : tcarry + (sex & 0x7FFFFFFFull);
  auto col_of = [&](uint32_t b) -> uint64_t {  // delimiters since the row start, token at bit b
    const uint64_t below = (1ull << b) - 1;
    const uint64_t r = RS & (below | (1ull << b));
    if (r) return (uint64_t)popc64(L & below & (~0ull << (63 - clz64(r))));
    return carry + popc64(L & below);
  };
  if (has_sp) {
    uint32_t nl = 0, nf = 0, nw = 0;
    if (has_lab && Lc == 0) {
      // column-0 labels are the row starts holding a token; a row's first
      // delimiter is the first after its start (row starts are sparse)
      nl = (uint32_t)popc64(RS & T);
      const uint64_t fr = RS & (0ull - RS);
      if (carry == 0 && (L & (fr ? fr - 1 : ~0ull))) nf = 1;  // the row carried in has none yet
      for (uint64_t rs = RS; rs; rs &= rs - 1) {
        const uint64_t r = rs & (0ull - rs), nx = (rs & (rs - 1)) & (0ull - (rs & (rs - 1)));
        nf += (L & (nx ? nx - 1 : ~0ull) & ~(r | (r - 1))) != 0;
      }
    } else if (has_lab) {
      for (uint64_t m = T; m; m &= m - 1) nl += col_of((uint32_t)ctz64(m)) == Lc;
    }
    if (has_w)
      for (uint64_t m = T; m; m &= m - 1) nw += col_of((uint32_t)ctz64(m)) == Wc;
    if (nl | nw) atomic_add_u32(&sh.nlab, nl | (nw << 16));
    if (nf) atomic_add_u32(&sh.nfirst, nf);
    bk.sync();
    // only tiles whose rows straddle their ends add, into one of kLabShards
    // lines (one device-wide counter saturates near 88 atomics/us,
    // MI355X_MICROARCH.md "dequeue")
    if (tid == 0) {
      uint64_t *sum = a.labsum + (uint64_t)(k % kLabShards) * 8;
      const uint32_t tl = sh.nlab & 0xFFFFu, tw = sh.nlab >> 16;
      if (has_lab && tl != nR) atomic_add_u64(&sum[0], (uint64_t)tl - (uint64_t)nR);
      if (has_w && tw != nR) atomic_add_u64(&sum[2], (uint64_t)tw - (uint64_t)nR);
      if (Lc == 0 && sh.nfirst != nR) atomic_add_u64(&sum[1], (uint64_t)sh.nfirst - (uint64_t)nR);
    }
  }
  if (k + 1 == a.ntiles && tid == 0) {
    const uint64_t rows = bRows + nR, vals = bVal + nT - rows * nsp;
    a.res[C_ROWS] = rows;
    a.res[C_INDEX] = vals;
    a.res[C_VALUE] = vals;
    a.res[C_WEIGHT] = has_w ? rows : 0;
    a.res[C_QID] = 0;
    a.res[C_LABEL] = has_lab ? rows : 0;
    a.res[C_FIELD] = 0;
    if (MODE == 2 && a.offset && rows < a.cap[C_ROWS] + 1) a.offset[rows] = vals;
  }
  if (MODE != 2) return;

  // ---- stores: values and column indices (labels), then row offsets
  auto put = [&](uint64_t g, uint32_t b, Val v) {  // g: global token rank
    const uint64_t c = col_of(b);
    const uint64_t sp_before = (c > Lc ? 1u : 0u) + (c > Wc ? 1u : 0u);
    if (has_sp) {
      const uint64_t bit = 1ull << b;
      const uint64_t row = eR + popc64(RS & ((bit - 1) | bit)) - 1;  // this token's row
      if (c == Lc) {
        if (row < a.cap[C_LABEL]) a.label[row] = v;
        else raise_error(a.err, E_CAPACITY, P + b);
        return;
      }
      if (c == Wc) {
        if (row < a.cap[C_WEIGHT]) a.weight[row] = v;
        else raise_error(a.err, E_CAPACITY, P + b);
        return;
      }
      g -= row * nsp + sp_before;  // labels and weights before this token
    }
    const uint64_t ci = c - sp_before;
    if (g < a.cap[C_VALUE] && g < a.cap[C_INDEX]) {
      put_val(g, v);
      if (a.wide) reinterpret_cast<uint64_t *>(a.index)[g] = ci;
      else reinterpret_cast<uint32_t *>(a.index)[g] = (uint32_t)ci;
    } else {
      raise_error(a.err, E_CAPACITY, P + b);
    }
  };
  if (!has_sp) {
    // list entry j of the pass starting at token s0: value rank bVal + s0 + j
    auto put_tok = [&](uint64_t g, uint32_t e, Val v) {
      const uint64_t ci = ((e >> 14) & ((1u << kColBits) - 1)) + ((e >> 31) ? tcarry : 0u);
      if (g < a.cap[C_VALUE] && g < a.cap[C_INDEX]) {
        put_val(g, v);
        if (a.wide) reinterpret_cast<uint64_t *>(a.index)[g] = ci;
        else reinterpret_cast<uint32_t *>(a.index)[g] = (uint32_t)ci;
      } else {
        raise_error(a.err, E_CAPACITY, t.tlo + (e & 0x3FFFu));
      }
    };
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const uint32_t j = (uint32_t)tid + (uint32_t)u * kFThreads;
      if (j < pe0) put_tok(bVal + j, sh.u.lst[j], vb[u]);
    }
    for (uint32_t p = 0; p < np; ++p) {
      const uint32_t s0 = p ? sh.pend[p - 1] : 0u, e0 = p ? sh.pend[p] : pe0;
      if (p) {  // block-uniform
        bk.sync();
        if (mypass == p) build(s0, e0);
        bk.sync();
      }
      for (uint32_t j = (uint32_t)tid + (p ? 0u : (uint32_t)kB * kFThreads); j < e0 - s0; j += kFThreads) {
        const uint32_t e = sh.u.lst[j];
        put_tok(bVal + s0 + j, e, dec_float(t.tlo + (e & 0x3FFFu)));
      }
    }
  } else {
    uint64_t m = T;
    uint64_t g = eT;
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      if (m) {
        put(g, (uint32_t)ctz64(m), vb[u]);
        m &= m - 1;
        ++g;
      }
    }
    for (; m; m &= m - 1, ++g) {
      const uint32_t b = (uint32_t)ctz64(m);
      put(g, b, dec_float(P + b));
    }
  }
  {
    uint64_t r = eR;
    for (uint64_t m = RS; m; m &= m - 1, ++r) {
      const int b = ctz64(m);
      if (r < a.cap[C_ROWS]) a.offset[r] = eT + popc64(T & ((1ull << b) - 1)) - r * nsp;
      else raise_error(a.err, E_CAPACITY, P + b);
    }
  }
  // ---- per-chunk exclusive counts at each chunk start in my segment
  if (a.chunk_tab) {
    for (uint32_t i = 0; i < sh.c.ncs; ++i) {
      const uint64_t x = sh.c.csl[i];
      if (x < P || x >= P + kSegB || x >= t.thi) continue;
      const uint64_t below = (1ull << (x - P)) - 1;
      uint64_t *row = a.chunk_tab + (uint64_t)(sh.c.c_first + i) * 8;
      const uint64_t rows = eR + popc64(RS & below);
      row[C_ROWS] = rows;
      row[C_INDEX] = row[C_VALUE] = eT + popc64(T & below) - rows * nsp;
      row[C_WEIGHT] = has_w ? rows : 0;
      row[C_QID] = 0;
      row[C_LABEL] = has_lab ? rows : 0;
      row[C_FIELD] = 0;
    }
  }
}

}  // namespace fcsv
}  // namespace dmlc_amd
