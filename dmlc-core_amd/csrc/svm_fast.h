// svm_fast.h -- the single-pass libsvm tile body for the "uniform grammar":
// every byte is a digitchar, blank, ':' or newline (no '#', no "qid:", no
// letters besides e/E, no dangling "x:" at a line end, no "a:b:c" chains),
// which is what libsvm files written by tools look like.  Inside that grammar
// the role of every digitchar run of LibSVMParser::ParseBlock
// (src/data/libsvm_parser.h:85-172, ParsePair include/dmlc/strtonum.h:667-703)
// is a function of the gap in front of it and of the previous run's role:
//
//   gap holds a newline / chunk start             -> label   (row)
//   gap holds ':'  and the previous run is a label -> weight
//   gap holds ':'  otherwise                       -> value
//   otherwise                                      -> index
//
// so the whole parse is bitmask arithmetic on 64-byte segments (one per
// thread) plus a short look-back to the previous run.  The kernel is single
// pass: a tile (16 KiB, 256 threads) classifies its bytes, publishes its
// counts, finds its output base by decoupled look-back over earlier tiles,
// then each thread decodes its own segment's runs role by role (SWAR digit
// conversion from LDS) and stores them.  Any byte or structure outside the grammar
// sets the gate word; the launcher then runs the exact tile kernels
// (libsvm_core.h) instead, so results are always the reference's.
//
// Written once against a block policy BK {tid, sync, exclusive} so the GPU
// kernel (libsvm.hip) and the test-only CPU emulator (tests/emu) share it.
#pragma once
#include "fast_common.h"

namespace dmlc_amd {
namespace fsvm {
using namespace fast;

enum : uint32_t { R_NONE = 0, R_L = 1, R_K = 2, R_I = 3, R_Q = 4 };

// After the single-pass kernel (qid_fix_kernel, and the emulator): its qid
// runs stand only when every row has one -- qid[r] is then row r's and each
// chunk's qid count its row count; a mix of rows with and without a qid goes
// to the exact kernels.  Returns true when the chunk rows' qid counts must be
// set to their row counts.
DA_HD bool qid_decide(uint64_t total, uint64_t *res, uint32_t *gate) {
  if (*gate || total == 0) return false;
  if (total != res[C_ROWS]) {
    *gate |= 1u;
    return false;
  }
  res[C_QID] = total;
  return true;
}

// ---- indexing_mode < 0 (libsvm_parser.h:165-171; libfm_parser.h:133-143)
// on the single-pass path: the write pass stores the ids as read and marks
// each ParseBlock unit holding a 0 id (umin[u] = 0, libfm: among fields and
// indices; ~0 otherwise); afterwards every id of a unit without a 0 id (its
// minimum is > 0) drops by one.  The units' index ranges are the chunk table's index column (tab,
// nunit rows of 8, complete after finish_kernel).  Entries [lo, hi) of
// the index array (and the field array, when set), stride `step` from lo.
DA_HD int unit_of_entry(const uint64_t *tab, int nunit, uint64_t i) {  // last unit whose range starts <= i
  int lo = 0, hi = nunit;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (tab[(uint64_t)mid * 8 + C_INDEX] <= i) lo = mid;
    else hi = mid;
  }
  return lo;
}
DA_HD void umin_fix(void *index, void *field, int wide, const uint64_t *tab, int nunit, const uint64_t *umin,
                    uint64_t total, uint64_t lo, uint64_t hi, uint64_t first, uint64_t step) {
  if (lo >= hi || nunit < 1) return;
  for (int u = unit_of_entry(tab, nunit, lo); u < nunit; ++u) {
    const uint64_t ulo = tab[(uint64_t)u * 8 + C_INDEX];
    if (ulo >= hi) break;
    const uint64_t uhi = u + 1 < nunit ? tab[(uint64_t)(u + 1) * 8 + C_INDEX] : total;
    if (umin[u] == 0) continue;  // a 0 among the unit's ids: kept (a unit without ids has an empty range)
    const uint64_t a = ulo > lo ? ulo : lo, b = uhi < hi ? uhi : hi;
    for (uint64_t i = a + first; i < b; i += step) {
      if (wide) {
        --reinterpret_cast<uint64_t *>(index)[i];
        if (field) --reinterpret_cast<uint64_t *>(field)[i];
      } else {
        --reinterpret_cast<uint32_t *>(index)[i];
        if (field) --reinterpret_cast<uint32_t *>(field)[i];
      }
    }
  }
}

// ---- "qid:<n>" (libsvm_parser.h:119-132) in the fast grammar.  The letters
// q, i, d classify as N and C together (fast_common.h class_of); qid_clean
// makes them blanks and the token's ':' a qid marker (N and C together), so
// the gap in front of a qid run carries a marker the role arithmetic sees
// like it sees a newline or a ':'.  Bytes [P, P + 64) with raw planes n, c;
// lead: the byte at P - 1 is a letter; at(p): the byte at p (0 outside the
// text).  Returns false on a letter outside a token or a token not followed
// by a digit (atoll's digits).
DA_HD bool is_qid_letter(uint32_t b) { return b == 'q' || b == 'i' || b == 'd'; }
// (inline: out of line, the call's stack frame cost the kernel 2.3x)
// Each run of letters is checked once, at its first letter: the token it
// must belong to starts where that letter's place in "qid" puts it, and the
// four bytes there (one word read, `wd`) must be "qid:" -- which also bounds
// the run to the token's three letters.  (Round 2 read five bytes per letter.)
constexpr uint32_t kQidWord = 0x3A646971u;  // "qid:" little-endian
// stray (optional): the letters of runs that are no "qid:" token -- bytes
// outside the grammar, which the dirty pass (dirty_rewrite) takes like any
// other; without it such letters fail the check.  A "qid:" token not followed
// by a digit always fails it (atoll's whitespace and sign, :126).
template <class At, class Wd>
DA_HD bool qid_clean(uint64_t P, uint64_t *n, uint64_t *c, bool lead, At at, Wd wd, uint64_t *stray = nullptr) {
  const uint64_t X = *n & *c;
  bool ok = true;
  uint64_t sx = 0;
  for (uint64_t m = X & ~(X << 1); m; m &= m - 1) {
    const uint64_t x = P + ctz64(m);
    const uint32_t b = at(x);
    const uint64_t s0 = x - (b == 'q' ? 0u : b == 'i' ? 1u : 2u);
    if (wd(s0) != kQidWord) {
      const uint64_t lb = m & (0 - m);
      sx |= X & ((X + lb) ^ X);  // the letter run from this bit
    }
  }
  if (stray) *stray = sx;
  else ok = sx == 0;
  uint64_t qc = 0;
  for (uint64_t m = *c & ~X & ((X << 1) | (lead ? 1u : 0u)); m; m &= m - 1) {
    const uint64_t x = P + ctz64(m);
    if (x >= 3 && wd(x - 3) == kQidWord) {
      qc |= m & (0 - m);
      ok = ok && is_digit(at(x + 1));
    }
  }
  *n = (*n & ~X) | qc;
  *c &= ~X;
  return ok;
}

// look-back counter slots (record words 0-3: aggregate, 4-7: inclusive prefix)
enum { Q_ROWS = 0, Q_INDEX = 1, Q_VALUE = 2, Q_WEIGHT = 3 };

struct Planes {  // slot 0: the segment before the tile; slot t+1: segment t
  uint64_t d[kFThreads + 1];  // digitchar
  uint64_t n[kFThreads + 1];  // newline
  uint64_t c[kFThreads + 1];  // ':'
};
// the lane that classifies the 16 bytes after the tile (besides its segment)
constexpr int kPostLane = kFWaves > 1 ? kWave : kFThreads - 1;
// run list entries (tile offsets) that fit in the planes' space, which the
// libsvm write pass no longer reads once the roles are known
constexpr int kListCap = (int)(sizeof(Planes) / sizeof(uint16_t));
// a pass of the run lists: the runs of consecutive segments, at most kPassRuns
// before its last segment starts (a segment holds <= 64 run starts)
constexpr uint32_t kPassRuns = (uint32_t)kListCap - kSegB;

// Per-line fallback (dirty_lines): a tile takes the lines holding bytes
// outside the grammar -- after its comments are blanked -- from a byte walk of
// the reference's line parse, at most kDirtyLines lines of at most
// kDirtyMaxLine bytes and kDirtyEntries runs in the tile.
constexpr int kDirtyLines = 4;
constexpr int kDirtyEntries = 40;
constexpr uint64_t kDirtyMaxLine = 256;
constexpr int kPendWords = (kTile / kPassRuns + 2) > kFWaves ? (kTile / kPassRuns + 2) : kFWaves;

struct Shared {  // LDS of one workgroup
  TileCommon c;
  uint32_t cls[kClsEntries];  // byte class table (fast_common.h class_of)
  DecTables dt;
  union {
    Planes m;
    uint16_t lst[kListCap];
  } u;
  uint32_t gw[2 * kFThreads + 2];  // digit plane as words: 2t, 2t+1 segment t; 2 kFThreads: the post-halo
  uint64_t pend[kPendWords];  // packed inclusive counts at the end of each pass (dirty_lines: wave masks)
  uint64_t prebad;            // pre-halo bytes outside the grammar (dirty_lines)
  uint64_t qfail[kFWaves];    // segments whose first-pass "qid:" check failed (the comment pass's plane path)
  uint32_t npass;
  uint32_t next;   // persistent form: the next tile id
  uint32_t nq;     // qid runs of the tile
  uint32_t hashy;  // a byte outside the grammar: comments to blank (pass 1)
  uint32_t ndl, ndr, dgate, nseg;
  uint32_t dl[kDirtyEntries];      // dirty lines' runs in the tile: tile offset | kind << 16
  int32_t dr[2 * kDirtyLines];     // dirty lines [lbegin, lend], tile-relative
};

struct Tile {
  const FastSvmArgs *a;
  Shared *sh;
  uint64_t tlo, thi;

  // masks of the absolute 64-byte segment g (full segments only when g < tlo/64)
  DA_HD void seg(uint64_t g, uint64_t *d, uint64_t *n, uint64_t *c) const {
    const uint64_t g0 = tlo >> 6;
    if (g < g0 + kFThreads && (g >= g0 || (tlo > 0 && g + 1 == g0))) {
      const uint64_t s = g + 1 - g0;
      *d = sh->u.m.d[s];
      *n = sh->u.m.n[s];
      *c = sh->u.m.c[s];
      return;
    }
    // beyond the staged bytes (a gap or run longer than the pre-halo): a
    // compact byte loop, kept out of line of the register budget
    uint64_t md = 0, mn = 0, mc = 0;
    const uint8_t *p = a->text + (g << 6);
#pragma unroll 1
    for (int i = 0; i < 64; ++i) {
      const uint32_t b = p[i];
      md |= (uint64_t)is_digitchar(b) << i;
      // a qid token's ':' is a marker (N and C), its letters blanks (qid_clean)
      const bool qm = b == ':' && (g << 6) + i >= 3 && p[i - 1] == 'd' && p[i - 2] == 'i' && p[i - 3] == 'q';
      mn |= (uint64_t)(is_nl(b) || qm) << i;
      mc |= (uint64_t)(b == ':') << i;
    }
    *d = md;
    *n = mn;
    *c = mc;
  }

  // last position in [lo, hi) whose bit is set in mask `kind` (0 D, 1 not-D,
  // 2 newline, 3 colon, 4 qid marker), or kNone
  DA_HD uint64_t last_bit(int kind, uint64_t lo, uint64_t hi) const {
    if (lo >= hi) return kNone;
    for (uint64_t g = (hi - 1) >> 6;; --g) {
      uint64_t d, n, c;
      seg(g, &d, &n, &c);
      uint64_t w = kind == 0 ? d : kind == 1 ? ~d : kind == 2 ? n & ~c : kind == 3 ? c & ~n : n & c;
      const uint64_t b0 = g << 6;
      if (hi - b0 < 64) w &= (1ull << (hi - b0)) - 1;
      if (lo > b0) w &= ~((1ull << (lo - b0)) - 1);
      if (w) return b0 + 63 - clz64(w);
      if (b0 <= lo) return kNone;
    }
  }

  DA_HD uint64_t floor_of(uint64_t p) const {  // last chunk start <= p
    uint64_t f = sh->c.cfloor;
    for (uint32_t i = 0; i < sh->c.ncs && sh->c.csl[i] <= p; ++i) f = sh->c.csl[i];
    return f;
  }
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

  // role of the run starting at q (q > its chunk start f, or == f)
  DA_HD uint32_t role_of(uint64_t q, uint64_t f) const {
    if (q == f) return R_L;
    const uint64_t p = last_bit(0, f, q);
    if (p == kNone) return R_L;
    if (last_bit(2, p + 1, q) != kNone) return R_L;
    if (last_bit(4, p + 1, q) != kNone) return R_Q;
    if (last_bit(3, p + 1, q) != kNone) return R_K;
    return R_I;
  }

  // The qid run at x (its token "qid:" at x - 4) stands where the reference
  // reads one: right after the line's label -- ParsePair skipped the blanks
  // after it (strtonum.h:667-703) -- or after label:weight with spaces only
  // in between (libsvm_parser.h:119-124); and it is 1-18 plain digits
  // (atoll, then the digitchar skip, :126-129).  Reads the staged text; a
  // line reaching back before it reads as not ok (the exact kernels decide).
  DA_HD bool qid_ok(uint64_t x) const {
    const uint8_t *txt = sh->c.text;
    const uint64_t base = tlo;
    auto at = [&](uint64_t p) -> uint32_t { return txt[p - base + kPre]; };
    uint32_t len = 0;
    while (len < 19 && is_digit(at(x + len))) ++len;
    if (len > 18 || is_digitchar(at(x + len))) return false;
    const uint64_t F = floor_of(x);
    const uint64_t lo = tlo >= (uint64_t)kPre ? tlo - kPre : 0;
    const uint64_t lim = F > lo ? F : lo;  // bytes before it are another line's, or not staged
    if (x < lim + 5) return false;
    uint64_t e = x - 4;  // the scan examines byte e - 1
    bool tab = false;
    while (e > lim && is_blank(at(e - 1))) tab |= at(--e) == '\t';
    if (e == lim || !is_digitchar(at(e - 1))) return false;  // no run before the token
    while (e > lim && is_digitchar(at(e - 1))) --e;
    if (e == F) return true;  // the line's label
    while (e > lim && is_blank(at(e - 1))) --e;
    if (e == F) return true;
    if (e == lim) return false;
    const uint32_t g = at(e - 1);
    if (is_nl(g)) return true;          // the line's label
    if (g != ':' || tab) return false;  // not label:weight, or a tab after the weight
    --e;
    while (e > lim && is_blank(at(e - 1))) --e;
    if (e == lim || !is_digitchar(at(e - 1))) return false;
    while (e > lim && is_digitchar(at(e - 1))) --e;
    if (e == F) return true;
    while (e > lim && is_blank(at(e - 1))) --e;
    if (e == F) return true;
    return e > lim && is_nl(at(e - 1));
  }
};

// Carry-in at a segment start P from the masks of the 64 bytes before it
// (bit i <-> P-64+i), when no chunk starts in (P-64, P] and the previous run
// and its gap lie inside those 64 bytes (the common case).  Returns false
// when the general look-back (Tile::last_bit) is needed.
DA_HD bool carry_fast(uint64_t d1, uint64_t n1r, uint64_t c1r, uint32_t *dc, uint32_t *ginl, uint32_t *ginc,
                      uint32_t *ginq, uint32_t *prole) {
  const uint64_t n1 = n1r & ~c1r, c1 = c1r & ~n1r, q1 = n1r & c1r;  // newline, ':', qid marker
  *dc = (uint32_t)(d1 >> 63);
  uint32_t qb;  // first bit of the last run that starts before P
  if (*dc) {
    const uint64_t nd = ~d1;
    if (!nd) return false;
    qb = 64 - clz64(nd);
    *ginl = *ginc = *ginq = 0;
  } else {
    if (!d1) return false;
    const uint32_t pb = 63 - clz64(d1);  // last digitchar, <= 62
    const uint64_t tg = ~0ull << (pb + 1);
    const uint64_t tgn = n1 & tg;
    *ginl = tgn != 0;
    const uint32_t ln = tgn ? 63 - clz64(tgn) : 0;
    const uint64_t after = !tgn ? tg : (ln == 63 ? 0ull : ~0ull << (ln + 1));
    *ginc = (c1 & after) != 0;
    *ginq = (q1 & after) != 0;
    const uint64_t nd = ~d1 & ((1ull << pb) - 1);
    if (!nd) return false;
    qb = 64 - clz64(nd);
  }
  // role of the run starting at bit qb (1 <= qb <= 63): its gap is (p2, qb)
  const uint64_t below = d1 & ((1ull << (qb - 1)) - 1);
  if (!below) return false;
  const uint32_t p2 = 63 - clz64(below);
  const uint64_t gm = ((1ull << qb) - 1) & ~((2ull << p2) - 1);
  *prole = (n1 & gm) ? R_L : (q1 & gm) ? R_Q : ((c1 & gm) ? R_K : R_I);
  return true;
}

// ---- '#' comments (libsvm_parser.h:67-83 IgnoreCommentAndBlank) in the fast
// grammar.  Where the reference calls IgnoreCommentAndBlank -- the line start
// and every pair end -- a '#' that is the first non-blank byte drops the rest
// of the line.  In the uniform grammar a pair end is the end of any digitchar
// run (ParsePair's endptr, strtonum.h:667-703), so a '#' whose nearest
// non-blank predecessor in the line is a run or the line start opens a
// comment; one after a ':' or a "qid:" token does not, and after the comment
// is blanked that ':' dangles at the line end (or the token lacks its digit),
// which the role checks already send to the exact kernels.
//
// So a comment is "from a '#' to the next newline or range start", found with
// the carry trick: X = bytes that do not end a comment, seeds A = '#' bytes;
// in X + A + cin a carry enters every byte of a run of X after its first seed
// (or from bit 0 when a comment is open before the segment), so the comment
// bytes are X & (A | carries), carries = (X + A + cin) ^ X ^ A.  Segments compose by the
// function (open before -> open after), two bits, by one block scan.  The
// tile's comment bytes -- and those of the staged halos -- become blanks in
// the LDS text and classification runs again; the tile start's state comes
// from the pre-halo alone (a comment open there has its '#' in the pre-halo),
// which the tile before checks: a comment open at its end whose '#' lies
// further back than the next tile's pre-halo raises the gate.
// A '#' opens a comment when the bytes between it and the previous digitchar
// (a pair end) or range start are blanks: "reachable" bytes.  A line start
// after a newline is not one -- ParseBlock's line begins at the previous
// line's '\n' (libsvm_parser.h:91-96), which IgnoreCommentAndBlank does not
// skip, so there ParsePair reads the '#' line's digits as the label and the
// exact kernels take it.
// Byte masks of 64 staged bytes (16-byte aligned), four bytes per SWAR step.
struct CmtMasks {
  uint64_t h, nl, bl, dg;  // '#', newline, blank, digitchar
};
DA_HD uint32_t swar_zero_hi(uint32_t t) {  // 0x80 in each zero byte of t
  return ~(((t & 0x7F7F7F7Fu) + 0x7F7F7F7Fu) | t) & 0x80808080u;
}
DA_HD uint32_t hi_nib(uint32_t m) { return (m * 0x00204081u) >> 28; }  // byte high bits -> 4 bits
DA_HD CmtMasks comment_masks(const uint8_t *p) {
  CmtMasks k{0, 0, 0, 0};
#pragma unroll 1
  for (int q = 0; q < 4; ++q) {
    uint32_t w[4];
    load16(p + 16 * q, w);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const uint32_t x = w[j];
      const uint32_t lo = (x | 0x80808080u) - 0x30303030u, hi = (x | 0x80808080u) - 0x3A3A3A3Au;
      const uint32_t dig = lo & ~hi & ~x & 0x80808080u;
      const uint32_t dc = dig | swar_zero_hi(x ^ 0x2B2B2B2Bu) | swar_zero_hi(x ^ 0x2D2D2D2Du) |
                          swar_zero_hi(x ^ 0x2E2E2E2Eu) | swar_zero_hi((x | 0x20202020u) ^ 0x65656565u);
      const uint32_t nl = swar_zero_hi(x ^ 0x0A0A0A0Au) | swar_zero_hi(x ^ 0x0D0D0D0Du);
      const uint32_t bl = swar_zero_hi(x ^ 0x20202020u) | swar_zero_hi(x ^ 0x09090909u);
      const int sh = 16 * q + 4 * j;
      k.h |= (uint64_t)hi_nib(swar_zero_hi(x ^ 0x23232323u)) << sh;
      k.nl |= (uint64_t)hi_nib(nl) << sh;
      k.bl |= (uint64_t)hi_nib(bl) << sh;
      k.dg |= (uint64_t)hi_nib(dc) << sh;
    }
  }
  return k;
}
// "Reachable" bytes of a block with reach-in r: after a digitchar or at a
// range start (S), through blanks.  *rout: the byte after the block is.
DA_HD uint64_t reach_of(const CmtMasks &k, uint64_t S, uint32_t r, uint32_t *rout) {
  const uint64_t ok = (k.dg << 1) | S, seeds = ok & k.bl;
  uint32_t ro;
  const uint64_t reach = ok | (add_carry(k.bl, seeds, r, &ro) ^ k.bl ^ seeds);
  *rout = ro | (uint32_t)(k.dg >> 63);
  return reach;
}
// reach-out as a function of reach-in (bit 0 = f(0), bit 1 = f(1))
DA_HD uint32_t reach_fn(const CmtMasks &k, uint64_t S) {
  uint32_t r0, r1;
  (void)reach_of(k, S, 0u, &r0);
  (void)reach_of(k, S, 1u, &r1);
  return r0 | (r1 << 1);
}
// comment-opening '#' (A) and comment ends (B) of a block with reach-in r
DA_HD void comment_ab(const CmtMasks &k, uint64_t S, uint32_t r, uint64_t *A, uint64_t *B) {
  uint32_t ro;
  *A = k.h & reach_of(k, S, r, &ro);
  *B = k.nl | (S & ~*A);  // a range start ends a comment, unless it opens one
}
// open-after as a function of open-before: bit 0 = f(0), bit 1 = f(1)
DA_HD uint32_t comment_fn(uint64_t A, uint64_t B) {
  uint32_t o0, o1;
  (void)add_carry(~B, A, 0u, &o0);
  (void)add_carry(~B, A, 1u, &o1);
  return o0 | (o1 << 1);
}
struct CommentFnCompose {  // a then b
  DA_HD uint32_t operator()(uint32_t a, uint32_t b) const {
    return ((b >> (a & 1u)) & 1u) | (((b >> ((a >> 1) & 1u)) & 1u) << 1);
  }
};
// blank the bytes of mask m in the 64 staged bytes at p
DA_HD void blank_bytes(uint8_t *p, uint64_t m) {
  for (; m; m &= m - 1) p[ctz64(m)] = ' ';
}
// The comment masks of a segment in the grammar, from its classification
// planes (no '#'; the other bytes are blanks).
DA_HD CmtMasks plane_cmt_masks(uint64_t D, uint64_t N, uint64_t C) {
  return CmtMasks{0, N & ~C, ~(D | N | C), D};
}
// The comment masks of the 64 staged bytes at p by the whole wave: lane =
// byte, one ballot per mask (all lanes; p wave-uniform).
template <class BK>
DA_HDF CmtMasks wave_cmt_masks(const uint8_t *p, BK &bk) {
  const uint32_t b = p[bk.tid() & (kWave - 1)];
  CmtMasks k;
  k.h = bk.ballot(b == '#');
  k.nl = bk.ballot(is_nl(b));
  k.bl = bk.ballot(is_blank(b));
  k.dg = bk.ballot(is_digitchar(b));
  return k;
}
// Lane `owner`'s mask M blanks bytes of the 64 staged bytes at p (p wave
// uniform), by the whole wave.
template <class BK>
DA_HDF void wave_blank(uint8_t *p, uint64_t M, uint32_t owner, BK &bk) {
  const uint64_t Ms = bk.shfl(M, (int)owner);
  const uint32_t lane = (uint32_t)bk.tid() & (kWave - 1);
  if ((Ms >> lane) & 1u) p[lane] = ' ';
}
// the comment bytes of a segment (A '#', B comment ends, cin open before it);
// *co: open after it
DA_HD uint64_t comment_mask(uint64_t A, uint64_t B, uint32_t cin, uint32_t *co) {
  const uint64_t X = ~B;
  return X & (A | (add_carry(X, A, cin, co) ^ X ^ A));
}
// chunk starts in [lo, lo + 64) as bits (the tile's list and the one after it)
DA_HD uint64_t cs_bits(const TileCommon &c, uint64_t lo) {
  uint64_t s = 0;
  for (uint32_t i = 0; i <= c.ncs; ++i) {
    const uint64_t x = i < c.ncs ? c.csl[i] : c.cnext;
    if (x >= lo && x < lo + 64) s |= 1ull << (x - lo);
  }
  if (c.cfloor >= lo && c.cfloor < lo + 64) s |= 1ull << (c.cfloor - lo);
  return s;
}
// Blanks the comments of the staged text (pre-halo, tile, post-halo); all
// threads.  Returns 1 (gate) when the tile after this one cannot see from its
// pre-halo that a comment is open at its start.
//
// A segment in the grammar (raw = 0) has no '#': its masks come from its
// classification planes D, N, C; the segments holding other bytes are read
// byte by byte, one segment at a time by their wave (lane = byte), and the
// comment bytes are blanked the same way -- per-lane byte loops would run
// every wave through the slowest lane's segment.
template <class BK>
DA_HDF uint32_t comment_erase(uint64_t tlo, uint64_t thi, uint64_t n, TileCommon &c, uint32_t *note, BK &bk,
                              uint64_t D, uint64_t N, uint64_t C, bool raw, uint32_t k, bool planes_ok,
                              uint64_t *Mplanes) {
  (void)k;  // (phase stamps of the diagnostic build)
  const int tid = bk.tid();
  const uint32_t lane = (uint32_t)tid & (kWave - 1), wbase = (uint32_t)tid - lane;
  uint8_t *txt = c.text;
  const uint64_t P = tlo + (uint64_t)tid * kSegB;
  CmtMasks km = plane_cmt_masks(D, N, C);
  for (uint64_t m = bk.ballot(raw); m; m &= m - 1) {  // wave-uniform
    const uint32_t s = (uint32_t)ctz64(m);
    const CmtMasks kk = wave_cmt_masks(txt + kPre + (wbase + s) * kSegB, bk);
    if (lane == s) km = kk;
  }
  // wave 0: the pre-halo's masks; wave 3: the post-halo's
  CmtMasks kh{0, 0, 0, 0}, kp[kPost / kSegB];
  if (tid < kWave && tlo > 0) kh = wave_cmt_masks(txt, bk);
  if (tid >= kFThreads - kWave)
    for (int s = 0; s < kPost / kSegB; ++s) kp[s] = wave_cmt_masks(txt + kPre + kTile + s * kSegB, bk);
  const uint64_t S = cs_bits(c, P);
  // the pre-halo read on its own (reach-in 0, no comment open before it): the
  // tile start's reach and comment state, as the tile before checks them
  uint64_t hA = 0, hB = 0;
  if (tid == 0 && tlo > 0) {
    const uint64_t Sh = cs_bits(c, tlo - kPre);
    uint32_t r0;
    (void)reach_of(kh, Sh, 0u, &r0);
    comment_ab(kh, Sh, 0u, &hA, &hB);
    const uint32_t c0 = comment_fn(hA, hB) & 1u;
    *note = 1u | (r0 << 1) | (c0 << 2);  // (stays nonzero: the caller's branch read it)
  }
  FAST_STAMP(k, 17);
  // The reach and comment state at each segment start, one barrier.  Both
  // per-segment maps (reach-in -> reach-out, open-in -> open-after) are
  // monotone: constant 0 (0b00), constant 1 (0b11) or the identity (0b10)
  // (add_carry's carry-out never falls when the carry-in rises), so a
  // segment's state is the constant of the nearest non-identity segment
  // before it, else the tile start's (*note).  In-wave by ballots; across
  // waves each wave publishes its reach map and its comment map for either
  // reach-in at its start (its leading segments' reach depends on it).
  const uint32_t fr = reach_fn(km, S);
  uint32_t fc0, fc1;
  {
    uint64_t A0, B0, A1, B1;
    comment_ab(km, S, 0u, &A0, &B0);
    comment_ab(km, S, 1u, &A1, &B1);
    fc0 = comment_fn(A0, B0);
    fc1 = comment_fn(A1, B1);
  }
  const uint64_t below = (1ull << lane) - 1;
  // the value at the lane's start from the wave's non-identity maps (nim) and
  // their constants (one): -1 when none lies before the lane
  auto anchor = [&](uint64_t nim, uint64_t one) -> int {
    const uint64_t b = nim & below;
    return b ? (int)((one >> (63 - clz64(b))) & 1u) : -1;
  };
  auto wave_map = [](uint64_t nim, uint64_t one) -> uint32_t {  // the wave's composed map
    return nim ? (((one >> (63 - clz64(nim))) & 1u) ? 3u : 0u) : 2u;
  };
  const uint64_t rn = bk.ballot(fr != 2u), r1 = bk.ballot(fr == 3u);
  const int ra = anchor(rn, r1);
  // the lane's comment map for wave reach-in 0 / 1
  const uint32_t g0 = ra >= 0 ? (ra ? fc1 : fc0) : fc0, g1 = ra >= 0 ? (ra ? fc1 : fc0) : fc1;
  const uint64_t cn0 = bk.ballot(g0 != 2u), c10 = bk.ballot(g0 == 3u);
  const uint64_t cn1 = bk.ballot(g1 != 2u), c11 = bk.ballot(g1 == 3u);
  const uint32_t wid = (uint32_t)tid / kWave;
  bk.wave_put(wave_map(rn, r1) | (wave_map(cn0, c10) << 2) | (wave_map(cn1, c11) << 4));
  bk.sync();
  uint32_t rw = (*note >> 1) & 1u, cw = (*note >> 2) & 1u;  // the tile start's reach / open state
  for (uint32_t w = 0; w < wid; ++w) {
    const uint32_t m = bk.wave_get((int)w);
    cw = (m >> (rw ? 4 : 2) >> cw) & 1u;  // the wave's comment map for its reach-in, applied
    rw = (m >> rw) & 1u;
  }
  FAST_STAMP(k, 18);
  const uint32_t r = ra >= 0 ? (uint32_t)ra : rw;
  const int ca = rw ? anchor(cn1, c11) : anchor(cn0, c10);
  const uint32_t cin = ca >= 0 ? (uint32_t)ca : cw;
  uint64_t A, B;
  comment_ab(km, S, r, &A, &B);
  uint32_t f_next = 0;  // the next tile's reading of its pre-halo (this segment)
  if (tid == kFThreads - 1) {
    uint64_t An, Bn;
    comment_ab(km, S, 0u, &An, &Bn);
    f_next = comment_fn(An, Bn) & 1u;
  }
  FAST_STAMP(k, 19);
  uint32_t co, gate = 0;
  const uint64_t M = comment_mask(A, B, cin, &co);
  // Every comment is blanked in the staged text (the per-line walk and the
  // decoders read it).  A segment whose first-pass "qid:" checks all held
  // (planes_ok) then takes its comment out of its planes (*Mplanes; the
  // caller clears the bits) instead of being classified again: its planes
  // are exactly the reclassified ones (the comment bytes read as blanks,
  // the rest as classified -- a qid token next to a comment fails the check)
#ifndef FSVM_CMT_BLANK  // A/B: every comment blanked and reclassified
  const bool via_planes = M != 0 && planes_ok;
#else
  const bool via_planes = false;
  (void)planes_ok;
#endif
  *Mplanes = via_planes ? M : 0;
  for (uint64_t m = bk.ballot(M != 0); m; m &= m - 1) {  // wave-uniform
    const uint32_t s = (uint32_t)ctz64(m);
    wave_blank(txt + kPre + (wbase + s) * kSegB, M, s, bk);
  }
  uint32_t changed = M != 0 && !via_planes;  // bit 0: my segment, bit 1: the pre-halo, bit 2: the post-halo
  if (tid < kWave && tlo > 0) {  // wave 0: lane 0's pre-halo comment bytes
    uint32_t ch;
    const uint64_t Mh = comment_mask(hA, hB, 0u, &ch);
    wave_blank(txt, Mh, 0u, bk);
    if (tid == 0 && Mh) changed |= 2u;
  }
  if (tid >= kFThreads - kWave) {  // the last wave: lane 63's post-halo comment bytes
    uint64_t Mp[kPost / kSegB] = {};
    if (tid == kFThreads - 1) {
      if (thi < n && P + kSegB == thi && !(cs_bits(c, thi) & 1u) && co != f_next) gate = 1;
      uint32_t ci = co, ri;
      (void)reach_of(km, S, r, &ri);
      for (int s = 0; s < kPost / kSegB; ++s) {
        const uint64_t Sp = cs_bits(c, tlo + kTile + (uint64_t)s * kSegB);
        uint64_t Ap, Bp;
        comment_ab(kp[s], Sp, ri, &Ap, &Bp);
        (void)reach_of(kp[s], Sp, ri, &ri);
        Mp[s] = comment_mask(Ap, Bp, ci, &ci);
        if (Mp[s]) changed |= 4u;
      }
    }
    for (int s = 0; s < kPost / kSegB; ++s) wave_blank(txt + kPre + kTile + s * kSegB, Mp[s], kWave - 1, bk);
  }
  return gate | (changed << 1);
}

// Runs, roles and counts of segment tid (positions P .. P+63).
struct SegOut {
  uint64_t L, W, I, V, Q;
  uint32_t bad;
};

DA_HD SegOut segment_roles(const Tile &t, int tid) {
  SegOut o;
  o.L = o.W = o.I = o.V = o.Q = 0;
  o.bad = 0;
  const FastSvmArgs &a = *t.a;
  const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
  if (P >= a.n) return o;
  const int nv = (int)mn<uint64_t>(64, a.n - P);
  const uint64_t valid = nv == 64 ? ~0ull : ((1ull << nv) - 1);
  const uint64_t D = t.sh->u.m.d[tid + 1], Nr = t.sh->u.m.n[tid + 1], Cr = t.sh->u.m.c[tid + 1];
  const uint64_t N = Nr & ~Cr, C = Cr & ~Nr, QM = Nr & Cr;  // newline, ':', qid marker
  uint64_t S = 0;
  for (uint32_t i = 0; i < t.sh->c.ncs; ++i) {
    const uint64_t x = t.sh->c.csl[i];
    if (x >= P && x < P + (uint64_t)nv) S |= 1ull << (x - P);
  }
  // ---- carry-in: state just before P
  uint32_t dc = 0, ginl = 0, ginc = 0, ginq = 0, prole = R_NONE;
  const uint64_t F = t.floor_of(P);
  if (P != F && !(F + 64 <= P && carry_fast(t.sh->u.m.d[tid], t.sh->u.m.n[tid], t.sh->u.m.c[tid], &dc, &ginl,
                                            &ginc, &ginq, &prole))) {
    dc = ginl = ginc = ginq = 0;
    prole = R_NONE;
    uint64_t d, n, c;
    t.seg((P - 1) >> 6, &d, &n, &c);
    dc = (uint32_t)(d >> 63) & 1u;
    if (dc) {
      const uint64_t x = t.last_bit(1, F, P);
      prole = t.role_of(x == kNone ? F : x + 1, F);
    } else {
      const uint64_t p = t.last_bit(0, F, P);
      if (p == kNone) {
        ginl = 1;
      } else {
        const uint64_t ln = t.last_bit(2, p + 1, P);
        ginl = ln != kNone;
        ginc = t.last_bit(3, ginl ? ln + 1 : p + 1, P) != kNone;
        ginq = t.last_bit(4, ginl ? ln + 1 : p + 1, P) != kNone;
        const uint64_t x = t.last_bit(1, F, p);
        prole = t.role_of(x == kNone ? F : x + 1, F);
      }
    }
  }
  // ---- roles inside the segment
  const uint64_t RS = (D & ~((D << 1) | dc)) | (D & S);
  const uint64_t G = ~D & valid;
  const uint64_t NS = N | S;
  uint32_t co;
  const uint64_t t1 = add_carry(G, NS & G, ginl, &co);
  const uint64_t L = RS & (t1 | S);
  const uint64_t G2 = G & ~NS;
  const uint64_t t2 = add_carry(G2, C & G2, ginc, &co);
  // a ':' gap that ends at a newline, a chunk start or the end of the text:
  // ParsePair then decodes past the line end (strtonum.h:684-692)
  if (t2 & (NS | ~valid)) o.bad = 1;
  if (co && (P + 64 >= a.n || t.is_cs(P + 64))) o.bad = 1;
  const uint64_t K = RS & t2 & ~L;
  uint64_t Q = 0;
  if (QM | ginq) {  // qid runs: the gap in front holds a qid marker
    uint32_t cq;
    const uint64_t t3 = add_carry(G2, QM & G2, ginq, &cq);
    if (t3 & (NS | ~valid)) o.bad = 1;
    if (cq && (P + 64 >= a.n || t.is_cs(P + 64))) o.bad = 1;
    Q = RS & t3 & ~L;
    if (Q & K) o.bad = 1;  // a ':' and a token in one gap ("l : qid:5" pairs l with 5)
    if (Q) {
      // qid_ok from the planes where the run before the token is the line's
      // label (role L: only blanks and the token between them, the common
      // "label qid:n" form): the value is 1-18 plain digits ending at a
      // non-digitchar -- the digitchar run at x and its G (digit) bits, read
      // as 128-bit windows over this segment and the next.  After a weight,
      // or near the tile's end, the byte walk (Tile::qid_ok).
      const uint64_t Zq = ~RS, xlq = L << 1;
      const uint64_t afterL = ((Zq + (xlq & Zq) + (prole == R_L ? 1u : 0u)) | xlq) & RS;
      uint64_t slow = Q & ~afterL;
      const bool lastseg = tid + 1 >= kFThreads;
      const uint64_t Dn = lastseg ? 0 : t.sh->u.m.d[tid + 2];
      const uint64_t Gc = t.sh->gw[2 * tid] | ((uint64_t)t.sh->gw[2 * tid + 1] << 32);
      const uint64_t Gn = lastseg ? 0 : t.sh->gw[2 * tid + 2] | ((uint64_t)t.sh->gw[2 * tid + 3] << 32);
      for (uint64_t m = Q & afterL; m; m &= m - 1) {
        const uint32_t b = ctz64(m);
        if (lastseg && b + 19 > 64) {
          slow |= 1ull << b;
          continue;
        }
        const uint64_t r = b ? (D >> b) | (Dn << (64 - b)) : D;
        const uint64_t g = b ? (Gc >> b) | (Gn << (64 - b)) : Gc;
        const uint32_t len = ~r ? (uint32_t)ctz64(~r) : 64u;  // >= 1: a run starts at b
        if (len > 18 || (~g & ((1ull << len) - 1))) o.bad = 1;
      }
      for (uint64_t m = slow; m; m &= m - 1)
        if (!t.qid_ok(P + ctz64(m))) o.bad = 1;
    }
  }
  const uint64_t Z = ~RS;
  const uint64_t xl = L << 1, xk = K << 1, xq = Q << 1;
  const uint64_t prevL = ((Z + (xl & Z) + (prole == R_L ? 1u : 0u)) | xl) & RS;
  const uint64_t prevK = ((Z + (xk & Z) + (prole == R_K ? 1u : 0u)) | xk) & RS;
  const uint64_t prevQ = ((Z + (xq & Z) + (prole == R_Q ? 1u : 0u)) | xq) & RS;
  if (K & prevK) o.bad = 1;  // "a:b:c": the pair grammar re-pairs (strtonum.h:684-702)
  if (K & prevQ) o.bad = 1;  // "qid:5:x": the digitchar skip stops at the ':' (libsvm_parser.h:127-129)
  o.L = L;
  o.W = K & prevL;
  o.V = K & ~prevL;
  o.Q = Q;
  o.I = RS & ~L & ~K & ~Q;
  return o;
}

// ---- libfm (LibFMParser::ParseBlock, libfm_parser.h:67-144) in the same
// uniform grammar.  A line is label[:weight] then ParseTriple groups
// field:index[:value] (strtonum.h:718-772).  With K = runs whose gap holds ':'
// and F = the other non-label runs (fields, v1), the roles are
//   W = K after a label, I = K after a field, V = K after an index;
// a K run after a value or weight ("f:i:v:x", "l:w:x") re-pairs in the
// reference and leaves the fast path, as does a dangling ':' at a line end.
// A field is stored only when its index follows (r >= 2); every field is
// still checked for a '-' sign (the reference decodes every v1).
enum : uint32_t { RF_NONE = 0, RF_L = 1, RF_W = 2, RF_F = 3, RF_I = 4, RF_V = 5, RF_BAD = 6 };

// role of the run starting at q (chunk start f <= q): walks back through
// the ':'-joined chain to its label or field (at most three runs)
DA_HD uint32_t fm_role_of(const Tile &t, uint64_t q, uint64_t f) {
  uint32_t nk = 0;  // ':' gaps walked over
  for (;;) {
    uint32_t base;
    if (q == f) {
      base = RF_L;
    } else {
      const uint64_t p = t.last_bit(0, f, q);
      if (p == kNone || t.last_bit(2, p + 1, q) != kNone) {
        base = RF_L;
      } else if (t.last_bit(3, p + 1, q) == kNone) {
        base = RF_F;
      } else {
        if (++nk > 2) return RF_BAD;
        const uint64_t x = t.last_bit(1, f, p);
        q = x == kNone ? f : x + 1;
        continue;
      }
    }
    if (nk == 0) return base;
    if (base == RF_L) return nk == 1 ? RF_W : RF_BAD;
    return nk == 1 ? RF_I : RF_V;
  }
}

struct SegOutFm {
  uint64_t L, W, I, V, F, RS;
  uint64_t q0;  // start of the last run that starts before the segment (kNone: none in its chunk)
  uint32_t bad;
};

// libfm carry-in from the 64 bytes before a segment (bit i <-> P-64+i), as
// carry_fast does for libsvm, when no chunk starts in them and the last run
// before P, its gap and the runs its role depends on lie inside them: the
// role follows the ':'-chain back to its label or field (fm_role_of) over at
// most three gaps.  *qlast: the window bit where that run starts.
// kind of the gap in front of the run at bit q: 0 newline, 1 ':', 2 plain;
// -1 when it or the run before it leaves the window (*qprev: that run's start)
DA_HD int fm_gap(uint64_t d1, uint64_t n1, uint64_t c1, uint32_t q, uint32_t *qprev) {
  const uint64_t below = d1 & ((1ull << q) - 1);
  if (!below) return -1;
  const uint32_t p = 63 - clz64(below);  // last byte of the run before
  const uint64_t gm = ((1ull << q) - 1) & ~((2ull << p) - 1);
  if (n1 & gm) return 0;
  const uint64_t nd = ~d1 & ((1ull << p) - 1);
  if (!nd) return -1;
  *qprev = 64 - clz64(nd);
  return (c1 & gm) ? 1 : 2;
}
DA_HD bool carry_fast_fm(uint64_t d1, uint64_t n1, uint64_t c1, uint32_t *dc, uint32_t *ginl, uint32_t *ginc,
                         uint32_t *prole, uint32_t *qlast) {
  *dc = (uint32_t)(d1 >> 63);
  uint32_t qb;
  if (*dc) {
    const uint64_t nd = ~d1;
    if (!nd) return false;
    qb = 64 - clz64(nd);
    *ginl = *ginc = 0;
  } else {
    if (!d1) return false;
    const uint32_t pb = 63 - clz64(d1);
    const uint64_t tg = ~0ull << (pb + 1);
    const uint64_t tgn = n1 & tg;
    *ginl = tgn != 0;
    const uint32_t ln = tgn ? 63 - clz64(tgn) : 0;
    const uint64_t after = !tgn ? tg : (ln == 63 ? 0ull : ~0ull << (ln + 1));
    *ginc = (c1 & after) != 0;
    const uint64_t nd = ~d1 & ((1ull << pb) - 1);
    if (!nd) return false;
    qb = 64 - clz64(nd);
  }
  *qlast = qb;
  uint32_t q2 = 0, q3 = 0, q4 = 0;
  const int g1 = fm_gap(d1, n1, c1, qb, &q2);
  if (g1 < 0) return false;
  if (g1 != 1) {
    *prole = g1 == 0 ? RF_L : RF_F;
    return true;
  }
  const int g2 = fm_gap(d1, n1, c1, q2, &q3);  // a ':' run: after a label W, after a field I
  if (g2 < 0) return false;
  if (g2 != 1) {
    *prole = g2 == 0 ? RF_W : RF_I;
    return true;
  }
  const int g3 = fm_gap(d1, n1, c1, q3, &q4);  // two ':' gaps: V after an index, else re-paired
  if (g3 < 0) return false;
  *prole = g3 == 2 ? RF_V : RF_BAD;
  return true;
}

// previous-run propagation: bit x of the result = the run before run start x
// has its start bit in X (cin: the run before the segment does)
DA_HD uint64_t prev_of(uint64_t RS, uint64_t X, uint32_t cin) {
  const uint64_t Z = ~RS, xs = X << 1;
  return ((Z + (xs & Z) + cin) | xs) & RS;
}

DA_HD SegOutFm segment_roles_fm(const Tile &t, int tid) {
  SegOutFm o;
  o.L = o.W = o.I = o.V = o.F = o.RS = 0;
  o.q0 = kNone;
  o.bad = 0;
  const FastSvmArgs &a = *t.a;
  const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
  if (P >= a.n) return o;
  const int nv = (int)mn<uint64_t>(64, a.n - P);
  const uint64_t valid = nv == 64 ? ~0ull : ((1ull << nv) - 1);
  const uint64_t D = t.sh->u.m.d[tid + 1], N = t.sh->u.m.n[tid + 1], C = t.sh->u.m.c[tid + 1];
  uint64_t S = 0;
  for (uint32_t i = 0; i < t.sh->c.ncs; ++i) {
    const uint64_t x = t.sh->c.csl[i];
    if (x >= P && x < P + (uint64_t)nv) S |= 1ull << (x - P);
  }
  // ---- carry-in: from the previous segment's masks, else the general
  // look-back over the LDS masks
  uint32_t dc = 0, ginl = 0, ginc = 0, prole = RF_NONE, qb = 0;
  const uint64_t F = t.floor_of(P);
  if (P != F && F + 64 <= P &&
      carry_fast_fm(t.sh->u.m.d[tid], t.sh->u.m.n[tid], t.sh->u.m.c[tid], &dc, &ginl, &ginc, &prole, &qb)) {
    o.q0 = P - 64 + qb;
  } else if (P != F) {
    dc = ginl = ginc = 0;
    prole = RF_NONE;
    uint64_t d, n, c;
    t.seg((P - 1) >> 6, &d, &n, &c);
    dc = (uint32_t)(d >> 63) & 1u;
    if (dc) {
      const uint64_t x = t.last_bit(1, F, P);
      o.q0 = x == kNone ? F : x + 1;
      prole = fm_role_of(t, o.q0, F);
    } else {
      const uint64_t p = t.last_bit(0, F, P);
      if (p == kNone) {
        ginl = 1;
      } else {
        const uint64_t ln = t.last_bit(2, p + 1, P);
        ginl = ln != kNone;
        ginc = t.last_bit(3, ginl ? ln + 1 : p + 1, P) != kNone;
        const uint64_t x = t.last_bit(1, F, p);
        o.q0 = x == kNone ? F : x + 1;
        prole = fm_role_of(t, o.q0, F);
      }
    }
  }
  if (prole == RF_BAD) o.bad = 1;
  // ---- roles inside the segment
  const uint64_t RS = (D & ~((D << 1) | dc)) | (D & S);
  const uint64_t G = ~D & valid;
  const uint64_t NS = N | S;
  uint32_t co;
  const uint64_t t1 = add_carry(G, NS & G, ginl, &co);
  const uint64_t L = RS & (t1 | S);
  const uint64_t G2 = G & ~NS;
  const uint64_t t2 = add_carry(G2, C & G2, ginc, &co);
  if (t2 & (NS | ~valid)) o.bad = 1;  // "x:" at a line end: ParseTriple decodes past it
  if (co && (P + 64 >= a.n || t.is_cs(P + 64))) o.bad = 1;
  const uint64_t K = RS & t2 & ~L;
  const uint64_t Fr = RS & ~L & ~K;
  const uint64_t W = K & prev_of(RS, L, prole == RF_L);
  const uint64_t I = K & prev_of(RS, Fr, prole == RF_F);
  const uint64_t V = K & prev_of(RS, I, prole == RF_I);
  if (K & ~(W | I | V)) o.bad = 1;
  // an index's field is the run before it; the first one's may start before
  // the segment (q0) -- further back than the staged pre-halo leaves the path
  if ((I & RS & (0 - RS)) && (o.q0 == kNone || o.q0 + kPre < t.tlo)) o.bad = 1;
  o.L = L;
  o.W = W;
  o.I = I;
  o.V = V;
  o.F = Fr;
  o.RS = RS;
  return o;
}

// The exact byte decoders: rare on this path (exponents, runs that may cross
// the 16-byte window or a chunk end, 9+ digit indices).
// (Measured: out of line they cost more than the code size saves, so they
// stay inline unless FSVM_OUTLINE_SLOW is defined.)
#if defined(FSVM_OUTLINE_SLOW) && defined(__HIP_DEVICE_COMPILE__)
#define FSVM_COLD __device__ __attribute__((noinline))
#else
#define FSVM_COLD DA_HD
#endif
// They read the text from global memory: no LDS pointer crosses the call.
FSVM_COLD float slow_float(const uint8_t *text, uint64_t q, uint64_t lim) {
  GSrc src{text, lim};
  uint64_t e;
  bool nan_err = false;
  return parse_float(src, q, &e, &nan_err);
}
FSVM_COLD bool slow_uint(const uint8_t *text, uint64_t q, uint64_t lim, int wide, uint64_t *v) {
  GSrc src{text, lim};
  return parse_uint(src, q, wide != 0, v);
}

// Classification of segment tid (parts bit 0), of the pre-halo (bit 1: lanes
// 0..15, OR-ed into slot 0) and of the 16 bytes after the tile (bit 2: lane
// kWave): the LDS planes and digit-plane words; returns the segment's grammar
// flag.  `first`: pass 0, which also notes bytes outside the grammar.
// Segment seg's masks m (classify64_lut's form) into the planes and the
// digit-plane words, "qid:" tokens cleaned; returns its grammar flag.
// The four text bytes at p as a little-endian word (0 past the text): two
// aligned LDS words when staged, else byte by byte through `at`.
template <class At>
DA_HD uint32_t text_word(const Tile &t, uint64_t p, At at) {
  if (p + kPre >= t.tlo && p + 4 <= t.a->n) {
    const uint64_t off = p + kPre - t.tlo;
    if (off + 8 <= (uint64_t)kStage) {
      const uint32_t *w = reinterpret_cast<const uint32_t *>(t.sh->c.text + (off & ~3ull));
      return funnel(w[1], w[0], (uint32_t)(off & 3u) * 8u);
    }
  }
  return at(p) | (at(p + 1) << 8) | (at(p + 2) << 16) | (at(p + 3) << 24);
}

template <bool FM, class At>
DA_HDF uint32_t commit_seg(const Tile &t, Shared &sh, int seg, At at, bool first, Masks m) {
  uint32_t bad = 0;
  const uint64_t P0 = t.tlo + (uint64_t)seg * kSegB;
  if ((m.n & m.c) || ((m.c & 1) && P0 > 0 && is_qid_letter(at(P0 - 1)))) {  // letters: "qid:" tokens
    auto wd = [&](uint64_t p) -> uint32_t { return text_word(t, p, at); };
    uint64_t stray = 0;  // letters of no "qid:" token: bytes outside the grammar (the digit plane marks them)
    if (FM || !qid_clean(P0, &m.n, &m.c, P0 > 0 && is_qid_letter(at(P0 - 1)), at, wd, &stray)) {
      bad = 1;
      if (!FM && first) atomic_or_u64(&sh.qfail[seg / kWave], 1ull << (seg % kWave));
    }
    if (stray) {
      m.g |= stray;
      m.bad = 1;
    }
  }
  sh.gw[2 * seg] = (uint32_t)m.g;
  sh.gw[2 * seg + 1] = (uint32_t)(m.g >> 32);
  sh.u.m.d[seg + 1] = m.d;
  sh.u.m.n[seg + 1] = m.n;
  sh.u.m.c[seg + 1] = m.c;
  bad |= m.bad;
  if (!FM && first && m.bad) sh.hashy = 1;
  if (!FM && first && (m.g & ~m.d)) atomic_add_u32(&sh.nseg, 1u);  // segments holding bytes outside the grammar
  return bad;
}

template <bool FM, class At>
DA_HDF uint32_t classify_tile(const Tile &t, Shared &sh, int tid, At at, bool first, uint32_t parts) {
  uint32_t bad = 0;
#ifdef FSVM_REGCLS  // A/B: the segment's classes in registers (fast_common.h classify64_reg)
  if (parts & 1u) bad = commit_seg<FM>(t, sh, tid, at, first, classify64_reg(sh.c.text + kPre + tid * kSegB));
#else
  if (parts & 1u) bad = commit_seg<FM>(t, sh, tid, at, first, classify64_lut(sh.c.text + kPre + tid * kSegB, sh.cls));
#endif
  if ((parts & 4u) && tid == kPostLane) {  // digits of the 16 bytes after the tile (windows of my last runs)
    uint32_t g = 0;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      uint32_t x;
      memcpy(&x, sh.c.text + kPre + kTile + 4 * i, 4);
      g |= classify_dword_lut(x, sh.cls).g << (4 * i);
    }
    sh.gw[2 * kFThreads] = g;
  }
  if ((parts & 2u) && tid < 16 && t.tlo > 0) {
    uint32_t x;
    memcpy(&x, sh.c.text + (kPre - kSegB) + 4 * tid, 4);
    const Nib b = classify_dword_lut(x, sh.cls);
    if (!FM && first && b.bad) sh.hashy = 1;
    if (!FM && b.bad) atomic_or_u64(&sh.prebad, (uint64_t)((b.g & ~b.d) | b.hi) << (4 * tid));  // (dirty_lines)
    uint64_t bn = b.n, bc = b.c;
    const uint64_t P0 = t.tlo - kSegB + 4 * tid;
    if (!FM && ((bn & bc) || (bc & 1))) {  // the bytes' owner tile checks them; here only their planes
      const bool lead = is_qid_letter(at(P0 - 1));
      auto wd = [&](uint64_t p) -> uint32_t { return text_word(t, p, at); };
      uint64_t stray = 0;
      if ((bn & bc) || lead) (void)qid_clean(P0, &bn, &bc, lead, at, wd, &stray);
      if (stray) {  // letters of no token: outside the grammar (dirty_lines / dirty_rewrite)
        if (first) sh.hashy = 1;
        atomic_or_u64(&sh.prebad, stray << (4 * tid));
      }
    }
    atomic_or_u64(&sh.u.m.d[0], (uint64_t)b.d << (4 * tid));
    atomic_or_u64(&sh.u.m.n[0], bn << (4 * tid));
    atomic_or_u64(&sh.u.m.c[0], bc << (4 * tid));
  }
  return bad;
}

// CSR stores (A/B FSVM_NT_STORE: non-temporal -- the outputs are written once)
template <class T>
DA_HD void out_store(T *p, T v) {
#if defined(FSVM_NT_STORE) && defined(__HIP_DEVICE_COMPILE__)
  __builtin_nontemporal_store(v, p);
#else
  *p = v;
#endif
}

// ---- per-line fallback.  A line holding bytes outside the grammar (after
// the tile's comments are blanked) -- a "# header" line of the next file that
// InputSplit put mid-chunk (input_split_base.cc:204-210), which the reference
// reads as a row (libsvm_parser.h:91-104), a word in a value -- takes its run
// positions from walk_line, the reference's line parse; the tile blanks the
// line in its staged text (classification and roles see an empty line), ORs
// the walked runs into its role masks and decodes them with the byte decoders.
// Everything else about the tile is unchanged.  A line the tile cannot walk
// cheaply or fully gates the call over to the exact kernels as before.
enum : uint32_t { DK_L = 1, DK_W = 2, DK_I = 3, DK_V = 4, DK_Q = 5 };
// ParseBlock's line from lb (libsvm_parser.h:85-160) as one byte loop over
// the staged text (offsets into txt): IgnoreCommentAndBlank (:67-83) at its
// start and at every pair end, ParsePair (strtonum.h:667-703) for
// label[:weight] and each index[:value] -- non-digitchars skipped to a run,
// blanks to a ':' -- and "qid:" after the label pair's spaces (:119-132).
// emit(kind, offset) in line order at the run each value is decoded from (a
// ':' at the line end: the line end itself).  The line ends at the first
// '\n' / '\r' after lb or at ue; returns that end, or -1 past lim.
// The staged bytes read a 4-byte word at a time (one LDS round trip per four
// bytes of a serial walk instead of one per byte).
struct WordCache {
  const uint8_t *txt;
  int32_t at = -4;
  uint32_t w = 0;
  DA_HD uint32_t operator()(int32_t p) {
    if ((p & ~3) != at) {
      at = p & ~3;
      w = *reinterpret_cast<const uint32_t *>(txt + at);
    }
    return (w >> (8 * (p & 3))) & 0xFFu;
  }
};
template <class Emit>
DA_HD int32_t walk_line(const uint8_t *txt, int32_t lb, int32_t ue, int32_t lim, Emit emit) {
  int32_t le = lb + 1;
  {  // the line end: a word at a time
    WordCache wc{txt};
    while (le < ue && !is_nl(wc(le))) {
      if (++le > lim) return -1;
    }
  }
  if (le > ue) le = ue;
  WordCache byte{txt};
  enum : uint32_t { ICB, SEEK, RUN, BL, SEEK2, RUN2, QSP };
  uint32_t st = ICB;
  bool head = true;  // the label pair; then the features
  for (int32_t p = lb; p < le;) {
    const uint32_t b = byte(p);
    if (st == ICB) {  // IgnoreCommentAndBlank
      if (b == '#') return le;
      if (is_blank(b)) ++p;
      else st = SEEK;
    } else if (st == SEEK || st == SEEK2) {  // ParsePair: to the next run
      if (is_digitchar(b)) {
        emit(st == SEEK ? (head ? DK_L : DK_I) : (head ? DK_W : DK_V), p);
        st = st == SEEK ? RUN : RUN2;
      } else {
        ++p;
      }
    } else if (st == RUN || st == RUN2) {  // the run (decoded by the caller)
      if (is_digitchar(b)) {
        ++p;
      } else if (st == RUN) {
        st = BL;
      } else {  // the pair's end (after a label pair: its qid)
        st = head ? QSP : ICB;
        head = false;
      }
    } else if (st == BL) {  // blanks, then a ':' or the pair's end
      if (is_blank(b)) {
        ++p;
      } else if (b == ':') {
        ++p;
        st = SEEK2;
      } else {
        st = head ? QSP : ICB;
        head = false;
      }
    } else {  // QSP: spaces, then "qid:<digits>"
      if (b == ' ') {
        ++p;
      } else {
        if (p + 3 < le && b == 'q' && byte(p + 1) == 'i' && byte(p + 2) == 'd' && byte(p + 3) == ':') {
          p += 4;
          emit(DK_Q, p);
          while (p < le && is_digitchar(byte(p))) ++p;
        }
        st = ICB;
      }
    }
  }
  if (st == SEEK2) emit(head ? DK_W : DK_V, le);  // "x:" at the line end: the value after it
  return le;
}

// The tile's segments (and halos) whose flag is set, classified again from
// the staged text (after blanking), each by its wave: lane = byte, one ballot
// per plane; parts: classify_tile's halo bits.  Returns the segment's flag.
template <class BK, class At>
DA_HDF uint32_t reclassify_blanked(const Tile &t, Shared &sh, uint32_t bad, bool changed, uint32_t parts, BK &bk,
                                   At at) {
  const int tid = bk.tid();
  const uint32_t lane = (uint32_t)tid & (kWave - 1), wbase = (uint32_t)tid - lane;
  for (uint64_t m = bk.ballot(changed); m; m &= m - 1) {  // wave-uniform
    const uint32_t sg = wbase + (uint32_t)ctz64(m);
    const uint32_t b = sh.c.text[kPre + sg * kSegB + lane];
    const uint32_t x = b >= 0x80u ? 0x00000100u : sh.cls[b];  // (>= 0x80: outside the grammar)
    Masks mm;
    mm.d = bk.ballot(x & 1u);
    mm.g = bk.ballot((x >> 8) & 1u);
    mm.n = bk.ballot((x >> 16) & 1u);
    mm.c = bk.ballot((x >> 24) & 1u);
    mm.bad = (mm.g & ~mm.d) != 0;
    if (sg == (uint32_t)tid) bad = commit_seg<false>(t, sh, tid, at, false, mm);
  }
  if (parts) (void)classify_tile<false>(t, sh, tid, at, false, parts);
  bk.sync();
  return bad;
}

// Bytes outside the grammar in segment s (G without D; the qid letters are N
// and C) and in the pre-halo.
DA_HD uint64_t outside_mask(const Tile &t, const Shared &sh, int s) {
  const uint64_t P = t.tlo + (uint64_t)s * kSegB;
  if (P >= t.a->n) return 0;
  const uint64_t g = sh.gw[2 * s] | ((uint64_t)sh.gw[2 * s + 1] << 32);
  return g & ~sh.u.m.d[s + 1];
}

// After the comment pass of a tile holding bytes outside the grammar: find
// their lines, walk them (thread 0, in text order), blank them and classify
// the blanked segments again.  Returns the segment's flag, with bit 0 set
// when the call must go to the exact kernels.
template <class BK, class At>
DA_HDF uint32_t dirty_lines(const Tile &t, Shared &sh, uint32_t bad, BK &bk, At at, uint32_t k) {
  (void)k;  // (phase stamps of the diagnostic build)
  const int tid = bk.tid();
  const uint32_t lane = (uint32_t)tid & (kWave - 1);
  const uint64_t wm = bk.ballot(outside_mask(t, sh, tid) != 0);
  if (lane == 0) sh.pend[tid / kWave] = wm;
  bk.sync();
  uint64_t any = sh.prebad;
  for (int w = 0; w < kFWaves; ++w) any |= sh.pend[w];
  if (!any) return bad;  // block-uniform
  const uint64_t n = t.a->n;
  const uint64_t slo = t.tlo >= (uint64_t)kPre ? t.tlo - kPre : 0;  // staged range
  const uint64_t shi = mn<uint64_t>(t.tlo + kTile + kPost, n);
  if (tid == 0) {
    uint32_t gate = 0, nl = 0, ne = 0;
    uint64_t cover = 0;
    const uint8_t *txt = sh.c.text;  // staged offset i <-> position tlo - kPre + i
    const int64_t base = (int64_t)t.tlo - kPre;
    const int32_t s_lo = (int32_t)((int64_t)slo - base), s_hi = (int32_t)((int64_t)shi - base);
    auto visit = [&](uint64_t x) {
      if (gate || x < cover) return;
      const uint64_t F = t.floor_of(x);
      if (F > x) {  // a pre-halo byte whose line ends at a unit start <= tlo
        cover = F;
        return;
      }
      const int32_t xs = (int32_t)((int64_t)x - base);
      if (x < t.tlo) {  // a pre-halo byte: only a line reaching into the tile is this tile's
        for (int32_t i = xs + 1; i <= kPre; ++i)
          if (is_nl(txt[i])) {
            cover = (uint64_t)(base + i);
            return;
          }
      }
      const int64_t fs = (int64_t)F - base;  // the unit start (may lie before the staged bytes)
      const int32_t stop = fs > (int64_t)s_lo ? (int32_t)fs : s_lo;
      int32_t lb = xs;  // the newline opening x's line, or its unit start
      WordCache wc{txt};
      while (lb > stop && !is_nl(wc(lb))) --lb;
      // no newline down to the staged start: the line starts before the staged bytes
      if ((!is_nl(wc(lb)) && (int64_t)lb != fs) || xs - lb > (int32_t)kDirtyMaxLine) {
        gate = 1;
        return;
      }
      const uint64_t ue = mn<uint64_t>(t.next_cs(x), n);
      const int32_t ues = (int32_t)mn<int64_t>((int64_t)ue - base, s_hi);
      const int32_t le = walk_line(txt, lb, ues, mn<int32_t>(lb + (int32_t)kDirtyMaxLine, s_hi),
                                   [&](uint32_t k, int32_t o) {
                                     if (k == DK_Q || ne >= (uint32_t)kDirtyEntries || o >= ues || is_nl(txt[o])) {
                                       gate = 1;  // a qid, too many runs, or a value read past the line end
                                       return;
                                     }
                                     sh.dl[ne++] = (uint32_t)o | (k << 16);  // staged offset
                                   });
      // unwalkable here: too long, ending past the staged bytes, or at a unit
      // end inside a line (the decoders would read on into the next unit)
      if (le < 0 || (le == ues && (uint64_t)(base + le) < n && !is_nl(txt[le]))) {
        gate = 1;
        return;
      }
      const uint64_t lend = (uint64_t)(base + le), lbg = (uint64_t)(base + lb);
      cover = lend;
      if (lend <= t.tlo) return;  // the previous tile's line
      // a line running on into the next tile must show it one of its bytes
      // outside the grammar in its pre-halo (the last 64 bytes of this tile)
      if (lend > t.thi && t.thi < n) {
        const uint64_t last = outside_mask(t, sh, kFThreads - 1);
        const uint64_t P = t.tlo + (uint64_t)(kFThreads - 1) * kSegB;
        const uint64_t from = lbg > P ? lbg - P : 0;
        if (!(last & (~0ull << from))) {
          gate = 1;
          return;
        }
      }
      if (nl >= (uint32_t)kDirtyLines) {
        gate = 1;
        return;
      }
      sh.dr[2 * nl] = (int32_t)((int64_t)lbg - (int64_t)t.tlo);
      sh.dr[2 * nl + 1] = (int32_t)(lend - t.tlo);
      ++nl;
    };
    for (uint64_t m = sh.prebad; m && t.tlo >= (uint64_t)kPre; m &= m - 1) visit(t.tlo - kPre + ctz64(m));
    for (int w = 0; w < kFWaves; ++w)
      for (uint64_t m = sh.pend[w]; m; m &= m - 1) {
        const int s = w * kWave + (int)ctz64(m);
        const uint64_t P = t.tlo + (uint64_t)s * kSegB;
        for (uint64_t b = outside_mask(t, sh, s); b; b &= b - 1) visit(P + ctz64(b));
      }
    sh.ndl = gate ? 0u : ne;
    sh.ndr = gate ? 0u : nl;
    sh.dgate = gate;
  }
  bk.sync();
  FAST_STAMP(k, 13);
  if (sh.dgate) return bad | 1u;
  const uint32_t nr = sh.ndr;
  if (nr == 0) return bad;
  // blank the lines (from the byte after the opening newline, or from the
  // unit start) in the staged text: my segment; wave 0 the pre-halo, the
  // last wave the post-halo
  auto blank_in = [&](uint64_t lo, uint64_t hi) -> bool {  // my staged bytes [lo, hi) of the lines
    bool ch = false;
    for (uint32_t r = 0; r < nr; ++r) {
      const uint64_t lb = (uint64_t)((int64_t)t.tlo + sh.dr[2 * r]), le = t.tlo + (uint64_t)sh.dr[2 * r + 1];
      const uint64_t b0 = is_nl(at(lb)) && t.floor_of(lb) != lb ? lb + 1 : lb;
      const uint64_t a0 = b0 > lo ? b0 : lo, a1 = le < hi ? le : hi;
      for (uint64_t p = a0; p < a1; ++p) {
        sh.c.text[p - t.tlo + kPre] = ' ';
        ch = true;
      }
    }
    return ch;
  };
  const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
  const bool changed = P < n && blank_in(P, mn<uint64_t>(P + kSegB, n));
  uint32_t parts = 0;
  if (tid < kWave && t.tlo > 0) {
    const uint64_t x = t.tlo - kPre + lane;
    if (x >= slo && blank_in(x, x + 1)) parts |= 2u;
  }
  if (tid >= kFThreads - kWave) {
    for (uint64_t x = t.thi + lane; x < shi; x += kWave)
      if (blank_in(x, x + 1)) parts |= 4u;
  }
  const uint64_t pm = bk.ballot((parts & 2u) != 0), qm = bk.ballot((parts & 4u) != 0);
  parts = (pm ? 2u : 0u) | (qm ? 4u : 0u);  // wave-level; made block-level below
  if (parts) atomic_or_u32(&sh.hashy, parts << 8);
  bk.sync();
  parts = (sh.hashy >> 8) & 6u;
  if (tid == 0 && (parts & 2u)) {
    sh.u.m.d[0] = sh.u.m.n[0] = sh.u.m.c[0] = 0;
    sh.prebad = 0;
  }
  bk.sync();
  bad = reclassify_blanked(t, sh, bad, changed, parts, bk, at);
  // the walked runs into the (blanked) planes as one-byte runs whose gaps make
  // the role arithmetic read them as walked: a ':' before a weight or value;
  // a label follows its line's newline or unit start (not blanked)
  {
    const uint32_t ne = sh.ndl;
    const int32_t s0 = kPre + tid * kSegB;  // my segment's staged offsets; the pre-halo: thread 0's slot 0
    uint64_t dd = 0, cc = 0, hd = 0, hc = 0;
    for (uint32_t i = 0; i < ne; ++i) {
      const uint32_t e = sh.dl[i];
      const int32_t o = (int32_t)(e & 0xFFFFu);
      const uint32_t kd = e >> 16;
      const bool kv = kd == DK_W || kd == DK_V;
      if (o >= s0 && o < s0 + kSegB) dd |= 1ull << (o - s0);
      if (kv && o - 1 >= s0 && o - 1 < s0 + kSegB) cc |= 1ull << (o - 1 - s0);
      if (tid == 0 && o < kPre) hd |= 1ull << o;
      if (tid == 0 && kv && o - 1 >= 0 && o - 1 < kPre) hc |= 1ull << (o - 1);
    }
    if (dd | cc) {
      sh.u.m.d[tid + 1] |= dd;
      sh.u.m.c[tid + 1] |= cc;
    }
    if (hd | hc) {
      sh.u.m.d[0] |= hd;
      sh.u.m.c[0] |= hc;
    }
  }
  bk.sync();
  return bad;
}

// ---- dirty rewrite (round 6): lines holding bytes outside the grammar at any
// length and density, without a walk.  Outside a "qid:" token, a byte X that
// is no digitchar, blank, newline or ':' acts in ParseBlock exactly like a
// blank (ParsePair skips it on the way to a run, strtonum.h:671-673 and
// :686-688; IgnoreCommentAndBlank stops at it, libsvm_parser.h:67-83 -- the
// comment pass already read it so) except in three places:
//   * a ':' pairs a value only when it is the first non-blank byte after the
//     run before it (:683-687) -- "5 x:3" is two indices, "5 :x 3" a pair;
//   * ParseFloat reads on past a sign into "inf" / "nan(...)" letters
//     (strtonum.h:133-175): a run of one sign followed by i / n;
//   * "qid:" after the label (libsvm_parser.h:119-132) -- a tile holding a
//     qid marker declines (the walk, dirty_lines, takes it).
// So the tile blanks every X byte and every ':' that is not the first
// non-blank byte after a run end in its staged text and classifies the
// changed segments again -- the role arithmetic then reads the reference's
// pairs.  The letter after a one-sign run ("-inf") becomes an 'e' instead: the
// run stays where it was, and the window decoder, seeing an exponent, hands
// the number to the byte decoder, which reads the text in HBM.  The first non-blank
// byte after each run end is a carry chain through the blanks: the gap
// starts E (a byte after a digitchar) added into the blank plane land on it.
// A segment whose result depends on the gap state at its start takes it from
// the segment before (through all-blank segments); a tile whose answer lies
// before its pre-halo declines.  Returns the tile's flags as dirty_lines;
// *took: false when the tile declined (block-uniform).
constexpr uint32_t kDeclined = 1u << 16;  // Shared::hashy: dirty_rewrite declined the tile
constexpr uint32_t kOutside = 1u << 17;   // Shared::hashy: bytes outside the grammar left after the comment pass
template <class BK, class At>
DA_HDF uint32_t dirty_rewrite(const Tile &t, Shared &sh, uint32_t bad, BK &bk, At at, uint32_t k, bool *took) {
  (void)k;
  const int tid = bk.tid();
  const uint32_t lane = (uint32_t)tid & (kWave - 1);
  const uint64_t n = t.a->n;
  const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
  const bool pre = t.tlo > 0;  // slot 0 holds the 64 bytes before the tile
  // nothing outside the grammar left (the comment pass took it all): done
  if ((P < n && outside_mask(t, sh, tid) != 0) || (tid == 0 && pre && sh.prebad != 0))
    atomic_or_u32(&sh.hashy, kOutside);
  bk.sync();
  if (!(sh.hashy & kOutside)) {  // block-uniform
    *took = true;
    return bad;
  }
  // outside bytes of slot s (0: the pre-halo)
  auto x_of = [&](int s) -> uint64_t { return s == 0 ? (pre ? sh.prebad : 0ull) : outside_mask(t, sh, s - 1); };
  // the gap state after slot s: 1 when its last non-blank byte is a
  // digitchar before its last byte (a gap with blanks only is open at its
  // end); through all-blank slots to the pre-halo, *unk past it
  auto pend_after = [&](int s, bool *unk) -> uint32_t {
    for (; s >= 0; --s) {
      if (s == 0 && !pre) return 0u;
      const uint64_t d = sh.u.m.d[s];
      const uint64_t nb = d | sh.u.m.n[s] | sh.u.m.c[s] | x_of(s);
      if (nb) {
        const int hb = 63 - clz64(nb);
        return ((d >> hb) & 1u) && hb < 63 ? 1u : 0u;
      }
    }
    *unk = true;
    return 0u;
  };
  // bytes of slot s to blank, for a gap state pin at its start and the
  // digitchar bit before it
  auto rewrite = [&](int s, uint64_t valid, uint32_t pin, uint64_t dprev) -> uint64_t {
    const uint64_t d = sh.u.m.d[s], c = sh.u.m.c[s], X = x_of(s) & valid;
    const uint64_t bl = ~(d | sh.u.m.n[s] | c | X) & valid;
    const uint64_t E = ~d & ((d << 1) | dprev) & valid;  // gap starts
    uint32_t co;
    const uint64_t land = (add_carry(bl, E & bl, pin, &co) | E) & ~bl & valid;  // first non-blank after a run end
    return X | (c & ~land);
  };
  uint32_t decline = 0;
  // a qid marker anywhere (the walk takes qid lines), and the rewrite of my segment
  uint64_t R = 0;
  if (P < n) {
    const int s = tid + 1;
    if (sh.u.m.n[s] & sh.u.m.c[s]) decline = 1;
    const uint64_t valid = n - P >= 64 ? ~0ull : (1ull << (n - P)) - 1;
    const uint64_t dprev = (sh.u.m.d[s - 1] >> 63) & 1u;
    const uint64_t r0 = rewrite(s, valid, 0u, dprev), r1 = rewrite(s, valid, 1u, dprev);
    R = r0;
    if (r0 != r1) {  // the gap state at my start decides: from the segments before
      bool unk = false;
      if (pend_after(s - 1, &unk)) R = r1;
      if (unk) decline = 1;
    }
  }
  // the pre-halo (thread 0): the byte before it read from HBM; the gap state
  // at its start is not staged -- it must not matter
  uint64_t Rpre = 0;
  if (tid == 0 && pre) {
    if (sh.u.m.n[0] & sh.u.m.c[0]) decline = 1;
    const uint64_t dp = t.tlo > (uint64_t)kPre && is_digitchar(at(t.tlo - kPre - 1)) ? 1u : 0u;
    Rpre = rewrite(0, ~0ull, 0u, dp);
    if (Rpre != rewrite(0, ~0ull, 1u, dp)) decline = 1;
  }
  if (decline) atomic_or_u32(&sh.hashy, kDeclined);
  bk.sync();
  if (sh.hashy & kDeclined) {  // block-uniform: the walk decides
    *took = false;
    return bad;
  }
  *took = true;
  // the letters after one-sign runs among R (x: the byte's position, bit:
  // its bit; d2: the digitchar planes' bits before it, `bit`-relative): 'e'
  auto inf_marks = [&](uint64_t P0, uint64_t m, uint64_t dcur, uint64_t dbefore) -> uint64_t {
    uint64_t em = 0;
    for (uint64_t mm = m & ((dcur << 1) | (dbefore >> 63)); mm; mm &= mm - 1) {  // bytes right after a run
      const int b = ctz64(mm);
      const uint64_t x = P0 + (uint64_t)b;
      const bool d2 = b >= 2 ? ((dcur >> (b - 2)) & 1u) : ((dbefore >> (62 + b)) & 1u);
      const uint32_t s0 = at(x - 1), l = at(x) | 0x20u;
      if (!d2 && (s0 == '+' || s0 == '-') && (l == 'i' || l == 'n')) em |= 1ull << b;
    }
    return em;
  };
  // R into the staged bytes (a word at a time): blanks, 'e' at em
  auto blank_words = [&](uint8_t *base, uint64_t m, uint64_t em) {
    uint32_t *w = reinterpret_cast<uint32_t *>(base);
    for (uint64_t mm = m; mm;) {
      const int q = ctz64(mm) >> 2;
      const uint32_t nib = (uint32_t)(m >> (4 * q)) & 0xFu, eib = (uint32_t)(em >> (4 * q)) & 0xFu;
      const uint32_t bm = ((nib * 0x00204081u) & 0x01010101u) * 0xFFu;
      const uint32_t be = ((eib * 0x00204081u) & 0x01010101u) * 0xFFu;
      w[q] = (w[q] & ~bm) | (0x20202020u & bm & ~be) | (0x65656565u & be);
      mm &= ~(0xFull << (4 * q));
    }
  };
  if (R) {
    const int s = tid + 1;
    blank_words(sh.c.text + kPre + tid * kSegB, R, inf_marks(P, R & x_of(s), sh.u.m.d[s], sh.u.m.d[s - 1]));
  }
  // the pre-halo: its bytes rewritten, its planes again (classify_tile part
  // 2); the post-halo: its outside bytes rewritten (the last runs' windows),
  // its digit word again (part 4)
  uint32_t parts = 0;
  if (tid == 0 && Rpre) {
    uint64_t dp = 0;  // the digitchar bits of the two bytes before the pre-halo, as bits 62-63
    for (uint64_t i = 1; i <= 2; ++i)
      if (t.tlo >= (uint64_t)kPre + i && is_digitchar(at(t.tlo - kPre - i))) dp |= 1ull << (64 - i);
    blank_words(sh.c.text, Rpre, inf_marks(t.tlo - kPre, Rpre & x_of(0), sh.u.m.d[0], dp));
    parts |= 2u;
  }
  const uint64_t shi = mn<uint64_t>(t.tlo + kTile + kPost, n);
  if (tid >= kFThreads - kWave) {
    // (read from HBM: the bytes before may be rewritten meanwhile)
    for (uint64_t x = t.thi + lane; x < shi; x += kWave) {
      const uint32_t b = gbyte(t.a->text, x);
      if (!is_digitchar(b) && !is_blank(b) && !is_nl(b) && b != ':') {
        const uint32_t s0 = gbyte(t.a->text, x - 1), l = b | 0x20u;
        const bool e = (s0 == '+' || s0 == '-') && !is_digitchar(gbyte(t.a->text, x - 2)) && (l == 'i' || l == 'n');
        sh.c.text[x - t.tlo + kPre] = e ? 'e' : ' ';
        parts |= 4u;
      }
    }
  }
  const uint64_t pm = bk.ballot((parts & 2u) != 0), qm = bk.ballot((parts & 4u) != 0);
  parts = (pm ? 2u : 0u) | (qm ? 4u : 0u);
  if (parts) atomic_or_u32(&sh.hashy, parts << 8);
  bk.sync();
  parts = (sh.hashy >> 8) & 6u;
  if (tid == 0 && (parts & 2u)) {
    sh.u.m.d[0] = sh.u.m.n[0] = sh.u.m.c[0] = 0;
    sh.prebad = 0;
  }
  bk.sync();
  return reclassify_blanked(t, sh, bad, R != 0, parts, bk, at);
}

// After the tile's aggregate is published (MODE 2, before the run lists):
// the walked lines' bytes back into the staged text and the digit plane, for
// the index windows.  (Done before the roles, its global round trip sat on
// the look-back chain: every later tile waits for a dirty tile's aggregate.)
template <class BK, class At>
DA_HDF void dirty_restore(const Tile &t, Shared &sh, BK &bk, At at) {
  const int tid = bk.tid();
  const uint64_t n = t.a->n;
  const uint32_t nr = sh.ndr;
  const uint64_t shi = mn<uint64_t>(t.tlo + kTile + kPost, n);
  const uint32_t parts = (sh.hashy >> 8) & 6u;
  const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
  // the lines' bytes back for the decoders (index windows: exact on any run
  // of digitchars; floats are decoded again at the end), digit-plane bits
  // from the bytes themselves (the table's G also marks bytes outside the
  // grammar)
  // (the bytes come back from global memory in 16-byte loads, all in flight
  // at once: a byte loop waited for one round trip per byte)
  auto restore = [&](uint64_t lo, uint64_t hi, uint64_t *dig) -> uint64_t {  // [lo, hi): 64 bytes from lo (16-aligned)
    uint64_t rm = 0;
    for (uint32_t r = 0; r < nr; ++r) {
      const uint64_t lb = (uint64_t)((int64_t)t.tlo + sh.dr[2 * r]), le = t.tlo + (uint64_t)sh.dr[2 * r + 1];
      const uint64_t b0 = is_nl(at(lb)) && t.floor_of(lb) != lb ? lb + 1 : lb;
      const uint64_t a0 = b0 > lo ? b0 : lo, a1 = le < hi ? le : hi;
      if (a0 < a1) rm |= (a1 - lo >= 64 ? ~0ull : (1ull << (a1 - lo)) - 1) & ~((1ull << (a0 - lo)) - 1);
    }
    if (!rm) return 0;
    uint32_t w[16];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint64_t g = lo + 16 * (uint64_t)q;
      if (g + 16 <= n) {
        load16(t.a->text + g, w + 4 * q);
      } else {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          uint32_t x = 0;
          for (int b = 0; b < 4; ++b) {
            const uint64_t pp = g + 4 * j + b;
            x |= (pp < n ? (uint32_t)gbyte(t.a->text, pp) : 0u) << (8 * b);
          }
          w[4 * q + j] = x;
        }
      }
    }
    uint32_t *lw = reinterpret_cast<uint32_t *>(sh.c.text + (lo - t.tlo + kPre));
    uint64_t dg = 0;
#pragma unroll
    for (int q = 0; q < 16; ++q) {
      const uint32_t nib = (uint32_t)(rm >> (4 * q)) & 0xFu;
      if (!nib) continue;
      const uint32_t bm = ((nib * 0x00204081u) & 0x01010101u) * 0xFFu, x = w[q];
      lw[q] = (lw[q] & ~bm) | (x & bm);
      const uint32_t d = ((x | 0x80808080u) - 0x30303030u) & ~((x | 0x80808080u) - 0x3A3A3A3Au) & ~x & 0x80808080u;
      dg |= (uint64_t)(hi_nib(d) & nib) << (4 * q);
    }
    *dig = dg;
    return rm;
  };
  if (P < n) {
    uint64_t dig = 0;
    const uint64_t rm = restore(P, mn<uint64_t>(P + kSegB, n), &dig);
    if (rm) {
      const uint64_t g = ((sh.gw[2 * tid] | ((uint64_t)sh.gw[2 * tid + 1] << 32)) & ~rm) | dig;
      sh.gw[2 * tid] = (uint32_t)g;
      sh.gw[2 * tid + 1] = (uint32_t)(g >> 32);
    }
  }
  if (parts & 4u) {  // the post-halo (kPost = 128 bytes): two lanes of the last wave, 64 bytes each
    if (tid >= kFThreads - 2) {
      const uint64_t lo = t.thi + (uint64_t)(tid - (kFThreads - 2)) * kSegB;
      uint64_t dig = 0;
      const uint64_t rm = lo < shi ? restore(lo, mn<uint64_t>(lo + kSegB, shi), &dig) : 0;
      if (tid == kFThreads - 2) sh.gw[2 * kFThreads] = (uint32_t)((sh.gw[2 * kFThreads] & ~rm) | dig);
    }
  }
}

// Pass 1 (libsvm): blank the comments and classify again what changed; all
// threads, after the chunk list is known.  bad0: the segment's pass-0 flag.
// (inline: out of line, the call frame's spills cost the kernel 2.2x, 3.97 ms
// on config 2)
template <class BK>
DA_HDF uint32_t comments_reclassify(const Tile t, Shared &sh, uint32_t bad0, BK &bk, uint32_t k) {
  (void)k;  // (phase stamps of the diagnostic build)
  const int tid = bk.tid();
  const FastSvmArgs &a = *t.a;
  uint64_t Mp = 0;
  const bool planes_ok = !((sh.qfail[tid / kWave] >> (tid % kWave)) & 1u);
  const uint32_t e = comment_erase(t.tlo, t.thi, a.n, sh.c, &sh.hashy, bk, sh.u.m.d[tid + 1], sh.u.m.n[tid + 1],
                                   sh.u.m.c[tid + 1], bad0 != 0, k, planes_ok, &Mp);
  if (Mp) {  // my segment's comment out of its planes; its flag: bytes outside the grammar left
    const uint64_t d = sh.u.m.d[tid + 1] & ~Mp;
    sh.u.m.d[tid + 1] = d;
    sh.u.m.n[tid + 1] &= ~Mp;
    sh.u.m.c[tid + 1] &= ~Mp;
    const uint64_t g = (sh.gw[2 * tid] | ((uint64_t)sh.gw[2 * tid + 1] << 32)) & ~Mp;
    sh.gw[2 * tid] = (uint32_t)g;
    sh.gw[2 * tid + 1] = (uint32_t)(g >> 32);
    bad0 = (g & ~d) != 0 ? 1u : 0u;
  }
  if (e & 12u) atomic_or_u32(&sh.hashy, (e & 12u) << 1);  // pre-halo / post-halo blanked: note bits 3 / 4
  if (tid == 0 && (e & 4u)) {
    sh.u.m.d[0] = sh.u.m.n[0] = sh.u.m.c[0] = 0;
    sh.prebad = 0;
  }
  bk.sync();
  FAST_STAMP(k, 16);
  auto at = [&](uint64_t p) -> uint32_t {
    if (p >= a.n) return 0u;
    return p + kPre >= t.tlo ? (uint32_t)sh.c.text[p - t.tlo + kPre] : gbyte(a.text, p);
  };
  // the blanked segments classified again, each by its wave (lane = byte)
  const uint32_t parts = (sh.hashy >> 2) & 6u;  // the halos (rare): classify_tile's lanes
  const uint32_t bad = reclassify_blanked(t, sh, bad0, (e >> 1) & 1u, parts, bk, at);
  return bad | (e & 1u);
}

// The tables every tile reads (byte classes, decoder constants): per tile,
// or once per workgroup in the persistent form.
template <class BK>
DA_HDF void init_tables(Shared &sh, BK &bk) {
  for (int i = bk.tid(); i < kClsEntries; i += kFThreads) sh.cls[i] = class_of((uint32_t)i);
  init_dec_tables(sh.dt, bk);
}

// MODE 1: count only (size query); MODE 2: parse and write.
//
// PERSIST (the kernel's workgroups loop over tiles, svm_fast_tile): `sr`
// already holds tile k's staged loads and the tables are in place; the tile
// takes the next tile id from the launch's ticket early on (one returning
// atomic, its latency hidden behind the tile's work) and issues that tile's
// loads into `sr` once its own register batch is stored, so the next tile's
// HBM latency overlaps this tile's stores.  Returns the next tile id (block
// uniform).  Deadlock-free in any residency: a tile id is handed out only to
// a resident workgroup, after every lower id was.
template <int MODE, bool FM = false, bool PERSIST = false, class BK>
DA_HDF uint32_t tile_p(const FastSvmArgs &a, Shared &sh, BK &bk, uint32_t k, StageRegs &sr) {
  // Tile k = workgroup k (its blockIdx).  The look-back needs every tile's
  // predecessors to become resident eventually; workgroups are dispatched in
  // index order on every XCD, so the least unstarted tile's XCD only holds
  // lower tiles, which finish.  (A device-wide ticket counter gave the same
  // guarantee for any dispatch order but saturates near 88 grabs/us -- it
  // capped the 131k-tile launch at ~1.5 ms.)  Should a predecessor ever not
  // publish, kSpinLimit bounds the wait and the exact kernels take over.
  const int tid = bk.tid();
  if (!PERSIST && a.skip_if_gated && *a.gate) return a.ntiles;  // fill phase after an exact-path count: block-uniform
  // after the lean kernel (svm_lean.h): resume at its first poisoned tile kf
  // (the word holds ~kf; 0: none poisoned, nothing left to do), tile kf's
  // exclusive prefix seeded by the lean inclusive prefix of tile kf - 1
  uint32_t kf = 0;
  const uint64_t *seed = nullptr;  // tile kf's exclusive prefix: the lean inclusive words of kf - 1 (marked)
  if (!PERSIST && a.lean_poison) {
    const uint64_t pw = *a.lean_poison;  // stable: the lean launch has finished
    kf = pw ? (uint32_t)mn<uint64_t>(~pw, (uint64_t)a.ntiles) : a.ntiles;
    if (k < kf) return a.ntiles;  // block-uniform
    if (k == kf && kf > 0) seed = a.lean_lb + (uint64_t)a.ntiles + (uint64_t)(kf - 1) * 4;
  }
  FAST_STAMP(k, 0);
  FAST_STAMP(k, 1);
  Tile t;
  t.a = &a;
  t.sh = &sh;
  t.tlo = (uint64_t)k * kTile;
  t.thi = mn<uint64_t>(t.tlo + kTile, a.n);
  uint32_t knext = a.ntiles;  // thread 0: the ticket's answer (PERSIST)
  if (PERSIST && tid == 0) knext = gridDim_x() + atomic_add_u32(a.ticket, 1u);
#if defined(FSVM_GLDS) && defined(__HIP_DEVICE_COMPILE__)
  if (!PERSIST) stage_issue_lds(a.text, a.n, t.tlo, sr, sh.c, bk);  // text loads first: the chunk search overlaps them
#else
  if (!PERSIST) stage_issue(a.text, a.n, t.tlo, sr, bk);  // text loads first: the chunk search overlaps them
#endif
#ifdef FSVM_PF_AHEAD  // A/B: touch tile k + FSVM_PF_AHEAD (same XCD) so its staging hits L2 / MALL
  uint32_t pfv = 0;
  {
    const uint64_t pk = (uint64_t)k + FSVM_PF_AHEAD, off = pk * kTile + (uint64_t)tid * kSegB;
    if (pk < a.ntiles && off < a.n) pfv = a.text[off];
  }
#endif
  ChunkProbe cp;  // wave 0: the window load stays in flight through classification
  if (tid < kWave) cp = chunk_list_begin(a.cs, a.nchunk, t.tlo, bk);
  FAST_STAMP(k, 11);
  if (tid == 0) {
    sh.u.m.d[0] = sh.u.m.n[0] = sh.u.m.c[0] = 0;
    sh.nq = 0;
    for (int w = 0; w < kFWaves; ++w) sh.qfail[w] = 0;
    sh.hashy = 0;
    sh.prebad = 0;
    sh.ndl = sh.ndr = sh.nseg = sh.dgate = 0;
  }
  if (!PERSIST) init_tables(sh, bk);
  stage_commit(a.text, a.n, t.tlo, sr, sh.c, bk);
  bk.sync();
  FAST_STAMP(k, 2);
#if defined(FSVM_ABL_STOP) && FSVM_ABL_STOP == 0  // timing ablation only: stage
  if (sh.c.text[tid] == 0xAB && sh.c.ncs == 7) a.res[15] = sh.c.cnext;
  return a.ntiles;
#endif
  // ---- classify: segment tid -> slot tid+1; lanes 0..15 also one word each
  // of the 64 bytes before the tile -> slot 0
  // a text byte (0 outside the text) for the qid token checks: staged, or
  // from global memory before the staged bytes
  auto at = [&](uint64_t p) -> uint32_t {
    if (p >= a.n) return 0u;
    return p + kPre >= t.tlo ? (uint32_t)sh.c.text[p - t.tlo + kPre] : gbyte(a.text, p);
  };
  uint32_t bad = classify_tile<FM>(t, sh, tid, at, true, 7u);
  FAST_STAMP(k, 9);
  if (tid < kWave) chunk_list_end(a.cs, a.nchunk, t.tlo, t.thi, cp, sh.c, bk);
  FAST_STAMP(k, 10);
  bk.sync();
  // a byte outside the grammar ('#' among them) in the tile or in the pre-halo:
  // blank the comments and classify again (block-uniform, libsvm only)
  if (!FM && __builtin_expect(sh.hashy != 0, 0)) {
#ifndef FSVM_NO_PRIO
    // until its aggregate is published, this tile holds up every later
    // tile's look-back: its waves go first (A/B: FSVM_NO_PRIO)
    prio_high();
#endif
    // The comment pass first, unless at most two segments (the pre-halo
    // counting as one) hold bytes outside the grammar and every '#' among
    // them opens a line (only blanks back to a newline: no comment to the
    // reference, libsvm_parser.h:91-96) -- a file header, one odd line:
    // then the walk takes their lines alone.
    // (nseg: counted by commit_seg before the classify barrier; stable until the next one)
    const uint32_t nseg = sh.nseg + (sh.prebad != 0 ? 1u : 0u);
    if (nseg <= 2u) {  // block-uniform: does every '#' of those segments open a line?
      // (thread 0 also takes the pre-halo's bytes, first)
      const uint64_t om = outside_mask(t, sh, tid);
      const bool pre = tid == 0 && sh.prebad && t.tlo >= (uint64_t)kPre;
      if (om || pre) {
        const uint64_t slo = t.tlo >= (uint64_t)kPre ? t.tlo - kPre : 0;
        uint64_t P = pre ? slo : t.tlo + (uint64_t)tid * kSegB, m = pre ? sh.prebad : om, rest = pre ? om : 0;
        for (;; m &= m - 1) {
          if (!m) {
            if (!rest) break;
            m = rest;
            rest = 0;
            P = t.tlo;
          }
          const uint64_t x = P + ctz64(m);
          if (at(x) != '#') continue;
          uint64_t y = x;
          while (y > slo && is_blank(at(y - 1))) --y;
          if (y == 0 || !is_nl(at(y - 1)) || t.is_cs(y)) {  // a comment, or not a line-start '#'
            atomic_or_u32(&sh.dgate, 1u);  // (dirty_lines sets it again later)
            break;
          }
        }
      }
      bk.sync();
    }
    if (nseg > 2u || sh.dgate) bad = comments_reclassify(t, sh, bad, bk, k);
    FAST_STAMP(k, 12);
    // lines still holding bytes outside the grammar: rewritten, else walked
    bool took = false;
    bad = dirty_rewrite(t, sh, bad, bk, at, k, &took);
    if (!took) bad = dirty_lines(t, sh, bad, bk, at, k);
    FAST_STAMP(k, 14);
  }
  if (tid == 0) bad |= sh.c.toomany;
  FAST_STAMP(k, 3);
#if defined(FSVM_ABL_STOP) && FSVM_ABL_STOP == 1  // timing ablation only: stage + classify
  if (sh.u.m.d[tid + 1] == 0x123456789ull) a.res[15] = sh.u.m.n[tid];
  return a.ntiles;
#endif
  // ---- roles, counts, eligibility
  SegOut so;
  so.Q = 0;
  uint64_t soF = 0, soRS = 0, soQ0 = kNone;  // libfm: field runs (v1), all run starts, the run before
  if constexpr (FM) {
    const SegOutFm sf = segment_roles_fm(t, tid);
    so.L = sf.L;
    so.W = sf.W;
    so.I = sf.I;
    so.V = sf.V;
    so.bad = sf.bad;
    soF = sf.F;
    soRS = sf.RS;
    soQ0 = sf.q0;
  } else {
    so = segment_roles(t, tid);
    if (so.Q) atomic_add_u32(&sh.nq, (uint32_t)popc64(so.Q));
  }
  if (so.bad | bad) atomic_or_u32(&sh.c.bad, 1u);
  // per-thread role counts packed in 16-bit fields (a tile holds < 2^16 runs)
  const uint64_t mine = (uint64_t)popc64(so.L) | ((uint64_t)popc64(so.W) << 16) |
                        ((uint64_t)popc64(so.I) << 32) | ((uint64_t)popc64(so.V) << 48);
  uint64_t totp;
#ifdef FSVM_DPP_SCAN
  const uint64_t ex = bk.exclusive_add(mine, &totp);
#elif defined(FSVM_SCAN1) && defined(__HIP_DEVICE_COMPILE__)
  const uint64_t ex = bk.exclusive1(mine, (uint64_t)0, AddU64(), &totp);
#else
  const uint64_t ex = bk.exclusive(mine, (uint64_t)0, AddU64(), &totp);
#endif
  FAST_STAMP(k, 4);
  const uint32_t nL = (uint32_t)(totp & 0xFFFF), nW = (uint32_t)((totp >> 16) & 0xFFFF),
                 nI = (uint32_t)((totp >> 32) & 0xFFFF), nV = (uint32_t)(totp >> 48);
#if defined(FSVM_ABL_STOP) && FSVM_ABL_STOP == 2  // + roles + block scan
  if (ex == 0x123456789ull) a.res[15] = totp;
  return a.ntiles;
#endif
#ifndef FSVM_NO_PRIO
  if (!FM) prio_normal();  // (every wave resets its own; one scalar instruction, no LDS read)
#endif
  // ---- publish this tile's aggregate
  const uint32_t cnt4[4] = {nL, nI, nV, nW};  // look-back slots Q_ROWS, Q_INDEX, Q_VALUE, Q_WEIGHT
  if (tid == 0) {
    publish_aggregate(a.lb, a.ntiles, k, cnt4, kf, seed);
    if (sh.c.bad) atomic_or_u32(a.gate, 1u);
    if (!FM && sh.nq) {  // the qid decision's sum (libsvm.hip), and the "some qid" word
      atomic_add_u64(a.qsum + (k % kLabShards) * 8, sh.nq);
      if (load_agent_u64(a.qsum + 1) == 0) store_agent_u64(a.qsum + 1, 1);
    }
  }
  const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
  const bool one_chunk = sh.c.ncs == 0;  // no chunk boundary before cnext
  // the window decoders are exact when their 16 bytes belong to the run's
  // chunk: the chunk end after tile offset o, tile-relative (clamped)
  const uint32_t lim1 = (uint32_t)mn<uint64_t>(sh.c.cnext - t.tlo, 0xFFFFFFFFull);
  auto limr_of = [&](uint32_t o) -> uint32_t {
    return one_chunk ? lim1 : (uint32_t)mn<uint64_t>(t.next_cs(t.tlo + o) - t.tlo, 0xFFFFFFFFull);
  };
  auto lim_of = [&](uint64_t q) { return one_chunk ? sh.c.cnext : t.next_cs(q); };
  // non-digit flags of the 16 window bytes at tile offset o (bits 16+ unused)
  auto ndig_at = [&](uint32_t o) -> uint32_t {
#if defined(FSVM_UAWIN) && defined(__HIP_DEVICE_COMPILE__)
    uint32_t x;  // the plane bytes from o / 8 on: one unaligned ds_read_b32
    __builtin_memcpy(&x, reinterpret_cast<const uint8_t *>(sh.gw) + (o >> 3), 4);
    return ~(x >> (o & 7u));
#endif
    const uint32_t i = o >> 5;
    return ~funnel(sh.gw[i + 1], sh.gw[i], o & 31u);
  };
  // The decoders take the run's tile offset o (the run starts at tlo + o).
  // win_*: the branch-free window form; *ok = false sends the run to the
  // byte decoders (slow_*), which also raise the sign error.
  // a float of a walked line (dirty_lines) takes the byte decoder: its window
  // need not look like the grammar's numbers (indices do not: any digitchar
  // run reads as ParseUnsignedInt reads it)
  const uint32_t ndr = FM ? 0u : sh.ndr;
  auto in_dirty = [&](uint32_t o) -> bool {
    for (uint32_t r = 0; r < ndr; ++r)
      if ((int32_t)o >= sh.dr[2 * r] && (int32_t)o < sh.dr[2 * r + 1]) return true;
    return false;
  };
  auto win_float = [&](uint32_t o, bool *ok) -> float {
#ifdef FSVM_ABL_NODEC  // timing ablation only (tools/build_variants.sh), never shipped
    *ok = true;
    return (float)o;
#endif
    const W16 wq = win_at_o(sh.c.text, o);
    const uint32_t w4[4] = {(uint32_t)wq.lo, (uint32_t)(wq.lo >> 32), (uint32_t)wq.hi, (uint32_t)(wq.hi >> 32)};
    bool k1;
    const float v = wfloat32m(w4, ndig_at(o), sh.dt, &k1);
    *ok = k1 && o + 16u <= limr_of(o) && (ndr == 0 || !in_dirty(o));
    return v;
  };
  // the id as read (<= 8 digits: 32 bits); ids_of applies indexing_mode > 0
  // in the index width
  auto win_index = [&](uint32_t o, bool *ok) -> uint32_t {
#ifdef FSVM_ABL_NODEC
    *ok = true;
    return o;
#endif
    const W16 wq = win_at_o(sh.c.text, o);
    const uint32_t w4[4] = {(uint32_t)wq.lo, (uint32_t)(wq.lo >> 32), (uint32_t)wq.hi, (uint32_t)(wq.hi >> 32)};
    uint64_t v;
    bool k1;
    const bool pos = wuint32m(w4, ndig_at(o), sh.dt, &v, &k1);
    *ok = k1 && pos && o + 16u <= limr_of(o);
    return (uint32_t)v;
  };
  auto ids_of = [&](uint32_t v) -> uint64_t { return (uint64_t)v - (a.indexing_mode > 0 ? 1u : 0u); };
  auto slow_flt = [&](uint32_t o) -> float { return slow_float(a.text, t.tlo + o, lim_of(t.tlo + o)); };
  auto slow_idx = [&](uint32_t o) -> uint64_t {
    uint64_t v = 0;
    if (!slow_uint(a.text, t.tlo + o, lim_of(t.tlo + o), a.wide, &v)) {
      raise_error(a.err, E_NEG_INDEX, t.tlo + o);
      v = 0;
    }
    return a.indexing_mode > 0 ? v - 1 : v;
  };
  // A run the window decoders leave (ok false: an exponent, a long number,
  // a window past its chunk, a '-' index) is not decoded in place: its
  // entry's bit goes to a per-thread mask (bit u: list entry tid + 256 u of
  // the pass) and one loop per pass runs the byte decoders on those entries
  // -- one inlined copy of them, off the hot loops' straight-line code.
#ifndef FSVM_KB
#define FSVM_KB 3
#endif
  constexpr int kB = FSVM_KB;  // runs per decoder decoded before the look-back
  static_assert(kB >= 1 && kB <= 5, "batch positions are packed 6 bits each");
  static_assert((kListCap + kFThreads - 1) / kFThreads <= 32, "slow-entry masks hold one bit per list round");
  uint32_t ib[kB];
  float fb[kB];
  uint32_t slowI = 0, slowF = 0;  // this pass's list rounds whose run takes the byte decoders
  // packed counts (fields as `mine`)
  auto fL = [](uint64_t x) { return (uint32_t)(x & 0xFFFF); };
  auto fW = [](uint64_t x) { return (uint32_t)((x >> 16) & 0xFFFF); };
  auto fI = [](uint64_t x) { return (uint32_t)((x >> 32) & 0xFFFF); };
  auto fV = [](uint64_t x) { return (uint32_t)(x >> 48); };

  // ---- libsvm: run lists.  Every run's tile offset goes to an LDS list in
  // output order -- indices, then values, labels, weights -- and the threads
  // decode the lists round-robin: each wave decodes ceil(runs / 256) runs per
  // list instead of its fullest lane's count, and the stores of consecutive
  // lanes are consecutive.  The lists reuse the planes' LDS; a tile with more
  // runs than fit is done in passes of consecutive segments.
  uint32_t np = 1, mypass = 0;
  uint64_t pe0 = totp;  // packed inclusive counts at the end of pass 0
  // libfm adds a field list after the indices: entry j = the staged offset
  // (tile offset + kPre) of index j's field run, the run before it
  auto build = [&](uint64_t s, uint64_t e) {  // my runs into the lists of the pass [s, e)
    const uint64_t rel = ex - s, cn = e - s;
    const uint32_t nIp = fI(cn), nVp = fV(cn), nLp = fL(cn);
    const uint32_t o0 = (uint32_t)tid * kSegB;
    // a mask's run starts, in order, from entry x on (one loop over the 64-bit
    // mask: two loops over its 32-bit halves measured slower, a VGPR spill)
    auto put_list = [&](uint64_t m, uint32_t x) {
      for (; m; m &= m - 1) sh.u.lst[x++] = (uint16_t)(o0 + ctz64(m));
    };
    put_list(so.I, fI(rel));
    uint32_t x;
    uint32_t fb0 = nIp;  // first float entry
    if constexpr (FM) {
      x = nIp + fI(rel);
      for (uint64_t m = so.I; m; m &= m - 1) {
        const uint64_t before = soRS & ((m & (0 - m)) - 1);
        const uint64_t fpos = before ? P + 63 - clz64(before) : soQ0;  // checked >= tlo - kPre (roles)
        sh.u.lst[x++] = (uint16_t)(fpos + kPre - t.tlo);
      }
      fb0 = 2 * nIp;
    }
    put_list(so.V, fb0 + fV(rel));
    put_list(so.L, fb0 + nVp + fL(rel));
    put_list(so.W, fb0 + nVp + nLp + fW(rel));
  };
  // (block-uniform: a tile whose dirty lines were walked)
  if (MODE == 2 && !FM && sh.ndr != 0 && !sh.dgate) dirty_restore(t, sh, bk, at);
  if (MODE == 2) {
    // (the block scan's barriers ordered every plane read before these writes)
    constexpr uint32_t kIW = FM ? 2u : 1u;  // list entries per index (libfm: + its field)
    if (nL + nW + kIW * nI + nV > kPassRuns) {  // block-uniform: several passes
      const uint32_t own = fL(mine) + fW(mine) + kIW * fI(mine) + fV(mine);
      const uint32_t tex = fL(ex) + fW(ex) + kIW * fI(ex) + fV(ex);
      mypass = tex / kPassRuns;
      if (tid == kFThreads - 1 || (tex + own) / kPassRuns != mypass) sh.pend[mypass] = ex + mine;
      if (tid == kFThreads - 1) sh.npass = mypass + 1;
      bk.sync();
      np = sh.npass;
      pe0 = sh.pend[0];
    }
    if (mypass == 0) build(0, pe0);
    bk.sync();
    FAST_STAMP(k, 5);
    // ---- first decode batch into registers (gives predecessors time to publish)
    const uint32_t nI0 = fI(pe0), nF0 = fV(pe0) + fL(pe0) + fW(pe0), fb0 = kIW * nI0;
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const uint32_t j = (uint32_t)tid + (uint32_t)u * kFThreads;
      ib[u] = 0;
      fb[u] = 0.f;
      bool oki = true, okf = true;
      if (j < nI0) ib[u] = win_index(sh.u.lst[j], &oki);
      if (j < nF0) fb[u] = win_float(sh.u.lst[fb0 + j], &okf);
      slowI |= (oki ? 0u : 1u) << u;
      slowF |= (okf ? 0u : 1u) << u;
    }
    FAST_STAMP(k, 6);
  }
  // ---- decoupled look-back by wave 0 (fast_common.h)
#ifdef FSVM_ABL_NOLB  // timing ablation only: write pass without look-back (bases k * counts, in bounds)
  if (MODE == 2 && tid < 4) {
    const int slot = tid == Q_ROWS ? C_ROWS : tid == Q_INDEX ? C_INDEX : tid == Q_VALUE ? C_VALUE : C_WEIGHT;
    const uint64_t c = cnt4[tid], cap = a.cap[slot];
    sh.c.base[tid] = cap > c + 64 ? mn<uint64_t>((uint64_t)k * c, cap - c - 64) : 0;
  }
  if (MODE != 2 && tid < kWave) {
#else
  if (tid < kWave) {
#endif
#ifdef FSVM_LB_PRIO  // A/B: the look-back wave ahead of the other tiles' waves
    prio_high();
#endif
    const uint32_t rounds =
        look_back(a.lb, a.ntiles, k, cnt4, a.gate, sh.c, bk, kf, seed);
#ifdef FSVM_LB_PRIO
    prio_normal();
#endif
#if defined(DMLC_AMD_STAMPS) && defined(__HIP_DEVICE_COMPILE__)
    if (tid == 0 && k < kStampTiles) g_stamps[(uint64_t)k * kStampSlots + 15] = rounds;
#else
    (void)rounds;
#endif
#ifdef DMLC_AMD_VALVE_TEST  // test-only build (lib/variants): the write pass of tile 1 hands over
    if (MODE == 2 && k == 1 && tid == 0) atomic_or_u32(a.gate, 2u);
#endif
  }
  if (PERSIST && tid == 0) sh.next = knext;
  bk.sync();
  FAST_STAMP(k, 7);
  const uint32_t kn = PERSIST ? sh.next : a.ntiles;
#if defined(FSVM_ABL_STOP) && FSVM_ABL_STOP == 3  // + first decode batch + look-back
  if (sh.c.base[0] == 0x123456789ull) a.res[15] = (uint64_t)ib[0] + (uint64_t)fb[0];
  return a.ntiles;
#endif
  const uint64_t bRows = sh.c.base[Q_ROWS], bIdx = sh.c.base[Q_INDEX], bVal = sh.c.base[Q_VALUE],
                 bW = sh.c.base[Q_WEIGHT];
  // ---- the last tile publishes the totals (dmlc_amd_result.count)
  if (k + 1 == a.ntiles && tid == 0) {
    const uint64_t rows = bRows + nL;
    a.res[C_ROWS] = rows;
    a.res[C_INDEX] = bIdx + nI;
    a.res[C_VALUE] = bVal + nV;
    a.res[C_WEIGHT] = bW + nW;
    a.res[C_QID] = 0;
    a.res[C_LABEL] = rows;
    a.res[C_FIELD] = FM ? bIdx + nI : 0;
    if (MODE == 2 && a.offset && rows < a.cap[C_ROWS] + 1) a.offset[rows] = bIdx + nI;
  }
  if (MODE != 2) {
    if (PERSIST && kn < a.ntiles) stage_issue(a.text, a.n, (uint64_t)kn * kTile, sr, bk);
    return kn;
  }

  // ---- stores
  const uint64_t eL = bRows + fL(ex), eW = bW + fW(ex), eI = bIdx + fI(ex), eV = bVal + fV(ex);
  // indexing_mode < 0 (umin_fix): whether a unit holds a 0 id -- all the
  // reference's rule needs (min_index > 0 <=> no id is 0).  A 0 id marks its
  // unit's word with a plain store of 0 (in a register first when the tile
  // lies inside one unit): no atomics, which on one word per unit serialise
  // (a wave minimum by atomicMin on every tile cost config 2 4.7x)
  const bool imin = a.indexing_mode < 0;
  bool zero = false;
  auto note_min = [&](uint64_t q, uint64_t v) {
    const uint64_t sv = a.wide ? v : (uint64_t)(uint32_t)v;
    if (sv != 0) return;
    if (one_chunk) {
      zero = true;
    } else {
      uint32_t u = sh.c.c_first - 1;
      for (uint32_t i = 0; i < sh.c.ncs; ++i) u += sh.c.csl[i] <= q ? 1u : 0u;
      store_flag_u64(&a.umin[u], 0);
    }
  };
#ifdef FSVM_INB  // A/B: every store of the tile in bounds (block-uniform): no per-store capacity branch
  const bool inb = bRows + nL <= a.cap[C_ROWS] && bIdx + nI <= a.cap[C_INDEX] && bVal + nV <= a.cap[C_VALUE] &&
                   bW + nW <= a.cap[C_WEIGHT] && (!FM || bIdx + nI <= a.cap[C_FIELD]);
#else
  constexpr bool inb = false;
#endif
  auto put_index = [&](uint64_t r, uint64_t v, uint64_t q) {
    if (imin) note_min(q, v);
#ifdef FSVM_ABL_NOSTORE  // timing ablation only
    if (v == 0x123456789ull) a.res[15] = r;
    return;
#endif
    if (inb) {
      if (a.wide) reinterpret_cast<uint64_t *>(a.index)[r] = v;
      else reinterpret_cast<uint32_t *>(a.index)[r] = (uint32_t)v;
      return;
    }
    if (r < a.cap[C_INDEX]) {
      if (a.wide) out_store(reinterpret_cast<uint64_t *>(a.index) + r, v);
      else out_store(reinterpret_cast<uint32_t *>(a.index) + r, (uint32_t)v);
    } else {
      raise_error(a.err, E_CAPACITY, q);
    }
  };
  auto put_value = [&](uint64_t r, float v, uint64_t q) {
#ifdef FSVM_ABL_NOSTORE
    if (v == 1234.5f) a.res[15] = r;
    return;
#endif
    if (r < a.cap[C_VALUE]) out_store(a.value + r, v);
    else raise_error(a.err, E_CAPACITY, q);
  };
  auto put_label = [&](uint64_t r, float v, uint64_t q) {
    if (r < a.cap[C_ROWS]) out_store(a.label + r, v);
    else raise_error(a.err, E_CAPACITY, q);
  };
  auto put_weight = [&](uint64_t r, float v, uint64_t q) {
    if (r < a.cap[C_WEIGHT]) a.weight[r] = v;
    else raise_error(a.err, E_CAPACITY, q);
  };
  // entry j of the float list of the pass starting at packed counts s
  auto put_float = [&](uint32_t j, float v, uint32_t o, uint64_t s, uint32_t nVp, uint32_t nLp) {
    if (inb) {  // one store through a selected address
      float *dst = j < nVp ? a.value + (bVal + fV(s) + j)
                           : j < nVp + nLp ? a.label + (bRows + fL(s) + (j - nVp))
                                           : a.weight + (bW + fW(s) + (j - nVp - nLp));
      *dst = v;
      return;
    }
    const uint64_t q = t.tlo + o;
    if (j < nVp) put_value(bVal + fV(s) + j, v, q);
    else if (j < nVp + nLp) put_label(bRows + fL(s) + (j - nVp), v, q);
    else put_weight(bW + fW(s) + (j - nVp - nLp), v, q);
  };
  // libfm: the field run at staged offset so (a window when it lies inside
  // its chunk; a '-' is raised by the sign check below)
  auto put_field = [&](uint64_t r, uint32_t so) {
    const uint64_t q = t.tlo + so - kPre;
    const uint64_t lim = lim_of(q);
    uint64_t v = 0;
    bool ok = false, pos = true;
    if (q + 16 <= lim) {
      const W16 wq = win_at(sh.c.text, t.tlo, q);
      const uint32_t w4[4] = {(uint32_t)wq.lo, (uint32_t)(wq.lo >> 32), (uint32_t)wq.hi, (uint32_t)(wq.hi >> 32)};
      pos = wuint32(w4, sh.dt, &v, &ok);
    }
    if (!ok) pos = slow_uint(a.text, q, lim, a.wide, &v);
    if (!pos) v = 0;
    if (a.indexing_mode > 0) --v;
    if (imin) note_min(q, v);
    if (r < a.cap[C_FIELD]) {
      if (a.wide) reinterpret_cast<uint64_t *>(a.field)[r] = v;
      else reinterpret_cast<uint32_t *>(a.field)[r] = (uint32_t)v;
    } else {
      raise_error(a.err, E_CAPACITY, q);
    }
  };
  // Row offsets, qids and the chunk table first: the segment's role masks
  // die here instead of staying live through the decode loops below.
  // each row's offset: the indices before its label
  uint64_t rl = eL;
  for (uint64_t m = so.L; m; m &= m - 1, ++rl) {
    const uint64_t below = (m & (0 - m)) - 1;
    if (inb || rl < a.cap[C_ROWS]) out_store(a.offset + rl, (uint64_t)(eI + popc64(so.I & below)));
    else raise_error(a.err, E_CAPACITY, P + ctz64(m));
  }
  if constexpr (!FM) {
    // qid runs (every row has one when this path stands, qid_fix_kernel):
    // row r's id, atoll of its digits (libsvm_parser.h:126-130)
    for (uint64_t m = so.Q; m; m &= m - 1) {
      const uint64_t bit = m & (0 - m), x = P + ctz64(m);
      const uint64_t r = eL + popc64(so.L & (bit - 1)) - 1;  // the row of the label before it
      // 1-18 digits (qid_ok), staged: the 16-byte window unless longer than 15
      const W16 w = win_at(sh.c.text, t.tlo, x);
      const uint32_t len = run_len(w.digits(), 0);
      uint64_t v = 0;
      if (len < 16) v = w.span16(0, len);
      else
        for (uint64_t q = x; is_digit(at(q)); ++q) v = v * 10 + (at(q) - '0');
      if (r < a.cap[C_QID]) a.qid[r] = v;
      else raise_error(a.err, E_CAPACITY, x);
    }
  } else {
    // every v1 is decoded by the reference: a '-' field is the sign error
    // even when its triple is dropped (strtonum.h:416, libfm_parser.h:104)
    for (uint64_t m = soF; m; m &= m - 1) {
      const uint64_t q = P + ctz64(m);
      if (sh.c.text[q - t.tlo + kPre] == '-') raise_error(a.err, E_NEG_INDEX, q);
    }
  }
  // ---- per-chunk exclusive counts at each chunk start in my segment
  if (a.chunk_tab) {
    for (uint32_t i = 0; i < sh.c.ncs; ++i) {
      const uint64_t x = sh.c.csl[i];
      if (x < P || x >= P + kSegB || x >= t.thi) continue;
      const uint64_t below = (1ull << (x - P)) - 1;
      uint64_t *row = a.chunk_tab + (uint64_t)(sh.c.c_first + i) * 8;
      const uint64_t rows = eL + popc64(so.L & below);
      row[C_ROWS] = rows;
      row[C_INDEX] = eI + popc64(so.I & below);
      row[C_VALUE] = eV + popc64(so.V & below);
      row[C_WEIGHT] = eW + popc64(so.W & below);
      row[C_QID] = 0;
      row[C_LABEL] = rows;
      row[C_FIELD] = FM ? row[C_INDEX] : 0;
    }
  }
  constexpr uint32_t kIW = FM ? 2u : 1u;  // list entries per index
  {  // the register batch (pass 0)
    const uint32_t nI0 = fI(pe0), nV0 = fV(pe0), nL0 = fL(pe0), nF0 = nV0 + nL0 + fW(pe0), fb0 = kIW * nI0;
#pragma unroll
    for (int u = 0; u < kB; ++u) {
      const uint32_t j = (uint32_t)tid + (uint32_t)u * kFThreads;
      if (j < nI0 && !((slowI >> u) & 1u)) put_index(bIdx + j, ids_of(ib[u]), t.tlo + sh.u.lst[j]);
      if (j < nF0 && !((slowF >> u) & 1u)) put_float(j, fb[u], sh.u.lst[fb0 + j], 0, nV0, nL0);
    }
  }
#ifndef FSVM_PF_LATE
  // the next tile's text loads, in flight through the rest of this tile
  if (PERSIST && kn < a.ntiles) stage_issue(a.text, a.n, (uint64_t)kn * kTile, sr, bk);
#endif
  for (uint32_t p = 0; p < np; ++p) {
    const uint64_t s = p ? sh.pend[p - 1] : 0, e = p ? sh.pend[p] : pe0;
    if (p) {  // block-uniform
      bk.sync();
      if (mypass == p) build(s, e);
      bk.sync();
      slowI = slowF = 0;
    }
    const uint64_t cn = e - s;
    const uint32_t nIp = fI(cn), nVp = fV(cn), nLp = fL(cn), nFp = nVp + nLp + fW(cn), fbp = kIW * nIp;
    const uint32_t u0 = p ? 0u : (uint32_t)kB;
#ifdef FSVM_UNR2
#pragma unroll 2
#endif
    for (uint32_t u = u0, j = (uint32_t)tid + u0 * kFThreads; j < nIp; ++u, j += kFThreads) {
      const uint32_t o = sh.u.lst[j];
      bool ok;
      const uint32_t v = win_index(o, &ok);
      if (ok) put_index(bIdx + fI(s) + j, ids_of(v), t.tlo + o);
      slowI |= (ok ? 0u : 1u) << u;
    }
#ifdef FSVM_UNR2
#pragma unroll 2
#endif
    for (uint32_t u = u0, j = (uint32_t)tid + u0 * kFThreads; j < nFp; ++u, j += kFThreads) {
      const uint32_t o = sh.u.lst[fbp + j];
      bool ok;
      const float v = win_float(o, &ok);
      if (ok) put_float(j, v, o, s, nVp, nLp);
      slowF |= (ok ? 0u : 1u) << u;
    }
    // the byte decoders on the runs the windows left (rare)
    for (uint32_t m = slowI; m; m &= m - 1) {
      const uint32_t j = (uint32_t)tid + (uint32_t)ctz32(m) * kFThreads, o = sh.u.lst[j];
      put_index(bIdx + fI(s) + j, slow_idx(o), t.tlo + o);
    }
    for (uint32_t m = slowF; m; m &= m - 1) {
      const uint32_t j = (uint32_t)tid + (uint32_t)ctz32(m) * kFThreads, o = sh.u.lst[fbp + j];
      put_float(j, slow_flt(o), o, s, nVp, nLp);
    }
    if constexpr (FM)
      for (uint32_t j = (uint32_t)tid; j < nIp; j += kFThreads) put_field(bIdx + fI(s) + j, sh.u.lst[nIp + j]);
  }
  if (imin && one_chunk) {  // block-uniform: one store per wave that saw a 0 id
    const uint64_t zm = bk.ballot(zero);
    if ((tid & (kWave - 1)) == 0 && zm) store_flag_u64(&a.umin[sh.c.c_first - 1], 0);
  }
  FAST_STAMP(k, 8);
#ifdef FSVM_PF_AHEAD
  if (pfv == 0xFFu && a.n == 1) a.res[15] = pfv;  // keeps the touch load alive (never true)
#endif
#ifdef FSVM_PF_LATE
  if (PERSIST && kn < a.ntiles) stage_issue(a.text, a.n, (uint64_t)kn * kTile, sr, bk);
#endif
  return kn;
}

template <int MODE, bool FM = false, class BK>
DA_HDF void tile(const FastSvmArgs &a, Shared &sh, BK &bk, uint32_t k) {
  StageRegs sr;
  (void)tile_p<MODE, FM, false>(a, sh, bk, k, sr);
}

}  // namespace fsvm

#if defined(__HIPCC__)
namespace {  // one private copy per kernel translation unit (no RDC)
// indexing_mode < 0 after the single-pass write pass (fsvm::umin_fix); every
// block first checks whether any unit needs the shift -- a unit with ids and
// no 0 id among them -- so 0-based input costs one small read per block.
// The shifted range stops at the caller's capacities: res[C_INDEX] is the
// exact count even when the write pass ran out of room (E_CAPACITY), and the
// entries past cap_index (cap_field for libfm's field ids) were never stored.
__global__ void __launch_bounds__(256) umin_fix_kernel(void *index, void *field, int wide, const uint64_t *tab,
                                                       int nunit, const uint64_t *umin, const uint64_t *res,
                                                       const uint32_t *gate, uint64_t cap_index,
                                                       uint64_t cap_field) {
  if (*gate) return;  // the exact kernels made this result (and applied the rule themselves)
  __shared__ int need;
  if (threadIdx.x == 0) need = 0;
  __syncthreads();
  uint64_t total = res[C_INDEX];
  for (int u = threadIdx.x; u < nunit; u += 256) {
    const uint64_t uhi = u + 1 < nunit ? tab[(uint64_t)(u + 1) * 8 + C_INDEX] : total;
    if (umin[u] != 0 && uhi > tab[(uint64_t)u * 8 + C_INDEX]) need = 1;  // ids, none of them 0
  }
  __syncthreads();
  if (!need) return;
  if (total > cap_index) total = cap_index;
  if (field && total > cap_field) total = cap_field;
  // a block of 4096 ids inside one unit to shift (the common case: units are
  // InputSplit chunks or their ranges): 16-byte loads, all in flight before
  // the stores; a block across a unit start, 64-bit ids or an unaligned
  // array take the element loop
  const bool vec = !wide && !field && ((uintptr_t)index & 15u) == 0;
  __shared__ int blk_u;
  for (uint64_t b = (uint64_t)blockIdx.x * 4096; b < total; b += (uint64_t)gridDim.x * 4096) {
    const uint64_t e = b + 4096 < total ? b + 4096 : total;
    __syncthreads();
    if (threadIdx.x == 0) {
      const int u = fsvm::unit_of_entry(tab, nunit, b);
      const uint64_t uhi = u + 1 < nunit ? tab[(uint64_t)(u + 1) * 8 + C_INDEX] : total;
      blk_u = (vec && e == b + 4096 && uhi >= e) ? u : -1;
    }
    __syncthreads();
    const int u = blk_u;
    if (u < 0) {
      fsvm::umin_fix(index, field, wide, tab, nunit, umin, total, b, e, threadIdx.x, 256);
      continue;
    }
    if (umin[u] == 0) continue;  // a 0 among the unit's ids: kept
    uint4 *p = reinterpret_cast<uint4 *>(static_cast<uint32_t *>(index) + b);
    uint4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = p[threadIdx.x + 256 * k];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      v[k].x -= 1u;
      v[k].y -= 1u;
      v[k].z -= 1u;
      v[k].w -= 1u;
      p[threadIdx.x + 256 * k] = v[k];
    }
  }
}
inline hipError_t launch_umin_fix(void *index, void *field, int wide, const uint64_t *tab, int nunit,
                                  const uint64_t *umin, const uint64_t *res, const uint32_t *gate,
                                  uint64_t cap_index, uint64_t cap_field, hipStream_t s) {
  if (nunit < 1 || !tab) return hipSuccess;
  uint64_t blocks = (cap_index + 4095) / 4096;
  blocks = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks);
  umin_fix_kernel<<<(unsigned)blocks, 256, 0, s>>>(index, field, wide, tab, nunit, umin, res, gate, cap_index,
                                                   cap_field);
  return hipGetLastError();
}
}  // namespace
#endif
}  // namespace dmlc_amd
