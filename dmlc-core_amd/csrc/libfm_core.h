// libfm_core.h -- the libfm tile body (LibFMParser::ParseBlock,
// src/data/libfm_parser.h:67-144; ParsePair strtonum.h:667-703 for the head,
// ParseTriple strtonum.h:718-772 for the features), written once against the
// block policy BK {tid, sync, min_u64, exclusive} so the GPU kernel
// (libfm.hip) and the test-only CPU emulator (tests/emu) run the same code.
//
// Decomposition: as libsvm_core.h (count -> scan -> write over tiles that own
// the line starts in their byte range, 8 KiB LDS windows, the owner of a line
// start parses its head and marks R1, the first feature run).  The feature
// runs of a line then follow ParseTriple's grammar as a 4-state machine whose
// per-segment transition functions compose in a block scan; one walk per
// segment records the role masks for every start state (walk_roles):
//
//   state  meaning (the role of the last run)      next run, gap's first non-blank
//   PRE    head / nothing yet                        -> PRE (no role until R1)
//   A      field  (ParseTriple v1)                   ':' -> B (index)   else -> A (field)
//   B      index  (v2)                               ':' -> C (value)   else -> A (field)
//   C      value  (v3)                               -> A (field)
//
// A field is emitted only when its index follows (r >= 2, libfm_parser.h:
// 111-120): the pair is written when the index run is reached, the field run
// found by scanning back over the gap.  A line ending in "v1:" / "v1:v2:"
// makes ParseTriple decode v2 / v3 at the line end (reading past it, as the
// reference does).  Every v1 is decoded by the reference, so a '-' field
// raises the sign error even when the triple is dropped (strtonum.h:416).
#pragma once
#include "libsvm_core.h"

namespace dmlc_amd {
namespace fm {

using svm::Seg;
using svm::r1_bit;
using svm::fn_apply;
using svm::FnCompose;
using svm::kIdentityFn;
using svm::first_line_start;
using svm::gap_fnb;

enum : uint32_t { S_PRE = 0, S_A = 1, S_B = 2, S_C = 3 };
// transition tables (entry i at bits 2i): gap's first non-blank is ':' or not
constexpr uint32_t kTColon = S_PRE | (S_B << 2) | (S_C << 4) | (S_A << 6);
constexpr uint32_t kTOther = S_PRE | (S_A << 2) | (S_A << 4) | (S_A << 6);
constexpr uint32_t kAllA = 0x55u, kAllPre = 0x00u;

struct Head {
  uint64_t label, wpos, r1;
  bool row, w;
};

// Head of the line starting at `ls` (libfm_parser.h:79-98: ParsePair<real_t,
// real_t>, then ParseTriple's first skip to R1).  `lim`: chunk end.  No
// comment or qid handling in this grammar.
template <typename F>
DA_HDF Head head_parse(const F &at, uint64_t ls, uint64_t lim) {
  Head h;
  h.label = h.wpos = h.r1 = kNone;
  h.row = h.w = false;
  auto eol = [&](uint64_t p) { return p >= lim || (p > ls && is_nl(at(p))); };
  uint64_t p = ls;
  while (!eol(p) && !is_digitchar(at(p))) ++p;
  if (eol(p)) return h;
  h.row = true;
  h.label = p;
  while (!eol(p) && is_digitchar(at(p))) ++p;
  while (!eol(p) && is_blank(at(p))) ++p;
  if (!eol(p) && at(p) == ':') {
    ++p;
    while (!eol(p) && !is_digitchar(at(p))) ++p;
    h.w = true;
    h.wpos = p;  // == line end for "label:" -- decoded there, as the reference does
    while (!eol(p) && is_digitchar(at(p))) ++p;
  }
  while (!eol(p) && !is_digitchar(at(p))) ++p;
  if (!eol(p)) h.r1 = p;
  return h;
}

// start of the digitchar run that ends before the gap ending at x
template <typename F>
DA_HD uint64_t prev_run(const F &at, uint64_t x, uint64_t floor) {
  while (x > floor && !is_digitchar(at(x - 1))) --x;
  while (x > floor && is_digitchar(at(x - 1))) --x;
  return x;
}

// Role masks of one segment for each state at its start (libsvm_core.h
// Roles, with ParseTriple's four states): bit i of pr[s] / va[s] = the run
// at lo + i is the index of a (field, index) pair / a value when the segment
// starts in state s; dp[s] / dv[s] = a dangling "v1:" / "v1:v2:" at the line
// end at lo + i, whose index / value ParseTriple decodes at lo + i + 1; neg:
// per state (byte s) the first run read as v1 that starts with '-' (0xFF:
// none) -- the reference decodes every v1, so it raises the sign error even
// when the triple is dropped (strtonum.h:416).  The block scan of the
// transition functions picks one set; counts are popcounts.  Round 6: one
// walk per window instead of three (compose, count, emit).
struct Roles {
  uint32_t pr[4], va[4], dp[4], dv[4];
  uint32_t neg;
};
DA_HD uint32_t pick(const uint32_t m[4], uint32_t s) {  // m[s] without a dynamic register index
  return s == 0 ? m[0] : s == 1 ? m[1] : s == 2 ? m[2] : m[3];
}

// Event walk over one segment: the transition function (4 x 2-bit entries,
// entry s = the state after the events when the segment starts in s) and
// the role masks.  ParseTriple (strtonum.h:718-772) for libfm_parser.h:
// 100-139: after the head (R1) runs are v1 / v2 / v3 by the ':' between them.
DA_HDF void walk_roles(const LibfmArgs &a, Src &src, const uint32_t *r1bits, uint64_t w0, const Seg &sg,
                       uint32_t &fn, Roles &R) {
  for (int s = 0; s < 4; ++s) R.pr[s] = R.va[s] = R.dp[s] = R.dv[s] = 0;
  R.neg = ~0u;
  uint32_t ev = sg.rs | sg.ls | sg.le;
  int chunk = sg.chunk;
  uint64_t cfloor = a.cs[chunk], cend = a.cs[chunk + 1];
  src.lim = a.lim(chunk);  // decoders read to the InputSplit chunk end
  while (ev) {
    const int i = ctz32(ev);
    ev &= ev - 1;
    const uint32_t bit = 1u << i;
    const uint64_t x = sg.lo + i;
    while (x >= cend) {  // entered the next chunk
      ++chunk;
      cfloor = a.cs[chunk];
      cend = a.cs[chunk + 1];
      src.lim = a.lim(chunk);
    }
    if (sg.ls & bit) fn = kAllPre;
    if (sg.rs & bit) {
      uint32_t amask = 0;  // states in which the run is a v1
      if (r1_bit(r1bits, w0, x)) {
        fn = kAllA;
        amask = 0xFu;
      } else if (fn != kAllPre) {
        const bool colon = (sg.xg & bit) ? gap_fnb(src, x, cfloor) == ':' : (sg.rc & bit) != 0u;
        for (int s = 0; s < 4; ++s) {
          const uint32_t e = (fn >> (2 * s)) & 3u;
          if (e == S_A && colon) R.pr[s] |= bit;
          else if (e == S_B && colon) R.va[s] |= bit;
          else if (e != S_PRE) amask |= 1u << s;
        }
        fn = fn_apply(fn, colon ? kTColon : kTOther);
      }
      if (amask && src(x) == '-')
        for (int s = 0; s < 4; ++s)
          if (((amask >> s) & 1u) && ((R.neg >> (8 * s)) & 0xFFu) == 0xFFu)
            R.neg = (R.neg & ~(0xFFu << (8 * s))) | ((uint32_t)i << (8 * s));
    }
    if (sg.le & bit) {  // "v1:" / "v1:v2:" at the line end: ParseTriple decodes at lend
      uint32_t fA = 0, fB = 0;
      for (int s = 0; s < 4; ++s) {
        const uint32_t e = (fn >> (2 * s)) & 3u;
        fA |= (e == S_A ? 1u : 0u) << s;
        fB |= (e == S_B ? 1u : 0u) << s;
      }
      if ((fA | fB) && gap_fnb(src, x + 1, cfloor) == ':')
        for (int s = 0; s < 4; ++s) {
          if ((fA >> s) & 1u) R.dp[s] |= bit;
          if ((fB >> s) & 1u) R.dv[s] |= bit;
        }
    }
  }
}

DA_HD int chunk_at(const LibfmArgs &a, int chunk, uint64_t x) {
  while (x >= a.cs[chunk + 1]) ++chunk;
  return chunk;
}

// The (field, index) pairs of the segment in position order (P: pairs at run
// starts, D: dangling pairs at line ends, index at lo + i + 1): f(rank, field
// value, index value, event position, chunk); the sign error is raised here.
template <typename F>
DA_HDF void for_pairs(const LibfmArgs &a, Src &src, const Seg &sg, uint32_t P, uint32_t D,
                      const fast::DecTables *dt, F &&f) {
  int chunk = sg.chunk;
  uint64_t cfloor = a.cs[chunk];
  src.lim = a.lim(chunk);
  uint64_t r = 0;
  for (uint32_t m = P | D; m; m &= m - 1, ++r) {
    const uint32_t i = (uint32_t)ctz32(m);
    const uint64_t x = sg.lo + i;
    if (x >= a.cs[chunk + 1]) {
      chunk = chunk_at(a, chunk, x);
      cfloor = a.cs[chunk];
      src.lim = a.lim(chunk);
    }
    const uint64_t ip = x + ((D >> i) & 1u);
    uint64_t fv, iv;
    bool ok = index_at(src, prev_run(src, ip, cfloor), a.wide != 0, dt, &fv);  // (exact_dec.h)
    ok = index_at(src, ip, a.wide != 0, dt, &iv) && ok;
    if (!ok) {
      raise_error(a.err, E_NEG_INDEX, x);
      fv = iv = 0;
    }
    f(r, fv, iv, x, chunk);
  }
}

// Write pass: the segment's pairs, values and rows at base + their rank in
// the segment (masks of its start state; libsvm_core.h emit).
DA_HDF void emit(const LibfmArgs &a, Src &src, const Seg &sg, uint32_t P, uint32_t V, uint32_t DP, uint32_t DV,
                 uint32_t neg, const Base64 &base, const fast::DecTables *dt) {
  if (neg != 0xFFu) raise_error(a.err, E_NEG_INDEX, sg.lo + neg);
  // ---- (field, index) pairs
  for_pairs(a, src, sg, P, DP, dt, [&](uint64_t rk, uint64_t fv, uint64_t iv, uint64_t x, int chunk) {
    if (a.indexing_mode > 0 || (a.indexing_mode < 0 && a.chunk_min[chunk] > 0)) {
      --fv;
      --iv;
    }
    const uint64_t r = base.c[C_INDEX] + rk;
    if (r < a.cap[C_INDEX] && r < a.cap[C_FIELD]) {
      if (a.wide) {
        reinterpret_cast<uint64_t *>(a.index)[r] = iv;
        reinterpret_cast<uint64_t *>(a.field)[r] = fv;
      } else {
        reinterpret_cast<uint32_t *>(a.index)[r] = (uint32_t)iv;
        reinterpret_cast<uint32_t *>(a.field)[r] = (uint32_t)fv;
      }
    } else {
      raise_error(a.err, E_CAPACITY, x);
    }
  });
  // ---- values (a v3 run, or the value read at the line end after "v1:v2:")
  {
    int chunk = sg.chunk;
    src.lim = a.lim(chunk);
    uint64_t vr = base.c[C_VALUE];
    for (uint32_t m = V | DV; m; m &= m - 1, ++vr) {
      const uint32_t i = (uint32_t)ctz32(m);
      const uint64_t x = sg.lo + i;
      if (x >= a.cs[chunk + 1]) {
        chunk = chunk_at(a, chunk, x);
        src.lim = a.lim(chunk);
      }
      bool nan_err = false;
      const float v = value_at(src, x + ((DV >> i) & 1u), dt, &nan_err);
      if (nan_err) raise_error(a.err, E_NAN_LITERAL, x);
      if (vr < a.cap[C_VALUE]) a.value[vr] = v;
      else raise_error(a.err, E_CAPACITY, x);
    }
  }
  // ---- rows: label[:weight] heads, row offsets, unit table rows
  if (sg.ls) {
    Cnt cnt = cnt_zero();  // rows / labels / weights so far in the segment
    int chunk = sg.chunk;
    uint64_t cfloor = a.cs[chunk], cend = a.cs[chunk + 1];
    src.lim = a.lim(chunk);
    for (uint32_t m = sg.ls; m; m &= m - 1) {
      const uint32_t i = (uint32_t)ctz32(m);
      const uint64_t x = sg.lo + i;
      while (x >= cend) {
        ++chunk;
        cfloor = a.cs[chunk];
        cend = a.cs[chunk + 1];
        src.lim = a.lim(chunk);
      }
      const uint32_t below = (1u << i) - 1u;
      cnt.c[C_INDEX] = cnt.c[C_FIELD] = (uint32_t)popc32((P | DP) & below);
      cnt.c[C_VALUE] = (uint32_t)popc32((V | DV) & below);
      if (x == cfloor) {
        uint64_t *row = a.chunk_tab + (uint64_t)chunk * 8;  // rows of 8 slots (dmlc_amd.h)
        for (int k = 0; k < C_N; ++k) row[k] = base.c[k] + cnt.c[k];
      }
      const Head h = head_parse(src, x, cend);
      if (h.row) {
        const uint64_t r = base.c[C_ROWS] + cnt.c[C_ROWS];
        bool nan_err = false;
        uint64_t e;
        if (r < a.cap[C_ROWS]) {
          a.label[r] = parse_float(src, h.label, &e, &nan_err);
          a.offset[r] = base.c[C_INDEX] + cnt.c[C_INDEX];
        } else {
          raise_error(a.err, E_CAPACITY, x);
        }
        if (h.w) {
          const uint64_t wr = base.c[C_WEIGHT] + cnt.c[C_WEIGHT];
          if (wr < a.cap[C_WEIGHT]) a.weight[wr] = parse_float(src, h.wpos, &e, &nan_err);
          else raise_error(a.err, E_CAPACITY, x);
        }
        if (nan_err) raise_error(a.err, E_NAN_LITERAL, x);
        cnt.c[C_ROWS]++;
        cnt.c[C_LABEL]++;
        cnt.c[C_WEIGHT] += h.w;
      }
    }
  }
}

// The tile body.  MODE 1 = count pass, MODE 2 = write pass.
template <int MODE, class BK>
DA_HDF void tile(const LibfmArgs &a, svm::Shared &sh, BK &bk, uint64_t k) {
  if (a.gate && *a.gate == 0) return;  // the uniform-grammar kernel handled this input
  const uint64_t tlo = k * a.tile_bytes;
  if (tlo >= a.n) return;
  const uint64_t thi = mn(tlo + a.tile_bytes, a.n);
  const int tid = bk.tid();
  const Cnt zero = cnt_zero();
  Cnt tot = zero;   // totals of this tile's previous windows (block-uniform)
  Cnt mine = zero;  // count pass: this thread's totals over all windows
  Base64 tbase;
  for (int i = 0; i < C_N; ++i) tbase.c[i] = MODE == 2 ? a.tile_base[k * C_N + i] : 0;

  uint64_t w0 = first_line_start(a, bk, tlo, a.n);
  if (w0 == kNone || w0 >= thi) {
    if (MODE == 1 && tid < C_N) a.tile_cnt[k * C_N + tid] = 0;
    return;
  }
  if (tid == 0) sh.pending[1] = kNone;
  fast::init_dec_tables(sh.dt, bk);
#ifdef FSVM_EXACT_BYTEDEC  // A/B only: the byte decoders everywhere
  const fast::DecTables *dtp = nullptr;
#else
  const fast::DecTables *dtp = &sh.dt;
#endif
  bk.sync();
  int j = 0;             // window counter
  uint32_t st0 = S_PRE;  // concrete state at the window start
  bool done = false;
  MinAcc macc;  // count pass, indexing_mode < 0: this thread's unit minimum
  MinAcc *mp = MODE == 1 && a.indexing_mode < 0 ? &macc : nullptr;
  Src src;
  src.g = a.text;
  src.lds = sh.win;
  // the count pass's records of this tile's windows (args.h LibsvmArgs.rec,
  // libsvm_core.h): the write pass takes the role masks and head counts from
  // them instead of walking the window again.  A window in which some start
  // state leaves both a dangling pair and a dangling value in one segment
  // (their kinds would need a fifth word) gets none: its meta word says so
  // and the write pass walks it, from the state the meta words carry.
  const bool recs = a.rec != nullptr;
  uint32_t *rec_t = recs ? a.rec + (uint64_t)k * a.rec_win * 4 * kThreads : nullptr;
  uint64_t *meta_t = recs ? a.rec_meta + (uint64_t)k * a.rec_win * 2 : nullptr;
  constexpr uint64_t kWalkWin = 1u << 8;
  bool prev_rec = false;  // write pass: window j-1 came from its record
  while (!done) {
    const bool has_rec = recs && (uint32_t)j < a.rec_win;
    const bool from_rec = MODE == 2 && has_rec && !(meta_t[j * 2 + 1] & kWalkWin);
    if (MODE == 2 && prev_rec && !from_rec) {  // walking again after recorded windows
      st0 = (uint32_t)(meta_t[(j - 1) * 2 + 1] & 3u);
      if (tid == 0) sh.pending[(j + 1) & 1] = meta_t[(j - 1) * 2];
      bk.sync();
    }
    prev_rec = from_rec;
    if (MODE == 1 && tid == 0) sh.walk_win = 0;
    const uint64_t pend = sh.pending[(j + 1) & 1];  // written during window j-1
    uint64_t wend = mn(w0 + (uint64_t)kWin, a.n);
    if (wend == a.n) done = true;
    if (wend > thi) {
      const uint64_t e = first_line_start(a, bk, mx(w0, thi), wend);
      if (e != kNone) {
        wend = e;
        done = true;
      }
    }
    if (wend == w0) break;
    if (tid == 0) sh.pending[j & 1] = (pend != kNone && pend >= wend) ? pend : kNone;
    const uint64_t abase = w0 & ~15ull;
    const uint64_t nunits = (wend - abase + 15) >> 4;
    for (uint64_t u = tid; u < nunits; u += kThreads) {
      const uint64_t g = abase + (u << 4);
      if (g + 16 <= a.n) {
        for (int q = 0; q < 4; ++q)
          reinterpret_cast<uint32_t *>(&sh.win[u << 4])[q] = reinterpret_cast<const uint32_t *>(a.text + g)[q];
      } else {
        for (int q = 0; q < 16; ++q) sh.win[(u << 4) + q] = g + q < a.n ? a.text[g + q] : 0;
      }
    }
    for (int i = tid; i < kWin / 32 + 1; i += kThreads) sh.r1bits[i] = 0;
    bk.sync();
    src.wbase = abase;
    src.wend = mn(abase + (nunits << 4), a.n);
    if (tid == 0 && pend != kNone && pend < wend)
      atomic_or_u32(&sh.r1bits[(pend - w0) >> 5], 1u << ((pend - w0) & 31));

    // ---- this thread's segment masks (libsvm_core.h)
    Seg sg;
    sg.lo = w0 + (uint64_t)tid * kSeg;
    sg.hi = mn(sg.lo + (uint64_t)kSeg, wend);
    sg.rs = sg.ls = sg.le = sg.rc = sg.rh = sg.xg = 0;
    sg.chunk = 0;
    if (sg.lo < sg.hi) {
      sg.chunk = chunk_of(a.cs, a.nchunk, sg.lo);
      src.lim = a.lim(sg.chunk);
      uint32_t dm, nl, cm = 0, bm = 0, hm = 0, csm = 0;
      const int len = (int)(sg.hi - sg.lo);
      if (from_rec) seg_masks(sh.win, (uint32_t)(sg.lo - abase), len, &dm, &nl);
      else seg_masks5(sh.win, (uint32_t)(sg.lo - abase), len, &dm, &nl, &cm, &bm, &hm);
      for (int c = sg.chunk; c < a.nchunk && a.cs[c] < sg.hi; ++c)
        if (a.cs[c] >= sg.lo) csm |= 1u << (a.cs[c] - sg.lo);
      const uint32_t prev = (sg.lo > 0 && !(csm & 1u) && is_digitchar(src(sg.lo - 1))) ? 1u : 0u;
      sg.rs = (dm & ~((dm << 1) | prev)) | (csm & dm);
      sg.ls = nl | csm;
      if (!from_rec) {  // gap classes (libsvm_core.h): run starts whose gap's first non-blank is ':'
        const uint32_t lenm = len >= 32 ? ~0u : ((1u << len) - 1u);
        const uint32_t G = ~dm & lenm, Bg = bm & G;
        const uint32_t F = (Bg + (G & ~(G << 1))) & ~Bg & G;
        sg.rc = (G + (F & cm)) & ~G & dm;
        const uint32_t rs0 = sg.rs & (0u - sg.rs);  // the first run's gap may begin before the segment
        sg.xg = (dm & (rs0 - 1u)) == 0u ? rs0 : 0u;
      }
      bool nxt = sg.hi == a.n;
      if (!nxt) {
        const uint64_t h = sg.hi;
        nxt = is_nl(h < src.wend ? (uint32_t)sh.win[h - abase] : gbyte(a.text, h)) || is_chunk_start(a.cs, a.nchunk, h);
      }
      sg.le = (sg.ls >> 1) | ((uint32_t)nxt << (len - 1));
    }

    // ---- head sections -> R1 marks, and the segment's row / weight counts
    uint32_t hrow = 0, hw = 0;
    if (sg.ls && !from_rec) {
      uint32_t m = sg.ls;
      int chunk = sg.chunk;
      while (m) {
        const int i = ctz32(m);
        m &= m - 1;
        const uint64_t x = sg.lo + i;
        while (x >= a.cs[chunk + 1]) ++chunk;
        src.lim = a.lim(chunk);
        const Head h = head_parse(src, x, a.cs[chunk + 1]);
        if (h.r1 != kNone) {
          if (h.r1 < wend) atomic_or_u32(&sh.r1bits[(h.r1 - w0) >> 5], 1u << ((h.r1 - w0) & 31));
          else sh.pending[j & 1] = h.r1;  // only the window's last line can get here
        }
        if (h.row) {
          ++hrow;
          hw += h.w;
        }
      }
    }
    bk.sync();

    // ---- role masks and transition function of my segment, then block scan
    // (or the count pass's record of them)
    uint32_t P, V, DP, DV, neg, st_next = S_PRE;
    uint32_t *rw = has_rec ? rec_t + (uint64_t)j * 4 * kThreads : nullptr;
    if (from_rec) {
      P = rw[tid];
      V = rw[kThreads + tid];
      const uint32_t d = rw[2 * kThreads + tid], hc = rw[3 * kThreads + tid];
      DP = (hc >> 24) & 1u ? 0u : d;  // bit 24: the dangling ends are values
      DV = d ^ DP;
      hrow = hc & 0x3Fu;
      hw = (hc >> 6) & 0x3Fu;
      neg = (hc >> 12) & 0xFFu;
    } else {
      uint32_t fn = kIdentityFn;
      Roles R;
      if (sg.lo < sg.hi) walk_roles(a, src, sh.r1bits, w0, sg, fn, R);
      else
        for (int s2 = 0; s2 < 4; ++s2) R.pr[s2] = R.va[s2] = R.dp[s2] = R.dv[s2] = 0, R.neg = ~0u;
      if (MODE == 1 && rw) {
        bool mixed = false;
        for (int s2 = 0; s2 < 4; ++s2) mixed = mixed || (R.dp[s2] && R.dv[s2]);
        if (mixed) sh.walk_win = 1;  // (read by thread 0 after the scan's barriers)
      }
      uint32_t fn_total;
      const uint32_t fn_ex = bk.exclusive(fn, kIdentityFn, FnCompose(), &fn_total);
      const uint32_t st = (fn_ex >> (2 * st0)) & 3u;
      st_next = (fn_total >> (2 * st0)) & 3u;
      P = pick(R.pr, st);
      V = pick(R.va, st);
      DP = pick(R.dp, st);
      DV = pick(R.dv, st);
      neg = (R.neg >> (8 * st)) & 0xFFu;
      if (MODE == 1 && rw) {  // the record for the write pass
        rw[tid] = P;
        rw[kThreads + tid] = V;
        rw[2 * kThreads + tid] = DP | DV;
        rw[3 * kThreads + tid] = hrow | (hw << 6) | (neg << 12) | ((DV != 0u ? 1u : 0u) << 24);
        if (tid == 0) {
          meta_t[j * 2] = sh.pending[j & 1];  // (set by the heads, before the scan's barriers)
          meta_t[j * 2 + 1] = st_next | (sh.walk_win ? kWalkWin : 0u);
        }
      }
    }

    // ---- counts by popcount, then (write pass) scan + emit
    Cnt c = zero;
    c.c[C_ROWS] = c.c[C_LABEL] = hrow;
    c.c[C_WEIGHT] = hw;
    c.c[C_INDEX] = c.c[C_FIELD] = (uint32_t)popc32(P | DP);
    c.c[C_VALUE] = (uint32_t)popc32(V | DV);
    if (MODE == 1) {
      if (mp && (P | DP))
        for_pairs(a, src, sg, P, DP, dtp, [&](uint64_t, uint64_t fv, uint64_t iv, uint64_t, int chunk) {
          if (!a.wide) {
            fv = (uint32_t)fv;
            iv = (uint32_t)iv;
          }
          mp->add(a.chunk_min, chunk, fv < iv ? fv : iv);
        });
      mine = CntAdd()(mine, c);
    } else {
      Cnt wtot;
      const Cnt ex = bk.exclusive(c, zero, CntAdd(), &wtot);
      if (sg.lo < sg.hi) {
        Base64 b;
        for (int i = 0; i < C_N; ++i) b.c[i] = tbase.c[i] + tot.c[i] + ex.c[i];
        emit(a, src, sg, P, V, DP, DV, neg, b, dtp);
      }
      tot = CntAdd()(tot, wtot);
    }
    st0 = st_next;
    w0 = wend;
    ++j;
    bk.sync();
  }
  if (mp) tile_min_flush(macc, a.chunk_min, bk);
  if (MODE == 1) {
    Cnt total;
    (void)bk.exclusive(mine, zero, CntAdd(), &total);
    if (tid < C_N) a.tile_cnt[k * C_N + tid] = total.c[tid];
  }
}

}  // namespace fm
}  // namespace dmlc_amd
