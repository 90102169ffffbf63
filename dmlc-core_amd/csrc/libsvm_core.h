// libsvm_core.h -- the libsvm tile body (LibSVMParser::ParseBlock,
// src/data/libsvm_parser.h:85-172, ParsePair strtonum.h:667-703), written once
// against a block policy BK {tid, sync, min_u64, exclusive} so the GPU kernel
// (libsvm.hip, BK = DevBlock) and the test-only CPU emulator (tests/emu) run
// the same per-thread code.
//
// Decomposition (DESIGN.md "libsvm tile kernel"):
//   * The text holds one or more InputSplit chunks; each chunk is one
//     ParseBlock (the reference with nthread = 1).  Line starts are the chunk
//     starts and every '\n' / '\r' after them (libsvm_parser.h:94-97, 155).
//   * Tile k owns the line starts in [k*T, (k+1)*T); its extent runs to the
//     first line start >= (k+1)*T, so no parse state crosses workgroups.
//   * The extent streams through 8 KiB LDS windows, 32 bytes per thread.
//   * The owner of a line start parses the head (label[:weight] [qid:n],
//     :99-132) sequentially and marks R1, the first feature run.  Feature runs
//     follow a 4-state role machine {PRE, FIRST(index), SECOND(value),
//     DEAD(comment)}; per-segment transition functions are composed with a
//     block scan.
#pragma once
#include "args.h"
#include "decode.h"
#include "exact_dec.h"

namespace dmlc_amd {
namespace svm {

enum : uint32_t { S_PRE = 0, S_F = 1, S_S = 2, S_D = 3 };
constexpr uint32_t kIdentityFn = 0xE4u;  // 4 x 2-bit entries, entry i -> i

DA_HD uint32_t fn_apply(uint32_t f, uint32_t T) {  // result[i] = T[f[i]]
  uint32_t r = 0;
  for (int i = 0; i < 4; ++i) r |= ((T >> (2 * ((f >> (2 * i)) & 3u))) & 3u) << (2 * i);
  return r;
}
struct FnCompose {  // "a then b"
  DA_HD uint32_t operator()(uint32_t a, uint32_t b) const { return fn_apply(a, b); }
};

struct Head {
  uint64_t label, wpos, qpos, r1;
  bool row, w, q;
};

// Head section of the line starting at `ls` (libsvm_parser.h:99-132, plus the
// first feature's IgnoreCommentAndBlank + ParsePair skip, :134-140).  `l0`:
// ls is a chunk start (comment recognition); `lim`: chunk end.  The line ends
// at the first '\n'/'\r' after ls, or lim.
template <typename F>
DA_HDF Head head_parse(const F &at, uint64_t ls, bool l0, uint64_t lim) {
  Head h;
  h.label = h.wpos = h.qpos = h.r1 = kNone;
  h.row = h.w = h.q = false;
  auto eol = [&](uint64_t p) { return p >= lim || (p > ls && is_nl(at(p))); };
  uint64_t p = ls;
  if (l0) {  // IgnoreCommentAndBlank, libsvm_parser.h:67-83, 103
    while (!eol(p)) {
      const uint32_t c = at(p);
      if (c == '#') return h;
      if (!is_blank(c)) break;
      ++p;
    }
  }
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
  while (p < lim && at(p) == ' ') ++p;  // :122-124 (bounded by the block end)
  if (!eol(p) && at(p) == 'q' && at(p + 1) == 'i' && at(p + 2) == 'd' && at(p + 3) == ':') {
    h.q = true;
    h.qpos = p + 4;
    p += 4;
    while (!eol(p) && is_digitchar(at(p))) ++p;
  }
  while (!eol(p)) {  // IgnoreCommentAndBlank before the first feature
    const uint32_t c = at(p);
    if (c == '#') return h;
    if (!is_blank(c)) break;
    ++p;
  }
  while (!eol(p) && !is_digitchar(at(p))) ++p;
  if (!eol(p)) h.r1 = p;
  return h;
}

// First non-blank byte of the gap that ends at x (exclusive) and starts after
// the previous digitchar; 0 when the gap is all blanks.  Stops at a line start.
template <typename F>
DA_HD uint32_t gap_fnb(const F &at, uint64_t x, uint64_t floor) {
  uint32_t fnb = 0;
  while (x > floor) {
    const uint32_t c = at(--x);
    if (is_digitchar(c)) break;
    if (!is_blank(c)) fnb = c;
    if (is_nl(c)) break;
  }
  return fnb;
}

struct Shared {  // LDS of one workgroup
  uint8_t win[kWin + 32];
  uint32_t r1bits[kWin / 32 + 1];
  uint64_t pending[2];  // R1 of a line whose head crossed a window, by window parity
  fast::DecTables dt;   // the window decoders' tables (fast_common.h)
  uint32_t walk_win;    // libfm count pass: this window gets no record (libfm_core.h)
};


struct Seg {
  uint64_t lo, hi;      // [lo, hi) absolute
  uint32_t rs, ls, le;  // run-start / line-start / line-end masks (bit i <-> lo + i)
  // run starts whose gap's first non-blank byte (gap_fnb) is ':' / '#', from
  // the segment's masks; xg: the first run start when no digitchar precedes
  // it in the segment -- its gap may begin before it (gap_fnb reads that one)
  uint32_t rc, rh, xg;
  int chunk;            // chunk of position lo
};

DA_HD bool r1_bit(const uint32_t *bits, uint64_t w0, uint64_t x) {
  const uint64_t o = x - w0;
  return (bits[o >> 5] >> (o & 31)) & 1u;
}

// Role masks of one segment for each role-machine state at its start: bit i
// of idx[s] / val[s] = the run starting at lo + i is an index / a value when
// the segment starts in state s; dng[s] = a dangling "idx:" at the line end
// at lo + i, whose value ParsePair decodes at lo + i + 1.  The block scan of
// the transition functions then picks one set, and the counts are popcounts.
struct Roles {
  uint32_t idx[4], val[4], dng[4];
};
DA_HD uint32_t pick(const uint32_t m[4], uint32_t s) {  // m[s] without a dynamic register index
  return s == 0 ? m[0] : s == 1 ? m[1] : s == 2 ? m[2] : m[3];
}

// Event walk over one segment: compose the role machine's transition
// function into fn (4 x 2-bit entries, entry s = the state after the events
// when the segment starts in s) and record the role masks.  ParsePair
// (strtonum.h:667-703) for libsvm_parser.h:134-161: a run is an index after
// the line head (R1) or a previous pair, a value when ':' is the first
// non-blank of the gap after an index; '#' as that first non-blank drops the
// rest of the line (IgnoreCommentAndBlank, :67-83).
DA_HDF void walk_roles(const LibsvmArgs &a, Src &src, const uint32_t *r1bits, uint64_t w0, const Seg &sg,
                       uint32_t &fn, Roles &R) {
  for (int s = 0; s < 4; ++s) R.idx[s] = R.val[s] = R.dng[s] = 0;
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
    if (sg.ls & bit) fn = 0u;  // every entry -> PRE
    if (sg.rs & bit) {
      if (r1_bit(r1bits, w0, x)) {
        fn = 0x55u;  // every entry -> FIRST, the run an index
        for (int s = 0; s < 4; ++s) R.idx[s] |= bit;
      } else if ((fn ^ (fn >> 1)) & 0x55u) {  // some entry is F or S
        const uint32_t g = (sg.xg & bit) ? gap_fnb(src, x, cfloor)
                           : (sg.rc & bit) ? (uint32_t)':' : (sg.rh & bit) ? (uint32_t)'#' : 0u;
        const uint32_t tF = g == '#' ? S_D : (g == ':' ? S_S : S_F);
        const uint32_t tS = g == '#' ? S_D : S_F;
        for (int s = 0; s < 4; ++s) {
          const uint32_t e = (fn >> (2 * s)) & 3u;
          if (e == S_F && tF == S_S) R.val[s] |= bit;
          else if ((e == S_F || e == S_S) && g != '#') R.idx[s] |= bit;
        }
        fn = fn_apply(fn, S_PRE | (tF << 2) | (tS << 4) | (S_D << 6));
      }
    }
    if (sg.le & bit) {  // "idx:" dangling at the line end: ParsePair decodes the value at lend
      uint32_t fF = 0;
      for (int s = 0; s < 4; ++s) fF |= (((fn >> (2 * s)) & 3u) == S_F ? 1u : 0u) << s;
      if (fF && gap_fnb(src, x + 1, cfloor) == ':')
        for (int s = 0; s < 4; ++s)
          if ((fF >> s) & 1u) R.dng[s] |= bit;
    }
  }
}

// Count pass, indexing_mode < 0: the unit minimum of the segment's indices
DA_HDF void index_min(const LibsvmArgs &a, Src &src, const Seg &sg, uint32_t I, MinAcc *macc,
                      const fast::DecTables *dt) {
  int chunk = sg.chunk;
  uint64_t cend = a.cs[chunk + 1];
  src.lim = a.lim(chunk);
  while (I) {
    const int i = ctz32(I);
    I &= I - 1;
    const uint64_t x = sg.lo + i;
    while (x >= cend) {
      ++chunk;
      cend = a.cs[chunk + 1];
      src.lim = a.lim(chunk);
    }
    uint64_t v;
    if (!index_at(src, x, a.wide != 0, dt, &v)) {
      raise_error(a.err, E_NEG_INDEX, x);
      v = 0;
    }
    macc->add(a.chunk_min, chunk, a.wide ? v : (uint64_t)(uint32_t)v);
  }
}

// Write pass: emit the segment's rows and entries at base + their rank in the
// segment (I / V / Dg: the role masks of its start state).  One loop per
// kind -- indices, values, rows -- so the lanes of a wave decode the same
// kind together; a rank is a popcount of the mask below the position.
DA_HD int chunk_at(const LibsvmArgs &a, int chunk, uint64_t x) {
  while (x >= a.cs[chunk + 1]) ++chunk;
  return chunk;
}
DA_HDF void emit(const LibsvmArgs &a, Src &src, const Seg &sg, uint32_t I, uint32_t V, uint32_t Dg,
                 const Base64 &base, const fast::DecTables *dt) {
  // ---- indices
  {
    int chunk = sg.chunk;
    src.lim = a.lim(chunk);
    uint64_t ir = base.c[C_INDEX];
    for (uint32_t m = I; m; m &= m - 1, ++ir) {
      const uint64_t x = sg.lo + ctz32(m);
      if (x >= a.cs[chunk + 1]) {
        chunk = chunk_at(a, chunk, x);
        src.lim = a.lim(chunk);
      }
      uint64_t v;
      if (!index_at(src, x, a.wide != 0, dt, &v)) {
        raise_error(a.err, E_NEG_INDEX, x);
        v = 0;
      }
      if (a.indexing_mode > 0 || (a.indexing_mode < 0 && a.chunk_min[chunk] > 0)) --v;
      if (ir < a.cap[C_INDEX]) {
        if (a.wide) reinterpret_cast<uint64_t *>(a.index)[ir] = v;
        else reinterpret_cast<uint32_t *>(a.index)[ir] = (uint32_t)v;
      } else {
        raise_error(a.err, E_CAPACITY, x);
      }
    }
  }
  // ---- values (a run after "idx:", or ParsePair's value read at the line
  // end after a dangling "idx:"; never both at one position)
  {
    int chunk = sg.chunk;
    src.lim = a.lim(chunk);
    uint64_t vr = base.c[C_VALUE];
    for (uint32_t m = V | Dg; m; m &= m - 1, ++vr) {
      const uint32_t i = (uint32_t)ctz32(m);
      const uint64_t x = sg.lo + i;
      if (x >= a.cs[chunk + 1]) {
        chunk = chunk_at(a, chunk, x);
        src.lim = a.lim(chunk);
      }
      bool nan_err = false;
      float v;
      if ((V >> i) & 1u) {
#ifdef FSVM_ABL_EXNODEC  // timing ablation only (tools/build_variants.sh), never shipped
        v = (float)(x & 7u);
#else
        v = value_at(src, x, dt, &nan_err);
#endif
      } else {
        uint64_t e;
        v = parse_float(src, x + 1, &e, &nan_err);
      }
      if (nan_err) raise_error(a.err, E_NAN_LITERAL, x);
      if (vr < a.cap[C_VALUE]) a.value[vr] = v;
      else raise_error(a.err, E_CAPACITY, x);
    }
  }
  // ---- rows: label[:weight] [qid:n] heads, row offsets, unit table rows
  if (sg.ls) {
    Cnt cnt = cnt_zero();  // rows / labels / weights / qids so far in the segment
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
      cnt.c[C_INDEX] = (uint32_t)popc32(I & below);
      cnt.c[C_VALUE] = (uint32_t)popc32((V | Dg) & below);
      const bool l0 = x == cfloor;
      if (l0) {
        uint64_t *row = a.chunk_tab + (uint64_t)chunk * 8;  // rows of 8 slots (dmlc_amd.h)
        for (int k = 0; k < C_N; ++k) row[k] = base.c[k] + cnt.c[k];
      }
      const Head h = head_parse(src, x, l0, cend);
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
        if (h.q) {
          const uint64_t qr = base.c[C_QID] + cnt.c[C_QID];
          if (qr < a.cap[C_QID]) a.qid[qr] = (uint64_t)c_strtoll(src, h.qpos, 10, &e);
          else raise_error(a.err, E_CAPACITY, x);
        }
        if (nan_err) raise_error(a.err, E_NAN_LITERAL, x);
        cnt.c[C_ROWS]++;
        cnt.c[C_LABEL]++;
        cnt.c[C_WEIGHT] += h.w;
        cnt.c[C_QID] += h.q;
      }
    }
  }
}

// Block-wide: first line start in [from, to), kNone if none.
template <class BK>
DA_HDF uint64_t first_line_start(const LibsvmArgs &a, BK &bk, uint64_t from, uint64_t to) {
  for (uint64_t base = from; base < to; base += kWin) {
    uint64_t best = kNone;
    const uint64_t lo = base + (uint64_t)bk.tid() * kSeg;
    const uint64_t hi = mn(lo + (uint64_t)kSeg, to);
    for (uint64_t p = lo; p < hi; ++p) {
      if (is_nl(a.text[p])) {
        best = p;
        break;
      }
    }
    if (lo < hi) {
      const int c = chunk_of(a.cs, a.nchunk, lo);
      const uint64_t s = a.cs[c] == lo ? lo : a.cs[c + 1];
      if (s < hi && s < best) best = s;
    }
    best = bk.min_u64(best);
    if (best != kNone) return best;
  }
  return kNone;
}

// The tile body.  MODE 1 = count pass, MODE 2 = write pass.
template <int MODE, class BK>
DA_HDF void tile(const LibsvmArgs &a, Shared &sh, BK &bk, uint64_t k) {
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
  uint32_t st0 = S_PRE;  // concrete role state at the window start
  bool done = false;
  MinAcc macc;  // count pass, indexing_mode < 0: this thread's unit minimum
  MinAcc *mp = MODE == 1 && a.indexing_mode < 0 ? &macc : nullptr;
  Src src;
  src.g = a.text;
  src.lds = sh.win;
  // the count pass's records of this tile's windows (args.h LibsvmArgs.rec):
  // the write pass takes the role masks and head counts from them instead of
  // walking the window again
  const bool recs = a.rec != nullptr;
  uint32_t *rec_t = recs ? a.rec + (uint64_t)k * a.rec_win * 4 * kThreads : nullptr;
  uint64_t *meta_t = recs ? a.rec_meta + (uint64_t)k * a.rec_win * 2 : nullptr;
  while (!done) {
    const bool from_rec = MODE == 2 && recs && (uint32_t)j < a.rec_win;
    if (MODE == 2 && recs && (uint32_t)j == a.rec_win) {  // the first window past the records
      st0 = (uint32_t)meta_t[(j - 1) * 2 + 1];
      if (tid == 0) sh.pending[(j + 1) & 1] = meta_t[(j - 1) * 2];
      bk.sync();
    }
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
    // a pending R1 beyond this window means its line spans the whole window
    if (tid == 0) sh.pending[j & 1] = (pend != kNone && pend >= wend) ? pend : kNone;
    // stage [abase, wend) into LDS (16-byte aligned base)
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

    // ---- this thread's segment masks
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
      // (a window with a count-pass record walks no roles: its run starts'
      // gap classes are not needed)
      if (from_rec) seg_masks(sh.win, (uint32_t)(sg.lo - abase), len, &dm, &nl);
      else seg_masks5(sh.win, (uint32_t)(sg.lo - abase), len, &dm, &nl, &cm, &bm, &hm);
      for (int c = sg.chunk; c < a.nchunk && a.cs[c] < sg.hi; ++c)
        if (a.cs[c] >= sg.lo) csm |= 1u << (a.cs[c] - sg.lo);
      const uint32_t prev = (sg.lo > 0 && !(csm & 1u) && is_digitchar(src(sg.lo - 1))) ? 1u : 0u;
      sg.rs = (dm & ~((dm << 1) | prev)) | (csm & dm);
      sg.ls = nl | csm;
      if (!from_rec) {  // gap classes: the carry from each gap start runs through its blanks to
         // its first non-blank; a ':' / '#' there is carried on through the gap
         // to the run start that ends it
        const uint32_t lenm = len >= 32 ? ~0u : ((1u << len) - 1u);
        const uint32_t G = ~dm & lenm, Bg = bm & G;
        const uint32_t F = (Bg + (G & ~(G << 1))) & ~Bg & G;
        sg.rc = (G + (F & cm)) & ~G & dm;
        sg.rh = (G + (F & hm)) & ~G & dm;
        const uint32_t rs0 = sg.rs & (0u - sg.rs);  // the first run's gap may begin before the segment
        sg.xg = (dm & (rs0 - 1u)) == 0u ? rs0 : 0u;
      }
      bool nxt = sg.hi == a.n;  // is position hi a line start (or the end of data)?
      if (!nxt) {
        const uint64_t h = sg.hi;
        nxt = is_nl(h < src.wend ? sh.win[h - abase] : a.text[h]) || is_chunk_start(a.cs, a.nchunk, h);
      }
      sg.le = (sg.ls >> 1) | ((uint32_t)nxt << (len - 1));
    }

    // ---- head sections -> R1 marks, and the segment's row / weight / qid
    // counts (libsvm_parser.h:99-132)
    uint32_t hrow = 0, hw = 0, hq = 0;
#ifdef FSVM_ABL_EX_NOHEADS  // timing ablation only
    if (false) {
#else
    if (sg.ls && !from_rec) {
#endif
      uint32_t m = sg.ls;
      int chunk = sg.chunk;
      while (m) {
        const int i = ctz32(m);
        m &= m - 1;
        const uint64_t x = sg.lo + i;
        while (x >= a.cs[chunk + 1]) ++chunk;
        src.lim = a.lim(chunk);
        const Head h = head_parse(src, x, x == a.cs[chunk], a.cs[chunk + 1]);
        if (h.r1 != kNone) {
          if (h.r1 < wend) atomic_or_u32(&sh.r1bits[(h.r1 - w0) >> 5], 1u << ((h.r1 - w0) & 31));
          else sh.pending[j & 1] = h.r1;  // only the window's last line can get here
        }
        if (h.row) {
          ++hrow;
          hw += h.w;
          hq += h.q;
        }
      }
    }
    bk.sync();

    // ---- role masks and transition function of my segment, then block scan
    // (or the count pass's record of them)
    uint32_t I, V, Dg, st_next = S_PRE;
    uint32_t *rw = recs && (uint32_t)j < a.rec_win ? rec_t + (uint64_t)j * 4 * kThreads : nullptr;
    if (from_rec) {
      I = rw[tid];
      V = rw[kThreads + tid];
      Dg = rw[2 * kThreads + tid];
      const uint32_t hc = rw[3 * kThreads + tid];
      hrow = hc & 0xFFu;
      hw = (hc >> 8) & 0xFFu;
      hq = hc >> 16;
    } else {
      uint32_t fn = kIdentityFn;
      Roles R;
#ifdef FSVM_ABL_EX_NOWALK  // timing ablation only
      if (false) walk_roles(a, src, sh.r1bits, w0, sg, fn, R);
#else
      if (sg.lo < sg.hi) walk_roles(a, src, sh.r1bits, w0, sg, fn, R);
#endif
      else
        for (int s2 = 0; s2 < 4; ++s2) R.idx[s2] = R.val[s2] = R.dng[s2] = 0;
      uint32_t fn_total;
      const uint32_t fn_ex = bk.exclusive(fn, kIdentityFn, FnCompose(), &fn_total);
      const uint32_t st = (fn_ex >> (2 * st0)) & 3u;
      st_next = (fn_total >> (2 * st0)) & 3u;
      I = pick(R.idx, st);
      V = pick(R.val, st);
      Dg = pick(R.dng, st);
      if (MODE == 1 && rw) {  // the record for the write pass
        rw[tid] = I;
        rw[kThreads + tid] = V;
        rw[2 * kThreads + tid] = Dg;
        rw[3 * kThreads + tid] = hrow | (hw << 8) | (hq << 16);
        if (tid == 0) {
          meta_t[j * 2] = sh.pending[j & 1];  // (set by the heads, before the scan's barriers)
          meta_t[j * 2 + 1] = st_next;
        }
      }
    }

    // ---- counts by popcount, then (write pass) scan + emit
    Cnt c = zero;
    c.c[C_ROWS] = c.c[C_LABEL] = hrow;
    c.c[C_WEIGHT] = hw;
    c.c[C_QID] = hq;
    c.c[C_INDEX] = (uint32_t)popc32(I);
    c.c[C_VALUE] = (uint32_t)popc32(V) + (uint32_t)popc32(Dg);
    if (MODE == 1) {
      if (mp && I) index_min(a, src, sg, I, mp, dtp);
      mine = CntAdd()(mine, c);
    } else {
      Cnt wtot;
      const Cnt ex = bk.exclusive(c, zero, CntAdd(), &wtot);
      if (sg.lo < sg.hi) {
        Base64 b;
        for (int i = 0; i < C_N; ++i) b.c[i] = tbase.c[i] + tot.c[i] + ex.c[i];
#ifndef FSVM_ABL_EX_NOEMIT  // timing ablation only (tools/build_variants.sh), never shipped
        emit(a, src, sg, I, V, Dg, b, dtp);
#endif
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

}  // namespace svm
}  // namespace dmlc_amd
