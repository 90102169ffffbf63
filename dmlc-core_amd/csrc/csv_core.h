// csv_core.h -- the CSV tile body (CSVParser<I,D>::ParseBlock,
// src/data/csv_parser.h:71-149), written once against a block policy BK so the
// GPU kernel (csv.hip) and the test-only CPU emulator (tests/emu) share it.
//
// Tile k owns the CSV line starts in [k*T, (k+1)*T): a line start is a
// non-'\n'/'\r' byte that follows one, or a chunk's first such byte; a line
// that begins with a UTF-8 BOM followed by a single line break absorbs the next
// line (text_parser.h:83-102, csv_parser.h:83-87).
// Fast lines (no BOM, a delimiter no decoder can consume): each field is
// decoded by the thread owning its first byte; its column is the number of
// delimiters since the line start, carried by a segmented block scan.  Slow
// lines (BOM, or a whitespace / alphanumeric / sign delimiter, where
// ParseFloat's whitespace skip changes the field structure) are parsed by the
// owner of the line start with an exact sequential restatement of the per-line
// loop (csv_parser.h:81-145).
#pragma once
#include "args.h"
#include "decode.h"
#include "exact_dec.h"

namespace dmlc_amd {
namespace csv {

// segmented column state: bit31 = reset (segment holds a line start),
// bit30 = slow line, bits 0..29 = delimiters since the (last) line start
struct ColCombine {
  DA_HD uint32_t operator()(uint32_t l, uint32_t r) const {
    if (r & 0x80000000u) return r;
    return (l & 0xC0000000u) | (((l & 0x3FFFFFFFu) + (r & 0x3FFFFFFFu)) & 0x3FFFFFFFu);
  }
};

DA_HD bool is_bom_at(const Src &at, uint64_t p) {
  return at(p) == 0xEFu && at(p + 1) == 0xBBu && at(p + 2) == 0xBFu;
}

// Exact CSV line-start predicate (see file comment).
DA_HDF bool csv_line_start(const Src &at, uint64_t x, uint64_t cfloor) {
  if (is_nl(at(x))) return false;
  if (x != cfloor && !is_nl(at(x - 1))) return false;
  // BOM units "EF BB BF <nl>" chained right before x: odd chain => x absorbed
  int k = 0;
  uint64_t y = x;
  while (y >= cfloor + 4 && is_nl(at(y - 1)) && at(y - 4) == 0xEFu && at(y - 3) == 0xBBu &&
         at(y - 2) == 0xBFu && (y - 4 == cfloor || is_nl(at(y - 5)))) {
    ++k;
    y -= 4;
  }
  return (k & 1) == 0;
}

template <typename T>
DA_HD void store_val(void *arr, int vtype, uint64_t i, float f, int64_t v) {
  if (vtype == 0) reinterpret_cast<float *>(arr)[i] = f;
  else if (vtype == 1) reinterpret_cast<int32_t *>(arr)[i] = (int32_t)v;
  else reinterpret_cast<int64_t *>(arr)[i] = v;
}

struct Field {
  float f;
  int64_t i;
  uint64_t end;
  bool nan_err;
};

DA_HD Field decode_field(const Src &at, int vtype, uint64_t p, const fast::DecTables *dt = nullptr) {
  Field r;
  r.nan_err = false;
  r.f = 0.f;
  r.i = 0;
  if (vtype == 0 && csv_value_at(at, p, dt, &r.f, &r.end)) return r;  // in registers (exact_dec.h)
  if (vtype == 0) {
    r.f = parse_float(at, p, &r.end, &r.nan_err);
  } else {
    r.i = c_strtoll(at, p, 0, &r.end);
    if (vtype == 1) r.i = (int64_t)(int32_t)r.i;
  }
  return r;
}

// Whether decode_field at p consumes a byte (endptr != p: the field holds a
// value, csv_parser.h:115-118) without decoding it -- the count pass needs
// no more for a value column.  ParseFloat (strtonum.h:95-264) consumes
// leading isspace bytes, a sign, "inf" / "infinity" / "nan" (any case; 3 or 8
// letters of infinity), digits, '.', an exponent 'e' / 'E' or the 'f' suffix;
// strtoll (base 0) consumes only when a decimal digit follows the optional
// blanks and sign (a "0x" prefix starts with one).
DA_HD bool field_consumed(const Src &at, int vtype, uint64_t p) {
  uint32_t c = at(p);
  if (vtype != 0) {
    while (is_cspace(c)) c = at(++p);
    if (c == '-' || c == '+') c = at(++p);
    return is_digit(c);
  }
  if (is_space(c) || c == '-' || c == '+' || is_digit(c) || c == '.' || (c | 32u) == 'e' || (c | 32u) == 'f')
    return true;
  if ((c | 32u) == 'n')
    return ((at(p + 1) | 32u) & 0xFFu) == 'a' && ((at(p + 2) | 32u) & 0xFFu) == 'n';
  if ((c | 32u) != 'i') return false;
  const char kInf[8] = {'i', 'n', 'f', 'i', 'n', 'i', 't', 'y'};
  int i = 1;
  while (i < 8 && ((at(p + i) | 32u) & 0xFFu) == (uint32_t)kInf[i]) ++i;
  return i == 3 || i == 8;
}

// csv_parser.h:81-145 for ONE line starting at `lbegin` (a CSV line start).
template <int MODE>
DA_HDF void csv_line_seq(const Src &at, const CsvArgs &a, uint64_t lbegin, uint64_t end, Cnt &cnt,
                             const Base64 &base) {
  {  // IgnoreUTF8BOM
    int count = 0;
    const uint32_t bom[3] = {0xEFu, 0xBBu, 0xBFu};
    while (lbegin != end && count < 3 && at(lbegin) == bom[count]) {
      ++count;
      ++lbegin;
    }
    if (count < 3) lbegin -= count;
  }
  if (lbegin == end) return;  // reference reads past `end` here (UB); the oracle stops too
  uint64_t lend = lbegin + 1;
  while (lend != end && !is_nl(at(lend))) ++lend;
  const uint64_t row = base.c[C_ROWS] + cnt.c[C_ROWS];
  if (MODE == 2) {
    if (row < a.cap[C_ROWS]) a.offset[row] = base.c[C_INDEX] + cnt.c[C_INDEX];
    else raise_error(a.err, E_CAPACITY, lbegin);
  }
  uint64_t p = lbegin;
  int col = 0;
  uint64_t idx = 0;
  float weight = u2f(0x7FC00000u);
  while (p != lend) {
    Field f = decode_field(at, a.vtype, p);
    if (MODE == 2 && f.nan_err) raise_error(a.err, E_NAN_LITERAL, p);
    if (col == a.label_column) {
      if (MODE == 2) {
        const uint64_t r = base.c[C_LABEL] + cnt.c[C_LABEL];
        if (r < a.cap[C_LABEL]) store_val<int>(a.label, a.vtype, r, f.f, f.i);
        else raise_error(a.err, E_CAPACITY, p);
      }
      cnt.c[C_LABEL]++;
    } else if (a.vtype == 0 && col == a.weight_column) {
      weight = f.f;
    } else {
      if (f.end != p) {
        if (MODE == 2) {
          const uint64_t r = base.c[C_INDEX] + cnt.c[C_INDEX];
          const uint64_t rv = base.c[C_VALUE] + cnt.c[C_VALUE];
          if (r < a.cap[C_INDEX] && rv < a.cap[C_VALUE]) {
            store_val<int>(a.value, a.vtype, rv, f.f, f.i);
            if (a.wide) reinterpret_cast<uint64_t *>(a.index)[r] = idx;
            else reinterpret_cast<uint32_t *>(a.index)[r] = (uint32_t)idx;
          } else {
            raise_error(a.err, E_CAPACITY, p);
          }
        }
        cnt.c[C_INDEX]++;
        cnt.c[C_VALUE]++;
      }
      idx++;
    }
    p = f.end >= lend ? lend : f.end;
    ++col;
    while (at(p) != a.delim && p != lend) ++p;
    if (p == lend && idx == 0) {
      raise_error(a.err, E_CSV_DELIM, p);
      return;
    }
    if (p != lend) ++p;
  }
  if (!(weight != weight)) {
    if (MODE == 2) {
      const uint64_t r = base.c[C_WEIGHT] + cnt.c[C_WEIGHT];
      if (r < a.cap[C_WEIGHT]) a.weight[r] = weight;
      else raise_error(a.err, E_CAPACITY, lbegin);
    }
    cnt.c[C_WEIGHT]++;
  }
  cnt.c[C_ROWS]++;
}

struct Seg {
  uint64_t lo, hi;
  uint32_t ls, dl, fs;  // line-start, delimiter, field-start masks
  uint32_t slow;        // slow flag per line start bit
  int chunk;
};

// value-column rank of column c (csv_parser.h:111-121: idx counts every column
// that is neither the label nor (float only) the weight column)
DA_HD uint64_t value_rank(const CsvArgs &a, uint64_t c) {
  uint64_t r = c;
  if (a.label_column >= 0 && (uint64_t)a.label_column < c) --r;
  if (a.vtype == 0 && a.weight_column >= 0 && (uint64_t)a.weight_column < c) --r;
  return r;
}
DA_HD bool is_value_col(const CsvArgs &a, uint64_t c) {
  return (int64_t)c != a.label_column && !(a.vtype == 0 && (int64_t)c == a.weight_column);
}

template <int MODE>  // 1 count, 2 emit
DA_HDF void walk(const CsvArgs &a, Src &src, const Seg &sg, uint32_t state, Cnt &cnt,
                     const Base64 &base, const fast::DecTables *dt) {
  // events: line and field starts; a field's column is the delimiters since
  // its line start, a popcount (col0 at bit `from`)
  uint32_t ev = sg.ls | sg.fs;
  int chunk = sg.chunk;
  uint64_t cend = a.cs[chunk + 1];
  src.lim = a.lim(chunk);  // decoders read to the InputSplit chunk end
  uint64_t col0 = state & 0x3FFFFFFFu;
  uint32_t from_mask = 0;  // bits below the current line's start
  bool slow = (state >> 30) & 1u;
  bool in_line = (state >> 31) & 1u;  // a line start has been seen (always true inside an extent)
  while (ev) {
    const int i = ctz32(ev);
    ev &= ev - 1;
    const uint64_t x = sg.lo + i;
    while (x >= cend) {
      ++chunk;
      cend = a.cs[chunk + 1];
      src.lim = a.lim(chunk);  // decoders read to the InputSplit chunk end
    }
    if ((sg.ls >> i) & 1u) {
      in_line = true;
      col0 = 0;
      from_mask = (1u << i) - 1u;
      slow = (sg.slow >> i) & 1u;
      // the chunk's first line: only newlines lie between its start and x
      // (a chunk row is the exclusive count at the chunk start, dmlc_amd.h)
      bool first = x == a.cs[chunk];
      if (MODE == 2 && !first) {
        uint64_t y = x;
        while (y > a.cs[chunk] && is_nl(src(y - 1))) --y;
        first = y == a.cs[chunk];
      }
      if (MODE == 2 && first) {
        uint64_t *row = a.chunk_tab + (uint64_t)chunk * 8;  // rows of 8 slots (dmlc_amd.h)
        for (int k = 0; k < C_N; ++k) row[k] = base.c[k] + cnt.c[k];
      }
      if (slow) {
        csv_line_seq<MODE>(src, a, x, cend, cnt, base);
      } else {
        if (MODE == 2) {
          const uint64_t r = base.c[C_ROWS] + cnt.c[C_ROWS];
          if (r < a.cap[C_ROWS]) a.offset[r] = base.c[C_INDEX] + cnt.c[C_INDEX];
          else raise_error(a.err, E_CAPACITY, x);
        }
        cnt.c[C_ROWS]++;
      }
    }
    if (!in_line || slow) continue;
    if ((sg.fs >> i) & 1u) {
      const uint64_t col = col0 + (uint32_t)popc32(sg.dl & ((1u << i) - 1u) & ~from_mask);
      const bool vc = is_value_col(a, col);
      Field f;
      if (MODE == 2 || (!vc && (int64_t)col != a.label_column)) {  // (the count pass decodes weights only)
        f = decode_field(src, a.vtype, x, dt);
      } else {
        f.f = 0.f;
        f.i = 0;
        f.nan_err = false;
        f.end = vc && field_consumed(src, a.vtype, x) ? x + 1 : x;
      }
      if (MODE == 2 && f.nan_err) raise_error(a.err, E_NAN_LITERAL, x);
      if ((int64_t)col == a.label_column) {
        if (MODE == 2) {
          const uint64_t r = base.c[C_LABEL] + cnt.c[C_LABEL];
          if (r < a.cap[C_LABEL]) store_val<int>(a.label, a.vtype, r, f.f, f.i);
          else raise_error(a.err, E_CAPACITY, x);
        }
        cnt.c[C_LABEL]++;
      } else if (!vc) {  // weight column (float)
        if (!(f.f != f.f)) {
          if (MODE == 2) {
            const uint64_t r = base.c[C_WEIGHT] + cnt.c[C_WEIGHT];
            if (r < a.cap[C_WEIGHT]) a.weight[r] = f.f;
            else raise_error(a.err, E_CAPACITY, x);
          }
          cnt.c[C_WEIGHT]++;
        }
      } else if (f.end != x) {
        if (MODE == 2) {
          const uint64_t r = base.c[C_INDEX] + cnt.c[C_INDEX];
          const uint64_t rv = base.c[C_VALUE] + cnt.c[C_VALUE];
          if (r < a.cap[C_INDEX] && rv < a.cap[C_VALUE]) {
            store_val<int>(a.value, a.vtype, rv, f.f, f.i);
            const uint64_t ix = value_rank(a, col);
            if (a.wide) reinterpret_cast<uint64_t *>(a.index)[r] = ix;
            else reinterpret_cast<uint32_t *>(a.index)[r] = (uint32_t)ix;
          } else {
            raise_error(a.err, E_CAPACITY, x);
          }
        }
        cnt.c[C_INDEX]++;
        cnt.c[C_VALUE]++;
      }
      // csv_parser.h:128-132: after the line's last field, no value column seen
      if (MODE == 2 && value_rank(a, col) + (vc ? 1 : 0) == 0) {
        uint64_t p = x;
        while (p < cend && !is_nl(src(p)) && src(p) != a.delim) ++p;
        if (p >= cend || is_nl(src(p))) raise_error(a.err, E_CSV_DELIM, p);
      }
    }
  }
}

template <class BK>
DA_HDF uint64_t first_line_start(const CsvArgs &a, BK &bk, uint64_t from, uint64_t to) {
  Src src;
  src.g = a.text;
  src.lds = nullptr;
  src.wbase = src.wend = 0;
  for (uint64_t base = from; base < to; base += kWin) {
    uint64_t best = kNone;
    const uint64_t lo = base + (uint64_t)bk.tid() * kSeg;
    const uint64_t hi = mn(lo + (uint64_t)kSeg, to);
    if (lo < hi) {
      int c = chunk_of(a.cs, a.nchunk, lo);
      for (uint64_t p = lo; p < hi; ++p) {
        while (p >= a.cs[c + 1]) ++c;
        src.lim = a.lim(c);
        if (csv_line_start(src, p, a.cs[c])) {
          best = p;
          break;
        }
      }
    }
    best = bk.min_u64(best);
    if (best != kNone) return best;
  }
  return kNone;
}

struct Shared {
  uint8_t win[kWin + 32];
  fast::DecTables dt;  // the window decoders' tables (exact_dec.h)
};

// The tile body.  MODE 1 = count pass, MODE 2 = write pass.
template <int MODE, class BK>
DA_HDF void tile(const CsvArgs &a, Shared &sh, BK &bk, uint64_t k) {
  const uint64_t tlo = k * a.tile_bytes;
  if (tlo >= a.n) return;
  if (a.gate && *a.gate == 0) return;  // the uniform-grammar kernel handled this input
  const uint64_t thi = mn(tlo + a.tile_bytes, a.n);
  const int tid = bk.tid();
  const Cnt zero = cnt_zero();
  Cnt tot = zero, mine = zero;
  Base64 tbase;
  for (int i = 0; i < C_N; ++i) tbase.c[i] = MODE == 2 ? a.tile_base[k * C_N + i] : 0;

  uint64_t w0 = first_line_start(a, bk, tlo, a.n);
  if (w0 == kNone || w0 >= thi) {
    if (MODE == 1 && tid < C_N) a.tile_cnt[k * C_N + tid] = 0;
    return;
  }
  uint32_t col0 = 0;  // column state at the window start (window 0 starts at a line start)
  uint32_t j = 0;     // window counter
  bool done = false;
  Src src;
  src.g = a.text;
  src.lds = sh.win;
  fast::init_dec_tables(sh.dt, bk);  // (read after the window's barrier)
#ifdef FSVM_EXACT_BYTEDEC  // A/B only: the byte decoders everywhere
  const fast::DecTables *dtp = nullptr;
#else
  const fast::DecTables *dtp = &sh.dt;
#endif
  while (!done) {
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
    bk.sync();
    src.wbase = abase;
    src.wend = mn(abase + (nunits << 4), a.n);

    Seg sg;
    sg.lo = w0 + (uint64_t)tid * kSeg;
    sg.hi = mn(sg.lo + (uint64_t)kSeg, wend);
    sg.ls = sg.dl = sg.fs = sg.slow = 0;
    sg.chunk = 0;
    uint32_t summary = 0;  // ColCombine element
    if (sg.lo < sg.hi) {
      sg.chunk = chunk_of(a.cs, a.nchunk, sg.lo);
      int c = sg.chunk;
      src.lim = a.lim(c);
      const int len = (int)(sg.hi - sg.lo);
      uint32_t nl, dl, ls = 0;
      seg_masks_csv(sh.win, (uint32_t)(sg.lo - abase), len, a.delim, &nl, &dl);
      // line starts: non-nl byte after an nl byte (or a chunk start), minus absorbed
      const uint32_t prev_nl = (sg.lo == 0 || is_nl(src(sg.lo - 1))) ? 1u : 0u;
      uint32_t cand = ~nl & ((nl << 1) | prev_nl);
      if (len < 32) cand &= (1u << len) - 1u;
      for (int cc = c; cc < a.nchunk && a.cs[cc] < sg.hi; ++cc)
        if (a.cs[cc] >= sg.lo && !((nl >> (a.cs[cc] - sg.lo)) & 1u)) cand |= 1u << (a.cs[cc] - sg.lo);
      uint32_t m = cand;
      while (m) {
        const int i = ctz32(m);
        m &= m - 1;
        const uint64_t x = sg.lo + i;
        while (x >= a.cs[c + 1]) ++c;
        src.lim = a.lim(c);
        if (csv_line_start(src, x, a.cs[c])) {
          ls |= 1u << i;
          if (!a.fast_delim || is_bom_at(src, x)) sg.slow |= 1u << i;
        }
      }
      src.lim = a.lim(sg.chunk);
      sg.ls = ls;
      sg.dl = dl & ~nl;
      // field starts: line starts of fast lines, and bytes after a delimiter that are not nl
      const uint32_t prev_dl = (sg.lo > 0 && src(sg.lo - 1) == a.delim && !(ls & 1u)) ? 1u : 0u;
      uint32_t fs = ((sg.dl << 1) | prev_dl) & ~nl;
      if (len < 32) fs &= (1u << len) - 1u;
      sg.fs = fs | (ls & ~sg.slow);
      if (ls) {
        const int last = 31 - clz32(ls);
        const uint32_t after = sg.dl & ~((1u << last) - 1u);  // delimiters at or after it
        summary = 0x80000000u | (((sg.slow >> last) & 1u) << 30) | (uint32_t)popc32(after);
      } else {
        summary = (uint32_t)popc32(sg.dl);
      }
    }
    uint32_t col_total;
    const uint32_t col_ex = bk.exclusive(summary, 0u, ColCombine(), &col_total);
    const uint32_t in_state = ColCombine()(col0 | 0x80000000u, col_ex);
    const uint32_t next0 = ColCombine()(col0 | 0x80000000u, col_total);

    Base64 nob;
    for (int i = 0; i < C_N; ++i) nob.c[i] = 0;
    Cnt cc = zero;
    // the count pass records each thread's window counts; the write pass
    // takes them instead of counting again (args.h CsvArgs.rec)
    uint32_t *rw = a.rec && j < a.rec_win ? a.rec + ((uint64_t)k * a.rec_win + j) * 4 * kThreads : nullptr;
    if (MODE == 2 && rw) {
      cc.c[C_ROWS] = rw[tid];
      cc.c[C_INDEX] = cc.c[C_VALUE] = rw[kThreads + tid];
      cc.c[C_LABEL] = rw[2 * kThreads + tid];
      cc.c[C_WEIGHT] = rw[3 * kThreads + tid];
    } else {
      if (sg.lo < sg.hi) walk<1>(a, src, sg, in_state, cc, nob, dtp);
      if (MODE == 1 && rw) {
        rw[tid] = cc.c[C_ROWS];
        rw[kThreads + tid] = cc.c[C_VALUE];
        rw[2 * kThreads + tid] = cc.c[C_LABEL];
        rw[3 * kThreads + tid] = cc.c[C_WEIGHT];
      }
    }
    if (MODE == 1) {
      mine = CntAdd()(mine, cc);
    } else {
      Cnt wtot;
      const Cnt ex = bk.exclusive(cc, zero, CntAdd(), &wtot);
      if (sg.lo < sg.hi) {
        Base64 b;
        for (int i = 0; i < C_N; ++i) b.c[i] = tbase.c[i] + tot.c[i] + ex.c[i];
        Cnt local = zero;
        walk<2>(a, src, sg, in_state, local, b, dtp);
      }
      tot = CntAdd()(tot, wtot);
    }
    col0 = next0 & 0x7FFFFFFFu;
    w0 = wend;
    ++j;
    bk.sync();
  }
  if (MODE == 1) {
    Cnt total;
    (void)bk.exclusive(mine, zero, CntAdd(), &total);
    if (tid < C_N) a.tile_cnt[k * C_N + tid] = total.c[tid];
  }
}

}  // namespace csv
}  // namespace dmlc_amd
