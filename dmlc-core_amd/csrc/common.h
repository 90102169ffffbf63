// common.h -- pieces shared by every tile body: sizes, counter slots, error
// codes, character classes (strtonum.h), the byte source and small helpers.
// Compiles as HIP device code and as plain C++ (test emulator).
#pragma once
#include "hd.h"

namespace dmlc_amd {

constexpr int kWave = 64;
constexpr int kThreads = 256;           // threads per tile workgroup (4 waves)
constexpr int kSeg = 32;                // bytes per thread per window
constexpr int kWin = kThreads * kSeg;   // 8 KiB window staged in LDS per step
constexpr int kWaves = kThreads / kWave;
constexpr uint64_t kNone = ~0ull;

// Counter slots carried through the tile scan; same order as dmlc_amd_result.
enum { C_ROWS = 0, C_INDEX, C_VALUE, C_WEIGHT, C_QID, C_LABEL, C_FIELD, C_N };

// Error codes (mirror the reference's fatal CHECKs; see include/dmlc_amd.h).
enum {
  E_OK = 0,
  E_NEG_INDEX = 1,    // strtonum.h:416 CHECK_EQ(sign, true)
  E_NAN_LITERAL = 2,  // strtonum.h:163 CHECK_EQ(*p, ')') "Invalid NAN literal"
  E_CSV_DELIM = 3,    // csv_parser.h:128-132 delimiter not found
  E_CAPACITY = 16,    // caller buffers too small (not a reference error)
};

// ---------------------------------------------------------- char classes --
DA_HD bool is_space(uint32_t c) {  // dmlc::isspace, strtonum.h:27-29
  return c == ' ' || c == '\t' || c == '\r' || c == '\n' || c == '\f';
}
DA_HD bool is_blank(uint32_t c) { return c == ' ' || c == '\t'; }  // strtonum.h:37-39
DA_HD bool is_digit(uint32_t c) { return c - '0' < 10u; }
DA_HD bool is_alpha(uint32_t c) { return (c | 32u) - 'a' < 26u; }
DA_HD bool is_digitchar(uint32_t c) {  // strtonum.h:70-72
  return is_digit(c) || c == '+' || c == '-' || c == '.' || c == 'e' || c == 'E';
}
DA_HD bool is_nl(uint32_t c) { return c == '\n' || c == '\r'; }
DA_HD bool is_cspace(uint32_t c) { return c == ' ' || c - '\t' < 5u; }  // glibc isspace

// ----------------------------------------------------------- byte source --
// Reads text bytes at absolute positions: from the staged LDS window when it
// holds them, otherwise from HBM.  Positions at or beyond `lim` (the end of
// the chunk being parsed) read as NUL -- what the reference sees after a
// std::string, and what the oracle restates.
struct Src {
  const uint8_t *g;
  uint64_t lim;
  const uint8_t *lds;  // LDS bytes for [wbase, wend)
  uint64_t wbase, wend;
  DA_HD uint32_t operator()(uint64_t p) const {
    if (p >= lim) return 0u;
    if (p >= wbase && p < wend) return lds[p - wbase];
    return g[p];
  }
};

// Counter vector for per-window scans (32-bit, window-local).
struct Cnt {
  uint32_t c[8];
};
struct CntAdd {
  DA_HD Cnt operator()(const Cnt &a, const Cnt &b) const {
    Cnt r;
    for (int i = 0; i < 8; ++i) r.c[i] = a.c[i] + b.c[i];
    return r;
  }
};
DA_HD Cnt cnt_zero() {
  Cnt z;
  for (int i = 0; i < 8; ++i) z.c[i] = 0;
  return z;
}
struct Base64 {  // absolute 64-bit ranks
  uint64_t c[C_N];
};

// indexing_mode < 0 (libsvm_parser.h:165-171): the minimum index of the
// ParseBlock unit a thread is walking, kept in registers and flushed to
// chunk_min[unit] when the walk enters another unit and once per tile
// (tile_min_flush), instead of one device atomic per index on a handful of
// addresses (which serialised the count pass: 437 ms on config 2).
struct MinAcc {
  int unit = -1;
  uint64_t v = ~0ull;
  DA_HD void add(uint64_t *cmin, int u, uint64_t x) {
    if (u != unit) {
      flush(cmin);
      unit = u;
      v = x;
    } else if (x < v) {
      v = x;
    }
  }
  DA_HD void flush(uint64_t *cmin) {
    if (unit >= 0) atomic_min_u64_if_lower((unsigned long long *)&cmin[unit], (unsigned long long)v);
    unit = -1;
    v = ~0ull;
  }
};
// Block-wide: the threads on the block's lowest unit reduce first (one atomic
// for the common tile inside one unit); any other unit flushes on its own.
template <class BK>
DA_HDF void tile_min_flush(MinAcc &m, uint64_t *cmin, BK &bk) {
  const uint64_t u0 = bk.min_u64(m.unit >= 0 ? (uint64_t)m.unit : ~0ull);
  const uint64_t m0 = bk.min_u64(m.unit >= 0 && (uint64_t)m.unit == u0 ? m.v : ~0ull);
  if (bk.tid() == 0 && u0 != ~0ull) atomic_min_u64_if_lower((unsigned long long *)&cmin[u0], (unsigned long long)m0);
  if (m.unit >= 0 && (uint64_t)m.unit != u0) m.flush(cmin);
  m.unit = -1;
}

// Record the first (lowest position) error: (pos << 16) | code, min wins.
DA_HD void raise_error(unsigned long long *err, uint32_t code, uint64_t pos) {
  atomic_min_u64(err, ((unsigned long long)(pos & 0xFFFFFFFFFFFFull) << 16) | code);
}

// Chunk containing position p (cs sorted, nchunk+1 entries, cs[nchunk] = n).
DA_HD int chunk_of(const uint64_t *cs, int nchunk, uint64_t p) {
  int lo = 0, hi = nchunk;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (cs[mid] <= p) lo = mid;
    else hi = mid;
  }
  return lo;
}

DA_HD bool is_chunk_start(const uint64_t *cs, int nchunk, uint64_t p) {
  return cs[chunk_of(cs, nchunk, p)] == p;
}

}  // namespace dmlc_amd
