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
// then decodes its runs token-parallel (one run per thread per step), writing
// index / value / label coalesced.  Any byte or structure outside the grammar
// sets the gate word; the launcher then runs the exact tile kernels
// (libsvm_core.h) instead, so results are always the reference's.
//
// Written once against a block policy BK {tid, sync, exclusive} so the GPU
// kernel (libsvm.hip) and the test-only CPU emulator (tests/emu) share it.
#pragma once
#include "args.h"
#include "decode.h"

namespace dmlc_amd {
namespace fsvm {

constexpr int kSegB = 64;                // bytes per thread (one 64-bit mask)
constexpr int kTile = kThreads * kSegB;  // 16 KiB of text per tile
constexpr int kPre = 64;                 // staged bytes before the tile (look-back)
constexpr int kPost = 128;               // staged bytes after it (runs crossing the end)
constexpr int kStage = kPre + kTile + kPost;
constexpr int kMaxCs = 32;               // chunk starts per tile the fast path accepts
constexpr int kMaxRuns = kTile / 2 + kMaxCs + 2;
constexpr uint64_t kAgg = 1ull << 62, kIncl = 2ull << 62, kValMask = (1ull << 62) - 1;
constexpr uint32_t kSpinLimit = 1u << 26;

enum : uint32_t { R_NONE = 0, R_L = 1, R_K = 2, R_I = 3 };
// look-back counter slots
enum { Q_ROWS = 0, Q_INDEX = 1, Q_VALUE = 2, Q_WEIGHT = 3 };

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

// Masks of the 64 bytes at p (16-byte aligned); bytes >= nvalid are outside
// the text and classify as blanks.
DA_HD Masks classify64(const uint8_t *p, int nvalid) {
  uint32_t dl = 0, dh = 0, nl = 0, nh = 0, cl = 0, ch = 0;
  uint32_t all = 0x80808080u, orv = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t w[4];
    load16(p + 16 * q, w);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int i = 4 * q + j;
      uint32_t x = w[j];
      uint32_t cls = classify4(x);
      const int nb = nvalid - 4 * i;
      if (nb < 4) {
        const uint32_t vm = nb <= 0 ? 0u : ((1u << (8 * nb)) - 1u);
        cls = (cls & vm) | (0x20202020u & ~vm);
        x &= vm;
      }
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

struct Shared {  // LDS of one workgroup
  alignas(16) uint8_t text[kStage];               // position p <-> text[p - tlo + kPre]
  uint64_t md[kThreads + 1];          // slot 0: the segment before the tile; slot t+1: segment t
  uint64_t mn[kThreads + 1];
  uint64_t mc[kThreads + 1];
  uint16_t runs[kMaxRuns];            // run starts (tile-relative), grouped L | W | I | V
  uint64_t csl[kMaxCs + 1];           // chunk starts in [tlo, thi]
  uint64_t cfloor, cnext, base[4];
  uint32_t ncs, c_first, tile, tot[5];
};

struct Cnt5 {
  uint32_t c[5];  // L, W, I, V, bad
};
struct Cnt5Add {
  DA_HD Cnt5 operator()(const Cnt5 &a, const Cnt5 &b) const {
    Cnt5 r;
    for (int i = 0; i < 5; ++i) r.c[i] = a.c[i] + b.c[i];
    return r;
  }
};

struct Tile {
  const FastSvmArgs *a;
  Shared *sh;
  uint64_t tlo, thi;

  // masks of the absolute 64-byte segment g (full segments only when g < tlo/64)
  DA_HD void seg(uint64_t g, uint64_t *d, uint64_t *n, uint64_t *c) const {
    const uint64_t g0 = tlo >> 6;
    if (g < g0 + kThreads && (g >= g0 || (tlo > 0 && g + 1 == g0))) {
      const uint64_t s = g + 1 - g0;
      *d = sh->md[s];
      *n = sh->mn[s];
      *c = sh->mc[s];
      return;
    }
    const Masks m = classify64(a->text + (g << 6), 64);
    *d = m.d;
    *n = m.n;
    *c = m.c;
  }

  // last position in [lo, hi) whose bit is set in mask `kind` (0 D, 1 not-D,
  // 2 newline, 3 colon), or kNone
  DA_HD uint64_t last_bit(int kind, uint64_t lo, uint64_t hi) const {
    if (lo >= hi) return kNone;
    for (uint64_t g = (hi - 1) >> 6;; --g) {
      uint64_t d, n, c;
      seg(g, &d, &n, &c);
      uint64_t w = kind == 0 ? d : kind == 1 ? ~d : kind == 2 ? n : c;
      const uint64_t b0 = g << 6;
      if (hi - b0 < 64) w &= (1ull << (hi - b0)) - 1;
      if (lo > b0) w &= ~((1ull << (lo - b0)) - 1);
      if (w) return b0 + 63 - clz64(w);
      if (b0 <= lo) return kNone;
    }
  }

  DA_HD uint64_t floor_of(uint64_t p) const {  // last chunk start <= p
    uint64_t f = sh->cfloor;
    for (uint32_t i = 0; i < sh->ncs && sh->csl[i] <= p; ++i) f = sh->csl[i];
    return f;
  }
  DA_HD uint64_t next_cs(uint64_t p) const {  // first chunk start > p
    for (uint32_t i = 0; i < sh->ncs; ++i)
      if (sh->csl[i] > p) return sh->csl[i];
    return sh->cnext;
  }
  DA_HD bool is_cs(uint64_t p) const {
    for (uint32_t i = 0; i < sh->ncs; ++i)
      if (sh->csl[i] == p) return true;
    return p == sh->cnext;
  }

  // role of the run starting at q (q > its chunk start f, or == f)
  DA_HD uint32_t role_of(uint64_t q, uint64_t f) const {
    if (q == f) return R_L;
    const uint64_t p = last_bit(0, f, q);
    if (p == kNone) return R_L;
    if (last_bit(2, p + 1, q) != kNone) return R_L;
    if (last_bit(3, p + 1, q) != kNone) return R_K;
    return R_I;
  }
};

// Runs, roles and counts of segment tid (positions P .. P+63).
struct SegOut {
  uint64_t L, W, I, V;
  uint32_t bad;
};

DA_HD SegOut segment_roles(const Tile &t, int tid) {
  SegOut o;
  o.L = o.W = o.I = o.V = 0;
  o.bad = 0;
  const FastSvmArgs &a = *t.a;
  const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
  if (P >= a.n) return o;
  const int nv = (int)mn<uint64_t>(64, a.n - P);
  const uint64_t valid = nv == 64 ? ~0ull : ((1ull << nv) - 1);
  const uint64_t D = t.sh->md[tid + 1], N = t.sh->mn[tid + 1], C = t.sh->mc[tid + 1];
  uint64_t S = 0;
  for (uint32_t i = 0; i < t.sh->ncs; ++i) {
    const uint64_t x = t.sh->csl[i];
    if (x >= P && x < P + (uint64_t)nv) S |= 1ull << (x - P);
  }
  // ---- carry-in: state just before P
  uint32_t dc = 0, ginl = 0, ginc = 0, prole = R_NONE;
  const uint64_t F = t.floor_of(P);
  if (P != F) {
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
  const uint64_t Z = ~RS;
  const uint64_t xl = L << 1, xk = K << 1;
  const uint64_t prevL = ((Z + (xl & Z) + (prole == R_L ? 1u : 0u)) | xl) & RS;
  const uint64_t prevK = ((Z + (xk & Z) + (prole == R_K ? 1u : 0u)) | xk) & RS;
  if (K & prevK) o.bad = 1;  // "a:b:c": the pair grammar re-pairs (strtonum.h:684-702)
  o.L = L;
  o.W = K & prevL;
  o.V = K & ~prevL;
  o.I = RS & ~L & ~K;
  return o;
}

DA_HD uint32_t lower_count(const uint16_t *r, uint32_t n, uint32_t x) {  // #entries < x (sorted)
  uint32_t lo = 0, hi = n;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (r[mid] < x) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// MODE 1: count only (size query); MODE 2: parse and write.
template <int MODE, class BK>
DA_HDF void tile(const FastSvmArgs &a, Shared &sh, BK &bk) {
  const int tid = bk.tid();
  if (tid == 0) {
    sh.tile = (a.skip_if_gated && *a.gate) ? ~0u : atomic_add_u32(a.ticket, 1);
  }
  bk.sync();
  const uint32_t k = sh.tile;
  if (k == ~0u) return;
  Tile t;
  t.a = &a;
  t.sh = &sh;
  t.tlo = (uint64_t)k * kTile;
  t.thi = mn<uint64_t>(t.tlo + kTile, a.n);

  // ---- chunk starts touching the tile (binary search once)
  if (tid == 0) {
    const int c0 = chunk_of(a.cs, a.nchunk, t.tlo);
    sh.cfloor = a.cs[c0];
    int c = c0;
    if (a.cs[c] < t.tlo) ++c;
    sh.c_first = (uint32_t)c;
    uint32_t m = 0;
    while (c < a.nchunk && a.cs[c] <= t.thi) {
      if (m < kMaxCs) sh.csl[m] = a.cs[c];
      ++m;
      ++c;
    }
    sh.ncs = m < kMaxCs ? m : kMaxCs;
    sh.cnext = a.cs[c];  // cs[nchunk] == n
    sh.tot[4] = m > kMaxCs;
  }
  // ---- stage [tlo - kPre, thi + kPost) into LDS
  {
    const uint64_t s0 = t.tlo >= (uint64_t)kPre ? t.tlo - kPre : 0;
    const uint64_t s1 = mn<uint64_t>(t.thi + kPost, a.n);
    uint8_t *dst = sh.text + (s0 + kPre - t.tlo);
    const uint64_t nunits = (s1 - s0 + 15) >> 4;
    for (uint64_t u = tid; u < nunits; u += kThreads) {
      const uint64_t g = s0 + (u << 4);
      if (g + 16 <= a.n) {
        uint32_t w[4];
        load16(a.text + g, w);
        memcpy(dst + (u << 4), w, 16);
      } else {
        for (int q = 0; q < 16; ++q) dst[(u << 4) + q] = g + q < a.n ? a.text[g + q] : 0;
      }
    }
  }
  bk.sync();
  // ---- classify: segment tid -> slot tid+1; thread 0 also the segment before the tile
  uint32_t bad = 0;
  {
    const uint64_t P = t.tlo + (uint64_t)tid * kSegB;
    const int nv = P < a.n ? (int)mn<uint64_t>(64, a.n - P) : 0;
    const Masks m = classify64(sh.text + kPre + tid * kSegB, nv);
    sh.md[tid + 1] = m.d;
    sh.mn[tid + 1] = m.n;
    sh.mc[tid + 1] = m.c;
    bad = m.bad;
    if (tid == 0) {
      if (t.tlo > 0) {
        const Masks p = classify64(sh.text, 64);
        sh.md[0] = p.d;
        sh.mn[0] = p.n;
        sh.mc[0] = p.c;
      } else {
        sh.md[0] = sh.mn[0] = sh.mc[0] = 0;
      }
      bad |= sh.tot[4];
    }
  }
  bk.sync();
  // ---- roles, counts, eligibility
  const SegOut so = segment_roles(t, tid);
  Cnt5 mine;
  mine.c[0] = (uint32_t)popc64(so.L);
  mine.c[1] = (uint32_t)popc64(so.W);
  mine.c[2] = (uint32_t)popc64(so.I);
  mine.c[3] = (uint32_t)popc64(so.V);
  mine.c[4] = bad | so.bad;
  Cnt5 zero;
  for (int i = 0; i < 5; ++i) zero.c[i] = 0;
  Cnt5 tot;
  const Cnt5 ex = bk.exclusive(mine, zero, Cnt5Add(), &tot);
  // ---- run lists (tile-relative offsets), grouped by role
  if (MODE == 2) {
    const uint32_t bL = ex.c[0], bW = tot.c[0] + ex.c[1], bI = tot.c[0] + tot.c[1] + ex.c[2],
                   bV = tot.c[0] + tot.c[1] + tot.c[2] + ex.c[3];
    const uint16_t off = (uint16_t)(tid * kSegB);
    uint64_t m;
    uint32_t j;
    for (m = so.L, j = bL; m; m &= m - 1) sh.runs[j++] = (uint16_t)(off + ctz64(m));
    for (m = so.W, j = bW; m; m &= m - 1) sh.runs[j++] = (uint16_t)(off + ctz64(m));
    for (m = so.I, j = bI; m; m &= m - 1) sh.runs[j++] = (uint16_t)(off + ctz64(m));
    for (m = so.V, j = bV; m; m &= m - 1) sh.runs[j++] = (uint16_t)(off + ctz64(m));
  }
  // ---- decoupled look-back: output base of this tile per counter
  if (tid < 4) {
    // lane -> counter: rows (L), index (I), value (V), weight (W)
    const uint64_t agg = tid == 0 ? tot.c[0] : tid == 1 ? tot.c[2] : tid == 2 ? tot.c[3] : tot.c[1];
    uint64_t *w = a.lb + (uint64_t)k * 4 + tid;
    uint64_t excl = 0;
    if (k == 0) {
      store_agent_u64(w, kIncl | agg);
    } else {
      store_agent_u64(w, kAgg | agg);
      uint64_t j = k - 1;
      uint32_t spins = 0;
      for (;;) {
        const uint64_t v = load_agent_u64(a.lb + j * 4 + tid);
        const uint64_t f = v & ~kValMask;
        if (f == 0) {
          if (++spins > kSpinLimit) {  // never expected: hand the input to the exact path
            atomic_or_u32(a.gate, 2u);
            break;
          }
          spin_pause();
          continue;
        }
        excl += v & kValMask;
        if (f == kIncl) break;
        --j;
      }
      store_agent_u64(w, kIncl | (excl + agg));
    }
    sh.base[tid] = excl;
    if (tid == 0 && tot.c[4]) atomic_or_u32(a.gate, 1u);
  }
  bk.sync();
  const uint64_t bRows = sh.base[Q_ROWS], bIdx = sh.base[Q_INDEX], bVal = sh.base[Q_VALUE],
                 bW = sh.base[Q_WEIGHT];
  // ---- the last tile publishes the totals (dmlc_amd_result.count)
  if (k + 1 == a.ntiles && tid == 0) {
    const uint64_t rows = bRows + tot.c[0];
    a.res[C_ROWS] = rows;
    a.res[C_INDEX] = bIdx + tot.c[2];
    a.res[C_VALUE] = bVal + tot.c[3];
    a.res[C_WEIGHT] = bW + tot.c[1];
    a.res[C_QID] = 0;
    a.res[C_LABEL] = rows;
    a.res[C_FIELD] = 0;
    if (MODE == 2 && a.offset && rows < a.cap[C_ROWS] + 1) a.offset[rows] = bIdx + tot.c[2];
  }
  if (MODE != 2) return;

  // ---- token-parallel decode + coalesced stores
  const uint32_t nL = tot.c[0], nW = tot.c[1], nI = tot.c[2], nV = tot.c[3];
  const uint16_t *rL = sh.runs, *rW = sh.runs + nL, *rI = rW + nW, *rV = rI + nI;
  Src src;
  src.g = a.text;
  src.wbase = t.tlo >= (uint64_t)kPre ? t.tlo - kPre : 0;
  src.wend = mn<uint64_t>(t.thi + kPost, a.n);
  src.lds = sh.text + (src.wbase + kPre - t.tlo);
  const bool simple_lim = sh.ncs == 0;  // no chunk boundary before cnext
  for (uint32_t j = tid; j < nI; j += kThreads) {
    const uint64_t q = t.tlo + rI[j];
    src.lim = simple_lim ? sh.cnext : t.next_cs(q);
    uint64_t v;
    if (!parse_uint(src, q, a.wide != 0, &v)) {
      raise_error(a.err, E_NEG_INDEX, q);
      v = 0;
    }
    if (a.indexing_mode > 0) --v;
    const uint64_t r = bIdx + j;
    if (r < a.cap[C_INDEX]) {
      if (a.wide) reinterpret_cast<uint64_t *>(a.index)[r] = v;
      else reinterpret_cast<uint32_t *>(a.index)[r] = (uint32_t)v;
    } else {
      raise_error(a.err, E_CAPACITY, q);
    }
  }
  for (uint32_t j = tid; j < nV; j += kThreads) {
    const uint64_t q = t.tlo + rV[j];
    src.lim = simple_lim ? sh.cnext : t.next_cs(q);
    uint64_t e;
    bool nan_err = false;
    const float v = parse_float(src, q, &e, &nan_err);
    const uint64_t r = bVal + j;
    if (r < a.cap[C_VALUE]) a.value[r] = v;
    else raise_error(a.err, E_CAPACITY, q);
  }
  for (uint32_t j = tid; j < nL; j += kThreads) {
    const uint64_t q = t.tlo + rL[j];
    src.lim = simple_lim ? sh.cnext : t.next_cs(q);
    uint64_t e;
    bool nan_err = false;
    const float v = parse_float(src, q, &e, &nan_err);
    const uint64_t r = bRows + j;
    if (r < a.cap[C_ROWS]) {
      a.label[r] = v;
      a.offset[r] = bIdx + lower_count(rI, nI, rL[j]);
    } else {
      raise_error(a.err, E_CAPACITY, q);
    }
  }
  for (uint32_t j = tid; j < nW; j += kThreads) {
    const uint64_t q = t.tlo + rW[j];
    src.lim = simple_lim ? sh.cnext : t.next_cs(q);
    uint64_t e;
    bool nan_err = false;
    const float v = parse_float(src, q, &e, &nan_err);
    const uint64_t r = bW + j;
    if (r < a.cap[C_WEIGHT]) a.weight[r] = v;
    else raise_error(a.err, E_CAPACITY, q);
  }
  // ---- per-chunk exclusive counts at each chunk start inside the tile
  if (a.chunk_tab) {
    for (uint32_t i = tid; i < sh.ncs; i += kThreads) {
      const uint64_t x = sh.csl[i];
      if (x >= t.thi) continue;
      const uint32_t rel = (uint32_t)(x - t.tlo);
      uint64_t *row = a.chunk_tab + (uint64_t)(sh.c_first + i) * 8;
      const uint64_t rows = bRows + lower_count(rL, nL, rel);
      row[C_ROWS] = rows;
      row[C_INDEX] = bIdx + lower_count(rI, nI, rel);
      row[C_VALUE] = bVal + lower_count(rV, nV, rel);
      row[C_WEIGHT] = bW + lower_count(rW, nW, rel);
      row[C_QID] = 0;
      row[C_LABEL] = rows;
      row[C_FIELD] = 0;
    }
  }
}

}  // namespace fsvm
}  // namespace dmlc_amd
