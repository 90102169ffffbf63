// libsvm.hip -- MI355X kernels for LibSVMParser::ParseBlock
// (src/data/libsvm_parser.h:85-172, strtonum.h ParsePair :667-703).
//
// Work decomposition (DESIGN.md "libsvm tile kernel"):
//   * The input is a device buffer of one or more InputSplit chunks (each chunk is
//     one ParseBlock, i.e. the reference with nthread = 1).
//   * Tile k owns every LINE START in [k*T, (k+1)*T); its extent runs from its
//     first line start to the first line start at or after (k+1)*T, so every line
//     is parsed by exactly one workgroup and no parse state crosses workgroups.
//   * A workgroup streams its extent through 8 KiB LDS windows; each of the 256
//     threads owns a 32-byte segment of the window.
//   * Per line the owner of the line start parses the head section sequentially
//     (label[:weight] [qid:n], libsvm_parser.h:99-132) and marks R1, the first
//     feature run.  Feature runs follow a 4-state role machine
//     {PRE, FIRST(index), SECOND(value), DEAD(comment)} whose per-segment
//     transition functions are composed with a block scan.
//   * count pass -> tile scan -> write pass (same walk, now decoding and storing
//     at scanned ranks).
#include "decode.h"
#include "dmlc_amd_kernels.h"
#include "scan.h"

namespace dmlc_amd {

namespace {

constexpr uint64_t kNone = ~0ull;
enum : uint32_t { S_PRE = 0, S_F = 1, S_S = 2, S_D = 3 };
constexpr uint32_t kIdentityFn = 0xE4u;  // entry i -> i

__device__ __forceinline__ uint32_t fn_apply(uint32_t f, uint32_t T) {
  // result[i] = T[f[i]]
  uint32_t r = 0;
#pragma unroll
  for (int i = 0; i < 4; ++i) r |= ((T >> (2 * ((f >> (2 * i)) & 3u))) & 3u) << (2 * i);
  return r;
}
struct FnCompose {  // "a then b"
  __device__ uint32_t operator()(uint32_t a, uint32_t b) const { return fn_apply(a, b); }
};

struct Head {
  uint64_t label, wpos, qpos, r1;
  bool row, w, q;
};

// Head section of one line (libsvm_parser.h:99-132 + first feature run, :134-140).
// `ls` = line start, `l0` = ls is a chunk start (comment recognition),
// `lim` = chunk end.  The line ends at the first '\n'/'\r' after ls, or lim.
template <typename F>
__device__ Head head_parse(const F &at, uint64_t ls, bool l0, uint64_t lim) {
  Head h;
  h.label = h.wpos = h.qpos = h.r1 = kNone;
  h.row = h.w = h.q = false;
  auto eol = [&](uint64_t p) { return p >= lim || (p > ls && is_nl(at(p))); };
  uint64_t p = ls;
  if (l0) {  // IgnoreCommentAndBlank at the block's first line
    while (!eol(p)) {
      uint32_t c = at(p);
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
    h.wpos = p;  // == line end for "label:" (decoded there, as the reference does)
    while (!eol(p) && is_digitchar(at(p))) ++p;
  }
  while (p < lim && at(p) == ' ') ++p;
  if (!eol(p) && at(p) == 'q' && at(p + 1) == 'i' && at(p + 2) == 'd' && at(p + 3) == ':') {
    h.q = true;
    h.qpos = p + 4;
    p += 4;
    while (!eol(p) && is_digitchar(at(p))) ++p;
  }
  while (!eol(p)) {  // IgnoreCommentAndBlank before the first feature
    uint32_t c = at(p);
    if (c == '#') return h;
    if (!is_blank(c)) break;
    ++p;
  }
  while (!eol(p) && !is_digitchar(at(p))) ++p;
  if (!eol(p)) h.r1 = p;
  return h;
}

// First non-blank byte of the gap that ends at `x` (exclusive) and starts after
// the previous digitchar; 0 if the gap is all blanks.  Stops at a line start.
template <typename F>
__device__ __forceinline__ uint32_t gap_fnb(const F &at, uint64_t x, uint64_t floor) {
  uint32_t fnb = 0;
  while (x > floor) {
    uint32_t c = at(--x);
    if (is_digitchar(c)) break;
    if (!is_blank(c)) fnb = c;
    if (is_nl(c)) break;
  }
  return fnb;
}

struct Tile {
  const LibsvmArgs *a;
  Src src;           // lim is updated per chunk
  const uint32_t *r1bits;
  uint64_t w0;       // window logical start (bits are relative to it)
};

struct Seg {
  uint64_t lo, hi;   // [lo, hi) absolute
  uint32_t rs, ls, le;  // run-start / line-start / line-end masks (bit i <-> lo + i)
  int chunk;         // chunk of position lo
};

__device__ __forceinline__ bool r1_bit(const uint32_t *bits, uint64_t w0, uint64_t x) {
  uint64_t o = x - w0;
  return (bits[o >> 5] >> (o & 31)) & 1u;
}

struct Base64 {
  uint64_t c[C_N];
};

template <int MODE>  // 0 = transition function, 1 = count, 2 = emit
__device__ void walk(Tile &t, const Seg &sg, uint32_t &st, Cnt &cnt, const Base64 &base) {
  const LibsvmArgs &a = *t.a;
  uint32_t ev = sg.rs | sg.ls | sg.le;
  int chunk = sg.chunk;
  uint64_t cfloor = a.cs[chunk], cend = a.cs[chunk + 1];
  t.src.lim = cend;
  while (ev) {
    const int i = __builtin_ctz(ev);
    ev &= ev - 1;
    const uint64_t x = sg.lo + i;
    if ((sg.ls >> i) & 1u) {
      while (x >= cend) {  // entered the next chunk
        ++chunk;
        cfloor = a.cs[chunk];
        cend = a.cs[chunk + 1];
        t.src.lim = cend;
      }
      if (MODE == 0) {
        st = 0u;  // all PRE
      } else {
        st = S_PRE;
        const bool l0 = x == cfloor;
        Head h = head_parse(t.src, x, l0, cend);
        if (MODE == 2 && l0) {
          uint64_t *row = a.chunk_tab + (uint64_t)chunk * C_N;
          for (int k = 0; k < C_N; ++k) row[k] = base.c[k] + cnt.c[k];
        }
        if (h.row) {
          if (MODE == 2) {
            const uint64_t r = base.c[C_ROWS] + cnt.c[C_ROWS];
            bool nan_err = false;
            uint64_t e;
            if (r < a.cap[C_ROWS]) {
              a.label[r] = parse_float(t.src, h.label, &e, &nan_err);
              a.offset[r] = base.c[C_INDEX] + cnt.c[C_INDEX];
            } else {
              raise_error(a.err, E_CAPACITY, x);
            }
            if (h.w) {
              const uint64_t wr = base.c[C_WEIGHT] + cnt.c[C_WEIGHT];
              if (wr < a.cap[C_WEIGHT]) a.weight[wr] = parse_float(t.src, h.wpos, &e, &nan_err);
              else raise_error(a.err, E_CAPACITY, x);
            }
            if (h.q) {
              const uint64_t qr = base.c[C_QID] + cnt.c[C_QID];
              if (qr < a.cap[C_QID]) a.qid[qr] = (uint64_t)c_strtoll(t.src, h.qpos, 10, &e);
              else raise_error(a.err, E_CAPACITY, x);
            }
            if (nan_err) raise_error(a.err, E_NAN_LITERAL, x);
          }
          cnt.c[C_ROWS]++;
          cnt.c[C_LABEL]++;
          cnt.c[C_WEIGHT] += h.w;
          cnt.c[C_QID] += h.q;
        }
      }
    }
    if ((sg.rs >> i) & 1u) {
      while (x >= cend) {
        ++chunk;
        cfloor = a.cs[chunk];
        cend = a.cs[chunk + 1];
        t.src.lim = cend;
      }
      if (MODE == 0) {
        if (r1_bit(t.r1bits, t.w0, x)) {
          st = 0x55u;  // all FIRST
        } else {
          // only entries currently in F or S depend on the gap
          const uint32_t fs = (st ^ (st >> 1)) & 0x55u;  // entry == 1 or 2
          if (fs) {
            const uint32_t g = gap_fnb(t.src, x, cfloor);
            const uint32_t tF = g == '#' ? S_D : (g == ':' ? S_S : S_F);
            const uint32_t tS = g == '#' ? S_D : S_F;
            st = fn_apply(st, S_PRE | (tF << 2) | (tS << 4) | (S_D << 6));
          }
        }
      } else {
        uint32_t role = 0;  // 0 none, 1 index, 2 value
        if (r1_bit(t.r1bits, t.w0, x)) {
          st = S_F;
          role = 1;
        } else if (st == S_F || st == S_S) {
          const uint32_t g = gap_fnb(t.src, x, cfloor);
          if (g == '#') st = S_D;
          else if (g == ':' && st == S_F) st = S_S, role = 2;
          else st = S_F, role = 1;
        }
        if (role == 1) {
          if (MODE == 2 || a.indexing_mode < 0) {
            uint64_t v;
            if (!parse_uint(t.src, x, a.wide, &v)) {
              raise_error(a.err, E_NEG_INDEX, x);
              v = 0;
            }
            if (MODE == 1) {
              atomicMin((unsigned long long *)&a.chunk_min[chunk], (unsigned long long)v);
            } else {
              if (a.indexing_mode > 0 || (a.indexing_mode < 0 && a.chunk_min[chunk] > 0)) --v;
              const uint64_t ir = base.c[C_INDEX] + cnt.c[C_INDEX];
              if (ir < a.cap[C_INDEX]) {
                if (a.wide) reinterpret_cast<uint64_t *>(a.index)[ir] = v;
                else reinterpret_cast<uint32_t *>(a.index)[ir] = (uint32_t)v;
              } else {
                raise_error(a.err, E_CAPACITY, x);
              }
            }
          }
          cnt.c[C_INDEX]++;
        } else if (role == 2) {
          if (MODE == 2) {
            const uint64_t vr = base.c[C_VALUE] + cnt.c[C_VALUE];
            bool nan_err = false;
            uint64_t e;
            float v = parse_float(t.src, x, &e, &nan_err);
            if (nan_err) raise_error(a.err, E_NAN_LITERAL, x);
            if (vr < a.cap[C_VALUE]) a.value[vr] = v;
            else raise_error(a.err, E_CAPACITY, x);
          }
          cnt.c[C_VALUE]++;
        }
      }
    }
    if (MODE != 0 && ((sg.le >> i) & 1u) && st == S_F) {
      // "idx:" dangling at the line end: ParsePair decodes the value at lend
      if (gap_fnb(t.src, x + 1, cfloor) == ':') {
        if (MODE == 2) {
          const uint64_t vr = base.c[C_VALUE] + cnt.c[C_VALUE];
          bool nan_err = false;
          uint64_t e;
          float v = parse_float(t.src, x + 1, &e, &nan_err);
          if (nan_err) raise_error(a.err, E_NAN_LITERAL, x);
          if (vr < a.cap[C_VALUE]) a.value[vr] = v;
          else raise_error(a.err, E_CAPACITY, x);
        }
        cnt.c[C_VALUE]++;
      }
    }
  }
}

__device__ __forceinline__ bool is_cs(const uint64_t *cs, int nchunk, uint64_t p) {
  int c = chunk_of(cs, nchunk, p);
  return cs[c] == p;
}

// Scan [from, from+kWin) of global memory for the first line start; returns
// kNone if none (block-uniform).
__device__ uint64_t first_line_start(const LibsvmArgs &a, uint64_t from, uint64_t to, uint64_t *scratch) {
  for (uint64_t base = from; base < to; base += kWin) {
    uint64_t best = kNone;
    const uint64_t lo = base + (uint64_t)threadIdx.x * kSeg;
    const uint64_t hi = min(lo + kSeg, to);
    for (uint64_t p = lo; p < hi; ++p) {
      if (is_nl(a.text[p])) {
        best = p;
        break;
      }
    }
    // chunk starts in [lo, hi)
    if (lo < hi) {
      int c = chunk_of(a.cs, a.nchunk, lo);
      uint64_t s = a.cs[c] == lo ? lo : a.cs[c + 1];
      if (s < hi && s < best) best = s;
    }
    best = block_min(best, scratch);
    if (best != kNone) return best;
  }
  return kNone;
}

template <int MODE>  // 1 = count pass, 2 = write pass
__global__ void __launch_bounds__(kThreads) libsvm_tile(LibsvmArgs a) {
  __shared__ __attribute__((aligned(16))) uint8_t win[kWin + 32];
  __shared__ uint32_t r1bits[kWin / 32 + 1];
  __shared__ uint32_t sfn[kWaves + 1];
  __shared__ Cnt scnt[kWaves + 1];
  __shared__ uint64_t s64[kWaves + 1];
  __shared__ uint64_t pending[2];  // R1 of a line whose head crossed a window, by window parity

  const uint64_t k = blockIdx.x;
  const uint64_t tlo = k * a.tile_bytes;
  if (tlo >= a.n) return;
  const uint64_t thi = min(tlo + a.tile_bytes, a.n);
  const int tid = threadIdx.x;

  Cnt zero;
#pragma unroll
  for (int i = 0; i < 8; ++i) zero.c[i] = 0;
  Cnt tot = zero;   // totals of this tile's previous windows (block-uniform)
  Cnt mine = zero;  // count pass: this thread's totals over all windows
  Base64 tbase;
#pragma unroll
  for (int i = 0; i < C_N; ++i) tbase.c[i] = MODE == 2 ? a.tile_base[k * C_N + i] : 0;

  uint64_t w0 = first_line_start(a, tlo, a.n, s64);
  if (w0 == kNone || w0 >= thi) {
    if (MODE == 1 && tid < C_N) a.tile_cnt[k * C_N + tid] = 0;
    return;
  }
  if (tid == 0) pending[1] = kNone;
  int j = 0;  // window counter
  uint32_t st0 = S_PRE;  // concrete role state at the window start
  bool done = false;
  Tile t;
  t.a = &a;
  t.r1bits = r1bits;
  t.src.g = a.text;
  t.src.lds = win;
  while (!done) {
    const uint64_t pend = pending[(j + 1) & 1];  // written during window j-1
    uint64_t wend = min(w0 + (uint64_t)kWin, a.n);
    if (wend == a.n) done = true;
    if (wend > thi) {
      const uint64_t e = first_line_start(a, max(w0, thi), wend, s64);
      if (e != kNone) {
        wend = e;
        done = true;
      }
    }
    if (wend == w0) break;
    // a pending R1 beyond this window means its line spans the whole window
    if (tid == 0) pending[j & 1] = (pend != kNone && pend >= wend) ? pend : kNone;
    // stage [abase, wend) into LDS (16-byte aligned base)
    const uint64_t abase = w0 & ~15ull;
    const uint64_t nunits = (wend - abase + 15) >> 4;
    for (uint64_t u = tid; u < nunits; u += kThreads) {
      const uint64_t g = abase + (u << 4);
      if (g + 16 <= a.n) {
        *reinterpret_cast<uint4 *>(&win[u << 4]) = *reinterpret_cast<const uint4 *>(a.text + g);
      } else {
        for (int j = 0; j < 16; ++j) win[(u << 4) + j] = g + j < a.n ? a.text[g + j] : 0;
      }
    }
    for (int i = tid; i < kWin / 32 + 1; i += kThreads) r1bits[i] = 0;
    __syncthreads();
    t.src.wbase = abase;
    t.src.wend = min(abase + (nunits << 4), a.n);
    t.w0 = w0;
    if (tid == 0 && pend != kNone && pend < wend)
      atomicOr(&r1bits[(pend - w0) >> 5], 1u << ((pend - w0) & 31));

    // ---- this thread's segment masks
    Seg sg;
    sg.lo = w0 + (uint64_t)tid * kSeg;
    sg.hi = min(sg.lo + kSeg, wend);
    sg.rs = sg.ls = sg.le = 0;
    sg.chunk = 0;
    if (sg.lo < sg.hi) {
      sg.chunk = chunk_of(a.cs, a.nchunk, sg.lo);
      t.src.lim = a.cs[sg.chunk + 1];
      uint32_t dm = 0, nl = 0, csm = 0;
      const int len = (int)(sg.hi - sg.lo);
      for (int i = 0; i < len; ++i) {
        const uint32_t c = win[sg.lo + i - abase];
        dm |= (uint32_t)is_digitchar(c) << i;
        nl |= (uint32_t)is_nl(c) << i;
      }
      for (int c = sg.chunk; c < a.nchunk && a.cs[c] < sg.hi; ++c)
        if (a.cs[c] >= sg.lo) csm |= 1u << (a.cs[c] - sg.lo);
      const uint32_t prev =
          (sg.lo > 0 && !(csm & 1u) && is_digitchar(t.src(sg.lo - 1))) ? 1u : 0u;
      sg.rs = (dm & ~((dm << 1) | prev)) | (csm & dm);
      sg.ls = nl | csm;
      bool nxt = sg.hi == a.n;  // is position hi a line start (or the end of data)?
      if (!nxt) {
        const uint64_t h = sg.hi;
        nxt = is_nl(h < t.src.wend ? win[h - abase] : a.text[h]) || is_cs(a.cs, a.nchunk, h);
      }
      sg.le = (sg.ls >> 1) | ((uint32_t)nxt << (len - 1));
    }

    // ---- phase B: head sections -> R1 marks
    if (sg.ls) {
      uint32_t m = sg.ls;
      int chunk = sg.chunk;
      while (m) {
        const int i = __builtin_ctz(m);
        m &= m - 1;
        const uint64_t x = sg.lo + i;
        while (x >= a.cs[chunk + 1]) ++chunk;
        t.src.lim = a.cs[chunk + 1];
        const Head h = head_parse(t.src, x, x == a.cs[chunk], a.cs[chunk + 1]);
        if (h.r1 != kNone) {
          if (h.r1 < wend) atomicOr(&r1bits[(h.r1 - w0) >> 5], 1u << ((h.r1 - w0) & 31));
          else pending[j & 1] = h.r1;  // only the last line of the window can get here
        }
      }
    }
    __syncthreads();

    // ---- role-machine transition function of my segment, then block scan
    uint32_t fn = kIdentityFn;
    Cnt dummy = zero;
    Base64 nob;
    if (sg.lo < sg.hi) walk<0>(t, sg, fn, dummy, nob);
    uint32_t fn_total;
    const uint32_t fn_ex = block_exclusive(fn, kIdentityFn, FnCompose(), sfn, &fn_total);
    const uint32_t st = (fn_ex >> (2 * st0)) & 3u;
    const uint32_t st_next = (fn_total >> (2 * st0)) & 3u;

    // ---- count walk
    Cnt c = zero;
    if (sg.lo < sg.hi) {
      uint32_t s2 = st;
      walk<1>(t, sg, s2, c, nob);
    }
    if (MODE == 1) {
      mine = CntAdd()(mine, c);
    } else {
      Cnt wtot;
      const Cnt ex = block_exclusive(c, zero, CntAdd(), scnt, &wtot);
      if (sg.lo < sg.hi) {
        Base64 b;
#pragma unroll
        for (int i = 0; i < C_N; ++i) b.c[i] = tbase.c[i] + tot.c[i] + ex.c[i];
        Cnt local = zero;
        uint32_t s3 = st;
        walk<2>(t, sg, s3, local, b);
      }
      tot = CntAdd()(tot, wtot);
    }
    st0 = st_next;
    w0 = wend;
    ++j;
    __syncthreads();
  }
  if (MODE == 1) {
    Cnt total;
    (void)block_exclusive(mine, zero, CntAdd(), scnt, &total);
    if (tid < C_N) a.tile_cnt[k * C_N + tid] = total.c[tid];
  }
}

__global__ void finalize_kernel(uint64_t *res) {
  if (res[8] == ~0ull) res[8] = 0;  // no error raised
}

}  // namespace

hipError_t launch_libsvm(const LibsvmArgs &a, uint64_t *res, bool count_only, hipStream_t s) {
  hipError_t e;
  if ((e = hipMemsetAsync(res, 0, 16 * sizeof(uint64_t), s)) != hipSuccess) return e;
  if ((e = hipMemsetAsync(res + 8, 0xFF, sizeof(uint64_t), s)) != hipSuccess) return e;
  if (a.indexing_mode < 0 &&
      (e = hipMemsetAsync(a.chunk_min, 0xFF, (size_t)a.nchunk * sizeof(uint64_t), s)) != hipSuccess)
    return e;
  if (!a.ntiles && !count_only && a.offset && (e = hipMemsetAsync(a.offset, 0, 8, s)) != hipSuccess)
    return e;  // empty input: offset = {0}
  if (a.ntiles) {
    libsvm_tile<1><<<a.ntiles, kThreads, 0, s>>>(a);
    tile_scan_kernel<<<1, kThreads, 0, s>>>(a.tile_cnt, const_cast<uint64_t *>(a.tile_base), a.ntiles,
                                            res, count_only ? nullptr : a.offset, a.cap[C_ROWS]);
    if (!count_only) libsvm_tile<2><<<a.ntiles, kThreads, 0, s>>>(a);
  }
  finalize_kernel<<<1, 1, 0, s>>>(res);
  return hipGetLastError();
}

}  // namespace dmlc_amd
