// svm_lean.h -- the lean single-pass libsvm tile: LibSVMParser::ParseBlock
// (src/data/libsvm_parser.h:85-172, ParsePair include/dmlc/strtonum.h:667-703)
// for the text every libsvm writer produces -- label[:weight] and
// index[:value] runs of digitchars separated by blanks and newlines -- with
// nothing else in the kernel: no comment pass, no qid, no per-line walk, no
// run lists.  It runs first; a tile holding anything else (a byte outside
// {digitchars, ':', blanks, newlines}, a dangling ':', an "a:b:c" chain, a
// carry it cannot see) POISONS: it publishes a poison status instead of its
// counts, every later tile's look-back stops there and exits, and the full
// single-pass kernel (svm_fast.h) resumes at the first poisoned tile with its
// look-back seeded by this kernel's inclusive prefix.  The output is the
// reference's either way; what the split buys is a kernel small enough for
// 8 workgroups per CU.
//
// Per tile (16 KiB, 256 threads, 64 bytes per thread; the full kernel's
// tile numbering, which the resume depends on):
//   * each thread loads its own 64 bytes into registers and classifies them
//     through the byte-class table (fast_common.h class_of), planes D / N / C
//     in registers; the text also goes to LDS for the decoders' windows;
//   * the carry-in of a segment is the previous segment's planes: lane t-1's
//     by a shuffle, and for lane 0 of each wave the 64 bytes before the wave
//     read lane = byte from global memory and turned into planes by ballots
//     (no barrier between classification and roles);
//   * roles by the carry arithmetic of svm_fast.h segment_roles;
//   * one block scan (one barrier) of the packed counts, the poison flag with it;
//   * wave run lists: each wave's index and value runs in rank order in
//     LDS (no block barrier), decoded round-robin by its lanes into
//     registers before the look-back (the look-back's polls find the
//     predecessors published), stored after it by consecutive lanes;
//   * decoupled look-back by wave 0 (fast_common.h scheme, plus the poison
//     state), one barrier, stores.
// Written against the block policy BK so the GPU kernel (libsvm.hip) and the
// test-only CPU emulator (tests/emu) share it.
#pragma once
#include "fast_common.h"
#include "svm_fast.h"

namespace dmlc_amd {
namespace lsvm {
using namespace fast;
using fsvm::R_I;
using fsvm::R_K;
using fsvm::R_L;
using fsvm::R_NONE;

constexpr int kLPost = 64;               // staged bytes after the tile (decoder windows of its last runs)
constexpr int kLStage = kTile + kLPost;  // the tile's text in LDS: position p <-> text[p - tlo]
constexpr uint64_t kSPoison = 3ull << 62;
#ifndef LSVM_LCAP
#define LSVM_LCAP 256
#endif
constexpr uint32_t kLCap = LSVM_LCAP;          // list entries per kind per wave
constexpr int kRounds = (int)kLCap / kWave;    // decode rounds per kind
static_assert(kLCap % kWave == 0, "whole rounds");

struct Shared {
  alignas(16) uint8_t text[kLStage];
  uint32_t cls[kClsEntries];  // byte classes (fast_common.h class_of)
  DecTables dt;
  uint64_t g0[kFWaves + 1];  // digit plane of each wave's first segment; [kFWaves]: the 32 bytes after the tile
  // wave run lists: index runs, value runs; an entry is the run's tile offset
  // (bits 0-13), bit 15: the owner's (a unit end within its window), bits
  // 16-31: its window's non-digit flags -- decoded in place into the value
  uint32_t lst[kFWaves][2][kLCap];
  uint64_t fail[kFWaves][2][kRounds];  // list entries the decoding lane left to the owner
  uint64_t wtot[kFWaves];  // packed counts of each wave (block scan)
  uint64_t base[4];        // output bases from the look-back
  uint32_t wbad[kFWaves];  // a segment of the wave poisons the tile
  uint32_t flags;          // bit 0: a tile before this one already poisoned; bit 1: the look-back met a poison
};

// ---- unit starts (ParseBlock units) around a wave's bytes.  Lane i holds
// v = cs[c0 + i] where c0 is the last unit whose start is <= lo; a 64-ary
// search finds it (fast_common.h chunk_list_begin, per wave).  Entries past
// cs[nchunk] read as ~0.
struct Units {
  uint64_t c0;  // unit index of lane 0's entry
  uint64_t v;   // this lane's entry, cs[c0 + lane] (~0 past cs[nchunk])
  uint32_t jf;  // the lane holding the last start <= lo (the floor)
};
// hi: the window must reach past it (else one more load re-centres it on the floor)
template <class BK>
DA_HDF Units units_around(const uint64_t *cs, int nchunk, uint64_t lo, uint64_t hi, uint32_t lane, BK &bk) {
  const uint64_t kBig = ~0ull;
  uint64_t c = 0, cnt = (uint64_t)nchunk;
  while (cnt > (uint64_t)kWave) {  // wave-uniform
    const uint64_t S = (cnt + kWave - 1) / kWave;
    const uint64_t v = (uint64_t)lane * S < cnt ? cs[c + (uint64_t)lane * S] : kBig;
    const uint64_t m = bk.ballot(v <= lo);  // lane 0 always holds (cs[c] <= lo)
    const uint64_t j = (uint64_t)(63 - clz64(m));
    const uint64_t nc = c + j * S;
    cnt = mn<uint64_t>(S, c + cnt - nc);
    c = nc;
  }
  uint64_t v = c + lane <= (uint64_t)nchunk ? cs[c + lane] : kBig;
  uint64_t m = bk.ballot(v <= lo && c + lane < (uint64_t)nchunk);
  uint32_t j = (uint32_t)(63 - clz64(m | 1u));
  if (j && !bk.ballot(v > hi)) {  // the window ends before hi: re-centre it on the floor
    c += j;
    v = c + lane <= (uint64_t)nchunk ? cs[c + lane] : kBig;
    j = 0;
  }
  Units u;
  u.c0 = c;
  u.v = v;
  u.jf = j;
  return u;
}

// ---- carry-in at a segment start P from the planes of W = [P-64, P) (bit
// i <-> P-64+i) and the bit fb of the segment's unit start F in W (-1: F
// lies before W).  The state svm_fast.h segment_roles needs: dc (byte P-1 is
// a digitchar of the unit), ginl / ginc (the gap open at P holds a newline /
// the unit start, or a ':' after its last newline), prole (the role of the
// last run starting before P).  False when W does not decide it (a run or a
// gap longer than W with no newline): the tile poisons.
DA_HD bool lean_carry(uint64_t d1, uint64_t n1, uint64_t c1, int fb, uint32_t *dc, uint32_t *ginl, uint32_t *ginc,
                      uint32_t *prole) {
  const uint64_t unit = fb >= 0 ? (~0ull << fb) : ~0ull;  // W's bytes in P's unit
  const uint64_t d = d1 & unit;
  // role of the run starting at bit q (the unit's first run: a label)
  auto role_at = [&](int q, uint32_t *r) -> bool {
    if (q == fb) {
      *r = R_L;
      return true;
    }
    const uint64_t lowq = q > 0 ? (~0ull >> (64 - q)) : 0ull;  // bits below q
    const uint64_t below = d & lowq;
    if (!below) {  // the gap reaches the unit start, or the start of W
      if (fb >= 0 || (n1 & lowq)) {
        *r = R_L;
        return true;
      }
      return false;
    }
    const int p2 = 63 - clz64(below);
    const uint64_t gm = lowq & ~(~0ull >> (63 - p2));  // bits p2+1 .. q-1
    *r = (n1 & gm) ? R_L : ((c1 & gm) ? R_K : R_I);
    return true;
  };
  *ginl = *ginc = 0;
  *prole = R_NONE;
  if ((d >> 63) & 1u) {  // the run at P-1 goes on into the segment
    *dc = 1;
    const uint64_t nd = ~d;
    if (!nd) {
      if (fb == 0) {
        *prole = R_L;
        return true;
      }
      return false;
    }
    return role_at(64 - clz64(nd), prole);
  }
  *dc = 0;
  if (!d) {  // no digitchar of the unit in W
    if (fb >= 0) {
      *ginl = 1;
      return true;
    }
    if (!n1) return false;
    *ginl = 1;
    const int ln = 63 - clz64(n1);
    *ginc = ln < 63 && (c1 >> (ln + 1)) != 0;
    return true;
  }
  const int pb = 63 - clz64(d);  // last digitchar, <= 62
  const uint64_t tg = ~0ull << (pb + 1);
  const uint64_t tgn = n1 & tg;
  if (tgn) {  // a newline after the last run: the next run is a label whatever came before
    *ginl = 1;
    const int ln = 63 - clz64(tgn);
    *ginc = ln < 63 && (c1 >> (ln + 1)) != 0;
    return true;
  }
  *ginc = (c1 & tg) != 0;
  const uint64_t nd = ~d & (pb > 0 ? (~0ull >> (64 - pb)) : 0ull);  // non-digitchars below pb
  if (!nd) {
    if (fb == 0) {
      *prole = R_L;
      return true;
    }
    return false;
  }
  return role_at(64 - clz64(nd), prole);
}

struct LeanRoles {
  uint64_t L, W, I, V;
  uint32_t bad;
};
// Roles of segment P's runs (svm_fast.h segment_roles without qid tokens).
// S: unit starts in the segment; nxt_cs: whether P + 64 starts a unit.
DA_HD LeanRoles lean_roles(uint64_t D, uint64_t N, uint64_t C, uint64_t S, uint64_t valid, bool at_end,
                           uint32_t dc, uint32_t ginl, uint32_t ginc, uint32_t prole) {
  LeanRoles o;
  o.bad = 0;
  const uint64_t RS = (D & ~((D << 1) | dc)) | (D & S);
  const uint64_t G = ~D & valid;
  const uint64_t NS = N | S;
  uint32_t co;
  const uint64_t t1 = add_carry(G, NS & G, ginl, &co);
  const uint64_t L = RS & (t1 | S);
  const uint64_t G2 = G & ~NS;
  const uint64_t t2 = add_carry(G2, C & G2, ginc, &co);
  // a ':' gap that ends at a newline, a unit start or the end of the text:
  // ParsePair decodes past the line end there (strtonum.h:684-692)
  if (t2 & (NS | ~valid)) o.bad = 1;
  if (co && at_end) o.bad = 1;
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

// Masks of 64 bytes held as 16 little-endian words, through the class table
// (fast_common.h classify64_lut's form).
// (The table reads go in groups of 16, fenced from the scheduler: left
// alone it hoists all 64 reads and their addresses, 128 VGPRs.)
DA_HD Masks classify_regs(const uint32_t w[16], const uint32_t *cls) {
  uint32_t acc[8];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int i = 4 * j + b;
      const uint32_t x = cls[(w[j] >> (8 * b)) & 0xFFu];
      if ((i & 7) == 0) acc[i >> 3] = x;
      else acc[i >> 3] |= x << (i & 7);
    }
#if defined(__HIP_DEVICE_COMPILE__)
    if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);
#endif
  }
  uint32_t pd[2], pg[2], pn[2], pc[2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const uint32_t t = perm_b32(acc[4 * h + 1], acc[4 * h], 0x05010400u);
    const uint32_t u = perm_b32(acc[4 * h + 3], acc[4 * h + 2], 0x05010400u);
    pd[h] = perm_b32(u, t, 0x05040100u);
    pg[h] = perm_b32(u, t, 0x07060302u);
    const uint32_t t2 = perm_b32(acc[4 * h + 1], acc[4 * h], 0x07030602u);
    const uint32_t u2 = perm_b32(acc[4 * h + 3], acc[4 * h + 2], 0x07030602u);
    pn[h] = perm_b32(u2, t2, 0x05040100u);
    pc[h] = perm_b32(u2, t2, 0x07060302u);
  }
  Masks m;
  m.d = pd[0] | ((uint64_t)pd[1] << 32);
  m.n = pn[0] | ((uint64_t)pn[1] << 32);
  m.c = pc[0] | ((uint64_t)pc[1] << 32);
  m.g = pg[0] | ((uint64_t)pg[1] << 32);
  m.hi = 0u;
  // outside the lean grammar: a byte the table marks G without D, or the
  // letters of "qid:" (N and C together)
  m.bad = ((m.g & ~m.d) | (m.n & m.c)) != 0;
  return m;
}

// the 16 staged bytes at tile offset o as four words
DA_HD void win16(const uint8_t *text, uint32_t o, uint32_t w[4]) {
  const uint32_t *p = reinterpret_cast<const uint32_t *>(text + (o & ~3u));
  const uint32_t sft = (o & 3u) * 8u;
  const uint32_t x0 = p[0], x1 = p[1], x2 = p[2], x3 = p[3], x4 = p[4];
  w[0] = funnel(x1, x0, sft);
  w[1] = funnel(x2, x1, sft);
  w[2] = funnel(x3, x2, sft);
  w[3] = funnel(x4, x3, sft);
}

// Lean look-back (wave 0): fast_common.h look_back with a poison state.  A
// round consumes predecessors up to the nearest inclusive one; an
// unpublished one ends the round, a poisoned one the tile.  Returns false
// when a poisoned predecessor was met (the tile then stores nothing).
template <class BK>
DA_HDF bool lean_look_back(uint64_t *lb, uint32_t ntiles, uint32_t k, const uint32_t cnt[4], uint32_t *gate,
                           uint64_t *base, BK &bk) {
  const uint32_t lane = (uint32_t)bk.tid() & (kWave - 1);
  uint64_t *st = lb, *incl = lb + ntiles;
  uint64_t j = k;
  uint32_t spins = 0;
  uint64_t acc[4] = {0, 0, 0, 0};
  bool done = k == 0, ok = true;
  while (!done) {
    uint64_t s = 0, w[4] = {kMark, kMark, kMark, kMark};  // before tile 0: an inclusive 0
    if (lane < j) {
      const uint64_t p = j - 1 - lane;
      s = load_agent_u64(st + p);
#pragma unroll
      for (int f = 0; f < 4; ++f) w[f] = load_agent_u64(incl + p * 4 + f);
    }
    const bool inc = (w[0] & w[1] & w[2] & w[3] & kMark) != 0;
    const uint64_t mi = bk.ballot(inc), mz = bk.ballot(!inc && (s >> 62) == 0);
    const uint64_t mp = bk.ballot(!inc && (s >> 62) == 3);
    uint64_t D = kWave;
    uint32_t stop = 0;  // 1 inclusive, 2 poison
    if (mz | mi | mp) {
      D = (uint64_t)ctz64(mz | mi | mp);
      stop = ((mi >> D) & 1u) ? 1u : (((mp >> D) & 1u) ? 2u : 0u);
    }
    uint32_t part[4] = {0, 0, 0, 0};
    if (lane < D) {
#pragma unroll
      for (int f = 0; f < 4; ++f) part[f] = (uint32_t)((s >> (15 * f)) & 0x7FFFu);
    }
#pragma unroll
    for (int f = 0; f < 4; ++f) acc[f] += bk.wave_sum(part[f]);
    if (stop == 2) {
      done = true;
      ok = false;
    } else if (stop == 1) {
      done = true;
#pragma unroll
      for (int f = 0; f < 4; ++f) acc[f] += bk.shfl(w[f] & ~kMark, (int)D);
    } else {
      j -= D;
      if (D == 0) {
        if (++spins > kSpinLimit) {  // never expected: hand the input to the exact path
          if (lane == 0) atomic_or_u32(gate, 2u);
          done = true;
          ok = false;
        }
        spin_pause();
      }
    }
  }
  if (ok && lane < 4) {
    const uint64_t v = acc[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3];
    base[lane] = v;
    if (k > 0) store_agent_u64(incl + (uint64_t)k * 4 + lane, kMark | (v + cnt[lane == 0 ? 0 : lane == 1 ? 1 : lane == 2 ? 2 : 3]));
  }
  return ok;
}

// The tile.  a.lean_lb: this kernel's look-back words; a.lean_poison: ~ the
// first poisoned tile (0: none), which the full kernel resumes at.
template <class BK>
DA_HDF void tile(const FastSvmArgs &a, Shared &sh, BK &bk, uint32_t k) {
  const int tid = bk.tid();
  const uint32_t lane = (uint32_t)tid & (kWave - 1), wid = (uint32_t)tid / kWave;
  const uint64_t n = a.n;
  const uint64_t tlo = (uint64_t)k * kTile;
  const uint64_t thi = mn<uint64_t>(tlo + kTile, n);
  const uint64_t P = tlo + (uint64_t)tid * kSegB;
  const uint64_t P0 = tlo + (uint64_t)wid * kWave * kSegB;  // the wave's first segment
  FAST_STAMP(k, 0);
  FAST_STAMP(k, 1);
  // ---- loads: my 64 bytes, the 64 bytes before my wave (lane = byte), the
  // post-halo (the last wave's lanes 60-63)
  // (a segment or post-halo piece reaching past the text end -- the last
  // tile only -- is staged byte by byte straight into LDS, blanks past n,
  // and read back: a compact loop off the register budget)
  uint32_t w[16];
  const bool wfull = P + kSegB <= n;
  if (wfull) {
#pragma unroll
    for (int q = 0; q < 4; ++q) load16(a.text + P + 16 * q, w + 4 * q);
  } else {
    uint8_t *dst = sh.text + (uint64_t)tid * kSegB;
#pragma unroll 1
    for (int i = 0; i < kSegB; ++i) dst[i] = P + i < n ? a.text[P + i] : (uint8_t)' ';
#pragma unroll
    for (int q = 0; q < 4; ++q) load16(dst + 16 * q, w + 4 * q);
  }
  const uint32_t prevb =
      P0 >= (uint64_t)kSegB && P0 - kSegB + lane < n ? (uint32_t)a.text[P0 - kSegB + lane] : (uint32_t)' ';
  uint32_t post[4] = {0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u};
  const int pl = tid - (kFThreads - kLPost / 16);  // post-halo lane 0..3
  bool pfull = false;
  if (pl >= 0) {
    const uint64_t g = tlo + kTile + 16 * (uint64_t)pl;
    pfull = g + 16 <= n;
    if (pfull) {
      load16(a.text + g, post);
    } else {
      uint8_t *dst = sh.text + kTile + 16 * pl;
#pragma unroll 1
      for (int i = 0; i < 16; ++i) dst[i] = g + i < n ? a.text[g + i] : (uint8_t)' ';
    }
  }
  // unit starts around the wave: the floor of P0 - 64 and every start up to
  // the wave's end + 80 (unit tests of P + 64, decode limits)
  const uint64_t ulo = P0 >= (uint64_t)kSegB ? P0 - kSegB : 0;
  const uint64_t whi = P0 + (uint64_t)kWave * kSegB + 80;
  const Units un = units_around(a.cs, a.nchunk, ulo, whi, lane, bk);
  // ---- tables, the poison word, barrier
  for (int i = tid; i < kClsEntries; i += kFThreads) sh.cls[i] = class_of((uint32_t)i);
  init_dec_tables(sh.dt, bk);
  // (the word holds ~ the first poisoned tile, 0: none; read past the
  // scalar and vector L1s, which another CU's atomic does not update)
  if (tid == 0) sh.flags = ~load_agent_u64(a.lean_poison) < (uint64_t)k ? 1u : 0u;
  bk.sync();
  FAST_STAMP(k, 2);
  if (sh.flags & 1u) {  // a tile before this one poisoned: the full kernel takes it from there
    if (tid == 0) store_agent_u64(a.lean_lb + k, kSPoison);  // (a look-back of a later tile must not wait for this one)
    return;
  }
  // text into LDS for the decoders' windows (my 64 bytes, the post-halo)
  if (wfull) {
    uint32_t *dst = reinterpret_cast<uint32_t *>(sh.text + (uint64_t)tid * kSegB);
#pragma unroll
    for (int q = 0; q < 16; ++q) dst[q] = w[q];
  }
  if (pfull) {
    uint32_t *pd = reinterpret_cast<uint32_t *>(sh.text + kTile + 16 * pl);
#pragma unroll
    for (int q = 0; q < 4; ++q) pd[q] = post[q];
  }
  // ---- classify my segment; the wave's carry segment by ballots
  const Masks m = classify_regs(w, sh.cls);
  uint32_t bad = P < n ? m.bad : 0u;
  if (lane == 0) sh.g0[wid] = m.g;  // (read after the scan barrier: the windows of the wave before)
  if (pl >= 0 && pl < 2) {  // digits of the first 32 bytes after the tile (windows of the last runs)
    const uint8_t *pp = sh.text + kTile + 16 * pl;
    uint32_t g = 0;
    for (int i = 0; i < 16; ++i) g |= (uint32_t)is_digit(pp[i]) << i;
    reinterpret_cast<uint16_t *>(&sh.g0[kFWaves])[pl] = (uint16_t)g;
    if (pl == 0) reinterpret_cast<uint32_t *>(&sh.g0[kFWaves])[1] = 0u;
  }
  const uint64_t gnx = bk.shfl(m.g, (int)((lane + 1) & (kWave - 1)));  // the next segment's (lane 63: below)
  uint64_t pd1, pn1, pc1;  // planes of the 64 bytes before the wave
  {
    const uint32_t x = sh.cls[prevb & 0xFFu];
    pd1 = bk.ballot((x & 1u) != 0);
    pn1 = bk.ballot(((x >> 16) & 1u) != 0);
    pc1 = bk.ballot(((x >> 24) & 1u) != 0);
  }
  // (every lane shuffles; lane 0 then takes the wave's carry segment)
  const uint64_t sd = bk.shfl_up(m.d, 1), sn = bk.shfl_up(m.n, 1), sc = bk.shfl_up(m.c, 1);
  const uint64_t d1 = lane == 0 ? pd1 : sd, n1 = lane == 0 ? pn1 : sn, c1 = lane == 0 ? pc1 : sc;
  // ---- my unit starts: the entries of the wave's window near my segment
  const int nv = P < n ? (int)mn<uint64_t>(64, n - P) : 0;
  const uint64_t valid = nv == 64 ? ~0ull : ((1ull << nv) - 1);
  uint64_t S = 0, F = bk.shfl(un.v, (int)un.jf), nxt;  // F: the last unit start <= P
  bool at_end = P + kSegB >= n;
  // the unit starts after the floor up to whi (usually none); the window
  // must reach past whi (else more than 63 unit starts lie here: poison)
  const uint64_t mw = bk.ballot(lane > un.jf && un.c0 + lane < (uint64_t)a.nchunk && un.v <= whi);
  {
    const uint64_t mb = bk.ballot(un.v > whi);
    if (!mb) bad = 1;
    nxt = mb ? bk.shfl(un.v, ctz64(mb)) : ~0ull;
    for (uint64_t mm = mw; mm; mm &= mm - 1) {  // wave-uniform
      const uint64_t x = bk.shfl(un.v, ctz64(mm));
      if (x <= P) F = x;
      if (x >= P + (uint64_t)nv && x < nxt) nxt = x;  // the first start after my segment (in it: S)
      if (x >= P && x < P + (uint64_t)nv) S |= 1ull << (x - P);
      if (x == P + kSegB) at_end = true;
    }
  }
  if (F == P) S |= 1u;  // a unit starts at my segment (the text start among them)
  if (P >= n) S = 0;
  // ---- carry-in and roles
  uint32_t dc = 0, ginl = 0, ginc = 0, prole = R_NONE;
  if (P < n && P != F) {
    const int fb = F + kSegB >= P ? (int)(F + kSegB - P) : -1;
    if (!lean_carry(d1, n1, c1, fb, &dc, &ginl, &ginc, &prole)) bad = 1;
  }
  LeanRoles ro;
  ro.L = ro.W = ro.I = ro.V = 0;
  ro.bad = 0;
  if (P < n) ro = lean_roles(m.d & valid, m.n & valid, m.c & valid, S, valid, at_end, dc, ginl, ginc, prole);
  bad |= ro.bad;
  FAST_STAMP(k, 3);
  // ---- block scan of the packed role counts (one barrier), poison flag with it
  const uint64_t mine = (uint64_t)popc64(ro.L) | ((uint64_t)popc64(ro.W) << 16) | ((uint64_t)popc64(ro.I) << 32) |
                        ((uint64_t)popc64(ro.V) << 48);
  uint64_t totp;
  uint64_t wpre;  // the wave's first segment's exclusive counts
  const uint64_t ex = bk.exclusive_add1(mine, bad != 0, sh.wtot, sh.wbad, &totp, &wpre);
  bool tile_bad = false;
  for (int q = 0; q < kFWaves; ++q) tile_bad |= sh.wbad[q] != 0;
  const uint32_t nL = (uint32_t)(totp & 0xFFFF), nW = (uint32_t)((totp >> 16) & 0xFFFF),
                 nI = (uint32_t)((totp >> 32) & 0xFFFF), nV = (uint32_t)(totp >> 48);
  if (tile_bad) {  // block-uniform
    if (tid == 0) {
      store_agent_u64(a.lean_lb + k, kSPoison);
      atomic_max_u64(reinterpret_cast<unsigned long long *>(a.lean_poison), ~(unsigned long long)k);
    }
    return;
  }
  const uint32_t cnt4[4] = {nL, nI, nV, nW};  // look-back slots fsvm Q_ROWS, Q_INDEX, Q_VALUE, Q_WEIGHT
  if (tid == 0) publish_aggregate(a.lean_lb, a.ntiles, k, cnt4);
  FAST_STAMP(k, 4);
#if defined(LSVM_ABL) && LSVM_ABL == 1  // timing ablation only: stage + classify + roles + scan
  if (ex == 0x123456789ull) a.res[15] = totp;
  return;
#endif
  // ---- wave run lists: the wave's first kLCap index runs and value runs in
  // wave rank order, decoded round-robin by the wave's lanes -- every lane
  // decodes about the wave's average, where each lane decoding its own runs
  // runs the wave for its fullest lane -- in place, before the look-back (its
  // polls then find the predecessors published).  The owner of a run keeps
  // what the lists do not take: ranks past kLCap, windows the decoders
  // refuse (the decoding lane marks them in the wave's failure words), runs
  // whose window reaches a unit end (their limit is the owner's).
  const uint32_t o0 = (uint32_t)tid * kSegB;
  const uint64_t lim_seg = nxt < n ? nxt : n;  // decode limit of runs after my last unit start
  // the limit of the run at bit b: the next unit start after it
  auto lim_of = [&](uint32_t b) -> uint64_t {
    const uint64_t above = S & (b >= 63 ? 0ull : (~0ull << (b + 1)));
    return above ? P + ctz64(above) : lim_seg;
  };
  // digit plane of the segment after mine (the next wave's first, or the bytes after the tile)
  const uint64_t gn = lane == kWave - 1 ? sh.g0[wid + 1] : gnx;
  // non-digit flags of the 16 window bytes at my bit b
  auto ndig_of = [&](uint32_t b) -> uint32_t {
    const uint64_t g = b ? (m.g >> b) | (gn << (64 - b)) : m.g;
    return ~(uint32_t)g & 0xFFFFu;
  };
  auto dec_float = [&](uint32_t o, uint32_t nd, bool *ok) -> float {
    uint32_t wq[4];
    win16(sh.text, o, wq);
    return wfloat32m(wq, nd, sh.dt, ok);
  };
  auto dec_index = [&](uint32_t o, uint32_t nd, bool *ok) -> uint32_t {
    uint32_t wq[4];
    win16(sh.text, o, wq);
    uint64_t v;
    bool k1;
    const bool pos = wuint32m(wq, nd, sh.dt, &v, &k1);
    *ok = k1 && pos;
    return (uint32_t)v;
  };
  const uint64_t wt = sh.wtot[wid];  // the wave's totals (packed)
  const uint64_t wex = ex - wpre;    // my wave-local exclusive counts
  const uint32_t wexI = (uint32_t)((wex >> 32) & 0xFFFF), wexV = (uint32_t)(wex >> 48);
  const uint32_t nIq = mn<uint32_t>((uint32_t)((wt >> 32) & 0xFFFF), kLCap), nVq = mn<uint32_t>((uint32_t)(wt >> 48), kLCap);
  uint32_t *li = sh.lst[wid][0], *lv = sh.lst[wid][1];
  {
    auto entry = [&](uint32_t b) -> uint32_t {
      return (o0 + b) | (P + b + 16 > lim_of(b) ? 0x8000u : 0u) | (ndig_of(b) << 16);
    };
    uint32_t r = wexI;
    for (uint64_t mm = ro.I; mm && r < kLCap; mm &= mm - 1, ++r) li[r] = entry((uint32_t)ctz64(mm));
    r = wexV;
    for (uint64_t mm = ro.V; mm && r < kLCap; mm &= mm - 1, ++r) lv[r] = entry((uint32_t)ctz64(mm));
  }
  bk.wave_sync();
  FAST_STAMP(k, 5);
#if defined(LSVM_ABL) && LSVM_ABL == 3  // timing ablation only: + run lists
  if (li[lane] == 0x12345678u) a.res[15] = lv[lane];
  return;
#endif
  bool anyfail = false;
  const uint32_t iv = a.indexing_mode > 0 ? 1u : 0u;
  const uint32_t nround = (mx<uint32_t>(nIq, nVq) + kWave - 1) / kWave;  // wave-uniform
#pragma unroll 1
  for (uint32_t u = 0; u < nround; ++u) {
    const uint32_t e = u * kWave + lane;
    bool okI = true, okV = true;
    if (e < nIq) {
      const uint32_t x = li[e];
      const uint32_t v = dec_index(x & 0x3FFFu, x >> 16, &okI);
      okI = okI && !(x & 0x8000u);
      li[e] = v - iv;  // the id (indexing_mode > 0: one lower; the 64-bit form widens it at the store)
    }
    if (e < nVq) {
      const uint32_t x = lv[e];
      const float v = dec_float(x & 0x3FFFu, x >> 16, &okV);
      okV = okV && !(x & 0x8000u);
      lv[e] = f2u(v);
    }
    const uint64_t fi = bk.ballot(!okI), fv = bk.ballot(!okV);
    if (lane == 0) {
      sh.fail[wid][0][u] = fi;
      sh.fail[wid][1][u] = fv;
    }
    anyfail |= (fi | fv) != 0;
  }
  bk.wave_sync();  // (the failure words and the decoded entries: every lane reads them below)
  FAST_STAMP(k, 6);
#if defined(LSVM_ABL) && LSVM_ABL == 4  // timing ablation only: + decode, no look-back
  if (li[lane] == 0x12345678u || anyfail) a.res[15] = lv[lane];
  return;
#endif
  // ---- look-back (wave 0), then the stores
  if (tid < kWave) {
    if (!lean_look_back(a.lean_lb, a.ntiles, k, cnt4, a.gate, sh.base, bk) && tid == 0) sh.flags |= 2u;
  }
  bk.sync();
  if (sh.flags & 2u) return;  // a poisoned tile before this one (block-uniform)
  FAST_STAMP(k, 7);
  const uint64_t bRows = sh.base[0], bIdx = sh.base[1], bVal = sh.base[2], bW = sh.base[3];
  if (k + 1 == a.ntiles && tid == 0) {  // the last tile publishes the totals
    const uint64_t rows = bRows + nL;
    a.res[C_ROWS] = rows;
    a.res[C_INDEX] = bIdx + nI;
    a.res[C_VALUE] = bVal + nV;
    a.res[C_WEIGHT] = bW + nW;
    a.res[C_QID] = 0;
    a.res[C_LABEL] = rows;
    a.res[C_FIELD] = 0;
    if (a.offset && rows < a.cap[C_ROWS] + 1) a.offset[rows] = bIdx + nI;
  }
  const uint64_t eL = bRows + (ex & 0xFFFF), eW = bW + ((ex >> 16) & 0xFFFF), eI = bIdx + ((ex >> 32) & 0xFFFF),
                 eV = bVal + (ex >> 48);
  const uint64_t eIw = bIdx + ((wpre >> 32) & 0xFFFF), eVw = bVal + (wpre >> 48);  // the wave's first entries
#if defined(LSVM_ABL) && LSVM_ABL == 2  // timing ablation only: no stores
  if (eL == 0x123456789ull) a.res[15] = eI + eV + eW;
  return;
#endif
  auto put_index = [&](uint64_t r, uint64_t v, uint64_t q) {
    if (r < a.cap[C_INDEX]) {
      if (a.wide) reinterpret_cast<uint64_t *>(a.index)[r] = v;
      else reinterpret_cast<uint32_t *>(a.index)[r] = (uint32_t)v;
    } else {
      raise_error(a.err, E_CAPACITY, q);
    }
  };
  auto put_value = [&](uint64_t r, float v, uint64_t q) {
    if (r < a.cap[C_VALUE]) a.value[r] = v;
    else raise_error(a.err, E_CAPACITY, q);
  };
  // the lists' entries: consecutive lanes store consecutive entries
#pragma unroll 1
  for (uint32_t u = 0; u < nround; ++u) {
    const uint32_t e = u * kWave + lane;
    const uint64_t fi = sh.fail[wid][0][u], fv = sh.fail[wid][1][u];
    if (e < nIq && !((fi >> lane) & 1u)) {
      const uint32_t v = li[e];  // (the 64-bit id of indexing_mode > 0 from a 0 wraps to ~0)
      put_index(eIw + e, a.wide ? (uint64_t)(v + iv) - iv : (uint64_t)v, eIw + e);
    }
    if (e < nVq && !((fv >> lane) & 1u)) put_value(eVw + e, u2f(lv[e]), eVw + e);
  }
  // the owner's runs: the window, else the byte decoders with the run's limit
  auto own_float = [&](uint32_t b) -> float {
    bool ok;
    const float v = dec_float(o0 + b, ndig_of(b), &ok);
    return ok && P + b + 16 <= lim_of(b) ? v : fsvm::slow_float(a.text, P + b, lim_of(b));
  };
  auto own_index = [&](uint32_t b) -> uint64_t {
    bool ok;
    const uint32_t v = dec_index(o0 + b, ndig_of(b), &ok);
    if (ok && P + b + 16 <= lim_of(b)) return (uint64_t)v - iv;
    uint64_t x = 0;
    if (!fsvm::slow_uint(a.text, P + b, lim_of(b), a.wide, &x)) {
      raise_error(a.err, E_NEG_INDEX, P + b);
      x = 0;
    }
    return x - iv;
  };
  auto failed = [&](int kind, uint32_t r) -> bool {
    return r >= kLCap || ((sh.fail[wid][kind][r >> 6] >> (r & 63)) & 1u);
  };
  if (bk.ballot(anyfail || wexI + (uint32_t)popc64(ro.I) > kLCap || wexV + (uint32_t)popc64(ro.V) > kLCap)) {
    uint32_t r = wexI;
    for (uint64_t mm = ro.I; mm; mm &= mm - 1, ++r) {
      const uint32_t b = (uint32_t)ctz64(mm);
      if (failed(0, r)) put_index(eIw + r, own_index(b), P + b);
    }
    r = wexV;
    for (uint64_t mm = ro.V; mm; mm &= mm - 1, ++r) {
      const uint32_t b = (uint32_t)ctz64(mm);
      if (failed(1, r)) put_value(eVw + r, own_float(b), P + b);
    }
  }
  // rows: each label, and its offset (the indices before it); weights
  {
    uint64_t r = eL;
    for (uint64_t mm = ro.L; mm; mm &= mm - 1, ++r) {
      const uint32_t b = (uint32_t)ctz64(mm);
      const float v = own_float(b);
      const uint64_t below = (mm & (0 - mm)) - 1;
      if (r < a.cap[C_ROWS]) {
        a.label[r] = v;
        a.offset[r] = eI + (uint64_t)popc64(ro.I & below);
      } else {
        raise_error(a.err, E_CAPACITY, P + b);
      }
    }
    r = eW;
    for (uint64_t mm = ro.W; mm; mm &= mm - 1, ++r) {
      const uint32_t b = (uint32_t)ctz64(mm);
      const float v = own_float(b);
      if (r < a.cap[C_WEIGHT]) a.weight[r] = v;
      else raise_error(a.err, E_CAPACITY, P + b);
    }
  }
  // the unit table: exclusive counts at each unit start in my segment
  if (a.chunk_tab) {  // (wave-uniform: the loop's shuffles need every lane)
    const uint64_t mt = bk.ballot(un.c0 + lane < (uint64_t)a.nchunk && un.v >= P0 && un.v < P0 + (uint64_t)kWave * kSegB);
    for (uint64_t mm = mt; mm; mm &= mm - 1) {
      const uint32_t j = (uint32_t)ctz64(mm);
      const uint64_t x = bk.shfl(un.v, (int)j);
      if (x < P || x >= P + (uint64_t)nv || x >= thi) continue;
      const uint64_t below = (1ull << (x - P)) - 1;
      uint64_t *row = a.chunk_tab + (un.c0 + j) * 8;
      const uint64_t rows = eL + popc64(ro.L & below);
      row[C_ROWS] = rows;
      row[C_INDEX] = eI + popc64(ro.I & below);
      row[C_VALUE] = eV + popc64(ro.V & below);
      row[C_WEIGHT] = eW + popc64(ro.W & below);
      row[C_QID] = 0;
      row[C_LABEL] = rows;
      row[C_FIELD] = 0;
    }
  }
  FAST_STAMP(k, 8);
}

}  // namespace lsvm
}  // namespace dmlc_amd
