// emu.cpp -- TEST INFRASTRUCTURE ONLY: CPU emulation of the HIP tile kernels.
//
// Runs the exact per-thread tile bodies of dmlc-core_amd/csrc/{libsvm,csv}_core.h
// with 256 std::threads per workgroup, a real barrier and a serial block scan,
// so kernel logic can be debugged (and run under AddressSanitizer) without a
// GPU.  Never part of the product: nothing in dmlc-core_amd/ links it.
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <thread>
#include <vector>

#include "csv_core.h"
#include "csv_fast.h"
#include "dmlc_amd.h"
#include "libfm_core.h"
#include "libsvm_core.h"
#include "svm_fast.h"
#include "svm_lean.h"

using namespace dmlc_amd;

namespace {

struct Barrier {
  std::mutex m;
  std::condition_variable cv;
  int n, waiting = 0;
  unsigned gen = 0;
  explicit Barrier(int n_) : n(n_) {}
  void wait() {
    std::unique_lock<std::mutex> lk(m);
    const unsigned g = gen;
    if (++waiting == n) {
      waiting = 0;
      ++gen;
      cv.notify_all();
    } else {
      cv.wait(lk, [&] { return gen != g; });
    }
  }
};

template <int NT>
struct BlockCtxT {
  static constexpr int kW = NT / kWave;
  Barrier bar{NT};
  std::vector<Barrier *> wbar;
  unsigned char bal[NT];
  uint32_t ws[NT];
  alignas(64) unsigned char scan[NT * 64];
  uint64_t mins[NT];
  uint64_t sh8[NT];
  uint32_t wv[NT / kWave];
  BlockCtxT() {
    for (int w = 0; w < kW; ++w) wbar.push_back(new Barrier(kWave));
  }
  ~BlockCtxT() {
    for (auto *b : wbar) delete b;
  }
};

// NT threads per workgroup: kThreads for the exact tiles, fast::kFThreads
// for the single-pass tiles
template <int NT>
struct HostBlockT {
  int t;
  BlockCtxT<NT> *ctx;
  int tid() const { return t; }
  void sync() { ctx->bar.wait(); }
  void wave_sync() { ctx->wbar[t / kWave]->wait(); }
  uint64_t ballot(bool p) {
    ctx->bal[t] = p;
    wave_sync();
    uint64_t m = 0;
    const int w0 = t / kWave * kWave;
    for (int i = 0; i < kWave; ++i) m |= (uint64_t)(ctx->bal[w0 + i] != 0) << i;
    wave_sync();
    return m;
  }
  template <typename T>
  T shfl(T v, int src) {
    static_assert(sizeof(T) <= 8, "shfl element");
    std::memcpy(&ctx->sh8[t], &v, sizeof(T));
    wave_sync();
    T r;
    std::memcpy(&r, &ctx->sh8[t / kWave * kWave + src], sizeof(T));
    wave_sync();
    return r;
  }
  void wave_put(uint32_t v) {  // DevBlockT::wave_put
    if (t % kWave == 0) ctx->wv[t / kWave] = v;
  }
  uint32_t wave_get(int w) { return ctx->wv[w]; }
  uint32_t wave_sum(uint32_t v) {
    ctx->ws[t] = v;
    wave_sync();
    uint32_t r = 0;
    const int w0 = t / kWave * kWave;
    for (int i = 0; i < kWave; ++i) r += ctx->ws[w0 + i];
    wave_sync();
    return r;
  }
  uint64_t min_u64(uint64_t v) {
    ctx->mins[t] = v;
    sync();
    uint64_t r = ~0ull;
    for (int i = 0; i < NT; ++i) r = ctx->mins[i] < r ? ctx->mins[i] : r;
    sync();
    return r;
  }
  template <typename T>
  T shfl_up(T v, int d) {  // lane - d's value (own below d)
    static_assert(sizeof(T) <= 8, "shfl element");
    std::memcpy(&ctx->sh8[t], &v, sizeof(T));
    wave_sync();
    T r = v;
    if (t % kWave >= d) std::memcpy(&r, &ctx->sh8[t - d], sizeof(T));
    wave_sync();
    return r;
  }
  // DevBlockT::exclusive_add1: packed counters, per-wave totals / flags to the caller's LDS
  uint64_t exclusive_add1(uint64_t v, bool flag, uint64_t *wtot, uint32_t *wbad, uint64_t *total, uint64_t *wpre) {
    const uint64_t fm = ballot(flag);
    struct Add {
      uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
    };
    const uint64_t ex = exclusive(v, (uint64_t)0, Add(), total);
    const uint64_t w0 = shfl(ex, 0);  // the wave's first lane
    if (t % kWave == kWave - 1) {
      wtot[t / kWave] = ex + v - w0;  // the wave's total
      wbad[t / kWave] = fm != 0 ? 1u : 0u;
    }
    *wpre = w0;
    sync();
    return ex;
  }
  uint64_t exclusive_add(uint64_t v, uint64_t *total) {  // DevBlock::exclusive_add (packed counters)
    struct Add {
      uint64_t operator()(uint64_t a, uint64_t b) const { return a + b; }
    };
    return exclusive(v, (uint64_t)0, Add(), total);
  }
  template <typename T, typename Op>
  T exclusive(T v, T identity, Op op, T *total) {
    static_assert(sizeof(T) <= 64, "scan element");
    T *buf = reinterpret_cast<T *>(ctx->scan);
    buf[t] = v;
    sync();
    T acc = identity;
    for (int i = 0; i < t; ++i) acc = op(acc, buf[i]);
    T all = acc;
    for (int i = t; i < NT; ++i) all = op(all, buf[i]);
    *total = all;
    sync();
    return acc;
  }
};
using HostBlock = HostBlockT<kThreads>;
using FastBlock = HostBlockT<fast::kFThreads>;

template <int NT = kThreads, typename Body>
void run_block(Body body) {
  BlockCtxT<NT> ctx;
  std::vector<std::thread> th;
  th.reserve(NT);
  for (int t = 0; t < NT; ++t)
    th.emplace_back([&, t] {
      HostBlockT<NT> bk{t, &ctx};
      body(bk);
    });
  for (auto &x : th) x.join();
}

void tile_scan(const std::vector<uint64_t> &cnt, std::vector<uint64_t> &base, uint64_t ntiles, uint64_t *res) {
  uint64_t run[C_N] = {0};
  for (uint64_t k = 0; k < ntiles; ++k)
    for (int i = 0; i < C_N; ++i) {
      base[k * C_N + i] = run[i];
      run[i] += cnt[k * C_N + i];
    }
  for (int i = 0; i < C_N; ++i) res[i] = run[i];
}

// mirrors the launchers' chunk-table pre-fill and finish_kernel (scan.h chunk_fixup_body)
void chunk_prefill(uint64_t *tab, int nchunk) {
  if (tab) std::memset(tab, 0xFF, (size_t)(nchunk > 0 ? nchunk : 0) * 8 * sizeof(uint64_t));
}
void chunk_fixup(uint64_t *tab, int nchunk, const uint64_t *res) {
  if (!tab) return;
  for (int c = nchunk - 1; c >= 0; --c) {
    uint64_t *row = tab + (uint64_t)c * 8;
    row[7] = 0;
    if (row[0] != ~0ull) continue;
    const uint64_t *nx = c + 1 < nchunk ? tab + (uint64_t)(c + 1) * 8 : res;
    for (int i = 0; i < 8; ++i) row[i] = i < 7 ? nx[i] : 0;
  }
}

}  // namespace

extern "C" int emu_parse(const uint8_t *text, uint64_t nbytes, const uint64_t *ccs, int nchunks_in,
                         const dmlc_amd_params *prm, const dmlc_amd_csr *out, uint64_t *chunk_table,
                         uint64_t *res /* 16 */) {
  // FillData ranges (nthread > 1) as ParseBlock units, as capi.cpp does with
  // range_kernel (ranges.hip): BackFindEndLine, text_parser.h:70-77,116-155
  const int upc = prm->nthread > 1 && nbytes > 0 ? prm->nthread : 1;
  std::vector<uint64_t> unit_starts;
  const uint64_t *cs = ccs;
  int nchunks = nchunks_in;
  if (upc > 1) {
    for (int c = 0; c < nchunks_in; ++c) {
      const uint64_t head = ccs[c], size = ccs[c + 1] - head, nstep = (size + upc - 1) / upc;
      for (int t = 0; t < upc; ++t) {
        const uint64_t sb = (uint64_t)t * nstep < size ? (uint64_t)t * nstep : size;
        uint64_t p = head + sb, r = head;
        for (; p > head; --p)
          if (p < head + size && (text[p] == '\n' || text[p] == '\r')) {
            r = p;
            break;
          }
        unit_starts.push_back(t == 0 ? head : r);
      }
    }
    unit_starts.push_back(nbytes);
    cs = unit_starts.data();
    nchunks = nchunks_in * upc;
  }
  const UnitLim ul{ccs, upc};
  const uint64_t T = prm->tile_bytes ? prm->tile_bytes : (256ull << 10);
  const uint64_t ntiles = (nbytes + T - 1) / T;
  const bool count_only = prm->flags & DMLC_AMD_FLAG_COUNT_ONLY;
  std::memset(res, 0, 16 * 8);
  res[8] = ~0ull;
  std::vector<uint64_t> tile_cnt(ntiles * C_N + 1), tile_base(ntiles * C_N + 1);
  std::vector<uint64_t> chunk_min(nchunks > 0 ? nchunks : 1, ~0ull), sink((nchunks > 0 ? nchunks : 1) * 8);
  unsigned long long *err = reinterpret_cast<unsigned long long *>(res + 8);
  if (!ntiles && !count_only && out->offset) out->offset[0] = 0;
  if (!count_only) chunk_prefill(chunk_table, nchunks);
  if (prm->format == DMLC_AMD_LIBSVM || prm->format == DMLC_AMD_LIBFM) {
    // mirrors launch_libsvm (libsvm.hip) / launch_libfm (libfm.hip): the
    // uniform-grammar kernel first, the exact tile kernels when it sets the
    // gate (or indexing_mode < 0 / FLAG_EXACT)
    const bool fm = prm->format == DMLC_AMD_LIBFM;
    const bool use_fast = nbytes > 0 && !(prm->flags & DMLC_AMD_FLAG_EXACT);
    const uint64_t nft = (nbytes + fsvm::kTile - 1) / fsvm::kTile;
    const bool imin = prm->indexing_mode < 0;
    std::vector<uint64_t> umin(nchunks > 0 ? nchunks : 1, ~0ull);
    uint64_t *ftab = chunk_table ? chunk_table : (imin ? sink.data() : nullptr);  // capi.cpp f.chunk_tab
    if (!count_only && ftab != chunk_table) chunk_prefill(ftab, nchunks);
    uint32_t gate = use_fast ? 0u : 1u;
    unsigned long long ferr = ~0ull;
    std::vector<uint64_t> lb(nft * 8 + 1, 0), qsum(kLabShards * 8, 0);
    LibfmArgs a;
    std::memset(&a, 0, sizeof(a));
    a.field = out->field;
    a.text = text;
    a.n = nbytes;
    a.cs = cs;
    a.nchunk = nchunks;
    a.ul = ul;
    a.tile_bytes = T;
    a.ntiles = (uint32_t)ntiles;
    a.wide = prm->index_bits == 64;
    a.indexing_mode = prm->indexing_mode;
    a.tile_cnt = tile_cnt.data();
    a.tile_base = tile_base.data();
    a.offset = out->offset;
    a.label = reinterpret_cast<float *>(out->label);
    a.weight = out->weight;
    a.qid = out->qid;
    a.index = out->index;
    a.value = reinterpret_cast<float *>(out->value);
    for (int i = 0; i < 8; ++i) a.cap[i] = out->cap[i];
    a.chunk_tab = chunk_table ? chunk_table : sink.data();
    a.chunk_min = chunk_min.data();
    a.err = err;
    a.gate = &gate;
    std::vector<uint32_t> rec;  // the exact libsvm / libfm kernels' count-pass records (capi.cpp)
    std::vector<uint64_t> rec_meta;
    if (!std::getenv("EMU_NOREC")) {  // (EMU_NOREC: records off, test_emu.py self-checks)
      const uint32_t rw = exact_rec_win(T, kWin);
      if (exact_rec_on(nbytes, exact_rec_bytes(ntiles, rw, kThreads))) {
        rec.assign(ntiles * rw * 4 * kThreads, 0xCDCDCDCDu);  // device memory is not zeroed either
        rec_meta.assign(ntiles * rw * 2, 0xCDCDCDCDCDCDCDCDull);
        a.rec = rec.data();
        a.rec_meta = rec_meta.data();
        a.rec_win = rw;
      }
    }
    if (use_fast) {
      FastSvmArgs f;
      std::memset(&f, 0, sizeof(f));
      f.text = text;
      f.n = nbytes;
      f.cs = cs;
      f.nchunk = nchunks;
      f.ntiles = (uint32_t)nft;
      f.wide = a.wide;
      f.indexing_mode = prm->indexing_mode;
      f.offset = a.offset;
      f.label = a.label;
      f.weight = a.weight;
      f.qid = a.qid;
      f.index = a.index;
      f.field = fm ? out->field : nullptr;
      f.value = a.value;
      for (int i = 0; i < 8; ++i) f.cap[i] = out->cap[i];
      f.chunk_tab = ftab;
      f.umin = umin.data();
      f.lb = lb.data();
      f.qsum = qsum.data();
      f.gate = &gate;
      f.err = &ferr;
      f.res = res;
      // the lean kernel first on a full call (libsvm.hip launch_libsvm)
      const char *le = std::getenv("DMLC_AMD_LEAN");
      // (off unless DMLC_AMD_LEAN=1, as in the product build: libsvm.hip LSVM_DEFAULT)
      const bool lean = !fm && !count_only && prm->indexing_mode >= 0 && le && le[0] && le[0] != '0';
      std::vector<uint64_t> llb(nft * 5 + 1, 0);
      if (lean) {
        f.lean_lb = llb.data();
        f.lean_poison = llb.data() + nft * 5;
        for (uint64_t k = 0; k < nft; ++k) {
          lsvm::Shared *sh = new lsvm::Shared;
          std::memset(sh, 0xCD, sizeof(*sh));
          run_block<fast::kFThreads>([&](FastBlock &bk) { lsvm::tile(f, *sh, bk, (uint32_t)k); });
          delete sh;
        }
        if (std::getenv("EMU_VERBOSE"))
          std::fprintf(stderr, "emu: lean poison=%lld\n", llb[nft * 5] ? (long long)~llb[nft * 5] : -1ll);
      }
      for (uint64_t k = 0; k < nft; ++k) {
        fsvm::Shared *sh = new fsvm::Shared;
        std::memset(sh, 0xCD, sizeof(*sh));
        run_block<fast::kFThreads>([&](FastBlock &bk) {
          if (fm) {
            if (count_only) fsvm::tile<1, true>(f, *sh, bk, (uint32_t)k);
            else fsvm::tile<2, true>(f, *sh, bk, (uint32_t)k);
          } else {
            if (count_only) fsvm::tile<1>(f, *sh, bk, (uint32_t)k);
            else fsvm::tile<2>(f, *sh, bk, (uint32_t)k);
          }
        });
        delete sh;
      }
      if (!fm) {  // qid_fix_kernel (libsvm.hip)
        uint64_t total = 0;
        for (int i = 0; i < kLabShards; ++i) total += qsum[i * 8];
        if (fsvm::qid_decide(total, res, &gate) && chunk_table && !count_only)
          for (int i = 0; i < nchunks; ++i)
            if (chunk_table[i * 8 + C_ROWS] != ~0ull) chunk_table[i * 8 + C_QID] = chunk_table[i * 8 + C_ROWS];
      }
    }
    if (gate) {
      for (uint64_t k = 0; k < ntiles; ++k) {
        svm::Shared *sh = new svm::Shared;
        std::memset(sh, 0xCD, sizeof(*sh));  // LDS is uninitialised on the GPU
        run_block([&](HostBlock &bk) {
          if (fm) fm::tile<1>(a, *sh, bk, k);
          else svm::tile<1>(a, *sh, bk, k);
        });
        delete sh;
      }
      tile_scan(tile_cnt, tile_base, ntiles, res);
      if (!count_only && out->offset && res[C_ROWS] < out->cap[C_ROWS] + 1) out->offset[res[C_ROWS]] = res[C_INDEX];
      if (!count_only) chunk_prefill(chunk_table, nchunks);  // the chunk-table reset in tile_scan_kernel (scan.h)
      if (!count_only)
        for (uint64_t k = 0; k < ntiles; ++k) {
          svm::Shared *sh = new svm::Shared;
          std::memset(sh, 0xCD, sizeof(*sh));
          run_block([&](HostBlock &bk) {
            if (fm) fm::tile<2>(a, *sh, bk, k);
            else svm::tile<2>(a, *sh, bk, k);
          });
          delete sh;
        }
    } else {
      res[8] = ferr;
      if (imin && !count_only && ftab) {  // finish_kernel, then umin_fix_kernel (svm_fast.h)
        chunk_fixup(ftab, nchunks, res);
        uint64_t tot = res[C_INDEX] < out->cap[C_INDEX] ? res[C_INDEX] : out->cap[C_INDEX];  // umin_fix_kernel's clamp
        if (fm && tot > out->cap[C_FIELD]) tot = out->cap[C_FIELD];
        fsvm::umin_fix(a.index, fm ? out->field : nullptr, a.wide, ftab, nchunks, umin.data(), tot, 0, tot, 0, 1);
      }
    }
    std::fprintf(stderr, "emu: %s path=%s\n", fm ? "libfm" : "libsvm", gate ? "exact" : "fast");
  } else if (prm->format == DMLC_AMD_CSV) {
    CsvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.text = text;
    a.n = nbytes;
    a.cs = cs;
    a.nchunk = nchunks;
    a.ul = ul;
    a.tile_bytes = T;
    a.ntiles = (uint32_t)ntiles;
    a.wide = prm->index_bits == 64;
    a.vtype = prm->value_type;
    a.label_column = prm->label_column;
    a.weight_column = prm->weight_column;
    a.delim = (uint32_t)prm->delimiter & 0xFFu;
    {
      const unsigned c = a.delim;
      a.fast_delim = !(c == ' ' || (c >= '\t' && c <= '\r') || (c >= '0' && c <= '9') ||
                       ((c | 32u) >= 'a' && (c | 32u) <= 'z') || c == '+' || c == '-' || c == '.' ||
                       c == '_' || c == '(' || c == ')' || c == 0);
    }
    a.tile_cnt = tile_cnt.data();
    a.tile_base = tile_base.data();
    a.offset = out->offset;
    a.label = out->label;
    a.weight = out->weight;
    a.index = out->index;
    a.value = out->value;
    for (int i = 0; i < 8; ++i) a.cap[i] = out->cap[i];
    a.chunk_tab = chunk_table ? chunk_table : sink.data();
    a.err = err;
    std::vector<uint32_t> rec;  // the exact CSV kernels' count-pass records (capi.cpp)
    {
      const uint32_t rw = exact_rec_win(T, kWin);
      if (exact_rec_on(nbytes, exact_rec_bytes(ntiles, rw, kThreads))) {
        rec.assign(ntiles * rw * 4 * kThreads, 0xCDCDCDCDu);
        a.rec = rec.data();
        a.rec_win = rw;
      }
    }
    // mirrors launch_csv (csv.hip): uniform-grammar kernel first, exact tile
    // kernels when it sets the gate (or the parameters are outside its form)
    const bool cols_ok = prm->value_type == DMLC_AMD_F32 ? csv_fast_columns_ok(prm->label_column, prm->weight_column)
                                                         : csv_fast_int_ok(prm->label_column);
    const bool use_fast = nbytes > 0 && cols_ok && a.fast_delim && !(prm->flags & DMLC_AMD_FLAG_EXACT);
    uint32_t gate = use_fast ? 0u : 1u;
    std::vector<uint64_t> labsum_v(kLabShards * 8, 0);
    uint64_t *labsum = labsum_v.data();
    unsigned long long ferr = ~0ull;
    if (use_fast) {
      const uint64_t nft = (nbytes + fast::kTile - 1) / fast::kTile;
      std::vector<uint64_t> lb(nft * 8 + 1, 0);
      FastCsvArgs f;
      std::memset(&f, 0, sizeof(f));
      f.text = text;
      f.n = nbytes;
      f.cs = cs;
      f.nchunk = nchunks;
      f.ntiles = (uint32_t)nft;
      f.wide = a.wide;
      f.delim = a.delim;
      f.label_col = prm->label_column;
      f.weight_col = prm->value_type == DMLC_AMD_F32 ? prm->weight_column : -1;
      f.vtype = prm->value_type;
      f.label = reinterpret_cast<float *>(out->label);
      f.weight = out->weight;
      f.labsum = labsum;
      f.offset = out->offset;
      f.index = out->index;
      f.value = out->value;
      for (int i = 0; i < 8; ++i) f.cap[i] = out->cap[i];
      f.chunk_tab = chunk_table;
      f.lb = lb.data();
      f.gate = &gate;
      f.err = &ferr;
      f.res = res;
      for (uint64_t k = 0; k < nft; ++k) {
        fcsv::Shared *sh = new fcsv::Shared;
        std::memset(sh, 0xCD, sizeof(*sh));
        const bool sp = f.label_col >= 0 || f.weight_col >= 0, iv = f.vtype != 0;
        if (count_only && iv) run_block<fast::kFThreads>([&](FastBlock &bk) { fcsv::tile<1, false, 1>(f, *sh, bk, (uint32_t)k); });
        else if (iv) run_block<fast::kFThreads>([&](FastBlock &bk) { fcsv::tile<2, false, 1>(f, *sh, bk, (uint32_t)k); });
        else if (count_only && sp) run_block<fast::kFThreads>([&](FastBlock &bk) { fcsv::tile<1, true, 0>(f, *sh, bk, (uint32_t)k); });
        else if (count_only) run_block<fast::kFThreads>([&](FastBlock &bk) { fcsv::tile<1, false, 0>(f, *sh, bk, (uint32_t)k); });
        else if (sp) run_block<fast::kFThreads>([&](FastBlock &bk) { fcsv::tile<2, true, 0>(f, *sh, bk, (uint32_t)k); });
        else run_block<fast::kFThreads>([&](FastBlock &bk) { fcsv::tile<2, false, 0>(f, *sh, bk, (uint32_t)k); });
        delete sh;
      }
      if (f.label_col >= 0 || f.weight_col >= 0) {  // label_check_kernel
        uint64_t s0 = 0, s1 = 0, s2 = 0;
        for (int i = 0; i < kLabShards; ++i) {
          s0 += labsum[i * 8];
          s1 += labsum[i * 8 + 1];
          s2 += labsum[i * 8 + 2];
        }
        if (s0 != 0 || s1 != 0 || s2 != 0) gate |= 1u;
      }
    }
    std::fprintf(stderr, "emu: csv path=%s\n", gate ? "exact" : "fast");
    if (!gate) {
      res[8] = ferr;
      if (res[8] == ~0ull) res[8] = 0;
      if (!count_only) chunk_fixup(chunk_table, nchunks, res);
      return 0;
    }
    for (uint64_t k = 0; k < ntiles; ++k) {
      csv::Shared *sh = new csv::Shared;
      std::memset(sh, 0xCD, sizeof(*sh));
      run_block([&](HostBlock &bk) { csv::tile<1>(a, *sh, bk, k); });
      delete sh;
    }
    tile_scan(tile_cnt, tile_base, ntiles, res);
    if (!count_only && out->offset && res[C_ROWS] < out->cap[C_ROWS] + 1) out->offset[res[C_ROWS]] = res[C_INDEX];
    if (!count_only) chunk_prefill(chunk_table, nchunks);  // the chunk-table reset in tile_scan_kernel (scan.h)
    if (!count_only)
      for (uint64_t k = 0; k < ntiles; ++k) {
        csv::Shared *sh = new csv::Shared;
        std::memset(sh, 0xCD, sizeof(*sh));
        run_block([&](HostBlock &bk) { csv::tile<2>(a, *sh, bk, k); });
        delete sh;
      }
  } else {
    return DMLC_AMD_ERR_ARG;
  }
  if (res[8] == ~0ull) res[8] = 0;
  if (!count_only) chunk_fixup(chunk_table, nchunks, res);
  return 0;
}

// ---------------------------------------------------------------- CLI mode
// emu <fmt> <index_bits> <vtype> <indexing_mode> <label_col> <weight_col> <delim_code> <tile>
//     <text_file> <chunks_file (uint64 LE, nchunks+1)> <out_prefix>
// Writes <out_prefix>.{res,offset,label,weight,qid,index,value,chunks} raw little-endian.
static std::vector<char> slurp(const char *p) {
  FILE *f = std::fopen(p, "rb");
  if (!f) return {};
  std::vector<char> v;
  char buf[1 << 16];
  size_t n;
  while ((n = std::fread(buf, 1, sizeof(buf), f)) > 0) v.insert(v.end(), buf, buf + n);
  std::fclose(f);
  return v;
}
static void dump(const std::string &p, const void *d, size_t n) {
  FILE *f = std::fopen(p.c_str(), "wb");
  if (n) std::fwrite(d, 1, n, f);
  std::fclose(f);
}

int main(int argc, char **argv) {
  if (argc != 12) {
    std::fprintf(stderr, "usage: see source\n");
    return 2;
  }
  dmlc_amd_params prm;
  std::memset(&prm, 0, sizeof(prm));
  prm.format = std::atoi(argv[1]);
  prm.index_bits = std::atoi(argv[2]);
  prm.value_type = std::atoi(argv[3]);
  prm.indexing_mode = std::atoi(argv[4]);
  prm.label_column = std::atoi(argv[5]);
  prm.weight_column = std::atoi(argv[6]);
  prm.delimiter = std::atoi(argv[7]);
  prm.tile_bytes = (uint32_t)std::atoi(argv[8]);
  if (const char *nt = std::getenv("EMU_NTHREAD")) prm.nthread = std::atoi(nt);
  std::vector<char> text = slurp(argv[9]);
  std::vector<char> craw = slurp(argv[10]);
  std::vector<uint64_t> cs(craw.size() / 8);
  std::memcpy(cs.data(), craw.data(), craw.size());
  const int nch = (int)cs.size() - 1;
  // exact-size heap copy of the text so ASan sees reads past its end
  uint8_t *t = (uint8_t *)std::malloc(text.size() ? text.size() : 1);
  std::memcpy(t, text.data(), text.size());
  uint64_t res[16];
  dmlc_amd_csr csr;
  std::memset(&csr, 0, sizeof(csr));
  const uint32_t xf = std::getenv("EMU_EXACT") ? DMLC_AMD_FLAG_EXACT : 0u;
  prm.flags = DMLC_AMD_FLAG_COUNT_ONLY | xf;
  emu_parse(t, text.size(), cs.data(), nch, &prm, &csr, nullptr, res);
  prm.flags = xf;
  const size_t vsz = prm.value_type == DMLC_AMD_I64 ? 8 : 4, isz = prm.index_bits == 64 ? 8 : 4;
  std::vector<uint64_t> offset(res[0] + 1);
  void *label = std::malloc(res[5] * vsz + 1), *value = std::malloc(res[2] * vsz + 1),
       *index = std::malloc(res[1] * isz + 1), *field = std::malloc(res[6] * isz + 1);
  std::vector<float> weight(res[3] + 1);
  std::vector<uint64_t> qid(res[4] + 1);
  const int upc = prm.nthread > 1 && !text.empty() ? prm.nthread : 1;
  std::vector<uint64_t> chunks((nch > 0 ? nch * upc : 1) * 8, 0);
  csr.offset = offset.data();
  csr.label = label;
  csr.weight = weight.data();
  csr.qid = qid.data();
  csr.index = index;
  csr.field = field;
  csr.value = value;
  uint64_t caps[8] = {res[0], res[1], res[2], res[3], res[4], res[5], res[6], 0};
  std::memcpy(csr.cap, caps, sizeof(caps));
  uint64_t res2[16];
  emu_parse(t, text.size(), cs.data(), nch, &prm, &csr, chunks.data(), res2);
  std::string o = argv[11];
  dump(o + ".res", res2, sizeof(res2));
  dump(o + ".offset", offset.data(), offset.size() * 8);
  dump(o + ".label", label, res2[5] * vsz);
  dump(o + ".weight", weight.data(), res2[3] * 4);
  dump(o + ".qid", qid.data(), res2[4] * 8);
  dump(o + ".index", index, res2[1] * isz);
  dump(o + ".field", field, res2[6] * isz);
  dump(o + ".value", value, res2[2] * vsz);
  dump(o + ".chunks", chunks.data(), chunks.size() * 8);
  std::free(t);
  std::free(label);
  std::free(value);
  std::free(index);
  std::free(field);
  return 0;
}
