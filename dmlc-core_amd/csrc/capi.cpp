// capi.cpp -- the extern "C" boundary (include/dmlc_amd.h) over the HIP kernels.
#include <hip/hip_runtime.h>

#include <cstring>
#include <vector>

#include "dmlc_amd.h"
#include "common.h"
#include "dmlc_amd_kernels.h"

namespace {

constexpr uint64_t kDefaultTile = 256ull << 10;  // bytes of text owned per workgroup (exact kernels)
constexpr uint64_t kFastTile = dmlc_amd::kFastTileBytes;  // fast_common.h kTile
constexpr int kSlots = 7;

uint64_t tile_of(const dmlc_amd_params *p) {
  return p && p->tile_bytes ? (uint64_t)p->tile_bytes : kDefaultTile;
}

struct Carve {
  char *p;
  size_t left;
  template <typename T>
  T *take(size_t n) {
    size_t bytes = (n * sizeof(T) + 255) & ~size_t(255);
    if (bytes > left) return nullptr;
    T *r = reinterpret_cast<T *>(p);
    p += bytes;
    left -= bytes;
    return r;
  }
};

// Delimiters that ParseFloat / strtoll can consume, which would make the field
// structure depend on decoding (csv_parser.h:99-127): handled by the exact
// per-line path instead of the field-parallel one.
bool csv_delim_fast(int d, int vtype) {
  const unsigned c = (unsigned)d & 0xFFu;
  if (c == ' ' || (c >= '\t' && c <= '\r')) return false;  // whitespace (incl. \v for strtoll)
  if ((c >= '0' && c <= '9') || ((c | 32u) >= 'a' && (c | 32u) <= 'z')) return false;
  if (c == '+' || c == '-' || c == '.' || c == '_' || c == '(' || c == ')') return false;
  if (c == 0) return false;
  (void)vtype;
  return true;
}

// ---- kernel timing (dmlc_amd_profile_begin / _end)
struct Profile {
  bool on = false;
  std::vector<hipEvent_t> ev;  // pairs: begin, end
  size_t used = 0;
  const char *kernel = "";
};
thread_local Profile g_prof;
thread_local hipError_t g_last_hip = hipSuccess;

}  // namespace

namespace dmlc_amd {
void prof_mark(int end, hipStream_t s, const char *kernel) {
  Profile &p = g_prof;
  if (!p.on) return;
  if (!end) {
    if (p.used + 2 > p.ev.size()) {
      for (int i = 0; i < 64; ++i) {
        hipEvent_t e;
        // no system-scope fence: a timing marker between kernels of one stream
        // (with it each marker cost the call about 5 us of GPU time)
        if (hipEventCreateWithFlags(&e, hipEventDisableSystemFence) != hipSuccess) return;
        p.ev.push_back(e);
      }
    }
    (void)hipEventRecord(p.ev[p.used], s);
    p.kernel = kernel;
  } else {
    (void)hipEventRecord(p.ev[p.used + 1], s);
    p.used += 2;
  }
}
}  // namespace dmlc_amd

extern "C" {

int dmlc_amd_profile_begin(void) {
  g_prof.on = true;
  g_prof.used = 0;
  return DMLC_AMD_OK;
}

int dmlc_amd_profile_end(double *total_ms, int *launches, const char **kernel) {
  Profile &p = g_prof;
  p.on = false;
  double t = 0;
  for (size_t i = 0; i + 1 < p.used; i += 2) {
    float ms = 0;
    if (hipEventSynchronize(p.ev[i + 1]) != hipSuccess ||
        hipEventElapsedTime(&ms, p.ev[i], p.ev[i + 1]) != hipSuccess)
      return DMLC_AMD_ERR_HIP;
    t += ms;
  }
  if (total_ms) *total_ms = t;
  if (launches) *launches = (int)(p.used / 2);
  if (kernel) *kernel = p.kernel;
  p.used = 0;
  return DMLC_AMD_OK;
}


int dmlc_amd_abi_version(void) { return DMLC_AMD_ABI_VERSION; }

#ifndef DMLC_AMD_BUILD_ID
#define DMLC_AMD_BUILD_ID "unknown"
#endif
const char *dmlc_amd_build_id(void) { return DMLC_AMD_BUILD_ID; }

int dmlc_amd_fast_geometry(uint32_t *tile_bytes, uint32_t *max_unit_starts) {
  if (tile_bytes) *tile_bytes = (uint32_t)dmlc_amd::kFastTileBytes;
  if (max_unit_starts) *max_unit_starts = (uint32_t)dmlc_amd::kFastMaxCs;
  return DMLC_AMD_OK;
}

int dmlc_amd_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

const char *dmlc_amd_error_string(int code) {
  switch (code) {
    case DMLC_AMD_OK: return "ok";
    case DMLC_AMD_ERR_NEG_INDEX: return "Check failed: sign == true";
    case DMLC_AMD_ERR_NAN_LITERAL: return "Check failed: *p == ')': Invalid NAN literal";
    case DMLC_AMD_ERR_CSV_DELIM: return "Delimiter is not found in the line";
    case DMLC_AMD_ERR_CAPACITY: return "output capacity exceeded";
    case DMLC_AMD_ERR_ARG: return "invalid argument";
    case DMLC_AMD_ERR_HIP: return "HIP runtime error";
    default: return "unknown error";
  }
}

// FillData ranges per chunk (dmlc_amd_params.nthread; 0 = 1)
int units_per_chunk(const dmlc_amd_params *p) { return p && p->nthread > 1 ? p->nthread : 1; }
constexpr int kMaxNthread = 1 << 12;

// the exact kernels' count-pass records (args.h exact_rec_*): bytes, 0 when
// they would outgrow the text
uint64_t rec_bytes_of(uint64_t nbytes, uint64_t T, uint64_t ntiles, const dmlc_amd_params *prm) {
  if (!prm) return 0;
  const uint64_t b = dmlc_amd::exact_rec_bytes(ntiles, dmlc_amd::exact_rec_win(T, dmlc_amd::kWin), dmlc_amd::kThreads);
  return dmlc_amd::exact_rec_on(nbytes, b) ? b : 0;
}

// single-pass look-back words: the full kernel's [5 nft] + its ticket; libsvm
// adds the lean kernel's [5 nft] + its poison word (libsvm.hip); CSV keeps
// one 8-word record per tile (csv_fast.h csv_look_back)
uint64_t lb_words_of(uint64_t nft, const dmlc_amd_params *prm) {
  if (prm && prm->format == DMLC_AMD_CSV) return nft * dmlc_amd::kCsvLbWords + 1;
  return prm && prm->format == DMLC_AMD_LIBSVM ? nft * 10 + 2 : nft * 5 + 1;
}

size_t dmlc_amd_workspace_bytes(uint64_t nbytes, int nchunks, const dmlc_amd_params *prm) {
  const uint64_t T = tile_of(prm);
  const uint64_t ntiles = (nbytes + T - 1) / T;
  const uint64_t nc = (nchunks > 0 ? (uint64_t)nchunks : 1) * (uint64_t)units_per_chunk(prm);
  const uint64_t nft = (nbytes + kFastTile - 1) / kFastTile;
  return (size_t)((2 * ntiles * kSlots + 2 * nc + nc * 8 + (nc + 1) + lb_words_of(nft, prm) + dmlc_amd::kLabShards * 8) *
                      sizeof(uint64_t) +
                  12 * 256 + rec_bytes_of(nbytes, T, ntiles, prm) + 2 * 256);
}

int dmlc_amd_parse(const void *d_text, uint64_t nbytes, const uint64_t *d_chunk_starts, int nchunks,
                   const dmlc_amd_params *prm, const dmlc_amd_csr *out, uint64_t *d_chunk_table,
                   void *d_workspace, size_t workspace_bytes, dmlc_amd_result *d_result,
                   void *stream) {
  if (!prm || !out || !d_result) return DMLC_AMD_ERR_ARG;
  if (prm->format < DMLC_AMD_LIBSVM || prm->format > DMLC_AMD_LIBFM) return DMLC_AMD_ERR_ARG;
  if (prm->index_bits != 32 && prm->index_bits != 64) return DMLC_AMD_ERR_ARG;
  if (prm->value_type < DMLC_AMD_F32 || prm->value_type > DMLC_AMD_I64) return DMLC_AMD_ERR_ARG;
  if (prm->format != DMLC_AMD_CSV && prm->value_type != DMLC_AMD_F32) return DMLC_AMD_ERR_ARG;
  if (nbytes && (!d_text || !d_chunk_starts || nchunks < 1)) return DMLC_AMD_ERR_ARG;
  if (prm->format == DMLC_AMD_CSV && prm->label_column >= 0 &&
      prm->label_column == prm->weight_column)
    return DMLC_AMD_ERR_ARG;  // csv_parser.h:59-60
  if (prm->nthread < 0 || prm->nthread > kMaxNthread) return DMLC_AMD_ERR_ARG;
  if (workspace_bytes < dmlc_amd_workspace_bytes(nbytes, nchunks, prm) || !d_workspace)
    return DMLC_AMD_ERR_ARG;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  const uint64_t T = tile_of(prm);
  const uint64_t ntiles = (nbytes + T - 1) / T;
  const int upc = units_per_chunk(prm);
  const uint64_t nunits = (uint64_t)(nchunks > 0 ? nchunks : 0) * (uint64_t)upc;
  if (nunits > (uint64_t)INT32_MAX) return DMLC_AMD_ERR_ARG;
  const int nc = nunits > 0 ? (int)nunits : 1;
  Carve cv{reinterpret_cast<char *>(d_workspace), workspace_bytes};
  uint64_t *tile_cnt = cv.take<uint64_t>(ntiles * kSlots + 1);
  uint64_t *tile_base = cv.take<uint64_t>(ntiles * kSlots + 1);
  uint64_t *chunk_min = cv.take<uint64_t>(nc);
  uint64_t *fast_min = cv.take<uint64_t>(nc);  // single-pass write pass, indexing_mode < 0 (svm_fast.h umin_fix)
  uint64_t *chunk_sink = cv.take<uint64_t>((size_t)nc * 8);
  uint64_t *units = cv.take<uint64_t>((size_t)nc + 1);  // ParseBlock unit starts (nthread > 1)
  const uint64_t nft = (nbytes + kFastTile - 1) / kFastTile;
  uint32_t *ctl = cv.take<uint32_t>(4);               // gate, gate after the count phase, recount flag
  unsigned long long *ferr = cv.take<unsigned long long>(1);
  uint64_t *lb = cv.take<uint64_t>(lb_words_of(nft, prm));
  uint64_t *labsum = cv.take<uint64_t>(dmlc_amd::kLabShards * 8);
  const uint64_t recb = rec_bytes_of(nbytes, T, ntiles, prm);
  const uint32_t rec_win = dmlc_amd::exact_rec_win(T, dmlc_amd::kWin);
  uint64_t *rec_meta = recb ? cv.take<uint64_t>(ntiles * rec_win * 2) : nullptr;
  uint32_t *rec = recb ? cv.take<uint32_t>(ntiles * rec_win * 4 * dmlc_amd::kThreads) : nullptr;
  if (recb && (!rec || !rec_meta)) return DMLC_AMD_ERR_ARG;
  if (!tile_cnt || !tile_base || !chunk_min || !fast_min || !chunk_sink || !units || !ctl || !ferr || !lb || !labsum)
    return DMLC_AMD_ERR_ARG;
  // FillData's thread ranges become the units the kernels parse; the
  // decoders still read to the end of the InputSplit chunk (args.h UnitLim)
  const uint64_t *ucs = d_chunk_starts;
  if (upc > 1 && nbytes > 0) {
    const hipError_t re = dmlc_amd::launch_ranges(reinterpret_cast<const uint8_t *>(d_text), d_chunk_starts,
                                                  nchunks, upc, nbytes, units, s);
    if (re != hipSuccess) {
      g_last_hip = re;
      return DMLC_AMD_ERR_HIP;
    }
    ucs = units;
  }
  const dmlc_amd::UnitLim ul{d_chunk_starts, upc};
  uint64_t *res = reinterpret_cast<uint64_t *>(d_result);
  const bool count_only = (prm->flags & DMLC_AMD_FLAG_COUNT_ONLY) != 0;
  const bool fill_only = (prm->flags & DMLC_AMD_FLAG_FILL_ONLY) != 0;
  if (count_only && fill_only) return DMLC_AMD_ERR_ARG;
  const int phase = count_only ? dmlc_amd::kPhaseCount
                               : (fill_only ? dmlc_amd::kPhaseFill : dmlc_amd::kPhaseFull);
  hipError_t e = hipSuccess;
  if (prm->format == DMLC_AMD_LIBSVM) {
    dmlc_amd::LibsvmArgs a;
    std::memset(&a, 0, sizeof(a));
    a.text = reinterpret_cast<const uint8_t *>(d_text);
    a.n = nbytes;
    a.cs = ucs;
    a.nchunk = (int)nunits;
    a.ul = ul;
    a.tile_bytes = T;
    a.ntiles = (uint32_t)ntiles;
    a.wide = prm->index_bits == 64;
    a.indexing_mode = prm->indexing_mode;
    a.tile_cnt = tile_cnt;
    a.tile_base = tile_base;
    a.offset = out->offset;
    a.label = reinterpret_cast<float *>(out->label);
    a.weight = out->weight;
    a.qid = out->qid;
    a.index = out->index;
    a.value = reinterpret_cast<float *>(out->value);
    for (int i = 0; i < 8; ++i) a.cap[i] = out->cap[i];
    a.chunk_tab = d_chunk_table ? d_chunk_table : chunk_sink;
    a.chunk_min = chunk_min;
    a.err = reinterpret_cast<unsigned long long *>(res + 8);
    a.gate = ctl;
    a.rec = rec;
    a.rec_meta = rec_meta;
    a.rec_win = rec ? rec_win : 0;
    dmlc_amd::FastSvmArgs f;
    std::memset(&f, 0, sizeof(f));
    f.text = a.text;
    f.n = nbytes;
    f.cs = ucs;
    f.nchunk = (int)nunits;
    f.ntiles = (uint32_t)nft;
    f.wide = a.wide;
    f.indexing_mode = prm->indexing_mode;
    f.skip_if_gated = phase == dmlc_amd::kPhaseFill;
    f.offset = a.offset;
    f.label = a.label;
    f.weight = a.weight;
    f.qid = a.qid;
    f.index = a.index;
    f.value = a.value;
    for (int i = 0; i < 8; ++i) f.cap[i] = out->cap[i];
    // indexing_mode < 0 needs the units' index ranges after the write pass:
    // the chunk table, or the workspace's when the caller passes none
    f.chunk_tab = d_chunk_table ? d_chunk_table : (prm->indexing_mode < 0 ? chunk_sink : nullptr);
    f.lb = lb;
    f.ticket = reinterpret_cast<uint32_t *>(lb + nft * dmlc_amd::kFastLbWords);  // zeroed with lb
    f.lean_lb = lb + nft * dmlc_amd::kFastLbWords + 1;
    f.lean_poison = f.lean_lb + nft * dmlc_amd::kFastLbWords;
    f.qsum = labsum;
    f.umin = fast_min;
    f.gate = ctl;
    f.err = ferr;
    f.res = res;
    const bool use_fast = nbytes > 0 && !(prm->flags & DMLC_AMD_FLAG_EXACT);
    e = dmlc_amd::launch_libsvm(a, f, use_fast, res, phase, s);
  } else if (prm->format == DMLC_AMD_CSV) {
    dmlc_amd::CsvArgs a;
    std::memset(&a, 0, sizeof(a));
    a.text = reinterpret_cast<const uint8_t *>(d_text);
    a.n = nbytes;
    a.cs = ucs;
    a.nchunk = (int)nunits;
    a.ul = ul;
    a.tile_bytes = T;
    a.ntiles = (uint32_t)ntiles;
    a.wide = prm->index_bits == 64;
    a.vtype = prm->value_type;
    a.label_column = prm->label_column;
    a.weight_column = prm->weight_column;
    a.delim = (uint32_t)prm->delimiter & 0xFFu;
    a.fast_delim = csv_delim_fast(prm->delimiter, prm->value_type);
    a.tile_cnt = tile_cnt;
    a.tile_base = tile_base;
    a.offset = out->offset;
    a.label = out->label;
    a.weight = out->weight;
    a.index = out->index;
    a.value = out->value;
    for (int i = 0; i < 8; ++i) a.cap[i] = out->cap[i];
    a.chunk_tab = d_chunk_table ? d_chunk_table : chunk_sink;
    a.err = reinterpret_cast<unsigned long long *>(res + 8);
    a.gate = ctl;
    a.rec = rec;
    a.rec_win = rec ? rec_win : 0;
    dmlc_amd::FastCsvArgs f;
    std::memset(&f, 0, sizeof(f));
    f.text = a.text;
    f.n = nbytes;
    f.cs = ucs;
    f.nchunk = (int)nunits;
    f.ntiles = (uint32_t)nft;
    f.wide = a.wide;
    f.delim = a.delim;
    f.skip_if_gated = phase == dmlc_amd::kPhaseFill;
    f.label_col = prm->label_column;
    // the weight column is ordinary for integer DTypes (csv_parser.h:113-114)
    f.weight_col = prm->value_type == DMLC_AMD_F32 ? prm->weight_column : -1;
    f.vtype = prm->value_type;
    f.label = reinterpret_cast<float *>(out->label);
    f.weight = out->weight;
    f.labsum = labsum;
    f.offset = a.offset;
    f.index = a.index;
    f.value = a.value;
    for (int i = 0; i < 8; ++i) f.cap[i] = out->cap[i];
    f.chunk_tab = d_chunk_table;
    f.lb = lb;
    f.gate = ctl;
    f.err = ferr;
    f.res = res;
    // the uniform-grammar CSV kernels: float values with the label / weight
    // columns they take, or integer values without a label column; a
    // delimiter the number decoders cannot consume (csv_fast.h)
    const bool cols_ok = prm->value_type == DMLC_AMD_F32
                             ? dmlc_amd::csv_fast_columns_ok(prm->label_column, prm->weight_column)
                             : dmlc_amd::csv_fast_int_ok(prm->label_column);
    const bool use_fast = nbytes > 0 && cols_ok && a.fast_delim && !(prm->flags & DMLC_AMD_FLAG_EXACT);
    e = dmlc_amd::launch_csv(a, f, use_fast, res, phase, s);
  } else {  // DMLC_AMD_LIBFM
    dmlc_amd::LibfmArgs a;
    std::memset(&a, 0, sizeof(a));
    a.text = reinterpret_cast<const uint8_t *>(d_text);
    a.n = nbytes;
    a.cs = ucs;
    a.nchunk = (int)nunits;
    a.ul = ul;
    a.tile_bytes = T;
    a.ntiles = (uint32_t)ntiles;
    a.wide = prm->index_bits == 64;
    a.indexing_mode = prm->indexing_mode;
    a.tile_cnt = tile_cnt;
    a.tile_base = tile_base;
    a.offset = out->offset;
    a.label = reinterpret_cast<float *>(out->label);
    a.weight = out->weight;
    a.index = out->index;
    a.field = out->field;
    a.value = reinterpret_cast<float *>(out->value);
    for (int i = 0; i < 8; ++i) a.cap[i] = out->cap[i];
    a.chunk_tab = d_chunk_table ? d_chunk_table : chunk_sink;
    a.chunk_min = chunk_min;
    a.err = reinterpret_cast<unsigned long long *>(res + 8);
    a.gate = ctl;
    a.rec = rec;
    a.rec_meta = rec_meta;
    a.rec_win = rec ? rec_win : 0;
    dmlc_amd::FastSvmArgs f;  // the single-pass kernel with the libfm roles (svm_fast.h)
    std::memset(&f, 0, sizeof(f));
    f.text = a.text;
    f.n = nbytes;
    f.cs = ucs;
    f.nchunk = (int)nunits;
    f.ntiles = (uint32_t)nft;
    f.wide = a.wide;
    f.indexing_mode = prm->indexing_mode;
    f.skip_if_gated = phase == dmlc_amd::kPhaseFill;
    f.offset = a.offset;
    f.label = a.label;
    f.weight = a.weight;
    f.index = a.index;
    f.field = a.field;
    f.value = a.value;
    for (int i = 0; i < 8; ++i) f.cap[i] = out->cap[i];
    f.chunk_tab = prm->indexing_mode < 0 ? a.chunk_tab : d_chunk_table;  // as libsvm's
    f.lb = lb;
    f.umin = fast_min;
    f.gate = ctl;
    f.err = ferr;
    f.res = res;
    const bool use_fast = nbytes > 0 && !(prm->flags & DMLC_AMD_FLAG_EXACT);
    e = dmlc_amd::launch_libfm(a, f, use_fast, res, phase, s);
  }
  if (e == hipSuccess && (prm->flags & DMLC_AMD_FLAG_MAX_INDEX) && phase != dmlc_amd::kPhaseCount) {
    // NumCol of the reference's BasicRowIter: maxima of what was written
    const int wide = prm->index_bits == 64;
    e = dmlc_amd::launch_max(out->index, wide, res + DMLC_AMD_INDEX, out->cap[DMLC_AMD_INDEX], res + 10, s);
    if (e == hipSuccess)
      e = dmlc_amd::launch_max(out->field, wide, res + DMLC_AMD_FIELD, out->cap[DMLC_AMD_FIELD], res + 11, s);
  }
  g_last_hip = e;
  return e == hipSuccess ? DMLC_AMD_OK : DMLC_AMD_ERR_HIP;
}

const char *dmlc_amd_last_hip_error(void) { return hipGetErrorString(g_last_hip); }

}  // extern "C"
