// hip_engine.h -- the host side of the MI355X parse path: a dmlc::Parser<I,D>
// whose ParseBlock work runs on one or more GPUs through the C ABI
// (include/dmlc_amd.h).  Header-only and written against the public dmlc
// headers alone (dmlc/data.h, dmlc/io.h, dmlc/logging.h), so the same code
// backs this build's own Parser::Create (host/data.cc) and the plugin that
// registers HIP parser types into an unmodified libdmlc (host/hip_plugin.cc).
//
// What it restates from the reference:
//   * TextParserBase::FillData (src/data/text_parser.h:116-155): every chunk
//     of the InputSplit is cut into nthread ranges, each one ParseBlock; the
//     parser's nthread is the reference's min(max(nprocs/2 - 4, 1), 2)
//     (text_parser.h:32-35, data.cc:31,42,53) unless DMLC_AMD_NTHREAD says
//     otherwise;
//   * ParserImpl::Next (src/data/parser.h:32-48): one RowBlock per non-empty
//     range, with RowBlockContainer::GetBlock's checks (row_block.h:171-189)
//     and offset[0] == 0; a block stays valid until the next Next();
//   * ThreadedParser (parser.h:74-137): parsing runs ahead of the consumer;
//     an error raised there surfaces from the consumer's Next() at the block
//     where the reference would raise it;
//   * the parameter checks of LibSVMParserParam / CSVParserParam /
//     LibFMParserParam (unknown key -> error, format must match).
//
// Pipeline: a reader thread fills pinned batches of whole
// chunks (batch_bytes, default 32 MiB) from a ChunkSource; W worker threads
// -- `per_device` per GPU, each with its own HIP stream, so one worker's
// host->device copy overlaps another's parse and device->host copy -- take
// batches in order, run one full dmlc_amd_parse (count and write in one call,
// outputs sized from an upper bound: no host round trip between the passes;
// a capacity overflow re-runs at the exact sizes), and copy the CSR back into
// the batch's own pinned arrays; the consumer takes batches in sequence.
// Several GPUs (DMLC_AMD_DEVICES) share the same queue: the multi-GPU
// dispatcher with host-side concatenation in input order.
#pragma once
#include <hip/hip_runtime_api.h>
#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <limits>
#include <map>
#include <memory>
#include <mutex>
#include <sstream>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "dmlc/data.h"
#include "dmlc/io.h"
#include "dmlc/logging.h"
#include "dmlc_amd.h"
#include "text_split.h"

namespace dmlc_amd {

inline void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw dmlc::Error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

// ------------------------------------------------------------ parameters --

// omp_get_num_procs() of the reference: the processors this process may run on
inline int available_procs() {
  cpu_set_t set;
  if (sched_getaffinity(0, sizeof(set), &set) == 0) return std::max(1, (int)CPU_COUNT(&set));
  const long n = sysconf(_SC_NPROCESSORS_ONLN);
  return n > 0 ? (int)n : 1;
}

// TextParserBase's thread count for the factories' request of 2
// (text_parser.h:32-35, data.cc:31,42,53); DMLC_AMD_NTHREAD overrides it.
inline int reference_nthread(int requested = 2) {
  if (const char *e = std::getenv("DMLC_AMD_NTHREAD")) {
    char *end = nullptr;
    const long v = std::strtol(e, &end, 10);
    if (end && *end == '\0' && v >= 1 && v <= 4096) return (int)v;
    LOG(WARNING) << "DMLC_AMD_NTHREAD='" << e << "' is not a thread count in [1, 4096]; ignored";
  }
  return std::min(std::max(available_procs() / 2 - 4, 1), requested);
}

inline size_t env_bytes(const char *name, size_t dflt, size_t lo) {
  const char *e = std::getenv(name);
  if (!e) return dflt;
  char *end = nullptr;
  const unsigned long long v = std::strtoull(e, &end, 10);
  if (!end || *end != '\0' || end == e || v < lo) {
    LOG(WARNING) << name << "='" << e << "' is not a byte count >= " << lo << "; using " << dflt;
    return dflt;
  }
  return (size_t)v;
}

inline int parse_int_param(const std::string &k, const std::string &v) {
  std::istringstream is(v);
  long x = 0;
  is >> x;
  if (is.fail() || !is.eof() || x < std::numeric_limits<int>::min() || x > std::numeric_limits<int>::max())
    throw dmlc::Error("Invalid Parameter format for " + k + " expect int but value='" + v + "'");
  return (int)x;
}

// The parser argument struct of `format` (LibSVMParserParam, libsvm_parser.h:26-41;
// CSVParserParam, csv_parser.h:26-42; LibFMParserParam, libfm_parser.h:26-40)
// as dmlc_amd_params.
template <typename IndexType, typename DType>
dmlc_amd_params make_params(const std::string &format, const std::map<std::string, std::string> &args) {
  static_assert(sizeof(IndexType) == 4 || sizeof(IndexType) == 8, "IndexType is uint32_t or uint64_t");
  dmlc_amd_params p;
  std::memset(&p, 0, sizeof(p));
  p.index_bits = (int)sizeof(IndexType) * 8;
  p.label_column = -1;
  p.weight_column = -1;
  p.delimiter = ',';
  std::vector<std::string> keys;
  if (format == "libsvm" || format == "libfm") {
    p.format = format == "libsvm" ? DMLC_AMD_LIBSVM : DMLC_AMD_LIBFM;
    keys = {"format", "indexing_mode"};
  } else if (format == "csv") {
    p.format = DMLC_AMD_CSV;
    keys = {"format", "label_column", "delimiter", "weight_column"};
  } else {
    throw dmlc::Error("Unknown data type " + format);
  }
  std::string fmt_arg = format;
  for (const auto &kv : args) {
    if (std::find(keys.begin(), keys.end(), kv.first) == keys.end()) {
      std::string msg = "Cannot find argument '" + kv.first + "', Possible Arguments:\n----------------\n";
      for (const auto &k : keys) msg += k + "\n";
      throw dmlc::Error(msg);
    }
    if (kv.first == "format") fmt_arg = kv.second;
    else if (kv.first == "indexing_mode") p.indexing_mode = parse_int_param(kv.first, kv.second);
    else if (kv.first == "label_column") p.label_column = parse_int_param(kv.first, kv.second);
    else if (kv.first == "weight_column") p.weight_column = parse_int_param(kv.first, kv.second);
    else if (kv.first == "delimiter") p.delimiter = kv.second.empty() ? 0 : (unsigned char)kv.second[0];
  }
  if (fmt_arg != format)
    throw dmlc::Error("Check failed: param_.format == \"" + format + "\" (" + fmt_arg + " vs. " + format + ")");
  if (p.format == DMLC_AMD_CSV && p.label_column == p.weight_column && p.label_column >= 0)
    throw dmlc::Error("Check failed: param_.label_column != param_.weight_column || param_.label_column < 0: "
                      "Must have distinct columns for labels and instance weights");
  if (std::is_same<DType, float>::value) p.value_type = DMLC_AMD_F32;
  else if (std::is_same<DType, int32_t>::value) p.value_type = DMLC_AMD_I32;
  else if (std::is_same<DType, int64_t>::value) p.value_type = DMLC_AMD_I64;
  else throw dmlc::Error("Only float32, int32, and int64 are supported for the time being");
  if (p.format != DMLC_AMD_CSV && p.value_type != DMLC_AMD_F32)
    throw dmlc::Error(format + " parses real_t values only");
  return p;
}

// ---------------------------------------------------------- chunk source --

// Whole InputSplit chunks, read into caller memory (a batch).
class ChunkSource {
 public:
  struct Fill {
    bool end;     // the part is exhausted (the chunks just read, if any, are its last)
    size_t need;  // > 0: not even one chunk fits in cap; call again with cap >= need
  };
  virtual ~ChunkSource() {}
  // Append chunks to dst (capacity cap) until at least max_bytes are there or
  // the next chunk might not fit; each chunk's end offset goes to *ends.
  virtual Fill FillChunks(char *dst, size_t cap, size_t max_bytes, std::vector<uint64_t> *ends) = 0;
  virtual void BeforeFirst() = 0;
  // Sources over mapped files (TextSplit::FillPieces): the chunks as pieces of
  // the mappings instead of a copy, and the mappings for HIP to register.
  // Default: no such form.
  virtual const std::vector<std::pair<const char *, size_t>> *Mappings() { return nullptr; }
  virtual Fill FillPieces(size_t, std::vector<uint64_t> *, std::vector<TextPiece> *) { return Fill{true, 0}; }
};

// Any dmlc::InputSplit (one copy per chunk out of the split's buffer).
class InputSplitSource : public ChunkSource {
 public:
  explicit InputSplitSource(dmlc::InputSplit *split) : split_(split) {}
  Fill FillChunks(char *dst, size_t cap, size_t max_bytes, std::vector<uint64_t> *ends) override {
    size_t pos = 0;
    while (pos < max_bytes) {
      const char *p;
      size_t n;
      if (has_pending_) {
        p = pending_.data();
        n = pending_.size();
      } else {
        if (done_) return Fill{true, 0};
        dmlc::InputSplit::Blob b;
        if (!split_->NextChunk(&b)) {
          done_ = true;
          return Fill{true, 0};
        }
        p = static_cast<const char *>(b.dptr);
        n = b.size;
      }
      if (pos + n > cap) {  // keep it for the next batch
        if (!has_pending_) {
          pending_.assign(p, p + n);
          has_pending_ = true;
        }
        return Fill{false, pos == 0 ? n : 0};
      }
      std::memcpy(dst + pos, p, n);
      pos += n;
      ends->push_back(pos);
      has_pending_ = false;
    }
    return Fill{false, 0};
  }
  void BeforeFirst() override {
    split_->BeforeFirst();
    has_pending_ = done_ = false;
  }

 private:
  std::unique_ptr<dmlc::InputSplit> split_;
  std::vector<char> pending_;
  bool has_pending_ = false, done_ = false;
};

// -------------------------------------------------------------- buffers --

// Process-wide cache of page-locked blocks: pinning is slow (hipHostMalloc
// maps and locks every page), and each parser holds a batch pool of several
// hundred MB, so parsers created one after another (a Parser per file or per
// epoch) reuse the blocks instead of pinning them again.  Blocks are kept for
// the life of the process.
class PinnedCache {
 public:
  static PinnedCache &get() {
    static PinnedCache *c = new PinnedCache();  // never destroyed: no HIP call at process exit
    return *c;
  }
  void *take(size_t bytes, size_t *got) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = free_.lower_bound(bytes);
      if (it != free_.end() && it->first <= 2 * bytes) {
        void *p = it->second;
        *got = it->first;
        free_.erase(it);
        return p;
      }
    }
    void *p = nullptr;
    hip_check(hipHostMalloc(&p, bytes, hipHostMallocPortable), "hipHostMalloc");
    *got = bytes;
    return p;
  }
  void give(void *p, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    free_.emplace(bytes, p);
  }

 private:
  std::mutex mu_;
  std::multimap<size_t, void *> free_;
};

template <typename T>
struct PinnedVec {  // page-locked host array, grown on demand (contents not kept)
  T *p = nullptr;
  size_t cap = 0;
  PinnedVec() = default;
  PinnedVec(const PinnedVec &) = delete;
  PinnedVec &operator=(const PinnedVec &) = delete;
  ~PinnedVec() {
    if (p) PinnedCache::get().give(p, cap * sizeof(T));
  }
  T *reserve(size_t n) {
    if (n > cap) {
      if (p) PinnedCache::get().give(p, cap * sizeof(T));
      size_t got = 0;
      p = static_cast<T *>(PinnedCache::get().take((n + n / 4 + 64) * sizeof(T), &got));
      cap = got / sizeof(T);
    }
    return p;
  }
};

// The same for device arrays, per device: a parser's workers hold a few
// hundred MB of HBM (text, workspace, CSR outputs); hipMalloc / hipFree of
// them cost ~10 ms per parser built and ~10 ms per parser destroyed (hipFree
// synchronises the device), the same order as parsing a 2 GB file
// (DESIGN.md 5.2).  Up to DMLC_AMD_HBM_CACHE_MB per device (default 8192 MiB,
// 0: no cache -- every block goes back to hipFree) are kept for reuse (HBM is
// 288 GB per GPU); blocks past that are freed, and an hipMalloc that fails
// frees the device's idle blocks and tries once more, so memory the cache
// holds never causes an out-of-memory error another allocation would not.
class DevCache {
 public:
  static DevCache &get() {
    static DevCache *c = new DevCache();  // never destroyed: no HIP call at process exit
    return *c;
  }
  // bytes kept per device (DMLC_AMD_HBM_CACHE_MB, read once)
  static size_t cap_bytes() {
    static const size_t cap = [] {
      const char *e = std::getenv("DMLC_AMD_HBM_CACHE_MB");
      if (!e || !*e) return size_t(8) << 30;
      char *end = nullptr;
      const unsigned long long mb = std::strtoull(e, &end, 10);
      if (end == e || *end) throw dmlc::Error(std::string("DMLC_AMD_HBM_CACHE_MB: not a number: ") + e);
      return (size_t)mb << 20;
    }();
    return cap;
  }
  void *take(int dev, size_t bytes, size_t *got) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto &fl = free_[dev];
      auto it = fl.lower_bound(bytes);
      if (it != fl.end() && it->first <= 2 * bytes) {
        void *p = it->second;
        *got = it->first;
        held_[dev] -= it->first;
        fl.erase(it);
        return p;
      }
    }
    void *p = nullptr;
    if (hipMalloc(&p, bytes) != hipSuccess) {
      (void)hipGetLastError();  // (clear the sticky error of the failed call)
      p = nullptr;
      if (trim(dev) == 0) hip_check(hipErrorOutOfMemory, "hipMalloc");
      hip_check(hipMalloc(&p, bytes), "hipMalloc");
    }
    *got = bytes;
    return p;
  }
  // false: not kept (the caller frees it)
  bool give(int dev, void *p, size_t bytes) {
    std::lock_guard<std::mutex> lk(mu_);
    if (held_[dev] + bytes > cap_bytes()) return false;
    free_[dev].emplace(bytes, p);
    held_[dev] += bytes;
    return true;
  }
  // frees the device's idle blocks (the calling thread's current device);
  // returns the bytes freed
  size_t trim(int dev) {
    std::multimap<size_t, void *> fl;
    {
      std::lock_guard<std::mutex> lk(mu_);
      fl.swap(free_[dev]);
      held_[dev] = 0;
    }
    size_t freed = 0;
    for (auto &kv : fl) {
      (void)hipFree(kv.second);
      freed += kv.first;
    }
    return freed;
  }
  // idle non-blocking streams of a device (the calling thread's current one)
  hipStream_t take_stream(int dev) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto &v = streams_[dev];
      if (!v.empty()) {
        hipStream_t s = v.back();
        v.pop_back();
        return s;
      }
    }
    hipStream_t s = nullptr;
    hip_check(hipStreamCreateWithFlags(&s, hipStreamNonBlocking), "hipStreamCreate");
    return s;
  }
  void give_stream(int dev, hipStream_t s) {
    std::lock_guard<std::mutex> lk(mu_);
    streams_[dev].push_back(s);
  }

 private:
  std::map<int, std::vector<hipStream_t>> streams_;
  std::mutex mu_;
  std::map<int, std::multimap<size_t, void *>> free_;
  std::map<int, size_t> held_;
};

struct DevBuf {  // device array, grown on demand (contents not kept)
  void *p = nullptr;
  size_t bytes = 0;
  int dev = -1;  // the device current when it was allocated
  DevBuf() = default;
  DevBuf(const DevBuf &) = delete;
  DevBuf &operator=(const DevBuf &) = delete;
  ~DevBuf() { release(); }
  void release() {
    if (p && !DevCache::get().give(dev, p, bytes)) (void)hipFree(p);
    p = nullptr;
    bytes = 0;
  }
  void *get(size_t n) {
    if (n > bytes) {
      release();
      if (hipGetDevice(&dev) != hipSuccess) throw dmlc::Error("hipGetDevice failed");
      size_t got = 0;
      p = DevCache::get().take(dev, n + n / 4 + 256, &got);
      bytes = got;
    }
    return p;
  }
};

// Counts of one block (a non-empty ParseBlock unit), for consumers that
// concatenate blocks (RowBlockIter) without reading past them.
struct BlockCounts {
  uint64_t rows, labels, weights, qids, entries, fields, values;
};

// One batch of InputSplit chunks and, once parsed, its CSR in pinned memory.
template <typename I, typename D>
struct Batch {
  uint64_t seq = 0;
  PinnedVec<char> text;
  std::vector<TextPiece> pieces;  // the text as pieces of registered mappings (text unused)
  std::vector<std::pair<size_t, size_t>> segs;  // (mapping, segment) the pieces lie in
  PinnedVec<uint64_t> starts;  // nchunks + 1
  size_t nchunks = 0, bytes = 0;
  bool end = false;
  // parse result
  dmlc_amd_result res;
  PinnedVec<uint64_t> off, tab, qid;
  PinnedVec<float> weight;
  PinnedVec<D> label, value;
  PinnedVec<I> index, field;
  std::vector<size_t> boff;  // per-block offsets rebased to 0 (rows + 1 per block)
  std::vector<dmlc::RowBlock<I, D>> blocks;
  std::vector<BlockCounts> counts;
  size_t fail_at = SIZE_MAX;    // blocks handed out before `error` is raised
  size_t fail_unit = SIZE_MAX;  // first failing ParseBlock unit (while building)
  std::string error;
  void clear_result() {
    blocks.clear();
    counts.clear();
    boff.clear();
    fail_at = fail_unit = SIZE_MAX;
    error.clear();
  }
};

// A registered segment of a mapped input file (HipTextParser::PrepPieces).
struct MapSeg {
  const char *p = nullptr;
  size_t len = 0;
  bool reg = false;
  uint64_t last_seq = 0;  // the last batch that used it (unregistered when that one is released)
};

struct EngineConfig {
  dmlc_amd_params prm;
  size_t batch_bytes = 32u << 20;
  std::vector<int> devices;  // empty: the calling thread's current device
  int per_device = 2;        // workers (HIP streams) per device
  int depth = 0;             // parsed batches ahead of the consumer (0: 2 per worker)
  bool max_index = false;    // reduce index/field maxima on the device (RowBlockIter::NumCol)
  bool stats = false;        // DMLC_AMD_STATS=1: per-stage times on stderr when the parser ends
  // H2D / D2H (DMLC_AMD_COPY): "kernel": the text by dmlc_amd_copy,
  // the batch's CSR arrays by one dmlc_amd_copy_n launch; "dma": one
  // hipMemcpyAsync per array.  (Measured on the MI355X box, DESIGN.md 5.2:
  // kernel copies 27 GB/s end to end, DMA 17 GB/s, and DMA with the CSR
  // gathered on the device into one D2H copy 18 GB/s -- although the SDMA
  // engines run both directions of 1 GiB copies at 97 GB/s together,
  // tools/e2e/link_probe.py)
  // "h2d_kernel" / "d2h_kernel": one direction by kernel, the other by DMA
  // (the SDMA engines and the copy kernels then carry different directions).
  // Default "d2h_kernel" (round 4: 28.8-30.3 GB/s against 25.7-28.4 for
  // "kernel" over two sweeps on config 2, profiles/r4_e2e_sweep_r4*.txt).
  enum CopyMode { kKernel, kDma, kH2DKernel, kD2HKernel } copy_mode = kD2HKernel;
  // DMLC_AMD_PRECOPY=0: the CSR copy-out waits for the parse's result on the
  // host (sizes exact) instead of being queued behind the parse with sizes
  // read on the device (dmlc_amd_copy_n_dev) -- for A/B timing
  bool precopy = true;
  bool h2d_kernel() const { return copy_mode == kKernel || copy_mode == kH2DKernel; }
  bool d2h_kernel() const { return copy_mode == kKernel || copy_mode == kD2HKernel; }

  // batch size, devices and workers from the environment
  // (DMLC_AMD_BATCH_BYTES, DMLC_AMD_DEVICES = "0,1,..." | "all", DMLC_AMD_WORKERS)
  void from_env() {
    batch_bytes = env_bytes("DMLC_AMD_BATCH_BYTES", batch_bytes, 1u << 20);
    if (const char *w = std::getenv("DMLC_AMD_WORKERS")) per_device = std::max(1, std::atoi(w));
    if (const char *st = std::getenv("DMLC_AMD_STATS")) stats = std::atoi(st) != 0;
    if (const char *pc = std::getenv("DMLC_AMD_PRECOPY")) precopy = std::atoi(pc) != 0;
    if (const char *c = std::getenv("DMLC_AMD_COPY")) {
      const std::string v(c);
      if (v == "kernel") copy_mode = kKernel;
      else if (v == "dma") copy_mode = kDma;
      else if (v == "h2d_kernel") copy_mode = kH2DKernel;
      else if (v == "d2h_kernel") copy_mode = kD2HKernel;
      else throw dmlc::Error("DMLC_AMD_COPY: expected kernel, dma, h2d_kernel or d2h_kernel, got " + v);
    }
    if (const char *d = std::getenv("DMLC_AMD_DEVICES")) {
      devices.clear();
      int n = 0;
      hip_check(hipGetDeviceCount(&n), "hipGetDeviceCount");
      if (std::string(d) == "all") {
        for (int i = 0; i < n; ++i) devices.push_back(i);
      } else {
        std::istringstream is(d);
        std::string tok;
        while (std::getline(is, tok, ',')) {
          const int dev = parse_int_param("DMLC_AMD_DEVICES", tok);
          if (dev < 0 || dev >= n) throw dmlc::Error("DMLC_AMD_DEVICES: no HIP device " + tok);
          devices.push_back(dev);
        }
      }
    }
  }
};

// ---------------------------------------------------------------- engine --

template <typename IndexType, typename DType>
class HipTextParser : public dmlc::Parser<IndexType, DType> {
 public:
  using Block = dmlc::RowBlock<IndexType, DType>;
  using B = Batch<IndexType, DType>;

  HipTextParser(ChunkSource *source, const EngineConfig &cfg) : src_(source), cfg_(cfg) {
    if (cfg_.devices.empty()) {
      int dev = 0;
      hip_check(hipGetDevice(&dev), "hipGetDevice");
      cfg_.devices.push_back(dev);
    }
    const int nworkers = (int)cfg_.devices.size() * std::max(1, cfg_.per_device);
    const int depth = cfg_.depth > 0 ? cfg_.depth : 2 * nworkers;
    for (int i = 0; i < nworkers + depth + 1; ++i) pool_.emplace_back(new B());
    for (int i = 0; i < nworkers; ++i) workers_.emplace_back(new Worker(cfg_.devices[i % cfg_.devices.size()]));
    RegisterMappings();
    Start();
  }
  ~HipTextParser() override {
    const Clock clk;
    Stop();
    const uint64_t stop_ns = clk.ns();
    if (cfg_.stats) PrintStats();
    workers_.clear();  // streams and HBM blocks back to DevCache, pinned blocks to PinnedCache
    pool_.clear();
    UnregisterAll();
    if (cfg_.stats) {
      std::fprintf(stderr, "{\"dmlc_amd_teardown\": {\"stop_s\": %.4f, \"free_s\": %.4f}}\n", stop_ns * 1e-9,
                   (clk.ns() - stop_ns) * 1e-9);
    }
  }

  void BeforeFirst() override {
    Stop();
    src_->BeforeFirst();
    Start();
  }

  bool Next() override {
    for (;;) {
      if (cur_ != nullptr) {
        if (blk_ < cur_->blocks.size() && blk_ < cur_->fail_at) {
          block_ = cur_->blocks[blk_];
          counts_ = cur_->counts[blk_];
          ++blk_;
          return true;
        }
        if (!cur_->error.empty()) throw dmlc::Error(cur_->error);
        const bool end = cur_->end;
        Release(cur_);
        cur_ = nullptr;
        if (end) {
          finished_ = true;
          return false;
        }
      }
      if (finished_) return false;
      cur_ = Take();
      blk_ = 0;
      bytes_read_ += cur_->bytes;
    }
  }

  const Block &Value() const override { return block_; }
  size_t BytesRead() const override { return bytes_read_; }

  // ---- for in-process consumers (RowBlockIter)
  const BlockCounts &ValueCounts() const { return counts_; }
  // index / field maxima of the batch holding the current block (cfg.max_index)
  uint64_t BatchMaxIndex() const { return cur_ ? cur_->res.max_index : 0; }
  uint64_t BatchMaxField() const { return cur_ ? cur_->res.max_field : 0; }
  bool BlockStartsBatch() const { return blk_ == 1; }

 private:
  struct Worker {
    explicit Worker(int d) : device(d) {}
    // runs on whichever thread destroys the parser: switch to the worker's
    // device for its stream and events, then give the caller its device back
    ~Worker() {
      if (stream) {
        int prev = -1;
        const bool have_prev = hipGetDevice(&prev) == hipSuccess;
        (void)hipSetDevice(device);
        for (auto &e : ev)
          if (e) (void)hipEventDestroy(e);
        (void)hipStreamSynchronize(stream);  // (idle: each batch ends with a sync)
        DevCache::get().give_stream(device, stream);
        if (have_prev && prev != device) (void)hipSetDevice(prev);
      }
    }
    int device;
    hipStream_t stream = nullptr;
    hipEvent_t ev[4] = {nullptr, nullptr, nullptr, nullptr};  // stats: H2D | parse | D2H boundaries
    DevBuf text, cs, res, tab, ws, off, label, weight, qid, index, field, value;
    uint64_t cap[7] = {0, 0, 0, 0, 0, 0, 0};
    uint64_t est[8] = {0, 0, 0, 0, 0, 0, 0, 0};  // copy-out bytes per CSR array, from earlier batches
    PinnedVec<dmlc_amd_result> hres;
  };

  // ---- threads
  void Start() {
    stop_ = false;
    reader_done_ = false;
    finished_ = false;
    read_error_.clear();
    free_.clear();
    todo_.clear();
    done_.clear();
    for (auto &b : pool_) free_.push_back(b.get());
    next_read_ = next_take_ = 0;
    cur_ = nullptr;
    blk_ = 0;
    bytes_read_ = 0;
    reader_ = std::thread([this] { ReadLoop(); });
    for (auto &w : workers_) {
      Worker *wp = w.get();
      threads_.emplace_back([this, wp] { WorkLoop(wp); });
    }
  }
  void Stop() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (reader_.joinable()) reader_.join();
    for (auto &t : threads_)
      if (t.joinable()) t.join();
    threads_.clear();
  }

  // ---- pipeline statistics (DMLC_AMD_STATS): seconds summed over batches;
  // the worker stages overlap each other and the reader, so the sums exceed
  // the wall time.  Device stages are timed with HIP events on each stream.
  enum { S_READ, S_H2D, S_PARSE, S_D2H, S_BUILD, S_WAIT, S_N };
  std::atomic<uint64_t> stat_ns_[S_N] = {};
  std::atomic<uint64_t> stat_batches_{0};
  bool pieces_ = false;  // batches as pieces of registered mappings (RegisterMappings)
  bool keep_ = false;    // registrations kept until the parser ends (RegisterMappings)
  std::vector<std::pair<const char *, size_t>> maps_;
  std::vector<std::vector<MapSeg>> segs_;  // per mapping, its 64 MiB segments
  std::mutex seg_mu_;
  struct Clock {
    std::chrono::steady_clock::time_point t0 = std::chrono::steady_clock::now();
    uint64_t ns() const {
      return (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
          .count();
    }
  };
  void PrintStats() const {
    static const char *kName[S_N] = {"read", "h2d", "parse", "d2h", "blocks", "consumer_wait"};
    std::string line = "{\"dmlc_amd_stats\": {\"batches\": " + std::to_string(stat_batches_.load()) +
                       ", \"workers\": " + std::to_string(workers_.size());
    for (int i = 0; i < S_N; ++i) {
      char buf[64];
      std::snprintf(buf, sizeof(buf), ", \"%s_s\": %.4f", kName[i], stat_ns_[i].load() * 1e-9);
      line += buf;
    }
    std::fprintf(stderr, "%s}}\n", line.c_str());
  }

  // Text from the page cache by DMA (round 6): when the source
  // maps its files, each batch's text goes to HBM as hipMemcpyAsync pieces of
  // the mappings -- no pread into a pinned block, so a host byte of text is
  // read once (by the DMA) instead of read, written and read again.  The
  // mappings are registered with HIP (read-only, portable) in 64 MiB
  // segments as the reader reaches them, and a segment is unregistered when
  // the last batch that used it is released, so the pinned part of the page
  // cache follows the pipeline instead of the whole input.  A batch whose
  // segment cannot be registered is staged through its pinned block
  // (memcpy) instead; DMLC_AMD_MMAP=0 keeps the pinned-copy form throughout.
  size_t seg_bytes_ = size_t(64) << 20;        // DMLC_AMD_MMAP_SEG_MB (A/B)
  unsigned reg_flags_ = hipHostRegisterReadOnly;  // + Portable when batches go to several devices
  void RegisterMappings() {
    const auto *maps = src_->Mappings();
    if (!maps || maps->empty()) return;
    const char *e = std::getenv("DMLC_AMD_MMAP");
    if (!e || e[0] != '1') return;  // opt-in (registration costs more than the copy it saves at 1 GPU)
    if (const char *sm = std::getenv("DMLC_AMD_MMAP_SEG_MB")) seg_bytes_ = (size_t)std::max(1, std::atoi(sm)) << 20;
    if (cfg_.devices.size() > 1 || (std::getenv("DMLC_AMD_MMAP_PORTABLE") && std::getenv("DMLC_AMD_MMAP_PORTABLE")[0] == '1'))
      reg_flags_ |= hipHostRegisterPortable;
    // segments stay registered across epochs (BeforeFirst re-reads the same
    // pages) while the input fits DMLC_AMD_MMAP_KEEP_MB (default: an eighth of
    // host memory, at most 64 GiB); past it each is unregistered when its
    // last batch is released
    size_t total = 0;
    for (const auto &m : *maps) total += m.second;
    size_t keep = std::min<size_t>((size_t)sysconf(_SC_PHYS_PAGES) * (size_t)sysconf(_SC_PAGESIZE) / 8,
                                   size_t(64) << 30);
    if (const char *k = std::getenv("DMLC_AMD_MMAP_KEEP_MB")) keep = (size_t)std::strtoull(k, nullptr, 10) << 20;
    keep_ = total <= keep;
    for (const auto &m : *maps) {
      maps_.push_back(m);
      std::vector<MapSeg> sv((m.second + seg_bytes_ - 1) / seg_bytes_);
      for (size_t i = 0; i < sv.size(); ++i) {
        sv[i].p = m.first + i * seg_bytes_;
        sv[i].len = std::min(seg_bytes_, m.second - i * seg_bytes_);
      }
      segs_.push_back(std::move(sv));
    }
    pieces_ = true;
  }
  size_t MapOf(const char *p) const {
    for (size_t i = 0; i < maps_.size(); ++i)
      if (p >= maps_[i].first && p < maps_[i].first + maps_[i].second) return i;
    throw dmlc::Error("dmlc_amd: a text piece outside the split's mappings");
  }
  // Reader: split the batch's pieces at segment boundaries (one registered
  // range per copy) and register the segments it reaches; false: a
  // registration failed (the caller stages the batch instead).
  bool PrepPieces(B *b, uint64_t seq) {
    std::vector<TextPiece> out;
    b->segs.clear();
    for (const TextPiece &pc : b->pieces) {
      if (!pc.src) {
        out.push_back(pc);
        continue;
      }
      const size_t m = MapOf(pc.src);
      const char *base = maps_[m].first;
      uint64_t o = (uint64_t)(pc.src - base), dst = pc.off;
      const uint64_t e = o + pc.len;
      while (o < e) {
        const uint64_t sg = o / seg_bytes_, se = std::min<uint64_t>(e, (sg + 1) * seg_bytes_);
        out.push_back(TextPiece{dst, base + o, se - o});
        dst += se - o;
        if (b->segs.empty() || b->segs.back() != std::make_pair(m, (size_t)sg)) b->segs.emplace_back(m, (size_t)sg);
        o = se;
      }
    }
    b->pieces.swap(out);
    std::lock_guard<std::mutex> lk(seg_mu_);
    for (const auto &ms : b->segs) {
      MapSeg &g = segs_[ms.first][ms.second];
      if (!g.reg) {
        if (hipHostRegister(const_cast<char *>(g.p), g.len, reg_flags_) !=
            hipSuccess) {
          (void)hipGetLastError();
          return false;
        }
        g.reg = true;
      }
      g.last_seq = seq;
    }
    return true;
  }
  // the batch's text gathered into its pinned block (a segment that could not be registered)
  void StagePieces(B *b) {
    b->text.reserve(b->bytes + 1);
    for (const TextPiece &pc : b->pieces) {
      if (pc.src) std::memcpy(b->text.p + pc.off, pc.src, pc.len);
      else b->text.p[pc.off] = '\n';
    }
    b->pieces.clear();
  }
  void ReleaseSegs(B *b) {
    if (b->segs.empty()) return;
    if (keep_) {  // kept for the next epoch; UnregisterAll at the end
      b->segs.clear();
      return;
    }
    std::lock_guard<std::mutex> lk(seg_mu_);
    for (const auto &ms : b->segs) {
      MapSeg &g = segs_[ms.first][ms.second];
      if (g.reg && g.last_seq == b->seq) {
        (void)hipHostUnregister(const_cast<char *>(g.p));
        g.reg = false;
      }
    }
    b->segs.clear();
  }
  void UnregisterAll() {
    std::lock_guard<std::mutex> lk(seg_mu_);
    for (auto &sv : segs_)
      for (MapSeg &g : sv)
        if (g.reg) {
          (void)hipHostUnregister(const_cast<char *>(g.p));
          g.reg = false;
        }
  }

  void ReadLoop() {
    try {
      std::vector<uint64_t> ends;
      for (;;) {
        B *b;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return stop_ || !free_.empty(); });
          if (stop_) return;
          b = free_.back();
          free_.pop_back();
        }
        b->clear_result();
        const Clock clk;
        // room for one more whole chunk past the target (8 MiB InputSplit buffers)
        size_t cap = cfg_.batch_bytes + (16u << 20);
        if (!pieces_) b->text.reserve(cap);
        ends.clear();
        ChunkSource::Fill f;
        b->pieces.clear();
        if (pieces_) {
          f = src_->FillPieces(cfg_.batch_bytes, &ends, &b->pieces);
        } else {
          for (;;) {
            f = src_->FillChunks(b->text.p, b->text.cap, cfg_.batch_bytes, &ends);
            if (f.need == 0) break;
            b->text.reserve(f.need + (16u << 20));  // a record longer than the room: grow, retry
          }
        }
        b->nchunks = ends.size();
        b->starts.reserve(ends.size() + 1);
        b->starts.p[0] = 0;
        for (size_t i = 0; i < ends.size(); ++i) b->starts.p[i + 1] = ends[i];
        b->bytes = ends.empty() ? 0 : ends.back();
        b->end = f.end;
        if (!b->pieces.empty()) {  // (only the reader advances next_read_)
          uint64_t seq;
          {
            std::lock_guard<std::mutex> lk(mu_);
            seq = next_read_;
          }
          if (!PrepPieces(b, seq)) StagePieces(b);
        }
        if (cfg_.stats) stat_ns_[S_READ] += clk.ns();
        {
          std::lock_guard<std::mutex> lk(mu_);
          b->seq = next_read_++;
          todo_.push_back(b);
          if (b->end) reader_done_ = true;
        }
        cv_.notify_all();
        if (b->end) return;
      }
    } catch (const std::exception &e) {
      std::lock_guard<std::mutex> lk(mu_);
      read_error_ = e.what();
      reader_done_ = true;
      cv_.notify_all();
    }
  }

  void WorkLoop(Worker *w) {
    bool ready = false;
    for (;;) {
      B *b;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return stop_ || !todo_.empty(); });
        if (stop_) return;
        b = todo_.front();
        todo_.pop_front();
      }
      try {
        if (!ready) {
          hip_check(hipSetDevice(w->device), "hipSetDevice");
          if (!w->stream) w->stream = DevCache::get().take_stream(w->device);
          ready = true;
        }
        if (b->nchunks > 0) Parse(w, b);
      } catch (const std::exception &e) {
        b->error = e.what();
        b->fail_at = 0;
        // kernels queued before the throw may still use this worker's HBM
        // blocks: drain them before the blocks can go to another worker
        if (w->stream) (void)hipStreamSynchronize(w->stream);
      }
      {
        std::lock_guard<std::mutex> lk(mu_);
        done_[b->seq] = b;
      }
      cv_.notify_all();
    }
  }

  B *Take() {
    const Clock clk;
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [&] { return done_.count(next_take_) || (!read_error_.empty() && next_take_ >= next_read_); });
    if (cfg_.stats) stat_ns_[S_WAIT] += clk.ns();
    auto it = done_.find(next_take_);
    if (it == done_.end()) throw dmlc::Error(read_error_);
    B *b = it->second;
    done_.erase(it);
    ++next_take_;
    return b;
  }
  void Release(B *b) {
    ReleaseSegs(b);  // (in sequence order: Take hands batches out in order)
    {
      std::lock_guard<std::mutex> lk(mu_);
      free_.push_back(b);
    }
    cv_.notify_all();
  }

  // ---- one batch on one device
  static uint64_t bound_of(size_t bytes) { return bytes / 2 + 2; }  // any slot's count, any format

  void Parse(Worker *w, B *b) {
    const hipStream_t s = w->stream;
    const int nch = (int)b->nchunks;
    const int upc = cfg_.prm.nthread > 1 ? cfg_.prm.nthread : 1;
    const size_t nunits = (size_t)nch * upc;
    void *d_text = w->text.get(b->bytes);
    uint64_t *d_cs = static_cast<uint64_t *>(w->cs.get((nch + 1) * 8));
    uint64_t *d_res = static_cast<uint64_t *>(w->res.get(sizeof(dmlc_amd_result)));
    uint64_t *d_tab = static_cast<uint64_t *>(w->tab.get(nunits * 64));
    dmlc_amd_result *hres = w->hres.reserve(1);
    const bool st = cfg_.stats;
    if (st && !w->ev[0])
      for (auto &e : w->ev) hip_check(hipEventCreate(&e), "hipEventCreate");
    if (st) hip_check(hipEventRecord(w->ev[0], s), "hipEventRecord");
    if (!b->pieces.empty()) {  // DMA straight from the registered mappings; inserted '\n's by memset
      for (const TextPiece &pc : b->pieces) {
        char *dst = static_cast<char *>(d_text) + pc.off;
        if (pc.src) hip_check(hipMemcpyAsync(dst, pc.src, pc.len, hipMemcpyHostToDevice, s), "H2D piece");
        else hip_check(hipMemsetAsync(dst, '\n', 1, s), "H2D newline");
      }
    } else {
      H2D(d_text, b->text.p, b->bytes, s);
    }
    hip_check(hipMemcpyAsync(d_cs, b->starts.p, (nch + 1) * 8, hipMemcpyHostToDevice, s), "H2D chunk starts");
    if (st) hip_check(hipEventRecord(w->ev[1], s), "hipEventRecord");
    dmlc_amd_params p = cfg_.prm;
    p.flags = cfg_.max_index ? DMLC_AMD_FLAG_MAX_INDEX : 0u;
    const size_t ws = dmlc_amd_workspace_bytes(b->bytes, nch, &p);
    void *d_ws = w->ws.get(ws);
    const uint64_t ub = bound_of(b->bytes);
    uint64_t want[7];
    for (int i = 0; i < 7; ++i) want[i] = std::max<uint64_t>(w->cap[i], ub);
    dmlc_amd_csr out;
    // The CSR copy-out by kernel is queued right behind the parse with its
    // sizes read on the device (dmlc_amd_copy_n_dev), into host arrays sized
    // from the worker's earlier batches: no host round trip between the parse
    // and the copy.  A batch larger than the estimate copies again after the
    // sync with its exact sizes.
    const size_t isz = sizeof(IndexType), dsz = sizeof(DType);
    const int kSlot[8] = {DMLC_AMD_ROWS, DMLC_AMD_LABEL, DMLC_AMD_WEIGHT, DMLC_AMD_QID,
                          DMLC_AMD_INDEX, DMLC_AMD_FIELD, DMLC_AMD_VALUE, -1};
    const uint64_t kScale[8] = {8, dsz, 4, 8, isz, isz, dsz, 0};
    const uint64_t kAdd[8] = {8, 0, 0, 0, 0, 0, 0, (uint64_t)nunits * 64};
    bool pre = false;  // the copy-out went with the parse
    uint64_t pre_max[8];
    void *pre_dst[8];
    for (int attempt = 0;; ++attempt) {
      Outputs(w, want, &out);
      CheckRc(dmlc_amd_parse(d_text, b->bytes, d_cs, nch, &p, &out, d_tab, d_ws, ws,
                             reinterpret_cast<dmlc_amd_result *>(d_res), s));
      // stats: the parse / D2H boundary right after the parse (the queued
      // copy-out and the result block count as D2H)
      if (st) hip_check(hipEventRecord(w->ev[2], s), "hipEventRecord");
      pre = attempt == 0 && cfg_.precopy && cfg_.d2h_kernel() && w->est[0] > 0;
      if (pre) {
        const void *src[8] = {out.offset, out.label, out.weight, out.qid, out.index, out.field, out.value, d_tab};
        pre_dst[0] = b->off.reserve(w->est[0] / 8 + 1);
        pre_dst[1] = b->label.reserve(w->est[1] / dsz + 1);
        pre_dst[2] = b->weight.reserve(w->est[2] / 4 + 1);
        pre_dst[3] = b->qid.reserve(w->est[3] / 8 + 1);
        pre_dst[4] = b->index.reserve(w->est[4] / isz + 1);
        pre_dst[5] = b->field.reserve(w->est[5] / isz + 1);
        pre_dst[6] = b->value.reserve(w->est[6] / dsz + 1);
        pre_dst[7] = b->tab.reserve(nunits * 8);
        // (an output the format does not have -- a NULL array -- is not copied)
        for (int i = 0; i < 8; ++i) pre_max[i] = !src[i] ? 0 : i == 7 ? (uint64_t)nunits * 64 : w->est[i];
        CheckRc(dmlc_amd_copy_n_dev(pre_dst, src, d_res, kSlot, kScale, kAdd, pre_max, 8, s));
      }
      hip_check(hipMemcpyAsync(hres, d_res, sizeof(dmlc_amd_result), hipMemcpyDeviceToHost, s), "D2H result");
      hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
      if ((hres->error & 0xFFFF) != DMLC_AMD_ERR_CAPACITY) break;
      if (attempt > 0) throw dmlc::Error("dmlc_amd_parse: output capacity exceeded at exact sizes");
      for (int i = 0; i < 7; ++i) want[i] = std::max<uint64_t>(want[i], hres->count[i]);  // exact: one re-run
    }
    b->res = *hres;
    const uint64_t *c = b->res.count;
    if (b->res.error) {  // the reference's ParseBlock raised inside this chunk
      const uint64_t pos = b->res.error >> 16;
      size_t chunk = 0;
      while (chunk + 1 < b->nchunks && b->starts.p[chunk + 1] <= pos) ++chunk;
      b->error = dmlc_amd_error_string((int)(b->res.error & 0xFFFF));
      b->fail_unit = chunk * upc;  // FillData rethrows for the whole chunk (text_parser.h:151)
    } else {
      b->fail_unit = SIZE_MAX;
    }
    // the CSR to the host: offsets, labels, weights, qids, indices, fields,
    // values, unit table
    const void *src[8] = {out.offset, out.label, out.weight, out.qid, out.index, out.field, out.value, d_tab};
    const uint64_t nb[8] = {(c[DMLC_AMD_ROWS] + 1) * 8, c[DMLC_AMD_LABEL] * sizeof(DType), c[DMLC_AMD_WEIGHT] * 4,
                            c[DMLC_AMD_QID] * 8, c[DMLC_AMD_INDEX] * sizeof(IndexType),
                            c[DMLC_AMD_FIELD] * sizeof(IndexType), c[DMLC_AMD_VALUE] * sizeof(DType),
                            (uint64_t)nunits * 64};
    void *dst[8] = {b->off.reserve(c[DMLC_AMD_ROWS] + 1), b->label.reserve(c[DMLC_AMD_LABEL] + 1),
                    b->weight.reserve(c[DMLC_AMD_WEIGHT] + 1), b->qid.reserve(c[DMLC_AMD_QID] + 1),
                    b->index.reserve(c[DMLC_AMD_INDEX] + 1), b->field.reserve(c[DMLC_AMD_FIELD] + 1),
                    b->value.reserve(c[DMLC_AMD_VALUE] + 1), b->tab.reserve(nunits * 8)};
    bool again = !pre;
    for (int i = 0; i < 8; ++i) {
      again = again || nb[i] > pre_max[i] || (nb[i] && dst[i] != pre_dst[i]);
      if (nb[i]) w->est[i] = std::max<uint64_t>(w->est[i], (nb[i] + nb[i] / 4 + 4095) & ~uint64_t(15));
    }
    if (again) {
      if (cfg_.d2h_kernel()) CheckRc(dmlc_amd_copy_n(dst, src, nb, 8, s));
      else
        for (int i = 0; i < 8; ++i) D2H(dst[i], src[i], nb[i], s);
    }
    if (st) hip_check(hipEventRecord(w->ev[3], s), "hipEventRecord");
    if (again) hip_check(hipStreamSynchronize(s), "hipStreamSynchronize");
    else if (st) hip_check(hipEventSynchronize(w->ev[3]), "hipEventSynchronize");
    const Clock clk;
    BuildBlocks(b, nunits, upc);
    if (st) {
      float ms[3] = {0, 0, 0};
      for (int i = 0; i < 3; ++i) hip_check(hipEventElapsedTime(&ms[i], w->ev[i], w->ev[i + 1]), "hipEventElapsedTime");
      stat_ns_[S_H2D] += (uint64_t)(ms[0] * 1e6);
      stat_ns_[S_PARSE] += (uint64_t)(ms[1] * 1e6);
      stat_ns_[S_D2H] += (uint64_t)(ms[2] * 1e6);
      stat_ns_[S_BUILD] += clk.ns();
      ++stat_batches_;
    }
  }

  // Bulk copies between the batch's page-locked arrays and HBM: by kernel
  // (dmlc_amd_copy) unless DMLC_AMD_COPY=dma
  void H2D(void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    if (cfg_.h2d_kernel()) CheckRc(dmlc_amd_copy(dst, src, bytes, s));
    else hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, s), "H2D");
  }
  void D2H(void *dst, const void *src, size_t bytes, hipStream_t s) {
    if (!bytes) return;
    if (cfg_.d2h_kernel()) CheckRc(dmlc_amd_copy(dst, src, bytes, s));
    else hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, s), "D2H");
  }

  void Outputs(Worker *w, const uint64_t *want, dmlc_amd_csr *out) {
    std::memset(out, 0, sizeof(*out));
    const bool csv = cfg_.prm.format == DMLC_AMD_CSV, fm = cfg_.prm.format == DMLC_AMD_LIBFM;
    const size_t vs = sizeof(DType), is = sizeof(IndexType);
    for (int i = 0; i < 7; ++i) w->cap[i] = want[i];
    out->offset = static_cast<uint64_t *>(w->off.get((want[DMLC_AMD_ROWS] + 1) * 8));
    out->label = w->label.get((want[DMLC_AMD_LABEL] + 1) * vs);
    out->weight = static_cast<float *>(w->weight.get((want[DMLC_AMD_WEIGHT] + 1) * 4));
    out->qid = csv || fm ? nullptr : static_cast<uint64_t *>(w->qid.get((want[DMLC_AMD_QID] + 1) * 8));
    out->index = w->index.get((want[DMLC_AMD_INDEX] + 1) * is);
    out->field = fm ? w->field.get((want[DMLC_AMD_FIELD] + 1) * is) : nullptr;
    out->value = w->value.get((want[DMLC_AMD_VALUE] + 1) * vs);
    for (int i = 0; i < 7; ++i) out->cap[i] = want[i];
    if (!out->qid) out->cap[DMLC_AMD_QID] = 0;
    if (!out->field) out->cap[DMLC_AMD_FIELD] = 0;
  }

  static void CheckRc(int rc) {
    if (rc == DMLC_AMD_OK) return;
    throw dmlc::Error(std::string("dmlc_amd_parse: ") + dmlc_amd_error_string(rc) +
                      (rc == DMLC_AMD_ERR_HIP ? std::string(" (") + dmlc_amd_last_hip_error() + ")" : ""));
  }

  // RowBlocks of the non-empty units, with the checks the reference applies:
  // ParseBlock's own (CSV label / weight counts, csv_parser.h:147-148; libfm
  // field == index, libfm_parser.h:127) fail the whole chunk; GetBlock's
  // (row_block.h:173-178) fail when the consumer reaches that block.
  void BuildBlocks(B *b, size_t nunits, int upc) {
    const uint64_t *tot = b->res.count;
    const bool csv = cfg_.prm.format == DMLC_AMD_CSV, fm = cfg_.prm.format == DMLC_AMD_LIBFM;
    size_t fail_unit = b->fail_unit;
    std::string fail_msg = b->error;
    auto fail = [&](size_t unit, const std::string &m) {
      if (unit < fail_unit) {
        fail_unit = unit;
        fail_msg = m;
      }
    };
    b->boff.reserve(tot[DMLC_AMD_ROWS] + nunits);
    b->boff.clear();
    std::vector<size_t> unit_of_block;
    for (size_t u = 0; u < nunits; ++u) {
      const uint64_t *r0 = b->tab.p + u * 8;
      const uint64_t *r1 = u + 1 < nunits ? b->tab.p + (u + 1) * 8 : tot;
      BlockCounts k;
      k.rows = r1[DMLC_AMD_ROWS] - r0[DMLC_AMD_ROWS];
      k.entries = r1[DMLC_AMD_INDEX] - r0[DMLC_AMD_INDEX];
      k.values = r1[DMLC_AMD_VALUE] - r0[DMLC_AMD_VALUE];
      k.labels = r1[DMLC_AMD_LABEL] - r0[DMLC_AMD_LABEL];
      k.weights = r1[DMLC_AMD_WEIGHT] - r0[DMLC_AMD_WEIGHT];
      k.qids = r1[DMLC_AMD_QID] - r0[DMLC_AMD_QID];
      k.fields = r1[DMLC_AMD_FIELD] - r0[DMLC_AMD_FIELD];
      const size_t chunk_unit = (u / upc) * upc;
      if (fm && k.fields != k.entries) fail(chunk_unit, "Check failed: out->field.size() == out->index.size()");
      if (csv && k.labels != 0 && k.labels != k.rows)
        fail(chunk_unit, "Check failed: out->label.size() == 0 || out->label.size() + 1 == out->offset.size()");
      if (csv && k.weights != 0 && k.weights != k.rows)
        fail(chunk_unit, "Check failed: out->weight.size() == 0 || out->weight.size() + 1 == out->offset.size()");
      if (k.rows == 0) continue;  // an empty container is no block (parser.h:36-38)
      if (k.labels != 0 && k.labels != k.rows) fail(u, "Check failed: label.size() + 1 == offset.size()");
      if (k.values != 0 && k.values != k.entries)
        fail(u, "Check failed: offset.back() == value.size() || value.size() == 0");
      // offsets of this block rebased to 0, as GetBlock's container holds them
      const size_t ob = b->boff.size();
      const uint64_t *o = b->off.p + r0[DMLC_AMD_ROWS];
      for (uint64_t i = 0; i <= k.rows; ++i) b->boff.push_back((size_t)(o[i] - o[0]));
      Block blk;
      blk.size = k.rows;
      blk.offset = reinterpret_cast<const size_t *>(ob);  // patched below (boff may still grow)
      blk.label = k.labels ? b->label.p + r0[DMLC_AMD_LABEL] : nullptr;
      blk.weight = k.weights ? b->weight.p + r0[DMLC_AMD_WEIGHT] : nullptr;
      blk.qid = k.qids ? b->qid.p + r0[DMLC_AMD_QID] : nullptr;
      blk.field = k.fields ? b->field.p + r0[DMLC_AMD_FIELD] : nullptr;
      blk.index = k.entries ? b->index.p + r0[DMLC_AMD_INDEX] : nullptr;
      blk.value = k.values ? b->value.p + r0[DMLC_AMD_VALUE] : nullptr;
      b->blocks.push_back(blk);
      b->counts.push_back(k);
      unit_of_block.push_back(u);
    }
    for (auto &blk : b->blocks) blk.offset = b->boff.data() + reinterpret_cast<size_t>(blk.offset);
    b->fail_at = SIZE_MAX;
    if (fail_unit != SIZE_MAX) {
      b->error = fail_msg;
      b->fail_at = std::lower_bound(unit_of_block.begin(), unit_of_block.end(), fail_unit) - unit_of_block.begin();
    }
  }

  std::unique_ptr<ChunkSource> src_;
  EngineConfig cfg_;
  std::vector<std::unique_ptr<B>> pool_;
  std::vector<std::unique_ptr<Worker>> workers_;
  std::thread reader_;
  std::vector<std::thread> threads_;
  std::mutex mu_;
  std::condition_variable cv_;
  std::vector<B *> free_;
  std::deque<B *> todo_;
  std::map<uint64_t, B *> done_;
  uint64_t next_read_ = 0, next_take_ = 0;
  bool stop_ = false, reader_done_ = false, finished_ = false;
  std::string read_error_;
  // consumer
  B *cur_ = nullptr;
  size_t blk_ = 0;
  size_t bytes_read_ = 0;
  Block block_;
  BlockCounts counts_;
};

}  // namespace dmlc_amd
