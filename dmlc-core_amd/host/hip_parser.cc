// hip_parser.cc -- dmlc::Parser<I,D> / RowBlockIter<I,D> backed by the MI355X
// parse path (include/dmlc_amd.h).  Host side of the drop-in boundary:
//
//   Parser<I,D>::Create(uri, part, nparts, type)      src/data.cc:152-186
//     "auto" -> the URI's format= argument or libsvm   src/data.cc:66-86
//     parser arguments from uri?k=v&...; an unknown key is an error
//       (Parameter::Init, include/dmlc/parameter.h:465-478)
//   Next()/Value(): one RowBlock per InputSplit chunk, i.e. the reference's
//     ParseBlock with nthread = 1 (src/data/text_parser.h:116-155); the block
//     stays valid until the next Next() (src/data/parser.h:109-111)
//   per-chunk consistency checks of RowBlockContainer::GetBlock
//     (src/data/row_block.h:171-189) and CSVParser (csv_parser.h:147-148)
//
// Pipeline per batch: InputSplit chunks (up to batch_bytes, default 256 MiB,
// env DMLC_AMD_BATCH_BYTES) -> pinned staging -> hipMemcpyAsync -> count pass ->
// exact-size device outputs -> write pass -> hipMemcpyAsync into pinned host
// arrays -> RowBlock views.  A prefetch thread fills the next batch's staging
// buffer from the InputSplit while the device parses the current one.
#include <hip/hip_runtime_api.h>

#include <condition_variable>
#include <cstdlib>
#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <type_traits>
#include <vector>

#include "dmlc/data.h"
#include "dmlc_amd.h"
#include "text_split.h"

namespace dmlc_amd {
namespace {

void hip_check(hipError_t e, const char *what) {
  if (e != hipSuccess) throw dmlc::Error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

// ---- URI sugar: path?k=v&k2=v2#cachefile (src/io/uri_spec.h:43-74)
struct UriSpec {
  std::string path;
  std::map<std::string, std::string> args;
  explicit UriSpec(const std::string &uri) {
    std::string u = uri;
    const size_t hash = u.find('#');
    if (hash != std::string::npos) u = u.substr(0, hash);  // disk cache: not used by this path
    const size_t q = u.find('?');
    path = u.substr(0, q);
    if (q == std::string::npos) return;
    std::string rest = u.substr(q + 1);
    size_t s = 0;
    while (s < rest.size()) {
      size_t e = rest.find('&', s);
      if (e == std::string::npos) e = rest.size();
      const std::string kv = rest.substr(s, e - s);
      const size_t eq = kv.find('=');
      if (eq == std::string::npos) throw dmlc::Error("Check failed: invalid uri argument \"" + kv + "\"");
      args[kv.substr(0, eq)] = kv.substr(eq + 1);
      s = e + 1;
    }
  }
};

int parse_int_arg(const std::string &k, const std::string &v) {
  char *end = nullptr;
  const long x = std::strtol(v.c_str(), &end, 10);
  if (v.empty() || *end != '\0') throw dmlc::Error("Invalid Parameter format for " + k + " expect int but value='" + v + "'");
  return (int)x;
}

template <typename T>
struct PinnedVec {  // page-locked host array, grown on demand
  T *p = nullptr;
  size_t cap = 0;
  ~PinnedVec() {
    if (p) (void)hipHostFree(p);
  }
  void reserve(size_t n, size_t keep = 0) {  // keeps the first `keep` elements
    if (n <= cap) return;
    T *q = nullptr;
    const size_t c = n + n / 4 + 64;
    hip_check(hipHostMalloc(reinterpret_cast<void **>(&q), c * sizeof(T), 0), "hipHostMalloc");
    if (p) {
      if (keep) std::memcpy(q, p, keep * sizeof(T));
      hip_check(hipHostFree(p), "hipHostFree");
    }
    p = q;
    cap = c;
  }
};

struct DevBuf {  // device array, grown on demand
  void *p = nullptr;
  size_t bytes = 0;
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  void *get(size_t n) {
    if (n > bytes) {
      if (p) hip_check(hipFree(p), "hipFree");
      p = nullptr;
      const size_t b = n + n / 4 + 256;
      hip_check(hipMalloc(&p, b), "hipMalloc");
      bytes = b;
    }
    return p;
  }
};

// One host-staged batch of InputSplit chunks.
struct Batch {
  PinnedVec<char> text;
  std::vector<uint64_t> starts;  // nchunks + 1
  size_t bytes = 0;
  bool end = false;
};

template <typename IndexType, typename DType>
class HipParser : public dmlc::Parser<IndexType, DType> {
 public:
  HipParser(const std::string &uri, unsigned part, unsigned nparts, const std::string &type)
      : spec_(uri) {
    std::string fmt = type;
    if (fmt == "auto") {
      auto it = spec_.args.find("format");
      fmt = it == spec_.args.end() ? "libsvm" : it->second;
    }
    std::memset(&prm_, 0, sizeof(prm_));
    prm_.index_bits = sizeof(IndexType) * 8;
    prm_.label_column = -1;
    prm_.weight_column = -1;
    prm_.delimiter = ',';
    if (fmt == "libsvm") {
      prm_.format = DMLC_AMD_LIBSVM;
    } else if (fmt == "csv") {
      prm_.format = DMLC_AMD_CSV;
    } else if (fmt == "libfm") {  // data.cc:206-209
      prm_.format = DMLC_AMD_LIBFM;
    } else {
      throw dmlc::Error("Unknown data type " + fmt);
    }
    for (const auto &kv : spec_.args) {  // LibSVMParserParam / CSVParserParam fields
      if (kv.first == "format") continue;
      if ((prm_.format == DMLC_AMD_LIBSVM || prm_.format == DMLC_AMD_LIBFM) && kv.first == "indexing_mode") {
        prm_.indexing_mode = parse_int_arg(kv.first, kv.second);
      } else if (prm_.format == DMLC_AMD_CSV && kv.first == "label_column") {
        prm_.label_column = parse_int_arg(kv.first, kv.second);
      } else if (prm_.format == DMLC_AMD_CSV && kv.first == "weight_column") {
        prm_.weight_column = parse_int_arg(kv.first, kv.second);
      } else if (prm_.format == DMLC_AMD_CSV && kv.first == "delimiter") {
        if (kv.second.empty()) throw dmlc::Error("Check failed: delimiter is empty");
        prm_.delimiter = (unsigned char)kv.second[0];
      } else {
        throw dmlc::Error("Cannot find argument '" + kv.first + "', Possible Arguments:");
      }
    }
    if (prm_.format == DMLC_AMD_CSV && prm_.label_column >= 0 && prm_.label_column == prm_.weight_column)
      throw dmlc::Error("Check failed: label_column != weight_column");
    if (sizeof(DType) == 4 && !std::is_same<DType, float>::value) prm_.value_type = DMLC_AMD_I32;
    if (sizeof(DType) == 8) prm_.value_type = DMLC_AMD_I64;
    if (prm_.format != DMLC_AMD_CSV && prm_.value_type != DMLC_AMD_F32)
      throw dmlc::Error("libsvm / libfm parsers support float values only");
    if (const char *b = std::getenv("DMLC_AMD_BATCH_BYTES")) batch_bytes_ = std::strtoull(b, nullptr, 10);
    if (const char *n = std::getenv("DMLC_AMD_PREFETCH_SLOTS")) nslots_ = std::max(2, std::atoi(n));
    hip_check(hipGetDevice(&device_), "hipGetDevice");
    hip_check(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking), "hipStreamCreate");
    split_.reset(new TextSplit(spec_.path, part, nparts));
    StartPrefetch();
  }

  ~HipParser() override {
    StopPrefetch();
    if (stream_) (void)hipStreamDestroy(stream_);
  }

  void BeforeFirst() override {
    StopPrefetch();
    split_->BeforeFirst();
    blocks_.clear();
    cur_ = 0;
    bytes_read_ = 0;
    StartPrefetch();
  }

  bool Next() override {
    while (cur_ >= blocks_.size()) {
      if (!ParseNextBatch()) return false;
    }
    block_ = blocks_[cur_++];
    return true;
  }

  const dmlc::RowBlock<IndexType, DType> &Value() const override { return block_; }
  size_t BytesRead() const override { return bytes_read_; }

 private:
  // ---- prefetch thread: fills batches from the InputSplit (2 slots)
  void StartPrefetch() {
    stop_ = false;
    ended_ = false;
    slots_.resize((size_t)nslots_);
    for (auto &b : slots_) b.reset(new Batch());
    filled_.clear();
    free_.clear();
    for (int i = nslots_ - 1; i >= 0; --i) free_.push_back(i);
    worker_ = std::thread([this] { PrefetchLoop(); });
  }
  void StopPrefetch() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      stop_ = true;
    }
    cv_.notify_all();
    if (worker_.joinable()) worker_.join();
  }
  void PrefetchLoop() {
    try {
      std::vector<uint64_t> ends;
      for (;;) {
        int slot;
        {
          std::unique_lock<std::mutex> lk(mu_);
          cv_.wait(lk, [&] { return stop_ || !free_.empty(); });
          if (stop_) return;
          slot = free_.back();
          free_.pop_back();
        }
        Batch &b = *slots_[slot];
        b.starts.assign(1, 0);
        b.bytes = 0;
        b.end = false;
        // chunks are read straight into the pinned batch (TextSplit::FillChunks:
        // no staging copies); room for one more 8 MiB chunk past the target
        b.text.reserve(batch_bytes_ + (16u << 20));
        for (;;) {
          ends.clear();
          const TextSplit::Fill f = split_->FillChunks(b.text.p, b.text.cap, batch_bytes_, &ends);
          if (f.need) {  // a record longer than the room left: grow and retry
            b.text.reserve(f.need + (16u << 20));
            continue;
          }
          b.starts.insert(b.starts.end(), ends.begin(), ends.end());
          b.bytes = b.starts.back();
          b.end = f.end;
          break;
        }
        {
          std::lock_guard<std::mutex> lk(mu_);
          filled_.push_back(slot);
        }
        cv_.notify_all();
        if (b.end) return;
      }
    } catch (const std::exception &e) {
      std::lock_guard<std::mutex> lk(mu_);
      error_ = e.what();
      cv_.notify_all();
    }
  }

  bool ParseNextBatch() {
    if (ended_) return false;
    int slot;
    {
      std::unique_lock<std::mutex> lk(mu_);
      cv_.wait(lk, [&] { return !filled_.empty() || !error_.empty(); });
      if (!error_.empty()) throw dmlc::Error(error_);
      slot = filled_.front();
      filled_.erase(filled_.begin());
    }
    Batch &b = *slots_[slot];
    const bool end = b.end;
    ended_ = end;
    const size_t nchunks = b.starts.size() - 1;
    if (nchunks > 0) {
      Parse(b);
      bytes_read_ += b.bytes;
    }
    {
      std::lock_guard<std::mutex> lk(mu_);
      free_.push_back(slot);
    }
    cv_.notify_all();
    return nchunks > 0 || !end;
  }

  void Parse(const Batch &b) {
    hip_check(hipSetDevice(device_), "hipSetDevice");  // callable from any thread
    const int nchunks = (int)(b.starts.size() - 1);
    char *d_text = static_cast<char *>(d_text_.get(b.bytes));
    uint64_t *d_cs = static_cast<uint64_t *>(d_cs_.get(b.starts.size() * 8));
    uint64_t *d_res = static_cast<uint64_t *>(d_res_.get(sizeof(dmlc_amd_result)));
    uint64_t *d_tab = static_cast<uint64_t *>(d_tab_.get((size_t)nchunks * 64));
    const size_t ws = dmlc_amd_workspace_bytes(b.bytes, nchunks, &prm_);
    void *d_ws = d_ws_.get(ws);
    hip_check(hipMemcpyAsync(d_text, b.text.p, b.bytes, hipMemcpyHostToDevice, stream_), "H2D text");
    hip_check(hipMemcpyAsync(d_cs, b.starts.data(), b.starts.size() * 8, hipMemcpyHostToDevice, stream_),
              "H2D chunk starts");
    // count pass (size query)
    dmlc_amd_params p = prm_;
    p.flags = DMLC_AMD_FLAG_COUNT_ONLY;
    dmlc_amd_csr none;
    std::memset(&none, 0, sizeof(none));
    Check(dmlc_amd_parse(d_text, b.bytes, d_cs, nchunks, &p, &none, nullptr, d_ws, ws,
                         reinterpret_cast<dmlc_amd_result *>(d_res), stream_));
    dmlc_amd_result res;
    hip_check(hipMemcpyAsync(&res, d_res, sizeof(res), hipMemcpyDeviceToHost, stream_), "D2H result");
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    RaiseParseError(res.error);
    const uint64_t *c = res.count;
    const size_t vsz = sizeof(DType), isz = sizeof(IndexType);
    // exact-size device outputs
    dmlc_amd_csr out;
    std::memset(&out, 0, sizeof(out));
    out.offset = static_cast<uint64_t *>(d_off_.get((c[DMLC_AMD_ROWS] + 1) * 8));
    out.label = d_label_.get((c[DMLC_AMD_LABEL] + 1) * vsz);
    out.weight = static_cast<float *>(d_weight_.get((c[DMLC_AMD_WEIGHT] + 1) * 4));
    out.qid = static_cast<uint64_t *>(d_qid_.get((c[DMLC_AMD_QID] + 1) * 8));
    out.index = d_index_.get((c[DMLC_AMD_INDEX] + 1) * isz);
    out.field = d_field_.get((c[DMLC_AMD_FIELD] + 1) * isz);
    out.value = d_value_.get((c[DMLC_AMD_VALUE] + 1) * vsz);
    for (int i = 0; i < 7; ++i) out.cap[i] = c[i];
    p.flags = DMLC_AMD_FLAG_FILL_ONLY;
    Check(dmlc_amd_parse(d_text, b.bytes, d_cs, nchunks, &p, &out, d_tab, d_ws, ws,
                         reinterpret_cast<dmlc_amd_result *>(d_res), stream_));
    // results into pinned host arrays
    h_off_.reserve(c[DMLC_AMD_ROWS] + 1);
    h_label_.reserve((c[DMLC_AMD_LABEL] + 1) * vsz);  // byte arrays
    h_weight_.reserve(c[DMLC_AMD_WEIGHT] + 1);
    h_qid_.reserve(c[DMLC_AMD_QID] + 1);
    h_index_.reserve((c[DMLC_AMD_INDEX] + 1) * isz);
    h_field_.reserve((c[DMLC_AMD_FIELD] + 1) * isz);
    h_value_.reserve((c[DMLC_AMD_VALUE] + 1) * vsz);
    h_tab_.reserve((size_t)nchunks * 8);
    auto d2h = [&](void *dst, const void *src, size_t bytes) {
      if (bytes) hip_check(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, stream_), "D2H");
    };
    d2h(h_off_.p, out.offset, (c[DMLC_AMD_ROWS] + 1) * 8);
    d2h(h_label_.p, out.label, c[DMLC_AMD_LABEL] * vsz);
    d2h(h_weight_.p, out.weight, c[DMLC_AMD_WEIGHT] * 4);
    d2h(h_qid_.p, out.qid, c[DMLC_AMD_QID] * 8);
    d2h(h_index_.p, out.index, c[DMLC_AMD_INDEX] * isz);
    d2h(h_field_.p, out.field, c[DMLC_AMD_FIELD] * isz);
    d2h(h_value_.p, out.value, c[DMLC_AMD_VALUE] * vsz);
    d2h(h_tab_.p, d_tab, (size_t)nchunks * 64);
    d2h(&res, d_res, sizeof(res));
    hip_check(hipStreamSynchronize(stream_), "hipStreamSynchronize");
    RaiseParseError(res.error);
    BuildBlocks(nchunks, res.count);
  }

  // RowBlock views per chunk, with the reference's per-block checks.
  void BuildBlocks(int nchunks, const uint64_t *tot) {
    blocks_.clear();
    cur_ = 0;
    for (int i = 0; i < nchunks; ++i) {
      const uint64_t *b0 = h_tab_.p + (size_t)i * 8;
      const uint64_t *b1 = i + 1 < nchunks ? h_tab_.p + (size_t)(i + 1) * 8 : tot;
      const uint64_t rows = b1[DMLC_AMD_ROWS] - b0[DMLC_AMD_ROWS];
      const uint64_t nidx = b1[DMLC_AMD_INDEX] - b0[DMLC_AMD_INDEX];
      const uint64_t nval = b1[DMLC_AMD_VALUE] - b0[DMLC_AMD_VALUE];
      const uint64_t nlab = b1[DMLC_AMD_LABEL] - b0[DMLC_AMD_LABEL];
      const uint64_t nw = b1[DMLC_AMD_WEIGHT] - b0[DMLC_AMD_WEIGHT];
      const uint64_t nq = b1[DMLC_AMD_QID] - b0[DMLC_AMD_QID];
      const uint64_t nf = b1[DMLC_AMD_FIELD] - b0[DMLC_AMD_FIELD];
      if (prm_.format == DMLC_AMD_LIBFM && nf != nidx)  // libfm_parser.h:127
        throw dmlc::Error("Check failed: out->field.size() == out->index.size()");
      if (prm_.format == DMLC_AMD_CSV) {  // csv_parser.h:147-148
        if (nlab != 0 && nlab != rows)
          throw dmlc::Error("Check failed: out->label.size() == 0 || out->label.size() + 1 == out->offset.size()");
        if (nw != 0 && nw != rows)
          throw dmlc::Error("Check failed: out->weight.size() == 0 || out->weight.size() + 1 == out->offset.size()");
      }
      if (rows == 0) continue;  // an empty container yields no block (parser.h:36-38)
      // RowBlockContainer::GetBlock, row_block.h:173-177
      if (nlab != 0 && nlab != rows) throw dmlc::Error("Check failed: label.size() + 1 == offset.size()");
      if (nval != 0 && nval != nidx)
        throw dmlc::Error("Check failed: offset.back() == value.size() || value.size() == 0");
      dmlc::RowBlock<IndexType, DType> blk;
      blk.size = rows;
      blk.offset = reinterpret_cast<const size_t *>(h_off_.p + b0[DMLC_AMD_ROWS]);
      blk.label = nlab ? reinterpret_cast<const DType *>(h_label_.p) + b0[DMLC_AMD_LABEL] : nullptr;
      blk.weight = nw ? h_weight_.p + b0[DMLC_AMD_WEIGHT] : nullptr;
      blk.qid = nq ? h_qid_.p + b0[DMLC_AMD_QID] : nullptr;
      blk.field = nf ? reinterpret_cast<const IndexType *>(h_field_.p) : nullptr;
      blk.index = reinterpret_cast<const IndexType *>(h_index_.p);
      blk.value = nval ? reinterpret_cast<const DType *>(h_value_.p) : nullptr;
      blocks_.push_back(blk);
    }
  }

  void Check(int rc) {
    if (rc == DMLC_AMD_OK) return;
    throw dmlc::Error(std::string("dmlc_amd_parse: ") + dmlc_amd_error_string(rc) +
                      (rc == DMLC_AMD_ERR_HIP ? std::string(" (") + dmlc_amd_last_hip_error() + ")" : ""));
  }

  static void RaiseParseError(uint64_t err) {
    if (err == 0) return;
    throw dmlc::Error(dmlc_amd_error_string((int)(err & 0xFFFF)));
  }

  UriSpec spec_;
  dmlc_amd_params prm_;
  std::unique_ptr<TextSplit> split_;
  // Device batches: a few InputSplit chunks each, several in flight, so the
  // reader, the copies and the parse overlap with short fill/drain phases
  // (measured on MI355X, 2.1 GB libsvm: 256 MiB batches 5.5 GB/s, 32 MiB 14.7; 3-4 slots no better).
  size_t batch_bytes_ = 32u << 20;
  int nslots_ = 2;
  int device_ = 0;
  hipStream_t stream_ = nullptr;
  // prefetch
  std::vector<std::unique_ptr<Batch>> slots_;
  std::vector<int> filled_, free_;
  std::thread worker_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false, ended_ = false;
  std::string error_;
  // device and pinned host buffers
  DevBuf d_text_, d_cs_, d_res_, d_tab_, d_ws_, d_off_, d_label_, d_weight_, d_qid_, d_index_, d_field_,
      d_value_;
  PinnedVec<uint64_t> h_off_, h_qid_, h_tab_;
  PinnedVec<float> h_weight_;
  PinnedVec<char> h_label_, h_index_, h_field_, h_value_;
  std::vector<dmlc::RowBlock<IndexType, DType>> blocks_;
  size_t cur_ = 0;
  size_t bytes_read_ = 0;
  dmlc::RowBlock<IndexType, DType> block_;
};

// In-memory RowBlockIter (the reference's BasicRowIter, basic_row_iter.h:61-79):
// every block concatenated with offset rebasing (RowBlockContainer::Push,
// row_block.h:126-168); NumCol = max index + 1.
template <typename IndexType, typename DType>
class HipRowIter : public dmlc::RowBlockIter<IndexType, DType> {
 public:
  explicit HipRowIter(dmlc::Parser<IndexType, DType> *parser) {
    std::unique_ptr<dmlc::Parser<IndexType, DType>> p(parser);
    offset_.push_back(0);
    while (p->Next()) {
      const auto &b = p->Value();
      const size_t base = offset_.back();
      for (size_t i = 0; i < b.size; ++i) offset_.push_back(base + b.offset[i + 1] - b.offset[0]);
      const size_t lo = b.offset[0], hi = b.offset[b.size];
      if (b.label) label_.insert(label_.end(), b.label, b.label + b.size);
      if (b.weight) weight_.insert(weight_.end(), b.weight, b.weight + b.size);
      if (b.qid) qid_.insert(qid_.end(), b.qid, b.qid + b.size);
      index_.insert(index_.end(), b.index + lo, b.index + hi);
      if (b.field) field_.insert(field_.end(), b.field + lo, b.field + hi);
      if (b.value) value_.insert(value_.end(), b.value + lo, b.value + hi);
      for (size_t j = lo; j < hi; ++j)
        if ((size_t)b.index[j] + 1 > num_col_) num_col_ = (size_t)b.index[j] + 1;
    }
    block_.size = offset_.size() - 1;
    block_.offset = offset_.data();
    block_.label = label_.empty() ? nullptr : label_.data();
    block_.weight = weight_.empty() ? nullptr : weight_.data();
    block_.qid = qid_.empty() ? nullptr : qid_.data();
    block_.field = field_.empty() ? nullptr : field_.data();
    block_.index = index_.empty() ? nullptr : index_.data();
    block_.value = value_.empty() ? nullptr : value_.data();
  }
  void BeforeFirst() override { at_start_ = true; }
  bool Next() override {
    if (!at_start_) return false;
    at_start_ = false;
    return true;
  }
  const dmlc::RowBlock<IndexType, DType> &Value() const override { return block_; }
  size_t NumCol() const override { return num_col_; }

 private:
  std::vector<size_t> offset_;
  std::vector<DType> label_;
  std::vector<float> weight_;
  std::vector<uint64_t> qid_;
  std::vector<IndexType> index_, field_;
  std::vector<DType> value_;
  size_t num_col_ = 0;
  bool at_start_ = true;
  dmlc::RowBlock<IndexType, DType> block_;
};

}  // namespace
}  // namespace dmlc_amd

namespace dmlc {

template <typename IndexType, typename DType>
Parser<IndexType, DType> *Parser<IndexType, DType>::Create(const char *uri, unsigned part_index,
                                                           unsigned num_parts, const char *type) {
  return new dmlc_amd::HipParser<IndexType, DType>(uri, part_index, num_parts, type ? type : "auto");
}

template <typename IndexType, typename DType>
RowBlockIter<IndexType, DType> *RowBlockIter<IndexType, DType>::Create(const char *uri, unsigned part_index,
                                                                       unsigned num_parts, const char *type) {
  return new dmlc_amd::HipRowIter<IndexType, DType>(
      Parser<IndexType, DType>::Create(uri, part_index, num_parts, type));
}

// the instantiations src/data.cc:189-221 registers
template class Parser<uint32_t, float>;
template class Parser<uint64_t, float>;
template class Parser<uint32_t, int32_t>;
template class Parser<uint64_t, int32_t>;
template class Parser<uint32_t, int64_t>;
template class Parser<uint64_t, int64_t>;
template class RowBlockIter<uint32_t, float>;
template class RowBlockIter<uint64_t, float>;
template class RowBlockIter<uint32_t, int32_t>;
template class RowBlockIter<uint64_t, int32_t>;
template class RowBlockIter<uint32_t, int64_t>;
template class RowBlockIter<uint64_t, int64_t>;

}  // namespace dmlc

// ---- test hook (C ABI): the InputSplit chunk sequence of a part, for
// tests/ to compare with the oracle on machines without a GPU.
extern "C" int dmlc_amd_host_split(const char *uri, unsigned part, unsigned nparts, uint64_t buffer_bytes,
                                   char **out_buf, uint64_t **out_off, uint64_t *out_n) {
  try {
    dmlc_amd::TextSplit split(uri, part, nparts, buffer_bytes);
    std::vector<char> all;
    std::vector<uint64_t> off(1, 0);
    while (split.NextChunk(&all)) off.push_back(all.size());
    *out_buf = static_cast<char *>(std::malloc(all.size() + 1));
    std::memcpy(*out_buf, all.data(), all.size());
    *out_off = static_cast<uint64_t *>(std::malloc(off.size() * 8));
    std::memcpy(*out_off, off.data(), off.size() * 8);
    *out_n = off.size() - 1;
    return 0;
  } catch (const std::exception &) {
    return DMLC_AMD_ERR_ARG;
  }
}

// Test hook: the same chunk sequence through TextSplit::FillChunks, the
// in-place reader of the device pipeline, with batches of batch_bytes into a
// buffer of cap bytes (small values exercise batch breaks and buffer growth).
extern "C" int dmlc_amd_host_split_inplace(const char *uri, unsigned part, unsigned nparts,
                                           uint64_t buffer_bytes, uint64_t batch_bytes, uint64_t cap,
                                           char **out_buf, uint64_t **out_off, uint64_t *out_n) {
  try {
    dmlc_amd::TextSplit split(uri, part, nparts, buffer_bytes);
    std::vector<char> all, buf(cap);
    std::vector<uint64_t> off(1, 0), ends;
    for (;;) {
      ends.clear();
      const dmlc_amd::TextSplit::Fill f = split.FillChunks(buf.data(), buf.size(), batch_bytes, &ends);
      if (f.need) {
        buf.resize(f.need);
        continue;
      }
      uint64_t prev = 0;
      for (uint64_t e : ends) {
        all.insert(all.end(), buf.data() + prev, buf.data() + e);
        off.push_back(all.size());
        prev = e;
      }
      if (f.end) break;
    }
    *out_buf = static_cast<char *>(std::malloc(all.size() + 1));
    std::memcpy(*out_buf, all.data(), all.size());
    *out_off = static_cast<uint64_t *>(std::malloc(off.size() * 8));
    std::memcpy(*out_off, off.data(), off.size() * 8);
    *out_n = off.size() - 1;
    return 0;
  } catch (const std::exception &) {
    return DMLC_AMD_ERR_ARG;
  }
}

extern "C" void dmlc_amd_host_free(void *p) { std::free(p); }
