// data.cc -- this build's src/data.cc: the parser registry, the registered
// HIP text parsers and the Parser / RowBlockIter factories.
//
//   Parser<I,D>::Create(uri, part, nparts, type)     src/data.cc:152-186
//     CreateParser_: URISpec (uri?args#cache),
//     "auto" -> format= or libsvm, registry lookup     src/data.cc:66-86
//   RowBlockIter<I,D>::Create -> BasicRowIter         src/data.cc:88-150
//   registrations: libsvm / libfm (real_t), csv
//     (real_t / int32_t / int64_t) x (u32 / u64)      src/data.cc:189-227
//
// The registered factories build HipTextParser (hip_engine.h) over this
// build's text InputSplit, read in place into pinned batches
// (TextSplit::FillChunks).  Programs may register more parser types with
// DMLC_REGISTER_DATA_PARSER; Create finds them by name the same way.
#include <algorithm>
#include <cstring>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <vector>

#include "dmlc/data.h"
#include "dmlc/logging.h"
#include "dmlc/registry.h"
#include "hip_engine.h"
#include "text_split.h"

namespace dmlc_amd {
namespace {

// io::URISpec (src/io/uri_spec.h:43-74): path?k=v&k2=v2#cachefile
struct UriSpec {
  std::string uri, cache_file;
  std::map<std::string, std::string> args;
  UriSpec(const std::string &full, unsigned part, unsigned nparts) {
    auto split = [](const std::string &s, char d) {
      std::vector<std::string> out;
      std::istringstream is(s);
      std::string item;
      while (std::getline(is, item, d)) out.push_back(item);
      return out;
    };
    const std::vector<std::string> name_cache = split(full, '#');
    if (name_cache.size() == 2) {
      std::ostringstream os;
      os << name_cache[1];
      if (nparts != 1) os << ".split" << nparts << ".part" << part;
      cache_file = os.str();
    } else {
      CHECK_EQ(name_cache.size(), 1U) << "only one `#` is allowed in file path for cachefile specification";
    }
    const std::vector<std::string> name_args = split(name_cache.empty() ? std::string() : name_cache[0], '?');
    if (name_args.size() == 2) {
      const std::vector<std::string> arg_list = split(name_args[1], '&');
      for (size_t i = 0; i < arg_list.size(); ++i) {
        std::istringstream is(arg_list[i]);
        std::pair<std::string, std::string> kv;
        CHECK(std::getline(is, kv.first, '=')) << "Invalid uri argument format for key in arg " << i + 1;
        CHECK(std::getline(is, kv.second)) << "Invalid uri argument format for value in arg " << i + 1;
        args.insert(kv);
      }
    } else {
      CHECK_EQ(name_args.size(), 1U) << "only one `#` is allowed in file path for cachefile specification";
    }
    uri = name_args.empty() ? std::string() : name_args[0];
  }
};

// Chunks of this build's InputSplit read straight into the batch (no copy).
class TextSplitSource : public ChunkSource {
 public:
  explicit TextSplitSource(TextSplit *s) : split_(s) {}
  Fill FillChunks(char *dst, size_t cap, size_t max_bytes, std::vector<uint64_t> *ends) override {
    const TextSplit::Fill f = split_->FillChunks(dst, cap, max_bytes, ends);
    return Fill{f.end, f.need};
  }
  void BeforeFirst() override { split_->BeforeFirst(); }
  const std::vector<std::pair<const char *, size_t>> *Mappings() override {
    return split_->Mapped() ? &split_->Mappings() : nullptr;
  }
  Fill FillPieces(size_t max_bytes, std::vector<uint64_t> *ends, std::vector<TextPiece> *pieces) override {
    const TextSplit::Fill f = split_->FillPieces(max_bytes, ends, pieces);
    return Fill{f.end, f.need};
  }

 private:
  std::unique_ptr<TextSplit> split_;
};

// Set by RowBlockIter::Create around its parser's construction: the parser
// then also reduces the index / field maxima on the device (NumCol).
thread_local bool g_want_max_index = false;

// The factory behind every registered text type: `format` is the name it
// is registered under.  nthread follows TextParserBase (text_parser.h:32-35).
template <typename I, typename D>
dmlc::Parser<I, D> *CreateHipParser(const std::string &format, const std::string &path,
                                    const std::map<std::string, std::string> &args, unsigned part,
                                    unsigned nparts) {
  EngineConfig cfg;
  cfg.prm = make_params<I, D>(format, args);
  cfg.prm.nthread = reference_nthread();
  cfg.max_index = g_want_max_index;
  cfg.from_env();
  return new HipTextParser<I, D>(new TextSplitSource(new TextSplit(path, part, nparts)), cfg);
}

template <typename I, typename D>
dmlc::Parser<I, D> *CreateLibSVMParser(const std::string &path, const std::map<std::string, std::string> &args,
                                       unsigned part, unsigned nparts) {
  return CreateHipParser<I, D>("libsvm", path, args, part, nparts);
}
template <typename I, typename D>
dmlc::Parser<I, D> *CreateLibFMParser(const std::string &path, const std::map<std::string, std::string> &args,
                                      unsigned part, unsigned nparts) {
  return CreateHipParser<I, D>("libfm", path, args, part, nparts);
}
template <typename I, typename D>
dmlc::Parser<I, D> *CreateCSVParser(const std::string &path, const std::map<std::string, std::string> &args,
                                    unsigned part, unsigned nparts) {
  return CreateHipParser<I, D>("csv", path, args, part, nparts);
}

template <typename I, typename D>
dmlc::Parser<I, D> *CreateParser_(const char *uri, unsigned part, unsigned nparts, const char *type) {
  std::string ptype = type ? type : "auto";
  UriSpec spec(uri, part, nparts);
  if (ptype == "auto") {
    auto it = spec.args.find("format");
    ptype = it == spec.args.end() ? std::string("libsvm") : it->second;
  }
  const dmlc::ParserFactoryReg<I, D> *e = dmlc::Registry<dmlc::ParserFactoryReg<I, D>>::Get()->Find(ptype);
  if (e == nullptr) LOG(FATAL) << "Unknown data type " << ptype;
  return (*e->body)(spec.uri, spec.args, part, nparts);
}

// RowBlockContainer::Push appends `size` weights / qids per block
// (row_block.h:131-135), so every block stays row-aligned in the container.
// A libsvm block where only some rows carry label:weight or qid: holds fewer
// (`own`, this build's parser); the reference reads past them there -- here
// the block's own values are followed by zeros up to its row count.
template <typename T>
void PushPadded(std::vector<T> *dst, const T *src, size_t size, size_t own) {
  if (src == nullptr) return;
  if (own > size) own = size;
  dst->insert(dst->end(), src, src + own);
  dst->resize(dst->size() + (size - own), T(0));
}

// BasicRowIter (src/data/basic_row_iter.h:24-79): every block of the parser
// concatenated as RowBlockContainer::Push does (row_block.h:126-168);
// NumCol = max_index + 1.  For this build's own parser the block counts and
// the index / field maxima come from the device (DMLC_AMD_FLAG_MAX_INDEX), so
// the copy is the only host pass over the data.
template <typename I, typename D>
class HipRowIter : public dmlc::RowBlockIter<I, D> {
 public:
  explicit HipRowIter(dmlc::Parser<I, D> *parser) {
    std::unique_ptr<dmlc::Parser<I, D>> p(parser);
    auto *hp = dynamic_cast<HipTextParser<I, D> *>(parser);
    offset_.push_back(0);
    while (p->Next()) {
      const dmlc::RowBlock<I, D> &b = p->Value();
      if (hp) Push(b, &hp->ValueCounts());
      else Push(b, nullptr);
      if (hp && hp->BlockStartsBatch()) {
        max_index_ = std::max<uint64_t>(max_index_, hp->BatchMaxIndex());
        max_field_ = std::max<uint64_t>(max_field_, hp->BatchMaxField());
      }
    }
    row_.size = offset_.size() - 1;
    // fewer weights / qids than rows (libsvm rows without label:weight or
    // qid:): a reader takes `size` of them, so the tail reads as zeros
    if (!weight_.empty() && weight_.size() < row_.size) weight_.resize(row_.size, 0.0f);
    if (!qid_.empty() && qid_.size() < row_.size) qid_.resize(row_.size, 0);
    row_.offset = offset_.data();
    row_.label = dmlc::BeginPtr(label_);
    row_.weight = dmlc::BeginPtr(weight_);
    row_.qid = dmlc::BeginPtr(qid_);
    row_.field = dmlc::BeginPtr(field_);
    row_.index = dmlc::BeginPtr(index_);
    row_.value = dmlc::BeginPtr(value_);
  }
  void BeforeFirst() override { at_head_ = true; }
  bool Next() override {
    if (!at_head_) return false;
    at_head_ = false;
    return true;
  }
  const dmlc::RowBlock<I, D> &Value() const override { return row_; }
  size_t NumCol() const override { return static_cast<size_t>(static_cast<I>(max_index_)) + 1; }

 private:
  // RowBlockContainer::Push: labels (zeros for a block without them -- the
  // reference copies from NULL there), `size` weights / qids per block
  // (PushPadded), entries with their maxima, offsets rebased.
  void Push(const dmlc::RowBlock<I, D> &b, const BlockCounts *k) {
    const size_t ndata = b.offset[b.size] - b.offset[0];
    const size_t nl = label_.size();
    label_.resize(nl + b.size);
    if (b.label) std::memcpy(label_.data() + nl, b.label, b.size * sizeof(D));
    PushPadded(&weight_, b.weight, b.size, k ? k->weights : b.size);
    PushPadded(&qid_, b.qid, b.size, k ? k->qids : b.size);
    if (b.field) {
      field_.insert(field_.end(), b.field, b.field + ndata);
      if (!k)
        for (size_t i = 0; i < ndata; ++i) max_field_ = std::max<uint64_t>(max_field_, b.field[i]);
    }
    index_.insert(index_.end(), b.index, b.index + ndata);
    if (!k)
      for (size_t i = 0; i < ndata; ++i) max_index_ = std::max<uint64_t>(max_index_, b.index[i]);
    if (b.value) value_.insert(value_.end(), b.value, b.value + ndata);
    const size_t shift = offset_.back();
    for (size_t i = 0; i < b.size; ++i) offset_.push_back(shift + b.offset[i + 1] - b.offset[0]);
  }

  std::vector<size_t> offset_;
  std::vector<D> label_, value_;
  std::vector<float> weight_;
  std::vector<uint64_t> qid_;
  std::vector<I> index_, field_;
  uint64_t max_index_ = 0, max_field_ = 0;
  bool at_head_ = true;
  dmlc::RowBlock<I, D> row_;
};

// ---- the #cache path: RowBlockContainer pages on disk (disk_row_iter.h)

// A page: the reference's RowBlockContainer (row_block.h:27-216) -- Push of
// RowBlocks with offset rebasing and index / field maxima, MemCostBytes,
// and the Save / Load byte format (each vector as u64 count + raw elements,
// then max_field and max_index as IndexType).
template <typename I, typename D>
struct Page {
  std::vector<size_t> offset{0};
  std::vector<D> label, value;
  std::vector<float> weight;
  std::vector<uint64_t> qid;
  std::vector<I> field, index;
  I max_field = 0, max_index = 0;

  void Clear() {
    offset.assign(1, 0);
    label.clear();
    value.clear();
    weight.clear();
    qid.clear();
    field.clear();
    index.clear();
    max_field = max_index = 0;
  }
  size_t Size() const { return offset.size() - 1; }
  size_t MemCostBytes() const {  // row_block.h:81-86 (labels and weights priced as real_t)
    return offset.size() * sizeof(size_t) + label.size() * sizeof(dmlc::real_t) +
           weight.size() * sizeof(dmlc::real_t) + qid.size() * sizeof(size_t) + field.size() * sizeof(I) +
           index.size() * sizeof(I) + value.size() * sizeof(D);
  }
  // row_block.h:126-168; a block without labels (label-less CSV) pushes zeros
  // where the reference copies from its NULL label pointer.  With the block's
  // counts known (this build's parser, k) only its own weights / qids are
  // read -- a libsvm block where some rows lack label:weight or qid: holds
  // fewer of them than rows -- and zeros pad them to the block's rows
  // (PushPadded), so later blocks stay row-aligned as in the reference.
  void Push(const dmlc::RowBlock<I, D> &b, const BlockCounts *k = nullptr) {
    const size_t n0 = label.size();
    label.resize(n0 + b.size);
    if (b.label) std::memcpy(label.data() + n0, b.label, b.size * sizeof(D));
    PushPadded(&weight, b.weight, b.size, k ? k->weights : b.size);
    PushPadded(&qid, b.qid, b.size, k ? k->qids : b.size);
    const size_t ndata = b.offset[b.size] - b.offset[0];
    if (b.field) {
      field.insert(field.end(), b.field, b.field + ndata);
      for (size_t i = 0; i < ndata; ++i) max_field = std::max(max_field, b.field[i]);
    }
    index.insert(index.end(), b.index, b.index + ndata);
    for (size_t i = 0; i < ndata; ++i) max_index = std::max(max_index, b.index[i]);
    if (b.value) value.insert(value.end(), b.value, b.value + ndata);
    const size_t shift = offset.back();
    for (size_t i = 0; i < b.size; ++i) offset.push_back(shift + b.offset[i + 1] - b.offset[0]);
  }
  void Save(dmlc::Stream *fo) const {
    fo->Write(offset);
    fo->Write(label);
    fo->Write(weight);
    fo->Write(qid);
    fo->Write(field);
    fo->Write(index);
    fo->Write(value);
    fo->Write(&max_field, sizeof(I));
    fo->Write(&max_index, sizeof(I));
  }
  bool Load(dmlc::Stream *fi) {
    if (!fi->Read(&offset)) return false;
    CHECK(fi->Read(&label)) << "Bad RowBlock format";
    CHECK(fi->Read(&weight)) << "Bad RowBlock format";
    CHECK(fi->Read(&qid)) << "Bad RowBlock format";
    CHECK(fi->Read(&field)) << "Bad RowBlock format";
    CHECK(fi->Read(&index)) << "Bad RowBlock format";
    CHECK(fi->Read(&value)) << "Bad RowBlock format";
    CHECK(fi->Read(&max_field, sizeof(I)) == sizeof(I)) << "Bad RowBlock format";
    CHECK(fi->Read(&max_index, sizeof(I)) == sizeof(I)) << "Bad RowBlock format";
    // a page of libsvm blocks where only some rows had label:weight / qid:
    // holds fewer of them than rows; a RowBlock reader takes `size` of each
    // (the reference's own pages read past the vector there): pad the
    // in-memory copy with zeros (the file keeps the reference's bytes)
    if (!weight.empty() && weight.size() < Size()) weight.resize(Size(), 0.0f);
    if (!qid.empty() && qid.size() < Size()) qid.resize(Size(), 0);
    return true;
  }
  // GetBlock (row_block.h:171-189) with its CHECKs
  dmlc::RowBlock<I, D> Block() const {
    CHECK(label.size() + 1 == offset.size());
    CHECK(offset.back() == index.size());
    CHECK(offset.back() == value.size() || value.size() == 0);
    dmlc::RowBlock<I, D> b;
    b.size = Size();
    b.offset = offset.data();
    b.label = dmlc::BeginPtr(label);
    b.weight = dmlc::BeginPtr(weight);
    b.qid = dmlc::BeginPtr(qid);
    b.field = dmlc::BeginPtr(field);
    b.index = dmlc::BeginPtr(index);
    b.value = dmlc::BeginPtr(value);
    return b;
  }
};

// DiskRowIter (disk_row_iter.h:40-137): with `uri#cachefile` the parsed rows
// are written once to the cache file in 64 MB pages (RowBlockContainer::Save)
// and the iterator reads the pages back; an existing cache file is reused
// without parsing.  NumCol: max_index + 1 over the pages built (as the
// reference); when an existing cache is reused the reference leaves it
// uninitialised -- here the pages are scanned once for it.
template <typename I, typename D>
class HipDiskRowIter : public dmlc::RowBlockIter<I, D> {
 public:
  static const size_t kPageSize = 64UL << 20UL;  // disk_row_iter.h:34
  HipDiskRowIter(dmlc::Parser<I, D> *parser, const std::string &cache_file) : cache_file_(cache_file) {
    std::unique_ptr<dmlc::Parser<I, D>> p(parser);
    if (!TryLoadCache()) {
      BuildCache(p.get());
      CHECK(TryLoadCache()) << "failed to build cache file " << cache_file_;
    } else {
      ScanNumCol();
    }
  }
  void BeforeFirst() override { fi_->Seek(0); }
  bool Next() override {
    if (!page_.Load(fi_.get())) return false;
    row_ = page_.Block();
    return true;
  }
  const dmlc::RowBlock<I, D> &Value() const override { return row_; }
  size_t NumCol() const override { return num_col_; }

 private:
  bool TryLoadCache() {
    fi_.reset(dmlc::SeekStream::CreateForRead(cache_file_.c_str(), true));
    return fi_ != nullptr;
  }
  void BuildCache(dmlc::Parser<I, D> *parser) {
    std::unique_ptr<dmlc::Stream> fo(dmlc::Stream::Create(cache_file_.c_str(), "w"));
    Page<I, D> data;
    num_col_ = 0;
    auto *hp = dynamic_cast<HipTextParser<I, D> *>(parser);
    while (parser->Next()) {
      data.Push(parser->Value(), hp ? &hp->ValueCounts() : nullptr);
      if (data.MemCostBytes() >= kPageSize) {
        num_col_ = std::max(num_col_, static_cast<size_t>(data.max_index) + 1);
        data.Save(fo.get());
        data.Clear();
      }
    }
    if (data.Size() != 0) {
      num_col_ = std::max(num_col_, static_cast<size_t>(data.max_index) + 1);
      data.Save(fo.get());
    }
  }
  void ScanNumCol() {
    num_col_ = 0;
    while (page_.Load(fi_.get())) num_col_ = std::max(num_col_, static_cast<size_t>(page_.max_index) + 1);
    fi_->Seek(0);
  }

  std::string cache_file_;
  std::unique_ptr<dmlc::SeekStream> fi_;
  size_t num_col_ = 0;
  Page<I, D> page_;
  dmlc::RowBlock<I, D> row_;
};

template <typename I, typename D>
dmlc::RowBlockIter<I, D> *CreateIter_(const char *uri, unsigned part, unsigned nparts, const char *type) {
  UriSpec spec(uri, part, nparts);
  // as the reference (data.cc:88-105): the parser is created from spec.uri,
  // i.e. WITHOUT the ?key=value arguments of the RowBlockIter uri
  g_want_max_index = spec.cache_file.empty();  // NumCol from the device maxima (this build's parsers)
  dmlc::Parser<I, D> *parser;
  try {
    parser = CreateParser_<I, D>(spec.uri.c_str(), part, nparts, type);
  } catch (...) {
    g_want_max_index = false;
    throw;
  }
  g_want_max_index = false;
  if (!spec.cache_file.empty()) return new HipDiskRowIter<I, D>(parser, spec.cache_file);
  return new HipRowIter<I, D>(parser);
}

}  // namespace
}  // namespace dmlc_amd

namespace dmlc {

template <typename I, typename D>
Parser<I, D> *Parser<I, D>::Create(const char *uri, unsigned part_index, unsigned num_parts, const char *type) {
  return dmlc_amd::CreateParser_<I, D>(uri, part_index, num_parts, type);
}
template <typename I, typename D>
RowBlockIter<I, D> *RowBlockIter<I, D>::Create(const char *uri, unsigned part_index, unsigned num_parts,
                                               const char *type) {
  return dmlc_amd::CreateIter_<I, D>(uri, part_index, num_parts, type);
}

template class Parser<uint32_t, real_t>;
template class Parser<uint64_t, real_t>;
template class Parser<uint32_t, int32_t>;
template class Parser<uint64_t, int32_t>;
template class Parser<uint32_t, int64_t>;
template class Parser<uint64_t, int64_t>;
template class RowBlockIter<uint32_t, real_t>;
template class RowBlockIter<uint64_t, real_t>;
template class RowBlockIter<uint32_t, int32_t>;
template class RowBlockIter<uint64_t, int32_t>;
template class RowBlockIter<uint32_t, int64_t>;
template class RowBlockIter<uint64_t, int64_t>;

// ---- registry (src/data.cc:189-227)
typedef ParserFactoryReg<uint32_t, real_t> Reg32flt;
typedef ParserFactoryReg<uint32_t, int32_t> Reg32int32;
typedef ParserFactoryReg<uint32_t, int64_t> Reg32int64;
typedef ParserFactoryReg<uint64_t, real_t> Reg64flt;
typedef ParserFactoryReg<uint64_t, int32_t> Reg64int32;
typedef ParserFactoryReg<uint64_t, int64_t> Reg64int64;
DMLC_REGISTRY_ENABLE(Reg32flt);
DMLC_REGISTRY_ENABLE(Reg32int32);
DMLC_REGISTRY_ENABLE(Reg32int64);
DMLC_REGISTRY_ENABLE(Reg64flt);
DMLC_REGISTRY_ENABLE(Reg64int32);
DMLC_REGISTRY_ENABLE(Reg64int64);

DMLC_REGISTER_DATA_PARSER(uint32_t, real_t, libsvm, dmlc_amd::CreateLibSVMParser<uint32_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, real_t, libsvm, dmlc_amd::CreateLibSVMParser<uint64_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, real_t, libfm, dmlc_amd::CreateLibFMParser<uint32_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, real_t, libfm, dmlc_amd::CreateLibFMParser<uint64_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, real_t, csv, dmlc_amd::CreateCSVParser<uint32_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, real_t, csv, dmlc_amd::CreateCSVParser<uint64_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, int32_t, csv, dmlc_amd::CreateCSVParser<uint32_t __DMLC_COMMA int32_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, int32_t, csv, dmlc_amd::CreateCSVParser<uint64_t __DMLC_COMMA int32_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, int64_t, csv, dmlc_amd::CreateCSVParser<uint32_t __DMLC_COMMA int64_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, int64_t, csv, dmlc_amd::CreateCSVParser<uint64_t __DMLC_COMMA int64_t>);

}  // namespace dmlc
