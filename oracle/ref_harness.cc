// ref_harness.cc -- TEST INFRASTRUCTURE ONLY.
//
// A thin extern "C" shim over the *genuine* dmlc-core reference, compiled from
// the unmodified sources under /root/reference by oracle/Makefile (target `ref`) into
// oracle/_ref/libdmlc_ref.so.  It is used (a) in this container to generate the
// golden fixtures under tests/golden/ and to pin the C restatement
// (oracle/dmlc_oracle.c), and (b) as bench.py's cpu_baseline ("kind":
// "reference") when oracle/_ref/ travelled to the GPU box.  It is never part
// of the product.
//
// The ParseBlock seam follows the fixture-subclass pattern of
// test/unittest_parser.cc:16-47 (ParseBlock is protected).
#include <dmlc/data.h>
#include <dmlc/io.h>
#include <dmlc/strtonum.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "../src/data/csv_parser.h"
#include "../src/data/libfm_parser.h"
#include "../src/data/libsvm_parser.h"
#include "dmlc_oracle.h"

using dmlc::data::RowBlockContainer;

// TextParserBase caps its thread count at max(omp_get_num_procs() / 2 - 4, 1)
// (text_parser.h:32-35): 1 in an 8-CPU build container, 2 on the 256-core GPU
// host.  To run the genuine FillData range split with nthread > 1 here, this
// test library answers omp_get_num_procs from DMLC_REF_NPROCS when that is set
// (bound inside this .so by -Bsymbolic, oracle/Makefile, whatever OpenMP
// runtime the process loaded first), and forwards to libgomp otherwise.
extern "C" int omp_get_num_procs(void) {
  if (const char *e = std::getenv("DMLC_REF_NPROCS")) return std::atoi(e);
  using Fn = int (*)(void);
  static Fn real = reinterpret_cast<Fn>(dlsym(RTLD_NEXT, "omp_get_num_procs"));
  return real ? real() : 1;
}

namespace {

// An InputSplit over chunks already in memory (the ParseNext seam below).
class MemSplit : public dmlc::InputSplit {
 public:
  MemSplit(const char *buf, const uint64_t *off, int n) : buf_(buf), off_(off), n_(n) {}
  size_t GetTotalSize(void) override { return (size_t)off_[n_]; }
  void BeforeFirst(void) override { i_ = 0; }
  bool NextRecord(Blob *) override { return false; }
  bool NextChunk(Blob *out) override {
    if (i_ >= n_) return false;
    // a private copy with a NUL after its end, like the InputSplit's own buffer
    cur_.assign(buf_ + off_[i_], buf_ + off_[i_ + 1]);
    cur_.push_back('\0');
    out->dptr = &cur_[0];
    out->size = (size_t)(off_[i_ + 1] - off_[i_]);
    ++i_;
    return true;
  }
  void ResetPartition(unsigned, unsigned) override { i_ = 0; }

 private:
  const char *buf_;
  const uint64_t *off_;
  int n_, i_ = 0;
  std::vector<char> cur_;
};

template <typename I, typename D>
struct SvmSeam : public dmlc::data::LibSVMParser<I, D> {
  SvmSeam(const std::map<std::string, std::string> &a, int nt)
      : dmlc::data::LibSVMParser<I, D>(nullptr, a, nt) {}
  void Call(const char *b, const char *e, RowBlockContainer<I, D> *o) { this->ParseBlock(b, e, o); }
};
template <typename I, typename D>
struct CsvSeam : public dmlc::data::CSVParser<I, D> {
  CsvSeam(const std::map<std::string, std::string> &a, int nt)
      : dmlc::data::CSVParser<I, D>(nullptr, a, nt) {}
  void Call(const char *b, const char *e, RowBlockContainer<I, D> *o) { this->ParseBlock(b, e, o); }
};
template <typename I, typename D>
struct FmSeam : public dmlc::data::LibFMParser<I, D> {
  FmSeam(const std::map<std::string, std::string> &a, int nt)
      : dmlc::data::LibFMParser<I, D>(nullptr, a, nt) {}
  void Call(const char *b, const char *e, RowBlockContainer<I, D> *o) { this->ParseBlock(b, e, o); }
};

template <typename T>
void *dup(const T *p, size_t n) {
  if (n == 0) return nullptr;
  void *q = std::malloc(n * sizeof(T));
  std::memcpy(q, p, n * sizeof(T));
  return q;
}

// Append a RowBlock the way BasicRowIter::Init does (RowBlockContainer::Push).
template <typename I, typename D>
void append(dmo_csr *o, const dmlc::RowBlock<I, D> &b) {
  size_t rows = b.size;
  uint64_t shift = o->offset[o->n_rows];
  o->offset = (uint64_t *)std::realloc(o->offset, (o->n_rows + rows + 1) * 8);
  for (size_t i = 0; i < rows; ++i) o->offset[o->n_rows + 1 + i] = shift + b.offset[i + 1] - b.offset[0];
  size_t nd = b.offset[rows] - b.offset[0];
  // CSV without label_column yields label == NULL (BeginPtr of an empty vector)
  if (b.label) {
    o->label = std::realloc(o->label, (o->n_label + rows) * sizeof(D) + 1);
    std::memcpy((char *)o->label + o->n_label * sizeof(D), b.label, rows * sizeof(D));
    o->n_label += rows;
  }
  o->n_rows += rows;
  if (b.weight) {
    o->weight = (float *)std::realloc(o->weight, (o->n_weight + rows) * 4);
    std::memcpy(o->weight + o->n_weight, b.weight, rows * 4);
    o->n_weight += rows;
  }
  if (b.qid) {
    o->qid = (uint64_t *)std::realloc(o->qid, (o->n_qid + rows) * 8);
    std::memcpy(o->qid + o->n_qid, b.qid, rows * 8);
    o->n_qid += rows;
  }
  o->index = (uint64_t *)std::realloc(o->index, (o->n_index + nd) * 8 + 8);
  for (size_t i = 0; i < nd; ++i) o->index[o->n_index + i] = b.index[b.offset[0] + i];
  o->n_index += nd;
  if (b.field) {
    o->field = (uint64_t *)std::realloc(o->field, (o->n_field + nd) * 8 + 8);
    for (size_t i = 0; i < nd; ++i) o->field[o->n_field + i] = b.field[b.offset[0] + i];
    o->n_field += nd;
  }
  if (b.value) {
    o->value = std::realloc(o->value, (o->n_value + nd) * sizeof(D) + 1);
    std::memcpy((char *)o->value + o->n_value * sizeof(D), b.value + b.offset[0], nd * sizeof(D));
    o->n_value += nd;
  }
  size_t nb = o->n_blocks + 1;
  auto grow = [&](uint64_t *&a, uint64_t v) {
    a = (uint64_t *)std::realloc(a, nb * 8);
    a[nb - 1] = v;
  };
  grow(o->block_rows, rows);
  grow(o->block_index, nd);
  grow(o->block_value, b.value ? nd : 0);
  grow(o->block_weight, b.weight ? rows : 0);
  grow(o->block_qid, b.qid ? rows : 0);
  o->n_blocks = nb;
}

// Block-level seam: take the container's vectors directly.  (A RowBlock view
// carries no weight/qid counts; BasicRowIter copies `size` entries from them,
// row_block.h:131-136, which reads past the vector when only some rows carry a
// weight or qid -- so goldens are taken from the ParseBlock output itself.)
template <typename I, typename D>
void append_container(dmo_csr *o, const RowBlockContainer<I, D> &c) {
  if (c.Size() == 0) return;
  (void)c.GetBlock();  // same consistency CHECKs as Next() -> GetBlock()
  dmlc::RowBlock<I, D> b = c.GetBlock();
  b.weight = nullptr;
  b.qid = nullptr;
  append(o, b);
  o->block_weight[o->n_blocks - 1] = c.weight.size();
  o->block_qid[o->n_blocks - 1] = c.qid.size();
  if (!c.weight.empty()) {
    o->weight = (float *)std::realloc(o->weight, (o->n_weight + c.weight.size()) * 4);
    std::memcpy(o->weight + o->n_weight, c.weight.data(), c.weight.size() * 4);
    o->n_weight += c.weight.size();
  }
  if (!c.qid.empty()) {
    o->qid = (uint64_t *)std::realloc(o->qid, (o->n_qid + c.qid.size()) * 8);
    std::memcpy(o->qid + o->n_qid, c.qid.data(), c.qid.size() * 8);
    o->n_qid += c.qid.size();
  }
}

std::map<std::string, std::string> args_of(const dmo_params *p) {
  std::map<std::string, std::string> a;
  if (p->format == DMO_FMT_CSV) {
    a["label_column"] = std::to_string(p->label_column);
    a["weight_column"] = std::to_string(p->weight_column);
    a["delimiter"] = std::string(1, (char)p->delimiter);
  } else {
    a["indexing_mode"] = std::to_string(p->indexing_mode);
  }
  return a;
}

template <typename I, typename D>
int block_csv(const char *buf, size_t n, const dmo_params *p, dmo_csr *o) {
  std::string s(buf, n);  // NUL after the end, as test/unittest_parser.cc has
  RowBlockContainer<I, D> c;
  CsvSeam<I, D>(args_of(p), 1).Call(s.data(), s.data() + n, &c);
  append_container(o, c);
  return 0;
}

// libsvm / libfm exist only for DType = real_t (LibSVMParser derives from
// TextParserBase<IndexType> with the default DType, libsvm_parser.h:48).
template <typename I>
int block_sparse(const char *buf, size_t n, const dmo_params *p, dmo_csr *o) {
  std::string s(buf, n);
  RowBlockContainer<I, float> c;
  if (p->format == DMO_FMT_LIBSVM) SvmSeam<I, float>(args_of(p), 1).Call(s.data(), s.data() + n, &c);
  else FmSeam<I, float>(args_of(p), 1).Call(s.data(), s.data() + n, &c);
  append_container(o, c);
  return 0;
}

// FillData over each chunk with the parser's own nthread (the genuine range
// split, text_parser.h:116-155); every non-empty container is one block, as
// ParserImpl::Next hands them out (parser.h:32-48).
template <class P, typename I, typename D>
int chunks_typed(const char *buf, const uint64_t *off, int n, const dmo_params *p, dmo_csr *o) {
  P parser(new MemSplit(buf, off, n), args_of(p), p->nthread > 0 ? p->nthread : 1);
  std::vector<RowBlockContainer<I, D>> data;
  while (parser.ParseNext(&data))
    for (const auto &c : data) append_container(o, c);
  return 0;
}

template <typename I, typename D>
int uri_typed(const char *uri, unsigned part, unsigned nparts, const char *type, dmo_csr *o,
              double *seconds) {
  auto t0 = std::chrono::steady_clock::now();
  std::unique_ptr<dmlc::Parser<I, D>> parser(dmlc::Parser<I, D>::Create(uri, part, nparts, type));
  while (parser->Next()) append(o, parser->Value());
  auto t1 = std::chrono::steady_clock::now();
  if (seconds) *seconds = std::chrono::duration<double>(t1 - t0).count();
  return 0;
}

template <typename F>
int guarded(dmo_csr *o, F f) {
  try {
    return f();
  } catch (const std::exception &e) {
    o->status = 1;
    std::snprintf(o->msg, sizeof(o->msg), "%s", e.what());
    return 1;
  }
}

}  // namespace

extern "C" {

// One ParseBlock over [buf, buf+n) with nthread = 1 (unittest_parser.cc seam).
int ref_parse_block(const char *buf, size_t n, const dmo_params *p, dmo_csr *o) {
  return guarded(o, [&] {
    bool i64 = p->index_bits == 64;
    if (p->format != DMO_FMT_CSV)
      return i64 ? block_sparse<uint64_t>(buf, n, p, o) : block_sparse<uint32_t>(buf, n, p, o);
    switch (p->value_kind) {
      case DMO_VAL_F32:
        return i64 ? block_csv<uint64_t, float>(buf, n, p, o) : block_csv<uint32_t, float>(buf, n, p, o);
      case DMO_VAL_I32:
        return i64 ? block_csv<uint64_t, int32_t>(buf, n, p, o) : block_csv<uint32_t, int32_t>(buf, n, p, o);
      default:
        return i64 ? block_csv<uint64_t, int64_t>(buf, n, p, o) : block_csv<uint32_t, int64_t>(buf, n, p, o);
    }
  });
}

// Chunks buf[off[i], off[i+1]) through TextParserBase::FillData with
// p->nthread ranges each (set DMLC_REF_NPROCS >= 2 * nthread + 8 so the
// reference's cap admits them).
int ref_parse_chunks(const char *buf, const uint64_t *off, int n, const dmo_params *p, dmo_csr *o) {
  using namespace dmlc::data;
  return guarded(o, [&] {
    const bool i64 = p->index_bits == 64;
    if (p->format == DMO_FMT_LIBSVM)
      return i64 ? chunks_typed<LibSVMParser<uint64_t, float>, uint64_t, float>(buf, off, n, p, o)
                 : chunks_typed<LibSVMParser<uint32_t, float>, uint32_t, float>(buf, off, n, p, o);
    if (p->format == DMO_FMT_LIBFM)
      return i64 ? chunks_typed<LibFMParser<uint64_t, float>, uint64_t, float>(buf, off, n, p, o)
                 : chunks_typed<LibFMParser<uint32_t, float>, uint32_t, float>(buf, off, n, p, o);
    switch (p->value_kind) {
      case DMO_VAL_F32:
        return i64 ? chunks_typed<CSVParser<uint64_t, float>, uint64_t, float>(buf, off, n, p, o)
                   : chunks_typed<CSVParser<uint32_t, float>, uint32_t, float>(buf, off, n, p, o);
      case DMO_VAL_I32:
        return i64 ? chunks_typed<CSVParser<uint64_t, int32_t>, uint64_t, int32_t>(buf, off, n, p, o)
                   : chunks_typed<CSVParser<uint32_t, int32_t>, uint32_t, int32_t>(buf, off, n, p, o);
      default:
        return i64 ? chunks_typed<CSVParser<uint64_t, int64_t>, uint64_t, int64_t>(buf, off, n, p, o)
                   : chunks_typed<CSVParser<uint32_t, int64_t>, uint32_t, int64_t>(buf, off, n, p, o);
    }
  });
}

// Parser<I,D>::Create(uri, part, nparts, type) -> Next()/Value() concatenation.
int ref_parse_uri(const char *uri, unsigned part, unsigned nparts, const char *type, int index_bits,
                  int value_kind, dmo_csr *o, double *seconds) {
  return guarded(o, [&] {
    bool i64 = index_bits == 64;
    switch (value_kind) {
      case DMO_VAL_F32:
        return i64 ? uri_typed<uint64_t, float>(uri, part, nparts, type, o, seconds)
                   : uri_typed<uint32_t, float>(uri, part, nparts, type, o, seconds);
      case DMO_VAL_I32:
        return i64 ? uri_typed<uint64_t, int32_t>(uri, part, nparts, type, o, seconds)
                   : uri_typed<uint32_t, int32_t>(uri, part, nparts, type, o, seconds);
      default:
        return i64 ? uri_typed<uint64_t, int64_t>(uri, part, nparts, type, o, seconds)
                   : uri_typed<uint32_t, int64_t>(uri, part, nparts, type, o, seconds);
    }
  });
}

// InputSplit::Create(uri, part, nparts, "text") chunk sequence.
int ref_split_chunks(const char *uri, unsigned part, unsigned nparts, dmo_chunks *out) {
  std::memset(out, 0, sizeof(*out));
  out->off = (uint64_t *)std::calloc(1, 8);
  std::unique_ptr<dmlc::InputSplit> split(dmlc::InputSplit::Create(uri, part, nparts, "text"));
  dmlc::InputSplit::Blob blob;
  while (split->NextChunk(&blob)) {
    uint64_t base = out->off[out->n_chunks];
    out->buf = (char *)std::realloc(out->buf, base + blob.size + 1);
    std::memcpy(out->buf + base, blob.dptr, blob.size);
    out->n_chunks++;
    out->off = (uint64_t *)std::realloc(out->off, (out->n_chunks + 1) * 8);
    out->off[out->n_chunks] = base + blob.size;
  }
  return (int)out->n_chunks;
}

float ref_parse_float(const char *s, size_t *consumed) {
  char *end = nullptr;
  float v = dmlc::ParseFloat<float>(s, &end);
  if (consumed) *consumed = (size_t)(end - s);
  return v;
}

// Pure ParseBlock throughput over pre-loaded line-aligned chunks (bench.py
// cpu_baseline).  Thread model: `nthread` std::threads started once, thread t
// parsing whole chunks t, t + nthread, ... with the format's own ParseBlock
// (LibSVMParser / CSVParser / LibFMParser).  That is the reference's total
// parse work at `nthread`-way parallelism; it is not FillData's per-chunk
// split into nthread ranges with an OpenMP fork/join per chunk, whose
// overhead it leaves out (an upper bound on the reference's rate).
double ref_bench_blocks(const char *buf, const uint64_t *off, int nchunks, int format, int nthread,
                        uint64_t *nnz_out) {
  std::map<std::string, std::string> a;
  auto t0 = std::chrono::steady_clock::now();
  std::vector<std::thread> th;
  std::vector<uint64_t> nnz(nthread, 0);
  for (int t = 0; t < nthread; ++t) {
    th.emplace_back([&, t] {
      RowBlockContainer<uint32_t, float> c;
      std::unique_ptr<SvmSeam<uint32_t, float>> svm;
      std::unique_ptr<CsvSeam<uint32_t, float>> csv;
      std::unique_ptr<FmSeam<uint32_t, float>> fm;
      if (format == DMO_FMT_CSV) csv.reset(new CsvSeam<uint32_t, float>(a, 1));
      else if (format == DMO_FMT_LIBFM) fm.reset(new FmSeam<uint32_t, float>(a, 1));
      else svm.reset(new SvmSeam<uint32_t, float>(a, 1));
      for (int k = t; k < nchunks; k += nthread) {
        const char *b = buf + off[k], *e = buf + off[k + 1];
        if (csv) csv->Call(b, e, &c);
        else if (fm) fm->Call(b, e, &c);
        else svm->Call(b, e, &c);
        nnz[t] += c.index.size();
      }
    });
  }
  for (auto &x : th) x.join();
  auto t1 = std::chrono::steady_clock::now();
  uint64_t s = 0;
  for (auto v : nnz) s += v;
  if (nnz_out) *nnz_out = s;
  return std::chrono::duration<double>(t1 - t0).count();
}

}  // extern "C"
