// host_api_test.cc -- TEST DRIVER: exercises the drop-in C++ API
// (include/dmlc/data.h: dmlc::Parser / RowBlockIter / the parser registry) on
// real files and dumps the concatenated result (RowBlockContainer::Push
// order, as BasicRowIter builds it) plus each block's row count, for
// tests/test_host_api.py to compare with the oracle.
//   host_api_test <uri> <part> <nparts> <type> <index_bits 32|64> <dtype f32|i32|i64> <out_prefix> [iter]
//   host_api_test --api <libsvm file>     RowBlock / Row CHECKs, MemCostBytes, a registered parser type
// Built twice: against this build's include/dmlc (tests/cpp/Makefile) and
// against the reference's own headers and library with the HIP plugin
// (oracle/Makefile target plugin) -- the same source on both sides of the
// drop-in boundary.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <memory>
#include <string>
#include <vector>

#include "dmlc/data.h"

template <typename T>
static void dump(const std::string &p, const std::vector<T> &v) {
  FILE *f = std::fopen(p.c_str(), "wb");
  if (!v.empty()) std::fwrite(v.data(), sizeof(T), v.size(), f);
  std::fclose(f);
}

template <typename I, typename D>
static int run(const char *uri, unsigned part, unsigned nparts, const char *type, const std::string &o,
               bool iter) {
  std::vector<uint64_t> offset(1, 0), qid, block_rows;
  std::vector<D> label, value;
  std::vector<float> weight;
  std::vector<I> index, field;
  size_t blocks = 0, bytes = 0, numcol = 0;
  bool rebased = true;
  auto push = [&](const dmlc::RowBlock<I, D> &b) {
    ++blocks;
    block_rows.push_back(b.size);
    if (b.offset[0] != 0) rebased = false;  // ParserImpl::Next's blocks start at 0 (GetBlock)
    const uint64_t base = offset.back();
    for (size_t i = 0; i < b.size; ++i) offset.push_back(base + b.offset[i + 1] - b.offset[0]);
    if (b.label) label.insert(label.end(), b.label, b.label + b.size);
    if (b.weight) weight.insert(weight.end(), b.weight, b.weight + b.size);
    if (b.qid) qid.insert(qid.end(), b.qid, b.qid + b.size);
    index.insert(index.end(), b.index + b.offset[0], b.index + b.offset[b.size]);
    if (b.field) field.insert(field.end(), b.field + b.offset[0], b.field + b.offset[b.size]);
    if (b.value) value.insert(value.end(), b.value + b.offset[0], b.value + b.offset[b.size]);
  };
  try {
    if (iter) {
      dmlc::RowBlockIter<I, D> *it = dmlc::RowBlockIter<I, D>::Create(uri, part, nparts, type);
      for (int pass = 0; pass < 2; ++pass) {  // BeforeFirst re-iteration
        it->BeforeFirst();
        if (pass == 1)
          while (it->Next()) push(it->Value());
        else
          while (it->Next()) {
          }
      }
      numcol = it->NumCol();
      delete it;
    } else {
      dmlc::Parser<I, D> *p = dmlc::Parser<I, D>::Create(uri, part, nparts, type);
      while (p->Next()) {
      }
      p->BeforeFirst();  // a full second pass must give the same blocks
      while (p->Next()) push(p->Value());
      bytes = p->BytesRead();
      delete p;
    }
  } catch (const dmlc::Error &e) {
    FILE *f = std::fopen((o + ".error").c_str(), "w");
    std::fputs(e.what(), f);
    std::fclose(f);
    return 3;
  }
  if (!rebased) return 4;
  dump(o + ".offset", offset);
  dump(o + ".label", label);
  dump(o + ".weight", weight);
  dump(o + ".qid", qid);
  dump(o + ".index", index);
  dump(o + ".field", field);
  dump(o + ".value", value);
  dump(o + ".blocks", block_rows);
  std::vector<uint64_t> meta = {blocks, bytes, numcol};
  dump(o + ".meta", meta);
  return 0;
}

// ---- the plugin API: a parser type registered by this program, found by
// Parser::Create through the registry (data.h DMLC_REGISTER_DATA_PARSER)
namespace {
// delegates to the registered "libsvm" parser and counts the blocks it hands out
class CountingParser : public dmlc::Parser<uint32_t, dmlc::real_t> {
 public:
  explicit CountingParser(dmlc::Parser<uint32_t, dmlc::real_t> *in) : in_(in) {}
  void BeforeFirst() override { in_->BeforeFirst(); }
  bool Next() override {
    const bool ok = in_->Next();
    blocks += ok;
    return ok;
  }
  const dmlc::RowBlock<uint32_t, dmlc::real_t> &Value() const override { return in_->Value(); }
  size_t BytesRead() const override { return in_->BytesRead(); }
  static size_t blocks;

 private:
  std::unique_ptr<dmlc::Parser<uint32_t, dmlc::real_t>> in_;
};
size_t CountingParser::blocks = 0;

dmlc::Parser<uint32_t, dmlc::real_t> *CreateCounting(const std::string &path,
                                                    const std::map<std::string, std::string> &args,
                                                    unsigned part, unsigned nparts) {
  const auto *e = dmlc::Registry<dmlc::ParserFactoryReg<uint32_t, dmlc::real_t>>::Find("libsvm");
  return new CountingParser((*e->body)(path, args, part, nparts));
}
}  // namespace

namespace dmlc {
DMLC_REGISTER_DATA_PARSER(uint32_t, real_t, counting_libsvm, CreateCounting);
}

template <typename F>
static bool raises(F f) {
  try {
    f();
  } catch (const dmlc::Error &) {
    return true;
  }
  return false;
}

static int api_checks(const char *path) {
  int bad = 0;
  auto expect = [&](bool ok, const char *what) {
    if (!ok) {
      std::fprintf(stderr, "api check failed: %s\n", what);
      ++bad;
    }
  };
  std::unique_ptr<dmlc::Parser<uint32_t>> p(dmlc::Parser<uint32_t>::Create(path, 0, 1, "counting_libsvm"));
  size_t rows = 0;
  while (p->Next()) {
    const dmlc::RowBlock<uint32_t> &b = p->Value();
    rows += b.size;
    expect(b.offset[0] == 0, "block offset[0] == 0");
    // MemCostBytes as reference data.h:200-219 counts it
    const size_t nd = b.offset[b.size];
    size_t cost = b.size * (sizeof(size_t) + sizeof(float)) + nd * sizeof(uint32_t);
    if (b.weight) cost += b.size * sizeof(float);
    if (b.qid) cost += b.size * sizeof(size_t);
    if (b.field) cost += nd * sizeof(uint32_t);
    if (b.value) cost += nd * sizeof(float);
    expect(b.MemCostBytes() == cost, "MemCostBytes");
    expect(raises([&] { (void)b[b.size]; }), "operator[] CHECK(rowid < size)");
    expect(raises([&] { (void)b.Slice(1, b.size + 1); }), "Slice CHECK(end <= size)");
    const dmlc::RowBlock<uint32_t> s = b.Slice(1, b.size);
    expect(s.size == b.size - 1 && s.offset == b.offset + 1, "Slice shares the arrays");
    const dmlc::Row<uint32_t> r = b[0];
    std::vector<float> w(1u << 20, 0.5f);
    float want = 0;
    for (size_t i = 0; i < r.length; ++i) want += 0.5f * r.get_value(i);
    expect(std::fabs(r.SDot(w.data(), w.size()) - want) < 1e-3f, "SDot");
    expect(raises([&] { (void)r.SDot(w.data(), 0); }), "SDot CHECK(index < size)");
    expect(r.get_weight() == 1.0f && r.get_qid() == 0, "Row defaults");
  }
  expect(rows > 0 && CountingParser::blocks > 0, "registered type parsed through Parser::Create");
  expect(raises([&] { delete dmlc::Parser<uint32_t>::Create(path, 0, 1, "no_such_type"); }), "unknown type raises");
  const auto names = dmlc::Registry<dmlc::ParserFactoryReg<uint32_t, dmlc::real_t>>::ListAllNames();
  for (const char *n : {"libsvm", "libfm", "csv", "counting_libsvm"})
    expect(std::find(names.begin(), names.end(), std::string(n)) != names.end(), "registered type names");
  return bad ? 5 : 0;
}

int main(int argc, char **argv) {
  if (argc == 3 && std::strcmp(argv[1], "--api") == 0) return api_checks(argv[2]);
  if (argc < 8) {
    std::fprintf(stderr, "usage: see source\n");
    return 2;
  }
  const unsigned part = std::atoi(argv[2]), nparts = std::atoi(argv[3]);
  const bool wide = std::strcmp(argv[5], "64") == 0, iter = argc > 8;
  const std::string dt = argv[6], o = argv[7];
  if (dt == "f32") return wide ? run<uint64_t, float>(argv[1], part, nparts, argv[4], o, iter)
                               : run<uint32_t, float>(argv[1], part, nparts, argv[4], o, iter);
  if (dt == "i32") return wide ? run<uint64_t, int32_t>(argv[1], part, nparts, argv[4], o, iter)
                               : run<uint32_t, int32_t>(argv[1], part, nparts, argv[4], o, iter);
  return wide ? run<uint64_t, int64_t>(argv[1], part, nparts, argv[4], o, iter)
              : run<uint32_t, int64_t>(argv[1], part, nparts, argv[4], o, iter);
}
