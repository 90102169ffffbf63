// host_api_test.cc -- TEST DRIVER: exercises the drop-in C++ API
// (include/dmlc/data.h: dmlc::Parser / RowBlockIter) on real files and dumps
// the concatenated result (RowBlockContainer::Push order, as BasicRowIter
// builds it) for tests/test_host_api.py to compare with the oracle.
//   host_api_test <uri> <part> <nparts> <type> <index_bits 32|64> <dtype f32|i32|i64> <out_prefix> [iter]
#include <cstdint>
#include <cstdio>
#include <cstring>
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
  std::vector<uint64_t> offset(1, 0), qid;
  std::vector<D> label, value;
  std::vector<float> weight;
  std::vector<I> index, field;
  size_t blocks = 0, bytes = 0, numcol = 0;
  auto push = [&](const dmlc::RowBlock<I, D> &b) {
    ++blocks;
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
  dump(o + ".offset", offset);
  dump(o + ".label", label);
  dump(o + ".weight", weight);
  dump(o + ".qid", qid);
  dump(o + ".index", index);
  dump(o + ".field", field);
  dump(o + ".value", value);
  std::vector<uint64_t> meta = {blocks, bytes, numcol};
  dump(o + ".meta", meta);
  return 0;
}

int main(int argc, char **argv) {
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
