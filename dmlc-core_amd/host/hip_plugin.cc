// hip_plugin.cc -- the MI355X text parsers as a plugin of an UNMODIFIED
// dmlc-core: compiled against the reference's own include/dmlc headers and
// linked with its libdmlc plus libdmlc_amd.so (the C ABI), it registers
//
//   libsvm_hip  Parser<uint32_t|uint64_t, real_t>
//   libfm_hip   Parser<uint32_t|uint64_t, real_t>
//   csv_hip     Parser<uint32_t|uint64_t, real_t|int32_t|int64_t>
//
// through DMLC_REGISTER_DATA_PARSER (reference include/dmlc/data.h:329-363),
// the same registry src/data.cc:189-227 fills, so a caller selects the GPU
// path with Parser<I,D>::Create(uri, part, nparts, "libsvm_hip") -- or
// "auto" with ?format=libsvm_hip -- and everything else stays the
// reference's: chunks come from its own InputSplit::Create(path, part,
// nparts, "text") (src/io unchanged), errors are its dmlc::Error.  The parse
// itself is hip_engine.h's HipTextParser (FillData ranges, per-range blocks,
// parse-ahead on the GPU).  INTEGRATION.md §3 shows the build lines;
// oracle/Makefile (target plugin) builds it with the reference's test driver.
#include <map>
#include <string>

#include "dmlc/data.h"
#include "dmlc/io.h"
#include "hip_engine.h"

namespace dmlc_amd {
namespace plugin {

template <typename I, typename D>
dmlc::Parser<I, D> *Create(const std::string &format, const std::string &path,
                           const std::map<std::string, std::string> &args, unsigned part, unsigned nparts) {
  std::map<std::string, std::string> a = args;
  auto f = a.find("format");  // "auto" with format=<format>_hip reaches this factory
  if (f != a.end() && f->second == format + "_hip") f->second = format;
  EngineConfig cfg;
  cfg.prm = make_params<I, D>(format, a);
  cfg.prm.nthread = reference_nthread();  // TextParserBase's cap of the factories' 2
  cfg.from_env();
  return new HipTextParser<I, D>(new InputSplitSource(dmlc::InputSplit::Create(path.c_str(), part, nparts, "text")),
                                 cfg);
}

template <typename I, typename D>
dmlc::Parser<I, D> *CreateLibSVM(const std::string &path, const std::map<std::string, std::string> &args,
                                 unsigned part, unsigned nparts) {
  return Create<I, D>("libsvm", path, args, part, nparts);
}
template <typename I, typename D>
dmlc::Parser<I, D> *CreateLibFM(const std::string &path, const std::map<std::string, std::string> &args,
                                unsigned part, unsigned nparts) {
  return Create<I, D>("libfm", path, args, part, nparts);
}
template <typename I, typename D>
dmlc::Parser<I, D> *CreateCSV(const std::string &path, const std::map<std::string, std::string> &args,
                              unsigned part, unsigned nparts) {
  return Create<I, D>("csv", path, args, part, nparts);
}

}  // namespace plugin
}  // namespace dmlc_amd

namespace dmlc {
DMLC_REGISTER_DATA_PARSER(uint32_t, real_t, libsvm_hip, dmlc_amd::plugin::CreateLibSVM<uint32_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, real_t, libsvm_hip, dmlc_amd::plugin::CreateLibSVM<uint64_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, real_t, libfm_hip, dmlc_amd::plugin::CreateLibFM<uint32_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, real_t, libfm_hip, dmlc_amd::plugin::CreateLibFM<uint64_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, real_t, csv_hip, dmlc_amd::plugin::CreateCSV<uint32_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, real_t, csv_hip, dmlc_amd::plugin::CreateCSV<uint64_t __DMLC_COMMA real_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, int32_t, csv_hip, dmlc_amd::plugin::CreateCSV<uint32_t __DMLC_COMMA int32_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, int32_t, csv_hip, dmlc_amd::plugin::CreateCSV<uint64_t __DMLC_COMMA int32_t>);
DMLC_REGISTER_DATA_PARSER(uint32_t, int64_t, csv_hip, dmlc_amd::plugin::CreateCSV<uint32_t __DMLC_COMMA int64_t>);
DMLC_REGISTER_DATA_PARSER(uint64_t, int64_t, csv_hip, dmlc_amd::plugin::CreateCSV<uint64_t __DMLC_COMMA int64_t>);
}  // namespace dmlc
