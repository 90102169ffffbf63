/*
 * dmlc/registry.h -- the global name -> entry registry dmlc-core's plugin
 * points use (reference include/dmlc/registry.h: Registry<E>::Get / Find /
 * __REGISTER__, FunctionRegEntryBase, DMLC_REGISTRY_ENABLE and
 * DMLC_REGISTRY_REGISTER).  Parser factories register here through
 * DMLC_REGISTER_DATA_PARSER (dmlc/data.h), so a library or program can add a
 * parser type that Parser<I,D>::Create(uri, part, nparts, "<name>") then finds.
 * This build's own implementation of that contract.
 */
#ifndef DMLC_REGISTRY_H_
#define DMLC_REGISTRY_H_

#include <map>
#include <string>
#include <vector>

#include "./base.h"
#include "./logging.h"

namespace dmlc {

/*! \brief description of one argument of a registered function */
struct ParamFieldInfo {
  std::string name;
  std::string type;
  std::string type_info_str;
  std::string description;
};

/*!
 * \brief registry of entries of type EntryType, one instance per type
 * (the instance is defined by DMLC_REGISTRY_ENABLE(EntryType) in exactly one
 * translation unit).
 */
template <typename EntryType>
class Registry {
 public:
  /*! \brief every registered entry, in registration order */
  static const std::vector<const EntryType *> &List() { return Get()->const_list_; }
  /*! \brief names of every entry, aliases included */
  static std::vector<std::string> ListAllNames() {
    std::vector<std::string> names;
    for (const auto &kv : Get()->fmap_) names.push_back(kv.first);
    return names;
  }
  /*! \brief the entry registered under `name`, or NULL */
  static const EntryType *Find(const std::string &name) {
    const auto &m = Get()->fmap_;
    auto it = m.find(name);
    return it == m.end() ? nullptr : it->second;
  }
  /*! \brief make `alias` another name of the entry `key_name` */
  void AddAlias(const std::string &key_name, const std::string &alias) {
    auto it = fmap_.find(key_name);
    CHECK(it != fmap_.end()) << "Cannot find entry " << key_name << " to alias";
    auto jt = fmap_.find(alias);
    if (jt != fmap_.end()) {
      CHECK(jt->second == it->second) << "Entry " << alias << " is already registered";
    } else {
      fmap_[alias] = it->second;
    }
  }
  /*! \brief register a new entry (a name may be registered once) */
  EntryType &__REGISTER__(const std::string &name) {
    CHECK_EQ(fmap_.count(name), 0U) << name << " already registered";
    EntryType *e = new EntryType();
    e->name = name;
    fmap_[name] = e;
    entry_list_.push_back(e);
    const_list_.push_back(e);
    return *e;
  }
  /*! \brief the entry `name`, registered now if it was not */
  EntryType &__REGISTER_OR_GET__(const std::string &name) {
    auto it = fmap_.find(name);
    return it == fmap_.end() ? __REGISTER__(name) : *it->second;
  }
  /*! \brief the singleton (defined by DMLC_REGISTRY_ENABLE) */
  static Registry *Get();

 private:
  Registry() = default;
  ~Registry() {
    for (EntryType *e : entry_list_) delete e;
  }
  std::vector<EntryType *> entry_list_;
  std::vector<const EntryType *> const_list_;
  std::map<std::string, EntryType *> fmap_;
};

/*!
 * \brief base of registry entries that carry a function: name, description,
 * argument list and the function itself (`body`).
 */
template <typename EntryType, typename FunctionType>
class FunctionRegEntryBase {
 public:
  std::string name;
  std::string description;
  std::vector<ParamFieldInfo> arguments;
  FunctionType body;
  std::string return_type;

  EntryType &set_body(FunctionType b) {
    body = b;
    return self();
  }
  EntryType &describe(const std::string &d) {
    description = d;
    return self();
  }
  EntryType &add_argument(const std::string &n, const std::string &type, const std::string &d) {
    ParamFieldInfo info;
    info.name = n;
    info.type = type;
    info.type_info_str = type;
    info.description = d;
    arguments.push_back(info);
    return self();
  }
  EntryType &add_arguments(const std::vector<ParamFieldInfo> &args) {
    arguments.insert(arguments.end(), args.begin(), args.end());
    return self();
  }
  EntryType &set_return_type(const std::string &t) {
    return_type = t;
    return self();
  }

 protected:
  EntryType &self() { return *static_cast<EntryType *>(this); }
};

}  // namespace dmlc

/*! \brief define the registry instance of EntryType (once per program; use inside namespace dmlc) */
#define DMLC_REGISTRY_ENABLE(EntryType)            \
  template <>                                      \
  Registry<EntryType> *Registry<EntryType>::Get() { \
    static Registry<EntryType> inst;               \
    return &inst;                                  \
  }

/*! \brief register an entry named `Name` at static-initialisation time */
#define DMLC_REGISTRY_REGISTER(EntryType, EntryTypeName, Name)                             \
  static DMLC_ATTRIBUTE_UNUSED EntryType &__make_##EntryTypeName##_##Name##__ = \
      ::dmlc::Registry<EntryType>::Get()->__REGISTER__(#Name)

/*! \brief tags that keep a registering object file linked into static builds */
#define DMLC_REGISTRY_FILE_TAG(UniqueTag) \
  int __dmlc_registry_file_tag_##UniqueTag##__() { return 0; }
#define DMLC_REGISTRY_LINK_TAG(UniqueTag)              \
  int __dmlc_registry_file_tag_##UniqueTag##__();       \
  static int DMLC_ATTRIBUTE_UNUSED __reg_file_tag_##UniqueTag##__ = __dmlc_registry_file_tag_##UniqueTag##__();

#endif  // DMLC_REGISTRY_H_
