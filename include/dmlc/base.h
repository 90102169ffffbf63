/*
 * dmlc/base.h -- the base layer of dmlc-core's public headers that the
 * parser API uses (this build's own header, API-compatible with the
 * reference's include/dmlc/base.h): the dmlc::Error exception that
 * LOG(FATAL) / CHECK throw (reference: DMLC_LOG_FATAL_THROW, base.h:33-35,
 * logging.h:437-452), BeginPtr (base.h:280-300: NULL for an empty vector --
 * what makes RowBlock.weight / qid / field / value NULL), and the macros the
 * registry and data headers build on.
 */
#ifndef DMLC_BASE_H_
#define DMLC_BASE_H_

#include <cstddef>
#include <cstdint>
#include <stdexcept>
#include <string>
#include <vector>

#define DMLC_USE_CXX11 1
#define DMLC_STRICT_CXX11 1
#define DMLC_ENABLE_STD_THREAD 1
#define DMLC_LOG_FATAL_THROW 1
#define DMLC_THROW_EXCEPTION noexcept(false)
#define DMLC_NO_EXCEPTION noexcept(true)
#define DMLC_ATTRIBUTE_UNUSED __attribute__((unused))
#define DMLC_STR_CONCAT_(a, b) a##b
#define DMLC_STR_CONCAT(a, b) DMLC_STR_CONCAT_(a, b)

namespace dmlc {

/*! \brief exception thrown by LOG(FATAL) / CHECK failures: malformed input, bad arguments, I/O errors */
struct Error : public std::runtime_error {
  explicit Error(const std::string &s) : std::runtime_error(s) {}
};

/*! \brief pointer to the first element, NULL for an empty vector */
template <typename T>
inline T *BeginPtr(std::vector<T> &v) {
  return v.empty() ? nullptr : v.data();
}
template <typename T>
inline const T *BeginPtr(const std::vector<T> &v) {
  return v.empty() ? nullptr : v.data();
}
inline char *BeginPtr(std::string &s) { return s.empty() ? nullptr : &s[0]; }
inline const char *BeginPtr(const std::string &s) { return s.empty() ? nullptr : s.data(); }

}  // namespace dmlc

#endif  // DMLC_BASE_H_
