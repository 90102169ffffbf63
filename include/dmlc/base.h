/*
 * dmlc/base.h -- the small part of dmlc-core's base/logging layer that the
 * parser API exposes to callers (this build's own header, API-compatible):
 * parse failures surface as dmlc::Error, as LOG(FATAL)/CHECK do in the
 * reference with DMLC_LOG_FATAL_THROW (include/dmlc/logging.h:437-452,
 * include/dmlc/base.h:33-35).
 */
#ifndef DMLC_BASE_H_
#define DMLC_BASE_H_

#include <stdexcept>
#include <string>

namespace dmlc {

/*! \brief exception thrown by the parser path on malformed input or I/O failure */
struct Error : public std::runtime_error {
  explicit Error(const std::string &s) : std::runtime_error(s) {}
};

}  // namespace dmlc

#endif  // DMLC_BASE_H_
