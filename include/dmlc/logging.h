/*
 * dmlc/logging.h -- CHECK / LOG macros with dmlc-core's contract
 * (reference include/dmlc/logging.h): LOG(FATAL) and a failed CHECK throw
 * dmlc::Error carrying the message ("Check failed: <expr>" followed by what
 * the caller streams), LOG(INFO|WARNING|ERROR) write a line to stderr.
 * This build's own implementation; callers written against the reference's
 * macros compile unchanged.
 */
#ifndef DMLC_LOGGING_H_
#define DMLC_LOGGING_H_

#include <cstdio>
#include <ctime>
#include <iostream>
#include <sstream>
#include <string>

#include "./base.h"

namespace dmlc {

/*! \brief "[hh:mm:ss] file:line: " prefix of every log line */
inline std::string LogPrefix(const char *file, int line) {
  char tb[16] = {0};
  const std::time_t t = std::time(nullptr);
  std::tm tm;
  localtime_r(&t, &tm);
  std::strftime(tb, sizeof(tb), "%H:%M:%S", &tm);
  std::ostringstream os;
  os << "[" << tb << "] " << file << ":" << line << ": ";
  return os.str();
}

/*! \brief a message that becomes a dmlc::Error when the statement ends */
class LogMessageFatal {
 public:
  LogMessageFatal(const char *file, int line) { os_ << LogPrefix(file, line); }
  std::ostringstream &stream() { return os_; }
  ~LogMessageFatal() DMLC_THROW_EXCEPTION { throw Error(os_.str()); }

 private:
  std::ostringstream os_;
};

/*! \brief a line written to stderr when the statement ends */
class LogMessage {
 public:
  LogMessage(const char *file, int line) { os_ << LogPrefix(file, line); }
  std::ostringstream &stream() { return os_; }
  ~LogMessage() {
    os_ << '\n';
    std::cerr << os_.str() << std::flush;
  }

 private:
  std::ostringstream os_;
};

/*! \brief swallows a stream expression so the conditional forms below have type void */
class LogMessageVoidify {
 public:
  void operator&(std::ostream &) {}
};

}  // namespace dmlc

#define LOG_FATAL ::dmlc::LogMessageFatal(__FILE__, __LINE__)
#define LOG_INFO ::dmlc::LogMessage(__FILE__, __LINE__)
#define LOG_WARNING ::dmlc::LogMessage(__FILE__, __LINE__)
#define LOG_ERROR ::dmlc::LogMessage(__FILE__, __LINE__)
#define LOG(severity) LOG_##severity.stream()
#define LOG_IF(severity, cond) !(cond) ? (void)0 : ::dmlc::LogMessageVoidify() & LOG(severity)

#define CHECK(x) \
  if (x) {       \
  } else         \
    ::dmlc::LogMessageFatal(__FILE__, __LINE__).stream() << "Check failed: " #x << ": "
#define DMLC_CHECK_OP_(x, y, op)                                                                      \
  if ((x)op(y)) {                                                                                    \
  } else                                                                                             \
    ::dmlc::LogMessageFatal(__FILE__, __LINE__).stream() << "Check failed: " #x " " #op " " #y " (" \
                                                         << (x) << " vs. " << (y) << ") "
#define CHECK_EQ(x, y) DMLC_CHECK_OP_(x, y, ==)
#define CHECK_NE(x, y) DMLC_CHECK_OP_(x, y, !=)
#define CHECK_LT(x, y) DMLC_CHECK_OP_(x, y, <)
#define CHECK_LE(x, y) DMLC_CHECK_OP_(x, y, <=)
#define CHECK_GT(x, y) DMLC_CHECK_OP_(x, y, >)
#define CHECK_GE(x, y) DMLC_CHECK_OP_(x, y, >=)
#define CHECK_NOTNULL(x) \
  ((x) == nullptr ? (::dmlc::LogMessageFatal(__FILE__, __LINE__).stream() << "Check notnull: " #x, (x)) : (x))

#endif  // DMLC_LOGGING_H_
