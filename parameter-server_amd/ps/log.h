// ps/log.h — LOG / CHECK macros with the reference's error convention: a failed
// CHECK throws ps_log::PSError (reference src/base/log.h:283-304,
// LOG_FATAL_THROW=1 in src/base/base.h:19-21).  LOG(INFO) prints only when
// PS_VERBOSE >= 1; WARNING and ERROR always print to stderr.
#pragma once
// the standard headers the reference's log.h brings in (log.h:24-45): harness
// code relies on them transitively (std::put_time in tests/LR_ps.cpp:54)
#include <chrono>
#include <ctime>
#include <fstream>
#include <iomanip>
#include <iostream>
#include <sstream>
#include <stdexcept>
#include <string>

#if defined(__GLIBCXX__) && defined(_GLIBCXX_RELEASE) && _GLIBCXX_RELEASE < 13 && __cplusplus >= 202002L
// C++20 streams std::chrono::duration (count + unit suffix); libstdc++ gained
// that operator in release 13.  tests/LR_ps.cpp:88 needs it, so older
// libstdc++ gets the same output format here — declared in the GLOBAL
// namespace (adding it to namespace std would be undefined behaviour): the
// harness's expression is in the global namespace, where ordinary lookup
// finds it.
template <class Rep, class Period>
std::ostream& operator<<(std::ostream& os, const std::chrono::duration<Rep, Period>& d) {
  os << d.count();
  if constexpr (std::is_same_v<Period, std::nano>) os << "ns";
  else if constexpr (std::is_same_v<Period, std::micro>) os << "\xC2\xB5s";
  else if constexpr (std::is_same_v<Period, std::milli>) os << "ms";
  else if constexpr (std::is_same_v<Period, std::ratio<1>>) os << "s";
  else if constexpr (std::is_same_v<Period, std::ratio<60>>) os << "min";
  else if constexpr (std::is_same_v<Period, std::ratio<3600>>) os << "h";
  else os << "[" << Period::num << "/" << Period::den << "]s";
  return os;
}
#endif

namespace ps_log {

class PSError : public std::runtime_error {
 public:
  explicit PSError(const std::string& s) : std::runtime_error(s) {}
};

enum Severity { INFO = 0, WARNING = 1, ERROR = 2, FATAL = 3 };

int Verbosity();
void Emit(int severity, const std::string& line);
/* per-node log file (argv[2] of ps::Start); empty = stderr only */
void InitLogging(const char* log_filename);

class LogMessage {
 public:
  LogMessage(const char* file, int line, int severity) : severity_(severity) {
    const char* base = file;
    for (const char* p = file; *p; ++p)
      if (*p == '/') base = p + 1;
    static const char kTag[] = "IWEF";
    s_ << '[' << kTag[severity & 3] << ' ' << base << ':' << line << "] ";
  }
  ~LogMessage() {
    if (severity_ >= WARNING || Verbosity() >= 1) Emit(severity_, s_.str());
  }
  std::ostream& stream() { return s_; }

 private:
  std::ostringstream s_;
  int severity_;
};

class LogMessageFatal {
 public:
  LogMessageFatal(const char* file, int line) {
    const char* base = file;
    for (const char* p = file; *p; ++p)
      if (*p == '/') base = p + 1;
    s_ << '[' << base << ':' << line << "] ";
  }
  ~LogMessageFatal() noexcept(false) {
    Emit(FATAL, s_.str());
    throw PSError(s_.str());
  }
  std::ostream& stream() { return s_; }

 private:
  std::ostringstream s_;
};

// Swallows the stream expression of a passing CHECK (the glog `voidify` trick).
struct Voidify {
  void operator&(std::ostream&) {}
};

template <typename T>
T CheckNotNull(const char* file, int line, const char* expr, T&& t) {
  if (t == nullptr) LogMessageFatal(file, line).stream() << "Check failed: " << expr << " must be non NULL";
  return std::forward<T>(t);
}

}  // namespace ps_log

#define PSLOG_STREAM_INFO ps_log::LogMessage(__FILE__, __LINE__, ps_log::INFO).stream()
#define PSLOG_STREAM_WARNING ps_log::LogMessage(__FILE__, __LINE__, ps_log::WARNING).stream()
#define PSLOG_STREAM_ERROR ps_log::LogMessage(__FILE__, __LINE__, ps_log::ERROR).stream()
#define PSLOG_STREAM_FATAL ps_log::LogMessageFatal(__FILE__, __LINE__).stream()

#define LOG(severity) ps_log::Voidify() & PSLOG_STREAM_##severity
#define LOG_IF(severity, cond) !(cond) ? (void)0 : ps_log::Voidify() & PSLOG_STREAM_##severity

#define CHECK(cond) \
  (cond) ? (void)0 : ps_log::Voidify() & ps_log::LogMessageFatal(__FILE__, __LINE__).stream() << "Check failed: " #cond " "

#define PS_CHECK_OP(a, b, op) \
  CHECK((a)op(b)) << "(" << (a) << " vs. " << (b) << ") "
#define CHECK_EQ(a, b) PS_CHECK_OP(a, b, ==)
#define CHECK_NE(a, b) PS_CHECK_OP(a, b, !=)
#define CHECK_LT(a, b) PS_CHECK_OP(a, b, <)
#define CHECK_LE(a, b) PS_CHECK_OP(a, b, <=)
#define CHECK_GT(a, b) PS_CHECK_OP(a, b, >)
#define CHECK_GE(a, b) PS_CHECK_OP(a, b, >=)
#define CHECK_NOTNULL(x) ps_log::CheckNotNull(__FILE__, __LINE__, #x, (x))

#define DCHECK(cond) CHECK(cond)
#define DCHECK_EQ(a, b) CHECK_EQ(a, b)
