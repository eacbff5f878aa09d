// log_env.cc — logging sink and the JSON config loader (reference
// src/base/log.h:53-58, src/internal/Env.cpp:28-83).
#include <cctype>
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <mutex>
#include <sstream>

#include "internal/Env.h"
#include "ps/log.h"

namespace ps_log {

static std::mutex g_log_mu;
static thread_local std::ofstream* t_log_file = nullptr;

int Verbosity() {
  static int v = [] {
    const char* e = std::getenv("PS_VERBOSE");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

void Emit(int severity, const std::string& line) {
  (void)severity;
  std::lock_guard<std::mutex> lk(g_log_mu);
  std::cerr << line << std::endl;
  if (t_log_file && t_log_file->good()) (*t_log_file) << line << std::endl;
}

void InitLogging(const char* log_filename) {
  if (!log_filename || !*log_filename) return;
  // one file per node thread; opened once and kept for the thread's lifetime
  if (!t_log_file) t_log_file = new std::ofstream(log_filename, std::ios::app);
}

}  // namespace ps_log

namespace ps {

namespace {

// Minimal parser for the flat config objects tests/local.py writes
// ({"KEY": "str" | 123 | 1.5 | true, ...}).  Nested values are skipped.
struct FlatJson {
  const std::string& s;
  size_t i = 0;
  explicit FlatJson(const std::string& str) : s(str) {}
  void ws() {
    while (i < s.size() && std::isspace((unsigned char)s[i])) ++i;
  }
  bool str(std::string* out) {
    ws();
    if (i >= s.size() || s[i] != '"') return false;
    ++i;
    out->clear();
    while (i < s.size() && s[i] != '"') {
      if (s[i] == '\\' && i + 1 < s.size()) {
        ++i;
        char c = s[i];
        out->push_back(c == 'n' ? '\n' : c == 't' ? '\t' : c);
      } else {
        out->push_back(s[i]);
      }
      ++i;
    }
    ++i;
    return true;
  }
  void skip_value() {
    ws();
    int depth = 0;
    bool in_str = false;
    for (; i < s.size(); ++i) {
      char c = s[i];
      if (in_str) {
        if (c == '\\') ++i;
        else if (c == '"') in_str = false;
        continue;
      }
      if (c == '"') in_str = true;
      else if (c == '{' || c == '[') ++depth;
      else if (c == '}' || c == ']') {
        if (depth == 0) return;
        --depth;
        if (depth == 0) { ++i; return; }
      } else if (c == ',' && depth == 0) return;
    }
  }
  bool value(std::string* out) {
    ws();
    if (i < s.size() && s[i] == '"') return str(out);
    if (i < s.size() && (s[i] == '{' || s[i] == '[')) {
      skip_value();
      return false;
    }
    size_t b = i;
    while (i < s.size() && s[i] != ',' && s[i] != '}' && !std::isspace((unsigned char)s[i])) ++i;
    std::string tok = s.substr(b, i - b);
    if (tok == "true") *out = "1";
    else if (tok == "false") *out = "0";
    else if (tok == "null") return false;
    else *out = tok;
    return true;
  }
  std::unordered_map<std::string, std::string> parse() {
    std::unordered_map<std::string, std::string> cfg;
    ws();
    CHECK(i < s.size() && s[i] == '{') << "config must be a JSON object";
    ++i;
    while (true) {
      ws();
      if (i < s.size() && s[i] == '}') break;
      std::string k, v;
      CHECK(str(&k)) << "bad config key near offset " << i;
      ws();
      CHECK(i < s.size() && s[i] == ':') << "bad config near offset " << i;
      ++i;
      if (value(&v)) cfg[k] = v;
      ws();
      if (i < s.size() && s[i] == ',') {
        ++i;
        continue;
      }
      break;
    }
    return cfg;
  }
};

}  // namespace

void ReadLocalConfigToEnv(std::string config_name) {
  if (config_name.size() > 5 && config_name.substr(config_name.size() - 5) != ".json") config_name += ".json";
  std::ifstream in(config_name);
  if (!in.good()) return;  // like the reference: a missing file leaves the Environment as is
  std::stringstream ss;
  ss << in.rdbuf();
  std::string content = ss.str();
  if (content.empty()) return;
  Environment::Init(FlatJson(content).parse());
}

}  // namespace ps

// ---- stage timing (internal/stage_time.h) -------------------------------------
#include "internal/stage_time.h"
#include "internal/PostOffice.h"

namespace ps {
namespace stage {
bool On() {
  static const bool on = [] {
    const char* e = std::getenv("PS_STAGE_TIMES");
    return e && std::atoi(e) != 0;
  }();
  return on;
}
void Print(const char* name, double ms, size_t bytes) {
  PostOffice* po = PostOffice::GetIfBound();
  std::fprintf(stderr, "[stage] node=%d %s %.3f ms %.1f MB\n", po ? po->my_id() : -1, name, ms, bytes / 1e6);
}
}  // namespace stage
}  // namespace ps
