// internal/Env.h — configuration: the JSON config file first, then getenv
// (reference src/internal/Env.h:23-96, Env.cpp:28-83).  Same class, same
// methods, same fallbacks; the include path is the one harnesses use
// (tests/src/LRServer.h:6).
#pragma once
#include <cstdlib>
#include <mutex>
#include <string>
#include <unordered_map>

#include "ps/log.h"

namespace ps {

class Environment {
 public:
  static void Init(const std::unordered_map<std::string, std::string>& cfg) {
    Environment* env = GetEnvironment();
    std::lock_guard<std::mutex> lk(env->mu_);
    for (auto& kv : cfg) env->cfg_[kv.first] = kv.second;
  }
  static const char* Get(const char* key) {
    Environment* env = GetEnvironment();
    std::lock_guard<std::mutex> lk(env->mu_);
    auto it = env->cfg_.find(key);
    if (it == env->cfg_.end()) return std::getenv(key);
    return it->second.c_str();
  }
  static const char* GetOrDefault(const char* key, const char* default_val) {
    const char* r = Get(key);
    return r ? r : default_val;
  }
  static const char* GetOrFail(const char* key) {
    const char* r = Get(key);
    CHECK(r != nullptr) << "Set valid config: " << key << " first!";
    return r;
  }
  static int GetInt(const char* key) { return GetIntOrDefault(key, 0); }
  static int GetIntOrDefault(const char* key, int default_val) {
    const char* r = Get(key);
    return r ? std::atoi(r) : default_val;
  }
  static int GetIntOrFail(const char* key) {
    const char* r = Get(key);
    CHECK(r != nullptr) << "Set valid config: " << key << " first!";
    return r ? std::atoi(r) : 0;
  }

 private:
  Environment() = default;
  static Environment* GetEnvironment() {
    static Environment env;
    return &env;
  }
  std::mutex mu_;
  std::unordered_map<std::string, std::string> cfg_;  // node-table entries are never erased
};

/* Load a flat JSON config ("x" or "x.json") into the Environment
 * (Env.cpp:28-83).  Values may be strings, integers, floats or booleans. */
void ReadLocalConfigToEnv(std::string config_filename);

}  // namespace ps
