// internal/stage_time.h — host stage timing of the request path (diagnostics).
//
// PS_STAGE_TIMES=1: every scoped stage prints one line to stderr when it ends,
//   [stage] node=<id> <name> <ms> ms <MB> MB
// (the vector -> SVector copy of a Push, the slicer and the Van send, the
// server's frame decode, its handle and its Response, the Pull merge, ...),
// so the time of one request of a harness such as the reference's
// test_kv_app_benchmark.cpp splits into its host stages.  Off by default: one
// cached getenv test per stage.
#pragma once
#include <chrono>
#include <cstddef>

namespace ps {
namespace stage {

bool On();
void Print(const char* name, double ms, size_t bytes);

class Scope {
 public:
  explicit Scope(const char* name, size_t bytes = 0) : name_(name), bytes_(bytes), on_(On()) {
    if (on_) t0_ = std::chrono::steady_clock::now();
  }
  ~Scope() {
    if (on_) Print(name_, std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0_).count(), bytes_);
  }
  Scope(const Scope&) = delete;
  Scope& operator=(const Scope&) = delete;

 private:
  const char* name_;
  size_t bytes_;
  bool on_;
  std::chrono::steady_clock::time_point t0_;
};

}  // namespace stage
}  // namespace ps
