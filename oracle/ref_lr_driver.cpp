// ref_lr_driver.cpp — runs the REFERENCE's own Adam (tests/src/Adam.h of
// SovietPower/Parameter-Server, #included where it lies under
// /root/reference; see oracle/Makefile) inside a replay of LRServer's BSP apply
// loop (tests/src/LRServer.h:171-177):
//     double grad = learning_rate_ * merge_buf_.vals[i];      // float * float, widened
//     if (adam_) grad = adam_->GetGrad(grad, i, current_iteration_);
//     weight_[i] -= grad;                                       // float -= double
// so the LR parity of this repo (psg_lr_apply_sum, oracle.lr_apply) is pinned by
// the reference's code, not only by restatements.  Test infrastructure only
// (tests/golden/make_lr_golden.py runs it to write the committed fixture).
//
// in:  int32 n, int32 rounds, int32 use_adam, float learning_rate,
//      float weight[n], then per round: int32 iteration, float merged[n]
// out: per round: float weight[n] after the round's apply
#include <cstdint>
#include <cstdio>
#include <vector>

#include "Adam.h"  // the reference's lr::Adam (tests/src/Adam.h)

int main(int argc, char** argv) {
  if (argc != 3) {
    std::fprintf(stderr, "usage: ref_lr_driver IN OUT\n");
    return 2;
  }
  FILE* in = std::fopen(argv[1], "rb");
  FILE* out = std::fopen(argv[2], "wb");
  if (!in || !out) return 3;
  int32_t n = 0, rounds = 0, use_adam = 0;
  float learning_rate = 0;
  if (std::fread(&n, 4, 1, in) != 1 || std::fread(&rounds, 4, 1, in) != 1 || std::fread(&use_adam, 4, 1, in) != 1 ||
      std::fread(&learning_rate, 4, 1, in) != 1)
    return 4;
  std::vector<float> weight(n), merged(n);
  if (std::fread(weight.data(), 4, n, in) != (size_t)n) return 5;
  // LRServer constructs Adam with its float learning rate (LRServer.h:83-84)
  lr::Adam* adam = use_adam ? new lr::Adam(n, learning_rate) : nullptr;
  for (int r = 0; r < rounds; ++r) {
    int32_t iteration = 0;
    if (std::fread(&iteration, 4, 1, in) != 1 || std::fread(merged.data(), 4, n, in) != (size_t)n) return 6;
    for (int32_t i = 0; i < n; ++i) {
      double grad = learning_rate * merged[i];
      if (adam) grad = adam->GetGrad(grad, i, iteration);
      weight[i] -= grad;
    }
    std::fwrite(weight.data(), 4, n, out);
  }
  delete adam;
  std::fclose(in);
  std::fclose(out);
  return 0;
}
