// psg_lr.hip — LRServer's sync-mode apply as one device kernel.
//
// Reference, per feature i once all NumWorkers() pushes are merged
// (tests/src/LRServer.h:171-177, tests/src/Adam.h:28-34):
//     double grad = learning_rate_ * merge_buf_.vals[i];   // float * float, widened
//     if (adam_) grad = adam_->GetGrad(grad, i, current_iteration_);
//     weight_[i] -= grad;                                  // in double, rounded to float
//   GetGrad(g, i, it):
//     m[i] = beta1 * m[i] + (1 - beta1) * g;
//     v[i] = beta2 * v[i] + (1 - beta2) * g * g;           // ((1-beta2)*g)*g
//     m_hat = m[i] / (1 - pow(beta1, it + 1));
//     v_hat = v[i] / (1 - pow(beta2, it + 1));
//     return learning_rate * m_hat / (sqrt(v_hat) + epsilon);
// The same operation order is kept and the library is built with
// -ffp-contract=off, so no multiply-add is fused: results are bit-identical to
// the reference's x86-64 build.  The two pow() terms are evaluated once on the
// host with the same libm call the reference makes.
//
// Bytes per feature: merged f32 4 + weight f32 r/w 8 (+ m, v f64 r/w 32 with
// Adam): HBM-bound, streamed.
#include <cmath>
#include <cstring>

#include "psg_internal.h"

struct psg_adam {
  uint64_t n;
  double lr, beta1, beta2, eps;
  double* m;
  double* v;
};

namespace psg {

template <bool ADAM>
__global__ __launch_bounds__(256) void k_lr_apply(float* __restrict__ w,
                                                  const float* __restrict__ merged, uint64_t n,
                                                  float lr, double* __restrict__ m,
                                                  double* __restrict__ v, double alr, double b1,
                                                  double b2, double eps, double c1, double c2) {
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBlock) {
    double grad = (double)(lr * merged[i]);
    if constexpr (ADAM) {
      double mi = b1 * m[i] + (1.0 - b1) * grad;
      double vi = b2 * v[i] + (1.0 - b2) * grad * grad;
      m[i] = mi;
      v[i] = vi;
      double m_hat = mi / c1;
      double v_hat = vi / c2;
      grad = alr * m_hat / (sqrt(v_hat) + eps);
    }
    w[i] = (float)((double)w[i] - grad);
  }
}

}  // namespace psg

using namespace psg;

extern "C" {

int psg_adam_create(uint64_t n, double learning_rate, double beta1, double beta2, double epsilon,
                    psg_adam** out) {
  PSG_REQUIRE(out && n > 0, PSG_ERR_INVALID, "psg_adam_create: bad arguments");
  *out = nullptr;
  psg_adam* a = new psg_adam();
  memset(a, 0, sizeof(*a));
  a->n = n;
  a->lr = learning_rate;
  a->beta1 = beta1;
  a->beta2 = beta2;
  a->eps = epsilon;
  hipError_t e = hipMalloc((void**)&a->m, n * sizeof(double));
  if (e == hipSuccess) e = hipMalloc((void**)&a->v, n * sizeof(double));
  if (e == hipSuccess) e = hipMemset(a->m, 0, n * sizeof(double));
  if (e == hipSuccess) e = hipMemset(a->v, 0, n * sizeof(double));
  if (e != hipSuccess) {
    psg_adam_destroy(a);
    return hip_fail(e, "psg_adam_create", __FILE__, __LINE__);
  }
  *out = a;
  return PSG_OK;
}

int psg_adam_destroy(psg_adam* a) {
  if (!a) return PSG_OK;
  if (a->m) (void)hipFree(a->m);
  if (a->v) (void)hipFree(a->v);
  delete a;
  return PSG_OK;
}

int psg_lr_apply(psg_store* weights, const float* merged, uint64_t n, float lr, psg_adam* adam,
                 int iteration, psg_stream stream) {
  PSG_REQUIRE(weights && weights->kind == PSG_STORE_DENSE && weights->dtype == PSG_F32,
              PSG_ERR_INVALID, "psg_lr_apply: weights must be an f32 DENSE store");
  PSG_REQUIRE(n <= weights->capacity, PSG_ERR_RANGE, "psg_lr_apply: %llu features > store slots",
              (unsigned long long)n);
  if (n == 0) return PSG_OK;
  PSG_REQUIRE(merged, PSG_ERR_INVALID, "psg_lr_apply: null merged");
  uint64_t b = (n + kBlock - 1) / kBlock;
  uint64_t cap = (uint64_t)max_stream_blocks();
  unsigned g = (unsigned)(b < cap ? b : cap);
  hipStream_t st = (hipStream_t)stream;
  if (adam) {
    PSG_REQUIRE(adam->n >= n, PSG_ERR_RANGE, "psg_lr_apply: Adam state holds %llu features",
                (unsigned long long)adam->n);
    const double c1 = 1 - std::pow(adam->beta1, iteration + 1);
    const double c2 = 1 - std::pow(adam->beta2, iteration + 1);
    k_lr_apply<true><<<g, kBlock, 0, st>>>((float*)weights->vals, merged, n, lr, adam->m, adam->v,
                                           adam->lr, adam->beta1, adam->beta2, adam->eps, c1, c2);
  } else {
    k_lr_apply<false><<<g, kBlock, 0, st>>>((float*)weights->vals, merged, n, lr, nullptr, nullptr,
                                            0, 0, 0, 0, 1, 1);
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

}  // extern "C"
