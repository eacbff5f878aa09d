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


namespace psg {

// One pass per BSP round: merge the round's gradients and apply the update.
//   s = ZERO ? ((0 + g_0[i]) + g_1[i]) + ... : (g_0[i] + g_1[i]) + ...   (f32 adds,
//       the arrival order of merge_buf_.vals[i] += req_data.vals[i], LRServer.h:158-160;
//       ZERO = the sync merge buffer that starts at 0, else async's raw push)
//   grad = (double)(lr * s); Adam (LRServer.h:171-174); w = (float)((double)w - grad)
// Four features per lane as 16-B vectors (f32 w / g, two f64x2 each for Adam's
// m and v); every gradient's loads are issued before the adds.  Bytes per
// feature: 4 * ng + 8 (+ 32 with Adam) — HBM-bound.
template <bool ADAM, bool ZERO>
__global__ __launch_bounds__(256) void k_lr_apply_sum(float* __restrict__ w, Grads g, int ng, uint64_t n,
                                                      float lr, double* __restrict__ m,
                                                      double* __restrict__ v, double alr, double b1,
                                                      double b2, double eps, double c1, double c2,
                                                      int vec) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t nv = vec ? n / 4 : 0;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < nv; j += stride) {
    f32x4 x[kMaxGrads];
#pragma unroll
    for (int k = 0; k < kMaxGrads; ++k)
      if (k < ng)
        x[k] = __builtin_bit_cast(f32x4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g.p[k]) + j));
    f32x4 s = ZERO ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} + x[0] : x[0];
#pragma unroll
    for (int k = 1; k < kMaxGrads; ++k)
      if (k < ng) s = s + x[k];
    f32x4 wv = __builtin_bit_cast(f32x4, *reinterpret_cast<const u32x4*>(w + 4 * j));
    double gr[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) gr[e] = (double)(lr * s[e]);
    if constexpr (ADAM) {
      f64x2* mp = reinterpret_cast<f64x2*>(m + 4 * j);
      f64x2* vp = reinterpret_cast<f64x2*>(v + 4 * j);
      f64x2 mm[2] = {mp[0], mp[1]}, vv[2] = {vp[0], vp[1]};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const double mi = b1 * mm[e >> 1][e & 1] + (1.0 - b1) * gr[e];
        const double vi = b2 * vv[e >> 1][e & 1] + (1.0 - b2) * gr[e] * gr[e];
        mm[e >> 1][e & 1] = mi;
        vv[e >> 1][e & 1] = vi;
        gr[e] = alr * (mi / c1) / (sqrt(vi / c2) + eps);
      }
      mp[0] = mm[0];
      mp[1] = mm[1];
      vp[0] = vv[0];
      vp[1] = vv[1];
    }
#pragma unroll
    for (int e = 0; e < 4; ++e) wv[e] = (float)((double)wv[e] - gr[e]);
    *reinterpret_cast<u32x4*>(w + 4 * j) = __builtin_bit_cast(u32x4, wv);
  }
  for (uint64_t i = nv * 4 + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    float s = ZERO ? 0.0f + g.p[0][i] : g.p[0][i];
    for (int k = 1; k < ng; ++k) s = s + g.p[k][i];
    double grad = (double)(lr * s);
    if constexpr (ADAM) {
      const double mi = b1 * m[i] + (1.0 - b1) * grad;
      const double vi = b2 * v[i] + (1.0 - b2) * grad * grad;
      m[i] = mi;
      v[i] = vi;
      grad = alr * (mi / c1) / (sqrt(vi / c2) + eps);
    }
    w[i] = (float)((double)w[i] - grad);
  }
}

int lr_apply_sum(psg_store* weights, uint64_t w_off, const float* const* grads, int ngrads,
                 int from_zero, uint64_t n, float lr, psg_adam* adam, uint64_t adam_off,
                 int iteration, hipStream_t st) {
  PSG_REQUIRE(weights && weights->kind == PSG_STORE_DENSE && weights->dtype == PSG_F32,
              PSG_ERR_INVALID, "LR apply: weights must be an f32 DENSE store");
  PSG_REQUIRE(w_off <= weights->capacity && n <= weights->capacity - w_off, PSG_ERR_RANGE,
              "LR apply: %llu features at slot %llu > store slots", (unsigned long long)n,
              (unsigned long long)w_off);
  PSG_REQUIRE(grads && ngrads >= 1 && ngrads <= kMaxGrads, PSG_ERR_INVALID,
              "LR apply: 1..%d gradient arrays per pass, got %d", kMaxGrads, ngrads);
  if (n == 0) return PSG_OK;
  Grads g = {};
  bool vec = true;
  float* w = (float*)weights->vals + w_off;
  for (int k = 0; k < ngrads; ++k) {
    PSG_REQUIRE(grads[k], PSG_ERR_INVALID, "LR apply: null gradient %d", k);
    g.p[k] = grads[k];
    vec = vec && aligned16(grads[k]);
  }
  vec = vec && aligned16(w);
  double *m = nullptr, *v = nullptr;
  double c1 = 1, c2 = 1;
  if (adam) {
    PSG_REQUIRE(adam_off <= adam->n && n <= adam->n - adam_off, PSG_ERR_RANGE,
                "LR apply: Adam state holds %llu features", (unsigned long long)adam->n);
    m = adam->m + adam_off;
    v = adam->v + adam_off;
    vec = vec && aligned16(m) && aligned16(v);
    // the two bias corrections of Adam.h:31-32, with the host libm pow the
    // reference calls
    c1 = 1 - std::pow(adam->beta1, iteration + 1);
    c2 = 1 - std::pow(adam->beta2, iteration + 1);
  }
  const uint64_t units = vec ? (n + 3) / 4 : n;
  uint64_t b = (units + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)max_stream_blocks();
  const unsigned grid = (unsigned)(b < cap ? (b ? b : 1) : cap);
  const int ve = vec ? 1 : 0;
  const double alr = adam ? adam->lr : 0, b1 = adam ? adam->beta1 : 0, b2 = adam ? adam->beta2 : 0,
               eps = adam ? adam->eps : 0;
  if (adam) {
    if (from_zero)
      k_lr_apply_sum<true, true><<<grid, kBlock, 0, st>>>(w, g, ngrads, n, lr, m, v, alr, b1, b2, eps, c1, c2, ve);
    else
      k_lr_apply_sum<true, false><<<grid, kBlock, 0, st>>>(w, g, ngrads, n, lr, m, v, alr, b1, b2, eps, c1, c2, ve);
  } else {
    if (from_zero)
      k_lr_apply_sum<false, true><<<grid, kBlock, 0, st>>>(w, g, ngrads, n, lr, m, v, 0, 0, 0, 0, 1, 1, ve);
    else
      k_lr_apply_sum<false, false><<<grid, kBlock, 0, st>>>(w, g, ngrads, n, lr, m, v, 0, 0, 0, 0, 1, 1, ve);
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
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
  PSG_REQUIRE(merged || n == 0, PSG_ERR_INVALID, "psg_lr_apply: null merged");
  const float* g[1] = {merged};
  // the merged buffer is applied as is: grad = (double)(lr * merged[i])
  return lr_apply_sum(weights, 0, g, 1, 0, n, lr, adam, 0, iteration, (hipStream_t)stream);
}

int psg_lr_apply_sum(psg_store* weights, const float* const* grads_host, int ngrads, int from_zero,
                     uint64_t n, float lr, psg_adam* adam, int iteration, psg_stream stream) {
  return lr_apply_sum(weights, 0, grads_host, ngrads, from_zero, n, lr, adam, 0, iteration,
                      (hipStream_t)stream);
}

}  // extern "C"
