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
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "psg_internal.h"


namespace psg {

// One pass per BSP round: merge the round's gradients and apply the update.
//   s = ZERO ? ((0 + g_0[i]) + g_1[i]) + ... : (g_0[i] + g_1[i]) + ...   (f32 adds,
//       the arrival order of merge_buf_.vals[i] += req_data.vals[i], LRServer.h:158-160;
//       ZERO = the sync merge buffer that starts at 0, else async's raw push)
//   grad = (double)(lr * s); Adam (LRServer.h:171-174); w = (float)((double)w - grad)
// SGD: four features per lane as 16-B vectors; Adam: two pairs per lane (see
// below); every gradient's loads are issued before the adds.  Bytes per
// feature: 4 * ng + 8 (+ 32 with Adam) — HBM-bound.
// the model's own arrays (w, m, v): non-temporal once they are well past the
// Infinity Cache (nt), default policy while a round's state can stay in it
template <typename V>
__device__ __forceinline__ V ld_nt(const V* p, int nt) {
  return nt ? __builtin_nontemporal_load(p) : *p;
}
template <typename V>
__device__ __forceinline__ void st_nt(V* p, V x, int nt) {
  if (nt) __builtin_nontemporal_store(x, p);
  else *p = x;
}

// Adam moments, three layouts (psg_adam.layout):
//   0      two arrays of n doubles, m and v;
//   1 BLK  one array holding, per 128 features, their 128 m values then their
//          128 v values (2 KiB), so a wave's m and v runs for the same features
//          are neighbours in memory — one stream of moment pairs instead of two;
//   2 QUAD one array holding, per 256 features (one wave tile of the QUAD lane
//          map: lane l owns features 4l..4l+3), four 1 KiB runs — the m of
//          features (4l, 4l+1) at lane offset 16 l, then the m of (4l+2, 4l+3),
//          then the same two for v — so every moment load and store of a wave is
//          one contiguous 1 KiB run with 16 B a lane, as are its f32 loads.
// Element accessors for feature i:
__device__ __forceinline__ uint64_t blk_m(uint64_t i) { return (i >> 7) * 256 + (i & 127); }
__device__ __forceinline__ uint64_t blk_v(uint64_t i) { return (i >> 7) * 256 + 128 + (i & 127); }
__device__ __forceinline__ uint64_t quad_m(uint64_t i) {
  return (i >> 8) * 512 + 128 * ((i >> 1) & 1) + 2 * ((i & 255) >> 2) + (i & 1);
}
__device__ __forceinline__ uint64_t quad_v(uint64_t i) { return quad_m(i) + 256; }
template <int LAY>
__device__ __forceinline__ double* mom_m(double* m, uint64_t i) {
  return LAY == 2 ? m + quad_m(i) : LAY == 1 ? m + blk_m(i) : m + i;
}
template <int LAY>
__device__ __forceinline__ double* mom_v(double* m, double* v, uint64_t i) {
  return LAY == 2 ? m + quad_v(i) : LAY == 1 ? m + blk_v(i) : v + i;
}

// MAXG: gradient slots the kernel keeps registers for; EXACT: a round of
// exactly MAXG frames (1..4: every slot loaded, no run-time frame test, so the
// registers of absent frames are not held), else up to kMaxGrads (ng at run
// time).  LAY: the moment layout (1, 2: m is the one array, v unused).
// COPY (measurement only, psg_lr_mix_copy): the same loads and stores with a
// copy's arithmetic (m += g, v -= g, w += g): this kernel's byte mix at the
// rate the box moves it, the ceiling the Adam apply is compared with.
template <bool ADAM, bool ZERO, int MAXG, int LAY, bool EXACT, bool COPY = false>
__global__ __launch_bounds__(256) void k_lr_apply_sum(float* __restrict__ w, Grads g, int ng, uint64_t n,
                                                      float lr, double* __restrict__ m,
                                                      double* __restrict__ v, double alr, double b1,
                                                      double b2, double eps, double c1, double c2,
                                                      int vec, int nt) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  uint64_t done = 0;  // features the vector loop covers
  if constexpr (!ADAM) {
    const uint64_t nv = vec ? n / 4 : 0;
    done = nv * 4;
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < nv; j += stride) {
      f32x4 x[MAXG];
#pragma unroll
      for (int k = 0; k < MAXG; ++k)
        if (EXACT || k < ng)
          x[k] = __builtin_bit_cast(f32x4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g.p[k]) + j));
      f32x4 s = ZERO ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} + x[0] : x[0];
#pragma unroll
      for (int k = 1; k < MAXG; ++k)
        if (EXACT || k < ng) s = s + x[k];
      f32x4 wv = __builtin_bit_cast(f32x4, ld_nt(reinterpret_cast<const u32x4*>(w + 4 * j), nt));
#pragma unroll
      for (int e = 0; e < 4; ++e) wv[e] = (float)((double)wv[e] - (double)(lr * s[e]));
      st_nt(reinterpret_cast<u32x4*>(w + 4 * j), __builtin_bit_cast(u32x4, wv), nt);
    }
  } else if constexpr (LAY == 2) {
    // Adam, QUAD: lane unit j owns features 4j..4j+3 (16-B f32 loads, one
    // 1 KiB run a wave instruction on every stream); T wave tiles per
    // iteration as below
    constexpr int T = EXACT ? 2 : 1;
    const uint64_t nu = vec ? n / 256 * 64 : 0;
    done = nu * 4;
    for (uint64_t j0 = (uint64_t)blockIdx.x * kBlock * T + threadIdx.x; j0 < nu; j0 += stride * T) {
      f32x4 x[T][MAXG], wv[T];
      f64x2 mo[T][4];  // m(4l, 4l+1), m(4l+2, 4l+3), v(4l, 4l+1), v(4l+2, 4l+3)
      uint64_t jq[T], mb[T];
      bool in[T];
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const uint64_t j = j0 + (uint64_t)t * kBlock;
        in[t] = j < nu;
        jq[t] = in[t] ? j : j0;  // a tile past the end repeats the first, unwritten
        mb[t] = (jq[t] >> 6) * 512 + 2 * (jq[t] & 63);
#pragma unroll
        for (int k = 0; k < MAXG; ++k)
          if (EXACT || k < ng)
            x[t][k] = __builtin_bit_cast(f32x4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(g.p[k]) + jq[t]));
        wv[t] = __builtin_bit_cast(f32x4, ld_nt(reinterpret_cast<const u32x4*>(w) + jq[t], nt));
#pragma unroll
        for (int r = 0; r < 4; ++r) mo[t][r] = ld_nt(reinterpret_cast<const f64x2*>(m + mb[t] + 128 * r), nt);
      }
#pragma unroll
      for (int t = 0; t < T; ++t) {
        f32x4 s = ZERO ? f32x4{0.0f, 0.0f, 0.0f, 0.0f} + x[t][0] : x[t][0];
#pragma unroll
        for (int k = 1; k < MAXG; ++k)
          if (EXACT || k < ng) s = s + x[t][k];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          if constexpr (COPY) {
            mo[t][e >> 1][e & 1] += (double)s[e];
            mo[t][2 + (e >> 1)][e & 1] -= (double)s[e];
            wv[t][e] += s[e];
            continue;
          }
          const double gr = (double)(lr * s[e]);
          const double mi = b1 * mo[t][e >> 1][e & 1] + (1.0 - b1) * gr;
          const double vi = b2 * mo[t][2 + (e >> 1)][e & 1] + (1.0 - b2) * gr * gr;
          mo[t][e >> 1][e & 1] = mi;
          mo[t][2 + (e >> 1)][e & 1] = vi;
          wv[t][e] = (float)((double)wv[t][e] - alr * (mi / c1) / (sqrt(vi / c2) + eps));
        }
        if (in[t]) {
#pragma unroll
          for (int r = 0; r < 4; ++r) st_nt(reinterpret_cast<f64x2*>(m + mb[t] + 128 * r), mo[t][r], nt);
          st_nt(reinterpret_cast<u32x4*>(w) + jq[t], __builtin_bit_cast(u32x4, wv[t]), nt);
        }
      }
    }
  } else {
    // Adam: 256 features per wave, lane l owning features 2l, 2l+1 of each
    // 128-feature half, so every load and store instruction of a wave is one
    // contiguous run (512 B of f32 pairs, 1 KiB of f64 pairs).  With four
    // consecutive features per lane the f64 moments moved at a 32-B lane
    // stride, each instruction writing half of every line (0.63 of HBM at 64 M
    // features).  T wave tiles per iteration, every load of the T tiles issued
    // before the first update: T = 2 for an exact frame count (the in-place
    // moment read-modify-write is the slow stream, and two tiles keep twice
    // its lines in flight: tools/probe_adam.hip), 1 for a run-time count (its
    // registers would halve the waves).
    constexpr int T = EXACT ? 2 : 1;
    typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
    typedef float f32x2 __attribute__((ext_vector_type(2)));
    const uint64_t nu = vec ? n / 256 * 64 : 0;  // lane units of whole wave tiles
    done = nu * 4;
    for (uint64_t j0 = (uint64_t)blockIdx.x * kBlock * T + threadIdx.x; j0 < nu; j0 += stride * T) {
      f32x2 x[T][MAXG][2];
      f32x2 wv[T][2];
      f64x2 mm[T][2], vv[T][2];
      uint64_t f0[T];
      bool in[T];
#pragma unroll
      for (int t = 0; t < T; ++t) {
        const uint64_t j = j0 + (uint64_t)t * kBlock;
        in[t] = j < nu;
        const uint64_t jj = in[t] ? j : j0;  // a tile past the end repeats the first, unwritten
        f0[t] = (jj >> 6) * 256 + 2 * (jj & 63);  // first pair; the second is f0 + 128
#pragma unroll
        for (int k = 0; k < MAXG; ++k)
          if (EXACT || k < ng)
#pragma unroll
            for (int h = 0; h < 2; ++h)
              x[t][k][h] = __builtin_bit_cast(
                  f32x2, __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(g.p[k] + f0[t] + 128 * h)));
        // the moment pairs of features f0 + 128 h (layout 1: group 2U + h of
        // the blocked array, U = f0 / 256, at lane offset f0 % 128)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          wv[t][h] = __builtin_bit_cast(f32x2, ld_nt(reinterpret_cast<const u32x2*>(w + f0[t] + 128 * h), nt));
          mm[t][h] = ld_nt(reinterpret_cast<const f64x2*>(mom_m<LAY>(m, f0[t] + 128 * h)), nt);
          vv[t][h] = ld_nt(reinterpret_cast<const f64x2*>(mom_v<LAY>(m, v, f0[t] + 128 * h)), nt);
        }
      }
#pragma unroll
      for (int t = 0; t < T; ++t) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          f32x2 s = ZERO ? f32x2{0.0f, 0.0f} + x[t][0][h] : x[t][0][h];
#pragma unroll
          for (int k = 1; k < MAXG; ++k)
            if (EXACT || k < ng) s = s + x[t][k][h];
#pragma unroll
          for (int e = 0; e < 2; ++e) {
            if constexpr (COPY) {
              mm[t][h][e] += (double)s[e];
              vv[t][h][e] -= (double)s[e];
              wv[t][h][e] += s[e];
              continue;
            }
            const double gr = (double)(lr * s[e]);
            const double mi = b1 * mm[t][h][e] + (1.0 - b1) * gr;
            const double vi = b2 * vv[t][h][e] + (1.0 - b2) * gr * gr;
            mm[t][h][e] = mi;
            vv[t][h][e] = vi;
            wv[t][h][e] = (float)((double)wv[t][h][e] - alr * (mi / c1) / (sqrt(vi / c2) + eps));
          }
          if (in[t]) {
            st_nt(reinterpret_cast<f64x2*>(mom_m<LAY>(m, f0[t] + 128 * h)), mm[t][h], nt);
            st_nt(reinterpret_cast<f64x2*>(mom_v<LAY>(m, v, f0[t] + 128 * h)), vv[t][h], nt);
            st_nt(reinterpret_cast<u32x2*>(w + f0[t] + 128 * h), __builtin_bit_cast(u32x2, wv[t][h]), nt);
          }
        }
      }
    }
  }
  for (uint64_t i = done + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    float s = ZERO ? 0.0f + g.p[0][i] : g.p[0][i];
    for (int k = 1; k < ng; ++k) s = s + g.p[k][i];
    double grad = (double)(lr * s);
    if constexpr (ADAM && COPY) {
      *mom_m<LAY>(m, i) += (double)s;
      *mom_v<LAY>(m, v, i) -= (double)s;
      w[i] += s;
      continue;
    } else if constexpr (ADAM) {
      double* mi_p = mom_m<LAY>(m, i);
      double* vi_p = mom_v<LAY>(m, v, i);
      const double mi = b1 * *mi_p + (1.0 - b1) * grad;
      const double vi = b2 * *vi_p + (1.0 - b2) * grad * grad;
      *mi_p = mi;
      *vi_p = vi;
      grad = alr * (mi / c1) / (sqrt(vi / c2) + eps);
    }
    w[i] = (float)((double)w[i] - grad);
  }
}

int lr_apply_sum(psg_store* weights, uint64_t w_off, const float* const* grads, int ngrads,
                 int from_zero, uint64_t n, float lr, psg_adam* adam, uint64_t adam_off,
                 int iteration, hipStream_t st, bool copy_mix) {
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
    PSG_REQUIRE(adam->layout == 0 || adam_off == 0, PSG_ERR_INVALID, "LR apply: interleaved Adam state at an offset");
    m = adam->m + (adam->layout ? 0 : adam_off);
    v = adam->layout ? nullptr : adam->v + adam_off;
    vec = vec && aligned16(m) && (adam->layout || aligned16(v));
    // the two bias corrections of Adam.h:31-32, with the host libm pow the
    // reference calls
    c1 = 1 - std::pow(adam->beta1, iteration + 1);
    c2 = 1 - std::pow(adam->beta2, iteration + 1);
  }
  const uint64_t units = vec ? (n + 3) / 4 : n;
  uint64_t b = (units + kBlock - 1) / kBlock;
  // 2 blocks of 256 per CU, grid-striding: at 64 M features SGD 0.87 / 0.81
  // (1 / 4 frames) and Adam 0.66 / 0.66 of 8 TB/s, against 0.77-0.83 / 0.69-0.76
  // and 0.64 / 0.65 with 8 per CU; 1 per CU starves SGD of loads in flight
  // (0.57), 3 and 4 sit between; no difference at 10 M features (two
  // interleaved rounds each, profiles/r4_ab_lr_bpc.txt).  PSG_LR_BPC=k: k per CU.
  static const int bpc = [] {
    const char* e = getenv("PSG_LR_BPC");
    const int k = e ? atoi(e) : 0;
    return k >= 1 && k <= 16 ? k : 2;
  }();
  const uint64_t cap = (uint64_t)max_stream_blocks() / 8 * bpc;
  const unsigned grid = (unsigned)(b < cap ? (b ? b : 1) : cap);
  const int ve = vec ? 1 : 0;
  // PSG_LR_NT=0/1 forces the policy (sweeps); default: non-temporal when the
  // model's arrays exceed 512 MiB
  static const int nt_env = [] {
    const char* e = getenv("PSG_LR_NT");
    return e ? atoi(e) : -1;
  }();
  const uint64_t state_bytes = n * (adam ? 20ull : 4ull);
  const int ntm = nt_env >= 0 ? (nt_env ? 1 : 0) : (state_bytes > (512ull << 20) ? 1 : 0);
  const double alr = adam ? adam->lr : 0, b1 = adam ? adam->beta1 : 0, b2 = adam ? adam->beta2 : 0,
               eps = adam ? adam->eps : 0;
  const int lay = adam ? adam->layout : 0;
  auto go = [&](auto adam_c, auto zero_c, auto lay_c) {
    constexpr bool A = decltype(adam_c)::value, Z = decltype(zero_c)::value;
    constexpr int B = decltype(lay_c)::value;
#define PSG_LR_LAUNCH(G, X)                                                                                    \
  do {                                                                                                         \
    if constexpr (A && Z) {                                                                                    \
      if (copy_mix) {                                                                                          \
        k_lr_apply_sum<A, Z, G, B, X, true>                                                                    \
            <<<grid, kBlock, 0, st>>>(w, g, ngrads, n, lr, m, v, alr, b1, b2, eps, c1, c2, ve, ntm);           \
        break;                                                                                                 \
      }                                                                                                        \
    }                                                                                                          \
    k_lr_apply_sum<A, Z, G, B, X><<<grid, kBlock, 0, st>>>(w, g, ngrads, n, lr, m, v, alr, b1, b2, eps, c1, c2, \
                                                           ve, ntm);                                           \
  } while (0)
    switch (ngrads) {
      case 1: PSG_LR_LAUNCH(1, true); break;
      case 2: PSG_LR_LAUNCH(2, true); break;
      case 3: PSG_LR_LAUNCH(3, true); break;
      case 4: PSG_LR_LAUNCH(4, true); break;
      default: PSG_LR_LAUNCH(kMaxGrads, false); break;
    }
#undef PSG_LR_LAUNCH
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using L0 = std::integral_constant<int, 0>;
  using L1 = std::integral_constant<int, 1>;
  using L2 = std::integral_constant<int, 2>;
  auto go_adam = [&](auto zero_c) {
    if (lay == 2) go(T_{}, zero_c, L2{});
    else if (lay == 1) go(T_{}, zero_c, L1{});
    else go(T_{}, zero_c, L0{});
  };
  if (adam && from_zero) go_adam(T_{});
  else if (adam) go_adam(F_{});
  else if (from_zero) go(F_{}, T_{}, L0{});
  else go(F_{}, F_{}, L0{});
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
  // PSG_ADAM_LAYOUT=0/1/2 (A/B; PSG_ADAM_BLOCKED=0 is layout 0): the moment
  // layout of k_lr_apply_sum, read at every create (tests switch it); default 1
  const int layout = [] {
    const char* e = getenv("PSG_ADAM_LAYOUT");
    if (e) return atoi(e) == 2 ? 2 : atoi(e) == 0 ? 0 : 1;
    const char* b = getenv("PSG_ADAM_BLOCKED");
    return b && atoi(b) == 0 ? 0 : 1;
  }();
  a->layout = layout;
  hipError_t e;
  if (layout) {
    const uint64_t words = layout == 2 ? (n + 255) / 256 * 512 : (n + 127) / 128 * 256;
    e = hipMalloc((void**)&a->m, words * sizeof(double));
    if (e == hipSuccess) e = hipMemset(a->m, 0, words * sizeof(double));
  } else {
    e = hipMalloc((void**)&a->m, n * sizeof(double));
    if (e == hipSuccess) e = hipMalloc((void**)&a->v, n * sizeof(double));
    if (e == hipSuccess) e = hipMemset(a->m, 0, n * sizeof(double));
    if (e == hipSuccess) e = hipMemset(a->v, 0, n * sizeof(double));
  }
  // null-stream memsets: done before the caller's (non-blocking) streams use
  // the moments
  if (e == hipSuccess) e = hipStreamSynchronize(nullptr);
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

int psg_lr_mix_copy(psg_store* weights, const float* const* grads_host, int ngrads, uint64_t n, psg_adam* adam,
                    psg_stream stream) {
  PSG_REQUIRE(adam, PSG_ERR_INVALID, "psg_lr_mix_copy: the Adam byte mix needs the moments");
  return lr_apply_sum(weights, 0, grads_host, ngrads, 1, n, 0.0f, adam, 0, 0, (hipStream_t)stream, true);
}

}  // extern "C"
