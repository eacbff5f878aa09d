// probe_adam.hip — where the LR Adam apply (psg_lr.hip, k_lr_apply_sum<ADAM>)
// loses against the copy ceiling.  Standalone (hipcc, no library): one f32
// weight array, NG f32 gradient frames and the blocked f64 moment array
// (per 128 features their m then their v), the Adam kernel's own lane mapping
// (lane l of a wave owns features 2l, 2l+1 of each 128-feature half), and
// bodies:
//   adam    the Adam update of psg_lr.hip (IEEE divide and sqrt, f64);
//   light   the same loads and stores, the update replaced by adds;
//   *_t2    the same with two wave tiles per iteration (twice the loads in flight).
// Also the plain streams of the same bytes: rmw (the moment array read and
// written back, 16 B per lane, grid-stride) and copy (1 GB read, 1 GB written).
// Prints ms and the fraction of 8 TB/s at the algorithmic bytes.
// Build: make -C tools  (tools/_bin/probe_adam)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <algorithm>
#include <vector>

#define CK(x)                                                              \
  do {                                                                     \
    hipError_t e = (x);                                                    \
    if (e != hipSuccess) {                                                 \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));               \
      exit(1);                                                             \
    }                                                                      \
  } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ uint64_t blk_m(uint64_t i) { return (i >> 7) * 256 + (i & 127); }
__device__ __forceinline__ uint64_t blk_v(uint64_t i) { return (i >> 7) * 256 + 128 + (i & 127); }

constexpr int NG = 4;

// MODE 0 adam, 1 light; T wave tiles per iteration
template <int MODE, int T>
__global__ __launch_bounds__(256) void k_probe(float* __restrict__ w, const float* __restrict__ g0,
                                               const float* __restrict__ g1, const float* __restrict__ g2,
                                               const float* __restrict__ g3, const double* __restrict__ m,
                                               double* __restrict__ mo, uint64_t n,
                                               float lr, double alr, double b1, double b2, double eps, double c1,
                                               double c2) {
  const float* g[NG] = {g0, g1, g2, g3};
  const uint64_t nu = n / 256 * 64;
  const uint64_t stride = (uint64_t)gridDim.x * 256;
  for (uint64_t j0 = (uint64_t)blockIdx.x * 256 * T + threadIdx.x; j0 < nu; j0 += stride * T) {
    f32x2 x[T][NG][2], wv[T][2];
    f64x2 mm[T][2], vv[T][2];
    uint64_t f0[T];
    bool ok[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const uint64_t j = j0 + (uint64_t)t * 256;
      ok[t] = j < nu;
      const uint64_t jj = ok[t] ? j : j0;
      f0[t] = (jj >> 6) * 256 + 2 * (jj & 63);
#pragma unroll
      for (int k = 0; k < NG; ++k)
#pragma unroll
        for (int h = 0; h < 2; ++h)
          x[t][k][h] = __builtin_bit_cast(
              f32x2, __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(g[k] + f0[t] + 128 * h)));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        wv[t][h] = __builtin_bit_cast(f32x2, __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(w + f0[t] + 128 * h)));
        mm[t][h] = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(m + blk_m(f0[t] + 128 * h)));
        vv[t][h] = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(m + blk_v(f0[t] + 128 * h)));
      }
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        f32x2 s = f32x2{0.0f, 0.0f} + x[t][0][h];
#pragma unroll
        for (int k = 1; k < NG; ++k) s = s + x[t][k][h];
#pragma unroll
        for (int e = 0; e < 2; ++e) {
          const double gr = (double)(lr * s[e]);
          if constexpr (MODE == 0) {
            const double mi = b1 * mm[t][h][e] + (1.0 - b1) * gr;
            const double vi = b2 * vv[t][h][e] + (1.0 - b2) * gr * gr;
            mm[t][h][e] = mi;
            vv[t][h][e] = vi;
            wv[t][h][e] = (float)((double)wv[t][h][e] - alr * (mi / c1) / (sqrt(vi / c2) + eps));
          } else {
            mm[t][h][e] += gr;
            vv[t][h][e] += gr;
            wv[t][h][e] = (float)((double)wv[t][h][e] - gr);
          }
        }
        if (ok[t]) {
          __builtin_nontemporal_store(mm[t][h], reinterpret_cast<f64x2*>(mo + blk_m(f0[t] + 128 * h)));
          __builtin_nontemporal_store(vv[t][h], reinterpret_cast<f64x2*>(mo + blk_v(f0[t] + 128 * h)));
          __builtin_nontemporal_store(__builtin_bit_cast(u32x2, wv[t][h]), reinterpret_cast<u32x2*>(w + f0[t] + 128 * h));
        }
      }
    }
  }
}

template <int NT, int U>
__global__ __launch_bounds__(256) void k_rmw(u32x4* __restrict__ a, uint64_t nv) {
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < nv; b += (uint64_t)gridDim.x * 256 * U) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * 256 < nv ? b + (uint64_t)u * 256 : b;
      x[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      x[u][0] += 1;
      if (b + (uint64_t)u * 256 < nv) {
        if (NT) __builtin_nontemporal_store(x[u], a + b + (uint64_t)u * 256);
        else a[b + (uint64_t)u * 256] = x[u];
      }
    }
  }
}
template <int NT, int U>
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ c, uint64_t nv) {
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < nv; b += (uint64_t)gridDim.x * 256 * U) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * 256 < nv ? b + (uint64_t)u * 256 : b;
      x[u] = NT ? __builtin_nontemporal_load(a + i) : a[i];
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + (uint64_t)u * 256 < nv) {
        if (NT) __builtin_nontemporal_store(x[u], c + b + (uint64_t)u * 256);
        else c[b + (uint64_t)u * 256] = x[u];
      }
  }
}

template <typename F>
static double time_ms(F f, int reps = 20) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int i = 0; i < 3; ++i) f();
  std::vector<float> t;
  for (int i = 0; i < reps; ++i) {
    CK(hipEventRecord(a, 0));
    f();
    CK(hipEventRecord(b, 0));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    t.push_back(ms);
  }
  std::sort(t.begin(), t.end());
  return t[t.size() / 2];
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (64ull << 20);
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int grid = cus * 8;
  float *w, *g[NG];
  double* m;
  CK(hipMalloc(&w, n * 4));
  for (int k = 0; k < NG; ++k) {
    CK(hipMalloc(&g[k], n * 4));
    CK(hipMemset(g[k], 0, n * 4));
  }
  CK(hipMalloc(&m, (n + 127) / 128 * 256 * 8));
  CK(hipMemset(w, 0, n * 4));
  CK(hipMemset(m, 0, (n + 127) / 128 * 256 * 8));
  const double per = 4.0 * NG + 8 + 32;
  auto report = [&](const char* name, double ms, double bytes) {
    printf("{\"kernel\": \"%s\", \"n\": %llu, \"ms\": %.4f, \"frac\": %.4f}\n", name, (unsigned long long)n, ms,
           bytes / (ms * 1e-3) / 8e12);
  };
  const double c1 = 1 - std::pow(0.9, 10), c2 = 1 - std::pow(0.999, 10);
  double* m2;
  CK(hipMalloc(&m2, (n + 127) / 128 * 256 * 8));
  CK(hipMemset(m2, 0, (n + 127) / 128 * 256 * 8));
#define P(NAME, MODE, T, SRC, DST) \
  report(NAME, time_ms([&] { k_probe<MODE, T><<<grid, 256>>>(w, g[0], g[1], g[2], g[3], SRC, DST, n, 0.01f, 0.01, 0.9, 0.999, 1e-8, c1, c2); }), per * n)
  P("adam", 0, 1, m, m);
  P("light", 1, 1, m, m);
  P("adam_t2", 0, 2, m, m);
  P("light_t2", 1, 2, m, m);
  P("adam_pingpong", 0, 1, m, m2);
  P("adam_t2_pingpong", 0, 2, m, m2);
  P("light_t2_pingpong", 1, 2, m, m2);
  const uint64_t mv = (n + 127) / 128 * 256 * 8 / 16;
  u32x4* mm = reinterpret_cast<u32x4*>(m);
  u32x4* dst = reinterpret_cast<u32x4*>(m2);
  report("rmw_nt_u1", time_ms([&] { k_rmw<1, 1><<<grid, 256>>>(mm, mv); }), 32.0 * n);
  report("rmw_nt_u2", time_ms([&] { k_rmw<1, 2><<<grid, 256>>>(mm, mv); }), 32.0 * n);
  report("rmw_def_u1", time_ms([&] { k_rmw<0, 1><<<grid, 256>>>(mm, mv); }), 32.0 * n);
  report("rmw_def_u2", time_ms([&] { k_rmw<0, 2><<<grid, 256>>>(mm, mv); }), 32.0 * n);
  report("copy_nt_u1", time_ms([&] { k_copy<1, 1><<<grid, 256>>>(mm, dst, mv); }), 32.0 * n);
  report("copy_nt_u2", time_ms([&] { k_copy<1, 2><<<grid, 256>>>(mm, dst, mv); }), 32.0 * n);
  report("copy_def_u2", time_ms([&] { k_copy<0, 2><<<grid, 256>>>(mm, dst, mv); }), 32.0 * n);
  CK(hipDeviceSynchronize());
  return 0;
}
