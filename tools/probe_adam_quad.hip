// probe_adam_quad.hip — the LR Adam apply (psg_lr.hip, k_lr_apply_sum<ADAM>)
// with 16-B loads on every stream.  Standalone (hipcc, no library), real
// (non-zero) data, 64 M features, NG = 4 gradient frames, fraction of 8 TB/s
// at 56 B/feature.  Variants:
//   pair   the library's lane map: lane l owns features 2l, 2l+1 of each
//          128-feature half (f32 loads 8 B a lane, 512 B a wave), the moments
//          blocked per 128 features (128 m then 128 v);
//   quad   lane l owns features 4l..4l+3 of a 256-feature wave tile (f32
//          loads 16 B a lane, 1 KiB a wave), the moments permuted per 256
//          features into four 1 KiB runs — m of features (4l, 4l+1) at lane
//          offset 16 l, then m (4l+2, 4l+3), then the same two for v — so every
//          load and store of the wave is one contiguous 1 KiB run;
//   *_t2   two wave tiles per iteration.
// Plus, in the same process, a 16-B copy of the same total bytes (28 B read and
// 28 B written per feature, two 1.9 GB buffers at 64 M), at several shapes:
// what a plain stream of the apply's byte volume reaches on this box.
// Build: make -C tools  (tools/_bin/probe_adam_quad)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <functional>
#include <vector>

#define CK(x)                                                \
  do {                                                       \
    hipError_t e = (x);                                      \
    if (e != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                               \
    }                                                        \
  } while (0)

typedef float f32x2 __attribute__((ext_vector_type(2)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

constexpr int NG = 4;

struct P {
  float* w;
  const float* g[NG];
  double* m;
  uint64_t n;
  float lr;
  double alr, b1, b2, eps, c1, c2;
};

__device__ __forceinline__ void adam1(double& m, double& v, float& w, float s, const P& p) {
  const double gr = (double)(p.lr * s);
  const double mi = p.b1 * m + (1.0 - p.b1) * gr;
  const double vi = p.b2 * v + (1.0 - p.b2) * gr * gr;
  m = mi;
  v = vi;
  w = (float)((double)w - p.alr * (mi / p.c1) / (sqrt(vi / p.c2) + p.eps));
}

__device__ __forceinline__ uint64_t blk_m(uint64_t i) { return (i >> 7) * 256 + (i & 127); }
__device__ __forceinline__ uint64_t blk_v(uint64_t i) { return (i >> 7) * 256 + 128 + (i & 127); }

template <int T>
__global__ __launch_bounds__(256) void k_pair(P p) {
  const uint64_t nu = p.n / 256 * 64, stride = (uint64_t)gridDim.x * 256;
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
          x[t][k][h] = __builtin_bit_cast(f32x2, __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p.g[k] + f0[t] + 128 * h)));
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        wv[t][h] = __builtin_bit_cast(f32x2, __builtin_nontemporal_load(reinterpret_cast<const u32x2*>(p.w + f0[t] + 128 * h)));
        mm[t][h] = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p.m + blk_m(f0[t] + 128 * h)));
        vv[t][h] = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p.m + blk_v(f0[t] + 128 * h)));
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
          double a = mm[t][h][e], b = vv[t][h][e];
          float c = wv[t][h][e];
          adam1(a, b, c, s[e], p);
          mm[t][h][e] = a;
          vv[t][h][e] = b;
          wv[t][h][e] = c;
        }
        if (ok[t]) {
          __builtin_nontemporal_store(mm[t][h], reinterpret_cast<f64x2*>(p.m + blk_m(f0[t] + 128 * h)));
          __builtin_nontemporal_store(vv[t][h], reinterpret_cast<f64x2*>(p.m + blk_v(f0[t] + 128 * h)));
          __builtin_nontemporal_store(__builtin_bit_cast(u32x2, wv[t][h]), reinterpret_cast<u32x2*>(p.w + f0[t] + 128 * h));
        }
      }
    }
  }
}

// quad: wave tile q (256 features) = lane units q*64 .. q*64+63; the moments
// of tile q live at p.m + q*512 doubles: [m(4l,4l+1)]x64 [m(4l+2,4l+3)]x64
// [v(4l,4l+1)]x64 [v(4l+2,4l+3)]x64
template <int T>
__global__ __launch_bounds__(256) void k_quad(P p) {
  const uint64_t nu = p.n / 256 * 64, stride = (uint64_t)gridDim.x * 256;
  for (uint64_t j0 = (uint64_t)blockIdx.x * 256 * T + threadIdx.x; j0 < nu; j0 += stride * T) {
    f32x4 x[T][NG], wv[T];
    f64x2 mo[T][4];
    bool ok[T];
    uint64_t mb[T], j1[T];
#pragma unroll
    for (int t = 0; t < T; ++t) {
      const uint64_t j = j0 + (uint64_t)t * 256;
      ok[t] = j < nu;
      j1[t] = ok[t] ? j : j0;
      mb[t] = (j1[t] >> 6) * 512 + 2 * (j1[t] & 63);
#pragma unroll
      for (int k = 0; k < NG; ++k)
        x[t][k] = __builtin_bit_cast(f32x4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p.g[k]) + j1[t]));
      wv[t] = __builtin_bit_cast(f32x4, __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(p.w) + j1[t]));
#pragma unroll
      for (int r = 0; r < 4; ++r) mo[t][r] = __builtin_nontemporal_load(reinterpret_cast<const f64x2*>(p.m + mb[t] + 128 * r));
    }
#pragma unroll
    for (int t = 0; t < T; ++t) {
      f32x4 s = f32x4{0.0f, 0.0f, 0.0f, 0.0f} + x[t][0];
#pragma unroll
      for (int k = 1; k < NG; ++k) s = s + x[t][k];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        double a = mo[t][e >> 1][e & 1], b = mo[t][2 + (e >> 1)][e & 1];
        float c = wv[t][e];
        adam1(a, b, c, s[e], p);
        mo[t][e >> 1][e & 1] = a;
        mo[t][2 + (e >> 1)][e & 1] = b;
        wv[t][e] = c;
      }
      if (ok[t]) {
#pragma unroll
        for (int r = 0; r < 4; ++r) __builtin_nontemporal_store(mo[t][r], reinterpret_cast<f64x2*>(p.m + mb[t] + 128 * r));
        __builtin_nontemporal_store(__builtin_bit_cast(u32x4, wv[t]), reinterpret_cast<u32x4*>(p.w) + j1[t]);
      }
    }
  }
}

template <int U>
__global__ __launch_bounds__(256) void k_copy(const u32x4* __restrict__ a, u32x4* __restrict__ c, uint64_t nv) {
  for (uint64_t b = (uint64_t)blockIdx.x * 256 * U + threadIdx.x; b < nv; b += (uint64_t)gridDim.x * 256 * U) {
    u32x4 x[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * 256 < nv ? b + (uint64_t)u * 256 : b;
      x[u] = __builtin_nontemporal_load(a + i);
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + (uint64_t)u * 256 < nv) __builtin_nontemporal_store(x[u], c + b + (uint64_t)u * 256);
  }
}

__global__ void k_fill(float* __restrict__ a, uint64_t n, uint32_t seed, float scale) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u + seed * 40503u;
    x ^= x >> 15;
    a[i] = scale * (float)((int)(x % 1001u) - 500);
  }
}
__global__ void k_fill_d(double* __restrict__ a, uint64_t n, uint32_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u + seed * 40503u;
    x ^= x >> 15;
    a[i] = 1e-6 * (double)(x % 1000u + 1);
  }
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : (64ull << 20);
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  if (n % 256) {
    fprintf(stderr, "n must be a multiple of 256\n");
    return 2;
  }
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  P p{};
  CK(hipMalloc(&p.w, n * 4));
  k_fill<<<1024, 256>>>(p.w, n, 3u, 1e-3f);
  for (int k = 0; k < NG; ++k) {
    float* g;
    CK(hipMalloc(&g, n * 4));
    k_fill<<<1024, 256>>>(g, n, 11u + k, 1.0f / 64);
    p.g[k] = g;
  }
  CK(hipMalloc(&p.m, n * 16));
  k_fill_d<<<1024, 256>>>(p.m, n * 2, 5u);
  const uint64_t cbytes = n * 28;  // copy of 28 B/feature read + 28 written = 56 B
  u32x4 *ca, *cb;
  CK(hipMalloc(&ca, cbytes));
  CK(hipMalloc(&cb, cbytes));
  k_fill<<<1024, 256>>>((float*)ca, cbytes / 4, 9u, 1.0f);
  k_fill<<<1024, 256>>>((float*)cb, cbytes / 4, 13u, 1.0f);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  p.n = n;
  p.lr = 0.01f;
  p.alr = 0.01;
  p.b1 = 0.9;
  p.b2 = 0.999;
  p.eps = 1e-8;
  p.c1 = 1 - std::pow(0.9, 10);
  p.c2 = 1 - std::pow(0.999, 10);
  struct V {
    const char* name;
    int per_cu;
    std::function<void(int)> f;
  };
  std::vector<V> vs = {
      {"pair T1 8/CU", 8, [&](int g) { k_pair<1><<<g, 256>>>(p); }},
      {"pair T2 8/CU", 8, [&](int g) { k_pair<2><<<g, 256>>>(p); }},
      {"pair T1 4/CU", 4, [&](int g) { k_pair<1><<<g, 256>>>(p); }},
      {"pair T2 4/CU", 4, [&](int g) { k_pair<2><<<g, 256>>>(p); }},
      {"pair T2 2/CU", 2, [&](int g) { k_pair<2><<<g, 256>>>(p); }},
      {"pair T2 1/CU", 1, [&](int g) { k_pair<2><<<g, 256>>>(p); }},
      {"pair T1 2/CU", 2, [&](int g) { k_pair<1><<<g, 256>>>(p); }},
      {"pair T4 2/CU", 2, [&](int g) { k_pair<4><<<g, 256>>>(p); }},
      {"pair T4 1/CU", 1, [&](int g) { k_pair<4><<<g, 256>>>(p); }},
      {"quad T1 8/CU", 8, [&](int g) { k_quad<1><<<g, 256>>>(p); }},
      {"quad T2 8/CU", 8, [&](int g) { k_quad<2><<<g, 256>>>(p); }},
      {"quad T2 4/CU", 4, [&](int g) { k_quad<2><<<g, 256>>>(p); }},
      {"copy U2 8/CU", 8, [&](int g) { k_copy<2><<<g, 256>>>(ca, cb, cbytes / 16); }},
      {"copy U1 4/CU", 4, [&](int g) { k_copy<1><<<g, 256>>>(ca, cb, cbytes / 16); }},
      {"copy U4 2/CU", 2, [&](int g) { k_copy<4><<<g, 256>>>(ca, cb, cbytes / 16); }},
      {"copy U8 2/CU", 2, [&](int g) { k_copy<8><<<g, 256>>>(ca, cb, cbytes / 16); }},
  };
  std::vector<std::vector<double>> res(vs.size());
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < rounds; ++r)
    for (size_t k = 0; k < vs.size(); ++k) {
      const int g = cus * vs[k].per_cu;
      for (int i = 0; i < 2; ++i) vs[k].f(g);
      std::vector<float> t;
      for (int i = 0; i < 15; ++i) {
        CK(hipEventRecord(a, 0));
        vs[k].f(g);
        CK(hipEventRecord(b, 0));
        CK(hipEventSynchronize(b));
        float ms;
        CK(hipEventElapsedTime(&ms, a, b));
        t.push_back(ms);
      }
      std::sort(t.begin(), t.end());
      res[k].push_back(t[t.size() / 2]);
    }
  printf("Adam apply, %llu features, %d frames, %d interleaved rounds; fraction of 8 TB/s at 56 B/feature\n",
         (unsigned long long)n, NG, rounds);
  for (size_t k = 0; k < vs.size(); ++k) {
    printf("%-20s", vs[k].name);
    for (double ms : res[k]) printf("  %.4f ms (%.3f)", ms, 56.0 * n / (ms * 1e-3) / 8e12);
    printf("\n");
  }
  return 0;
}
