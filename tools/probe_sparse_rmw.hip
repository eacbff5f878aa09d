// probe_sparse_rmw.hip — the store-value traffic of a keyed Push that asks for
// every other key of its store (k_resolve_apply's apply step at every 2nd key:
// lane l owns request keys 4l..4l+3, at store slots 8l, 8l+2, 8l+4, 8l+6 of
// its tile).  Standalone, real data, 10 M request values into a 20 M-slot f32
// store, interleaved rounds.  Variants:
//   scalar      4-B loads and 4-B stores of the 4 slots (the library today)
//   vec_load    two 16-B loads of the lane's 8 slots, 4-B stores of the 4
//   vec_full    two 16-B loads, the 4 slots updated, both vectors stored back
//               (every byte of every line written: no partially written line)
// Build: make -C tools  (tools/_bin/probe_sparse_rmw)
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                \
  do {                                                       \
    hipError_t e = (x);                                      \
    if (e != hipSuccess) {                                   \
      fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e)); \
      exit(1);                                               \
    }                                                        \
  } while (0)

typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ __launch_bounds__(256) void k_rmw(float* __restrict__ store, const float* __restrict__ vals, uint64_t n) {
  // n request keys, a multiple of 4; lane unit j owns keys 4j..4j+3 at slots 8j + 2k
  const uint64_t units = n / 4;
  for (uint64_t j = (uint64_t)blockIdx.x * 256 + threadIdx.x; j < units; j += (uint64_t)gridDim.x * 256) {
    const f32x4 v = __builtin_nontemporal_load(reinterpret_cast<const f32x4*>(vals) + j);
    float* s = store + 8 * j;
    if constexpr (MODE == 0) {
      float x[4];
#pragma unroll
      for (int k = 0; k < 4; ++k) x[k] = s[2 * k];
#pragma unroll
      for (int k = 0; k < 4; ++k) s[2 * k] = x[k] + v[k];
    } else {
      f32x4 a = reinterpret_cast<const f32x4*>(s)[0], b = reinterpret_cast<const f32x4*>(s)[1];
      a[0] += v[0];
      a[2] += v[1];
      b[0] += v[2];
      b[2] += v[3];
      if constexpr (MODE == 1) {
        s[0] = a[0];
        s[2] = a[2];
        s[4] = b[0];
        s[6] = b[2];
      } else {
        reinterpret_cast<f32x4*>(s)[0] = a;
        reinterpret_cast<f32x4*>(s)[1] = b;
      }
    }
  }
}

__global__ void k_fill(float* __restrict__ a, uint64_t n, uint32_t seed) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    uint32_t x = (uint32_t)i * 2654435761u + seed * 40503u;
    x ^= x >> 15;
    a[i] = (float)(x % 1000u);
  }
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? strtoull(argv[1], nullptr, 10) : 10000000ull;
  const int rounds = argc > 2 ? atoi(argv[2]) : 3;
  int cus = 256;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  float *store, *vals;
  CK(hipMalloc(&store, 2 * n * 4));
  CK(hipMalloc(&vals, n * 4));
  k_fill<<<1024, 256>>>(store, 2 * n, 1u);
  k_fill<<<1024, 256>>>(vals, n, 5u);
  CK(hipDeviceSynchronize());
  const char* names[3] = {"scalar", "vec_load", "vec_full"};
  std::vector<std::vector<float>> res(3);
  hipEvent_t a, b;
  CK(hipEventCreate(&a));
  CK(hipEventCreate(&b));
  for (int r = 0; r < rounds; ++r)
    for (int m = 0; m < 3; ++m)
      for (int bpc : {8}) {
        auto go = [&] {
          const unsigned g = (unsigned)(cus * bpc);
          if (m == 0) k_rmw<0><<<g, 256>>>(store, vals, n);
          else if (m == 1) k_rmw<1><<<g, 256>>>(store, vals, n);
          else k_rmw<2><<<g, 256>>>(store, vals, n);
        };
        for (int i = 0; i < 3; ++i) go();
        std::vector<float> t;
        for (int i = 0; i < 20; ++i) {
          CK(hipEventRecord(a, 0));
          go();
          CK(hipEventRecord(b, 0));
          CK(hipEventSynchronize(b));
          float ms;
          CK(hipEventElapsedTime(&ms, a, b));
          t.push_back(ms);
        }
        std::sort(t.begin(), t.end());
        res[m].push_back(t[t.size() / 2]);
      }
  printf("store RMW at every 2nd slot: %llu values into %llu slots, %d rounds; TB/s of the lines touched (vals 4 + store 8 r + 8 w per value)\n",
         (unsigned long long)n, (unsigned long long)(2 * n), rounds);
  for (int m = 0; m < 3; ++m) {
    printf("%-10s", names[m]);
    for (float ms : res[m]) printf("  %.4f ms (%.2f TB/s)", ms, 20.0 * n / (ms * 1e-3) / 1e12);
    printf("\n");
  }
  return 0;
}
