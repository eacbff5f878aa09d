// probe_push_small.hip — launch shape of the dense Push (store += vals, 12 B
// per float) and Pull (out = store, 8 B) at the LR steady state's size (the
// 10 M-key cached stretch, a 40 MB store that stays in the Infinity Cache
// between requests), timed the way bench.py times them: Push then Pull on one
// stream, an event before, between and after, medians over 30 steps, shapes
// interleaved over rounds, one process.
//   make -C tools  (tools/_bin/probe_push_small)
//   probe_push_small [floats] [rounds]
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                                 \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) {                                                                   \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                           \
    }                                                                                         \
  } while (0)

// the library's k_dense_vec shape: U vectors per lane, grid stride; request
// stream non-temporal, store default policy
template <int U, int BS, bool PUSH, bool SNT = false>
__global__ __launch_bounds__(BS) void k_op(u32x4* __restrict__ store, const u32x4* __restrict__ vals,
                                           u32x4* __restrict__ out, uint64_t nvec) {
  const uint64_t tile = (uint64_t)BS * U, gs = (uint64_t)gridDim.x * tile;
  for (uint64_t b = (uint64_t)blockIdx.x * tile + threadIdx.x; b < nvec; b += gs) {
    u32x4 s[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * BS;
      if (i < nvec) {
        if (PUSH) v[u] = __builtin_nontemporal_load(vals + i);
        s[u] = SNT ? __builtin_nontemporal_load(store + i) : store[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * BS;
      if (i < nvec) {
        if (PUSH) {
          const u32x4 r = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, s[u]) + __builtin_bit_cast(f32x4, v[u]));
          if (SNT) __builtin_nontemporal_store(r, store + i);
          else store[i] = r;
        } else {
          __builtin_nontemporal_store(s[u], out + i);
        }
      }
    }
  }
}

// each block one contiguous slab (nvec / grid vectors)
template <int U, int BS, bool PUSH>
__global__ __launch_bounds__(BS) void k_op_chunk(u32x4* __restrict__ store, const u32x4* __restrict__ vals,
                                                 u32x4* __restrict__ out, uint64_t nvec) {
  const uint64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = (uint64_t)blockIdx.x * per, hi = std::min<uint64_t>(nvec, lo + per);
  for (uint64_t b = lo + threadIdx.x; b < hi; b += (uint64_t)BS * U) {
    u32x4 s[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * BS;
      if (i < hi) {
        if (PUSH) v[u] = __builtin_nontemporal_load(vals + i);
        s[u] = store[i];
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t i = b + (uint64_t)u * BS;
      if (i < hi) {
        if (PUSH) {
          store[i] = __builtin_bit_cast(u32x4, __builtin_bit_cast(f32x4, s[u]) + __builtin_bit_cast(f32x4, v[u]));
        } else {
          __builtin_nontemporal_store(s[u], out + i);
        }
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

struct Shape {
  std::string name;
  void (*push)(u32x4*, const u32x4*, u32x4*, uint64_t, int, hipStream_t);
  void (*pull)(u32x4*, const u32x4*, u32x4*, uint64_t, int, hipStream_t);
  int blocks_per_cu;
};

template <int U, int BS, bool PUSH, bool CHUNK, bool SNT = false>
void go(u32x4* st, const u32x4* v, u32x4* o, uint64_t nvec, int blocks, hipStream_t s) {
  const uint64_t need = (nvec + (uint64_t)BS * U - 1) / ((uint64_t)BS * U);
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>(need, (uint64_t)blocks));
  if (CHUNK)
    k_op_chunk<U, BS, PUSH><<<g, BS, 0, s>>>(st, v, o, nvec);
  else
    k_op<U, BS, PUSH, SNT><<<g, BS, 0, s>>>(st, v, o, nvec);
}

int main(int argc, char** argv) {
  const uint64_t n = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 10000000ull;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 4;
  const uint64_t nvec = n / 4;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4 *st = nullptr, *v = nullptr, *o = nullptr;
  CK(hipMalloc(&st, n * 4));
  CK(hipMalloc(&v, n * 4));
  CK(hipMalloc(&o, n * 4));
  // integer-valued floats, as bench.py's synthetic data (all-zero buffers
  // measured up to 20 % faster than real values: not a workload)
  k_fill<<<1024, 256>>>((float*)st, n, 1u);
  k_fill<<<1024, 256>>>((float*)v, n, 7u);
  CK(hipGetLastError());
  CK(hipDeviceSynchronize());
  hipStream_t s;
  CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  std::vector<Shape> shapes = {
      {"U1 B256 8/CU", go<1, 256, true, false>, go<1, 256, false, false>, 8},
      {"U2 B256 2/CU", go<2, 256, true, false>, go<2, 256, false, false>, 2},
      {"U1 B256 4/CU", go<1, 256, true, false>, go<1, 256, false, false>, 4},
      {"U1 B512 2/CU", go<1, 512, true, false>, go<1, 512, false, false>, 2},
      {"U1 B512 4/CU", go<1, 512, true, false>, go<1, 512, false, false>, 4},
      {"U1 B512 4/CU store nt", go<1, 512, true, false, true>, go<1, 512, false, false, true>, 4},
      {"U1 B256 8/CU store nt", go<1, 256, true, false, true>, go<1, 256, false, false, true>, 8},
      {"U2 B256 2/CU store nt", go<2, 256, true, false, true>, go<2, 256, false, false, true>, 2},
      {"U1 B512 3/CU", go<1, 512, true, false>, go<1, 512, false, false>, 3},
      {"U1 B1024 2/CU", go<1, 1024, true, false>, go<1, 1024, false, false>, 2},
      {"U1 B1024 1/CU", go<1, 1024, true, false>, go<1, 1024, false, false>, 1},
      {"U2 B512 2/CU", go<2, 512, true, false>, go<2, 512, false, false>, 2},
      {"U2 B256 4/CU", go<2, 256, true, false>, go<2, 256, false, false>, 4},
      {"U2 B1024 1/CU", go<2, 1024, true, false>, go<2, 1024, false, false>, 1},
  };

  const int steps = 30;
  std::vector<hipEvent_t> ev(2 * steps + 1);
  for (auto& e : ev) CK(hipEventCreate(&e));
  std::vector<std::vector<float>> push(shapes.size()), pull(shapes.size()), stepms(shapes.size());
  for (int r = 0; r < rounds; ++r) {
    for (size_t k = 0; k < shapes.size(); ++k) {
      const int blocks = cus * shapes[k].blocks_per_cu;
      for (int w = 0; w < 3; ++w) {
        shapes[k].push(st, v, o, nvec, blocks, s);
        shapes[k].pull(st, v, o, nvec, blocks, s);
      }
      CK(hipEventRecord(ev[0], s));
      for (int i = 0; i < steps; ++i) {
        shapes[k].push(st, v, o, nvec, blocks, s);
        CK(hipEventRecord(ev[2 * i + 1], s));
        shapes[k].pull(st, v, o, nvec, blocks, s);
        CK(hipEventRecord(ev[2 * i + 2], s));
      }
      CK(hipStreamSynchronize(s));
      std::vector<float> a, b;
      for (int i = 0; i < steps; ++i) {
        float x = 0, y = 0;
        CK(hipEventElapsedTime(&x, ev[2 * i], ev[2 * i + 1]));
        CK(hipEventElapsedTime(&y, ev[2 * i + 1], ev[2 * i + 2]));
        a.push_back(x);
        b.push_back(y);
      }
      std::sort(a.begin(), a.end());
      std::sort(b.begin(), b.end());
      push[k].push_back(a[steps / 2]);
      pull[k].push_back(b[steps / 2]);
      // unperturbed: steps back to back, one event pair around them all
      CK(hipEventRecord(ev[0], s));
      for (int i = 0; i < steps; ++i) {
        shapes[k].push(st, v, o, nvec, blocks, s);
        shapes[k].pull(st, v, o, nvec, blocks, s);
      }
      CK(hipEventRecord(ev[1], s));
      CK(hipStreamSynchronize(s));
      float t = 0;
      CK(hipEventElapsedTime(&t, ev[0], ev[1]));
      stepms[k].push_back(t / steps);
    }
  }
  std::printf("dense Push / Pull at %llu floats, %d rounds x %d steps; fractions of 8 TB/s at 12 / 8 B per float\n",
              (unsigned long long)n, rounds, steps);
  for (size_t k = 0; k < shapes.size(); ++k) {
    auto med = [](std::vector<float> x) {
      std::sort(x.begin(), x.end());
      return x[x.size() / 2];
    };
    const float pm = med(push[k]), lm = med(pull[k]), sm = med(stepms[k]);
    std::printf("%-26s push %.2f us (%.3f)  pull %.2f us (%.3f)  step unperturbed %.2f us (Push+Pull %.1f GB/s)\n",
                shapes[k].name.c_str(), pm * 1e3, 12.0 * n / (pm * 1e-3) / 8e12, lm * 1e3, 8.0 * n / (lm * 1e-3) / 8e12,
                sm * 1e3, 8.0 * n / (sm * 1e-3) / 1e9);
  }
  return 0;
}
