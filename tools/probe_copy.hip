// probe_copy.hip — what a 1 GiB float4 copy (read 1 GiB, write 1 GiB: the
// 256 M-float Pull's exact traffic) reaches on this MI355X, by kernel shape,
// all in one process on the same two buffers, interleaved rounds.
//   make -C tools  (tools/_bin/probe_copy)
//   probe_copy [MiB] [rounds]
// Variants: grid-stride with U vectors per lane in flight and B blocks per CU,
// non-temporal (nt) or default loads / stores, and a chunked form where each
// block copies one contiguous slab.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                         \
  do {                                                                                \
    hipError_t e_ = (x);                                                              \
    if (e_ != hipSuccess) {                                                           \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(2);                                                                   \
    }                                                                                 \
  } while (0)

template <int NT>
__device__ __forceinline__ u32x4 ld(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int NT>
__device__ __forceinline__ void st(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int U, int NTL, int NTS, int BS>
__global__ __launch_bounds__(BS) void k_copy_stride(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                    uint64_t nvec) {
  const uint64_t tile = (uint64_t)BS * U, gs = (uint64_t)gridDim.x * tile;
  for (uint64_t b = (uint64_t)blockIdx.x * tile + threadIdx.x; b < nvec; b += gs) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + (uint64_t)u * BS < nvec) v[u] = ld<NTL>(src + b + (uint64_t)u * BS);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + (uint64_t)u * BS < nvec) st<NTS>(dst + b + (uint64_t)u * BS, v[u]);
  }
}

// each block one contiguous slab of nvec / gridDim vectors
template <int U, int NTL, int NTS, int BS>
__global__ __launch_bounds__(BS) void k_copy_chunk(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                   uint64_t nvec) {
  const uint64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  const uint64_t lo = (uint64_t)blockIdx.x * per, hi = std::min<uint64_t>(nvec, lo + per);
  for (uint64_t b = lo + threadIdx.x; b < hi; b += (uint64_t)BS * U) {
    u32x4 v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + (uint64_t)u * BS < hi) v[u] = ld<NTL>(src + b + (uint64_t)u * BS);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (b + (uint64_t)u * BS < hi) st<NTS>(dst + b + (uint64_t)u * BS, v[u]);
  }
}

struct Variant {
  std::string name;
  void (*launch)(const u32x4*, u32x4*, uint64_t, int, hipStream_t);
  int bpc;
};

template <int U, int NTL, int NTS, int BS, bool CHUNK>
void launch(const u32x4* s, u32x4* d, uint64_t nvec, int blocks, hipStream_t st) {
  if (CHUNK)
    k_copy_chunk<U, NTL, NTS, BS><<<blocks, BS, 0, st>>>(s, d, nvec);
  else
    k_copy_stride<U, NTL, NTS, BS><<<blocks, BS, 0, st>>>(s, d, nvec);
}

int main(int argc, char** argv) {
  const uint64_t mib = argc > 1 ? std::strtoull(argv[1], nullptr, 10) : 1024;
  const int rounds = argc > 2 ? std::atoi(argv[2]) : 4;
  const uint64_t bytes = mib << 20, nvec = bytes / 16;
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  u32x4 *src = nullptr, *dst = nullptr;
  CK(hipMalloc(&src, bytes));
  CK(hipMalloc(&dst, bytes));
  // a byte pattern that varies along the buffer (not one repeated value)
  {
    std::vector<unsigned char> h(bytes < (64u << 20) ? bytes : (64u << 20));
    for (size_t i = 0; i < h.size(); ++i) h[i] = (unsigned char)((i * 2654435761u) >> 13);
    for (uint64_t off = 0; off < bytes; off += h.size())
      CK(hipMemcpy((char*)src + off, h.data(), std::min<uint64_t>(h.size(), bytes - off), hipMemcpyHostToDevice));
  }
  CK(hipMemset(dst, 0, bytes));
  CK(hipDeviceSynchronize());
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  std::vector<Variant> vs = {
      {"stride U1 nt/nt B256 4/CU", launch<1, 1, 1, 256, false>, 4},
      {"stride U2 nt/nt B256 2/CU", launch<2, 1, 1, 256, false>, 2},
      {"stride U4 nt/nt B256 2/CU", launch<4, 1, 1, 256, false>, 2},
      {"stride U4 nt/nt B256 3/CU", launch<4, 1, 1, 256, false>, 3},
      {"stride U4 nt/nt B256 4/CU", launch<4, 1, 1, 256, false>, 4},
      {"stride U8 nt/nt B256 1/CU", launch<8, 1, 1, 256, false>, 1},
      {"stride U8 nt/nt B256 2/CU", launch<8, 1, 1, 256, false>, 2},
      {"stride U4 nt/nt B512 1/CU", launch<4, 1, 1, 512, false>, 1},
      {"stride U2 nt/nt B512 2/CU", launch<2, 1, 1, 512, false>, 2},
      {"stride U4 nt/def B256 2/CU", launch<4, 1, 0, 256, false>, 2},
      {"stride U4 def/nt B256 2/CU", launch<4, 0, 1, 256, false>, 2},
      {"stride U16 nt/nt B256 1/CU", launch<16, 1, 1, 256, false>, 1},
  };

  std::vector<std::vector<float>> ms(vs.size());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  const int reps = 10;
  for (int r = 0; r < rounds; ++r) {
    for (size_t k = 0; k < vs.size(); ++k) {
      const int blocks = cus * vs[k].bpc;
      for (int w = 0; w < 2; ++w) vs[k].launch(src, dst, nvec, blocks, st);
      CK(hipEventRecord(e0, st));
      for (int i = 0; i < reps; ++i) vs[k].launch(src, dst, nvec, blocks, st);
      CK(hipEventRecord(e1, st));
      CK(hipEventSynchronize(e1));
      float t = 0;
      CK(hipEventElapsedTime(&t, e0, e1));
      ms[k].push_back(t / reps);
    }
  }
  std::printf("copy %llu MiB (read + write = %.2f GB per launch), %d CUs, %d rounds x %d launches\n",
              (unsigned long long)mib, 2.0 * bytes / 1e9, cus, rounds, reps);
  for (size_t k = 0; k < vs.size(); ++k) {
    auto v = ms[k];
    std::sort(v.begin(), v.end());
    const float med = v[v.size() / 2], best = v[0];
    std::printf("%-30s median %.4f ms  %.3f TB/s (%.3f of 8)  best %.3f TB/s\n", vs[k].name.c_str(), med,
                2.0 * bytes / (med * 1e-3) / 1e12, 2.0 * bytes / (med * 1e-3) / 8e12, 2.0 * bytes / (best * 1e-3) / 1e12);
  }
  return 0;
}
