// probe_pmc_shapes.hip — calibrate rocprofv3's HBM byte counters on gfx950 for
// the access shapes the keyed store kernels use.
//
// MI355X_MICROARCH.md ("HBM") documents one shape only: a wide (16 B / lane)
// coalesced streaming read, for which FETCH_SIZE reports exactly half of the
// bytes; "other access widths are uncalibrated".  The keyed kernels
// (csrc/psg_store.hip k_resolve_apply, k_ident_*, k_slots_vec) also read 8-B
// and 4-B values per lane, gather scattered 4-B store values, and write single
// slots or 32-B spans of a line.  Each kernel below touches a KNOWN set of
// 128-B lines with one of those shapes, over 512 MiB (twice the Infinity
// Cache), so a pass of
//   rocprofv3 --pmc FETCH_SIZE | WRITE_SIZE | TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum TCC_BUBBLE_sum
//             | TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum
// gives, per shape, the counter against the bytes the shape moves (lines
// touched x 128 B for reads; for writes, the bytes written and the lines
// they fall in).  tools/pmc_calib.py turns the passes into the factor table
// (profiles/r5_pmc_calibration.json) that tools/pmc_summary.py applies.
//
// Shapes (names are the kernel names the CSV carries):
//   p_rd16       16-B loads, coalesced, every line            (the guide's case)
//   p_rd8        8-B loads, coalesced, every line              (request keys, 8 B / lane)
//   p_rd4        4-B loads, coalesced, every line              (request values, 4 B / lane)
//   p_rd4_half   4-B loads of every other word                 (a sparse request's store values)
//   p_gather4    one 4-B load in each line, lines in random order  (scattered store values)
//   p_gather8    one 8-B load in each line, random order           (scattered store keys)
//   p_wr16       16-B stores, coalesced, every line
//   p_wr4        4-B stores, coalesced, every line
//   p_wr4_half   4-B stores to every other word (each line half written)
//   p_span32     32-B spans (two 16-B stores) at a 64-B stride (each line half written)
//   p_scatter4   one 4-B store in each line, random order
//   p_rmw4       one 4-B load + add + store in each line, random order (a sparse slot RMW)
// usage: probe_pmc_shapes [reps]
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                   \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned long long u64;

constexpr u64 kBytes = u64(512) << 20;     // the region every shape covers
constexpr u64 kLines = kBytes / 128;       // 4 M lines
constexpr u64 kOdd = 0x9E3779B97F4A7C15ull;  // odd: i -> i * kOdd mod 2^22 permutes the lines

__device__ __forceinline__ u64 perm(u64 i) { return (i * kOdd) & (kLines - 1); }
__device__ __forceinline__ u64 gid() { return (u64)blockIdx.x * blockDim.x + threadIdx.x; }
__device__ __forceinline__ u64 gstride() { return (u64)gridDim.x * blockDim.x; }

// a sink that keeps the loads alive: one word per block, written only when the
// (never true) sum matches a magic value
__device__ __forceinline__ void sink(unsigned v, unsigned* out) {
  if (v == 0x12345678u) out[blockIdx.x] = v;
}

__global__ void p_rd16(const u32x4* a, unsigned* out) {
  unsigned acc = 0;
  for (u64 i = gid(); i < kBytes / 16; i += gstride()) {
    const u32x4 v = a[i];
    acc ^= v[0] ^ v[1] ^ v[2] ^ v[3];
  }
  sink(acc, out);
}
__global__ void p_rd8(const u64* a, unsigned* out) {
  unsigned acc = 0;
  for (u64 i = gid(); i < kBytes / 8; i += gstride()) acc ^= (unsigned)a[i] ^ (unsigned)(a[i] >> 32);
  sink(acc, out);
}
__global__ void p_rd4(const unsigned* a, unsigned* out) {
  unsigned acc = 0;
  for (u64 i = gid(); i < kBytes / 4; i += gstride()) acc ^= a[i];
  sink(acc, out);
}
__global__ void p_rd4_half(const unsigned* a, unsigned* out) {
  unsigned acc = 0;
  for (u64 i = gid(); i < kBytes / 8; i += gstride()) acc ^= a[2 * i];
  sink(acc, out);
}
__global__ void p_gather4(const unsigned* a, unsigned* out) {
  unsigned acc = 0;
  for (u64 i = gid(); i < kLines; i += gstride()) acc ^= a[perm(i) * 32 + (i & 31)];
  sink(acc, out);
}
__global__ void p_gather8(const u64* a, unsigned* out) {
  unsigned acc = 0;
  for (u64 i = gid(); i < kLines; i += gstride()) acc ^= (unsigned)a[perm(i) * 16 + (i & 15)];
  sink(acc, out);
}
__global__ void p_wr16(u32x4* b) {
  for (u64 i = gid(); i < kBytes / 16; i += gstride()) b[i] = u32x4{(unsigned)i, 1u, 2u, 3u};
}
__global__ void p_wr4(unsigned* b) {
  for (u64 i = gid(); i < kBytes / 4; i += gstride()) b[i] = (unsigned)i;
}
__global__ void p_wr4_half(unsigned* b) {
  for (u64 i = gid(); i < kBytes / 8; i += gstride()) b[2 * i] = (unsigned)i;
}
__global__ void p_span32(u32x4* b) {
  for (u64 i = gid(); i < kBytes / 64; i += gstride()) {
    b[4 * i] = u32x4{(unsigned)i, 1u, 2u, 3u};
    b[4 * i + 1] = u32x4{(unsigned)i, 5u, 6u, 7u};
  }
}
__global__ void p_scatter4(unsigned* b) {
  for (u64 i = gid(); i < kLines; i += gstride()) b[perm(i) * 32 + (i & 31)] = (unsigned)i;
}
__global__ void p_rmw4(unsigned* b) {
  for (u64 i = gid(); i < kLines; i += gstride()) {
    unsigned* p = b + perm(i) * 32 + (i & 31);
    *p = *p + 1u;
  }
}

int main(int argc, char** argv) {
  const int reps = argc > 1 ? std::atoi(argv[1]) : 3;
  void *a, *b, *c;
  unsigned* out;
  CK(hipMalloc(&a, kBytes));
  CK(hipMalloc(&b, kBytes));
  CK(hipMalloc(&c, kBytes));  // evicts the Infinity Cache between shapes
  CK(hipMalloc(&out, 1 << 20));
  CK(hipMemset(a, 1, kBytes));
  CK(hipMemset(b, 2, kBytes));
  CK(hipDeviceSynchronize());
  const dim3 g(2048), t(256);
  for (int r = 0; r < reps; ++r) {
#define RUN(k, ...)                                   \
  do {                                                \
    CK(hipMemsetAsync(c, r, kBytes, 0));              \
    hipLaunchKernelGGL(k, g, t, 0, 0, __VA_ARGS__);   \
    CK(hipGetLastError());                            \
  } while (0)
    RUN(p_rd16, (const u32x4*)a, out);
    RUN(p_rd8, (const u64*)a, out);
    RUN(p_rd4, (const unsigned*)a, out);
    RUN(p_rd4_half, (const unsigned*)a, out);
    RUN(p_gather4, (const unsigned*)a, out);
    RUN(p_gather8, (const u64*)a, out);
    RUN(p_wr16, (u32x4*)b);
    RUN(p_wr4, (unsigned*)b);
    RUN(p_wr4_half, (unsigned*)b);
    RUN(p_span32, (u32x4*)b);
    RUN(p_scatter4, (unsigned*)b);
    RUN(p_rmw4, (unsigned*)b);
#undef RUN
  }
  CK(hipDeviceSynchronize());
  std::printf("probe_pmc_shapes: %d reps of 12 shapes over %llu MiB\n", reps, kBytes >> 20);
  return 0;
}
