// tools/probe_latency.hip — what the host waits for after a kernel ends
// (round 6: the drop-in line's idle gaps between a server's last pass and the
// next request's slicer).  For a tiny kernel and for a ~40 µs copy kernel:
//   word   the kernel's last block stores a tag into pinned host memory (vector
//          store, system scope); the host spins on it
//   event  hipEventRecord behind the kernel; the host polls hipEventQuery
//   sync   hipStreamSynchronize
// and the launch itself (hipLaunchKernel's host time).  Times are host wall
// clock from just before the launch, median of 200.
#include <hip/hip_runtime.h>
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                  \
  do {                                                                         \
    hipError_t e_ = (x);                                                       \
    if (e_ != hipSuccess) {                                                    \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));             \
      std::exit(1);                                                            \
    }                                                                          \
  } while (0)

using clk = std::chrono::steady_clock;

__global__ void k_copy_tag(const float4* __restrict__ a, float4* __restrict__ b, size_t n, unsigned* count,
                           unsigned* word, unsigned tag) {
  const size_t stride = (size_t)gridDim.x * blockDim.x;
  for (size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += stride) b[i] = a[i];
  if (!word) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    __threadfence();
    const unsigned prev = atomicAdd(count, 1u);
    if (prev == gridDim.x - 1) {
      *count = 0;
      __threadfence_system();
      __hip_atomic_store(word, tag, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    }
  }
}

static double us_since(clk::time_point t0) {
  return std::chrono::duration<double, std::micro>(clk::now() - t0).count();
}

int main() {
  CK(hipSetDevice(0));
  hipStream_t st;
  CK(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  hipEvent_t ev;
  CK(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  unsigned* word = nullptr;
  CK(hipHostMalloc((void**)&word, 64, hipHostMallocCoherent));
  *word = 0;
  unsigned* count = nullptr;
  CK(hipMalloc((void**)&count, 64));
  CK(hipMemset(count, 0, 64));
  const size_t big = (size_t)160 << 20;  // 160 MiB each way: ~40 µs at ~8 TB/s
  float4 *a = nullptr, *b = nullptr;
  CK(hipMalloc((void**)&a, big));
  CK(hipMalloc((void**)&b, big));
  CK(hipMemset(a, 0, big));
  CK(hipDeviceSynchronize());
  unsigned tag = 0;
  for (int sz = 0; sz < 2; ++sz) {
    const size_t n = sz ? big / sizeof(float4) : 1024;
    const unsigned grid = sz ? 2048 : 4;
    for (int mode = 0; mode < 3; ++mode) {
      std::vector<double> launch, done;
      for (int it = 0; it < 220; ++it) {
        ++tag;
        const auto t0 = clk::now();
        k_copy_tag<<<grid, 256, 0, st>>>(a, b, n, count, mode == 0 ? word : nullptr, tag);
        if (mode == 1) CK(hipEventRecord(ev, st));
        const double tl = us_since(t0);
        if (mode == 0) {
          const auto tw = clk::now();
          while (__atomic_load_n(word, __ATOMIC_ACQUIRE) != tag) {
            if (std::chrono::duration<double>(clk::now() - tw).count() > 2.0) {
              std::fprintf(stderr, "word never came\n");
              std::exit(1);
            }
            __builtin_ia32_pause();
          }
        } else if (mode == 1) {
          hipError_t q;
          while ((q = hipEventQuery(ev)) == hipErrorNotReady) __builtin_ia32_pause();
          CK(q);
        } else {
          CK(hipStreamSynchronize(st));
        }
        const double td = us_since(t0);
        if (mode == 0) CK(hipStreamSynchronize(st));  // the kernel's tail before the next launch
        if (it >= 20) launch.push_back(tl), done.push_back(td);
      }
      std::sort(launch.begin(), launch.end());
      std::sort(done.begin(), done.end());
      const char* names[] = {"word", "event", "sync"};
      std::printf("{\"kernel\": \"%s\", \"wait\": \"%s\", \"launch_us_p50\": %.2f, \"done_us_p50\": %.2f, "
                  "\"done_us_p10\": %.2f, \"done_us_p90\": %.2f}\n",
                  sz ? "copy 160 MiB" : "tiny", names[mode], launch[launch.size() / 2], done[done.size() / 2],
                  done[done.size() / 10], done[done.size() * 9 / 10]);
    }
  }
  CK(hipFree(a));
  CK(hipFree(b));
  CK(hipFree(count));
  CK(hipHostFree(word));
  return 0;
}
