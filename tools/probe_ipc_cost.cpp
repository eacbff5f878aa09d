// probe_ipc_cost.cpp — per-call host cost of the runtime calls on the TCP Van's
// HBM-frame path (process mode): hipMemGetAddressRange, hipIpcGetMemHandle,
// hipPointerGetAttribute(BUFFER_ID), hipStreamWriteValue32, hipStreamSynchronize.
// build: make -C tools  (tools/_bin/probe_ipc_cost)
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstring>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { std::printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)
using clk = std::chrono::steady_clock;
static double us(clk::time_point a, clk::time_point b, int n) { return std::chrono::duration<double, std::micro>(b - a).count() / n; }
int main() {
  void* p = nullptr;
  CK(hipMalloc(&p, 80 << 20));
  const int N = 2000;
  hipDeviceptr_t base; size_t size;
  auto t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)((char*)p + 4096)));
  auto t1 = clk::now();
  std::printf("hipMemGetAddressRange      %.2f us\n", us(t0, t1, N));
  hipIpcMemHandle_t h;
  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipIpcGetMemHandle(&h, p));
  t1 = clk::now();
  std::printf("hipIpcGetMemHandle         %.2f us\n", us(t0, t1, N));
  unsigned long long id = 0;
  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)((char*)p + 4096)));
  t1 = clk::now();
  std::printf("hipPointerGetAttribute(ID) %.2f us (id %llu)\n", us(t0, t1, N), id);
  hipPointerAttribute_t a;
  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipPointerGetAttributes(&a, (char*)p + 4096));
  t1 = clk::now();
  std::printf("hipPointerGetAttributes    %.2f us\n", us(t0, t1, N));
  hipStream_t s; CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  CK(hipStreamSynchronize(s));
  t0 = clk::now();
  for (int i = 0; i < N; ++i) CK(hipStreamSynchronize(s));
  t1 = clk::now();
  std::printf("hipStreamSynchronize idle  %.2f us\n", us(t0, t1, N));
  uint32_t* hw; CK(hipHostMalloc((void**)&hw, 64, hipHostMallocMapped | hipHostMallocCoherent));
  uint32_t* dw; CK(hipHostGetDevicePointer((void**)&dw, hw, 0));
  t0 = clk::now();
  for (int i = 1; i <= N; ++i) {
    CK(hipStreamWriteValue32(s, dw, i, 0));
    while (*(volatile uint32_t*)hw != (uint32_t)i) __builtin_ia32_pause();
  }
  t1 = clk::now();
  std::printf("writeValue32 + poll        %.2f us\n", us(t0, t1, N));
  t0 = clk::now();
  for (int i = 0; i < N; ++i) { CK(hipMemsetAsync(p, 0, 4, s)); CK(hipStreamSynchronize(s)); }
  t1 = clk::now();
  std::printf("memset(4B) + sync          %.2f us\n", us(t0, t1, N));
  // a second allocation reusing the freed address: does the buffer id change?
  CK(hipFree(p));
  void* q = nullptr; CK(hipMalloc(&q, 80 << 20));
  unsigned long long id2 = 0;
  CK(hipPointerGetAttribute(&id2, HIP_POINTER_ATTRIBUTE_BUFFER_ID, (hipDeviceptr_t)q));
  hipIpcMemHandle_t h2; CK(hipIpcGetMemHandle(&h2, q));
  std::printf("realloc: same address %d, buffer id %llu -> %llu, handle same %d\n", p == q, id, id2,
              memcmp(&h, &h2, sizeof(h)) == 0);
  return 0;
}
