// psg_runtime.hip — runtime entry points of the psg C-ABI: errors, device,
// memory, streams, events, seeded synthetic data.
#include <cstring>
#include <mutex>
#include <vector>

#include "psg_internal.h"

namespace psg {

static thread_local std::string g_err;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_err = buf;
}
void clear_error() { g_err.clear(); }

int hip_fail(hipError_t e, const char* what, const char* file, int line) {
  set_error("%s failed: %s (%s:%d)", what, hipGetErrorString(e), file, line);
  return e == hipErrorOutOfMemory ? PSG_ERR_OOM : PSG_ERR_HIP;
}

int max_stream_blocks() {
  static int cached[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  if (cached[dev] == 0) {
    int cus = 256;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess) cus = 256;
    cached[dev] = cus * 8;
  }
  return cached[dev];
}

__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

template <typename T>
__global__ __launch_bounds__(256) void k_synth(T* __restrict__ out, uint64_t n, uint64_t seed,
                                               int mode, double lo, double hi) {
  const double inv24 = 1.0 / 16777216.0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t r = splitmix64(seed + i) >> 40;  // 24 random bits
    double v;
    if (mode == 0) {
      v = floor((double)r * (hi - lo) * inv24) + lo;
    } else {
      v = lo + ((double)r * inv24) * (hi - lo);
    }
    // f16 / bf16 go through f32 (two RNE steps), restated exactly by the oracle.
    if constexpr (sizeof(T) < 4) out[i] = (T)(float)v; else out[i] = (T)v;
  }
}

__global__ __launch_bounds__(256) void k_keys_arith(uint64_t* __restrict__ keys, uint64_t n,
                                                    uint64_t base, uint64_t step) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    keys[i] = base + i * step;
}

// Position-keyed checksum of n 64-bit words: sum_i splitmix64(w_i ^ (i * phi))
// (mod 2^64).  One wave-reduced partial per block; the host adds the partials.
__global__ __launch_bounds__(256) void k_checksum(const uint64_t* __restrict__ w, uint64_t n,
                                                  uint64_t* __restrict__ partials) {
  uint64_t h = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    h += splitmix64(__builtin_nontemporal_load(w + i) ^ (i * 0x9e3779b97f4a7c15ull));
  for (int o = 32; o > 0; o >>= 1) {  // 64-bit butterfly as two 32-bit shuffles
    const uint32_t lo = __shfl_xor((uint32_t)h, o, 64), hi = __shfl_xor((uint32_t)(h >> 32), o, 64);
    h += ((uint64_t)hi << 32) | lo;
  }
  __shared__ uint64_t part[kBlock / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int k = 0; k < kBlock / 64; ++k) t += part[k];
    partials[blockIdx.x] = t;
  }
}

// Closed-form check of a pulled vector: got[i] == scale * sum_{w < nseeds} of
// the integer-valued synth value of (seed0 + w, i + offset), computed in double
// (exact for the integer sums the bench and tests use).  Per block: mismatch
// count and the smallest mismatching index (plain stores, the host reduces).
template <typename T>
__global__ __launch_bounds__(256) void k_verify_synth_sum(const T* __restrict__ got, uint64_t n,
                                                          uint64_t seed0, int nseeds, uint64_t offset,
                                                          double lo, double hi, double scale,
                                                          uint64_t* __restrict__ part) {
  const double inv24 = 1.0 / 16777216.0;
  uint64_t bad = 0, first = ~0ull;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x) {
    double e = 0.0;
    for (int w = 0; w < nseeds; ++w) {
      const uint64_t r = splitmix64(seed0 + (uint64_t)w + offset + i) >> 40;
      e += floor((double)r * (hi - lo) * inv24) + lo;
    }
    e *= scale;
    double g;
    if constexpr (sizeof(T) < 4) g = (double)(float)got[i]; else g = (double)got[i];
    if (g != e) {
      bad++;
      if (i < first) first = i;
    }
  }
  for (int o = 32; o > 0; o >>= 1) {
    bad += __shfl_xor(bad, o, 64);
    const uint64_t f = __shfl_xor(first, o, 64);
    first = f < first ? f : first;
  }
  __shared__ uint64_t sb[kBlock / 64], sf[kBlock / 64];
  if ((threadIdx.x & 63) == 0) {
    sb[threadIdx.x >> 6] = bad;
    sf[threadIdx.x >> 6] = first;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t b = 0, f = ~0ull;
    for (int k = 0; k < kBlock / 64; ++k) {
      b += sb[k];
      f = sf[k] < f ? sf[k] : f;
    }
    part[2 * blockIdx.x] = b;
    part[2 * blockIdx.x + 1] = f;
  }
}

// The key-list hash of LR key caching (tests/src/LRServer.h:11-29):
// seed = n; for each key x: seed ^= splitmix64(x), whose XOR-fold is
// order-free, so one XOR reduction over the keys computes it.  Per-block
// partials, XOR-ed on the host.
__global__ __launch_bounds__(256) void k_key_list_hash(const uint64_t* __restrict__ keys, uint64_t n,
                                                       uint64_t* __restrict__ partials) {
  uint64_t h = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * blockDim.x)
    h ^= splitmix64(keys[i]);
  for (int o = 32; o > 0; o >>= 1) {
    const uint32_t lo = __shfl_xor((uint32_t)h, o, 64), hi = __shfl_xor((uint32_t)(h >> 32), o, 64);
    h ^= ((uint64_t)hi << 32) | lo;
  }
  __shared__ uint64_t part[kBlock / 64];
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = h;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint64_t t = 0;
    for (int k = 0; k < kBlock / 64; ++k) t ^= part[k];
    partials[blockIdx.x] = t;
  }
}

static unsigned grid_for(uint64_t n) {
  uint64_t b = (n + kBlock - 1) / kBlock;
  uint64_t cap = (uint64_t)max_stream_blocks();
  if (b > cap) b = cap;
  if (b == 0) b = 1;
  return (unsigned)b;
}

}  // namespace psg

using namespace psg;

extern "C" {

int psg_abi_version(void) { return PSG_ABI_VERSION; }
const char* psg_last_error(void) { return g_err.c_str(); }

int psg_device_count(int* n) {
  PSG_REQUIRE(n, PSG_ERR_INVALID, "psg_device_count: null out");
  PSG_HIP(hipGetDeviceCount(n));
  return PSG_OK;
}
int psg_set_device(int device) {
  PSG_HIP(hipSetDevice(device));
  return PSG_OK;
}
int psg_get_device(int* device) {
  PSG_REQUIRE(device, PSG_ERR_INVALID, "psg_get_device: null out");
  PSG_HIP(hipGetDevice(device));
  return PSG_OK;
}

int psg_device_pci_bus_id(int device, char* buf, int len) {
  PSG_REQUIRE(buf && len > 0, PSG_ERR_INVALID, "psg_device_pci_bus_id: null or empty buffer");
  PSG_HIP(hipDeviceGetPCIBusId(buf, len, device));
  buf[len - 1] = 0;
  return PSG_OK;
}
int psg_device_sync(void) {
  PSG_HIP(hipDeviceSynchronize());
  return PSG_OK;
}
int psg_enable_peer_access(int device, int peer) {
  if (device == peer) return PSG_OK;
  int cur = 0, can = 0;
  PSG_HIP(hipGetDevice(&cur));
  PSG_HIP(hipDeviceCanAccessPeer(&can, device, peer));
  PSG_REQUIRE(can, PSG_ERR_UNSUPPORTED, "GPU %d cannot access GPU %d", device, peer);
  PSG_HIP(hipSetDevice(device));
  hipError_t e = hipDeviceEnablePeerAccess(peer, 0);
  if (e == hipErrorPeerAccessAlreadyEnabled) (void)hipGetLastError();
  (void)hipSetDevice(cur);
  if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
    return hip_fail(e, "hipDeviceEnablePeerAccess", __FILE__, __LINE__);
  return PSG_OK;
}

int psg_malloc(void** dptr, size_t bytes) {
  PSG_REQUIRE(dptr, PSG_ERR_INVALID, "psg_malloc: null out");
  *dptr = nullptr;
  if (bytes == 0) return PSG_OK;
  PSG_HIP(hipMalloc(dptr, ipc_alloc_bytes(bytes)));
  return PSG_OK;
}
int psg_free(void* dptr) {
  if (dptr) PSG_HIP(hipFree(dptr));
  return PSG_OK;
}
int psg_host_alloc(void** hptr, size_t bytes) {
  PSG_REQUIRE(hptr, PSG_ERR_INVALID, "psg_host_alloc: null out");
  *hptr = nullptr;
  if (bytes == 0) return PSG_OK;
  PSG_HIP(hipHostMalloc(hptr, bytes, hipHostMallocDefault));
  return PSG_OK;
}
int psg_host_free(void* hptr) {
  if (hptr) PSG_HIP(hipHostFree(hptr));
  return PSG_OK;
}
int psg_host_register(void* hptr, size_t bytes) {
  PSG_REQUIRE(hptr && bytes, PSG_ERR_INVALID, "psg_host_register: empty range");
  PSG_HIP(hipHostRegister(hptr, bytes, hipHostRegisterDefault));
  return PSG_OK;
}
int psg_host_unregister(void* hptr) {
  PSG_HIP(hipHostUnregister(hptr));
  return PSG_OK;
}

int psg_memcpy(void* dst, const void* src, size_t bytes, int kind, psg_stream stream) {
  if (bytes == 0) return PSG_OK;
  PSG_REQUIRE(dst && src, PSG_ERR_INVALID, "psg_memcpy: null pointer");
  hipMemcpyKind k;
  switch (kind) {
    case 0: k = hipMemcpyHostToDevice; break;
    case 1: k = hipMemcpyDeviceToHost; break;
    case 2: k = hipMemcpyDeviceToDevice; break;
    case 3: k = hipMemcpyDefault; break;
    default: set_error("psg_memcpy: bad kind %d", kind); return PSG_ERR_INVALID;
  }
  PSG_HIP(hipMemcpyAsync(dst, src, bytes, k, (hipStream_t)stream));
  return PSG_OK;
}
int psg_memset(void* dptr, int value, size_t bytes, psg_stream stream) {
  if (bytes == 0) return PSG_OK;
  PSG_REQUIRE(dptr, PSG_ERR_INVALID, "psg_memset: null pointer");
  PSG_HIP(hipMemsetAsync(dptr, value, bytes, (hipStream_t)stream));
  return PSG_OK;
}

int psg_stream_create(psg_stream* stream) {
  PSG_REQUIRE(stream, PSG_ERR_INVALID, "psg_stream_create: null out");
  hipStream_t s;
  PSG_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  *stream = (psg_stream)s;
  return PSG_OK;
}
int psg_stream_create_priority(psg_stream* stream, int priority) {
  PSG_REQUIRE(stream, PSG_ERR_INVALID, "psg_stream_create_priority: null out");
  int least = 0, greatest = 0;
  PSG_HIP(hipDeviceGetStreamPriorityRange(&least, &greatest));
  hipStream_t s;
  PSG_HIP(hipStreamCreateWithPriority(&s, hipStreamNonBlocking, priority ? greatest : least));
  *stream = (psg_stream)s;
  return PSG_OK;
}
int psg_stream_destroy(psg_stream stream) {
  if (stream) PSG_HIP(hipStreamDestroy((hipStream_t)stream));
  return PSG_OK;
}
int psg_stream_sync(psg_stream stream) {
  PSG_HIP(hipStreamSynchronize((hipStream_t)stream));
  return PSG_OK;
}
int psg_event_create(psg_event* ev) {
  PSG_REQUIRE(ev, PSG_ERR_INVALID, "psg_event_create: null out");
  hipEvent_t e;
  PSG_HIP(hipEventCreate(&e));
  *ev = (psg_event)e;
  return PSG_OK;
}
int psg_event_create_timing(psg_event* ev) {
  PSG_REQUIRE(ev, PSG_ERR_INVALID, "psg_event_create_timing: null out");
  hipEvent_t e;
  PSG_HIP(hipEventCreateWithFlags(&e, hipEventDisableSystemFence));
  *ev = (psg_event)e;
  return PSG_OK;
}
int psg_event_destroy(psg_event ev) {
  if (ev) PSG_HIP(hipEventDestroy((hipEvent_t)ev));
  return PSG_OK;
}
int psg_event_record(psg_event ev, psg_stream stream) {
  PSG_HIP(hipEventRecord((hipEvent_t)ev, (hipStream_t)stream));
  return PSG_OK;
}
int psg_event_sync(psg_event ev) {
  PSG_HIP(hipEventSynchronize((hipEvent_t)ev));
  return PSG_OK;
}
int psg_event_elapsed_ms(psg_event start, psg_event stop, float* ms) {
  PSG_REQUIRE(ms, PSG_ERR_INVALID, "psg_event_elapsed_ms: null out");
  PSG_HIP(hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
  return PSG_OK;
}

int psg_stream_wait_event(psg_stream stream, psg_event ev) {
  PSG_REQUIRE(ev, PSG_ERR_INVALID, "psg_stream_wait_event: null event");
  PSG_HIP(hipStreamWaitEvent((hipStream_t)stream, (hipEvent_t)ev, 0));
  return PSG_OK;
}

int psg_fill_synth(void* dptr, uint64_t n, int dtype, uint64_t seed, int mode, double lo,
                   double hi, psg_stream stream) {
  if (n == 0) return PSG_OK;
  PSG_REQUIRE(dptr, PSG_ERR_INVALID, "psg_fill_synth: null pointer");
  PSG_REQUIRE(mode == 0 || mode == 1, PSG_ERR_INVALID, "psg_fill_synth: bad mode %d", mode);
  hipStream_t s = (hipStream_t)stream;
  unsigned g = grid_for(n);
  switch (dtype) {
    case PSG_F32: k_synth<float><<<g, kBlock, 0, s>>>((float*)dptr, n, seed, mode, lo, hi); break;
    case PSG_F64: k_synth<double><<<g, kBlock, 0, s>>>((double*)dptr, n, seed, mode, lo, hi); break;
    case PSG_F16: k_synth<_Float16><<<g, kBlock, 0, s>>>((_Float16*)dptr, n, seed, mode, lo, hi); break;
    case PSG_BF16: k_synth<__bf16><<<g, kBlock, 0, s>>>((__bf16*)dptr, n, seed, mode, lo, hi); break;
    default: set_error("psg_fill_synth: bad dtype %d", dtype); return PSG_ERR_UNSUPPORTED;
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int psg_fill_keys_arith(uint64_t* keys, uint64_t n, uint64_t base, uint64_t step,
                        psg_stream stream) {
  if (n == 0) return PSG_OK;
  PSG_REQUIRE(keys, PSG_ERR_INVALID, "psg_fill_keys_arith: null pointer");
  k_keys_arith<<<grid_for(n), kBlock, 0, (hipStream_t)stream>>>(keys, n, base, step);
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int psg_checksum(const void* dptr, uint64_t nbytes, uint64_t* sum_host, psg_stream stream) {
  PSG_REQUIRE(sum_host, PSG_ERR_INVALID, "psg_checksum: null out");
  PSG_REQUIRE(nbytes % 8 == 0 && ((uintptr_t)dptr & 7u) == 0, PSG_ERR_INVALID,
              "psg_checksum: need 8-B aligned pointer and a multiple of 8 bytes");
  *sum_host = 0;
  if (nbytes == 0) return PSG_OK;
  PSG_REQUIRE(dptr, PSG_ERR_INVALID, "psg_checksum: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const uint64_t n = nbytes / 8;
  const unsigned g = grid_for(n);
  uint64_t* part = nullptr;
  PSG_HIP(hipMalloc((void**)&part, (size_t)g * sizeof(uint64_t)));
  std::vector<uint64_t> host(g);
  k_checksum<<<g, kBlock, 0, s>>>((const uint64_t*)dptr, n, part);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess)
    e = hipMemcpyAsync(host.data(), part, (size_t)g * sizeof(uint64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(part);
  if (e != hipSuccess) return hip_fail(e, "psg_checksum", __FILE__, __LINE__);
  uint64_t h = 0;
  for (uint64_t x : host) h += x;
  *sum_host = h;
  return PSG_OK;
}

int psg_key_list_hash(const uint64_t* keys, uint64_t n, uint64_t* hash_host, psg_stream stream) {
  PSG_REQUIRE(hash_host, PSG_ERR_INVALID, "psg_key_list_hash: null out");
  *hash_host = n;
  if (n == 0) return PSG_OK;
  PSG_REQUIRE(keys, PSG_ERR_INVALID, "psg_key_list_hash: null keys");
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = grid_for(n);
  uint64_t* part = nullptr;
  PSG_HIP(hipMalloc((void**)&part, (size_t)g * sizeof(uint64_t)));
  std::vector<uint64_t> host(g);
  k_key_list_hash<<<g, kBlock, 0, s>>>(keys, n, part);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess)
    e = hipMemcpyAsync(host.data(), part, (size_t)g * sizeof(uint64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(part);
  if (e != hipSuccess) return hip_fail(e, "psg_key_list_hash", __FILE__, __LINE__);
  uint64_t h = n;
  for (uint64_t x : host) h ^= x;
  *hash_host = h;
  return PSG_OK;
}

int psg_verify_synth_sum(const void* dptr, uint64_t n, int dtype, uint64_t seed0, int nseeds,
                         uint64_t offset, double lo, double hi, double scale,
                         uint64_t* mismatches_host, uint64_t* first_bad_host, psg_stream stream) {
  PSG_REQUIRE(mismatches_host, PSG_ERR_INVALID, "psg_verify_synth_sum: null out");
  PSG_REQUIRE(nseeds >= 0, PSG_ERR_INVALID, "psg_verify_synth_sum: nseeds < 0");
  *mismatches_host = 0;
  if (first_bad_host) *first_bad_host = UINT64_MAX;
  if (n == 0) return PSG_OK;
  PSG_REQUIRE(dptr, PSG_ERR_INVALID, "psg_verify_synth_sum: null pointer");
  hipStream_t s = (hipStream_t)stream;
  const unsigned g = grid_for(n);
  uint64_t* part = nullptr;
  PSG_HIP(hipMalloc((void**)&part, (size_t)g * 2 * sizeof(uint64_t)));
  switch (dtype) {
    case PSG_F32:
      k_verify_synth_sum<float><<<g, kBlock, 0, s>>>((const float*)dptr, n, seed0, nseeds, offset, lo, hi, scale, part);
      break;
    case PSG_F64:
      k_verify_synth_sum<double><<<g, kBlock, 0, s>>>((const double*)dptr, n, seed0, nseeds, offset, lo, hi, scale, part);
      break;
    case PSG_F16:
      k_verify_synth_sum<_Float16><<<g, kBlock, 0, s>>>((const _Float16*)dptr, n, seed0, nseeds, offset, lo, hi, scale, part);
      break;
    case PSG_BF16:
      k_verify_synth_sum<__bf16><<<g, kBlock, 0, s>>>((const __bf16*)dptr, n, seed0, nseeds, offset, lo, hi, scale, part);
      break;
    default:
      (void)hipFree(part);
      set_error("psg_verify_synth_sum: bad dtype %d", dtype);
      return PSG_ERR_UNSUPPORTED;
  }
  std::vector<uint64_t> host((size_t)g * 2);
  hipError_t e = hipGetLastError();
  if (e == hipSuccess)
    e = hipMemcpyAsync(host.data(), part, host.size() * sizeof(uint64_t), hipMemcpyDeviceToHost, s);
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  (void)hipFree(part);
  if (e != hipSuccess) return hip_fail(e, "psg_verify_synth_sum", __FILE__, __LINE__);
  uint64_t bad = 0, first = UINT64_MAX;
  for (unsigned b = 0; b < g; ++b) {
    bad += host[2 * b];
    first = host[2 * b + 1] < first ? host[2 * b + 1] : first;
  }
  *mismatches_host = bad;
  if (first_bad_host) *first_bad_host = first;
  return PSG_OK;
}

}  // extern "C"
