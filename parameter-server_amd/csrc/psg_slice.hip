// psg_slice.hip — worker-side key-range slicing and the pull merge.
//
//   psg_server_ranges  PostOffice::GetServerRanges (src/internal/PostOffice.cpp:211-221)
//   psg_slice          KVWorker<V>::DefaultSlicer  (src/ps/KVApp.h:515-574)
//   psg_merge          AddPullCB merge lambda      (src/ps/KVApp.h:673-726)
//
// The slicer's work is ns+1 lower_bounds over the sorted key array.  One
// 256-lane block per boundary runs a 256-ary search: each round every lane
// probes one evenly spaced key and __syncthreads_count gives the bracket, so a
// 10 M-key array takes 3 rounds of one coalesced-free parallel probe instead of
// 24 dependent loads.  With lens, the value bound of each slice is a per-slice
// sum of lens (KVApp.h:565-569), done as a 2-D grid of chunk partial sums.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "psg_internal.h"

namespace psg {

constexpr int kMaxTargets = 64;
struct Targets {
  uint64_t v[kMaxTargets];
  uint64_t hint[kMaxTargets];  // the bound this key array had last time (UINT64_MAX: none)
};

// pos_sys (may be NULL): the same bound into pinned host memory, tagged —
// bits [0, 40) the position, [40, 64) the request's tag — as ONE system-scope
// store per bound, so the host reads each bound as soon as its word carries
// the tag: no copy launch, no stream synchronisation, and no ordering between
// words to rely on (each word validates itself).
constexpr int kPosBits = 40;
__global__ __launch_bounds__(256) void k_bounds(const uint64_t* __restrict__ keys, uint64_t n,
                                                Targets t, uint64_t* __restrict__ pos,
                                                uint64_t* __restrict__ pos_sys, uint64_t tag) {
  const uint64_t target = t.v[blockIdx.x];
  uint64_t lo = 0, hi = n;  // the answer (first index with keys >= target) is in [lo, hi]
  // The bound this array had at its last slice (a worker slices the same key
  // array request after request): confirmed by the two keys around it — one
  // round of loads instead of the search's three under the load of the
  // servers' kernels.  (The keys are sorted, as the slicer requires.)
  const uint64_t h = t.hint[blockIdx.x];
  if (h <= n) {
    __shared__ int s_ok[2];
    if (threadIdx.x < 2) {
      const uint64_t i = h - 1 + threadIdx.x;  // keys[h - 1] < target <= keys[h]
      s_ok[threadIdx.x] = threadIdx.x == 0 ? (h == 0 || keys[i] < target) : (h == n || keys[i] >= target);
    }
    __syncthreads();
    if (s_ok[0] && s_ok[1]) {
      lo = hi = h;
    }
  }
  while (hi - lo > (uint64_t)kBlock) {
    const uint64_t step = (hi - lo + kBlock - 1) / kBlock;
    const uint64_t p = lo + (uint64_t)threadIdx.x * step;
    const int pred = (p < hi) && (keys[p] < target);
    const uint64_t c = (uint64_t)__syncthreads_count(pred);
    if (c == 0) {
      hi = lo;
      break;
    }
    const uint64_t nlo = lo + (c - 1) * step + 1;
    const uint64_t pc = lo + c * step;
    hi = pc < hi ? pc : hi;
    lo = nlo;
  }
  const uint64_t p = lo + threadIdx.x;
  const int pred = (p < hi) && (keys[p] < target);
  const uint64_t c = lo == hi ? 0 : (uint64_t)__syncthreads_count(pred);
  if (threadIdx.x == 0) {
    pos[blockIdx.x] = lo + c;
    if (pos_sys)
      __hip_atomic_store(pos_sys + blockIdx.x, (lo + c) | (tag << kPosBits), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
  }
}

constexpr uint64_t kLenChunk = 16384;  // lens per block

// sums[seg] += sum(lens[pos[seg] + chunk*kLenChunk ...]) for blockIdx = (chunk, seg)
__global__ __launch_bounds__(256) void k_seg_len_sum(const int* __restrict__ lens,
                                                     const uint64_t* __restrict__ pos,
                                                     unsigned long long* __restrict__ sums) {
  const int seg = blockIdx.y;
  const uint64_t b = pos[seg], e = pos[seg + 1];
  const uint64_t c0 = b + (uint64_t)blockIdx.x * kLenChunk;
  if (c0 >= e) return;
  const uint64_t c1 = c0 + kLenChunk < e ? c0 + kLenChunk : e;
  long long acc = 0;
  for (uint64_t i = c0 + threadIdx.x; i < c1; i += kBlock) acc += lens[i];
  // wave reduce then one atomic per wave
  for (int d = 32; d > 0; d >>= 1) acc += __shfl_down(acc, d, 64);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(&sums[seg], (unsigned long long)acc);
}

constexpr int kMaxSegs = 32;
struct SegTable {
  const char* src[kMaxSegs];
  uint64_t count[kMaxSegs];
  uint64_t dst_off[kMaxSegs];
};

// Row y copies segment y into dst at dst_off (elements of type W).
template <typename W>
__global__ __launch_bounds__(256) void k_merge_copy(SegTable t, char* __restrict__ dst) {
  const int y = blockIdx.y;
  const W* __restrict__ src = (const W*)t.src[y];
  W* __restrict__ d = (W*)dst + t.dst_off[y];
  const uint64_t n = t.count[y];
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBlock)
    d[i] = src[i];
}

template <typename W>
static void launch_merge(const SegTable& t, int nseg, uint64_t maxcount, char* dst,
                         hipStream_t st) {
  uint64_t bx = (maxcount + kBlock - 1) / kBlock;
  uint64_t cap = (uint64_t)max_stream_blocks() / (uint64_t)nseg + 1;
  if (bx > cap) bx = cap;
  if (bx == 0) bx = 1;
  k_merge_copy<W><<<dim3((unsigned)bx, (unsigned)nseg), kBlock, 0, st>>>(t, dst);
}

// Per-thread, per-GPU scratch of the slicer: the bounds / length sums in HBM
// and pinned mirrors, so a request costs no allocation (a worker slices every
// Push and Pull).  Kept for the thread's lifetime.
struct SliceScratch {
  uint64_t* pos_dev = nullptr;
  unsigned long long* sums_dev = nullptr;
  uint64_t* pos_host = nullptr;
  uint64_t* pos_map = nullptr;      // tagged bounds, pinned + mapped (k_bounds' pos_sys)
  uint64_t* pos_map_dev = nullptr;
  uint64_t tag = 0;
  int cap = 0;
  // the bounds of the last key arrays sliced (the next slice's hints)
  struct Last {
    const uint64_t* keys = nullptr;
    uint64_t n = 0;
    int nb = 0;
    uint64_t begin0 = 0;
    std::vector<uint64_t> pos;
    uint64_t use = 0;
  } last[8];
  uint64_t clock = 0;
};
static thread_local std::map<int, SliceScratch> t_slice_scratch;

static int get_slice_scratch(int nb, SliceScratch** out) {
  int dev = 0;
  PSG_HIP(hipGetDevice(&dev));
  SliceScratch& s = t_slice_scratch[dev];
  if (s.cap < nb) {
    if (s.pos_dev) (void)hipFree(s.pos_dev);
    if (s.sums_dev) (void)hipFree(s.sums_dev);
    if (s.pos_host) (void)hipHostFree(s.pos_host);
    if (s.pos_map) (void)hipHostFree(s.pos_map);
    const uint64_t tag = s.tag;
    s = SliceScratch();
    s.tag = tag;
    const int cap = std::max(nb, 64);
    PSG_HIP(hipMalloc((void**)&s.pos_dev, cap * sizeof(uint64_t)));
    PSG_HIP(hipMalloc((void**)&s.sums_dev, cap * sizeof(unsigned long long)));
    PSG_HIP(hipHostMalloc((void**)&s.pos_host, cap * sizeof(uint64_t), hipHostMallocDefault));
    PSG_HIP(hipHostMalloc((void**)&s.pos_map, cap * sizeof(uint64_t), hipHostMallocMapped | hipHostMallocCoherent));
    PSG_HIP(hipHostGetDevicePointer((void**)&s.pos_map_dev, s.pos_map, 0));
    memset(s.pos_map, 0, cap * sizeof(uint64_t));
    s.cap = cap;
  }
  *out = &s;
  return PSG_OK;
}

}  // namespace psg

using namespace psg;

extern "C" {

int psg_server_ranges(int num_servers, uint64_t* begins_host, uint64_t* ends_host) {
  PSG_REQUIRE(num_servers > 0 && begins_host && ends_host, PSG_ERR_INVALID,
              "psg_server_ranges: bad arguments");
  const uint64_t kMaxKey = UINT64_MAX;
  for (int i = 0; i < num_servers; ++i) {
    begins_host[i] = kMaxKey / (uint64_t)num_servers * (uint64_t)i;
    ends_host[i] = i != num_servers - 1 ? kMaxKey / (uint64_t)num_servers * (uint64_t)(i + 1) : kMaxKey;
  }
  return PSG_OK;
}

int psg_slice_hint(const uint64_t* keys, uint64_t n, int num_servers, uint64_t begin0, uint64_t* key_pos_host,
                   int* found) {
  PSG_REQUIRE(found && key_pos_host && num_servers > 0, PSG_ERR_INVALID, "psg_slice_hint: bad arguments");
  *found = 0;
  const int nb = num_servers + 1;
  SliceScratch* sc = nullptr;
  PSG_TRY(get_slice_scratch(nb, &sc));
  for (auto& l : sc->last)
    if (l.keys == keys && l.n == n && l.nb == nb && l.begin0 == begin0 && (int)l.pos.size() == nb) {
      for (int i = 0; i < nb; ++i) key_pos_host[i] = l.pos[i];
      l.use = ++sc->clock;
      *found = 1;
      break;
    }
  return PSG_OK;
}

int psg_slice(const uint64_t* keys, uint64_t n, const int* lens, uint64_t num_vals, int num_servers,
              const uint64_t* begins_host, const uint64_t* ends_host, uint64_t* key_pos_host,
              uint64_t* val_pos_host, psg_stream stream) {
  PSG_REQUIRE(num_servers > 0 && begins_host && ends_host && key_pos_host, PSG_ERR_INVALID,
              "psg_slice: bad arguments");
  for (int i = 1; i < num_servers; ++i)
    PSG_REQUIRE(ends_host[i - 1] == begins_host[i], PSG_ERR_INVALID,
                "psg_slice: ranges %d and %d are not adjacent (CHECK_EQ, KVApp.h:531)", i - 1, i);
  const int nb = num_servers + 1;
  if (n == 0) {
    for (int i = 0; i < nb; ++i) key_pos_host[i] = 0;
    if (val_pos_host)
      for (int i = 0; i < nb; ++i) val_pos_host[i] = 0;
    return PSG_OK;
  }
  PSG_REQUIRE(keys, PSG_ERR_INVALID, "psg_slice: null keys");
  uint64_t k = 0;
  if (!lens) {
    k = num_vals / n;
    PSG_REQUIRE(k * n == num_vals, PSG_ERR_INVALID,
                "psg_slice: %llu vals for %llu keys is not a whole value length (KVApp.h:551)",
                (unsigned long long)num_vals, (unsigned long long)n);
  }
  hipStream_t st = (hipStream_t)stream;
  SliceScratch* sc = nullptr;
  PSG_TRY(get_slice_scratch(nb, &sc));
  uint64_t* pos_dev = sc->pos_dev;
  unsigned long long* sums_dev = sc->sums_dev;
  int rc = PSG_OK;
  // the bounds come back tagged through pinned memory (k_bounds' pos_sys),
  // read as soon as every word carries this request's tag; n < 2^40 keys
  static const bool poll_on = [] {  // PSG_SLICE_POLL=0: a copy + stream sync instead (A/B)
    const char* e = getenv("PSG_SLICE_POLL");
    return !(e && atoi(e) == 0);
  }();
  const bool tagged = poll_on && n < (1ull << kPosBits);
  sc->tag = (sc->tag + 1) & ((1ull << (64 - kPosBits)) - 1);
  if (sc->tag == 0) sc->tag = 1;
  const uint64_t tag = sc->tag;
  // hints: this array's bounds at its last slice against the same ranges
  SliceScratch::Last* hint = nullptr;
  for (auto& l : sc->last)
    if (l.keys == keys && l.n == n && l.nb == nb && l.begin0 == begins_host[0]) hint = &l;
  for (int b0 = 0; b0 < nb; b0 += kMaxTargets) {
    Targets t;
    const int cnt = std::min(kMaxTargets, nb - b0);
    for (int j = 0; j < cnt; ++j) {
      const int b = b0 + j;
      t.v[j] = b == 0 ? begins_host[0] : ends_host[b - 1];
      t.hint[j] = hint ? hint->pos[b] : UINT64_MAX;
    }
    k_bounds<<<cnt, kBlock, 0, st>>>(keys, n, t, pos_dev + b0, tagged ? sc->pos_map_dev + b0 : nullptr, tag);
  }
  hipError_t e = hipGetLastError();
  bool got = false;
  if (e == hipSuccess && tagged) {
    // spin for ~2 ms at most (then the stream sync below reports any fault)
    const volatile uint64_t* w = sc->pos_map;
    auto t0 = std::chrono::steady_clock::now();
    for (uint32_t spin = 0; !got; ++spin) {
      int b = 0;
      while (b < nb && (w[b] >> kPosBits) == tag) ++b;
      if (b == nb) {
        std::atomic_thread_fence(std::memory_order_acquire);
        for (int i = 0; i < nb; ++i) key_pos_host[i] = w[i] & ((1ull << kPosBits) - 1);
        got = true;
        break;
      }
      if ((spin & 255) == 255 && std::chrono::steady_clock::now() - t0 > std::chrono::milliseconds(2)) break;
      __builtin_ia32_pause();
    }
  }
  if (e == hipSuccess && !got) {
    e = hipMemcpyAsync(sc->pos_host, pos_dev, nb * sizeof(uint64_t), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e == hipSuccess) memcpy(key_pos_host, sc->pos_host, nb * sizeof(uint64_t));
  }
  if (e != hipSuccess) {
    rc = hip_fail(e, "psg_slice bounds", __FILE__, __LINE__);
  } else {
    // remember these bounds for the next slice of this array (LRU of 8)
    SliceScratch::Last* l = hint;
    if (!l) {
      l = &sc->last[0];
      for (auto& c : sc->last)
        if (c.use < l->use) l = &c;
    }
    l->keys = keys;
    l->n = n;
    l->nb = nb;
    l->begin0 = begins_host[0];
    l->pos.assign(key_pos_host, key_pos_host + nb);
    l->use = ++sc->clock;
  }
  if (rc != PSG_OK) {
  } else if (key_pos_host[num_servers] != n) {
    // a key at or above the last range's end: CHECK_EQ(pos[n], send.keys.size()),
    // KVApp.h:544.  (Keys below ranges[0].begin are dropped, as in the
    // reference; with GetServerRanges ranges[0].begin is 0.)
    set_error("psg_slice: %llu of %llu keys fall above the last server range (KVApp.h:544)",
              (unsigned long long)(n - key_pos_host[num_servers]), (unsigned long long)n);
    rc = PSG_ERR_INVALID;
  } else if (val_pos_host) {
    if (!lens) {
      for (int i = 0; i < nb; ++i) val_pos_host[i] = key_pos_host[i] * k;
    } else {
      uint64_t maxseg = 0;
      for (int i = 0; i < num_servers; ++i)
        maxseg = std::max<uint64_t>(maxseg, key_pos_host[i + 1] - key_pos_host[i]);
      e = hipMemsetAsync(sums_dev, 0, num_servers * sizeof(unsigned long long), st);
      if (e == hipSuccess && maxseg > 0) {
        dim3 g((unsigned)((maxseg + kLenChunk - 1) / kLenChunk), (unsigned)num_servers);
        k_seg_len_sum<<<g, kBlock, 0, st>>>(lens, pos_dev, sums_dev);
        e = hipGetLastError();
      }
      std::vector<unsigned long long> sums(num_servers, 0);
      if (e == hipSuccess)
        e = hipMemcpyAsync(sums.data(), sums_dev, num_servers * sizeof(unsigned long long),
                           hipMemcpyDeviceToHost, st);
      if (e == hipSuccess) e = hipStreamSynchronize(st);
      if (e != hipSuccess) {
        rc = hip_fail(e, "psg_slice lens", __FILE__, __LINE__);
      } else {
        // the reference's running val_begin/val_end start at 0 (KVApp.h:548)
        val_pos_host[0] = 0;
        for (int i = 0; i < num_servers; ++i) val_pos_host[i + 1] = val_pos_host[i] + sums[i];
      }
    }
  }
  return rc;
}

int psg_merge(psg_segment* segs, int nsegs, int elem_size, void* dst, uint64_t dst_count,
              psg_stream stream) {
  PSG_REQUIRE(nsegs >= 0 && (nsegs == 0 || segs), PSG_ERR_INVALID, "psg_merge: bad segments");
  PSG_REQUIRE(elem_size == 1 || elem_size == 2 || elem_size == 4 || elem_size == 8 ||
                  elem_size == 16,
              PSG_ERR_INVALID, "psg_merge: elem_size %d", elem_size);
  uint64_t total = 0;
  for (int i = 0; i < nsegs; ++i) {
    PSG_REQUIRE(segs[i].count == 0 || segs[i].vals, PSG_ERR_INVALID, "psg_merge: null segment %d", i);
    total += segs[i].count;
  }
  PSG_REQUIRE(total == dst_count, PSG_ERR_INVALID,
              "psg_merge: replies hold %llu values, expected %llu (lost some servers?, KVApp.h:691)",
              (unsigned long long)total, (unsigned long long)dst_count);
  if (total == 0) return PSG_OK;
  PSG_REQUIRE(dst, PSG_ERR_INVALID, "psg_merge: null dst");
  // order replies by first key (KVApp.h:694-696)
  std::vector<psg_segment> v(segs, segs + nsegs);
  std::stable_sort(v.begin(), v.end(),
                   [](const psg_segment& a, const psg_segment& b) { return a.first_key < b.first_key; });
  hipStream_t st = (hipStream_t)stream;
  uint64_t off = 0;
  for (size_t b0 = 0; b0 < v.size(); b0 += kMaxSegs) {
    SegTable t;
    int cnt = 0;
    uint64_t maxcount = 0;
    bool vec16 = psg::aligned16(dst);
    for (size_t j = b0; j < v.size() && cnt < kMaxSegs; ++j) {
      t.src[cnt] = (const char*)v[j].vals;
      t.count[cnt] = v[j].count;
      t.dst_off[cnt] = off;
      const uint64_t bytes = v[j].count * elem_size;
      vec16 = vec16 && psg::aligned16(v[j].vals) && ((off * elem_size) % 16 == 0) && (bytes % 16 == 0);
      off += v[j].count;
      maxcount = std::max(maxcount, v[j].count);
      ++cnt;
    }
    if (vec16) {
      // re-express in 16-byte units
      for (int j = 0; j < cnt; ++j) {
        t.count[j] = t.count[j] * elem_size / 16;
        t.dst_off[j] = t.dst_off[j] * elem_size / 16;
      }
      launch_merge<u32x4>(t, cnt, maxcount * elem_size / 16, (char*)dst, st);
    } else {
      switch (elem_size) {
        case 1: launch_merge<uint8_t>(t, cnt, maxcount, (char*)dst, st); break;
        case 2: launch_merge<uint16_t>(t, cnt, maxcount, (char*)dst, st); break;
        case 4: launch_merge<uint32_t>(t, cnt, maxcount, (char*)dst, st); break;
        case 8: launch_merge<uint64_t>(t, cnt, maxcount, (char*)dst, st); break;
        default: launch_merge<u32x4>(t, cnt, maxcount, (char*)dst, st); break;
      }
    }
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

}  // extern "C"
