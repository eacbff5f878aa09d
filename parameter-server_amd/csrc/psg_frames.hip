// psg_frames.hip — a run of queued Push requests on one key list, applied in
// one pass.
//
// The reference server drains its queue one message at a time
// (src/internal/Customer.cpp:52-70) and applies each Push with
// `store[key] += vals[i]` (src/ps/KVApp.h:446-454).  When k Pushes on the same
// key list sit in the queue one behind the other (nw workers of a BSP round,
// test_kv_app_multi_workers.cpp's customers), the store ends as
//     s_i = (((s_i + v_0[i]) + v_1[i]) + ...) + v_{k-1}[i]
// and that is exactly what one pass computes: the store is read and written
// once instead of k times, and the k frames are added in arrival order, so the
// result is bit for bit the reference's (every dtype rounds after each add,
// as k separate requests do).  HBM bytes per key, f32:
//     k requests          k * (vals 4 + store 8)        = 12k
//     one pass            store 8 + vals 4k             = 8 + 4k
// plus, for full key lists, the keys: every list must be read to know that it
// IS the same list (k_frames_check: 8 per list, plus the reference it is
// compared with).  psg_store.hip (psg_store_push_frames) drives the kernels:
//   identity  the lists equal a stretch of the store's keys K[D, D + n):
//             k_frames_base finds D, k_frames_check compares every list with
//             it, k_frames_apply adds the frames to V[D, D + n)
//             (16 + 12k B / key, against 28k for k identity requests);
//   slots     lists 1..k-1 equal list 0, resolved to slots once:
//             k_frames_check, then k_frames_slots;
//   cached    LR key caching names the list by its hash: no keys at all,
//             k_frames_apply on a stretch of slots (8 + 4k) or k_frames_slots.
// A check that fails makes the apply write nothing and raise a host flag; the
// requests then run one after the other, so the store always sees exactly the
// reference's sequence.
#include <cstdlib>

#include "psg_internal.h"

namespace psg {

namespace {

struct FramePtrs {
  const void* p[kMaxFrames];
};

template <int NT>
__device__ __forceinline__ u32x4 ld16(const u32x4* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p);
  else return *p;
}
template <int NT>
__device__ __forceinline__ void st16(u32x4* p, u32x4 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p);
  else *p = v;
}

// The base of a stretch: D = lower_bound(K, q0[0]) when K[D] == q0[0] and n
// slots fit from D, else UINT64_MAX.  One wave.
__global__ __launch_bounds__(64) void k_frames_base(const uint64_t* __restrict__ K, uint64_t S,
                                                    const uint64_t* __restrict__ q0, uint64_t n,
                                                    uint64_t* __restrict__ base) {
  const uint64_t key = q0[0];
  const uint64_t D = lower_bound_wave(K, S, key);
  const bool ok = D < S && K[D] == key && n <= S - D;
  if (threadIdx.x == 0) *base = ok ? D : UINT64_MAX;
}

// Every list j in [j0, k) equals ref[off + i] for i < n, where off = *base
// (base == NULL: 0).  Two keys a lane per 16-B load of every list when the
// arrays are 16-B aligned (uniform), then the scalar rest; every list's load
// of one pair is in flight together.  Any mismatch (or a stretch that was not
// found) writes seq into *rej.  Bytes: the reference 8 + 8 per list compared.
template <int MAXF>
__global__ __launch_bounds__(256) void k_frames_check(const uint64_t* __restrict__ ref,
                                                      const uint64_t* __restrict__ base, FramePtrs keys, int j0,
                                                      int k, uint64_t n, int vec, int* __restrict__ rej, int seq) {
  int bad = 0;
  uint64_t off = 0;
  if (base) {
    off = *base;
    if (off == UINT64_MAX) bad = 1;
  }
  if (!bad) {
    const uint64_t* r = ref + off;
    const uint64_t stride = (uint64_t)gridDim.x * kBlock;
    const uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
    uint64_t done = 0;
    if (vec && (off & 1) == 0) {
      const uint64_t np = n / 2;
      done = np * 2;
      for (uint64_t i = gid; i < np; i += stride) {
        const u64x2 a = *reinterpret_cast<const u64x2*>(r + 2 * i);
        u64x2 c[MAXF];
#pragma unroll
        for (int j = 0; j < MAXF; ++j)
          if (j >= j0 && j < k) c[j] = __builtin_nontemporal_load(reinterpret_cast<const u64x2*>(keys.p[j]) + i);
#pragma unroll
        for (int j = 0; j < MAXF; ++j)
          if (j >= j0 && j < k && (c[j][0] != a[0] || c[j][1] != a[1])) bad = 1;
      }
    }
    for (uint64_t i = done + gid; i < n; i += stride) {
      const uint64_t a = r[i];
#pragma unroll
      for (int j = 0; j < MAXF; ++j)
        if (j >= j0 && j < k && static_cast<const uint64_t*>(keys.p[j])[i] != a) bad = 1;
    }
  }
  if (__ballot(bad) && (threadIdx.x & 63) == 0) *rej = seq;
}

// The gate every applying kernel reads first: a failed check (or no stretch)
// means nothing is written, and the host hears of it through *flag (pinned).
__device__ __forceinline__ bool frames_gated(const uint64_t* base, const int* rej, int seq, int* flag,
                                             uint64_t* off) {
  *off = 0;
  bool bad = false;
  if (base) {
    *off = *base;
    bad = *off == UINT64_MAX;
  }
  if (rej && *rej == seq) bad = true;
  if (bad && blockIdx.x == 0 && threadIdx.x == 0) *flag = 1;
  return bad;
}

// store[off + i] = ((store[off + i] + v_0[i]) + v_1[i]) + ... for i < n, with
// off = *base (base == NULL: 0): one 16-B store vector and every frame's 16-B
// vector in flight per lane (MAXF registers of 16 B), the adds in frame order.
// The frames stream non-temporally (read once); the store keeps the cache
// policy of a Push (NT bit 1: past the Infinity Cache, non-temporal too).
template <int DT, int MAXF, int NT>
__global__ __launch_bounds__(256) void k_frames_apply(typename Elem<DT>::T* __restrict__ store, FramePtrs vals, int k,
                                                      uint64_t n, int vec, const uint64_t* __restrict__ base,
                                                      const int* __restrict__ rej, int seq, int* __restrict__ flag) {
  using E = Elem<DT>;
  using T = typename E::T;
  uint64_t off;
  if (frames_gated(base, rej, seq, flag, &off)) return;
  T* st = store + off;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  uint64_t done = 0;
  if (vec && (off % E::kVec) == 0) {
    const uint64_t nv = n / E::kVec;
    done = nv * E::kVec;
    u32x4* sv = reinterpret_cast<u32x4*>(st);
    for (uint64_t i = gid; i < nv; i += stride) {
      u32x4 v[MAXF];
      u32x4 s = ld16<(NT >> 1) & 1>(sv + i);
#pragma unroll
      for (int j = 0; j < MAXF; ++j)
        if (j < k) v[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(vals.p[j]) + i);
#pragma unroll
      for (int j = 0; j < MAXF; ++j)
        if (j < k) s = E::add(s, v[j]);
      st16<(NT >> 1) & 1>(sv + i, s);
    }
  }
  for (uint64_t i = done + gid; i < n; i += stride) {
    T s = st[i];
#pragma unroll
    for (int j = 0; j < MAXF; ++j)
      if (j < k) s = E::add1(s, static_cast<const T*>(vals.p[j])[i]);
    st[i] = s;
  }
}

// store[slots[i]] = ((store[slots[i]] + v_0[i]) + ...) for i < n (slots unique:
// psg_store_resolve's lists are).  4-B values: four slots a lane from one 16-B
// load, every frame's 16-B vector in flight, and one 16-B store read-modify-
// write when the four slots are consecutive and aligned (a cached list that
// covers a stretch); else four scalar ones.  Bytes: slot 4 + store 8 + 4k.
template <int DT, int MAXF>
__global__ __launch_bounds__(256) void k_frames_slots(typename Elem<DT>::T* __restrict__ store,
                                                      const uint32_t* __restrict__ slots, FramePtrs vals, int k,
                                                      uint64_t n, int vec, const int* __restrict__ rej, int seq,
                                                      int* __restrict__ flag) {
  using E = Elem<DT>;
  using T = typename E::T;
  uint64_t off;
  if (frames_gated(nullptr, rej, seq, flag, &off)) return;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t gid = (uint64_t)blockIdx.x * kBlock + threadIdx.x;
  uint64_t done = 0;
  if constexpr (sizeof(T) == 4) {
    if (vec) {
      typedef T t4 __attribute__((ext_vector_type(4)));
      const uint64_t nq = n / 4;
      done = nq * 4;
      for (uint64_t q = gid; q < nq; q += stride) {
        const u32x4 sl = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(slots) + q);
        u32x4 v[MAXF];
#pragma unroll
        for (int j = 0; j < MAXF; ++j)
          if (j < k) v[j] = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(vals.p[j]) + q);
        const uint32_t p0 = sl[0];
        if (sl[1] == p0 + 1 && sl[2] == p0 + 2 && sl[3] == p0 + 3 && (p0 & 3) == 0) {
          u32x4* sp = reinterpret_cast<u32x4*>(store + p0);
          u32x4 s = *sp;
#pragma unroll
          for (int j = 0; j < MAXF; ++j)
            if (j < k) s = E::add(s, v[j]);
          *sp = s;
        } else {
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            T s = store[sl[e]];
#pragma unroll
            for (int j = 0; j < MAXF; ++j)
              if (j < k) s = E::add1(s, __builtin_bit_cast(t4, v[j])[e]);
            store[sl[e]] = s;
          }
        }
      }
    }
  }
  for (uint64_t i = done + gid; i < n; i += stride) {
    const uint32_t p = slots[i];
    T s = store[p];
#pragma unroll
    for (int j = 0; j < MAXF; ++j)
      if (j < k) s = E::add1(s, static_cast<const T*>(vals.p[j])[i]);
    store[p] = s;
  }
}

unsigned frames_grid(uint64_t units, int bpc) {
  const uint64_t cap = (uint64_t)(max_stream_blocks() / 8) * (uint64_t)bpc;
  uint64_t b = (units + kBlock - 1) / kBlock;
  if (b > cap) b = cap;
  return b ? (unsigned)b : 1u;
}

// frames kept in registers: the smallest instantiation that holds k
template <typename F>
int by_maxf(int k, F&& f) {
  if (k <= 2) return f(std::integral_constant<int, 2>());
  if (k <= 4) return f(std::integral_constant<int, 4>());
  if (k <= 8) return f(std::integral_constant<int, 8>());
  return f(std::integral_constant<int, 16>());
}

bool all_aligned(const void* const* p, int k) {
  for (int j = 0; j < k; ++j)
    if (!aligned16(p[j])) return false;
  return true;
}

// Blocks of 256 per CU of the frame kernels: 8 for a run over at most 64 MiB
// of store values, 2 past it — k = 8 frames on 64 M floats took 437 us at 2
// against 452-474 at 4-16, on 10 M 67-69 us at any (profiles/r5_frames_bpc_sweep.txt).
// PSG_FRAMES_BPC (A/B) sets it for every size.
int frames_bpc(uint64_t store_bytes) {
  static const int v = [] {
    const char* e = getenv("PSG_FRAMES_BPC");
    const int b = e ? atoi(e) : 0;
    return b >= 1 && b <= 16 ? b : 0;
  }();
  if (v) return v;
  return store_bytes > (64ull << 20) ? 2 : 8;
}

template <int DT>
int apply_t(void* store_vals, uint64_t store_elems, const void* const* vals, int k, uint64_t n,
            const uint64_t* base, const int* rej, int seq, int* flag, hipStream_t st) {
  using T = typename Elem<DT>::T;
  FramePtrs f = {};
  for (int j = 0; j < k; ++j) f.p[j] = vals[j];
  const int vec = aligned16(store_vals) && all_aligned(vals, k) ? 1 : 0;
  // past the Infinity Cache the store is read and written once: non-temporal
  const int nt = (uint64_t)sizeof(T) * store_elems > (512ull << 20) ? 2 : 0;
  const unsigned g = frames_grid(vec ? n / Elem<DT>::kVec : n, frames_bpc(n * sizeof(T)));
  return by_maxf(k, [&](auto mc) -> int {
    constexpr int M = decltype(mc)::value;
    if (nt)
      k_frames_apply<DT, M, 2><<<g, kBlock, 0, st>>>((T*)store_vals, f, k, n, vec, base, rej, seq, flag);
    else
      k_frames_apply<DT, M, 0><<<g, kBlock, 0, st>>>((T*)store_vals, f, k, n, vec, base, rej, seq, flag);
    PSG_HIP(hipGetLastError());
    return PSG_OK;
  });
}

template <int DT>
int slots_t(void* store_vals, const uint32_t* slots, const void* const* vals, int k, uint64_t n, const int* rej,
            int seq, int* flag, hipStream_t st) {
  using T = typename Elem<DT>::T;
  FramePtrs f = {};
  for (int j = 0; j < k; ++j) f.p[j] = vals[j];
  const int vec = sizeof(T) == 4 && aligned16(slots) && all_aligned(vals, k) ? 1 : 0;
  const unsigned g = frames_grid(vec ? n / 4 : n, frames_bpc(0));
  return by_maxf(k, [&](auto mc) -> int {
    constexpr int M = decltype(mc)::value;
    k_frames_slots<DT, M><<<g, kBlock, 0, st>>>((T*)store_vals, slots, f, k, n, vec, rej, seq, flag);
    PSG_HIP(hipGetLastError());
    return PSG_OK;
  });
}

}  // namespace

int frames_base(const uint64_t* K, uint64_t S, const uint64_t* q0, uint64_t n, uint64_t* base, hipStream_t st) {
  k_frames_base<<<1, 64, 0, st>>>(K, S, q0, n, base);
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int frames_check(const uint64_t* ref, const uint64_t* base, const uint64_t* const* keys, int j0, int k, uint64_t n,
                 int* rej, int seq, hipStream_t st) {
  if (j0 >= k) return PSG_OK;
  FramePtrs f = {};
  bool vec = aligned16(ref);
  for (int j = 0; j < k; ++j) {
    f.p[j] = keys[j];
    if (j >= j0) vec = vec && aligned16(keys[j]);
  }
  const unsigned g = frames_grid(vec ? n / 2 : n, frames_bpc(0));
  return by_maxf(k, [&](auto mc) -> int {
    constexpr int M = decltype(mc)::value;
    k_frames_check<M><<<g, kBlock, 0, st>>>(ref, base, f, j0, k, n, vec ? 1 : 0, rej, seq);
    PSG_HIP(hipGetLastError());
    return PSG_OK;
  });
}

int frames_apply(int dtype, void* store_vals, uint64_t store_elems, const void* const* vals, int k, uint64_t n,
                 const uint64_t* base, const int* rej, int seq, int* flag, hipStream_t st) {
  switch (dtype) {
    case PSG_F32: return apply_t<PSG_F32>(store_vals, store_elems, vals, k, n, base, rej, seq, flag, st);
    case PSG_F64: return apply_t<PSG_F64>(store_vals, store_elems, vals, k, n, base, rej, seq, flag, st);
    case PSG_F16: return apply_t<PSG_F16>(store_vals, store_elems, vals, k, n, base, rej, seq, flag, st);
    case PSG_BF16: return apply_t<PSG_BF16>(store_vals, store_elems, vals, k, n, base, rej, seq, flag, st);
    default: set_error("unsupported dtype %d", dtype); return PSG_ERR_UNSUPPORTED;
  }
}

int frames_slots(int dtype, void* store_vals, const uint32_t* slots, const void* const* vals, int k, uint64_t n,
                 const int* rej, int seq, int* flag, hipStream_t st) {
  switch (dtype) {
    case PSG_F32: return slots_t<PSG_F32>(store_vals, slots, vals, k, n, rej, seq, flag, st);
    case PSG_F64: return slots_t<PSG_F64>(store_vals, slots, vals, k, n, rej, seq, flag, st);
    case PSG_F16: return slots_t<PSG_F16>(store_vals, slots, vals, k, n, rej, seq, flag, st);
    case PSG_BF16: return slots_t<PSG_BF16>(store_vals, slots, vals, k, n, rej, seq, flag, st);
    default: set_error("unsupported dtype %d", dtype); return PSG_ERR_UNSUPPORTED;
  }
}

}  // namespace psg
