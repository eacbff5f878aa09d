// psg_dense.hip — the element-wise accumulate kernels of the value store.
//
// Reference loop (src/ps/KVApp.h:446-454, KVServerDefaultHandle::operator()):
//     for i < n:  if push: store[key_i] += vals[i];  if pull: res.vals[i] = store[key_i];
// For a dense request the keys are consecutive, so key_i -> slot off + i and
// the loop is a pure streaming op, bound by HBM:
//     PUSH       read vals + read store + write store         12 B / f32 element
//     PULL       read store + write out                         8 B / f32 element
//     PUSH|PULL  read vals + read store + write store + write out 16 B / f32 element
// No MFMA (0 flops of reuse).  Every lane moves 16 B per access (one
// global_load_dwordx4, 1 KiB per wave instruction), each thread keeps U such
// vectors of every stream in flight, blocks grid-stride over 256*U-vector
// tiles (cdna_hip_programming.md Guidelines 11, 13, Appendix B 'Element-wise').
// The once-read request stream (vals) and the write-only reply stream (out)
// use non-temporal loads/stores (+20 % over default policy in the sweep); the
// store keeps the default policy while it can live in the Infinity Cache.
// Measured HBM traffic of the Push kernel = 1.00003 x the 12 B/elem algorithmic
// bytes (profiles/pmc_push_traffic.json): no re-reads.
#include <cstdlib>
#include <type_traits>

#include "psg_internal.h"

namespace psg {

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

// Vector kernel over nvec 16-byte vectors.  OP bits: PSG_PUSH, PSG_PULL.
// BS threads per block (256, or 512 / 1024 for the shapes dense_cfg picks).
template <int DT, int OP, int U, int NT, int BS = 256>
__global__ __launch_bounds__(BS) void k_dense_vec(u32x4* __restrict__ store,
                                                  const u32x4* __restrict__ vals,
                                                  u32x4* __restrict__ out, uint64_t nvec) {
  using E = Elem<DT>;
  constexpr int kBlock = BS;
  const uint64_t tile = (uint64_t)kBlock * U;
  const uint64_t gstride = (uint64_t)gridDim.x * tile;
  for (uint64_t base = (uint64_t)blockIdx.x * tile + threadIdx.x; base < nvec; base += gstride) {
    u32x4 s[U], v[U];
    if (base + (uint64_t)(U - 1) * kBlock < nvec) {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if constexpr ((OP & PSG_PUSH) != 0) v[u] = ld16<NT & 1>(vals + i);
        s[u] = ld16<(NT >> 1) & 1>(store + i);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if constexpr ((OP & PSG_PUSH) != 0) {
          s[u] = E::add(s[u], v[u]);
          st16<(NT >> 1) & 1>(store + i, s[u]);
        }
        if constexpr ((OP & PSG_PULL) != 0) st16<NT & 1>(out + i, s[u]);
      }
    } else {
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nvec) {
          if constexpr ((OP & PSG_PUSH) != 0) v[u] = ld16<NT & 1>(vals + i);
          s[u] = ld16<(NT >> 1) & 1>(store + i);
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const uint64_t i = base + (uint64_t)u * kBlock;
        if (i < nvec) {
          if constexpr ((OP & PSG_PUSH) != 0) {
            s[u] = E::add(s[u], v[u]);
            st16<(NT >> 1) & 1>(store + i, s[u]);
          }
          if constexpr ((OP & PSG_PULL) != 0) st16<NT & 1>(out + i, s[u]);
        }
      }
    }
  }
}

// Element kernel: misaligned operands and the sub-16-byte tail.
template <int DT, int OP>
__global__ __launch_bounds__(256) void k_dense_elem(typename Elem<DT>::T* __restrict__ store,
                                                    const typename Elem<DT>::T* __restrict__ vals,
                                                    typename Elem<DT>::T* __restrict__ out,
                                                    uint64_t n) {
  using E = Elem<DT>;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBlock) {
    typename E::T s = store[i];
    if constexpr ((OP & PSG_PUSH) != 0) {
      s = E::add1(s, vals[i]);
      store[i] = s;
    }
    if constexpr ((OP & PSG_PULL) != 0) out[i] = s;
  }
}

// Slot-indexed request: the gather/scatter form used by the SORTED store and
// by cached slot lists.  UINT32_MAX slots are skipped (a pull yields 0).
template <int DT, int OP>
__global__ __launch_bounds__(256) void k_slots(typename Elem<DT>::T* __restrict__ store,
                                               const uint32_t* __restrict__ slots,
                                               const typename Elem<DT>::T* __restrict__ vals,
                                               typename Elem<DT>::T* __restrict__ out, uint64_t n) {
  using E = Elem<DT>;
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n;
       i += (uint64_t)gridDim.x * kBlock) {
    const uint32_t p = slots[i];
    typename E::T s = (typename E::T)0.0f;
    if (p != 0xffffffffu) {
      s = store[p];
      if constexpr ((OP & PSG_PUSH) != 0) {
        s = E::add1(s, vals[i]);
        store[p] = s;
      }
    }
    if constexpr ((OP & PSG_PULL) != 0) out[i] = s;
  }
}

// The same for 4-byte values, four slots per lane: 16-B loads of the slots and
// the request values, 16-B stores of the replies, and — when the four slots
// are consecutive and 16-B aligned (a cached slot list that covers a stretch
// of the store, the steady state of LR key caching) — one 16-B load and store
// of the store values instead of four.  U groups of four in flight per lane.
// Bytes per key: slot 4 + value 4 + store 4 read / 4 written (+ reply 4).
// Slots must be unique within a request (psg_store_resolve's lists are).
template <int DT, int OP, int U>
__global__ __launch_bounds__(256) void k_slots_vec(typename Elem<DT>::T* __restrict__ store,
                                                   const u32x4* __restrict__ slots,
                                                   const u32x4* __restrict__ vals,
                                                   u32x4* __restrict__ out, uint64_t nq) {
  using T = typename Elem<DT>::T;
  static_assert(sizeof(T) == 4, "4-byte values");
  const uint64_t stride = (uint64_t)gridDim.x * kBlock * U;
  for (uint64_t j0 = (uint64_t)blockIdx.x * kBlock * U + threadIdx.x; j0 < nq; j0 += stride) {
    u32x4 sl[U], v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = j0 + (uint64_t)u * kBlock;
      if (j < nq) {
        sl[u] = __builtin_nontemporal_load(slots + j);
        if constexpr ((OP & PSG_PUSH) != 0) v[u] = __builtin_nontemporal_load(vals + j);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t j = j0 + (uint64_t)u * kBlock;
      if (j >= nq) continue;
      // whole-vector bit casts only: __builtin_bit_cast of a vector ELEMENT
      // (x[k]) reads element 0 with this compiler, so elements are taken from
      // vectors of T
      typedef T t4 __attribute__((ext_vector_type(4)));
      t4 o = {(T)0.0f, (T)0.0f, (T)0.0f, (T)0.0f};
      t4 vv = {(T)0.0f, (T)0.0f, (T)0.0f, (T)0.0f};
      if constexpr ((OP & PSG_PUSH) != 0) vv = __builtin_bit_cast(t4, v[u]);
      const uint32_t p0 = sl[u][0];
      if (p0 != 0xffffffffu && sl[u][1] == p0 + 1 && sl[u][2] == p0 + 2 && sl[u][3] == p0 + 3 && (p0 & 3) == 0) {
        u32x4* sp = reinterpret_cast<u32x4*>(store + p0);
        t4 x = __builtin_bit_cast(t4, *sp);
        if constexpr ((OP & PSG_PUSH) != 0) {
          x = x + vv;
          *sp = __builtin_bit_cast(u32x4, x);
        }
        o = x;
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          const uint32_t p = sl[u][k];
          T y = (T)0.0f;
          if (p != 0xffffffffu) {
            y = store[p];
            if constexpr ((OP & PSG_PUSH) != 0) {
              y = y + vv[k];
              store[p] = y;
            }
          }
          o[k] = y;
        }
      }
      if constexpr ((OP & PSG_PULL) != 0) __builtin_nontemporal_store(__builtin_bit_cast(u32x4, o), out + j);
    }
  }
}

// ---- tuning knobs ------------------------------------------------------------
// Defaults from the MI355X sweep (profiles/r1_sweep_dense_{64M,256M}.json):
// 2 vectors per stream in flight per lane, 2 blocks of 256 per CU (512 blocks
// grid-striding), non-temporal request/reply streams.  Once the store itself
// is well past the 256 MiB Infinity Cache (> 512 MiB) its loads and stores go
// non-temporal too (nt = 3): at 256 M floats that was +3..6 % on the Pull.
// PSG_DENSE_{UNROLL,NT,BPC} override them, for tools/sweep_dense.py only.
struct DenseCfg {
  int unroll = 2;
  int nt = -1;  // -1: by store size
  int blocks_per_cu = 2;
  int block = 256;  // threads per block: 256, 512 or 1024 (PSG_DENSE_BLOCK)
};
static DenseCfg dense_cfg() {
  static DenseCfg cfg = [] {
    DenseCfg c;
    if (const char* e = getenv("PSG_DENSE_UNROLL")) c.unroll = atoi(e);
    if (const char* e = getenv("PSG_DENSE_NT")) c.nt = atoi(e);
    if (const char* e = getenv("PSG_DENSE_BPC")) c.blocks_per_cu = atoi(e);
    if (const char* e = getenv("PSG_DENSE_BLOCK")) c.block = atoi(e);
    if (c.block != 256 && c.block != 512 && c.block != 1024) c.block = 256;
    if (c.unroll != 1 && c.unroll != 2 && c.unroll != 4 && c.unroll != 8) c.unroll = 2;
    if (c.blocks_per_cu < 1 || c.blocks_per_cu > 32) c.blocks_per_cu = 2;
    if (c.nt < -1 || c.nt > 3) c.nt = -1;
    return c;
  }();
  return cfg;
}
// PSG_DENSE_PULL_{UNROLL,NT,BPC}: the same knobs for the Pull alone (sweeps).
static DenseCfg dense_pull_override() {
  static DenseCfg cfg = [] {
    DenseCfg c;
    c.unroll = c.blocks_per_cu = 0;
    c.nt = -1;
    if (const char* e = getenv("PSG_DENSE_PULL_UNROLL")) c.unroll = atoi(e);
    if (const char* e = getenv("PSG_DENSE_PULL_NT")) c.nt = atoi(e);
    if (const char* e = getenv("PSG_DENSE_PULL_BPC")) c.blocks_per_cu = atoi(e);
    if (c.unroll != 1 && c.unroll != 2 && c.unroll != 4 && c.unroll != 8) c.unroll = 0;
    if (c.blocks_per_cu < 1 || c.blocks_per_cu > 32) c.blocks_per_cu = 0;
    if (c.nt < -1 || c.nt > 3) c.nt = -1;
    return c;
  }();
  return cfg;
}
static DenseCfg dense_cfg_for_size(uint64_t store_bytes, int op);
static DenseCfg dense_cfg_for(uint64_t store_bytes, int op) {
  DenseCfg c = dense_cfg_for_size(store_bytes, op);
  if (op == PSG_PULL) {
    const DenseCfg& o = dense_pull_override();
    if (o.unroll) c.unroll = o.unroll;
    if (o.nt >= 0) c.nt = o.nt;
    if (o.blocks_per_cu) c.blocks_per_cu = o.blocks_per_cu;
  }
  return c;
}
static DenseCfg dense_cfg_for_size(uint64_t store_bytes, int op) {
  DenseCfg c = dense_cfg();
  if (c.nt >= 0) return c;  // explicit sweep settings
  if (store_bytes <= (64ull << 20)) {
    // a request of at most 64 MiB (a 10 M-key cached stretch, an LR model):
    // 1 vector per lane at 8 blocks/CU — more waves in flight over the short
    // launch's ramp and tail.  10 M floats Push+Pull, 4 interleaved rounds:
    // 2,454-2,517 GB/s against 2,419-2,435 at 2 x 2/CU
    // (profiles/r3_ab_dense_shape_10M.txt)
    // (PSG_DENSE_UNROLL / PSG_DENSE_BPC, when set, still win: A/B runs)
    // Round 4: the same 2048 threads per CU as 4 blocks of 512
    // (tools/probe_push_small.hip, 10 M integer-valued floats, 4 interleaved
    // rounds, one process): Push 21.8 vs 23.0 us, an unperturbed Push+Pull
    // step 31.3 vs 32.7 us, the best of 11 shapes (profiles/r4_probe_push_shapes.txt)
    // — half the workgroups to dispatch and retire on a ~20 us launch.  (The
    // same probe on all-zero buffers ran ~20 % faster for every shape: the
    // probes and the bench use real values.)
    static const bool env_u = getenv("PSG_DENSE_UNROLL") != nullptr;
    static const bool env_b = getenv("PSG_DENSE_BPC") != nullptr;
    static const bool env_k = getenv("PSG_DENSE_BLOCK") != nullptr;
    // PSG_DENSE_SMALL_NT / PSG_DENSE_MID_NT: this class's Push / the next
    // class's cache policy bits (A/B)
    static const int small_nt = [] {
      const char* e = getenv("PSG_DENSE_SMALL_NT");
      const int v = e ? atoi(e) : -1;
      return v >= 0 && v <= 3 ? v : 1;
    }();
    c.nt = (op & PSG_PUSH) ? small_nt : 1;
    if (!env_u) c.unroll = 1;
    if (!env_b) c.blocks_per_cu = 4;
    if (!env_k) c.block = 512;
  } else if (store_bytes <= (512ull << 20)) {
    static const int mid_nt = [] {
      const char* e = getenv("PSG_DENSE_MID_NT");
      const int v = e ? atoi(e) : -1;
      return v >= 0 && v <= 3 ? v : 1;
    }();
    c.nt = mid_nt;
  } else {
    // past the Infinity Cache, all non-temporal.  Pull (the Pull-only sweep
    // profiles/r1_sweep_pull_256M.json): 1 vector per lane at 4 blocks/CU
    // (0.80 of 8 TB/s, up from 0.72 with 2 vectors per lane).  Push: 2 vectors
    // per lane at 2 blocks/CU — consecutive Pushes into one store (several
    // workers in a row) run at 0.770 of HBM against 0.686 with 1 vector
    // (profiles/r2_sweep_b2b_push_256M.json), for 0.774 vs 0.786 when a Pull
    // sits between them (profiles/r1_sweep_dense_256M.json)
    c.nt = 3;
    if (op == PSG_PULL) {
      c.unroll = 1;
      c.blocks_per_cu = 4;
    } else {
      c.unroll = 2;
      c.blocks_per_cu = 2;
    }
  }
  return c;
}

static unsigned stream_grid(uint64_t units, uint64_t per_block, int bpc) {
  int cus = max_stream_blocks() / 8;
  uint64_t cap = (uint64_t)cus * bpc;
  uint64_t b = (units + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b == 0) b = 1;
  return (unsigned)b;
}

template <int DT, int OP, int U, int NT, int BS = 256>
static void launch_vec(void* store, const void* vals, void* out, uint64_t nvec, int bpc,
                       hipStream_t s) {
  unsigned g = stream_grid(nvec, (uint64_t)BS * U, bpc);
  k_dense_vec<DT, OP, U, NT, BS><<<g, BS, 0, s>>>((u32x4*)store, (const u32x4*)vals, (u32x4*)out, nvec);
}

template <int DT, int OP>
static void dispatch_vec(const DenseCfg& c, void* store, const void* vals, void* out,
                         uint64_t nvec, hipStream_t s) {
#define PSG_V(U, NT)                                                                \
  if (c.unroll == U && c.nt == NT && c.block == 256) {                              \
    launch_vec<DT, OP, U, NT>(store, vals, out, nvec, c.blocks_per_cu, s);           \
    return;                                                                         \
  }
#define PSG_VB(U, NT, BS)                                                           \
  if (c.unroll == U && c.nt == NT && c.block == BS) {                               \
    launch_vec<DT, OP, U, NT, BS>(store, vals, out, nvec, c.blocks_per_cu, s);       \
    return;                                                                         \
  }
  PSG_V(1, 0) PSG_V(1, 1) PSG_V(1, 2) PSG_V(1, 3) PSG_V(2, 0) PSG_V(2, 1) PSG_V(2, 2) PSG_V(2, 3)
  PSG_V(4, 0) PSG_V(4, 1) PSG_V(4, 2) PSG_V(4, 3) PSG_V(8, 0) PSG_V(8, 1) PSG_V(8, 2) PSG_V(8, 3)
  PSG_VB(1, 1, 512) PSG_VB(1, 3, 512) PSG_VB(2, 1, 512) PSG_VB(2, 3, 512)
  PSG_VB(1, 1, 1024) PSG_VB(1, 3, 1024) PSG_VB(2, 1, 1024) PSG_VB(2, 3, 1024)
#undef PSG_VB
#undef PSG_V
  // a shape without an instantiation: the same threads per CU in 256-thread
  // blocks (unroll and nt are validated by dense_cfg: the 256 table has them all)
  if (c.block == 256) return;
  DenseCfg d = c;
  d.block = 256;
  d.blocks_per_cu = c.blocks_per_cu * c.block / 256;
  dispatch_vec<DT, OP>(d, store, vals, out, nvec, s);
}

template <int DT, int OP>
static int run_dense(void* store, const void* vals, void* out, uint64_t n, hipStream_t s) {
  using T = typename Elem<DT>::T;
  constexpr int kVec = Elem<DT>::kVec;
  const bool need_vals = (OP & PSG_PUSH) != 0, need_out = (OP & PSG_PULL) != 0;
  bool vec_ok = aligned16(store) && (!need_vals || aligned16(vals)) && (!need_out || aligned16(out));
  uint64_t nvec = vec_ok ? n / kVec : 0;
  if (nvec) dispatch_vec<DT, OP>(dense_cfg_for(n * sizeof(T), OP), store, vals, out, nvec, s);
  uint64_t done = nvec * kVec;
  if (done < n) {
    uint64_t rest = n - done;
    unsigned g = stream_grid(rest, kBlock, 8);
    k_dense_elem<DT, OP><<<g, kBlock, 0, s>>>((T*)store + done,
                                             need_vals ? (const T*)vals + done : nullptr,
                                             need_out ? (T*)out + done : nullptr, rest);
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

template <int DT>
static int run_dense_op(int op, void* store, const void* vals, void* out, uint64_t n,
                        hipStream_t s) {
  switch (op) {
    case PSG_PUSH: return run_dense<DT, PSG_PUSH>(store, vals, out, n, s);
    case PSG_PULL: return run_dense<DT, PSG_PULL>(store, vals, out, n, s);
    case PSG_PUSH | PSG_PULL: return run_dense<DT, PSG_PUSH | PSG_PULL>(store, vals, out, n, s);
    default: set_error("bad request flags %d", op); return PSG_ERR_INVALID;
  }
}

int dense_request(int dtype, int op, void* store_vals, const void* vals, void* out, uint64_t n,
                  hipStream_t stream) {
  if (n == 0) return PSG_OK;
  switch (dtype) {
    case PSG_F32: return run_dense_op<PSG_F32>(op, store_vals, vals, out, n, stream);
    case PSG_F64: return run_dense_op<PSG_F64>(op, store_vals, vals, out, n, stream);
    case PSG_F16: return run_dense_op<PSG_F16>(op, store_vals, vals, out, n, stream);
    case PSG_BF16: return run_dense_op<PSG_BF16>(op, store_vals, vals, out, n, stream);
    default: set_error("unsupported dtype %d", dtype); return PSG_ERR_UNSUPPORTED;
  }
}

template <int DT>
static int run_slots(int op, void* store, const uint32_t* slots, const void* vals, void* out,
                     uint64_t n, hipStream_t s) {
  using T = typename Elem<DT>::T;
  if constexpr (sizeof(T) == 4) {
    const bool need_vals = (op & PSG_PUSH) != 0, need_out = (op & PSG_PULL) != 0;
    const uint64_t nq = (aligned16(slots) && (!need_vals || aligned16(vals)) && (!need_out || aligned16(out)))
                            ? n / 4 : 0;
    if (nq) {
      // one group of four per lane at 8 blocks/CU: 10 M cached keys, Push+Pull
      // 1,711 GB/s against 1,689 at 2 groups x 4 blocks/CU (3 runs each);
      // PSG_SLOTS_U / PSG_SLOTS_BPC override it for sweeps
      static const int su = [] { const char* e = getenv("PSG_SLOTS_U"); return e ? atoi(e) : 1; }();
      static const int sb = [] {
        const char* e = getenv("PSG_SLOTS_BPC");
        const int v = e ? atoi(e) : 8;
        return v >= 1 && v <= 32 ? v : 8;
      }();
      auto go = [&](auto uc) {
        constexpr int U = decltype(uc)::value;
        const unsigned g = stream_grid(nq, (uint64_t)kBlock * U, sb);
        switch (op) {
          case PSG_PUSH:
            k_slots_vec<DT, PSG_PUSH, U><<<g, kBlock, 0, s>>>((T*)store, (const u32x4*)slots, (const u32x4*)vals,
                                                              (u32x4*)out, nq);
            break;
          case PSG_PULL:
            k_slots_vec<DT, PSG_PULL, U><<<g, kBlock, 0, s>>>((T*)store, (const u32x4*)slots, (const u32x4*)vals,
                                                              (u32x4*)out, nq);
            break;
          default:
            k_slots_vec<DT, PSG_PUSH | PSG_PULL, U><<<g, kBlock, 0, s>>>(
                (T*)store, (const u32x4*)slots, (const u32x4*)vals, (u32x4*)out, nq);
        }
      };
      if (su == 1) go(std::integral_constant<int, 1>());
      else if (su == 4) go(std::integral_constant<int, 4>());
      else go(std::integral_constant<int, 2>());
      PSG_HIP(hipGetLastError());
      const uint64_t done = nq * 4;
      if (done == n) return PSG_OK;
      slots += done;
      vals = need_vals ? (const void*)((const T*)vals + done) : nullptr;
      out = need_out ? (void*)((T*)out + done) : nullptr;
      n -= done;
    }
  }
  unsigned g = stream_grid(n, kBlock, 8);
  switch (op) {
    case PSG_PUSH:
      k_slots<DT, PSG_PUSH><<<g, kBlock, 0, s>>>((T*)store, slots, (const T*)vals, (T*)out, n);
      break;
    case PSG_PULL:
      k_slots<DT, PSG_PULL><<<g, kBlock, 0, s>>>((T*)store, slots, (const T*)vals, (T*)out, n);
      break;
    case PSG_PUSH | PSG_PULL:
      k_slots<DT, PSG_PUSH | PSG_PULL><<<g, kBlock, 0, s>>>((T*)store, slots, (const T*)vals,
                                                            (T*)out, n);
      break;
    default: set_error("bad request flags %d", op); return PSG_ERR_INVALID;
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int slot_request(int dtype, int op, void* store_vals, const uint32_t* slots, const void* vals,
                 void* out, uint64_t n, hipStream_t stream) {
  if (n == 0) return PSG_OK;
  switch (dtype) {
    case PSG_F32: return run_slots<PSG_F32>(op, store_vals, slots, vals, out, n, stream);
    case PSG_F64: return run_slots<PSG_F64>(op, store_vals, slots, vals, out, n, stream);
    case PSG_F16: return run_slots<PSG_F16>(op, store_vals, slots, vals, out, n, stream);
    case PSG_BF16: return run_slots<PSG_BF16>(op, store_vals, slots, vals, out, n, stream);
    default: set_error("unsupported dtype %d", dtype); return PSG_ERR_UNSUPPORTED;
  }
}

}  // namespace psg

extern "C" int psg_copy(void* dst, const void* src, uint64_t bytes, int unroll, int blocks_per_cu,
                        psg_stream stream) {
  using namespace psg;
  if (bytes == 0) return PSG_OK;
  PSG_REQUIRE(dst && src && aligned16(dst) && aligned16(src) && bytes % 16 == 0, PSG_ERR_INVALID,
              "psg_copy: 16-B aligned pointers and a multiple of 16 bytes");
  PSG_REQUIRE((unroll == 1 || unroll == 2 || unroll == 4 || unroll == 8) && blocks_per_cu >= 1 && blocks_per_cu <= 16,
              PSG_ERR_INVALID, "psg_copy: unroll 1/2/4/8, 1..16 blocks per CU");
  DenseCfg c;
  c.unroll = unroll;
  c.nt = 3;  // non-temporal loads (the "store" operand is the source) and stores
  c.blocks_per_cu = blocks_per_cu;
  // a Pull with the source as its store: load 16 B, store 16 B, nothing else
  dispatch_vec<PSG_F32, PSG_PULL>(c, const_cast<void*>(src), nullptr, dst, bytes / 16, (hipStream_t)stream);
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}
