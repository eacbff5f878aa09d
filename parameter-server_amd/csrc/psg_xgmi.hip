// psg_xgmi.hip — one-shot BSP exchange over xGMI without RCCL.
//
// MI355X links every GPU of a node to every other GPU (7 xGMI links per GPU).
// A ring collective moves each byte over one link per step; here every rank
// maps its peers' buffers (hipIpc handles, exchanged by the caller) and
// touches all of them in ONE kernel, so all 7 links carry traffic at once and
// the reduction is fused with the store update:
//
//   Push (psg_xgmi_push)  rank r:  shard[i] = ((shard[i] + v_0[r*blk+i]) + v_1[..]) + ...
//                         summed in rank order 0..N-1 (deterministic), reading
//                         N-1 peers' request vectors in place — the
//                         reduce-scatter and the accumulate of psg_comm_push in
//                         one pass over HBM.
//   Pull (psg_xgmi_pull)  rank r:  out[w*blk + i] = shard_w[i] for every w —
//                         the all-gather, reading N-1 peers' shards in place.
//   Pull as writes (psg_xgmi_pull_write)  rank r:  out_w[r*blk + i] = shard[i]
//                         for every w — the same all-gather pushed out over
//                         the links (egress) while the Push reads (ingress).
//
// Ordering between ranks is the caller's: all Pushes must be complete before
// any Pull reads a shard, and every Pull complete before the next Push
// changes a shard (a node barrier after each phase; psg_node_barrier is one).
// Per-rank traffic: Push reads (N-1)/N of its block from peers; Pull reads
// (N-1)/N of the vector — the same bytes as RS + AG, in one hop each.
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>

#include "psg_internal.h"

namespace psg {

constexpr int kMaxPeers = 16;

struct Peers {
  const u32x4* p[kMaxPeers];
};

// store += sum_w src_w (16-B vectors), sources added in rank order.
template <int DT>
__global__ __launch_bounds__(256) void k_xgmi_push(u32x4* __restrict__ store, Peers src, int nsrc,
                                                   uint64_t nvec) {
  using E = Elem<DT>;
  for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < nvec;
       j += (uint64_t)gridDim.x * kBlock) {
    u32x4 v[kMaxPeers];
#pragma unroll
    for (int w = 0; w < kMaxPeers; ++w)
      if (w < nsrc) v[w] = __builtin_nontemporal_load(src.p[w] + j);
    u32x4 acc = store[j];
#pragma unroll
    for (int w = 0; w < kMaxPeers; ++w)
      if (w < nsrc) acc = E::add(acc, v[w]);
    store[j] = acc;
  }
}

// out[w*ostride ...] = shard_w (16-B vectors, nvec of them); blockIdx.y = w.
// Four loads in flight per lane before the stores: a read of a peer's HBM over
// xGMI waits microseconds, and Little's law at ~1 TB/s of ingress needs several
// MB in flight across the chip (512 blocks x 256 lanes x 64 B = 8 MB).
constexpr int kPullU = 4;
__global__ __launch_bounds__(256) void k_xgmi_pull(u32x4* __restrict__ out, Peers shard, uint64_t nvec,
                                                   uint64_t ostride) {
  const int w = blockIdx.y;
  const u32x4* __restrict__ s = shard.p[w];
  u32x4* __restrict__ o = out + (uint64_t)w * ostride;
  const uint64_t tile = (uint64_t)kBlock * kPullU;
  for (uint64_t base = (uint64_t)blockIdx.x * tile + threadIdx.x; base < nvec;
       base += (uint64_t)gridDim.x * tile) {
    u32x4 v[kPullU];
#pragma unroll
    for (int u = 0; u < kPullU; ++u) {
      const uint64_t j = base + (uint64_t)u * kBlock;
      if (j < nvec) v[u] = __builtin_nontemporal_load(s + j);
    }
#pragma unroll
    for (int u = 0; u < kPullU; ++u) {
      const uint64_t j = base + (uint64_t)u * kBlock;
      if (j < nvec) __builtin_nontemporal_store(v[u], o + j);
    }
  }
}

// The Pull as writes: v = shard[j] (local HBM, read once), then one
// non-temporal 16-B store of v into every rank's output (remote stores over
// xGMI are posted: no round trip per access, unlike the reads of k_xgmi_pull).
// Two vectors per lane in flight.
struct Outs {
  u32x4* p[kMaxPeers];
};
constexpr int kScatterU = 2;
__global__ __launch_bounds__(256) void k_xgmi_scatter(const u32x4* __restrict__ shard, Outs outs, int nout,
                                                      uint64_t nvec) {
  const uint64_t tile = (uint64_t)kBlock * kScatterU;
  for (uint64_t base = (uint64_t)blockIdx.x * tile + threadIdx.x; base < nvec;
       base += (uint64_t)gridDim.x * tile) {
    u32x4 v[kScatterU];
#pragma unroll
    for (int u = 0; u < kScatterU; ++u) {
      const uint64_t j = base + (uint64_t)u * kBlock;
      if (j < nvec) v[u] = __builtin_nontemporal_load(shard + j);
    }
#pragma unroll
    for (int w = 0; w < kMaxPeers; ++w) {
      if (w >= nout) break;
#pragma unroll
      for (int u = 0; u < kScatterU; ++u) {
        const uint64_t j = base + (uint64_t)u * kBlock;
        if (j < nvec) __builtin_nontemporal_store(v[u], outs.p[w] + j);
      }
    }
  }
}

// ---- keyed exchange on cached slots (LR key caching across GPUs) ------------
// Every worker pushes values for the SAME key list (LR-like, configs[3]); the
// list's segment r belongs to shard r, whose SORTED store resolved it once to
// slots (psg_store_resolve).  Push: rank r reads segment r of every rank's
// value vector in place and adds them in rank order to its store slots
// (store[slot] + v_0 + v_1 + ..., the arrival order 0..N-1 of the N Push
// requests, KVApp.h:446-449).  Pull: rank r gathers every owner's segment from
// the owner's store through the owner's slots (KVApp.h:452 + the merge of
// :713-720).  Four keys per lane; 16-B loads of the slots and values, and a
// 16-B store read-modify-write when the four slots are consecutive.
template <int DT>
__global__ __launch_bounds__(256) void k_xgmi_push_slots(typename Elem<DT>::T* __restrict__ store,
                                                         const uint32_t* __restrict__ slots, Peers src,
                                                         int nsrc, uint64_t n, int vec) {
  using E = Elem<DT>;
  using T = typename E::T;
  const uint64_t nq = vec ? n / 4 : 0;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  if constexpr (sizeof(T) == 4) {
    typedef T t4 __attribute__((ext_vector_type(4)));
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < nq; j += stride) {
      const u32x4 sl = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(slots) + j);
      t4 v[kMaxPeers];
#pragma unroll
      for (int w = 0; w < kMaxPeers; ++w)
        if (w < nsrc) v[w] = __builtin_bit_cast(t4, __builtin_nontemporal_load(src.p[w] + j));
      const uint32_t p0 = sl[0];
      if (sl[1] == p0 + 1 && sl[2] == p0 + 2 && sl[3] == p0 + 3 && (p0 & 3) == 0) {
        u32x4* sp = reinterpret_cast<u32x4*>(store + p0);
        t4 x = __builtin_bit_cast(t4, *sp);
#pragma unroll
        for (int w = 0; w < kMaxPeers; ++w)
          if (w < nsrc) x = x + v[w];
        *sp = __builtin_bit_cast(u32x4, x);
      } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          T x = store[sl[k]];
#pragma unroll
          for (int w = 0; w < kMaxPeers; ++w)
            if (w < nsrc) x = x + v[w][k];
          store[sl[k]] = x;
        }
      }
    }
  }
  for (uint64_t i = nq * 4 + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const uint32_t p = slots[i];
    T x = store[p];
    for (int w = 0; w < nsrc; ++w) x = E::add1(x, reinterpret_cast<const T*>(src.p[w])[i]);
    store[p] = x;
  }
}

// The keyed Pull as writes: rank r reads its segment through its own slots
// (local) and writes it into out_w[seg_off + i] of every rank w.  Four keys
// per lane with 16-B slot loads, a 16-B store read when the four slots are
// consecutive, and 16-B posted stores when the segment is 16-B aligned in the
// outputs (vec); element stores otherwise.
template <typename T>
__global__ __launch_bounds__(256) void k_xgmi_scatter_slots(const T* __restrict__ store,
                                                            const uint32_t* __restrict__ slots, Outs outs,
                                                            int nout, uint64_t seg_off, uint64_t n, int vec) {
  const uint64_t stride = (uint64_t)gridDim.x * kBlock;
  const uint64_t nq = vec ? n / 4 : 0;
  if constexpr (sizeof(T) == 4) {
    for (uint64_t j = (uint64_t)blockIdx.x * kBlock + threadIdx.x; j < nq; j += stride) {
      const u32x4 sl = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(slots) + j);
      const uint32_t p0 = sl[0];
      u32x4 v;
      if (sl[1] == p0 + 1 && sl[2] == p0 + 2 && sl[3] == p0 + 3 && (p0 & 3) == 0) {
        v = *reinterpret_cast<const u32x4*>(store + p0);
      } else {
        const uint32_t* s32 = reinterpret_cast<const uint32_t*>(store);
        v = u32x4{s32[sl[0]], s32[sl[1]], s32[sl[2]], s32[sl[3]]};
      }
#pragma unroll
      for (int w = 0; w < kMaxPeers; ++w) {
        if (w >= nout) break;
        __builtin_nontemporal_store(v, reinterpret_cast<u32x4*>(reinterpret_cast<T*>(outs.p[w]) + seg_off) + j);
      }
    }
  }
  for (uint64_t i = nq * 4 + (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += stride) {
    const T v = store[slots[i]];
    for (int w = 0; w < nout; ++w) reinterpret_cast<T*>(outs.p[w])[seg_off + i] = v;
  }
}

struct SlotPeers {
  const uint32_t* slots[kMaxPeers];
  uint64_t off[kMaxPeers];
  uint64_t cnt[kMaxPeers];
};

// out[off_w + i] = store_w[slots_w[i]]; blockIdx.y = w.
template <typename T>
__global__ __launch_bounds__(256) void k_xgmi_pull_slots(T* __restrict__ out, Peers stores, SlotPeers sp) {
  const int w = blockIdx.y;
  const T* __restrict__ st = reinterpret_cast<const T*>(stores.p[w]);
  const uint32_t* __restrict__ sl = sp.slots[w];
  T* __restrict__ o = out + sp.off[w];
  const uint64_t n = sp.cnt[w];
  for (uint64_t i = (uint64_t)blockIdx.x * kBlock + threadIdx.x; i < n; i += (uint64_t)gridDim.x * kBlock)
    o[i] = st[sl[i]];
}

}  // namespace psg

struct psg_xgmi {
  int nranks, rank;
  void* vals[psg::kMaxPeers];
  void* stores[psg::kMaxPeers];
  void* outs[psg::kMaxPeers];  // psg_xgmi_set_outs (the write form of the Pull)
};

struct psg_barrier {
  struct Shared {
    std::atomic<int> count;
    std::atomic<int> generation;
    std::atomic<int> broken;  // set by a rank whose wait timed out: every later wait fails
    std::atomic<int> ready;   // kReady once rank 0 has created the segment
  };
  static constexpr int kReady = 0x50534742;
  Shared* sh;
  int nranks, rank;
  std::string name;
};

using namespace psg;

extern "C" {

int psg_ipc_handle_bytes(void) { return (int)sizeof(hipIpcMemHandle_t); }

int psg_ipc_export(const void* dptr, void* handle_out) {
  PSG_REQUIRE(dptr && handle_out, PSG_ERR_INVALID, "psg_ipc_export: null argument");
  hipIpcMemHandle_t h;
  PSG_HIP(hipIpcGetMemHandle(&h, const_cast<void*>(dptr)));
  memcpy(handle_out, &h, sizeof(h));
  return PSG_OK;
}

// Exported handles, by allocation: hipIpcGetMemHandle costs ~3 us a call on
// MI355X (profiles/r3_probe_ipc_cost.txt), and the process-mode Van exports
// every HBM frame of every request (keys, values, the direct-reply slice).  An
// entry is keyed by the allocation's base AND its runtime buffer id (unique
// per allocation, 0.07 us to read), so an address freed and allocated again
// never reuses a stale handle.
namespace {
struct ExportEntry {
  uint64_t buffer_id;
  size_t size;
  hipIpcMemHandle_t handle;
};
std::mutex g_export_mu;
std::unordered_map<uintptr_t, ExportEntry> g_exports;
constexpr size_t kMaxExports = 4096;
}  // namespace

int psg_ipc_export_range(const void* dptr, void* handle_out, uint64_t* offset_out) {
  PSG_REQUIRE(dptr && handle_out && offset_out, PSG_ERR_INVALID, "psg_ipc_export_range: null argument");
  hipDeviceptr_t base = nullptr;
  size_t size = 0;
  PSG_HIP(hipMemGetAddressRange(&base, &size, (hipDeviceptr_t)const_cast<void*>(dptr)));
  static const bool cache_on = [] {  // PSG_IPC_EXPORT_CACHE=0: export every time (A/B)
    const char* e = getenv("PSG_IPC_EXPORT_CACHE");
    return !(e && atoi(e) == 0);
  }();
  unsigned long long id = 0;
  const bool have_id = cache_on &&
      hipPointerGetAttribute(&id, HIP_POINTER_ATTRIBUTE_BUFFER_ID, base) == hipSuccess && id != 0;
  if (!have_id) (void)hipGetLastError();
  *offset_out = (uint64_t)((const char*)dptr - (const char*)base);
  if (have_id) {
    std::lock_guard<std::mutex> lk(g_export_mu);
    auto it = g_exports.find((uintptr_t)base);
    if (it != g_exports.end() && it->second.buffer_id == id && it->second.size == size) {
      memcpy(handle_out, &it->second.handle, sizeof(hipIpcMemHandle_t));
      return PSG_OK;
    }
  }
  hipIpcMemHandle_t h;
  PSG_HIP(hipIpcGetMemHandle(&h, (void*)base));
  memcpy(handle_out, &h, sizeof(h));
  if (have_id) {
    std::lock_guard<std::mutex> lk(g_export_mu);
    if (g_exports.size() >= kMaxExports) g_exports.clear();
    g_exports[(uintptr_t)base] = ExportEntry{id, size, h};
  }
  return PSG_OK;
}

int psg_ipc_open(const void* handle, void** dptr_out) {
  PSG_REQUIRE(handle && dptr_out, PSG_ERR_INVALID, "psg_ipc_open: null argument");
  hipIpcMemHandle_t h;
  memcpy(&h, handle, sizeof(h));
  PSG_HIP(hipIpcOpenMemHandle(dptr_out, h, hipIpcMemLazyEnablePeerAccess));
  return PSG_OK;
}

int psg_ipc_close(void* dptr) {
  if (dptr) PSG_HIP(hipIpcCloseMemHandle(dptr));
  return PSG_OK;
}

int psg_xgmi_create(int nranks, int rank, void* const* peer_vals, void* const* peer_stores,
                    psg_xgmi** out) {
  PSG_REQUIRE(out && peer_vals && peer_stores && nranks > 0 && nranks <= kMaxPeers && rank >= 0 &&
                  rank < nranks,
              PSG_ERR_INVALID, "psg_xgmi_create: bad arguments (at most %d ranks)", kMaxPeers);
  psg_xgmi* x = new psg_xgmi();
  memset(x, 0, sizeof(*x));
  x->nranks = nranks;
  x->rank = rank;
  for (int r = 0; r < nranks; ++r) {
    PSG_REQUIRE(peer_vals[r] && peer_stores[r], PSG_ERR_INVALID, "psg_xgmi_create: null peer %d", r);
    PSG_REQUIRE(aligned16(peer_vals[r]) && aligned16(peer_stores[r]), PSG_ERR_INVALID,
                "psg_xgmi_create: peer %d buffers not 16-B aligned", r);
    x->vals[r] = peer_vals[r];
    x->stores[r] = peer_stores[r];
  }
  *out = x;
  return PSG_OK;
}

int psg_xgmi_destroy(psg_xgmi* x) {
  delete x;
  return PSG_OK;
}

int psg_xgmi_push_range(psg_xgmi* x, psg_store* shard, uint64_t n_total, uint64_t off, uint64_t cnt,
                        psg_stream stream) {
  PSG_REQUIRE(x && shard && shard->kind == PSG_STORE_DENSE, PSG_ERR_INVALID,
              "psg_xgmi_push: need a DENSE shard");
  PSG_REQUIRE(n_total % (uint64_t)x->nranks == 0, PSG_ERR_INVALID, "psg_xgmi_push: n_total %% nranks");
  const uint64_t blk = n_total / (uint64_t)x->nranks;
  PSG_REQUIRE(shard->capacity >= blk, PSG_ERR_RANGE, "psg_xgmi_push: shard too small");
  PSG_REQUIRE(off <= blk && cnt <= blk - off, PSG_ERR_RANGE, "psg_xgmi_push: range [%llu, +%llu) outside the block",
              (unsigned long long)off, (unsigned long long)cnt);
  PSG_REQUIRE(shard->vals == x->stores[x->rank], PSG_ERR_INVALID, "psg_xgmi_push: shard is not this rank's store");
  const int es = shard->esize;
  PSG_REQUIRE((blk * es) % 16 == 0 && (off * es) % 16 == 0 && (cnt * es) % 16 == 0, PSG_ERR_INVALID,
              "psg_xgmi_push: block, offset and count must be multiples of 16 B");
  const uint64_t nvec = cnt * es / 16;
  if (nvec == 0) return PSG_OK;
  Peers src;
  for (int w = 0; w < x->nranks; ++w)
    src.p[w] = (const u32x4*)((const char*)x->vals[w] + ((uint64_t)x->rank * blk + off) * es);
  u32x4* dst = (u32x4*)((char*)shard->vals + off * es);
  uint64_t g = (nvec + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)max_stream_blocks() / 4;  // 2 per CU
  if (g > cap) g = cap;
  hipStream_t st = (hipStream_t)stream;
  switch (shard->dtype) {
    case PSG_F32: k_xgmi_push<PSG_F32><<<(unsigned)g, kBlock, 0, st>>>(dst, src, x->nranks, nvec); break;
    case PSG_F64: k_xgmi_push<PSG_F64><<<(unsigned)g, kBlock, 0, st>>>(dst, src, x->nranks, nvec); break;
    case PSG_F16: k_xgmi_push<PSG_F16><<<(unsigned)g, kBlock, 0, st>>>(dst, src, x->nranks, nvec); break;
    default: k_xgmi_push<PSG_BF16><<<(unsigned)g, kBlock, 0, st>>>(dst, src, x->nranks, nvec); break;
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int psg_xgmi_push(psg_xgmi* x, psg_store* shard, uint64_t n_total, psg_stream stream) {
  PSG_REQUIRE(x && shard, PSG_ERR_INVALID, "psg_xgmi_push: null argument");
  return psg_xgmi_push_range(x, shard, n_total, 0, n_total / (uint64_t)x->nranks, stream);
}

// LR BSP Push over xGMI: rank r reads block r of every rank's gradient vector
// (N-1 of them over the links) and applies the merged gradient to its weight
// shard in ONE kernel — merge from 0 in rank order (one arrival order of
// LRServer.h:158-160), then SGD / Adam (LRServer.h:171-177).
int psg_xgmi_lr_push(psg_xgmi* x, psg_store* weights, uint64_t n_total, float lr, psg_adam* adam,
                     int iteration, psg_stream stream) {
  PSG_REQUIRE(x && weights && weights->kind == PSG_STORE_DENSE && weights->dtype == PSG_F32,
              PSG_ERR_INVALID, "psg_xgmi_lr_push: need an f32 DENSE weight shard");
  PSG_REQUIRE(n_total % (uint64_t)x->nranks == 0, PSG_ERR_INVALID, "psg_xgmi_lr_push: n_total %% nranks");
  PSG_REQUIRE(weights->vals == x->stores[x->rank], PSG_ERR_INVALID,
              "psg_xgmi_lr_push: weights are not this rank's registered shard");
  PSG_REQUIRE(x->nranks <= kMaxGrads, PSG_ERR_INVALID, "psg_xgmi_lr_push: at most %d ranks", kMaxGrads);
  const uint64_t blk = n_total / (uint64_t)x->nranks;
  const float* g[kMaxPeers];
  for (int w = 0; w < x->nranks; ++w) g[w] = (const float*)x->vals[w] + (uint64_t)x->rank * blk;
  return lr_apply_sum(weights, 0, g, x->nranks, 1, blk, lr, adam, 0, iteration, (hipStream_t)stream);
}

int psg_xgmi_push_slots(psg_xgmi* x, psg_store* shard, const uint32_t* slots, uint64_t seg_off, uint64_t seg_n,
                        psg_stream stream) {
  PSG_REQUIRE(x && shard, PSG_ERR_INVALID, "psg_xgmi_push_slots: null argument");
  PSG_REQUIRE(shard->vals == x->stores[x->rank], PSG_ERR_INVALID,
              "psg_xgmi_push_slots: shard is not this rank's registered store");
  if (seg_n == 0) return PSG_OK;
  PSG_REQUIRE(slots, PSG_ERR_INVALID, "psg_xgmi_push_slots: null slots");
  const int es = shard->esize;
  Peers src;
  bool vec = aligned16(slots) && aligned16(shard->vals) && es == 4;
  for (int w = 0; w < x->nranks; ++w) {
    src.p[w] = (const u32x4*)((const char*)x->vals[w] + seg_off * es);
    vec = vec && aligned16(src.p[w]);
  }
  const uint64_t units = vec ? seg_n / 4 : seg_n;
  uint64_t g = (units + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)max_stream_blocks() / 4;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  hipStream_t st = (hipStream_t)stream;
  switch (shard->dtype) {
    case PSG_F32:
      k_xgmi_push_slots<PSG_F32><<<(unsigned)g, kBlock, 0, st>>>((float*)shard->vals, slots, src, x->nranks, seg_n, vec);
      break;
    case PSG_F64:
      k_xgmi_push_slots<PSG_F64><<<(unsigned)g, kBlock, 0, st>>>((double*)shard->vals, slots, src, x->nranks, seg_n, 0);
      break;
    case PSG_F16:
      k_xgmi_push_slots<PSG_F16><<<(unsigned)g, kBlock, 0, st>>>((_Float16*)shard->vals, slots, src, x->nranks, seg_n, 0);
      break;
    default:
      k_xgmi_push_slots<PSG_BF16><<<(unsigned)g, kBlock, 0, st>>>((__bf16*)shard->vals, slots, src, x->nranks, seg_n, 0);
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int psg_xgmi_pull_slots(psg_xgmi* x, psg_store* shard, const uint32_t* const* peer_slots,
                        const uint64_t* seg_off_host, const uint64_t* seg_n_host, void* out, psg_stream stream) {
  PSG_REQUIRE(x && shard && peer_slots && seg_off_host && seg_n_host && out, PSG_ERR_INVALID,
              "psg_xgmi_pull_slots: null argument");
  Peers st;
  SlotPeers sp;
  uint64_t most = 0;
  for (int w = 0; w < x->nranks; ++w) {
    PSG_REQUIRE(peer_slots[w] || seg_n_host[w] == 0, PSG_ERR_INVALID, "psg_xgmi_pull_slots: null slots of rank %d", w);
    st.p[w] = (const u32x4*)x->stores[w];
    sp.slots[w] = peer_slots[w];
    sp.off[w] = seg_off_host[w];
    sp.cnt[w] = seg_n_host[w];
    most = seg_n_host[w] > most ? seg_n_host[w] : most;
  }
  if (most == 0) return PSG_OK;
  uint64_t gx = (most + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)max_stream_blocks() / 2 / (uint64_t)x->nranks + 1;
  if (gx > cap) gx = cap;
  const dim3 grid((unsigned)gx, (unsigned)x->nranks);
  hipStream_t s = (hipStream_t)stream;
  switch (shard->esize) {
    case 4: k_xgmi_pull_slots<uint32_t><<<grid, kBlock, 0, s>>>((uint32_t*)out, st, sp); break;
    case 8: k_xgmi_pull_slots<uint64_t><<<grid, kBlock, 0, s>>>((uint64_t*)out, st, sp); break;
    default: k_xgmi_pull_slots<uint16_t><<<grid, kBlock, 0, s>>>((uint16_t*)out, st, sp); break;
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int psg_xgmi_pull_write_slots(psg_xgmi* x, psg_store* shard, const uint32_t* slots, uint64_t seg_off,
                              uint64_t seg_n, psg_stream stream) {
  PSG_REQUIRE(x && shard, PSG_ERR_INVALID, "psg_xgmi_pull_write_slots: null argument");
  PSG_REQUIRE(x->outs[0] != nullptr, PSG_ERR_INVALID, "psg_xgmi_pull_write_slots: no outputs (psg_xgmi_set_outs)");
  PSG_REQUIRE(shard->vals == x->stores[x->rank], PSG_ERR_INVALID,
              "psg_xgmi_pull_write_slots: shard is not this rank's registered store");
  if (seg_n == 0) return PSG_OK;
  PSG_REQUIRE(slots, PSG_ERR_INVALID, "psg_xgmi_pull_write_slots: null slots");
  const int es = shard->esize;
  Outs o;
  for (int w = 0; w < x->nranks; ++w) o.p[w] = (u32x4*)x->outs[w];
  const int vec = (es == 4 && aligned16(slots) && aligned16(shard->vals) && (seg_off * es) % 16 == 0) ? 1 : 0;
  const uint64_t units = vec ? seg_n / 4 : seg_n;
  uint64_t g = (units + kBlock - 1) / kBlock;
  const uint64_t cap = (uint64_t)max_stream_blocks() / 4;
  if (g > cap) g = cap;
  if (g == 0) g = 1;
  hipStream_t st = (hipStream_t)stream;
  switch (es) {
    case 4:
      k_xgmi_scatter_slots<uint32_t><<<(unsigned)g, kBlock, 0, st>>>((const uint32_t*)shard->vals, slots, o,
                                                                     x->nranks, seg_off, seg_n, vec);
      break;
    case 8:
      k_xgmi_scatter_slots<uint64_t><<<(unsigned)g, kBlock, 0, st>>>((const uint64_t*)shard->vals, slots, o,
                                                                     x->nranks, seg_off, seg_n, 0);
      break;
    default:
      k_xgmi_scatter_slots<uint16_t><<<(unsigned)g, kBlock, 0, st>>>((const uint16_t*)shard->vals, slots, o,
                                                                     x->nranks, seg_off, seg_n, 0);
  }
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int psg_xgmi_pull_range(psg_xgmi* x, psg_store* shard, void* out, uint64_t n_total, uint64_t off,
                        uint64_t cnt, psg_stream stream) {
  PSG_REQUIRE(x && shard && out, PSG_ERR_INVALID, "psg_xgmi_pull: null argument");
  PSG_REQUIRE(n_total % (uint64_t)x->nranks == 0, PSG_ERR_INVALID, "psg_xgmi_pull: n_total %% nranks");
  const int es = shard->esize;
  const uint64_t blk = n_total / (uint64_t)x->nranks;
  PSG_REQUIRE(off <= blk && cnt <= blk - off, PSG_ERR_RANGE, "psg_xgmi_pull: range [%llu, +%llu) outside the block",
              (unsigned long long)off, (unsigned long long)cnt);
  PSG_REQUIRE((blk * es) % 16 == 0 && (off * es) % 16 == 0 && (cnt * es) % 16 == 0 && aligned16(out),
              PSG_ERR_INVALID, "psg_xgmi_pull: blocks, offset, count and out must be 16-B aligned");
  const uint64_t nvec = cnt * es / 16;
  if (nvec == 0) return PSG_OK;
  Peers sh;
  for (int w = 0; w < x->nranks; ++w) sh.p[w] = (const u32x4*)((const char*)x->stores[w] + off * es);
  uint64_t gx = (nvec + (uint64_t)kBlock * kPullU - 1) / ((uint64_t)kBlock * kPullU);
  const uint64_t cap = (uint64_t)max_stream_blocks() / 4 / (uint64_t)x->nranks + 1;
  if (gx > cap) gx = cap;
  k_xgmi_pull<<<dim3((unsigned)gx, (unsigned)x->nranks), kBlock, 0, (hipStream_t)stream>>>(
      (u32x4*)((char*)out + off * es), sh, nvec, blk * es / 16);
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int psg_xgmi_pull(psg_xgmi* x, psg_store* shard, void* out, uint64_t n_total, psg_stream stream) {
  PSG_REQUIRE(x && shard, PSG_ERR_INVALID, "psg_xgmi_pull: null argument");
  return psg_xgmi_pull_range(x, shard, out, n_total, 0, n_total / (uint64_t)x->nranks, stream);
}

int psg_xgmi_set_outs(psg_xgmi* x, void* const* peer_outs) {
  PSG_REQUIRE(x && peer_outs, PSG_ERR_INVALID, "psg_xgmi_set_outs: null argument");
  for (int r = 0; r < x->nranks; ++r) {
    PSG_REQUIRE(peer_outs[r] && aligned16(peer_outs[r]), PSG_ERR_INVALID,
                "psg_xgmi_set_outs: output %d null or not 16-B aligned", r);
    x->outs[r] = peer_outs[r];
  }
  return PSG_OK;
}

int psg_xgmi_pull_write_range(psg_xgmi* x, psg_store* shard, uint64_t n_total, uint64_t off, uint64_t cnt,
                              psg_stream stream) {
  PSG_REQUIRE(x && shard && shard->kind == PSG_STORE_DENSE, PSG_ERR_INVALID,
              "psg_xgmi_pull_write: need a DENSE shard");
  PSG_REQUIRE(x->outs[0] != nullptr, PSG_ERR_INVALID, "psg_xgmi_pull_write: no outputs (psg_xgmi_set_outs)");
  PSG_REQUIRE(n_total % (uint64_t)x->nranks == 0, PSG_ERR_INVALID, "psg_xgmi_pull_write: n_total %% nranks");
  const int es = shard->esize;
  const uint64_t blk = n_total / (uint64_t)x->nranks;
  PSG_REQUIRE(shard->capacity >= blk, PSG_ERR_RANGE, "psg_xgmi_pull_write: shard too small");
  PSG_REQUIRE(shard->vals == x->stores[x->rank], PSG_ERR_INVALID,
              "psg_xgmi_pull_write: shard is not this rank's store");
  PSG_REQUIRE(off <= blk && cnt <= blk - off, PSG_ERR_RANGE,
              "psg_xgmi_pull_write: range [%llu, +%llu) outside the block", (unsigned long long)off,
              (unsigned long long)cnt);
  PSG_REQUIRE((blk * es) % 16 == 0 && (off * es) % 16 == 0 && (cnt * es) % 16 == 0, PSG_ERR_INVALID,
              "psg_xgmi_pull_write: block, offset and count must be multiples of 16 B");
  const uint64_t nvec = cnt * es / 16;
  if (nvec == 0) return PSG_OK;
  Outs o;
  for (int w = 0; w < x->nranks; ++w)
    o.p[w] = (u32x4*)((char*)x->outs[w] + ((uint64_t)x->rank * blk + off) * es);
  uint64_t g = (nvec + (uint64_t)kBlock * kScatterU - 1) / ((uint64_t)kBlock * kScatterU);
  const uint64_t cap = (uint64_t)max_stream_blocks() / 4;  // 2 per CU
  if (g > cap) g = cap;
  k_xgmi_scatter<<<(unsigned)g, kBlock, 0, (hipStream_t)stream>>>(
      (const u32x4*)((const char*)shard->vals + off * es), o, x->nranks, nvec);
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int psg_xgmi_pull_write(psg_xgmi* x, psg_store* shard, uint64_t n_total, psg_stream stream) {
  PSG_REQUIRE(x && shard, PSG_ERR_INVALID, "psg_xgmi_pull_write: null argument");
  return psg_xgmi_pull_write_range(x, shard, n_total, 0, n_total / (uint64_t)x->nranks, stream);
}

// ---- node barrier: a sense-counting barrier in a POSIX shared-memory page --
// Rank 0 creates the segment exclusively (a name left over by a crashed job is
// an error, never a stale count); the other ranks wait for it to appear.  A
// wait that times out has already counted itself in, so it poisons the
// barrier: every later wait on it, in any rank, fails instead of releasing a
// phase early.
int psg_node_barrier_create(const char* name, int nranks, int rank, psg_barrier** out) {
  PSG_REQUIRE(name && out && nranks > 0 && rank >= 0 && rank < nranks, PSG_ERR_INVALID,
              "psg_node_barrier_create: bad arguments");
  std::string nm = std::string("/") + name;
  int fd = -1;
  if (rank == 0) {
    fd = shm_open(nm.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    PSG_REQUIRE(fd >= 0, PSG_ERR_INVALID, "shm_open(%s, O_EXCL) failed: %s (a stale segment of another job?)",
                nm.c_str(), strerror(errno));
    if (ftruncate(fd, 4096) != 0) {
      close(fd);
      shm_unlink(nm.c_str());
      set_error("ftruncate(%s) failed", nm.c_str());
      return PSG_ERR_INVALID;
    }
  } else {
    for (int tries = 0; (fd = shm_open(nm.c_str(), O_RDWR, 0600)) < 0; ++tries) {
      PSG_REQUIRE(errno == ENOENT && tries < 60000, PSG_ERR_COMM,
                  "node barrier %s: rank 0 never created it (%s)", nm.c_str(), strerror(errno));
      usleep(1000);
    }
    // rank 0 creates the object empty and sizes it next: mapping it before
    // that would fault (SIGBUS) on the first access
    struct stat sb;
    for (int tries = 0; fstat(fd, &sb) == 0 && sb.st_size < 4096; ++tries) {
      if (tries >= 60000) {
        close(fd);
        set_error("node barrier %s: never sized by rank 0", nm.c_str());
        return PSG_ERR_COMM;
      }
      usleep(1000);
    }
  }
  void* p = mmap(nullptr, 4096, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  PSG_REQUIRE(p != MAP_FAILED, PSG_ERR_INVALID, "mmap(%s) failed", nm.c_str());
  auto* sh = (psg_barrier::Shared*)p;  // zero-filled on creation
  if (rank == 0) {
    sh->ready.store(psg_barrier::kReady, std::memory_order_release);
  } else {
    // rank 0 may not have sized the segment yet: wait for its ready mark
    for (int tries = 0; sh->ready.load(std::memory_order_acquire) != psg_barrier::kReady; ++tries) {
      if (tries >= 60000) {
        munmap(p, 4096);
        set_error("node barrier %s: never became ready", nm.c_str());
        return PSG_ERR_COMM;
      }
      usleep(1000);
    }
  }
  psg_barrier* b = new psg_barrier();
  b->sh = sh;
  b->nranks = nranks;
  b->rank = rank;
  b->name = nm;
  *out = b;
  return PSG_OK;
}

int psg_node_barrier_wait(psg_barrier* b, double timeout_s) {
  PSG_REQUIRE(b, PSG_ERR_INVALID, "psg_node_barrier_wait: null barrier");
  PSG_REQUIRE(!b->sh->broken.load(std::memory_order_acquire), PSG_ERR_COMM,
              "node barrier %s is broken (a rank timed out in it)", b->name.c_str());
  const int gen = b->sh->generation.load(std::memory_order_acquire);
  if (b->sh->count.fetch_add(1, std::memory_order_acq_rel) + 1 == b->nranks) {
    b->sh->count.store(0, std::memory_order_relaxed);
    b->sh->generation.fetch_add(1, std::memory_order_acq_rel);
    return PSG_OK;
  }
  struct timespec t0, t;
  clock_gettime(CLOCK_MONOTONIC, &t0);
  for (uint64_t spin = 0; b->sh->generation.load(std::memory_order_acquire) == gen; ++spin) {
    if ((spin & 1023) == 1023) {
      PSG_REQUIRE(!b->sh->broken.load(std::memory_order_acquire), PSG_ERR_COMM,
                  "node barrier %s is broken (a rank timed out in it)", b->name.c_str());
      clock_gettime(CLOCK_MONOTONIC, &t);
      const double el = (t.tv_sec - t0.tv_sec) + 1e-9 * (t.tv_nsec - t0.tv_nsec);
      if (el >= timeout_s) {
        b->sh->broken.store(1, std::memory_order_release);
        set_error("node barrier %s: timed out after %.1f s (barrier now broken)", b->name.c_str(), el);
        return PSG_ERR_COMM;
      }
      if (el > 1e-3) usleep(20);
    }
  }
  return PSG_OK;
}

int psg_node_barrier_destroy(psg_barrier* b) {
  if (!b) return PSG_OK;
  munmap(b->sh, 4096);
  if (b->rank == 0) shm_unlink(b->name.c_str());
  delete b;
  return PSG_OK;
}

}  // extern "C"
