// psg_internal.h — shared internals of the psg C-ABI implementation (gfx950).
//
// Error convention: every extern "C" entry returns an int status; the message
// of the last failure is kept per thread (psg_last_error).  This replaces the
// reference's CHECK -> ps_log::PSError throw (src/base/log.h:283-304), which
// must not cross a C ABI.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <cstdarg>
#include <cstdio>
#include <deque>
#include <string>
#include <vector>

#include "../../include/psg.h"

namespace psg {

void set_error(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
void clear_error();

// Status from a HIP call, with the message recorded.
int hip_fail(hipError_t e, const char* what, const char* file, int line);

}  // namespace psg

#define PSG_HIP(call)                                                   \
  do {                                                                  \
    hipError_t e_ = (call);                                             \
    if (e_ != hipSuccess) return psg::hip_fail(e_, #call, __FILE__, __LINE__); \
  } while (0)

#define PSG_REQUIRE(cond, code, ...)   \
  do {                                 \
    if (!(cond)) {                     \
      psg::set_error(__VA_ARGS__);     \
      return (code);                   \
    }                                  \
  } while (0)

#define PSG_TRY(expr)             \
  do {                            \
    int rc_ = (expr);             \
    if (rc_ != PSG_OK) return rc_; \
  } while (0)

namespace psg {

// ---- element types --------------------------------------------------------
inline int dtype_size(int dtype) {
  switch (dtype) {
    case PSG_F32: return 4;
    case PSG_F64: return 8;
    case PSG_F16: return 2;
    case PSG_BF16: return 2;
    default: return 0;
  }
}

// 16-byte raw vector: the unit of every streaming load/store (one
// global_load_dwordx4 per lane, 1 KiB per wave instruction).
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef double f64x2 __attribute__((ext_vector_type(2)));
typedef uint64_t u64x2 __attribute__((ext_vector_type(2)));

// Per-dtype arithmetic on one 16-B vector.  Sub-32-bit types accumulate in
// f32 and round once (RNE): with p(f32)=24 >= 2*p(f16)+2 the double rounding
// is innocuous, so this equals exact-sum-rounded-to-half arithmetic.
template <int DT> struct Elem;
template <> struct Elem<PSG_F32> {
  typedef float T;
  static constexpr int kVec = 4;
  __device__ static inline u32x4 add(u32x4 a, u32x4 b) {
    f32x4 r = __builtin_bit_cast(f32x4, a) + __builtin_bit_cast(f32x4, b);
    return __builtin_bit_cast(u32x4, r);
  }
  __device__ static inline T add1(T a, T b) { return a + b; }
};
template <> struct Elem<PSG_F64> {
  typedef double T;
  static constexpr int kVec = 2;
  __device__ static inline u32x4 add(u32x4 a, u32x4 b) {
    f64x2 r = __builtin_bit_cast(f64x2, a) + __builtin_bit_cast(f64x2, b);
    return __builtin_bit_cast(u32x4, r);
  }
  __device__ static inline T add1(T a, T b) { return a + b; }
};
template <> struct Elem<PSG_F16> {
  typedef _Float16 T;
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  typedef float f8 __attribute__((ext_vector_type(8)));
  static constexpr int kVec = 8;
  __device__ static inline u32x4 add(u32x4 a, u32x4 b) {
    f8 fa = __builtin_convertvector(__builtin_bit_cast(h8, a), f8);
    f8 fb = __builtin_convertvector(__builtin_bit_cast(h8, b), f8);
    h8 r = __builtin_convertvector(fa + fb, h8);
    return __builtin_bit_cast(u32x4, r);
  }
  __device__ static inline T add1(T a, T b) { return (T)((float)a + (float)b); }
};
template <> struct Elem<PSG_BF16> {
  typedef __bf16 T;
  typedef __bf16 b8 __attribute__((ext_vector_type(8)));
  typedef float f8 __attribute__((ext_vector_type(8)));
  static constexpr int kVec = 8;
  __device__ static inline u32x4 add(u32x4 a, u32x4 b) {
    f8 fa = __builtin_convertvector(__builtin_bit_cast(b8, a), f8);
    f8 fb = __builtin_convertvector(__builtin_bit_cast(b8, b), f8);
    b8 r = __builtin_convertvector(fa + fb, b8);
    return __builtin_bit_cast(u32x4, r);
  }
  __device__ static inline T add1(T a, T b) { return (T)((float)a + (float)b); }
};

// ---- launch geometry --------------------------------------------------------
// Streaming kernels: 256-thread blocks, grid capped at 256 CUs x 8 blocks and
// grid-strided beyond (cdna_hip_programming.md Guideline 11).
constexpr int kBlock = 256;
int max_stream_blocks();

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }

#ifdef __HIPCC__
// lower_bound by one wave: 64 lanes probe 64 evenly spaced keys per round and
// a ballot brackets the answer, so a 10 M-key store takes 4 rounds of one
// parallel load instead of 24 dependent loads.  Wave-uniform result.
__device__ __forceinline__ uint64_t lower_bound_wave(const uint64_t* __restrict__ a, uint64_t S,
                                                     uint64_t key) {
  const int lane = threadIdx.x & 63;
  uint64_t lo = 0, hi = S;  // the answer is in [lo, hi]
  while (hi - lo > 64) {
    const uint64_t step = (hi - lo + 63) / 64;
    const uint64_t p = lo + (uint64_t)lane * step;
    const bool pred = p < hi && a[p] < key;
    const uint64_t c = (uint64_t)__popcll(__ballot(pred));
    if (c == 0) return lo;
    const uint64_t pc = lo + c * step;
    lo = lo + (c - 1) * step + 1;
    hi = pc < hi ? pc : hi;
  }
  const uint64_t p = lo + (uint64_t)lane;
  const bool pred = p < hi && a[p] < key;
  return lo + (uint64_t)__popcll(__ballot(pred));
}
#endif

// Bytes to hipMalloc for an array a peer process may map (hipIpc): the HIP
// runtime may carve allocations below 2 MiB out of a shared block, and such a
// pointer's IPC handle cannot always be opened ("invalid device pointer"), so
// arrays of 64 KiB and more are rounded up to whole 2 MiB pages.
inline size_t ipc_alloc_bytes(size_t bytes) {
  constexpr size_t kPage = 2u << 20;
  return bytes < (64u << 10) ? bytes : (bytes + kPage - 1) / kPage * kPage;
}

// ---- store ------------------------------------------------------------------
}  // namespace psg

namespace psg {
// A fused keyed request launched and not yet reaped (psg_store_handle_async).
struct InflightReq {
  uint64_t ticket;
  int op;
  const uint64_t* q;
  uint64_t n;
  const void* vals;
  void* out;
  uint32_t ring;  // its completion word: ring_host[ring]
  uint32_t tag;   // the 24-bit tag that word will carry
  int wc;         // window-cache entry it ran on
  hipStream_t stream;
  int want_land;  // a Pull answered when reaped (psg_store_handle): its reply must be in memory then
  int land;       // ... and land_ev[ring] was recorded behind its kernels to say so
  int ident;      // sent as an identity request (k_ident_check / k_ident_apply)
  int mident;     // its validation pass marked the tiles that are stretches of the store (chunk_ok)
  int nt;         // threads per block (tile = 4 keys a lane) of its resolve-and-apply launch
  int seq;        // its sequence number (reject words, tile words)
  uint32_t tw_ring;  // the ring slot whose tile words its validation wrote (a follow-up keeps it)
  int lean;       // applied by k_tile_apply (its stretch and coded tiles; general ones follow up)
  int vl;         // 1: validated as its list's verified copy (k_list_check); 2: a learning request
};
constexpr int kRing = 64;  // completion words per store (requests in flight + 1)
struct RunSeen;            // psg_runs.hip (below)
}  // namespace psg

struct psg_store {
  int kind;
  int dtype;
  int esize;
  int device;
  uint64_t key_begin, key_end;
  uint64_t size;      // keys present
  uint64_t capacity;  // slots allocated
  void* vals;         // device, capacity * esize
  uint64_t* keys;     // device, SORTED only
  // scratch for SORTED requests (grown on demand)
  uint32_t* slots;
  uint32_t* slots2;  // slots after an insert (second resolve)
  uint64_t* wlo;     // per-tile store-key windows of the resolve
  uint64_t slots_cap;
  int* flags;        // device view of flags_host: the kernels raise flags there
  int* flags_host;   // pinned host int[4]: any key absent / out of range / unsorted
  // Device words (psg_store.hip, kRej* / kPending): the validation pass sets
  // [0] / [1] to the request's sequence number when a key is out of range /
  // out of order (every store-writing kernel of that request reads them first
  // and writes nothing); [2] != 0 gates every later fused request until the
  // host has done an earlier request's follow-up (insert, out-of-order path).
  int* reject_dev;
  int seq;           // request sequence number (never 0 after the first request)
  // completion events (psg_store.hip, stream_done / wait_landed): one for the
  // host's waits on a stream, one per ring slot for a synchronous Pull's reply
  hipEvent_t done_ev;
  hipEvent_t land_ev[psg::kRing];
  // k_resolve_apply's arrival counters, one set per ring slot: 8 shard
  // counters and a top counter, 64-bit, each on its own 256 B; zeroed by the
  // block that completes the request
  uint64_t* done_ctr;
  // completion words of the fused requests: tag << 8 | flags, written by the
  // kernel with one system-scope store (pinned host memory, kRing words)
  uint32_t* ring_host;
  uint32_t* ring_dev;
  std::vector<hipStream_t> unlanded;  // streams whose reaped async Pulls psg_store_wait still synchronises
  uint32_t ring_next;
  uint32_t tag;
  // fused requests in flight, in launch (= stream) order
  std::deque<psg::InflightReq> inflight;
  uint64_t next_ticket;
  // the first failure of an asynchronous request not yet reported by psg_store_wait
  int async_rc;
  std::string async_msg;
  // scratch of the out-of-order path (psg_store.hip, general_request)
  void* gbuf;
  uint64_t gbuf_bytes;
  // K's generation: bumped whenever the sorted key array changes (insert,
  // clear), so a cached window of an older K is never trusted.
  uint32_t gen;
  // Store-key windows per request tile, cached per request key array (the
  // LR / benchmark steady state sends the same key list again and again).
  struct WinCache {
    const uint64_t* q;   // request keys (device pointer) the entry was filled for
    uint64_t n;
    void* win;           // device psg::Win[ntiles]
    uint32_t* codes;     // device: 1024 lane codes per tile (k_validate_code), reused while they verify
    uint64_t cap_tiles;
    uint64_t last_use;
    int trusted;         // skip the search pre-pass; the kernel still verifies
    int strikes;         // kernel-detected stale windows for this (q, n)
    uint32_t ident_fail; // K's generation at which an identity request on this list was not one
    uint32_t ident_ok;   // K's generation at which an identity request on this list completed as one
    uint64_t ident_trial;  // ticket of the identity attempt in flight before either is known (0: none)
    int nt;              // the block size (tile size / 4) its windows were filled for
    uint32_t lean_fail;  // K's generation at which a k_tile_apply on this list left general tiles
    // the verified copy of the list (k_validate_code's learn, k_list_check):
    // the keys a learning request validated, valid while K keeps copy_gen
    uint64_t* copy;
    uint64_t copy_cap;      // keys it holds room for
    uint32_t copy_gen;      // K's generation it was validated against (0: none)
    uint32_t vl_fail;       // K's generation at which a Push of this list differed from its copy
    uint64_t learn_ticket;  // the last learning request launched (its reap validates the copy)
  } wc[4];
  uint64_t wc_clock;
  uint64_t counters[PSG_NCOUNTERS];  // psg_store_counters
  // per request tile of the current fused Push (device): its tile word —
  // stretch / coded / general for the request that wrote it
  int* chunk_ok;      // per ring slot, per tile: the tile words of the request in that slot (psg_store.hip)
  uint64_t chunk_cap;  // tiles per ring slot
  // the layout of the current run of queued requests (psg_runs.hip, device
  // psg::RunDesc), and how the last runs went (psg_store_run)
  void* run_desc;
  psg::RunSeen* run_seen;  // pinned host: what the last classify saw
  // list positions learnt from strided runs: a list (device pointer, n) whose
  // first key sat at slot pos0 of K generation gen, in a layout of period P
  struct RunPos {
    const uint64_t* q;
    uint64_t n;
    uint64_t pos0;
    uint32_t P;
    uint32_t gen;
    uint64_t last_use;
  } run_pos[64];
  uint64_t run_clock;
  int run_last;       // PSG_RUN_* the last run was served as
  uint32_t run_fail_gen;  // K's generation at which a run with Pulls was not strided
  int run_fail_count;     // ... and how many runs since were served one by one without trying
  // psg_store_run_status: per-request codes of a run served one by one (a
  // request refused for a key outside the range does not stop the run)
  int* run_status = nullptr;
};

struct psg_adam {
  uint64_t n;
  double lr, beta1, beta2, eps;
  // the moments of Adam.h:40-41 in one of psg_lr.hip's layouts: 1 (default)
  // per 128 features their 128 m then their 128 v values, 2 per 256 features
  // four 1 KiB runs of the QUAD lane map (both in m; v unused), 0 two arrays of
  // n doubles; 16-B aligned (hipMalloc)
  double* m;
  double* v;
  int layout;
};

namespace psg {
// Gradient arrays one LR apply pass merges (LRServer's BSP round: one per worker).
constexpr int kMaxGrads = 16;
struct Grads {
  const float* p[kMaxGrads];
};
// weights[w_off + i] -= update(sum_k grads[k][i]) for i < n, Adam state at
// adam_off; the merge and the apply of LRServer.h:158-177 in one pass.
// psg_lr.hip.
// copy_mix (psg_lr_mix_copy, measurement only): the same pass with a copy's
// arithmetic in place of the Adam update.
int lr_apply_sum(psg_store* weights, uint64_t w_off, const float* const* grads, int ngrads,
                 int from_zero, uint64_t n, float lr, psg_adam* adam, uint64_t adam_off,
                 int iteration, hipStream_t st, bool copy_mix = false);
// Dense element-wise request on slot range [off, off + n) of a store value
// array.  op = PSG_PUSH | PSG_PULL bits.  Implemented in psg_dense.hip.
int dense_request(int dtype, int op, void* store_vals, const void* vals, void* out,
                  uint64_t n, hipStream_t stream);
// Slot-indexed request (gather/scatter).  psg_dense.hip.
int slot_request(int dtype, int op, void* store_vals, const uint32_t* slots,
                 const void* vals, void* out, uint64_t n, hipStream_t stream);
// A run of queued Pushes on one key list applied in one pass (psg_frames.hip).
// frames_base: *base = D, the slot of q0[0] in K[0..S) when K[D .. D + n) can
//   hold the list, else UINT64_MAX (one wave);
// frames_check: lists keys[j0..k) equal ref[*base + i] (base NULL: ref[i]) for
//   i < n, else *rej = seq;
// frames_apply: store[*base + i] (base NULL: store[i]) += vals[0][i], then
//   vals[1][i], ... in order — unless *base is UINT64_MAX or *rej == seq, when
//   it writes nothing and sets *flag (pinned host int);
// frames_slots: the same on store[slots[i]] (slots unique).
constexpr int kMaxFrames = 16;
int frames_base(const uint64_t* K, uint64_t S, const uint64_t* q0, uint64_t n, uint64_t* base, hipStream_t st);
int frames_check(const uint64_t* ref, const uint64_t* base, const uint64_t* const* keys, int j0, int k, uint64_t n,
                 int* rej, int seq, hipStream_t st);
int frames_apply(int dtype, void* store_vals, uint64_t store_elems, const void* const* vals, int k, uint64_t n,
                 const uint64_t* base, const int* rej, int seq, int* flag, hipStream_t st);
int frames_slots(int dtype, void* store_vals, const uint32_t* slots, const void* const* vals, int k, uint64_t n,
                 const int* rej, int seq, int* flag, hipStream_t st);
// A run of queued requests on interleaved key lists (psg_runs.hip): request j
// holds every P-th key of the store from its own phase,
//     keys_j[i] == K[D + p_j + P * i]   for i < n_j,
// with the phases p_j distinct — so the lists are pairwise disjoint, every
// store slot is touched by at most one request, and the requests commute: one
// pass over the slots [D, D + span) serves them all with the result of the
// queued sequence.  That is the reference benchmark's key layout
// (tests/test_kv_app_benchmark.cpp:47-52, `kMaxKey / num * i + rank`) at
// nw workers: each server's store holds the nw lists interleaved, P = nw.
constexpr int kRunMaxPeriod = 64;
enum { RUN_NONE = 0, RUN_SAME = 1, RUN_STRIDED = 2 };
struct RunDesc {
  uint64_t D;     // the store slot of the run's lowest first key
  uint64_t rows;  // rows [0, rows): slots D + P * row + phase
  uint32_t P;     // period
  int cls;        // RUN_*: what run_classify found (from first keys only)
  int8_t map[kRunMaxPeriod];  // phase -> request, -1: a phase no request holds
};
// what run_classify saw, mirrored to pinned host memory for the host's cache
// of list positions (psg_store_run): the slot of each list's first key
struct RunSeen {
  RunDesc d;
  uint64_t pos[16];
  int found[16];
};
struct RunFrames {
  const uint64_t* q[kMaxFrames];  // keys of request j (device)
  const void* v[kMaxFrames];      // its pushed values (PSG_PUSH)
  void* o[kMaxFrames];            // its reply values (PSG_PULL)
  uint64_t n[kMaxFrames];         // its keys
  int op[kMaxFrames];             // PSG_PUSH | PSG_PULL bits
  uint64_t lo, hi;                // the store's key range: a key outside it fails the check
};
// run_classify: one block; from the requests' first keys (and the second key of
//   request pl, which gives P) writes *desc and *seen (pinned host); *same_base
//   = D when every list starts at one slot and allow_same (a run of Pushes on
//   one list: the frames path), else UINT64_MAX.
// run_pass: one lane per row, over rows [0, rows), when the layout (*desc when
//   desc != NULL — run_classify's — else `given`) is RUN_STRIDED; else it only
//   raises *flag (when flag != NULL).  mode RUN_CHECK compares every key with
//   its slot's store key and writes seq into *bad on a mismatch; RUN_APPLY
//   applies the run (Pushes add, Pulls read, PushPulls both) unless *bad ==
//   seq, when it writes nothing and raises *flag; RUN_PULL_CHECKED does both
//   for a run without Pushes (nothing in the store is written, so a mismatch
//   just raises *flag and the replies are not used).
enum { RUN_CHECK = 0, RUN_APPLY = 1, RUN_PULL_CHECKED = 2 };
int run_classify(const uint64_t* K, uint64_t S, const RunFrames& f, int k, int pl, int allow_same, RunDesc* desc,
                 RunSeen* seen, uint64_t* same_base, hipStream_t st);
int run_pass(int mode, int dtype, void* store_vals, const uint64_t* K, uint64_t S, const RunFrames& f, int k,
             uint64_t max_rows, const RunDesc* desc, const RunDesc& given, int* bad, int seq, int* flag,
             hipStream_t st);
// Stable LSD radix sort on bits [0, bits) of keys[n], carrying u32 values
// (iota: the values are the positions 0..n-1 and vals is not read).  Ping-pongs
// between (keys, vals) and (keys_alt, vals_alt); *result = 0 or 1 names the
// pair holding the sorted output.  counts: radix_counts_elems(n) u32 of
// scratch.  psg_sort.hip.
uint64_t radix_counts_elems(uint64_t n);
int radix_sort_u32(uint32_t* keys, uint32_t* vals, uint64_t n, int bits, bool iota, uint32_t* keys_alt,
                   uint32_t* vals_alt, uint32_t* counts, hipStream_t st, int* result);
int radix_sort_u64(uint64_t* keys, uint32_t* vals, uint64_t n, int bits, bool iota, uint64_t* keys_alt,
                   uint32_t* vals_alt, uint32_t* counts, hipStream_t st, int* result);
}  // namespace psg
