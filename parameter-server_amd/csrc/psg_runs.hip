// psg_runs.hip — a run of queued requests on interleaved key lists, served in
// one pass over the store.
//
// The reference server takes its queued messages one at a time
// (src/internal/Customer.cpp:52-70) and serves each with its own loop over the
// request's keys (src/ps/KVApp.h:446-454: `store[key] += val` for a Push,
// `res.vals[i] = store[key]` for a Pull).  In the reference benchmark's layout
// (tests/test_kv_app_benchmark.cpp:47-52, tests/test_kv_app.cpp:27) worker r
// sends the keys kMaxKey / num * i + r, so at nw workers every server's store
// holds nw lists interleaved key by key, and each request is every nw-th key of
// the store: on its own it touches every line of the store's keys and values
// (8 nw + 8 nw bytes of lines per key it sends, against 16).  When the requests
// of several workers sit in the queue one behind the other, their lists are
// distinct phases of one period,
//     keys_j[i] == K[D + p_j + P * i],   p_j distinct, 0 <= p_j < P,
// hence pairwise disjoint: each store slot belongs to at most one request, no
// two requests touch one value, and the order of the run changes no result
// (a Pull reads slots no Push of the run writes).  One pass over the rows
// D + P * i + [0, P) then serves the whole run and reads and writes each line
// once:
//     check (a run with Pushes): request key 8 + store key 8   per key
//     apply: Push  value 4 + store 8; Pull  store 4 + reply 4  per key
// i.e. 28 B per pushed key and 24 per pulled key — what one identity request
// moves — for the whole run.
//
// One lane per 16-B chunk of the store's values: every wave instruction on the
// store's keys and values is one contiguous run, and row i of request j is
// element i of its arrays, so the lanes that share a phase read that
// request's keys, values and replies as contiguous runs too (P = 4, f32: one
// lane per row, every request one stream).  The phase -> request map is
// uniform across the block (LDS).
//
// run_classify looks at first keys only (one block, one wave per request); the
// passes verify every key.  A mismatch anywhere makes the apply write nothing
// (the check pass's word), so the caller (psg_store_run) serves the run request
// by request from the store it found.
#include <cstdlib>

#include "psg_internal.h"

namespace psg {

namespace {

__global__ __launch_bounds__(1024) void k_run_classify(const uint64_t* __restrict__ K, uint64_t S, RunFrames f,
                                                       int k, int pl, int allow_same, RunDesc* __restrict__ desc,
                                                       RunSeen* __restrict__ seen, uint64_t* __restrict__ same_base) {
  __shared__ uint64_t pos[kMaxFrames];
  __shared__ int found[kMaxFrames];
  __shared__ uint64_t pos2;
  __shared__ int found2;
  __shared__ RunDesc d;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (w < k) {
    const uint64_t key = f.q[w][0];
    const uint64_t p = lower_bound_wave(K, S, key);
    if (lane == 0) {
      pos[w] = p;
      found[w] = p < S && K[p] == key;
    }
    if (w == pl) {
      const uint64_t key2 = f.q[w][1];
      const uint64_t p2 = lower_bound_wave(K, S, key2);
      if (lane == 0) {
        pos2 = p2;
        found2 = p2 < S && K[p2] == key2;
      }
    }
  }
  if (threadIdx.x < kRunMaxPeriod) d.map[threadIdx.x] = -1;
  __syncthreads();
  if (threadIdx.x == 0) {
    d.D = 0;
    d.rows = 0;
    d.P = 0;
    d.cls = RUN_NONE;
    uint64_t base = UINT64_MAX;
    bool ok = true;
    uint64_t D = UINT64_MAX;
    for (int j = 0; j < k; ++j) {
      ok = ok && found[j];
      D = pos[j] < D ? pos[j] : D;
    }
    if (ok) {
      bool same = allow_same != 0;
      for (int j = 1; j < k; ++j) same = same && pos[j] == pos[0];
      if (same && f.n[0] <= S - pos[0]) {
        d.cls = RUN_SAME;
        d.D = D;
        base = D;
      } else if (pl >= 0 && found2 && pos2 > pos[pl] && pos2 - pos[pl] >= 2 && pos2 - pos[pl] <= kRunMaxPeriod) {
        const uint32_t P = (uint32_t)(pos2 - pos[pl]);
        bool strided = true;
        uint64_t rows = 0, span = 0;
        for (int j = 0; j < k && strided; ++j) {
          const uint64_t p = pos[j] - D;
          if (p >= P || d.map[p] >= 0) {
            strided = false;
            break;
          }
          d.map[p] = (int8_t)j;
          rows = f.n[j] > rows ? f.n[j] : rows;
          const uint64_t last = p + (uint64_t)P * (f.n[j] - 1) + 1;
          span = last > span ? last : span;
        }
        if (strided && span <= S - D && rows < 0xffffffffull) {
          d.cls = RUN_STRIDED;
          d.D = D;
          d.P = P;
          d.rows = rows;
        }
      }
    }
    *same_base = base;
  }
  __syncthreads();
  // the layout for the passes, and a host-readable copy of it with the first
  // keys' slots (psg_store_run caches them per list)
  if (threadIdx.x < sizeof(RunDesc) / 4) {
    reinterpret_cast<int*>(desc)[threadIdx.x] = reinterpret_cast<const int*>(&d)[threadIdx.x];
    reinterpret_cast<int*>(&seen->d)[threadIdx.x] = reinterpret_cast<const int*>(&d)[threadIdx.x];
  }
  if (threadIdx.x < (unsigned)k) {
    seen->pos[threadIdx.x] = pos[threadIdx.x];
    seen->found[threadIdx.x] = found[threadIdx.x];
  }
}

template <int DT, int MODE, int U, int NT>
__global__ __launch_bounds__(256) void k_run_pass(typename Elem<DT>::T* __restrict__ store,
                                                  const uint64_t* __restrict__ K, uint64_t S, RunFrames f,
                                                  const RunDesc* __restrict__ dp, RunDesc given,
                                                  int* __restrict__ bad, int seq, int* __restrict__ flag) {
  using E = Elem<DT>;
  using T = typename E::T;
  constexpr int V = E::kVec;
  // per phase: the request's arrays, its keys, its op (0: no request)
  __shared__ const uint64_t* sq[kRunMaxPeriod];
  __shared__ const T* sv[kRunMaxPeriod];
  __shared__ T* so[kRunMaxPeriod];
  __shared__ uint32_t sn[kRunMaxPeriod];
  __shared__ int sop[kRunMaxPeriod];
  __shared__ int8_t smap[kRunMaxPeriod];
  __shared__ uint64_t sD, srows;
  __shared__ uint32_t sP;
  __shared__ int sgo;
  const RunDesc* d = dp ? dp : &given;
  if (threadIdx.x < kRunMaxPeriod) smap[threadIdx.x] = d->map[threadIdx.x];
  if (threadIdx.x == 0) {
    sD = d->D;
    srows = d->rows;
    sP = d->P;
    int go = d->cls == RUN_STRIDED;
    if (MODE == RUN_APPLY && *bad == seq) go = 0;
    sgo = go;
    if (!go && flag && blockIdx.x == 0) *flag = 1;
  }
  __syncthreads();
  if (!sgo) return;
  if (threadIdx.x < kRunMaxPeriod) {
    const int ph = threadIdx.x;
    const int mj = ph < (int)sP ? smap[ph] : -1;
    const uint64_t* q = nullptr;
    const T* v = nullptr;
    T* o = nullptr;
    uint32_t n = 0;
    int op = 0;
    // compile-time indices into the kernel argument (no private copy of it)
#pragma unroll
    for (int j = 0; j < kMaxFrames; ++j)
      if (j == mj) {
        q = f.q[j];
        v = static_cast<const T*>(f.v[j]);
        o = static_cast<T*>(f.o[j]);
        n = (uint32_t)f.n[j];
        op = f.op[j];
      }
    sq[ph] = q;
    sv[ph] = v;
    so[ph] = o;
    sn[ph] = n;
    sop[ph] = op;
  }
  __syncthreads();
  const uint64_t D = sD, rows = srows;
  const uint32_t P = sP;
  // One lane per 16-B chunk of store values (V slots) over the rows' slots
  // [D, D + P rows): every wave instruction on the store's keys and values is
  // one contiguous run, whatever P.  A chunk's slots are consecutive phases,
  // wrapping into the next row: one division per chunk.  U chunks per lane at
  // a time (kBlock apart, so each wave instruction stays one contiguous run):
  // every load of the U chunks is issued before the first one is used.
  const uint64_t end = D + (uint64_t)P * rows;
  const uint64_t c0 = D / V, c1 = (end + V - 1) / V;
  const uint64_t stride = (uint64_t)gridDim.x * kBlock * U;
  int mismatch = 0;
  for (uint64_t t0 = c0 + (uint64_t)blockIdx.x * kBlock * U + threadIdx.x; t0 < c1; t0 += stride) {
    int ph[U][V], ops[U][V];
    uint32_t rw[U][V];
    bool whole[U], anypush[U];
    uint64_t a0[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const uint64_t t = t0 + (uint64_t)u * kBlock;
      a0[u] = t * V;
      // the phase and row of the chunk's first slot (slots before D: none)
      const uint64_t m0 = a0[u] >= D ? a0[u] - D : 0;
      uint32_t r = (uint32_t)(m0 / P);
      uint32_t p = (uint32_t)(m0 - (uint64_t)r * P);
      anypush[u] = false;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const uint64_t a = a0[u] + e;
        const bool in = t < c1 && a >= D && a < end;
        ph[u][e] = in ? (int)p : 0;
        rw[u][e] = r;
        ops[u][e] = in && r < sn[p] ? sop[p] : 0;
        anypush[u] = anypush[u] || (ops[u][e] & PSG_PUSH);
        if (a >= D && ++p == P) {
          p = 0;
          ++r;
        }
      }
      whole[u] = a0[u] + V <= S;
    }
    // every load of the U chunks first, then the arithmetic, then the writes
    uint64_t kk[U][V], qq[U][V];
    T y[U][V], av[U][V];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      bool anyop = false;
#pragma unroll
      for (int e = 0; e < V; ++e) anyop = anyop || ops[u][e];
      if constexpr (MODE != RUN_APPLY) {
        if (anyop && whole[u]) {
          const u64x2* kp = reinterpret_cast<const u64x2*>(K + a0[u]);
#pragma unroll
          for (int h = 0; h < V / 2; ++h) {
            const u64x2 x = NT ? __builtin_nontemporal_load(kp + h) : kp[h];
            kk[u][2 * h] = x[0];
            kk[u][2 * h + 1] = x[1];
          }
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e) kk[u][e] = ops[u][e] ? K[a0[u] + e] : 0;
        }
#pragma unroll
        for (int e = 0; e < V; ++e)
          qq[u][e] = ops[u][e] ? (NT ? __builtin_nontemporal_load(sq[ph[u][e]] + rw[u][e]) : sq[ph[u][e]][rw[u][e]])
                               : 0;
      }
      if constexpr (MODE != RUN_CHECK) {
        if (anyop && whole[u]) {
          typedef T tv __attribute__((ext_vector_type(V)));
          const tv w = __builtin_bit_cast(tv, *reinterpret_cast<const u32x4*>(store + a0[u]));
#pragma unroll
          for (int e = 0; e < V; ++e) y[u][e] = w[e];
        } else {
#pragma unroll
          for (int e = 0; e < V; ++e) y[u][e] = ops[u][e] ? store[a0[u] + e] : T(0);
        }
#pragma unroll
        for (int e = 0; e < V; ++e)
          av[u][e] = (ops[u][e] & PSG_PUSH)
                         ? (NT ? __builtin_nontemporal_load(sv[ph[u][e]] + rw[u][e]) : sv[ph[u][e]][rw[u][e]])
                         : T(0);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if constexpr (MODE != RUN_APPLY) {
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (ops[u][e] && (qq[u][e] != kk[u][e] || kk[u][e] < f.lo || kk[u][e] >= f.hi)) mismatch = 1;
      }
      if constexpr (MODE != RUN_CHECK) {
        T x[V];
#pragma unroll
        for (int e = 0; e < V; ++e) x[e] = (ops[u][e] & PSG_PUSH) ? E::add1(y[u][e], av[u][e]) : y[u][e];
#pragma unroll
        for (int e = 0; e < V; ++e)
          if (ops[u][e] & PSG_PULL) __builtin_nontemporal_store(x[e], so[ph[u][e]] + rw[u][e]);
        if (MODE == RUN_APPLY && anypush[u]) {
          if (whole[u]) {
            typedef T tv __attribute__((ext_vector_type(V)));
            tv w;
#pragma unroll
            for (int e = 0; e < V; ++e) w[e] = x[e];
            // the chunk's slots no request of the run holds go back unchanged:
            // only this stream writes the store
            *reinterpret_cast<u32x4*>(store + a0[u]) = __builtin_bit_cast(u32x4, w);
          } else {
#pragma unroll
            for (int e = 0; e < V; ++e)
              if (ops[u][e] & PSG_PUSH) store[a0[u] + e] = x[e];
          }
        }
      }
    }
  }
  if constexpr (MODE != RUN_APPLY) {
    if (__ballot(mismatch) && (threadIdx.x & 63) == 0) {
      if (MODE == RUN_CHECK) *bad = seq;
      else if (flag) *flag = 1;
    }
  }
}

template <int DT>
int pass_t(int mode, void* store_vals, const uint64_t* K, uint64_t S, const RunFrames& f, uint64_t max_rows,
           const RunDesc* desc, const RunDesc& given, int* bad, int seq, int* flag, hipStream_t st) {
  using T = typename Elem<DT>::T;
  // one lane per 16-B chunk, grid-strided past the cap: PSG_RUN_BPC blocks of
  // 256 per CU (default 8, the streaming grid; up to 256, i.e. no cap)
  static const int bpc = [] {
    const char* e = getenv("PSG_RUN_BPC");
    const int v = e ? atoi(e) : 0;
    return v >= 1 && v <= 256 ? v : 8;
  }();
  // PSG_RUN_U (A/B): chunks per lane in flight (1 or 2; default 1 — two
  // measured slower, profiles/r6_strided_units_ab.txt); PSG_RUN_NT=0 (A/B):
  // the request arrays and store keys read as plain loads — faster for a run
  // alone (check 0.65 -> 0.72, apply 0.65 -> 0.69, Pull 0.70 -> 0.74 at P = 4)
  // but slower in the drop-in job, where N servers' passes share the chip
  // (0.642 vs 0.585 ms a step at N = 4, profiles/r6_strided_units_ab.txt)
  static const int units = [] {
    const char* e = getenv("PSG_RUN_U");
    return e && atoi(e) == 2 ? 2 : 1;
  }();
  static const int nt = [] {
    const char* e = getenv("PSG_RUN_NT");
    return e && atoi(e) == 0 ? 0 : 1;
  }();
  uint64_t b = (max_rows + (uint64_t)kBlock * units - 1) / ((uint64_t)kBlock * units);
  const uint64_t cap = (uint64_t)max_stream_blocks() / 8 * (uint64_t)bpc;
  if (b > cap) b = cap;
  const unsigned g = b ? (unsigned)b : 1u;
#define PSG_RUN_LAUNCH(M, UU, N) \
  k_run_pass<DT, M, UU, N><<<g, kBlock, 0, st>>>((T*)store_vals, K, S, f, desc, given, bad, seq, flag)
#define PSG_RUN_BY_U(M)                                   \
  do {                                                    \
    if (units == 2) PSG_RUN_LAUNCH(M, 2, 1);              \
    else if (nt) PSG_RUN_LAUNCH(M, 1, 1);                 \
    else PSG_RUN_LAUNCH(M, 1, 0);                         \
  } while (0)
  switch (mode) {
    case RUN_CHECK: PSG_RUN_BY_U(RUN_CHECK); break;
    case RUN_APPLY: PSG_RUN_BY_U(RUN_APPLY); break;
    default: PSG_RUN_BY_U(RUN_PULL_CHECKED); break;
  }
#undef PSG_RUN_BY_U
#undef PSG_RUN_LAUNCH
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

}  // namespace

int run_classify(const uint64_t* K, uint64_t S, const RunFrames& f, int k, int pl, int allow_same, RunDesc* desc,
                 RunSeen* seen, uint64_t* same_base, hipStream_t st) {
  k_run_classify<<<1, 1024, 0, st>>>(K, S, f, k, pl, allow_same, desc, seen, same_base);
  PSG_HIP(hipGetLastError());
  return PSG_OK;
}

int run_pass(int mode, int dtype, void* store_vals, const uint64_t* K, uint64_t S, const RunFrames& f, int k,
             uint64_t max_rows, const RunDesc* desc, const RunDesc& given, int* bad, int seq, int* flag,
             hipStream_t st) {
  (void)k;
  switch (dtype) {
    case PSG_F32: return pass_t<PSG_F32>(mode, store_vals, K, S, f, max_rows, desc, given, bad, seq, flag, st);
    case PSG_F64: return pass_t<PSG_F64>(mode, store_vals, K, S, f, max_rows, desc, given, bad, seq, flag, st);
    case PSG_F16: return pass_t<PSG_F16>(mode, store_vals, K, S, f, max_rows, desc, given, bad, seq, flag, st);
    case PSG_BF16: return pass_t<PSG_BF16>(mode, store_vals, K, S, f, max_rows, desc, given, bad, seq, flag, st);
    default: set_error("unsupported dtype %d", dtype); return PSG_ERR_UNSUPPORTED;
  }
}

}  // namespace psg
