// ps_oracle.cpp — CPU restatement of the reference's KV hot path.
//
// TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
// cpu_baseline leg of bench.py load this library, as the checker / the timed
// CPU baseline.  The product path (parameter-server_amd/) never links, loads or
// calls it.
//
// Each function restates one reference algorithm, cited by file:line in the
// reference repository (SovietPower/Parameter-Server, mounted read-only at
// /root/reference in the build container).  The reference itself cannot be
// built here: every translation unit on its KV path includes Van.h / Message.h
// through PostOffice.h, and the Van implementation needs the protobuf 3.21
// generated code (src/internal/meta.pb.{h,cc}) and libprotobuf, which this
// image does not have.  The restatement is therefore pinned by the
// reference's own known-answer tests (tests/test_kv_app.cpp:20-61,
// tests/test_kv_app_multi_workers.cpp:27-65, tests/test_my.cpp:29-75 and the
// SVector Slice semantics of src/utility/test/SVector_test.cpp:411-462), which
// tests/test_oracle.py replays — see DESIGN.md "Oracle".
//
// The store is a std::unordered_map<uint64_t, V> exactly like
// KVServerDefaultHandle::store (src/ps/KVApp.h:457), so the CPU baseline times
// the reference's own data structure and loop.
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <chrono>
#include <cmath>
#include <unordered_map>
#include <vector>

namespace {

enum { F32 = 0, F64 = 1, F16 = 2, BF16 = 3 };
enum { PUSH = 1, PULL = 2 };

// ---- f16 / bf16 storage with RNE conversions (no _Float16 in g++ 11) -------
inline uint32_t f2u(float f) { uint32_t u; memcpy(&u, &f, 4); return u; }
inline float u2f(uint32_t u) { float f; memcpy(&f, &u, 4); return f; }

inline float half_to_float(uint16_t h) {
  uint32_t s = (uint32_t)(h >> 15) << 31, e = (h >> 10) & 0x1f, m = h & 0x3ff;
  if (e == 0) {
    if (m == 0) return u2f(s);
    float v = std::ldexp((float)m, -24);  // subnormal, exact
    return s ? -v : v;
  }
  if (e == 31) return u2f(s | 0x7f800000u | (m << 13));
  return u2f(s | ((e - 15 + 127) << 23) | (m << 13));
}
inline uint16_t float_to_half(float f) {  // round to nearest even
  uint32_t u = f2u(f), s = (u >> 16) & 0x8000;
  uint32_t a = u & 0x7fffffffu;
  if (a >= 0x7f800000u) return (uint16_t)(s | 0x7c00 | (a > 0x7f800000u ? 0x200 : 0));
  if (a >= 0x477ff000u) return (uint16_t)(s | 0x7c00);  // >= 65520 rounds to inf
  if (a < 0x38800000u) {                                // subnormal or zero in half
    float v = u2f(a);
    float q = v * 16777216.0f;  // units of 2^-24, exact scaling
    float r = std::nearbyint(q);  // RNE (default rounding mode)
    return (uint16_t)(s | (uint32_t)r);
  }
  uint32_t e = (a >> 23) - 127 + 15, m = a & 0x7fffff;
  uint32_t h = (e << 10) | (m >> 13);
  uint32_t rem = m & 0x1fff;
  if (rem > 0x1000 || (rem == 0x1000 && (h & 1))) h++;
  return (uint16_t)(s | h);
}
inline float bf16_to_float(uint16_t b) { return u2f((uint32_t)b << 16); }
inline uint16_t float_to_bf16(float f) {
  uint32_t u = f2u(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  uint32_t r = u + 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(r >> 16);
}

template <int DT> struct Num;
template <> struct Num<F32> {
  typedef float S;
  static S add(S a, S b) { return a + b; }
  static S zero() { return 0.0f; }
  static S from_double(double v) { return (float)v; }
};
template <> struct Num<F64> {
  typedef double S;
  static S add(S a, S b) { return a + b; }
  static S zero() { return 0.0; }
  static S from_double(double v) { return v; }
};
template <> struct Num<F16> {
  typedef uint16_t S;
  static S add(S a, S b) { return float_to_half(half_to_float(a) + half_to_float(b)); }
  static S zero() { return 0; }
  static S from_double(double v) { return float_to_half((float)v); }
};
template <> struct Num<BF16> {
  typedef uint16_t S;
  static S add(S a, S b) { return float_to_bf16(bf16_to_float(a) + bf16_to_float(b)); }
  static S zero() { return 0; }
  static S from_double(double v) { return float_to_bf16((float)v); }
};

struct StoreBase {
  int dtype;
  virtual ~StoreBase() {}
};
template <int DT>
struct Store : StoreBase {
  typedef typename Num<DT>::S S;
  std::unordered_map<uint64_t, S> store;
};

// KVServerDefaultHandle<V>::operator() (src/ps/KVApp.h:435-456): one request,
// in key order, `store[key] += vals[i]` then `res.vals[i] = store[key]`.
template <int DT>
void handle(Store<DT>* st, int flags, const uint64_t* keys, uint64_t first_key, const void* vals,
            void* out, uint64_t n) {
  typedef typename Num<DT>::S S;
  const S* v = (const S*)vals;
  S* o = (S*)out;
  auto& store = st->store;
  for (uint64_t i = 0; i < n; ++i) {
    const uint64_t key = keys ? keys[i] : first_key + i;
    if (flags & PUSH) {
      S& ref = store[key];  // operator[] inserts 0 on first touch (KVApp.h:449)
      ref = Num<DT>::add(ref, v[i]);
    }
    if (flags & PULL) o[i] = store[key];  // inserts 0 for an absent key (KVApp.h:452)
  }
}

inline uint64_t splitmix64(uint64_t x) {
  x += 0x9e3779b97f4a7c15ull;
  x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
  x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}

// All (key, value) pairs sorted by key.
template <int DT>
void dump_t(Store<DT>* st, uint64_t* keys, void* vals) {
  typedef typename Num<DT>::S S;
  std::vector<std::pair<uint64_t, S>> kv(st->store.begin(), st->store.end());
  std::sort(kv.begin(), kv.end(), [](const auto& a, const auto& b) { return a.first < b.first; });
  S* v = (S*)vals;
  for (size_t i = 0; i < kv.size(); ++i) {
    keys[i] = kv[i].first;
    v[i] = kv[i].second;
  }
}
}  // namespace

extern "C" {

void* oracle_store_new(int dtype) {
  StoreBase* s = nullptr;
  switch (dtype) {
    case F32: s = new Store<F32>(); break;
    case F64: s = new Store<F64>(); break;
    case F16: s = new Store<F16>(); break;
    case BF16: s = new Store<BF16>(); break;
    default: return nullptr;
  }
  s->dtype = dtype;
  return s;
}

void oracle_store_free(void* s) { delete (StoreBase*)s; }

void oracle_store_reserve(void* s, uint64_t n) {
  StoreBase* b = (StoreBase*)s;
  switch (b->dtype) {
    case F32: ((Store<F32>*)b)->store.reserve(n); break;
    case F64: ((Store<F64>*)b)->store.reserve(n); break;
    case F16: ((Store<F16>*)b)->store.reserve(n); break;
    case BF16: ((Store<BF16>*)b)->store.reserve(n); break;
  }
}

// keys == NULL: consecutive keys first_key + i.  Values are raw element bits of
// the dtype (f16 / bf16 as uint16).
int oracle_handle(void* s, int flags, const uint64_t* keys, uint64_t first_key, const void* vals,
                  void* out, uint64_t n) {
  StoreBase* b = (StoreBase*)s;
  if (!b || flags < 1 || flags > 3) return 1;
  switch (b->dtype) {
    case F32: handle<F32>((Store<F32>*)b, flags, keys, first_key, vals, out, n); break;
    case F64: handle<F64>((Store<F64>*)b, flags, keys, first_key, vals, out, n); break;
    case F16: handle<F16>((Store<F16>*)b, flags, keys, first_key, vals, out, n); break;
    case BF16: handle<BF16>((Store<BF16>*)b, flags, keys, first_key, vals, out, n); break;
    default: return 1;
  }
  return 0;
}

uint64_t oracle_store_size(void* s) {
  StoreBase* b = (StoreBase*)s;
  switch (b->dtype) {
    case F32: return ((Store<F32>*)b)->store.size();
    case F64: return ((Store<F64>*)b)->store.size();
    case F16: return ((Store<F16>*)b)->store.size();
    case BF16: return ((Store<BF16>*)b)->store.size();
  }
  return 0;
}

void oracle_store_dump(void* s, uint64_t* keys, void* vals) {
  StoreBase* b = (StoreBase*)s;
  switch (b->dtype) {
    case F32: dump_t((Store<F32>*)b, keys, vals); break;
    case F64: dump_t((Store<F64>*)b, keys, vals); break;
    case F16: dump_t((Store<F16>*)b, keys, vals); break;
    case BF16: dump_t((Store<BF16>*)b, keys, vals); break;
  }
}

// PostOffice::GetServerRanges (src/internal/PostOffice.cpp:211-221).
void oracle_server_ranges(int ns, uint64_t* begins, uint64_t* ends) {
  const uint64_t kMaxKey = UINT64_MAX;
  for (int i = 0; i < ns; ++i) {
    begins[i] = kMaxKey / ns * i;
    ends[i] = i != ns - 1 ? kMaxKey / ns * (i + 1) : kMaxKey;
  }
}

// KVWorker<V>::DefaultSlicer (src/ps/KVApp.h:515-574).  Returns 0, or 1 when
// a reference CHECK would throw (non-adjacent ranges :531, keys past the last
// range :544, vals not a multiple of keys :551, lens size :553).
// key_pos[ns+1]; val_pos[ns+1]: start/end offsets of each slice's values.
int oracle_slice(const uint64_t* keys, uint64_t n, const int* lens, uint64_t nlens,
                 uint64_t num_vals, int ns, const uint64_t* begins, const uint64_t* ends,
                 uint64_t* key_pos, uint64_t* val_pos) {
  std::vector<size_t> pos(ns + 1);
  const uint64_t* begin = keys;
  const uint64_t* end = keys + n;
  for (int i = 0; i < ns; ++i) {
    if (i == 0) {
      pos[0] = std::lower_bound(begin, end, begins[0]) - begin;
      begin += pos[0];
    } else if (ends[i - 1] != begins[i]) {
      return 1;
    }
    size_t len = std::lower_bound(begin, end, ends[i]) - begin;
    begin += len;
    pos[i + 1] = pos[i] + len;
  }
  if (pos[ns] != n) return 1;
  for (int i = 0; i <= ns; ++i) key_pos[i] = pos[i];
  if (n == 0) {
    for (int i = 0; i <= ns; ++i) val_pos[i] = 0;
    return 0;
  }
  uint64_t k = 0, val_begin = 0, val_end = 0;
  if (nlens == 0) {
    k = num_vals / n;
    if (k * n != num_vals) return 1;
  } else if (nlens != n) {
    return 1;
  }
  // val_pos[i] = start of slice i; an empty slice starts where the previous ended
  for (int i = 0; i < ns; ++i) {
    if (nlens) {
      val_pos[i] = val_begin;
      for (size_t j = pos[i]; j < pos[i + 1]; ++j) val_end += (uint64_t)lens[j];
      val_begin = val_end;
    } else {
      val_pos[i] = pos[i] * k;
    }
  }
  val_pos[ns] = nlens ? val_end : pos[ns] * k;
  return 0;
}

// The AddPullCB merge (src/ps/KVApp.h:680-720): replies sorted by first key,
// values concatenated.  Returns 1 when the totals do not match (:691, :701).
int oracle_merge(int nsegs, const void* const* seg_vals, const uint64_t* seg_counts,
                 const uint64_t* seg_first_keys, int elem_size, void* dst, uint64_t dst_count) {
  std::vector<int> order(nsegs);
  uint64_t total = 0;
  for (int i = 0; i < nsegs; ++i) {
    order[i] = i;
    total += seg_counts[i];
  }
  if (total != dst_count) return 1;
  std::sort(order.begin(), order.end(),
            [&](int a, int b) { return seg_first_keys[a] < seg_first_keys[b]; });
  char* p = (char*)dst;
  for (int i : order) {
    memcpy(p, seg_vals[i], seg_counts[i] * elem_size);
    p += seg_counts[i] * elem_size;
  }
  return 0;
}

// LRServer sync apply + Adam (tests/src/LRServer.h:171-177, tests/src/Adam.h:28-34),
// same types and operation order.  m, v may be NULL (no Adam).
void oracle_lr_apply(float* weight, const float* merged, uint64_t n, float learning_rate,
                     double* m, double* v, double adam_lr, double beta1, double beta2,
                     double epsilon, int iteration) {
  for (uint64_t i = 0; i < n; ++i) {
    double grad = learning_rate * merged[i];
    if (m) {
      m[i] = beta1 * m[i] + (1 - beta1) * grad;
      v[i] = beta2 * v[i] + (1 - beta2) * grad * grad;
      double m_hat = m[i] / (1 - std::pow(beta1, iteration + 1));
      double v_hat = v[i] / (1 - std::pow(beta2, iteration + 1));
      grad = adam_lr * m_hat / (std::sqrt(v_hat) + epsilon);
    }
    weight[i] -= grad;
  }
}

// The device generator psg_fill_synth, restated (element i depends on seed, i).
void oracle_synth(void* out, uint64_t n, int dtype, uint64_t seed, int mode, double lo,
                  double hi) {
  const double inv24 = 1.0 / 16777216.0;
  for (uint64_t i = 0; i < n; ++i) {
    uint64_t r = splitmix64(seed + i) >> 40;
    double x = mode == 0 ? std::floor((double)r * (hi - lo) * inv24) + lo
                         : lo + ((double)r * inv24) * (hi - lo);
    switch (dtype) {
      case F32: ((float*)out)[i] = (float)x; break;
      case F64: ((double*)out)[i] = x; break;
      case F16: ((uint16_t*)out)[i] = float_to_half((float)x); break;
      case BF16: ((uint16_t*)out)[i] = float_to_bf16((float)x); break;
    }
  }
}

// glibc srand/rand, as the reference tests draw their values
// (tests/test_kv_app.cpp:26-30: srand(rank + 7); vals[i] = rand() % 1000).
void oracle_glibc_rand_mod(int seed, int mod, uint64_t n, float* out) {
  srand((unsigned)seed);
  for (uint64_t i = 0; i < n; ++i) out[i] = (float)(rand() % mod);
}

// CPU baseline: the reference handler on the test_kv_app_benchmark layout
// (tests/test_kv_app_benchmark.cpp:43-52, keys kMaxKey/num*i + rank) — one
// inserting Push, then `reps` steady Push and Pull requests, single thread (the
// reference runs ReqHandle on one Customer thread, src/internal/Customer.cpp:52-70).
// Times in seconds per request.
void oracle_bench(uint64_t num, int reps, double* first_push_s, double* push_s, double* pull_s) {
  std::vector<uint64_t> keys(num);
  std::vector<float> vals(num), out(num);
  srand(7);
  for (uint64_t i = 0; i < num; ++i) {
    keys[i] = UINT64_MAX / num * i;
    vals[i] = (float)(rand() % 1000);
  }
  Store<F32> st;
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  handle<F32>(&st, PUSH, keys.data(), 0, vals.data(), nullptr, num);
  auto t1 = clk::now();
  *first_push_s = std::chrono::duration<double>(t1 - t0).count();
  double tp = 0, tl = 0;
  for (int r = 0; r < reps; ++r) {
    auto a = clk::now();
    handle<F32>(&st, PUSH, keys.data(), 0, vals.data(), nullptr, num);
    auto b = clk::now();
    handle<F32>(&st, PULL, keys.data(), 0, nullptr, out.data(), num);
    auto c = clk::now();
    tp += std::chrono::duration<double>(b - a).count();
    tl += std::chrono::duration<double>(c - b).count();
  }
  *push_s = reps ? tp / reps : 0;
  *pull_s = reps ? tl / reps : 0;
}

// CPU baseline on the GPU bench's own workload (configs[1]): keys
// key_base + i * key_step (step 1: the DENSE layout, keys 0..num-1 of server
// 0's range) and the bench's integer-valued synthetic values (seed, 0..999).
// Same handler and timing split as oracle_bench.
void oracle_bench_layout(uint64_t num, int reps, uint64_t key_base, uint64_t key_step,
                         uint64_t seed, double* first_push_s, double* push_s, double* pull_s) {
  std::vector<uint64_t> keys(num);
  std::vector<float> vals(num), out(num);
  for (uint64_t i = 0; i < num; ++i) keys[i] = key_base + i * key_step;
  oracle_synth(vals.data(), num, F32, seed, 0, 0.0, 1000.0);
  Store<F32> st;
  using clk = std::chrono::steady_clock;
  auto t0 = clk::now();
  handle<F32>(&st, PUSH, keys.data(), 0, vals.data(), nullptr, num);
  auto t1 = clk::now();
  *first_push_s = std::chrono::duration<double>(t1 - t0).count();
  double tp = 0, tl = 0;
  for (int r = 0; r < reps; ++r) {
    auto a = clk::now();
    handle<F32>(&st, PUSH, keys.data(), 0, vals.data(), nullptr, num);
    auto b = clk::now();
    handle<F32>(&st, PULL, keys.data(), 0, nullptr, out.data(), num);
    auto c = clk::now();
    tp += std::chrono::duration<double>(b - a).count();
    tl += std::chrono::duration<double>(c - b).count();
  }
  *push_s = reps ? tp / reps : 0;
  *pull_s = reps ? tl / reps : 0;
}

}  // extern "C"
