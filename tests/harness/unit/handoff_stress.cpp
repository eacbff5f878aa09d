// handoff_stress.cpp — does a reply handed out by the store's completion wait
// really hold the request's values?  (GPUTEST_r03: the LR handle's Pull reply,
// copied to the host right after psg_store_sync returned, held the values of
// an EARLIER reply over a tail of the buffer.)
//
// Each iteration updates the store so that every value has a known new value,
// pulls into ONE reply buffer, waits the way a server does before answering,
// and copies the reply to pageable host memory on the same stream — the
// sequence of KVServerLRHandle's Pull (ps/lr_handle.h) and of
// KVServerDefaultHandle's Pulls (ps/kv_app.h).  Every element is checked; any
// stale element is counted.
//
//   handoff_stress dense   <n> <iters> [threads]  DENSE store: handle, psg_store_sync
//   handoff_stress stretch <n> <iters> [threads]  SORTED store, psg_store_handle_stretch,
//                                                 psg_store_sync (the cached-list path)
//   handoff_stress keyed   <n> <iters> [threads]  SORTED store, a synchronous keyed
//                                                 PushPull: psg_store_handle's own wait
//   handoff_stress lr      <n> <iters> [threads]  KVServerLRHandle's BSP round exactly:
//                                                 three gradient frames copied in from
//                                                 pageable memory, psg_lr_apply_sum,
//                                                 psg_store_sync, the Pull, psg_store_sync,
//                                                 the reply out to pageable memory
// threads > 1 runs that many independent copies at once, each on its own
// stream and store (the thread-mode cluster: every node a thread).
// Prints "HANDOFF <mode> n=<n> iters=<iters> threads=<t> stale_iters=<k>
// stale_elems=<m>" and exits 0 when nothing was stale, 3 otherwise.
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "psg.h"

#define CK(x)                                                                       \
  do {                                                                              \
    int rc_ = (x);                                                                  \
    if (rc_ != PSG_OK) {                                                            \
      std::fprintf(stderr, "%s:%d %s -> %d: %s\n", __FILE__, __LINE__, #x, rc_,    \
                   psg_last_error());                                               \
      std::exit(2);                                                                 \
    }                                                                               \
  } while (0)

namespace {
std::atomic<int> g_stale_iters{0};
std::atomic<uint64_t> g_stale_elems{0};
std::mutex g_mu;
std::string g_first;

void Run(const std::string& mode, uint64_t n, int iters) {
  CK(psg_set_device(0));
  psg_stream st = nullptr;
  CK(psg_stream_create(&st));
  void *ones = nullptr, *out = nullptr, *keys = nullptr;
  CK(psg_malloc(&ones, n * 4));
  CK(psg_malloc(&out, n * 4));
  {
    std::vector<float> h(n, 1.0f);
    CK(psg_memcpy(ones, h.data(), n * 4, 0, st));
    std::vector<float> z(n, -1.0f);
    CK(psg_memcpy(out, z.data(), n * 4, 0, st));
    CK(psg_stream_sync(st));
  }
  psg_store* s = nullptr;
  // lr: three gradient frames of dyadic values (k + 1) / 64, merged 6 / 64 =
  // 3 / 32 per round; with lr = 1 every weight is exactly -(it + 1) * 3 / 32
  std::vector<std::vector<float>> grad_host;
  void* frames[3] = {nullptr, nullptr, nullptr};
  if (mode == "lr") {
    for (int k = 0; k < 3; ++k) {
      grad_host.emplace_back(n, (float)(k + 1) / 64.0f);
      CK(psg_malloc(&frames[k], n * 4));
    }
  }
  if (mode == "dense" || mode == "lr") {
    CK(psg_store_create(PSG_STORE_DENSE, PSG_F32, 0, n, n, &s));
  } else {
    CK(psg_store_create(PSG_STORE_SORTED, PSG_F32, 0, ~0ull, 0, &s));
    std::vector<uint64_t> hk(n);
    for (uint64_t i = 0; i < n; ++i) hk[i] = 1000 + 3 * i;
    CK(psg_malloc(&keys, n * 8));
    CK(psg_memcpy(keys, hk.data(), n * 8, 0, st));
    CK(psg_stream_sync(st));
    // insert every key with 0: a Pull of absent keys inserts them (KVApp.h:452)
    CK(psg_store_handle(s, PSG_PULL, (const uint64_t*)keys, 0, nullptr, out, n, st));
    CK(psg_stream_sync(st));
  }
  uint64_t first = 0;
  void* slots = nullptr;
  if (mode == "stretch") {
    CK(psg_malloc(&slots, n * 4));
    CK(psg_store_resolve(s, (const uint64_t*)keys, n, 0, (uint32_t*)slots, st));
    CK(psg_store_slots_stretch(s, (const uint32_t*)slots, n, &first, st));
    if (first == UINT64_MAX) {
      std::fprintf(stderr, "the key list is not a stretch of the store\n");
      std::exit(2);
    }
    CK(psg_stream_sync(st));
  }
  std::vector<float> host(n);
  for (int it = 0; it < iters; ++it) {
    const float want = mode == "lr" ? -(float)(it + 1) * 3.0f / 32.0f : (float)(it + 1);
    if (mode == "lr") {
      for (int k = 0; k < 3; ++k) {  // detail::ToDevice of each worker's frame
        CK(psg_memcpy(frames[k], grad_host[k].data(), n * 4, 0, st));
        CK(psg_stream_sync(st));
      }
      const float* g[3] = {(const float*)frames[0], (const float*)frames[1], (const float*)frames[2]};
      CK(psg_lr_apply_sum(s, g, 3, 1, n, 1.0f, nullptr, 0, st));
      CK(psg_store_sync(s, st));
      CK(psg_store_handle(s, PSG_PULL, nullptr, 0, nullptr, out, n, st));
      CK(psg_store_sync(s, st));
    } else if (mode == "dense") {
      CK(psg_store_handle(s, PSG_PUSH, nullptr, 0, ones, nullptr, n, st));
      CK(psg_store_handle(s, PSG_PULL, nullptr, 0, nullptr, out, n, st));
      CK(psg_store_sync(s, st));
    } else if (mode == "stretch") {
      CK(psg_store_handle_stretch(s, PSG_PUSH | PSG_PULL, first, ones, out, n, st));
      CK(psg_store_sync(s, st));
    } else {
      CK(psg_store_handle(s, PSG_PUSH | PSG_PULL, (const uint64_t*)keys, 0, ones, out, n, st));
    }
    // the server's answer: the reply to the host (detail::ToHost)
    CK(psg_memcpy(host.data(), out, n * 4, 1, st));
    CK(psg_stream_sync(st));
    uint64_t bad = 0, first_bad = 0;
    for (uint64_t i = 0; i < n; ++i) {
      if (host[i] != want) {
        if (bad == 0) first_bad = i;
        ++bad;
      }
    }
    if (bad) {
      if (g_stale_iters.fetch_add(1) == 0) {
        std::lock_guard<std::mutex> lk(g_mu);
        char buf[160];
        std::snprintf(buf, sizeof(buf), " first: iter=%d index=%llu got=%g want=%g", it,
                      (unsigned long long)first_bad, host[first_bad], want);
        g_first = buf;
      }
      g_stale_elems += bad;
    }
  }
  CK(psg_store_destroy(s));
  for (void* p : {ones, out, keys, slots, frames[0], frames[1], frames[2]}) CK(psg_free(p));
  CK(psg_stream_destroy(st));
}
}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    std::fprintf(stderr, "usage: handoff_stress dense|stretch|keyed|lr <n> <iters> [threads]\n");
    return 1;
  }
  const std::string mode = argv[1];
  const uint64_t n = std::strtoull(argv[2], nullptr, 10);
  const int iters = std::atoi(argv[3]);
  const int threads = argc > 4 ? std::atoi(argv[4]) : 1;
  if (n == 0 || iters <= 0 || threads < 1 || threads > 16 ||
      (mode != "dense" && mode != "stretch" && mode != "keyed" && mode != "lr")) {
    std::fprintf(stderr, "bad arguments\n");
    return 1;
  }
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) ts.emplace_back(Run, mode, n, iters);
  for (auto& t : ts) t.join();
  std::printf("HANDOFF %s n=%llu iters=%d threads=%d stale_iters=%d stale_elems=%llu%s\n", mode.c_str(),
              (unsigned long long)n, iters, threads, g_stale_iters.load(),
              (unsigned long long)g_stale_elems.load(), g_first.c_str());
  std::fflush(stdout);
  return g_stale_iters.load() ? 3 : 0;
}
