// device.cc — GPU plumbing of the host runtime, all through the psg C-ABI.
#include "internal/device.h"

#include <sys/mman.h>

#include <algorithm>
#include <condition_variable>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "internal/PostOffice.h"
#include "internal/shm_pool.h"
#include "ps/log.h"
#include "ps/svector.h"

namespace ps {
namespace device {

void Check(int rc, const char* what) {
  if (rc != PSG_OK) ps_log::LogMessageFatal(__FILE__, __LINE__).stream() << what << ": " << psg_last_error();
}

int Count() {
  static int n = [] {
    int c = 0;
    if (psg_device_count(&c) != PSG_OK) c = 0;
    return c;
  }();
  return n;
}

void Use(int dev) {
  if (dev < 0) return;
  Check(psg_set_device(dev), "psg_set_device");
}

namespace {
// Streams live as long as the process: destroying them from thread_local
// destructors could run after the HIP runtime has been torn down.
struct ThreadStreams {
  std::map<int, psg_stream> by_dev;
};
thread_local ThreadStreams t_streams;

// Caching HBM pool: freed blocks are kept per (device, rounded size) and
// reused, so per-request reply / staging buffers cost no hipMalloc after
// warm-up.  Sizes round up to 64 KiB granules (or the next power of two
// above 64 MiB).
struct Pool {
  std::mutex mu;
  std::map<std::pair<int, size_t>, std::vector<void*>> free;
  std::map<size_t, bool> pinning;   // a block of this class is being pinned
  static size_t Round(size_t b) {
    if (b <= (64u << 20)) return (b + 65535) & ~size_t(65535);
    size_t r = size_t(64) << 20;
    while (r < b) r <<= 1;
    return r;
  }
};
Pool& GlobalPool() {
  static Pool* p = new Pool();  // never destroyed: blocks may outlive static teardown
  return *p;
}
}  // namespace

psg_stream ThreadStream() {
  int dev = 0;
  Check(psg_get_device(&dev), "psg_get_device");
  auto it = t_streams.by_dev.find(dev);
  if (it != t_streams.by_dev.end()) return it->second;
  psg_stream s = nullptr;
  // A worker's thread stream is of high priority (PS_WORKER_STREAM_PRIORITY=0:
  // the default): its kernels are the slicer's bounds and the merges, a few
  // microseconds each, on every request's critical path, while the servers'
  // store kernels run for tens — nodes run as threads of one process share
  // its few hardware queues (GPU_MAX_HW_QUEUES), and a bounds kernel queued
  // behind a store kernel waits for it.
  static const bool prio_on = [] {
    const char* e = std::getenv("PS_WORKER_STREAM_PRIORITY");
    return !(e && std::atoi(e) == 0);
  }();
  PostOffice* po = PostOffice::GetIfBound();
  if (prio_on && po && po->is_worker())
    Check(psg_stream_create_priority(&s, 1), "psg_stream_create_priority");
  else
    Check(psg_stream_create(&s), "psg_stream_create");
  t_streams.by_dev[dev] = s;
  return s;
}

std::shared_ptr<void> Alloc(size_t bytes, int dev) {
  CHECK_GE(dev, 0) << "device allocation without a GPU";
  if (bytes == 0) return nullptr;
  Pool& pool = GlobalPool();
  const size_t rb = Pool::Round(bytes);
  void* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(pool.mu);
    auto& fl = pool.free[{dev, rb}];
    if (!fl.empty()) {
      p = fl.back();
      fl.pop_back();
    }
  }
  // PS_POOL_POISON=1 (tests): a block handed out again is first filled with
  // 0xff bytes (NaN floats), synchronously, so a reader that overtakes the
  // block's next writer sees NaN instead of the plausible values it held
  static const bool poison = [] {
    const char* e = std::getenv("PS_POOL_POISON");
    return e && std::atoi(e) != 0;
  }();
  int cur = 0;
  if (!p || poison) Check(psg_get_device(&cur), "psg_get_device");
  if (!p) {
    if (cur != dev) Use(dev);
    int rc = psg_malloc(&p, rb);
    if (cur != dev) Use(cur);
    Check(rc, "psg_malloc");
  } else if (poison) {
    if (cur != dev) Use(dev);
    psg_stream s = ThreadStream();
    Check(psg_memset(p, 0xff, rb, s), "psg_memset(poison)");
    Check(psg_stream_sync(s), "psg_stream_sync");
    if (cur != dev) Use(cur);
  }
  return std::shared_ptr<void>(p, [dev, rb](void* q) {
    Pool& pl = GlobalPool();
    std::lock_guard<std::mutex> lk(pl.mu);
    pl.free[{dev, rb}].push_back(q);
  });
}

// Pinned host blocks for large host arrays (>= 1 MiB): H2D / D2H of such a
// frame then runs without the runtime's pageable staging.  Pooled like the HBM
// blocks (device key -1).  Opt-in (PS_PINNED_HOST=1) since round 5: a size
// class is pinned in the background the first time it is seen, and that
// hipHostMalloc slowed the very copy it was meant to help — the cold 120 MB
// Push of test_kv_app_benchmark took 26-35 ms with it and 2.2-2.7 ms without
// (profiles/r5_dropin_variants.txt).  Host frames rarely reach the GPU now:
// a worker stages its vectors into HBM itself once its servers take HBM
// frames, and every host <-> HBM copy of the runtime goes through its own
// pinned staging blocks (StageToDevice / StageToHost).
std::shared_ptr<void> HostAlloc(size_t bytes) {
  // process mode: large host arrays live in shared memory, so a frame to a
  // peer process is a mapping (internal/shm_pool.h)
  if (shm::Enabled()) {
    if (auto p = shm::Alloc(bytes)) return p;
  }
  static const bool enabled = [] {
    const char* e = std::getenv("PS_PINNED_HOST");
    return Count() > 0 && e && std::atoi(e) != 0;
  }();
  if (!enabled || bytes < (1u << 20)) return nullptr;
  Pool& pool = GlobalPool();
  const size_t rb = Pool::Round(bytes);
  void* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(pool.mu);
    auto& fl = pool.free[{-1, rb}];
    if (!fl.empty()) {
      p = fl.back();
      fl.pop_back();
    } else {
      // pinning costs far more than one copy and must not stall a request:
      // the size class gets a block pinned in the background, which a later
      // request of that size picks up (a training loop); this one stays
      // pageable (a one-shot Push, test_kv_app_benchmark's repeat = 1)
      if (!pool.pinning[rb]) {
        pool.pinning[rb] = true;
        std::thread([rb] {
          void* q = nullptr;
          const bool ok = psg_host_alloc(&q, rb) == PSG_OK;
          Pool& pl = GlobalPool();
          std::lock_guard<std::mutex> lk2(pl.mu);
          if (ok) pl.free[{-1, rb}].push_back(q);
          pl.pinning[rb] = false;
        }).detach();
      }
      return nullptr;
    }
  }
  return std::shared_ptr<void>(p, [rb](void* q) {
    Pool& pl = GlobalPool();
    std::lock_guard<std::mutex> lk(pl.mu);
    pl.free[{-1, rb}].push_back(q);
  });
}

// Heap blocks of >= 4 MiB on transparent huge pages, recycled: a block freed
// by its last SVector goes back to a pool by size class (2 MiB steps) instead
// of to the kernel, so the next frame of that size is already faulted in.  A
// fresh block costs its first touch — 2 MiB faults, spread over the copy
// threads of HostCopy / HostZero (120 MB: ~2 ms on the GPU host against ~10 ms
// on 4 KiB pages, profiles/r5_probe_host_faults.txt) — and a freed one that
// would take the pool past PS_HOST_POOL_MB (default 1024) is returned.  A
// request takes the smallest pooled block of its size up to twice it, so
// frames of varying sizes share blocks instead of each pinning its own class.
namespace {
struct HugePool {
  std::mutex mu;
  std::map<size_t, std::vector<void*>> free;
  size_t held = 0;
  size_t cap = [] {
    const char* e = std::getenv("PS_HOST_POOL_MB");
    const long v = e ? std::atol(e) : 1024;
    return (size_t)(v < 0 ? 0 : v) << 20;
  }();
};
HugePool& Huge() {
  static HugePool* p = new HugePool();  // never destroyed: blocks may outlive static teardown
  return *p;
}
}  // namespace

std::shared_ptr<void> HugeAlloc(size_t bytes) {
  constexpr size_t kHuge = size_t(2) << 20;
  if (bytes < 2 * kHuge) return nullptr;
  size_t rb = (bytes + kHuge - 1) & ~(kHuge - 1);
  HugePool& hp = Huge();
  void* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(hp.mu);
    for (auto it = hp.free.lower_bound(rb); it != hp.free.end() && it->first <= 2 * rb; ++it) {
      if (it->second.empty()) continue;
      p = it->second.back();
      it->second.pop_back();
      hp.held -= it->first;
      rb = it->first;  // the block's own class goes back with it
      break;
    }
  }
  if (!p) {
    p = std::aligned_alloc(kHuge, rb);
    if (!p) return nullptr;
    (void)madvise(p, rb, MADV_HUGEPAGE);
  }
  return std::shared_ptr<void>(p, [rb](void* q) {
    HugePool& pl = Huge();
    {
      std::lock_guard<std::mutex> lk(pl.mu);
      if (pl.held + rb <= pl.cap) {
        pl.free[rb].push_back(q);
        pl.held += rb;
        return;
      }
    }
    std::free(q);
  });
}

void EnableAllPeerAccess() {
  const int n = Count();
  for (int a = 0; a < n; ++a)
    for (int b = 0; b < n; ++b)
      if (a != b) Check(psg_enable_peer_access(a, b), "psg_enable_peer_access");
}

namespace {
// One copy by the runtime on the thread stream, waited for.
void RuntimeCopy(void* dst, const void* src, size_t bytes, int kind) {
  psg_stream s = ThreadStream();
  // a few bytes out of HBM (a hashed key list's one key): through a pinned
  // per-thread word, not a pageable destination the runtime stages itself
  constexpr size_t kSmall = 64;
  thread_local void* small = nullptr;
  if (kind == 1 && bytes <= kSmall) {
    if (!small && psg_host_alloc(&small, kSmall) != PSG_OK) small = nullptr;
    if (small) {
      Check(psg_memcpy(small, src, bytes, kind, s), "psg_memcpy");
      Check(psg_stream_sync(s), "psg_stream_sync");
      std::memcpy(dst, small, bytes);
      return;
    }
  }
  Check(psg_memcpy(dst, src, bytes, kind, s), "psg_memcpy");
  Check(psg_stream_sync(s), "psg_stream_sync");
}
}  // namespace

// Host <-> HBM copies of request and reply frames go through this runtime's
// own pinned staging blocks (StageToDevice / StageToHost: a DMA into or out of
// a pinned block, an event waited for, a host memcpy), not the HIP runtime's
// pageable-memory path: what the host reads is then exactly what the DMA
// wrote once its event completed.  (A hardening step: the runtime's pageable
// staging is not ours to reason about.  GPUTEST_r03's stale LR reply, first
// blamed on it, was the reference LRServer's own constructor race —
// LRServer.h:70 vs 81-87, DESIGN.md "Parity".)
void CopySync(void* dst, const void* src, size_t bytes, int kind) {
  if (!bytes) return;
  if (kind == 0 && bytes > 64) return StageToDevice(dst, src, bytes);
  if (kind == 1 && bytes > 64) return StageToHost(dst, src, bytes);
  RuntimeCopy(dst, src, bytes, kind);
}

namespace {
// Two pinned staging blocks per thread and the events that tell when the DMA
// out of / into each one is done.  A thread that ends hands them to a global
// free list (no HIP call at thread exit, which may come after the runtime's
// teardown), and the next thread that stages takes them from there.
constexpr size_t kStageChunk = size_t(16) << 20;
struct StagePair {
  void* block[2] = {nullptr, nullptr};
  psg_event done[2] = {nullptr, nullptr};
};
std::mutex g_stage_mu;
std::vector<StagePair>* g_stage_free = new std::vector<StagePair>();  // never destroyed

struct Staging {
  StagePair p;
  bool pending[2] = {false, false};
  bool ok = false;
  bool tried = false;
  ~Staging() {
    if (!ok) return;
    std::lock_guard<std::mutex> lk(g_stage_mu);
    g_stage_free->push_back(p);
  }
};
thread_local Staging t_stage;

Staging* GetStaging() {
  Staging& st = t_stage;
  if (!st.tried) {
    st.tried = true;
    {
      std::lock_guard<std::mutex> lk(g_stage_mu);
      if (!g_stage_free->empty()) {
        st.p = g_stage_free->back();
        g_stage_free->pop_back();
        st.ok = true;
      }
    }
    if (!st.ok) {
      st.ok = true;
      for (int b = 0; b < 2 && st.ok; ++b)
        st.ok = psg_host_alloc(&st.p.block[b], kStageChunk) == PSG_OK && psg_event_create(&st.p.done[b]) == PSG_OK;
    }
  }
  return st.ok ? &st : nullptr;
}
}  // namespace

void StageToDevice(void* dst_dev, const void* src_host, size_t bytes) {
  if (!bytes) return;
  psg_stream s = ThreadStream();
  Staging* st = GetStaging();
  if (!st) {  // no pinned memory: the runtime's own pageable path
    RuntimeCopy(dst_dev, src_host, bytes, 0);
    return;
  }
  int b = 0;
  for (size_t off = 0; off < bytes; off += kStageChunk, b ^= 1) {
    const size_t len = std::min(kStageChunk, bytes - off);
    if (st->pending[b]) Check(psg_event_sync(st->p.done[b]), "psg_event_sync");  // block b's last DMA
    HostCopy(st->p.block[b], (const char*)src_host + off, len);
    Check(psg_memcpy((char*)dst_dev + off, st->p.block[b], len, 0, s), "psg_memcpy H2D");
    Check(psg_event_record(st->p.done[b], s), "psg_event_record");
    st->pending[b] = true;
  }
  Check(psg_stream_sync(s), "psg_stream_sync");
  st->pending[0] = st->pending[1] = false;
}

void StageToHost(void* dst_host, const void* src_dev, size_t bytes) {
  if (!bytes) return;
  psg_stream s = ThreadStream();
  Staging* st = GetStaging();
  if (!st) {
    RuntimeCopy(dst_host, src_dev, bytes, 1);
    return;
  }
  const size_t n = (bytes + kStageChunk - 1) / kStageChunk;
  auto issue = [&](size_t c) {
    const size_t off = c * kStageChunk, len = std::min(kStageChunk, bytes - off);
    Check(psg_memcpy(st->p.block[c & 1], (const char*)src_dev + off, len, 1, s), "psg_memcpy D2H");
    Check(psg_event_record(st->p.done[c & 1], s), "psg_event_record");
  };
  issue(0);
  for (size_t c = 0; c < n; ++c) {
    // chunk c + 1 goes on PCIe while chunk c is copied out of its block
    if (c + 1 < n) issue(c + 1);
    Check(psg_event_sync(st->p.done[c & 1]), "psg_event_sync");
    const size_t off = c * kStageChunk, len = std::min(kStageChunk, bytes - off);
    HostCopy((char*)dst_host + off, st->p.block[c & 1], len);
  }
  st->pending[0] = st->pending[1] = false;
}

void SliceKeys(const uint64_t* keys, size_t n, const int* lens, size_t num_vals,
               const std::vector<Range>& ranges, std::vector<uint64_t>* key_pos,
               std::vector<uint64_t>* val_pos) {
  const size_t ns = ranges.size();
  std::vector<uint64_t> b(ns), e(ns);
  for (size_t i = 0; i < ns; ++i) {
    b[i] = ranges[i].begin;
    e[i] = ranges[i].end;
  }
  key_pos->assign(ns + 1, 0);
  val_pos->assign(ns + 1, 0);
  Check(psg_slice(keys, n, lens, num_vals, (int)ns, b.data(), e.data(), key_pos->data(), val_pos->data(),
                  ThreadStream()),
        "psg_slice");
}

void Merge(std::vector<psg_segment>* segs, int elem_size, void* dst, uint64_t dst_count) {
  psg_stream s = ThreadStream();
  Check(psg_merge(segs->data(), (int)segs->size(), elem_size, dst, dst_count, s), "psg_merge");
  Check(psg_stream_sync(s), "psg_stream_sync");
}

psg_comm* CreateComm(int group) {
  PostOffice* po = PostOffice::Get();
  const std::vector<int>& ids = po->GetNodeIDs(group);
  auto me = std::find(ids.begin(), ids.end(), po->my_id());
  CHECK(me != ids.end()) << "node " << po->my_id() << " is not in group " << group;
  CHECK_GE(po->device(), 0) << "CreateComm: this node has no GPU";
  std::string mine;
  if (po->my_id() == *std::min_element(ids.begin(), ids.end())) {
    mine.resize((size_t)psg_comm_id_bytes());
    Check(psg_comm_get_id(&mine[0]), "psg_comm_get_id");
  }
  const std::string uid = po->GroupBroadcast(group, mine);
  CHECK_EQ(uid.size(), (size_t)psg_comm_id_bytes()) << "RCCL id from the group's root";
  psg_comm* c = nullptr;
  Check(psg_comm_init(uid.data(), (int)ids.size(), (int)(me - ids.begin()), &c), "psg_comm_init");
  return c;
}

}  // namespace device

namespace {
// HostFill's byte value that asks for the pages to be faulted in instead
// (PrefaultHost); MADV_POPULATE_WRITE (Linux 5.14) spelt out for older headers
constexpr int kPopulate = 0x100;
constexpr int kMadvPopulateWrite = 23;
// A persistent pool for large host copies (vector -> SVector, staging blocks).
// Spawning the helper threads per call cost more than the copy it split: a
// 16 MiB staging chunk copied by 4 fresh threads spent ~25 us on thread
// creation and join alone.  One job at a time; the caller runs part 0 and
// the workers take the rest by an atomic ticket OF THAT JOB: every job has its
// own ticket and part counters, and a worker drains only the job it took
// under the lock, so a worker still leaving an old job can never run a part
// of the next one (or count one of its parts twice).  Never destroyed: its
// threads may still be parked when static destructors run.
class CopyPool {
 public:
  explicit CopyPool(int nthreads) {
    for (int i = 0; i < nthreads; ++i) std::thread([this] { Work(); }).detach();
  }
  /* src == nullptr: fill dst with the byte `fill` */
  void Run(char* dst, const char* src, size_t bytes, int parts, size_t chunk, int fill = 0) {
    std::lock_guard<std::mutex> job_lk(job_mu_);
    auto job = std::make_shared<Job>();
    job->dst = dst;
    job->src = src;
    job->fill = fill;
    job->bytes = bytes;
    job->chunk = chunk;
    job->parts = parts;
    job->left.store(parts, std::memory_order_relaxed);
    {
      std::lock_guard<std::mutex> lk(mu_);
      job_ = job;
      ++gen_;
    }
    cv_.notify_all();
    Part(*job, 0);
    Drain(*job);
    // every part of THIS job done (a worker that took a ticket may still be
    // copying its part: wait for the count, not for the tickets)
    while (job->left.load(std::memory_order_acquire) != 0) std::this_thread::yield();
  }

 private:
  struct Job {
    char* dst = nullptr;
    const char* src = nullptr;
    int fill = 0;
    size_t bytes = 0, chunk = 0;
    int parts = 0;
    std::atomic<int> next{1}, left{0};
  };
  static void Part(Job& j, int i) {
    const size_t off = j.chunk * (size_t)i;
    if (off < j.bytes) {
      const size_t len = std::min(j.chunk, j.bytes - off);
      if (j.src) {
        std::memcpy(j.dst + off, j.src + off, len);
      } else if (j.fill == kPopulate) {
        // fault the part's whole pages in without writing through the
        // caller's objects (the kernel zero-fills fresh pages anyway)
        const uintptr_t a = ((uintptr_t)(j.dst + off) + 4095) & ~uintptr_t(4095);
        const uintptr_t b = ((uintptr_t)(j.dst + off + len)) & ~uintptr_t(4095);
        if (b > a) (void)madvise((void*)a, b - a, kMadvPopulateWrite);
      } else {
        std::memset(j.dst + off, j.fill, len);
      }
    }
    j.left.fetch_sub(1, std::memory_order_acq_rel);
  }
  static void Drain(Job& j) {
    for (int i; (i = j.next.fetch_add(1, std::memory_order_acq_rel)) < j.parts;) Part(j, i);
  }
  void Work() {
    uint64_t seen = 0;
    for (;;) {
      std::shared_ptr<Job> j;
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return gen_ != seen; });
        seen = gen_;
        j = job_;
      }
      if (j) Drain(*j);
    }
  }
  std::mutex job_mu_, mu_;
  std::condition_variable cv_;
  uint64_t gen_ = 0;
  std::shared_ptr<Job> job_;
};
}  // namespace

namespace {
constexpr size_t kSplit = size_t(4) << 20;  // below this one memcpy / memset
constexpr size_t kPart = size_t(1) << 20;   // smallest part handed to a worker
int CopyThreads() {
  static const int nthreads = [] {
    unsigned hc = std::thread::hardware_concurrency();
    const char* e = std::getenv("PS_COPY_THREADS");
    int n = e ? std::atoi(e) : (int)std::min<unsigned>(hc ? hc / 2 : 4, 8u);
    return std::max(1, n);
  }();
  return nthreads;
}
CopyPool* Pool() {
  static CopyPool* pool = new CopyPool(CopyThreads() - 1);
  return pool;
}
}  // namespace

void HostCopy(void* dst, const void* src, size_t bytes) {
  const int nthreads = CopyThreads();
  if (bytes < kSplit || nthreads == 1) {
    std::memcpy(dst, src, bytes);
    return;
  }
  const int parts = (int)std::min<size_t>((size_t)nthreads, bytes / kPart);
  const size_t chunk = (bytes / parts + 4095) & ~size_t(4095);
  Pool()->Run((char*)dst, (const char*)src, bytes, parts, chunk);
}

void HostFill(void* dst, int byte, size_t bytes) {
  const int nthreads = CopyThreads();
  if (bytes < kSplit || nthreads == 1) {
    std::memset(dst, byte, bytes);
    return;
  }
  const int parts = (int)std::min<size_t>((size_t)nthreads, bytes / kPart);
  const size_t chunk = (bytes / parts + 4095) & ~size_t(4095);
  Pool()->Run((char*)dst, nullptr, bytes, parts, chunk, byte);
}

void PrefaultHost(void* p, size_t bytes) {
  if (bytes < kSplit) return;
  // the whole 2 MiB pages inside [p, p + bytes) on huge pages, then every page
  // faulted in by the kernel (MADV_POPULATE_WRITE), in parallel — no store
  // through the caller's memory, which may be a vector's unused capacity
  constexpr uintptr_t kHuge = uintptr_t(2) << 20;
  const uintptr_t a = ((uintptr_t)p + kHuge - 1) & ~(kHuge - 1);
  const uintptr_t b = ((uintptr_t)p + bytes) & ~(kHuge - 1);
  if (b > a) (void)madvise((void*)a, b - a, MADV_HUGEPAGE);
  const int nthreads = CopyThreads();
  const int parts = (int)std::max<size_t>(1, std::min<size_t>((size_t)nthreads, bytes / kPart));
  const size_t chunk = (bytes / parts + 4095) & ~size_t(4095);
  Pool()->Run((char*)p, nullptr, bytes, parts, chunk, kPopulate);
}

}  // namespace ps
