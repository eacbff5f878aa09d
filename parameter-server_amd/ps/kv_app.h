// ps/kv_app.h — KVWorker / KVServer / KVServerDefaultHandle: the reference's
// KV app surface (src/ps/KVApp.h:27-458) over the MI355X data path.
//
// What runs where
//   worker  Push/Pull/PushPull build one request; the slicer cuts it by the
//           servers' key ranges — with std::lower_bound for host key arrays
//           (as KVApp.h:515-574) and with the psg_slice HIP kernel for key
//           arrays in HBM; one message per non-empty slice (frames zero-copy).
//   server  KVServerDefaultHandle keeps the value store in HBM (psg_store,
//           SORTED layout) and runs every request as the psg_store_handle
//           kernel.  HBM frames (a worker that holds its keys / values on a
//           GPU, or a host-vector request the worker staged into HBM,
//           detail::StageFrame) are read in place, over xGMI when the
//           worker's GPU is another one; host frames are copied into HBM.
//   merge   Pull replies are concatenated in key order: memcpy for host
//           replies (KVApp.h:713-720), the psg_merge kernel for HBM replies.
// Custom request handles registered with SetRequestHandle see host frames
// (HBM frames are copied to host first), exactly like the reference; a handle
// that can consume HBM frames registers with SetDeviceRequestHandle.
#pragma once
#include <fcntl.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <type_traits>
#include <unordered_map>
#include <utility>
#include <vector>

#include "internal/PostOffice.h"
#include "internal/customer.h"
#include "internal/device.h"
#include "internal/stage_time.h"
#include "ps/base.h"
#include "ps/range.h"
#include "ps/simple_app.h"
#include "ps/svector.h"

namespace ps {

/* keys (unique, ascending), vals, optional per-key value lengths (KVApp.h:27-37) */
template <typename Value>
struct KVPairs {
  SVector<Key> keys;
  SVector<Value> vals;
  SVector<int> lens;
  int priority = 0;
};

/* meta of one request (KVApp.h:42-57) */
struct KVMeta {
  int cmd;
  bool push;
  bool pull;
  int sender;
  int timestamp;
  int customer_id;
};

namespace detail {
template <typename T>
int DeviceOf(const std::vector<T>*) { return -1; }
template <typename T>
int DeviceOf(const SVector<T>* v) { return v->device(); }

/* host copy of an HBM array (no-op for host arrays) */
template <typename T>
SVector<T> ToHost(const SVector<T>& v) {
  if (!v.on_device() || v.empty()) return v;
  SVector<T> h = SVector<T>::Uninitialized(v.size());
  device::CopySync(h.data(), v.data(), v.size() * sizeof(T), 1);
  return h;
}
/* HBM copy of a host array on GPU dev (no-op for HBM arrays) */
template <typename T>
SVector<T> ToDevice(const SVector<T>& v, int dev) {
  if (v.on_device() || v.empty()) return v;
  SVector<T> d = SVector<T>::OnDevice(v.size(), dev);
  device::CopySync(d.data(), v.data(), v.size() * sizeof(T), 0);
  return d;
}
/* the same, enqueued on the thread stream without waiting (the caller's
 * later work on that stream is ordered after it; keep `v` alive until then) */
template <typename T>
SVector<T> ToDeviceAsync(const SVector<T>& v, int dev) {
  if (v.on_device() || v.empty()) return v;
  SVector<T> d = SVector<T>::OnDevice(v.size(), dev);
  device::Check(psg_memcpy(d.data(), v.data(), v.size() * sizeof(T), 0, device::ThreadStream()),
                "psg_memcpy H2D");
  return d;
}
// The copy a host-vector Push / Pull makes of the caller's array
// (KVApp.h:119-121, 155).  On a node with a GPU, once every server has
// answered that its handle takes HBM frames (Meta::hbm_handle: the default
// handle, SetDeviceRequestHandle), a large array (>= 4 MiB) is copied straight
// into HBM by the pipelined staging (device::StageToDevice): the request then
// takes the HBM path (device slicer, HBM frames, no H2D on the server) and the
// host copy overlaps the PCIe transfer.  Otherwise — a host handle such as
// test_kv_app_benchmark's, which would copy the frames back — or with
// PS_STAGE_TO_HBM=0, it is the reference's host SVector copy.
// PS_STAGE_MIN_BYTES moves the 4 MiB threshold (tests: the reference's
// test_kv_app.cpp, 10,000 keys, then runs its CHECKs on the HBM path —
// device slicer, HBM frames — with its own host vectors).
template <typename T>
SVector<T> StageFrame(const std::vector<T>& v, bool servers_take_hbm) {
  static const bool on = [] {
    const char* e = std::getenv("PS_STAGE_TO_HBM");
    return !(e && std::atoi(e) == 0);
  }();
  static const size_t min_bytes = [] {
    const char* e = std::getenv("PS_STAGE_MIN_BYTES");
    return e ? (size_t)std::atoll(e) : (size_t(4) << 20);
  }();
  const int dev = PostOffice::Get()->device();
  if (!on || !servers_take_hbm || dev < 0 || v.empty() || v.size() * sizeof(T) < min_bytes) return SVector<T>(v);
  SVector<T> d = SVector<T>::OnDevice(v.size(), dev);
  device::StageToDevice(d.data(), v.data(), v.size() * sizeof(T));
  return d;
}
// The key-list hash of LR key caching: the std::hash<ps::SVector<uint64_t>>
// specialisation of tests/src/LRServer.h:11-29, which the reference worker
// also uses (LRWorker.h:214-219), restated so a server finds the list a
// worker names.  psg_key_list_hash computes the same on device keys.
inline uint64_t KeyListHash(const Key* keys, size_t n) {
  uint64_t seed = n;
  for (size_t i = 0; i < n; ++i) {
    uint64_t x = keys[i] + 0x9e3779b97f4a7c15ull;
    x = (x ^ (x >> 30)) * 0xbf58476d1ce4e5b9ull;
    x = (x ^ (x >> 27)) * 0x94d049bb133111ebull;
    seed ^= x ^ x >> 31;
  }
  return seed;
}

/* PS_PUSH_RUNS=0: a server handles every queued Push on its own, never a run
 * of them in one pass (A/B; KVServer::OnReceive). */
inline bool PushRunsOn() {
  static const bool on = [] {
    const char* e = std::getenv("PS_PUSH_RUNS");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
/* PS_MIXED_RUNS=0: a run holds Pushes of one shape only, never the Pulls and
 * PushPulls of distinct senders queued with them (A/B; KVServer::OnReceive). */
inline bool MixedRunsOn() {
  static const bool on = [] {
    const char* e = std::getenv("PS_MIXED_RUNS");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
/* PS_RUN_GATHER_US: how long a server waits for the requests of the senders
 * it has heard from lately to join a run (KVServer::OnReceive); default 120
 * (the reference benchmark's layout at ns = nw = 4 on one GPU: 477-487 GB/s
 * with no wait, 574-609 with 120 us, noisier past it:
 * profiles/r6_dropin_gather_sweep.txt); 0: a run holds what is queued when it
 * starts. */
inline int RunGatherMicros() {
  static const int us = [] {
    const char* e = std::getenv("PS_RUN_GATHER_US");
    return e ? std::atoi(e) : 120;
  }();
  return us;
}
/* PS_RUN_GATHER_AUTO=<cap µs> (default 0: off): the gather window follows how
 * long this server's recent runs took (at least PS_RUN_GATHER_US, at most the
 * cap) — a sender missing from a run is most likely waiting for another
 * server's run of about that length before it sends its next request. */
inline int RunGatherAutoCap() {
  static const int us = [] {
    const char* e = std::getenv("PS_RUN_GATHER_AUTO");
    return e ? std::atoi(e) : 0;
  }();
  return us;
}
/* PS_RUN_GATHER_ORDINAL (default 1): the gather waits only for the recent
 * senders that are behind the run — those this server has taken fewer
 * requests from than the run's lowest ordinal (its n-th request from each) —
 * and for up to PS_RUN_GATHER_ORD_US (default 1000) µs.  A sender that is not
 * behind has had this round's request served already and may itself wait for
 * this server's answer to another; one that is behind is held up only by
 * servers serving lower ordinals, so the waits form no cycle.  0: wait for
 * every recent sender for PS_RUN_GATHER_US (A/B). */
inline bool RunGatherOrdinal() {
  static const bool on = [] {
    const char* e = std::getenv("PS_RUN_GATHER_ORDINAL");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
inline int RunGatherOrdMicros() {
  static const int us = [] {
    const char* e = std::getenv("PS_RUN_GATHER_ORD_US");
    return e ? std::atoi(e) : 1000;
  }();
  return us;
}
/* PS_TRACE_REQUESTS=<file>: every request a KVServer hands to its handle is
 * appended to <file> as one line "server sender timestamp push pull keys
 * run_size run_pos" (run_size 1 for a request handled on its own) — the
 * arrival order a test replays through the oracle.  One write(2) per line on
 * an O_APPEND descriptor, so the servers of a job may share the file. */
inline void TraceRequest(int server, const KVMeta& m, size_t keys, size_t run_size, size_t run_pos) {
  static const int fd = [] {
    const char* e = std::getenv("PS_TRACE_REQUESTS");
    return e && *e ? ::open(e, O_WRONLY | O_CREAT | O_APPEND, 0644) : -1;
  }();
  if (fd < 0) return;
  char line[160];
  const int len = std::snprintf(line, sizeof(line), "%d %d %d %d %d %zu %zu %zu\n", server, m.sender, m.timestamp,
                                (int)m.push, (int)m.pull, keys, run_size, run_pos);
  if (len > 0) (void)!::write(fd, line, (size_t)len);
}

/* A worker sends an HBM key list it sliced before on the bounds it had then,
 * unconfirmed, when every server checks its slices (KVWorker::Send);
 * PS_SPEC_SLICE=0: every request is sliced first (A/B). */
inline bool SpecSliceOn() {
  static const bool on = [] {
    const char* e = std::getenv("PS_SPEC_SLICE");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
/* PS_TRACE_GATHER=<file> (diagnostics): one line per gathered run, "server
 * head_sender head_ordinal run_size why waited_us" — why the gather ended:
 * 0 run full, 1 no sender behind (or no window), 2 a queued message that
 * may not join, 3 the window timed out. */
inline void TraceGather(int server, int sender, uint64_t ordinal, size_t size, int why, double us) {
  static const int fd = [] {
    const char* e = std::getenv("PS_TRACE_GATHER");
    return e && *e ? ::open(e, O_WRONLY | O_CREAT | O_APPEND, 0644) : -1;
  }();
  if (fd < 0) return;
  char line[128];
  const int len = std::snprintf(line, sizeof(line), "%d %d %llu %zu %d %.1f\n", server, sender,
                                (unsigned long long)ordinal, size, why, us);
  if (len > 0) (void)!::write(fd, line, (size_t)len);
}

/* ZPull offers the servers its HBM output (Meta::direct_reply); PS_DIRECT_REPLY=0
 * turns the offer off (A/B): every reply is then merged by psg_merge. */
inline bool DirectReplyOn() {
  static const bool on = [] {
    const char* e = std::getenv("PS_DIRECT_REPLY");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}
}  // namespace detail

template <typename Value>
struct KVServerDefaultHandle;

template <typename Value>
class KVWorker : public SimpleApp {
 public:
  using Data = KVPairs<Value>;
  using Callback = std::function<void()>;
  using SlicedKVs = std::vector<std::pair<bool, Data>>;
  using Slicer = std::function<void(Data& send, const std::vector<Range>& ranges, SlicedKVs* sliced)>;

  KVWorker(int app_id, int customer_id) : SimpleApp() {
    slicer_ = [this](Data& send, const std::vector<Range>& ranges, SlicedKVs* sliced) {
      DefaultSlicer(send, ranges, sliced);
    };
    app_id_ = app_id;
    customer_ = new Customer(app_id, customer_id, [this](const Message& m) { OnReceive(m); });
  }
  ~KVWorker() override {
    delete customer_;
    customer_ = nullptr;
  }

  /* KVApp.h:112-122: the vectors are copied into SVectors (into HBM on a
   * node with a GPU, detail::StageFrame; the lens stay on the host) */
  int Push(const std::vector<Key>& keys, const std::vector<Value>& vals,
           const std::vector<int>& lens = {}, int cmd = 0, const Callback& cb = nullptr,
           int priority = 0) {
    if (!lens.empty()) return ZPush(SVector<Key>(keys), SVector<Value>(vals), SVector<int>(lens), cmd, cb, priority);
    const bool hbm = servers_take_hbm_.load();
    SVector<Key> skeys;
    SVector<Value> svals;
    {
      stage::Scope t("worker.push.copy", keys.size() * sizeof(Key) + vals.size() * sizeof(Value));
      skeys = detail::StageFrame(keys, hbm);
      svals = detail::StageFrame(vals, hbm);
    }
    return ZPush(skeys, svals, SVector<int>(), cmd, cb, priority);
  }

  /* KVApp.h:148-162 */
  int Pull(const std::vector<Key>& keys, std::vector<Value>* vals, std::vector<int>* lens = nullptr,
           int cmd = 0, const Callback& cb = nullptr, int priority = 0) {
    SVector<Key> skeys;
    {
      stage::Scope t("worker.pull.copy_keys", keys.size() * sizeof(Key));
      skeys = lens ? SVector<Key>(keys) : detail::StageFrame(keys, servers_take_hbm_.load());
    }
    int ts = AddPullCB(skeys, vals, lens, cmd, cb);
    Data kvs;
    kvs.keys = skeys;
    kvs.priority = priority;
    Send(ts, false, true, cmd, kvs);
    return ts;
  }

  /* KVApp.h:188-213 */
  int PushPull(const std::vector<Key>& keys, const std::vector<Value>& vals, std::vector<Value>* outs,
               std::vector<int>* lens = nullptr, int cmd = 0, const Callback& cb = nullptr,
               int priority = 0) {
    CHECK_NOTNULL(outs);
    if (outs->empty())
      outs->resize(vals.size());
    else
      CHECK_EQ(vals.size(), outs->size());
    const bool hbm = servers_take_hbm_.load();
    SVector<Key> skeys = lens ? SVector<Key>(keys) : detail::StageFrame(keys, hbm);
    SVector<Value> svals = lens ? SVector<Value>(vals) : detail::StageFrame(vals, hbm);
    auto souts = new SVector<Value>(outs->data(), outs->size());
    SVector<int>* slens = lens ? new SVector<int>(lens->data(), lens->size()) : nullptr;
    return ZPushPull(skeys, svals, souts, slens, cmd,
                     [souts, slens, cb]() {
                       delete souts;
                       delete slens;
                       if (cb) cb();
                     },
                     priority);
  }

  void Wait(int timestamp) override { customer_->WaitRequest(timestamp); }

  /* zero-copy forms (KVApp.h:234-291); SVectors may live in HBM */
  int ZPush(const SVector<Key>& keys, const SVector<Value>& vals, const SVector<int>& lens = {},
            int cmd = 0, const Callback& cb = nullptr, int priority = 0) {
    int ts = customer_->NewRequest(kServerGroup);
    AddCallback(ts, cb);
    Data kvs;
    kvs.keys = keys;
    kvs.vals = vals;
    kvs.lens = lens;
    kvs.priority = priority;
    Send(ts, true, false, cmd, kvs);
    return ts;
  }
  int ZPull(const SVector<Key>& keys, SVector<Value>* vals, SVector<int>* lens = nullptr, int cmd = 0,
            const Callback& cb = nullptr, int priority = 0) {
    int ts = AddPullCB(keys, vals, lens, cmd, cb);
    Data kvs;
    kvs.keys = keys;
    kvs.priority = priority;
    // HBM keys and a sized HBM output, no lens: offer each server its slice of
    // the output (the request's vals frame), so a handle that can write its
    // reply there does, and the merge copy disappears (detail::DirectReply)
    const bool direct = vals && lens == nullptr && keys.on_device() && keys.size() && vals->on_device() &&
                        vals->size() && vals->size() % keys.size() == 0 && detail::DirectReplyOn();
    if (direct) kvs.vals = *vals;
    Send(ts, false, true, cmd, kvs, direct);
    return ts;
  }
  int ZPushPull(const SVector<Key>& keys, const SVector<Value>& vals, SVector<Value>* outs,
                SVector<int>* lens = nullptr, int cmd = 0, const Callback& cb = nullptr,
                int priority = 0) {
    int ts = AddPullCB(keys, outs, lens, cmd, cb);
    Data kvs;
    kvs.keys = keys;
    kvs.vals = vals;
    kvs.priority = priority;
    if (lens) kvs.lens = *lens;  // the reference forwards the output lens (KVApp.h:287-288)
    // as ZPull: offer each server its slice of the HBM output (outs mirrors vals)
    const bool direct = outs && lens == nullptr && keys.on_device() && keys.size() && outs->on_device() &&
                        outs->size() == vals.size() && vals.on_device() && detail::DirectReplyOn();
    Send(ts, true, true, cmd, kvs, direct, direct ? outs : nullptr);
    return ts;
  }

  /* slices its servers refused (Refused; PS_SPEC_SLICE) */
  uint64_t refused_slices() const { return refused_.load(); }
  void set_slicer(const Slicer& slicer) {
    default_slicer_ = false;
    CHECK(static_cast<bool>(slicer));
    slicer_ = slicer;
  }

 private:
  struct Reply {
    Data kv;
    int sender;
    bool direct = false;  // the server wrote the values into the output in place
  };
  // servers whose replies said their handle takes HBM frames
  void NoteHbmServer(int sender) {
    std::lock_guard<std::mutex> lk(mu_);
    const int ns = PostOffice::Get()->num_servers();
    if (hbm_server_.size() != (size_t)ns) hbm_server_.assign(ns, 0);
    const int r = PostOffice::IDToRank(sender);
    if (r < ns && !hbm_server_[r]) {
      hbm_server_[r] = 1;
      if (++hbm_count_ == ns) servers_take_hbm_ = true;
    }
  }
  std::vector<char> hbm_server_;
  int hbm_count_ = 0;
  std::atomic<bool> servers_take_hbm_{false};
  // servers whose handle takes unconfirmed slices (Meta::spec_slice in their
  // replies); all of them: the worker may send the slicer's hints unconfirmed
  void NoteSpecServer(int sender) {
    std::lock_guard<std::mutex> lk(mu_);
    const int ns = PostOffice::Get()->num_servers();
    if (spec_server_.size() != (size_t)ns) spec_server_.assign(ns, 0);
    const int r = PostOffice::IDToRank(sender);
    if (r < ns && !spec_server_[r]) {
      spec_server_[r] = 1;
      if (++spec_count_ == ns) servers_take_spec_ = true;
    }
  }
  std::vector<char> spec_server_;
  int spec_count_ = 0;
  std::atomic<bool> servers_take_spec_{false};
  // a request sent on unconfirmed slices: what a refusal needs to re-send
  struct SpecSend {
    bool push = false, pull = false, direct = false, has_outs = false;
    int cmd = 0;
    Data kvs;
    SVector<Value> outs;
    std::vector<uint64_t> pos;  // the hinted key bounds, num_servers + 1
  };
  std::unordered_map<int, SpecSend> spec_sends_;
  std::unordered_map<const void*, bool> spec_stale_;  // key arrays a refusal proved re-sliced since
  bool default_slicer_ = true;
  std::atomic<uint64_t> refused_{0};
  void SendOne(int timestamp, bool push, bool pull, int cmd, int priority, const Data& whole, const Data& kv,
               bool direct, const SVector<Value>* outs, int server_rank, bool spec);
  void Refused(const Message& msg);
  void SendPieces(int timestamp, const SpecSend& sp, uint64_t a, uint64_t b, const std::vector<uint64_t>& pos,
                  int* sent);

  void AddCallback(int timestamp, const Callback& cb) {
    if (!cb) return;
    std::lock_guard<std::mutex> lk(mu_);
    callbacks_[timestamp] = cb;
  }
  void RunCallback(int timestamp);
  void Send(int timestamp, bool push, bool pull, int cmd, const Data& kvs, bool direct = false,
            const SVector<Value>* outs = nullptr);
  void OnReceive(const Message& msg) override;
  void DefaultSlicer(Data& send, const std::vector<Range>& ranges, SlicedKVs* sliced);
  template <typename C, typename D>
  int AddPullCB(const SVector<Key>& keys, C* vals, D* lens, int cmd, const Callback& cb);
  template <typename C, typename D>
  void MergePull(const SVector<Key>& keys, std::vector<Reply>& kvs, C* vals, D* lens);

  std::unordered_map<int, std::vector<Reply>> recv_kvs_;
  std::unordered_map<int, Callback> callbacks_;
  std::mutex mu_;
  Slicer slicer_;
};

/* one request of a run of queued requests (KVServer::OnReceive) */
template <typename Value>
struct KVRunItem {
  KVMeta meta;
  KVPairs<Value> data;
  SVector<Value> out;  // the output slice a Pull offered for its reply (direct reply), else empty
  bool spec = false;   // its slice is the worker's unconfirmed hint (Meta::spec_slice)
};

template <typename Value>
class KVServer : public SimpleApp {
 public:
  using ReqHandle = std::function<void(const KVMeta& req_meta, const KVPairs<Value>& req_data, KVServer* server)>;
  /* A run of requests queued one behind the other (see OnReceive), in arrival
   * order; the handle answers every one of them. */
  using RunHandle = std::function<void(std::vector<KVRunItem<Value>>& run, KVServer* server)>;
  static constexpr int kMaxRun = 16;  // requests a run holds at most (psg_store_run)

  explicit KVServer(int app_id) : SimpleApp() {
    app_id_ = app_id;
    customer_ = new Customer(app_id, app_id, [this](const Message& m) { OnReceive(m); });
  }
  ~KVServer() override {
    delete customer_;
    customer_ = nullptr;
  }

  /* a host handle: sees host frames (KVApp.h:405-408) */
  void SetRequestHandle(const ReqHandle& request_handle) {
    CHECK(static_cast<bool>(request_handle)) << "invalid request handle";
    Install(request_handle, false);
  }
  /* the default handle keeps its store in HBM and takes frames where they are,
   * and serves a run of queued Pushes on one key list in one pass */
  void SetRequestHandle(const KVServerDefaultHandle<Value>& h) {
    Install(h, true, [hd = h](std::vector<KVRunItem<Value>>& run, KVServer* server) mutable { hd.Run(run, server); });
  }
  /* a handle that consumes HBM frames itself */
  void SetDeviceRequestHandle(const ReqHandle& request_handle) {
    CHECK(static_cast<bool>(request_handle)) << "invalid request handle";
    Install(request_handle, true);
  }

  /* reply to a request (KVApp.h:491-513); frames may be host or HBM */
  void Response(const KVMeta& req, const KVPairs<Value>& res = KVPairs<Value>());
  /* For a run handle: reply to one request of a run; `direct` says the handle
   * wrote the Pull's values into the output slice the request offered
   * (KVRunItem::out), so the reply carries its keys and no values. */
  void RunResponse(const KVMeta& req, const KVPairs<Value>& res, bool direct) { Reply(req, res, direct); }
  /* For a run handle: refuse a request whose unconfirmed slice (KVRunItem::spec)
   * holds a key outside this server's range — nothing of it was applied; the
   * worker re-sends its keys sliced for real. */
  void RunRefuse(const KVMeta& req) { Reply(req, KVPairs<Value>(), false, true); }
  /* this server takes unconfirmed slices: its handle checks every key of a run
   * against its own range and refuses a wrong slice instead of failing */
  bool TakesSpecSlices() const {
    return static_cast<bool>(run_handle_) && device_frames_.load() && detail::PushRunsOn() && detail::MixedRunsOn();
  }
  /* For a run handle: serve one request of a run with the installed handle, as
   * if it had been taken on its own (its output offer included). */
  void ServeOne(const KVRunItem<Value>& item) {
    direct_out_ = item.out;
    direct_ts_ = item.meta.timestamp;
    direct_sender_ = item.meta.sender;
    direct_taken_ = false;
    request_handle_(item.meta, item.data, this);
    direct_out_ = SVector<Value>();
    direct_taken_ = false;
  }

 private:
  void OnReceive(const Message& msg) override;
  void Reply(const KVMeta& req, const KVPairs<Value>& res, bool direct, bool refused = false);
  void Install(const ReqHandle& h, bool device_frames, const RunHandle& run = nullptr) {
    {
      std::lock_guard<std::mutex> lk(handle_mu_);
      request_handle_ = h;
      run_handle_ = run;
      device_frames_ = device_frames;
    }
    handle_cv_.notify_all();
  }
  /* a request a run may hold: a Push, Pull or PushPull with keys and no lens
   * ([keys, vals], [keys, out] for a Pull offering its output, [keys, vals, out]
   * for such a PushPull) */
  static bool PlainRequest(const Message& m) {
    if (!m.meta.request || m.meta.simple_app || m.meta.control.cmd != Control::EMPTY) return false;
    if (!(m.meta.push || m.meta.pull)) return false;
    const size_t want = (m.meta.direct_reply && m.meta.push && m.meta.pull) ? 3 : 2;
    return m.data.size() == want && m.data[0].size() > 0 && (!m.meta.push || m.data[1].size() > 0);
  }
  static KVMeta MetaOf(const Message& msg) {
    KVMeta meta;
    meta.cmd = msg.meta.head;
    meta.push = msg.meta.push;
    meta.pull = msg.meta.pull;
    meta.sender = msg.meta.sender;
    meta.timestamp = msg.meta.timestamp;
    meta.customer_id = msg.meta.customer_id;
    return meta;
  }
  RunHandle run_handle_;
  // the senders of the last requests this server took (the gather window's
  // target: how many requests one step brings), a ring of 64
  int recent_[64] = {};
  unsigned recent_n_ = 0;
  int gather_idle_ = 0;  // gather windows in a row that timed out with nothing gained
  int gather_cool_ = 0;  // requests left to take without a window
  double run_us_ = 0;    // this server's recent run times (moving average, µs)
  // requests taken from each sender so far (a request's ordinal: the n-th from
  // its sender)
  std::unordered_map<int, uint64_t> taken_;
  // senders a window timed out waiting for: not waited for again until they
  // send (a worker that skips this server, or has stopped)
  std::unordered_map<int, bool> stalled_;
  uint64_t Take(int sender) {
    stalled_.erase(sender);
    return ++taken_[sender];
  }
  // a recent sender outside the run that this server has taken fewer than m
  // requests from (its next request is the run's round or an earlier one);
  // mark: note every such sender as stalled instead
  bool SendersBehind(const std::vector<KVRunItem<Value>>& items, uint64_t m, bool mark = false) {
    const unsigned n = recent_n_ < 64 ? recent_n_ : 64;
    bool any = false;
    for (unsigned i = 0; i < n; ++i) {
      const int w = recent_[i];
      bool in = false;
      for (const auto& it : items) in = in || it.meta.sender == w;
      if (in || stalled_.count(w)) continue;
      auto t = taken_.find(w);
      if ((t == taken_.end() ? 0 : t->second) < m) {
        if (!mark) return true;
        stalled_[w] = true;
        any = true;
      }
    }
    return any;
  }
  void NoteSender(int sender) { recent_[recent_n_++ & 63] = sender; }
  size_t RecentSenders(int sender) {
    NoteSender(sender);
    const unsigned n = recent_n_ < 64 ? recent_n_ : 64;
    int seen[64];
    size_t c = 0;
    for (unsigned i = 0; i < n; ++i) {
      bool dup = false;
      for (size_t j = 0; j < c && !dup; ++j) dup = seen[j] == recent_[i];
      if (!dup) seen[c++] = recent_[i];
    }
    return c < (size_t)kMaxRun ? c : (size_t)kMaxRun;
  }
  // The customer thread may receive a request before the program installs its
  // handle (it is created with the KVServer); it waits for the handle instead
  // of failing the reference's CHECK (KVApp.h:487) on that race.
  ReqHandle request_handle_;
  std::atomic<bool> device_frames_{false};
  std::mutex handle_mu_;
  std::condition_variable handle_cv_;
  // the output slice a direct-reply Pull offers while its handle runs (the
  // customer thread runs one handle at a time), and whether the handle took it
  // (atomics: a handle may answer a deferred request from another thread)
  SVector<Value> direct_out_;
  std::atomic<int> direct_ts_{-1}, direct_sender_{-1};
  std::atomic<bool> direct_taken_{false};

 public:
  /* For a handle that answers a Pull from HBM: the caller's output slice for
   * this request's values when the worker offered one of n values (ZPull
   * with HBM keys and a sized HBM output), else an empty SVector.  A handle
   * that takes it must write the reply values there (ordered before its
   * Response) and then Response with keys and no values, from inside the
   * handle (a deferred Response is not marked as written in place). */
  SVector<Value> TakeDirectOut(size_t n) {
    if (direct_out_.size() != n || !direct_out_.on_device()) return SVector<Value>();
    direct_taken_ = true;
    return direct_out_;
  }
};

/* The default handle (KVApp.h:433-458): `store[key] += val` for a push,
 * `res.vals[i] = store[key]` (post-update) for a pull, absent keys inserted
 * with 0 — with the store in HBM (psg_store, SORTED) and the loop as HIP
 * kernels per request.  One value per key (the reference's CHECK at :441).
 *
 * KVServerDefaultHandle<V>(true) also serves the key-cache protocol of the
 * reference's LR server (LRServer.h:127-142) on this store: a request with
 * more than one key is handled as usual and its key list is cached under its
 * hash (detail::KeyListHash / psg_key_list_hash), resolved once to store
 * slots; a request with ONE key names a cached list by that hash and runs on
 * the cached slots (psg_store_handle_slots: 16 B / key for a Push instead of
 * a validation pass plus the resolve).  The slots are re-resolved after the
 * store inserts keys.  As in the reference, a one-key request is then always
 * read as a hash, and every list should go to one server (LR_ps runs ns = 1). */
template <typename Value>
struct KVServerDefaultHandle {
  struct Cached {
    SVector<Key> keys;        // the list (HBM), kept for a re-resolve
    SVector<uint32_t> slots;  // its store slots (HBM)
    uint64_t store_size = 0;  // the store's size when resolved (an insert moves slots)
    // the first slot when the slots are a stretch of the store (the list covers
    // its range: LRServer.h:144's every-feature list), else UINT64_MAX: then a
    // request needs no slot stream (psg_store_handle_stretch)
    uint64_t stretch = UINT64_MAX;
  };
  struct State {
    psg_store* store = nullptr;
    bool key_cache = false;
    std::unordered_map<uint64_t, Cached> cache;
    ~State() {
      if (store) psg_store_destroy(store);
    }
  };
  std::shared_ptr<State> state = std::make_shared<State>();

  explicit KVServerDefaultHandle(bool use_key_cache = false) { state->key_cache = use_key_cache; }

  void operator()(const KVMeta& req_meta, const KVPairs<Value>& req_data, KVServer<Value>* server) {
    size_t n = req_data.keys.size();
    KVPairs<Value> res;
    const int dev = PostOffice::Get()->device();
    CHECK_GE(dev, 0) << "KVServerDefaultHandle: the value store lives in HBM and this node has no GPU";
    constexpr int dt = device::DType<Value>();
    CHECK_GE(dt, 0) << "KVServerDefaultHandle: value type not supported by the HBM store";
    if (!state->store)
      device::Check(psg_store_create(PSG_STORE_SORTED, dt, 0, kMaxKey, 0, &state->store), "psg_store_create");
    const bool on_dev = req_data.keys.on_device();
    const int flags = (req_meta.push ? PSG_PUSH : 0) | (req_meta.pull ? PSG_PULL : 0);
    psg_stream s = device::ThreadStream();
    SVector<Value> dout;
    bool direct = false;
    if (state->key_cache && n == 1 && flags) {
      // a cached list named by its hash (LRServer.h:129-135)
      Key h = 0;
      if (on_dev) device::CopySync(&h, req_data.keys.data(), sizeof(Key), 1);
      else h = req_data.keys[0];
      auto it = state->cache.find(h);
      CHECK(it != state->cache.end()) << "Keys don't exist with hash value: " << h;
      Cached& c = it->second;
      n = c.keys.size();
      if (req_meta.push) CHECK_EQ(n, req_data.vals.size());
      Refresh(c, s);
      SVector<Value> dvals;
      if (req_meta.push) dvals = detail::ToDeviceAsync(req_data.vals, dev);
      if (req_meta.pull) dout = PullOutput(server, n, dev, &direct);
      if (c.stretch != UINT64_MAX)
        device::Check(psg_store_handle_stretch(state->store, flags, c.stretch, dvals.data(), dout.data(), n, s),
                      "psg_store_handle_stretch");
      else
        device::Check(psg_store_handle_slots(state->store, flags, c.slots.data(), dvals.data(), dout.data(), n, s),
                      "psg_store_handle_slots");
      // answered once the kernel has ended: a polled word, not a stream wait
      device::Check(psg_store_sync(state->store, s), "psg_store_sync");
    } else if (n && flags) {
      if (req_meta.push) CHECK_EQ(n, req_data.vals.size());
      SVector<Key> dkeys = detail::ToDeviceAsync(req_data.keys, dev);
      SVector<Value> dvals;
      if (req_meta.push) dvals = detail::ToDeviceAsync(req_data.vals, dev);
      if (req_meta.pull) dout = PullOutput(server, n, dev, &direct);
      {
        stage::Scope t(req_meta.push ? "server.handle.store.push" : "server.handle.store.pull");
        device::Check(psg_store_handle(state->store, flags, dkeys.data(), 0, dvals.data(), dout.data(), n, s),
                      "psg_store_handle");
      }
      // psg_store_handle returns once the request's keys and vals are no longer
      // read and a Pull's reply is in memory (psg.h), so it can be answered
      // now.  Later requests on this thread's stream are ordered behind it.
      if (state->key_cache) Remember(dkeys, on_dev, on_dev ? 0 : detail::KeyListHash(req_data.keys.data(), n), s);
    } else if (req_meta.push) {
      CHECK_EQ(n, req_data.vals.size());
    }
    if (req_meta.pull) {
      res.keys = req_data.keys;
      // written into the worker's output in place (TakeDirectOut): no values
      if (!direct) res.vals = on_dev ? dout : detail::ToHost(dout);
    }
    server->Response(req_meta, res);
  }

  /* A run of requests queued one behind the other (KVServer::OnReceive), with
   * the result of handling them one at a time in that order (KVApp.h:446-454
   * per request).  Full key lists go to psg_store_run, which reads and writes
   * the store once for the whole run when the lists are one list (Pushes) or
   * interleave (distinct phases of one period of the store: the reference
   * benchmark's layout), and serves them request by request otherwise.  With
   * the key cache, a run of Pushes naming one cached list by its hash is one
   * pass over the cached slots or stretch (psg_store_push_slots_frames).
   * Every request is answered after the run is served. */
  void Run(std::vector<KVRunItem<Value>>& run, KVServer<Value>* server) {
    bool all_push = true, hashed = false;
    for (const auto& it : run) {
      all_push = all_push && it.meta.push && !it.meta.pull;
      hashed = hashed || it.data.keys.size() == 1;
    }
    if (all_push) {
      std::vector<KVMeta> metas;
      std::vector<KVPairs<Value>> datas;
      std::vector<char> spec;
      for (const auto& it : run) {
        metas.push_back(it.meta);
        datas.push_back(it.data);
        spec.push_back(it.spec ? 1 : 0);
      }
      PushRun(metas, datas, server, spec);
      return;
    }
    if (state->key_cache && hashed) {
      // a one-key request names a cached list (LRServer.h:129-135): on its own
      for (const auto& it : run) server->ServeOne(it);
      return;
    }
    const int dev = PostOffice::Get()->device();
    CHECK_GE(dev, 0) << "KVServerDefaultHandle: the value store lives in HBM and this node has no GPU";
    constexpr int dt = device::DType<Value>();
    CHECK_GE(dt, 0) << "KVServerDefaultHandle: value type not supported by the HBM store";
    if (!state->store)
      device::Check(psg_store_create(PSG_STORE_SORTED, dt, 0, kMaxKey, 0, &state->store), "psg_store_create");
    psg_stream s = device::ThreadStream();
    const size_t k = run.size();
    std::vector<int> ops(k);
    std::vector<uint64_t> ns(k);
    std::vector<SVector<Key>> dkeys(k);
    std::vector<SVector<Value>> dvals(k), douts(k);
    std::vector<const uint64_t*> kp(k);
    std::vector<const void*> vp(k, nullptr);
    std::vector<void*> op(k, nullptr);
    std::vector<char> direct(k, 0);
    for (size_t j = 0; j < k; ++j) {
      const auto& it = run[j];
      const size_t n = it.data.keys.size();
      ops[j] = (it.meta.push ? PSG_PUSH : 0) | (it.meta.pull ? PSG_PULL : 0);
      ns[j] = n;
      if (it.meta.push) CHECK_EQ(n, it.data.vals.size());  // one value per key (KVApp.h:441)
      dkeys[j] = detail::ToDeviceAsync(it.data.keys, dev);
      kp[j] = dkeys[j].data();
      if (it.meta.push) {
        dvals[j] = detail::ToDeviceAsync(it.data.vals, dev);
        vp[j] = dvals[j].data();
      }
      if (it.meta.pull) {
        direct[j] = it.out.size() == n && it.out.on_device();
        douts[j] = direct[j] ? it.out : SVector<Value>::OnDevice(n, dev);
        op[j] = douts[j].data();
      }
    }
    std::vector<int> status(k, PSG_OK);
    bool any_spec = false;
    for (const auto& it : run) any_spec = any_spec || it.spec;
    {
      stage::Scope t("server.handle.store.run");
      ServeRun(any_spec, (int)k, ops.data(), kp.data(), ns.data(), vp.data(), op.data(), s, status.data(),
               [&](int j) { return run[j].spec; });
    }
    // a request refused for a key outside this shard: fatal, as a CHECK,
    // unless its slice was the worker's unconfirmed hint
    for (size_t j = 0; j < k; ++j)
      if (status[j] != PSG_OK && !run[j].spec) device::Check(status[j], "psg_store_run");
    if (state->key_cache)
      for (size_t j = 0; j < k; ++j)
        if (status[j] == PSG_OK)
          Remember(dkeys[j], run[j].data.keys.on_device(),
                   run[j].data.keys.on_device() ? 0 : detail::KeyListHash(run[j].data.keys.data(), ns[j]), s);
    for (size_t j = 0; j < k; ++j) {
      if (status[j] != PSG_OK) {
        server->RunRefuse(run[j].meta);
        continue;
      }
      KVPairs<Value> res;
      if (run[j].meta.pull) {
        res.keys = run[j].data.keys;
        if (!direct[j]) res.vals = run[j].data.keys.on_device() ? douts[j] : detail::ToHost(douts[j]);
      }
      server->RunResponse(run[j].meta, res, direct[j] != 0);
    }
  }

  /* A run of Pushes of one shape (Run). */
  void PushRun(const std::vector<KVMeta>& metas, const std::vector<KVPairs<Value>>& datas, KVServer<Value>* server,
               const std::vector<char>& spec = {}) {
    std::vector<int> status(datas.size(), PSG_OK);
    const int dev = PostOffice::Get()->device();
    CHECK_GE(dev, 0) << "KVServerDefaultHandle: the value store lives in HBM and this node has no GPU";
    constexpr int dt = device::DType<Value>();
    CHECK_GE(dt, 0) << "KVServerDefaultHandle: value type not supported by the HBM store";
    if (!state->store)
      device::Check(psg_store_create(PSG_STORE_SORTED, dt, 0, kMaxKey, 0, &state->store), "psg_store_create");
    psg_stream s = device::ThreadStream();
    const size_t k = datas.size();
    const size_t n = datas[0].keys.size();
    for (const auto& d : datas) {
      CHECK_EQ(d.keys.size(), n);
      if (!(state->key_cache && n == 1)) CHECK_EQ(n, d.vals.size());  // one value per key (KVApp.h:441)
    }
    std::vector<SVector<Value>> dvals(k);
    std::vector<const void*> vp(k);
    if (state->key_cache && n == 1) {
      // cached lists named by their hashes (LRServer.h:129-135); consecutive
      // requests naming one list are one pass
      std::vector<Key> h(k);
      for (size_t j = 0; j < k; ++j) {
        if (datas[j].keys.on_device()) device::CopySync(&h[j], datas[j].keys.data(), sizeof(Key), 1);
        else h[j] = datas[j].keys[0];
      }
      for (size_t i = 0; i < k;) {
        size_t e = i + 1;
        while (e < k && h[e] == h[i]) ++e;
        auto it = state->cache.find(h[i]);
        CHECK(it != state->cache.end()) << "Keys don't exist with hash value: " << h[i];
        Cached& c = it->second;
        Refresh(c, s);
        for (size_t j = i; j < e; ++j) {
          CHECK_EQ(c.keys.size(), datas[j].vals.size());
          dvals[j] = detail::ToDeviceAsync(datas[j].vals, dev);
          vp[j] = dvals[j].data();
        }
        const bool stretch = c.stretch != UINT64_MAX;
        device::Check(psg_store_push_slots_frames(state->store, stretch ? nullptr : c.slots.data(),
                                                  stretch ? c.stretch : 0, vp.data() + i, (int)(e - i),
                                                  c.keys.size(), s),
                      "psg_store_push_slots_frames");
        i = e;
      }
      device::Check(psg_store_sync(state->store, s), "psg_store_sync");
    } else {
      std::vector<SVector<Key>> dkeys(k);
      std::vector<const uint64_t*> kp(k);
      for (size_t j = 0; j < k; ++j) {
        dkeys[j] = detail::ToDeviceAsync(datas[j].keys, dev);
        dvals[j] = detail::ToDeviceAsync(datas[j].vals, dev);
        kp[j] = dkeys[j].data();
        vp[j] = dvals[j].data();
      }
      std::vector<int> ops(k, PSG_PUSH);
      std::vector<uint64_t> ns(k, n);
      bool any_spec = false;
      for (char c : spec) any_spec = any_spec || c;
      ServeRun(any_spec, (int)k, ops.data(), kp.data(), ns.data(), vp.data(), nullptr, s, status.data(),
               [&](int j) { return j < (int)spec.size() && spec[j] != 0; });
      for (size_t j = 0; j < k; ++j)
        if (status[j] != PSG_OK && !(j < spec.size() && spec[j])) device::Check(status[j], "psg_store_run");
      if (state->key_cache)
        for (size_t j = 0; j < k; ++j)
          if (status[j] == PSG_OK)
            Remember(dkeys[j], datas[j].keys.on_device(),
                     datas[j].keys.on_device() ? 0 : detail::KeyListHash(datas[j].keys.data(), n), s);
    }
    for (size_t j = 0; j < metas.size(); ++j) {
      if (status[j] != PSG_OK) server->RunRefuse(metas[j]);
      else server->Response(metas[j], KVPairs<Value>());
    }
  }

  /* A run through psg_store_run_status.  A run holding unconfirmed slices
   * (KVRunItem::spec) is served against this server's own key range, so a
   * slice with a key outside it is refused (nothing of it applied); a request
   * of the run that is not such a slice and was refused only for that
   * narrower range is then served again on the whole range. */
  template <typename IsSpec>
  void ServeRun(bool any_spec, int k, const int* ops, const uint64_t* const* kp, const uint64_t* ns,
                const void* const* vp, void* const* op, psg_stream s, int* status, IsSpec is_spec) {
    int served = 0;
    if (!any_spec) {
      const int rc = psg_store_run_status(state->store, k, ops, kp, ns, vp, op, s, &served, status);
      if (rc != PSG_OK) device::Check(rc, "psg_store_run");
      return;
    }
    const auto& r = PostOffice::Get()->GetServerRanges()[PostOffice::IDToRank(PostOffice::Get()->my_id())];
    device::Check(psg_store_set_key_range(state->store, r.begin, r.end), "psg_store_set_key_range");
    const int rc = psg_store_run_status(state->store, k, ops, kp, ns, vp, op, s, &served, status);
    device::Check(psg_store_set_key_range(state->store, 0, kMaxKey), "psg_store_set_key_range");
    if (rc != PSG_OK) device::Check(rc, "psg_store_run");
    for (int j = 0; j < k; ++j) {
      if (status[j] != PSG_ERR_RANGE || is_spec(j)) continue;
      const int rc1 = psg_store_run_status(state->store, 1, ops + j, kp + j, ns + j, vp + j, op ? op + j : nullptr, s,
                                           &served, status + j);
      if (rc1 != PSG_OK) device::Check(rc1, "psg_store_run");
    }
  }

  psg_store* store() const { return state->store; }
  size_t cached_key_lists() const { return state->cache.size(); }
  /* (key, value) pairs in key order, copied to host */
  void Dump(std::vector<Key>* keys, std::vector<Value>* vals) const {
    keys->clear();
    vals->clear();
    if (!state->store) return;
    psg_store_info info;
    device::Check(psg_store_get_info(state->store, &info), "psg_store_get_info");
    keys->resize(info.size);
    vals->resize(info.size);
    device::Check(psg_store_dump(state->store, keys->data(), vals->data()), "psg_store_dump");
  }

 private:
  uint64_t StoreSize() const {
    psg_store_info info;
    device::Check(psg_store_get_info(state->store, &info), "psg_store_get_info");
    return info.size;
  }
  // cache a full list under its hash (LRServer.h:136-141: the first one wins)
  // a Pull's output: the worker's own slice when it offered one of n values
  // (written in place: no reply frame, no merge), else a fresh HBM array
  static SVector<Value> PullOutput(KVServer<Value>* server, size_t n, int dev, bool* direct) {
    SVector<Value> d = server->TakeDirectOut(n);
    *direct = !d.empty();
    return *direct ? d : SVector<Value>::OnDevice(n, dev);
  }

  // worker_frame: dkeys is the request's own HBM frame (the worker's buffer,
  // or its hipIpc mapping), which the worker may rewrite once the request is
  // answered (psg.h) — the cache keeps a server-owned copy, as the reference
  // keeps its received copy (LRServer.h:139), so a later re-resolve never
  // reads another list, and no worker frame stays mapped.
  void Remember(const SVector<Key>& dkeys, bool worker_frame, uint64_t host_hash, psg_stream s) {
    const size_t n = dkeys.size();
    uint64_t h = host_hash;
    if (dkeys.on_device() && host_hash == 0)
      device::Check(psg_key_list_hash(dkeys.data(), n, &h, s), "psg_key_list_hash");
    if (state->cache.count(h)) return;
    Cached c;
    const int dev = PostOffice::Get()->device();
    if (worker_frame) {
      c.keys = SVector<Key>::OnDevice(n, dev);
      device::Check(psg_memcpy(c.keys.data(), dkeys.data(), n * sizeof(Key), 2 /* D2D */, s), "psg_memcpy D2D");
    } else {
      c.keys = dkeys;  // already the server's copy (ToDeviceAsync of a host frame)
    }
    c.slots = SVector<uint32_t>::OnDevice(n, dev);
    device::Check(psg_store_resolve(state->store, c.keys.data(), n, 0, c.slots.data(), s), "psg_store_resolve");
    device::Check(psg_store_slots_stretch(state->store, c.slots.data(), n, &c.stretch, s), "psg_store_slots_stretch");
    c.store_size = StoreSize();
    state->cache.emplace(h, std::move(c));
  }
  void Refresh(Cached& c, psg_stream s) {
    const uint64_t size = StoreSize();
    if (size == c.store_size) return;
    device::Check(psg_store_resolve(state->store, c.keys.data(), c.keys.size(), 0, c.slots.data(), s),
                  "psg_store_resolve");
    device::Check(psg_store_slots_stretch(state->store, c.slots.data(), c.keys.size(), &c.stretch, s),
                  "psg_store_slots_stretch");
    c.store_size = size;
  }
};

// ============================================================================
// KVServer

template <typename Value>
void KVServer<Value>::OnReceive(const Message& msg) {
  if (msg.meta.simple_app) {
    SimpleApp::OnReceive(msg);
    return;
  }
  const KVMeta meta = MetaOf(msg);
  const uint64_t ordinal = Take(meta.sender);
  bool device_frames, installed;
  RunHandle run;
  {
    std::unique_lock<std::mutex> lk(handle_mu_);
    handle_cv_.wait_for(lk, std::chrono::seconds(30), [this] { return static_cast<bool>(request_handle_); });
    installed = static_cast<bool>(request_handle_);
    device_frames = device_frames_;
    run = run_handle_;
  }
  CHECK(installed) << "no request handle installed 30 s after the first request";
  stage::Scope t_recv(meta.push ? "server.request.push" : "server.request.pull");
  KVPairs<Value> data;
  const size_t n = msg.data.size();
  direct_out_ = SVector<Value>();
  direct_taken_ = false;
  if (n && msg.meta.direct_reply && meta.pull) {
    // the last frame is not request data: it is where this Pull's (or
    // PushPull's) values may go — [keys, out] or [keys, vals, out]
    CHECK_EQ(n, meta.push ? (size_t)3 : (size_t)2);
    data.keys = msg.data[0];
    if (meta.push) data.vals = msg.data[1];
    if (device_frames) {
      direct_out_ = msg.data[n - 1];
      direct_ts_ = meta.timestamp;
      direct_sender_ = meta.sender;
    } else {
      data.keys = detail::ToHost(data.keys);
      data.vals = detail::ToHost(data.vals);
    }
  } else if (n) {
    CHECK_GE(n, (size_t)2);
    data.keys = msg.data[0];
    data.vals = msg.data[1];
    if (n > 2) {
      CHECK_EQ(n, (size_t)3);
      data.lens = msg.data[2];
      CHECK_EQ(data.lens.size(), data.keys.size());
    }
    if (!device_frames) {
      data.keys = detail::ToHost(data.keys);
      data.vals = detail::ToHost(data.vals);
      data.lens = detail::ToHost(data.lens);
    }
  }
  // A run of queued requests.  The reference's receive thread handles the
  // queued messages one at a time, in queue order (Customer.cpp:52-70); a
  // plain request taken here (no lens) may bring along the requests queued
  // right behind it — the very messages the thread would handle next, so
  // nothing is reordered — and the run's handle (KVServerDefaultHandle::Run)
  // serves them as that sequence:
  //   Pushes of one shape (one pass when their lists are one list: nw workers
  //     of a BSP round, or a worker's Pushes in flight), and
  //   requests of distinct senders, Pushes and Pulls (one pass when their
  //     lists interleave: the reference benchmark's `kMaxKey / num * i + rank`
  //     at nw workers, tests/test_kv_app_benchmark.cpp:47-52);
  // request by request otherwise.
  if (run && device_frames && detail::PushRunsOn() && PlainRequest(msg)) {
    const size_t kbytes = msg.data[0].size(), vbytes = msg.data[1].size();
    auto push_shape = [&](const Message& m) {
      return m.meta.push && !m.meta.pull && !m.meta.direct_reply && m.data.size() == 2 && m.data[0].size() == kbytes &&
             m.data[1].size() == vbytes;
    };
    bool all_push = push_shape(msg), distinct = true;
    std::vector<KVRunItem<Value>> items(1);
    items[0].meta = meta;
    items[0].data = data;
    items[0].out = direct_out_;
    items[0].spec = msg.meta.spec_slice;
    auto mate = [&](const Message& m) {
      if (m.meta.app_id != msg.meta.app_id || !PlainRequest(m)) return false;
      if (all_push && push_shape(m)) return true;
      if (!distinct || !detail::MixedRunsOn()) return false;
      for (const auto& it : items)
        if (it.meta.sender == m.meta.sender) return false;
      return true;
    };
    // The gather window (PS_RUN_GATHER_US, default 120; 0: off): when fewer
    // requests are queued than the senders this server has heard from lately,
    // wait up to that long for theirs to arrive — the requests of one step
    // reach a server microseconds apart, and a request taken alone costs a
    // whole pass over the store's lines.  The wait ends as soon as the head of
    // the queue is a message that may not join (PopIf's refusal: a message
    // that arrives while the window checks its senders is still taken).
    // A window that keeps timing out with nothing gained (a sender stopped
    // sending) is skipped for the next 64 requests.
    // With the ordinal rule (detail::RunGatherOrdinal) the window waits only
    // for the senders behind the run, for up to PS_RUN_GATHER_ORD_US.
    const bool by_ordinal = detail::RunGatherOrdinal() && detail::RunGatherMicros() > 0;
    int gather_us = gather_cool_ > 0 ? 0 : by_ordinal ? detail::RunGatherOrdMicros() : detail::RunGatherMicros();
    if (gather_us > 0 && !by_ordinal && detail::RunGatherAutoCap() > 0)
      gather_us = std::min(detail::RunGatherAutoCap(), std::max(gather_us, (int)run_us_));
    if (gather_cool_ > 0) --gather_cool_;
    const size_t want = gather_us > 0 ? RecentSenders(meta.sender) : 0;
    uint64_t low = ordinal;  // the run's lowest ordinal
    const auto t_gather = std::chrono::steady_clock::now();
    bool waited = false;
    Message next;
    int why = 0;
    while ((int)items.size() < kMaxRun) {
      bool refused = false;
      if (!customer_->TakeQueued(mate, &next, &refused)) {
        // (the head of the queue may not join: the run ends here, in queue order)
        if (refused) {
          why = 2;
          break;
        }
        const bool more = gather_us > 0 && (by_ordinal ? SendersBehind(items, low) : items.size() < want);
        if (!more) {
          why = 1;
          break;
        }
        if (std::chrono::steady_clock::now() - t_gather > std::chrono::microseconds(gather_us)) {
          if (by_ordinal) (void)SendersBehind(items, low, true);
          if (!waited && ++gather_idle_ >= 4) {
            gather_idle_ = 0;
            gather_cool_ = 64;
          }
          why = 3;
          break;
        }
        __builtin_ia32_pause();
        continue;
      }
      if (items.size() >= 1 && std::chrono::steady_clock::now() - t_gather > std::chrono::microseconds(1)) {
        waited = true;  // a request joined after the wait began
        gather_idle_ = 0;
      }
      NoteSender(next.meta.sender);
      low = std::min(low, Take(next.meta.sender));
      KVRunItem<Value> it;
      it.meta = MetaOf(next);
      for (const auto& o : items) distinct = distinct && o.meta.sender != it.meta.sender;
      all_push = all_push && push_shape(next);
      it.data.keys = next.data[0];
      if (next.meta.push) it.data.vals = next.data[1];
      if (next.meta.direct_reply) it.out = next.data[next.data.size() - 1];
      it.spec = next.meta.spec_slice;
      items.push_back(std::move(it));
    }
    // (a plain request on its own goes to the run handle too: the store
    // serves it as a strided pass when it knows its list's place in a learnt
    // interleaved layout, else as one request)
    detail::TraceGather(PostOffice::Get()->my_id(), meta.sender, ordinal, items.size(), why,
                        std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_gather).count());
    if (items.size() > 1 || detail::MixedRunsOn()) {
      direct_out_ = SVector<Value>();
      for (size_t j = 0; j < items.size(); ++j)
        detail::TraceRequest(PostOffice::Get()->my_id(), items[j].meta, items[j].data.keys.size(), items.size(), j);
      const auto t_run = std::chrono::steady_clock::now();
      run(items, this);
      const double us = std::chrono::duration<double, std::micro>(std::chrono::steady_clock::now() - t_run).count();
      run_us_ = run_us_ > 0 ? 0.75 * run_us_ + 0.25 * us : us;
      return;
    }
  }
  CHECK(!msg.meta.spec_slice) << "an unconfirmed slice reached a handle that does not check it";
  detail::TraceRequest(PostOffice::Get()->my_id(), meta, data.keys.size(), 1, 0);
  // called in place: a handle keeps its state across requests (KVApp.h:457)
  {
    stage::Scope t("server.handle");
    request_handle_(meta, data, this);
  }
  direct_out_ = SVector<Value>();
  direct_taken_ = false;
}

template <typename Value>
void KVServer<Value>::Response(const KVMeta& req, const KVPairs<Value>& res) {
  // the handle wrote this Pull's values into the worker's output in place
  Reply(req, res,
        direct_taken_.load() && req.timestamp == direct_ts_.load() && req.sender == direct_sender_.load());
}

template <typename Value>
void KVServer<Value>::Reply(const KVMeta& req, const KVPairs<Value>& res, bool direct, bool refused) {
  stage::Scope t("server.response", res.keys.size() * sizeof(Key) + res.vals.size() * sizeof(Value));
  Message msg;
  msg.meta.app_id = customer_->app_id();
  msg.meta.customer_id = req.customer_id;
  msg.meta.request = false;
  msg.meta.push = req.push;
  msg.meta.pull = req.pull;
  msg.meta.head = req.cmd;
  msg.meta.timestamp = req.timestamp;
  msg.meta.receiver = req.sender;
  // tells the worker that HBM frames reach this handle without a copy back
  msg.meta.hbm_handle = device_frames_.load();
  msg.meta.direct_reply = direct;
  if (msg.meta.direct_reply) CHECK(res.vals.empty()) << "a direct reply carries no values";
  // tells the worker it may send this server unconfirmed slices (KVWorker::Send)
  msg.meta.spec_slice = TakesSpecSlices();
  msg.meta.refused = refused;
  if (refused) CHECK(res.keys.empty() && !direct) << "a refusal carries nothing";
  if (res.keys.size()) {
    msg.AddData(res.keys);
    msg.AddData(res.vals);
    if (res.lens.size()) msg.AddData(res.lens);
  }
  PostOffice::Get()->van()->Send(msg);
}

// ============================================================================
// KVWorker

template <typename Value>
void KVWorker<Value>::DefaultSlicer(Data& send, const std::vector<Range>& ranges, SlicedKVs* sliced) {
  const size_t n = ranges.size();
  sliced->resize(n);
  std::vector<uint64_t> pos(n + 1, 0), vpos(n + 1, 0);
  const size_t nkeys = send.keys.size();
  if (send.keys.on_device() && n == 1 && send.lens.empty()) {
    // one server owns [0, kMaxKey): the slice is the whole request, no kernel
    // and no host sync.  The one key the reference's slicer would reject
    // (kMaxKey itself, KVApp.h:544) is rejected by the server's range check.
    CHECK_EQ(nkeys ? send.vals.size() / nkeys * nkeys : send.vals.size(), send.vals.size());
    pos[1] = nkeys;
    vpos[1] = send.vals.size();
  } else if (send.keys.on_device()) {
    stage::Scope t("worker.slice.device", nkeys * sizeof(Key));
    if (send.lens.size()) {
      CHECK_EQ(send.keys.size(), send.lens.size());
      CHECK(send.lens.on_device()) << "device keys need device lens";
    }
    device::SliceKeys(send.keys.data(), nkeys, send.lens.size() ? send.lens.data() : nullptr,
                      send.vals.size(), ranges, &pos, &vpos);
  } else {
    const Key* begin = send.keys.begin();
    const Key* end = send.keys.end();
    for (size_t i = 0; i < n; ++i) {
      if (i == 0) {
        pos[0] = std::lower_bound(begin, end, ranges[0].begin) - begin;
        begin += pos[0];
      } else {
        CHECK_EQ(ranges[i - 1].end, ranges[i].begin);
      }
      size_t len = std::lower_bound(begin, end, ranges[i].end) - begin;
      begin += len;
      pos[i + 1] = pos[i] + len;
    }
    CHECK_EQ(pos[n], nkeys);
    if (nkeys) {
      if (send.lens.empty()) {
        const size_t k = send.vals.size() / nkeys;
        CHECK_EQ(k * nkeys, send.vals.size());
        for (size_t i = 0; i <= n; ++i) vpos[i] = pos[i] * k;
      } else {
        CHECK_EQ(nkeys, send.lens.size());
        SVector<int> hl = detail::ToHost(send.lens);
        uint64_t acc = 0;
        for (size_t i = 0; i < n; ++i) {
          vpos[i] = acc;
          for (size_t j = pos[i]; j < pos[i + 1]; ++j) acc += hl[j];
        }
        vpos[n] = acc;
      }
    }
  }
  for (size_t i = 0; i < n; ++i) {
    auto& s = sliced->at(i);
    s.first = pos[i + 1] != pos[i];
    if (!s.first) continue;
    s.second.keys = send.keys.Slice(pos[i], pos[i + 1]);
    s.second.vals = send.vals.Slice(vpos[i], vpos[i + 1]);
    if (send.lens.size()) s.second.lens = send.lens.Slice(pos[i], pos[i + 1]);
  }
}

template <typename Value>
void KVWorker<Value>::Send(int timestamp, bool push, bool pull, int cmd, const Data& kvs, bool direct,
                           const SVector<Value>* outs) {
  stage::Scope t_send(push ? "worker.send.push" : "worker.send.pull");
  SlicedKVs sliced;
  const std::vector<Range>& ranges = PostOffice::Get()->GetServerRanges();
  const size_t ns = ranges.size();
  // Unconfirmed slices (PS_SPEC_SLICE=0: off): an HBM key list this thread sliced
  // before is sent on the bounds it had then, without the slicer's kernel and
  // readback, when every server's handle checks each key against its own
  // range (a wrong bound puts some key outside its server's range; that
  // server refuses its slice, applying nothing, and Refused re-sends those
  // keys sliced for real).  Not with lens, a custom slicer, or a Pull merged
  // on the host (its replies must be the servers' slices).
  bool spec = false;
  std::vector<uint64_t> hint;
  const size_t nkeys = kvs.keys.size();
  if (detail::SpecSliceOn() && default_slicer_ && ns > 1 && nkeys && kvs.keys.on_device() && kvs.lens.empty() &&
      (!pull || direct) && servers_take_spec_.load()) {
    bool stale = false;
    {
      std::lock_guard<std::mutex> lk(mu_);
      stale = spec_stale_.erase(kvs.keys.data()) > 0;
    }
    int found = 0;
    hint.assign(ns + 1, 0);
    if (!stale)
      device::Check(psg_slice_hint(kvs.keys.data(), nkeys, (int)ns, ranges[0].begin, hint.data(), &found),
                    "psg_slice_hint");
    if (found && hint[ns] == nkeys) {
      const size_t per = kvs.vals.size() / nkeys;
      CHECK_EQ(per * nkeys, kvs.vals.size());
      sliced.resize(ns);
      for (size_t i = 0; i < ns; ++i) {
        auto& sl = sliced[i];
        sl.first = hint[i + 1] != hint[i];
        if (!sl.first) continue;
        sl.second.keys = kvs.keys.Slice(hint[i], hint[i + 1]);
        sl.second.vals = kvs.vals.Slice(hint[i] * per, hint[i + 1] * per);
      }
      spec = true;
      SpecSend sp;
      sp.push = push;
      sp.pull = pull;
      sp.direct = direct;
      sp.cmd = cmd;
      sp.kvs = kvs;
      sp.has_outs = outs != nullptr;
      if (outs) sp.outs = *outs;
      sp.pos = hint;
      std::lock_guard<std::mutex> lk(mu_);
      spec_sends_[timestamp] = std::move(sp);
    }
  }
  if (!spec) slicer_(const_cast<Data&>(kvs), ranges, &sliced);
  int skipped = 0;
  for (auto& sl : sliced)
    if (!sl.first) ++skipped;
  customer_->AddResponse(timestamp, skipped);
  if ((size_t)skipped == sliced.size()) RunCallback(timestamp);
  for (size_t i = 0; i < sliced.size(); ++i) {
    if (!sliced[i].first) continue;
    SendOne(timestamp, push, pull, cmd, kvs.priority, kvs, sliced[i].second, direct, outs, (int)i, spec);
  }
}

// One server's slice of a request (Send, SendPieces): `kv` is a slice of
// `whole`, the request as the caller gave it.
template <typename Value>
void KVWorker<Value>::SendOne(int timestamp, bool push, bool pull, int cmd, int priority, const Data& whole,
                              const Data& kv, bool direct, const SVector<Value>* outs, int server_rank, bool spec) {
  Message msg;
  msg.meta.app_id = customer_->app_id();
  msg.meta.customer_id = customer_->customer_id();
  msg.meta.request = true;
  msg.meta.push = push;
  msg.meta.pull = pull;
  msg.meta.head = cmd;
  msg.meta.timestamp = timestamp;
  msg.meta.receiver = PostOffice::ServerRankToID(server_rank);
  msg.meta.priority = priority;
  msg.meta.direct_reply = direct;
  msg.meta.spec_slice = spec;
  SVector<Value> out_slice;
  if (direct && outs) {
    // a PushPull: the output slice at this server's values' offset, found
    // from where its vals slice sits in the request (a slicer that copied
    // the values instead of slicing them gets no offer)
    const Value* base = whole.vals.data();
    const Value* v = kv.vals.data();
    if (kv.vals.size() && v >= base && v + kv.vals.size() <= base + whole.vals.size()) {
      const size_t off = (size_t)(v - base);
      out_slice = outs->Slice(off, off + kv.vals.size());
    } else {
      msg.meta.direct_reply = false;
    }
  }
  bool drop_vals = false;
  if (direct && !outs) {
    // a Pull whose vals frame is the caller's output: offered only when this
    // server's vals slice is the output at its keys' offset (a custom slicer
    // that copied or remapped the values gets no offer, and a plain Pull
    // request without values, as the reference sends)
    const Key* kbase = whole.keys.data();
    const Key* k = kv.keys.data();
    const size_t per = whole.keys.size() ? whole.vals.size() / whole.keys.size() : 0;
    const bool keys_inside = kv.keys.size() && k >= kbase && k + kv.keys.size() <= kbase + whole.keys.size();
    const bool ok = keys_inside && per && kv.vals.size() == kv.keys.size() * per &&
                    kv.vals.data() == whole.vals.data() + (size_t)(k - kbase) * per;
    if (!ok) {
      msg.meta.direct_reply = false;
      drop_vals = true;
    }
  }
  if (kv.keys.size()) {
    msg.AddData(kv.keys);
    msg.AddData(drop_vals ? SVector<Value>() : kv.vals);
    if (kv.lens.size()) msg.AddData(kv.lens);
    if (msg.meta.direct_reply && outs) msg.AddData(out_slice);
  }
  PostOffice::Get()->van()->Send(msg);
}

// A server refused its unconfirmed slice [pos[r], pos[r+1]) of request
// `timestamp` (a key outside its range: the key list changed since it was
// last sliced; nothing of that slice was applied).  The list is sliced for
// real and those keys go to the servers that own them, as requests of the same
// timestamp; the request now waits for their replies too.  The servers that
// took their slices hold exactly their keys (each accepted slice lies in its
// server's range), so every key is still applied once.
template <typename Value>
void KVWorker<Value>::Refused(const Message& msg) {
  const int ts = msg.meta.timestamp;
  ++refused_;
  SpecSend sp;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = spec_sends_.find(ts);
    CHECK(it != spec_sends_.end()) << "a refusal of request " << ts << ", which was not sent on unconfirmed slices";
    sp = it->second;
    spec_stale_[sp.kvs.keys.data()] = true;  // the sender's thread slices it for real next time
  }
  const int r = PostOffice::IDToRank(msg.meta.sender);
  const std::vector<Range>& ranges = PostOffice::Get()->GetServerRanges();
  CHECK_LT((size_t)r + 1, sp.pos.size());
  std::vector<uint64_t> pos, vpos;
  device::SliceKeys(sp.kvs.keys.data(), sp.kvs.keys.size(), nullptr, sp.kvs.vals.size(), ranges, &pos, &vpos);
  int sent = 0;
  SendPieces(ts, sp, sp.pos[r], sp.pos[r + 1], pos, &sent);
  // (before this reply is counted: the request now waits for `sent` more)
  customer_->ExpectMore(ts, sent);
}

template <typename Value>
void KVWorker<Value>::SendPieces(int timestamp, const SpecSend& sp, uint64_t a, uint64_t b,
                                 const std::vector<uint64_t>& pos, int* sent) {
  const size_t n = sp.kvs.keys.size();
  const size_t per = n ? sp.kvs.vals.size() / n : 0;
  *sent = 0;
  for (size_t i = 0; i + 1 < pos.size(); ++i) {
    const uint64_t lo = std::max<uint64_t>(a, pos[i]), hi = std::min<uint64_t>(b, pos[i + 1]);
    if (lo >= hi) continue;
    Data kv;
    kv.keys = sp.kvs.keys.Slice(lo, hi);
    kv.vals = sp.kvs.vals.Slice(lo * per, hi * per);
    SendOne(timestamp, sp.push, sp.pull, sp.cmd, sp.kvs.priority, sp.kvs, kv, sp.direct,
            sp.has_outs ? &sp.outs : nullptr, (int)i, false);
    ++*sent;
  }
}

template <typename Value>
void KVWorker<Value>::OnReceive(const Message& msg) {
  if (msg.meta.simple_app) {
    SimpleApp::OnReceive(msg);
    return;
  }
  const int ts = msg.meta.timestamp;
  if (msg.meta.hbm_handle && !servers_take_hbm_.load()) NoteHbmServer(msg.meta.sender);
  if (msg.meta.spec_slice && !servers_take_spec_.load()) NoteSpecServer(msg.meta.sender);
  if (msg.meta.refused) {
    Refused(msg);
    return;  // (counted as a reply; the re-sent pieces are waited for)
  }
  if (msg.meta.pull) {
    CHECK_GE(msg.data.size(), (size_t)2);
    Reply r;
    r.kv.keys = msg.data[0];
    r.kv.vals = msg.data[1];
    if (msg.data.size() > 2) r.kv.lens = msg.data[2];
    r.sender = msg.meta.sender;
    r.direct = msg.meta.direct_reply;
    std::lock_guard<std::mutex> lk(mu_);
    recv_kvs_[ts].push_back(std::move(r));
  }
  // the tracker is bumped after this handle returns (Customer.cpp:58-67)
  if (customer_->GetResponse(ts) == customer_->NumExpected(ts) - 1) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      spec_sends_.erase(ts);
    }
    RunCallback(ts);
  }
}

template <typename Value>
void KVWorker<Value>::RunCallback(int timestamp) {
  Callback cb;
  {
    std::lock_guard<std::mutex> lk(mu_);
    auto it = callbacks_.find(timestamp);
    if (it == callbacks_.end()) return;
    cb = std::move(it->second);
    callbacks_.erase(it);
  }
  CHECK(static_cast<bool>(cb));
  cb();
}

template <typename Value>
template <typename C, typename D>
int KVWorker<Value>::AddPullCB(const SVector<Key>& keys, C* vals, D* lens, int cmd, const Callback& cb) {
  (void)cmd;
  int ts = customer_->NewRequest(kServerGroup);
  AddCallback(ts, [this, ts, keys, vals, lens, cb]() mutable {
    std::vector<Reply> kvs;
    {
      std::lock_guard<std::mutex> lk(mu_);
      auto it = recv_kvs_.find(ts);
      if (it != recv_kvs_.end()) {
        kvs.swap(it->second);
        recv_kvs_.erase(it);
      }
    }
    MergePull(keys, kvs, vals, lens);
    if (cb) cb();
  });
  return ts;
}

template <typename Value>
template <typename C, typename D>
void KVWorker<Value>::MergePull(const SVector<Key>& keys, std::vector<Reply>& kvs, C* vals, D* lens) {
  stage::Scope t_merge("worker.pull.merge", keys.size() * sizeof(Value));
  size_t total_key = 0, total_val = 0;
  int ndev = 0, ndirect = 0;
  for (const auto& r : kvs) {
    const auto& s = r.kv;
    if (!s.keys.on_device() && !keys.on_device() && s.keys.size()) {
      Range range = FindRange(keys, s.keys.front(), s.keys.back() + 1);
      CHECK_EQ(range.size(), s.keys.size()) << "unmatched keys size from one server";
    }
    if (lens) CHECK_EQ(s.lens.size(), s.keys.size());
    total_key += s.keys.size();
    if (r.direct) {
      // written in place: its slice of the output, keys x values per key
      CHECK(!lens && vals && keys.size()) << "a direct reply needs a sized output and no lens";
      total_val += s.keys.size() * (vals->size() / keys.size());
      ++ndirect;
      continue;
    }
    total_val += s.vals.size();
    ndev += s.vals.on_device() ? 1 : 0;
  }
  CHECK_EQ(total_key, keys.size()) << "lost some servers?";
  CHECK(ndev == 0 || ndev + ndirect == (int)kvs.size()) << "pull replies mix host and HBM frames";
  // order the replies by their first key (KVApp.h:694-696); replies whose keys
  // are in HBM are ordered by server rank, which the default ranges make the same
  if (!keys.on_device()) {
    std::sort(kvs.begin(), kvs.end(), [](const Reply& a, const Reply& b) {
      return a.kv.keys.front() < b.kv.keys.front();
    });
  } else {
    std::sort(kvs.begin(), kvs.end(), [](const Reply& a, const Reply& b) { return a.sender < b.sender; });
  }
  CHECK_NOTNULL(vals);
  const int out_dev = detail::DeviceOf(vals);
  if (vals->empty()) {
    CHECK_LT(out_dev, 0) << "an HBM pull output must be sized by the caller";
    stage::Scope t("worker.pull.merge.resize_output", total_val * sizeof(Value));
    // the reference resizes the caller's vector (KVApp.h:703-711); its fresh
    // pages are faulted in first, in parallel and on huge pages (PrefaultHost)
    // — a 40 MB reply's resize took 6.4-8 ms one 4 KiB fault at a time
    if (out_dev < 0) {
      vals->reserve(total_val);
      PrefaultHost(vals->data(), total_val * sizeof(Value));
    }
    vals->resize(total_val);
  } else {
    CHECK_EQ(vals->size(), total_val);
  }
  if (ndirect == (int)kvs.size()) {
    // every server wrote its values in place: nothing to merge
  } else if (ndev == 0 && out_dev < 0) {
    stage::Scope t("worker.pull.merge.copy", total_val * sizeof(Value));
    Value* p = vals->data();
    for (const auto& r : kvs) {
      if (r.kv.vals.size()) HostCopy(p, r.kv.vals.data(), r.kv.vals.size() * sizeof(Value));
      p += r.kv.vals.size();
    }
  } else if (total_val) {
    std::vector<psg_segment> segs;
    std::vector<SVector<Value>> staged;  // host replies going to an HBM output
    const int my_dev = PostOffice::Get()->device();
    const size_t per_key = keys.size() ? total_val / keys.size() : 0;
    std::vector<uint64_t> offs;  // where each segment goes in the output
    uint64_t done_vals = 0;      // values of the replies before j (direct ones included)
    for (size_t j = 0; j < kvs.size(); ++j) {
      if (kvs[j].direct) {
        done_vals += kvs[j].kv.keys.size() * per_key;
        continue;
      }
      const SVector<Value>& v = kvs[j].kv.vals;
      const Value* src = v.data();
      if (!v.on_device() && v.size()) {
        staged.push_back(detail::ToDevice(v, out_dev >= 0 ? out_dev : my_dev));
        src = staged.back().data();
      }
      segs.push_back(psg_segment{src, v.size(), (uint64_t)j});  // j: already in order
      offs.push_back(done_vals);
      done_vals += v.size();
    }
    if (out_dev >= 0 && ndirect == 0) {
      device::Merge(&segs, sizeof(Value), vals->data(), total_val);
    } else if (out_dev >= 0) {
      // some servers wrote in place: copy the other replies to their slices
      for (size_t t = 0; t < segs.size(); ++t) {
        std::vector<psg_segment> one{segs[t]};
        device::Merge(&one, sizeof(Value), vals->data() + offs[t], segs[t].count);
      }
    } else {
      SVector<Value> tmp = SVector<Value>::OnDevice(total_val, my_dev);
      device::Merge(&segs, sizeof(Value), tmp.data(), total_val);
      device::StageToHost(vals->data(), tmp.data(), total_val * sizeof(Value));
    }
  }
  if (lens) {
    CHECK_LT(detail::DeviceOf(lens), 0) << "pull lens are returned in host memory";
    if (lens->empty())
      lens->resize(keys.size());
    else
      CHECK_EQ(lens->size(), keys.size());
    int* p = lens->data();
    for (const auto& r : kvs) {
      SVector<int> hl = detail::ToHost(r.kv.lens);
      if (hl.size()) std::memcpy(p, hl.data(), hl.size() * sizeof(int));
      p += hl.size();
    }
  }
}

}  // namespace ps
