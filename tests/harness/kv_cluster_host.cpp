// kv_cluster_host.cpp — exercises the host runtime (Customer, PostOffice,
// local Van, DefaultSlicer on host keys, pull merge, barriers, callbacks,
// priorities, lens) with a host-memory request handle, so it runs without a
// GPU.  Built and run by tests/test_host_runtime.py; every check is a CHECK,
// so a wrong result exits non-zero.
#include <atomic>
#include <cstdlib>
#include <cmath>
#include <map>
#include <mutex>
#include <unordered_map>

#include "ps/ps.h"

using namespace ps;

// A host store keyed by Key, one value per key, or `lens[i]` values per key
// when lens travel (test code: the product handle keeps its store in HBM).
struct HostHandle {
  struct State {
    std::mutex mu;
    std::unordered_map<Key, std::vector<float>> store;
  };
  std::shared_ptr<State> st = std::make_shared<State>();

  void operator()(const KVMeta& meta, const KVPairs<float>& req, KVServer<float>* server) {
    std::lock_guard<std::mutex> lk(st->mu);
    const size_t n = req.keys.size();
    KVPairs<float> res;
    // a push carries its lens; a pull returns the stored length of every key
    std::vector<size_t> off(n + 1, 0);
    for (size_t i = 0; i < n; ++i) {
      size_t len = 1;
      if (req.lens.size()) {
        len = (size_t)req.lens[i];
      } else if (!meta.push) {
        auto it = st->store.find(req.keys[i]);
        len = it == st->store.end() ? 1 : std::max<size_t>(1, it->second.size());
      }
      off[i + 1] = off[i] + len;
    }
    if (meta.push) CHECK_EQ(off[n], req.vals.size());
    if (meta.pull) {
      res.keys = req.keys;
      res.vals.resize(off[n]);
      res.lens.resize(n);
      for (size_t i = 0; i < n; ++i) res.lens[i] = (int)(off[i + 1] - off[i]);
    }
    for (size_t i = 0; i < n; ++i) {
      auto& v = st->store[req.keys[i]];
      const size_t len = off[i + 1] - off[i];
      if (v.size() < len) v.resize(len, 0.f);
      for (size_t j = 0; j < len; ++j) {
        if (meta.push) v[j] += req.vals[off[i] + j];
        if (meta.pull) res.vals[off[i] + j] = v[j];
      }
    }
    server->Response(meta, res);
  }
};

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  if (IsServer()) {
    auto server = new KVServer<float>(0);
    server->SetRequestHandle(HostHandle());
    RegisterExitCallback([server]() { delete server; });
  }
  if (IsWorker()) {
    KVWorker<float> kv(0, 0);
    const int rank = MyRank(), nw = NumWorkers();
    // keys per request: argv[4] when given (large requests exercise the
    // shared-memory frames of process mode), else 20000
    const int num = argc > 4 ? std::atoi(argv[4]) : 20000;
    // disjoint keys per worker (test_kv_app.cpp layout)
    std::vector<Key> keys(num);
    std::vector<float> vals(num);
    for (int i = 0; i < num; ++i) {
      keys[i] = kMaxKey / num * i + rank;
      vals[i] = (float)((i * 7 + rank) % 1000);
    }
    std::vector<int> ts;
    for (int r = 0; r < 10; ++r) ts.push_back(kv.Push(keys, vals));
    for (int t : ts) kv.Wait(t);
    std::vector<float> rets;
    kv.Wait(kv.Pull(keys, &rets));
    CHECK_EQ(rets.size(), (size_t)num);
    for (int i = 0; i < num; ++i) CHECK_EQ(rets[i], vals[i] * 10) << "i=" << i;
    std::vector<float> outs;
    kv.Wait(kv.PushPull(keys, vals, &outs));
    for (int i = 0; i < num; ++i) CHECK_EQ(outs[i], vals[i] * 11);

    // shared keys: every worker adds into the same store entries
    std::vector<Key> shared(num);
    for (int i = 0; i < num; ++i) shared[i] = kMaxKey / num * i + 12345;
    std::vector<float> one(num, 1.0f + rank);
    kv.Wait(kv.Push(shared, one));
    Barrier(0, kWorkerGroup);
    std::vector<float> got;
    kv.Wait(kv.Pull(shared, &got));
    const float expect = (float)(nw * (nw + 1) / 2);
    for (int i = 0; i < num; ++i) CHECK_EQ(got[i], expect);
    Barrier(0, kWorkerGroup);

    // lens: key i carries (i % 3) + 1 values; pull returns values and lens
    const int nl = 999;
    std::vector<Key> lk(nl);
    std::vector<int> lens(nl);
    std::vector<float> lv;
    for (int i = 0; i < nl; ++i) {
      lk[i] = kMaxKey / nl * i + 777 + rank;
      lens[i] = i % 3 + 1;
      for (int j = 0; j < lens[i]; ++j) lv.push_back((float)(i + j));
    }
    kv.Wait(kv.Push(lk, lv, lens));
    std::vector<float> lo;
    std::vector<int> ll;
    kv.Wait(kv.Pull(lk, &lo, &ll, 0, nullptr));
    CHECK_EQ(lo.size(), lv.size());
    for (size_t j = 0; j < lv.size(); ++j) CHECK_EQ(lo[j], lv[j]);
    for (int i = 0; i < nl; ++i) CHECK_EQ(ll[i], lens[i]);

    // callbacks run once the request completed; zero-copy ZPull into an SVector
    std::atomic<int> fired{0};
    SVector<Key> sk(keys);
    SVector<float> sv;
    int t = kv.ZPull(sk, &sv, nullptr, 0, [&fired]() { fired++; });
    kv.Wait(t);
    CHECK_EQ(fired.load(), 1);
    for (int i = 0; i < num; ++i) CHECK_EQ(sv[i], vals[i] * 11);

    // empty request completes without any message
    std::vector<float> none;
    kv.Wait(kv.Pull(std::vector<Key>{}, &none));
    CHECK(none.empty());
    std::cout << "worker " << rank << " ok" << std::endl;
  }
  Finalize(0, true);
  return 0;
}
