// ps/lr_handle.h — the LR server's request handle with the model in HBM.
//
// Reference: lr::LRServer::RequestHandle (tests/src/LRServer.h:122-207) with
// Adam (tests/src/Adam.h:28-34).  Sync mode (SYNC_MODE=0): every worker's
// gradient Push is accumulated into a merge buffer in arrival order
// (`merge_buf_.vals[i] += req_data.vals[i]`, :158-160) and answered only when
// NumWorkers() pushes have arrived; then `weight -= lr * merge` (optionally
// through Adam) runs once and all deferred responses go out (:163-177).  Async
// mode (SYNC_MODE=1) applies every push at once (:179-189).  A push with
// cmd == 1 from worker 0 ends an iteration (:193-195).  A Pull returns the
// weights (:196-206).  Key caching (USE_KEY_CACHING, :127-142): a request with
// more than one key is cached under the hash of its key list; a request with
// ONE key names a cached list by that hash (the worker side: LRWorker.h:214-219).
//
// Here the weights are a DENSE psg store in HBM and a BSP round is ONE kernel:
// the round's gradient frames are kept (referenced, not copied) in arrival
// order and psg_lr_apply_sum merges them from 0 and applies SGD / Adam in the
// same pass — no merge buffer is written, read back or cleared.  Same f32 adds
// in the same arrival order and the same f32/f64 update, so the model is
// bit-identical to the reference's.  Keys must be 0..n-1, one per feature, as
// the reference's CHECK_EQ(n, weight_.size()) (:145) requires.  Register with
// KVServer::SetDeviceRequestHandle.
#pragma once
#include <memory>
#include <unordered_map>
#include <vector>

#include "ps/kv_app.h"

namespace ps {

struct KVServerLRHandle {
  struct State {
    psg_store* weights = nullptr;
    psg_adam* adam = nullptr;
    psg_store* fold = nullptr;       // merge of rounds with more than 16 workers
    bool folded = false;
    std::vector<SVector<float>> grads;  // this round's gradient frames, arrival order
    std::vector<KVMeta> pending;
    std::unordered_map<uint64_t, SVector<Key>> key_cache;
    uint64_t n = 0;
    float lr = 0.01f;
    bool sync = true;
    bool use_key_cache = false;
    int iteration = 0;
    ~State() {
      if (adam) psg_adam_destroy(adam);
      if (fold) psg_store_destroy(fold);
      if (weights) psg_store_destroy(weights);
    }
  };
  std::shared_ptr<State> st = std::make_shared<State>();
  static constexpr int kMaxGrads = 16;  // gradient frames one psg_lr_apply_sum pass merges

  /* init_weight: the model at start (LRServer's InitWeight, LRServer.h:36-63);
   * sync: SYNC_MODE == 0; use_adam: USE_ADAM set (Adam gets the f32 learning
   * rate widened to double, as LRServer.h:83-84 constructs it); use_key_cache:
   * USE_KEY_CACHING set. */
  KVServerLRHandle(const std::vector<float>& init_weight, float learning_rate, bool sync,
                   bool use_adam, int start_iteration = 0, bool use_key_cache = false) {
    State& s = *st;
    s.n = init_weight.size();
    s.lr = learning_rate;
    s.sync = sync;
    s.use_key_cache = use_key_cache;
    s.iteration = start_iteration;
    const int dev = PostOffice::Get()->device();
    CHECK_GE(dev, 0) << "KVServerLRHandle: the model lives in HBM and this node has no GPU";
    CHECK_GT(s.n, 0u);
    device::Check(psg_store_create(PSG_STORE_DENSE, PSG_F32, 0, s.n, s.n, &s.weights), "psg_store_create");
    if (use_adam)
      device::Check(psg_adam_create(s.n, (double)learning_rate, 0.9, 0.999, 1e-8, &s.adam), "psg_adam_create");
    psg_store_info info;
    device::Check(psg_store_get_info(s.weights, &info), "psg_store_get_info");
    device::CopySync(info.vals, init_weight.data(), s.n * sizeof(float), 0);
  }

  void operator()(const KVMeta& meta, const KVPairs<float>& req, KVServer<float>* server) {
    State& s = *st;
    size_t n = req.keys.size();
    if (s.use_key_cache) n = ResolveKeyCache(s, req.keys);
    CHECK_EQ(n, s.n) << "Unmatched keys";
    psg_stream strm = device::ThreadStream();
    if (meta.push) {
      CHECK_EQ(n, req.vals.size());
      // the frame itself (HBM) or its async staging copy: referenced until the apply
      SVector<float> g = detail::ToDevice(req.vals, PostOffice::Get()->device());
      if (s.sync) {
        s.grads.push_back(g);
        s.pending.push_back(meta);
        const bool last = (int)s.pending.size() == NumWorkersOfJob();
        if (!last && (int)s.grads.size() == kMaxGrads) FoldGrads(s, strm);
        if (last) {
          ApplyRound(s, strm, /*from_zero=*/true);
          for (const auto& r : s.pending) server->Response(r);
          s.pending.clear();
        }
      } else {
        s.grads.push_back(g);
        ApplyRound(s, strm, /*from_zero=*/false);
        server->Response(meta);
      }
      if (meta.cmd == 1 && meta.sender == PostOffice::WorkerRankToID(0)) ++s.iteration;
    }
    if (meta.pull) {
      KVPairs<float> res;
      res.keys = req.keys;
      auto dout = SVector<float>::OnDevice(n, PostOffice::Get()->device());
      device::Check(psg_store_handle(s.weights, PSG_PULL, nullptr, 0, nullptr, dout.data(), n, strm), "pull");
      device::Check(psg_store_sync(s.weights, strm), "psg_store_sync");  // the reply in memory
      res.vals = req.keys.on_device() ? dout : detail::ToHost(dout);
      server->Response(meta, res);
    }
  }

  /* host copy of the model */
  std::vector<float> GetWeight() const {
    std::vector<float> w(st->n);
    psg_store_info info;
    device::Check(psg_store_get_info(st->weights, &info), "psg_store_get_info");
    device::CopySync(w.data(), info.vals, st->n * sizeof(float), 1);
    return w;
  }
  int iteration() const { return st->iteration; }
  size_t cached_key_lists() const { return st->key_cache.size(); }

 private:
  static int NumWorkersOfJob() { return PostOffice::Get()->num_workers(); }

  // LRServer.h:127-142: one key names a cached list, more than one key is cached.
  static size_t ResolveKeyCache(State& s, const SVector<Key>& keys) {
    SVector<Key> hk = detail::ToHost(keys);
    if (hk.size() == 1) {
      auto it = s.key_cache.find(hk[0]);
      CHECK(it != s.key_cache.end()) << "Keys don't exist with hash value: " << hk[0];
      return it->second.size();
    }
    const uint64_t h = detail::KeyListHash(hk.data(), hk.size());
    if (s.key_cache.count(h) == 0) s.key_cache[h] = hk;
    return hk.size();
  }

  // More than kMaxGrads workers in a round: the first frames are merged into a
  // fold buffer (0 + g0 + g1 + ..., the same adds in the same order), which
  // then heads the list of the final pass.
  static void FoldGrads(State& s, psg_stream strm) {
    if (!s.fold)
      device::Check(psg_store_create(PSG_STORE_DENSE, PSG_F32, 0, s.n, s.n, &s.fold), "psg_store_create");
    if (!s.folded) device::Check(psg_store_clear(s.fold, strm), "psg_store_clear");
    for (const auto& g : s.grads)
      device::Check(psg_store_handle(s.fold, PSG_PUSH, nullptr, 0, g.data(), nullptr, s.n, strm), "fold push");
    device::Check(psg_store_sync(s.fold, strm), "psg_store_sync");
    s.grads.clear();
    s.folded = true;
  }

  static void ApplyRound(State& s, psg_stream strm, bool from_zero) {
    std::vector<const float*> g;
    if (s.folded) {
      psg_store_info fi;
      device::Check(psg_store_get_info(s.fold, &fi), "psg_store_get_info");
      g.push_back((const float*)fi.vals);
    }
    for (const auto& x : s.grads) g.push_back(x.data());
    device::Check(psg_lr_apply_sum(s.weights, g.data(), (int)g.size(), from_zero && !s.folded ? 1 : 0, s.n,
                                   s.lr, s.adam, s.iteration, strm),
                  "psg_lr_apply_sum");
    device::Check(psg_store_sync(s.weights, strm), "psg_store_sync");  // frames are released below
    s.grads.clear();
    s.folded = false;
  }
};

}  // namespace ps
