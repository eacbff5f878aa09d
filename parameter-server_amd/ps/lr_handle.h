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
// weights (:196-206).
//
// Here the weights and the merge buffer are DENSE psg stores in HBM; the merge
// is the psg_store_handle accumulate kernel (same per-element f32 adds in the
// same arrival order), the update is psg_lr_apply (same f32/f64 operation
// order, bit-identical).  Keys must be 0..n-1, one per feature, as the
// reference's CHECK_EQ(n, weight_.size()) (:145) requires.  Register with
// KVServer::SetDeviceRequestHandle.
#pragma once
#include <memory>
#include <vector>

#include "ps/kv_app.h"

namespace ps {

struct KVServerLRHandle {
  struct State {
    psg_store* weights = nullptr;
    psg_store* merge = nullptr;
    psg_adam* adam = nullptr;
    std::vector<KVMeta> pending;
    uint64_t n = 0;
    float lr = 0.01f;
    bool sync = true;
    int iteration = 0;
    ~State() {
      if (adam) psg_adam_destroy(adam);
      if (merge) psg_store_destroy(merge);
      if (weights) psg_store_destroy(weights);
    }
  };
  std::shared_ptr<State> st = std::make_shared<State>();

  /* init_weight: the model at start (LRServer's InitWeight, LRServer.h:36-63);
   * sync: SYNC_MODE == 0; use_adam: USE_ADAM set (Adam gets the f32 learning
   * rate widened to double, as LRServer.h:83-84 constructs it). */
  KVServerLRHandle(const std::vector<float>& init_weight, float learning_rate, bool sync,
                   bool use_adam, int start_iteration = 0) {
    State& s = *st;
    s.n = init_weight.size();
    s.lr = learning_rate;
    s.sync = sync;
    s.iteration = start_iteration;
    const int dev = PostOffice::Get()->device();
    CHECK_GE(dev, 0) << "KVServerLRHandle: the model lives in HBM and this node has no GPU";
    CHECK_GT(s.n, 0u);
    device::Check(psg_store_create(PSG_STORE_DENSE, PSG_F32, 0, s.n, s.n, &s.weights), "psg_store_create");
    device::Check(psg_store_create(PSG_STORE_DENSE, PSG_F32, 0, s.n, s.n, &s.merge), "psg_store_create");
    if (use_adam)
      device::Check(psg_adam_create(s.n, (double)learning_rate, 0.9, 0.999, 1e-8, &s.adam), "psg_adam_create");
    psg_store_info info;
    device::Check(psg_store_get_info(s.weights, &info), "psg_store_get_info");
    device::CopySync(info.vals, init_weight.data(), s.n * sizeof(float), 0);
  }

  void operator()(const KVMeta& meta, const KVPairs<float>& req, KVServer<float>* server) {
    State& s = *st;
    const size_t n = req.keys.size();
    CHECK_EQ(n, s.n) << "Unmatched keys";
    psg_stream strm = device::ThreadStream();
    if (meta.push) {
      CHECK_EQ(n, req.vals.size());
      SVector<float> g = detail::ToDevice(req.vals, PostOffice::Get()->device());
      if (s.sync) {
        device::Check(psg_store_handle(s.merge, PSG_PUSH, nullptr, 0, g.data(), nullptr, n, strm),
                      "merge push");
        s.pending.push_back(meta);
        if ((int)s.pending.size() == NumWorkersOfJob()) {
          psg_store_info mi;
          device::Check(psg_store_get_info(s.merge, &mi), "psg_store_get_info");
          device::Check(psg_lr_apply(s.weights, (const float*)mi.vals, n, s.lr, s.adam, s.iteration, strm),
                        "psg_lr_apply");
          device::Check(psg_store_clear(s.merge, strm), "psg_store_clear");
          device::Check(psg_stream_sync(strm), "psg_stream_sync");
          for (const auto& r : s.pending) server->Response(r);
          s.pending.clear();
        }
      } else {
        device::Check(psg_lr_apply(s.weights, g.data(), n, s.lr, s.adam, s.iteration, strm), "psg_lr_apply");
        device::Check(psg_stream_sync(strm), "psg_stream_sync");
        server->Response(meta);
      }
      if (meta.cmd == 1 && meta.sender == PostOffice::WorkerRankToID(0)) ++s.iteration;
    }
    if (meta.pull) {
      KVPairs<float> res;
      res.keys = req.keys;
      auto dout = SVector<float>::OnDevice(n, PostOffice::Get()->device());
      device::Check(psg_store_handle(s.weights, PSG_PULL, nullptr, 0, nullptr, dout.data(), n, strm), "pull");
      device::Check(psg_stream_sync(strm), "psg_stream_sync");
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

 private:
  static int NumWorkersOfJob() { return PostOffice::Get()->num_workers(); }
};

}  // namespace ps
