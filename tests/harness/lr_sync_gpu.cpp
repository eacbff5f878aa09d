// lr_sync_gpu.cpp — the LR server flow (tests/src/LRServer.h, LRWorker.h of the
// reference) with the model and the BSP merge in HBM (ps::KVServerLRHandle).
//
// Workers run E epochs of B batches: Pull the weights, Push a gradient, the
// last batch of an epoch with cmd = 1 (LRWorker.h:188-210).  The gradients
// are dyadic (multiples of 1/64), so their sum is exact in any arrival order
// and the final model can be compared bit for bit with a replay of the
// reference's update (LRServer.h:171-177, Adam.h:28-34) done here on the CPU.
// With key_cache = 1 the server caches key lists and the workers send the
// list's hash after their first request (USE_KEY_CACHING: LRServer.h:127-142,
// LRWorker.h:214-219).
// usage: lr_sync_gpu [-ns 1] [-nw W] sync(0|1) adam(0|1) epochs batches features [key_cache]
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ps/lr_handle.h"
#include "ps/ps.h"

using namespace ps;

static float grad_of(int rank, int epoch, int batch, int i) {
  return (float)(((i * 7 + rank * 3 + epoch * 5 + batch) % 11) - 5) / 64.0f;
}

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  const int sync_mode = argc > 4 ? std::atoi(argv[4]) : 0;
  const bool use_adam = argc > 5 ? std::atoi(argv[5]) != 0 : false;
  const int epochs = argc > 6 ? std::atoi(argv[6]) : 3;
  const int batches = argc > 7 ? std::atoi(argv[7]) : 4;
  const int n = argc > 8 ? std::atoi(argv[8]) : 123;
  const bool key_cache = argc > 9 ? std::atoi(argv[9]) != 0 : false;
  const float lr = 0.01f;
  std::vector<float> w0(n);
  for (int i = 0; i < n; ++i) w0[i] = (float)((i % 13) - 6) / 16.0f;

  if (IsServer()) {
    auto server = new KVServer<float>(0);
    server->SetDeviceRequestHandle(KVServerLRHandle(w0, lr, sync_mode == 0, use_adam, 0, key_cache));
    RegisterExitCallback([server]() { delete server; });
  }
  if (IsWorker()) {
    KVWorker<float> kv(0, 0);
    const int rank = MyRank(), nw = NumWorkers();
    std::vector<Key> keys(n);
    for (int i = 0; i < n; ++i) keys[i] = i;
    std::vector<float> w, g(n);
    for (int e = 0; e < epochs; ++e) {
      for (int b = 0; b < batches; ++b) {
        kv.Wait(kv.Pull(keys, &w));
        if (key_cache && keys.size() > 1) {  // LRWorker::CacheKey (LRWorker.h:214-219)
          const Key h = detail::KeyListHash(keys.data(), keys.size());
          keys = std::vector<Key>{h};
        }
        CHECK_EQ(w.size(), (size_t)n);
        for (int i = 0; i < n; ++i) g[i] = grad_of(rank, e, b, i);
        kv.Wait(kv.Push(keys, g, {}, b == batches - 1 ? 1 : 0));
      }
    }
    Barrier(0, kWorkerGroup);
    kv.Wait(kv.Pull(keys, &w));
    if (rank == 0) {
      // Replay of LRServer::RequestHandle, round by round.  In sync mode the
      // server advances the iteration when worker 0's cmd = 1 push is handled
      // (LRServer.h:193-195): before that round's apply unless worker 0's push
      // was the round's last to arrive.  So the last round of epoch e applied
      // Adam with iteration e or e + 1, by arrival order; the model must equal
      // the replay of one of those 2^epochs patterns bit for bit.
      const double alr = lr;  // Adam(num_feature, learning_rate_) widens the float
      const double b1 = 0.9, b2 = 0.999, eps = 1e-8;
      const int rounds_per_worker = epochs * batches;
      const int workers_per_apply = sync_mode == 0 ? nw : 1;
      const int patterns = (sync_mode == 0 && use_adam && nw > 1) ? 1 << epochs : 1;
      int matched = -1;
      int first_bad = -1;
      for (int pat = 0; pat < patterns && matched < 0; ++pat) {
        std::vector<float> ref = w0;
        std::vector<double> m(n, 0.0), v(n, 0.0);
        int iteration = 0;
        for (int r = 0; r < rounds_per_worker; ++r) {
          const int e = r / batches, b = r % batches;
          const int it = iteration + ((b == batches - 1 && ((pat >> e) & 1)) ? 1 : 0);
          for (int wk = 0; wk < nw; wk += workers_per_apply) {
            std::vector<float> merged(n, 0.0f);
            for (int k = wk; k < wk + workers_per_apply; ++k)
              for (int i = 0; i < n; ++i) merged[i] += grad_of(k, e, b, i);
            for (int i = 0; i < n; ++i) {
              double grad = lr * merged[i];
              if (use_adam) {
                m[i] = b1 * m[i] + (1 - b1) * grad;
                v[i] = b2 * v[i] + (1 - b2) * grad * grad;
                double m_hat = m[i] / (1 - std::pow(b1, it + 1));
                double v_hat = v[i] / (1 - std::pow(b2, it + 1));
                grad = alr * m_hat / (std::sqrt(v_hat) + eps);
              }
              ref[i] -= grad;
            }
          }
          if (b == batches - 1) ++iteration;
        }
        int bad = -1;
        for (int i = 0; i < n && bad < 0; ++i)
          if (w[i] != ref[i]) bad = i;
        if (bad < 0) matched = pat;
        else if (first_bad < 0) first_bad = bad;
      }
      CHECK_GE(matched, 0) << "no arrival pattern's replay matches; first differing feature " << first_bad;
      std::printf("lr model matches the reference update: n=%d workers=%d sync=%d adam=%d pattern=%d\n", n,
                  nw, sync_mode, (int)use_adam, matched);
    }
  }
  Finalize(0, true);
  return 0;
}
