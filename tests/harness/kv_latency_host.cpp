// kv_latency_host.cpp — the round trip of a small request through the host
// runtime: 1 server whose handle answers at once (test_kv_app_benchmark's
// EmptyHandler), 1 worker timing ITERS synchronous Push + Wait of KEYS keys.
// No GPU.  Thread mode (one process) or -procs (the TCP Van between two
// processes): the difference is the transport's cost per request.
//   LAT_ITERS=20000 LAT_KEYS=1 LAT_MODE=processes kv_latency_host -ns 1 -nw 1 [-procs]
// Prints one JSON line {"mode", "iters", "keys", "us_per_request"} from the
// worker.
#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "ps/ps.h"

using namespace ps;

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  // parameters by environment (in process mode every node is started with
  // the launcher's own argv): LAT_ITERS, LAT_KEYS, LAT_MODE (a label)
  const char* ei = std::getenv("LAT_ITERS");
  const char* ek = std::getenv("LAT_KEYS");
  const char* em = std::getenv("LAT_MODE");
  const long iters = ei ? std::atol(ei) : 20000;
  const long nkeys = ek ? std::atol(ek) : 1;
  // LAT_WORK_US: the handle busy-waits this long first (a request's device
  // time, e.g. ~50 us for a 10 M-key keyed Push), so the waiting threads of the
  // worker outlast their spin as they do behind a real request
  const char* ew = std::getenv("LAT_WORK_US");
  const long work_us = ew ? std::atol(ew) : 0;
  if (IsServer()) {
    auto server = new KVServer<float>(0);
    server->SetRequestHandle([work_us](const KVMeta& meta, const KVPairs<float>& req, KVServer<float>* s) {
      if (work_us > 0) {
        const auto t0 = std::chrono::steady_clock::now();
        while (std::chrono::steady_clock::now() - t0 < std::chrono::microseconds(work_us)) {
        }
      }
      KVPairs<float> res;
      if (meta.pull) {
        res.keys = req.keys;
        res.vals.resize(req.keys.size());
      }
      s->Response(meta, res);
    });
    RegisterExitCallback([server]() { delete server; });
  }
  if (IsWorker()) {
    KVWorker<float> kv(0, 0);
    std::vector<Key> keys(nkeys);
    std::vector<float> vals(nkeys, 1.0f);
    for (long i = 0; i < nkeys; ++i) keys[i] = (Key)(i * 7919 + 1);
    for (int w = 0; w < 1000; ++w) kv.Wait(kv.Push(keys, vals));
    std::vector<double> us;
    for (int rep = 0; rep < 5; ++rep) {
      const auto t0 = std::chrono::steady_clock::now();
      for (long i = 0; i < iters / 5; ++i) kv.Wait(kv.Push(keys, vals));
      const auto t1 = std::chrono::steady_clock::now();
      us.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count() / (double)(iters / 5));
    }
    std::sort(us.begin(), us.end());
    printf("{\"mode\": \"%s\", \"iters\": %ld, \"keys\": %ld, \"work_us\": %ld, \"us_per_request\": %.2f, \"min\": %.2f, \"max\": %.2f}\n",
           em ? em : "?", iters, nkeys, work_us, us[us.size() / 2], us.front(), us.back());
    fflush(stdout);
  }
  Finalize(0, true);
  return 0;
}
