// lr_ref_pin.cpp — the LR server of the reference (tests/src/LRServer.h with
// Adam.h, compiled from the reference tree as it lies, unmodified) and this
// runtime's HBM LR handle (ps::KVServerLRHandle) driven by the same worker
// requests, so the model each one ends with can be compared bit for bit.
//
//   PIN_MODE=ref  the server node runs lr::LRServer: its RequestHandle
//                 (LRServer.h:122-207) merges and applies on the CPU;
//   PIN_MODE=gpu  the server node runs KVServerLRHandle on HBM, started from
//                 the weights the reference's own InitWeight draws
//                 (LRServer.h:36-63, seed 0).
//
// Workers: E epochs of B batches, Pull then Push of a gradient, the last batch
// of an epoch with cmd = 1 (LRWorker.h:188-210).  PIN_GRAD=real draws
// real-valued gradients (only with one worker or async: the merge order is then
// fixed), PIN_GRAD=dyadic multiples of 1/64 (exact in any merge order).  At the
// end worker 0 Pulls the model and prints it as one line of hex words:
//   MODEL <rank> <n> <bits of w[0]> <bits of w[1]> ...     (every worker)
// and, with PIN_MODE=gpu, the server's own model (KVServerLRHandle::GetWeight)
// when the job ends, so a wrong final model can be told apart from a wrong reply:
//   SERVER_MODEL <n> <bits of w[0]> ...
// The reference server reads its settings from the environment as LR_ps does:
// NUM_FEATURE, LEARNING_RATE, SYNC_MODE, USE_ADAM, ITERATION, DATA_DIR.
// usage: PIN_MODE=ref|gpu PIN_EPOCHS=E PIN_BATCHES=B lr_ref_pin -ns 1 -nw W
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "LRServer.h"
#include "ps/lr_handle.h"
#include "ps/ps.h"

using namespace ps;

static float grad_of(bool real, int rank, int epoch, int batch, int i) {
  if (real) return (float)std::sin(0.37 * i + 1.3 * epoch + 0.71 * batch + 2.9 * rank) * 0.8f;
  return (float)(((i * 7 + rank * 3 + epoch * 5 + batch) % 11) - 5) / 64.0f;
}

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  const char* mode_env = std::getenv("PIN_MODE");
  const char* grad_env = std::getenv("PIN_GRAD");
  const std::string mode = mode_env ? mode_env : "ref";
  const bool real = grad_env && std::strcmp(grad_env, "real") == 0;
  const int epochs = Environment::GetIntOrDefault("PIN_EPOCHS", 3);
  const int batches = Environment::GetIntOrDefault("PIN_BATCHES", 4);
  const int n = Environment::GetIntOrFail("NUM_FEATURE");

  if (IsServer()) {
    if (mode == "ref") {
      auto server = new lr::LRServer(0);
      RegisterExitCallback([server]() { delete server; });
    } else {
      // the reference's InitWeight for the starting model (srand(0), rand())
      std::vector<lr::FType> w0(n);
      int total = 0, current = 0;
      lr::InitWeight(w0, 0, total, current);
      const float lr_rate = std::stof(std::string(Environment::GetOrFail("LEARNING_RATE")));
      auto server = new KVServer<float>(0);
      KVServerLRHandle handle(w0, lr_rate, Environment::GetInt("SYNC_MODE") == 0,
                              Environment::Get("USE_ADAM") != nullptr, current, false);
      server->SetDeviceRequestHandle(handle);
      RegisterExitCallback([server, handle]() {
        const std::vector<float> w = handle.GetWeight();
        std::string line = "SERVER_MODEL " + std::to_string(w.size());
        char buf[16];
        for (float x : w) {
          uint32_t bits;
          std::memcpy(&bits, &x, 4);
          std::snprintf(buf, sizeof(buf), " %08x", bits);
          line += buf;
        }
        std::printf("%s\n", line.c_str());
        std::fflush(stdout);
        delete server;
      });
    }
  }
  // Workers start once the server is fully built.  The reference's LRServer
  // installs its request handle BEFORE it sizes and initialises weight_
  // (LRServer.h:68-86: SetRequestHandle, then weight_.resize and InitWeight),
  // and LR_ps.cpp starts its workers right after ps::Start (LR_ps.cpp:120-124):
  // with 200,000 features a first BSP round could be applied while InitWeight
  // was still writing the tail of weight_, which then overwrote the round
  // there (the GPUTEST_r03 failure).  The barrier closes that
  // window for both servers of this harness.
  Barrier(0, kAllNodes);
  if (IsWorker()) {
    KVWorker<float> kv(0, 0);
    const int rank = MyRank();
    std::vector<Key> keys(n);
    for (int i = 0; i < n; ++i) keys[i] = i;
    std::vector<float> w, g(n);
    // PIN_TRACE=K: worker 0 also prints the last K features of every Pull reply
    // (the model after each BSP round), so a test can find the round at which a
    // wrong model first appears:  PULL <epoch> <batch> <first feature> <bits> ...
    const int trace = Environment::GetIntOrDefault("PIN_TRACE", 0);
    for (int e = 0; e < epochs; ++e) {
      for (int b = 0; b < batches; ++b) {
        kv.Wait(kv.Pull(keys, &w));
        CHECK_EQ(w.size(), (size_t)n);
        if (trace > 0 && rank == 0) {
          const int first = n > trace ? n - trace : 0;
          std::string line = "PULL " + std::to_string(e) + " " + std::to_string(b) + " " + std::to_string(first);
          char buf[16];
          for (int i = first; i < n; ++i) {
            uint32_t bits;
            std::memcpy(&bits, &w[i], 4);
            std::snprintf(buf, sizeof(buf), " %08x", bits);
            line += buf;
          }
          std::printf("%s\n", line.c_str());
          std::fflush(stdout);
        }
        for (int i = 0; i < n; ++i) g[i] = grad_of(real, rank, e, b, i);
        kv.Wait(kv.Push(keys, g, {}, b == batches - 1 ? 1 : 0));
      }
    }
    Barrier(0, kWorkerGroup);
    kv.Wait(kv.Pull(keys, &w));
    {
      std::string line = "MODEL " + std::to_string(rank) + " " + std::to_string(n);
      char buf[16];
      for (int i = 0; i < n; ++i) {
        uint32_t bits;
        std::memcpy(&bits, &w[i], 4);
        std::snprintf(buf, sizeof(buf), " %08x", bits);
        line += buf;
      }
      std::printf("%s\n", line.c_str());
      std::fflush(stdout);
    }
  }
  Finalize(0, true);
  return 0;
}
