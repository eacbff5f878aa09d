// kv_bench_dropin.cpp — the drop-in API's own bench line (bench.py --workload
// dropin): device-resident ZPush then ZPull through KVWorker / KVServer
// (KVServerDefaultHandle, HBM store) at ns servers and nw workers, timed per
// step the way test_kv_app_benchmark.cpp:57-81 times one Push and one Pull,
// but over `steps` steps after `warmup` untimed ones, every worker between
// two barriers.
//   layout 0  test_kv_app_benchmark's keys: worker r pushes keys kMaxKey/num*i + r
//             (tests/test_kv_app_benchmark.cpp:47-52), so with nw workers each
//             server's store holds nw interleaved lists and every request is
//             a sparse subset of it;
//   layout 1  one shared list kMaxKey/num*i: the BSP shape, where a server
//             finds the workers' Pushes queued and serves them as runs.
// Values are integer-valued synthetic floats (psg_fill_synth mode 0, seed 7 +
// rank), so after P Pushes every pulled value has a closed form; each worker
// checks its whole pulled vector on the device (psg_verify_synth_sum) and
// prints
//   {"rank", "n", "workers", "servers", "layout", "steps", "warmup",
//    "ms_per_step", "push_ms", "pull_ms", "mismatches"}
// and each server, at exit, its store's counters (which paths served the
// requests: {"server", "fused", "ident", "runs", "run_frames", "strided_runs",
// "strided_frames"}).
// usage: kv_bench_dropin [-ns S] [-nw W] [-procs] num_keys steps warmup layout
#include <chrono>
#include <cstdio>
#include <cstdlib>

#include "internal/device.h"
#include "ps/ps.h"

using namespace ps;
using clk = std::chrono::steady_clock;

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  if (IsServer()) {
    auto server = new KVServer<float>(0);
    KVServerDefaultHandle<float> h;
    server->SetRequestHandle(h);
    const int id = PostOffice::Get()->my_id();
    RegisterExitCallback([server, h, id]() {
      // how the store served the job's requests (psg_store_counters)
      uint64_t c[PSG_NCOUNTERS] = {};
      if (h.store()) device::Check(psg_store_counters(h.store(), c, PSG_NCOUNTERS), "psg_store_counters");
      std::printf("{\"server\": %d, \"fused\": %llu, \"ident\": %llu, \"runs\": %llu, \"run_frames\": %llu, "
                  "\"strided_runs\": %llu, \"strided_frames\": %llu, \"strided_single\": %llu}\n",
                  id, (unsigned long long)c[PSG_CTR_FUSED], (unsigned long long)c[PSG_CTR_IDENT],
                  (unsigned long long)c[PSG_CTR_RUNS], (unsigned long long)c[PSG_CTR_RUN_FRAMES],
                  (unsigned long long)c[PSG_CTR_STRIDED_RUNS], (unsigned long long)c[PSG_CTR_STRIDED_FRAMES],
                  (unsigned long long)c[PSG_CTR_STRIDED_SINGLE]);
      std::fflush(stdout);
      delete server;
    });
  }
  if (IsWorker()) {
    const long num = argc > 4 ? std::atol(argv[4]) : 10000000;
    const int steps = argc > 5 ? std::atoi(argv[5]) : 10;
    const int warmup = argc > 6 ? std::atoi(argv[6]) : 3;
    const int layout = argc > 7 ? std::atoi(argv[7]) : 0;
    const int rank = MyRank();
    const int dev = PostOffice::Get()->device();
    KVWorker<float> kv(0, 0);
    psg_stream s = device::ThreadStream();
    auto keys = SVector<Key>::OnDevice(num, dev);
    auto vals = SVector<float>::OnDevice(num, dev);
    auto out = SVector<float>::OnDevice(num, dev);
    device::Check(psg_fill_keys_arith(keys.data(), num, layout == 0 ? (uint64_t)rank : 0, kMaxKey / num, s),
                  "fill keys");
    device::Check(psg_fill_synth(vals.data(), num, PSG_F32, 7 + rank, 0, 0.0, 100.0, s), "fill vals");
    device::Check(psg_stream_sync(s), "sync");
    for (int w = 0; w < warmup; ++w) {
      kv.Wait(kv.ZPush(keys, vals));
      kv.Wait(kv.ZPull(keys, &out));
    }
    Barrier(0, kWorkerGroup);
    double push_ms = 0, pull_ms = 0;
    const auto t0 = clk::now();
    for (int r = 0; r < steps; ++r) {
      const auto a = clk::now();
      kv.Wait(kv.ZPush(keys, vals));
      const auto b = clk::now();
      kv.Wait(kv.ZPull(keys, &out));
      push_ms += std::chrono::duration<double, std::milli>(b - a).count();
      pull_ms += std::chrono::duration<double, std::milli>(clk::now() - b).count();
    }
    const double ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count();
    Barrier(0, kWorkerGroup);
    // every worker's last Pull saw its own Pushes; with one shared list it saw
    // the others' too only after the barrier: pull once more there
    if (layout == 1) kv.Wait(kv.ZPull(keys, &out));
    const int pushes = warmup + steps;
    uint64_t bad = 0, first = 0;
    if (layout == 0)
      device::Check(psg_verify_synth_sum(out.data(), num, PSG_F32, 7 + rank, 1, 0, 0.0, 100.0, (double)pushes, &bad,
                                         &first, s),
                    "verify");
    else
      device::Check(psg_verify_synth_sum(out.data(), num, PSG_F32, 7, NumWorkers(), 0, 0.0, 100.0, (double)pushes,
                                         &bad, &first, s),
                    "verify");
    std::printf("{\"rank\": %d, \"n\": %ld, \"workers\": %d, \"servers\": %d, \"layout\": %d, \"steps\": %d, "
                "\"warmup\": %d, \"ms_per_step\": %.5f, \"push_ms\": %.5f, \"pull_ms\": %.5f, \"mismatches\": %llu}\n",
                rank, num, NumWorkers(), NumServers(), layout, steps, warmup, ms / steps, push_ms / steps,
                pull_ms / steps, (unsigned long long)bad);
    std::fflush(stdout);
  }
  Finalize(0, true);
  return 0;
}
