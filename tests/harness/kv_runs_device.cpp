// kv_runs_device.cpp — nw workers pushing ONE key list through the KV API: the
// BSP shape of test_kv_app_multi_workers.cpp (customers on shared keys) and of
// an LR round, where a server finds several workers' Pushes queued one behind
// the other and serves them as a run (KVServer::OnReceive,
// KVServerDefaultHandle::PushRun, psg_store_push_frames).
//
// Every worker holds its own copy of the list (keys kMaxKey / num * i, in HBM)
// and its own real-valued frame (psg_fill_synth seed 7 + rank, [-1, 1)), so
// the order of the additions shows in the low bits: the test replays the
// servers' trace of arrivals (PS_TRACE_REQUESTS) through the oracle and
// compares worker 0's final Pull bit for bit.
//   1. an untimed ZPush (inserts the keys) and ZPull per worker, a barrier;
//   2. `repeat` timed ZPushes per worker, each waited for, a barrier;
//   3. worker 0 ZPulls and writes the values to $PS_RUNS_OUT (raw f32).
// With key_cache = 1 (one server) the timed Pushes name the list by its hash.
// layout 0 gives every worker the reference benchmark's own keys instead,
// kMaxKey / num * i + rank (tests/test_kv_app_benchmark.cpp:47-52): the lists
// interleave in every server's store, and the requests of distinct workers
// queued at a server form strided runs (psg_store_run).  pull_each = 1 makes
// every timed step a ZPush then a ZPull, each waited for — the benchmark's
// step — so runs mix Pushes and Pulls; each worker then also writes its last
// timed Pull to $PS_RUNS_OUT.<rank>.last and prints its timestamp, and every
// worker writes its final Pull to $PS_RUNS_OUT.<rank>.
// Each worker prints {"rank", "n", "push_ms", "last_pull_ts"}; each server
// prints its store's counters at exit ({"server", "runs", "run_frames",
// "strided_runs", "strided_frames", ...}).
// usage: kv_runs_device [-ns S] [-nw W] [num_keys] [repeat] [key_cache] [layout] [pull_each]
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "internal/device.h"
#include "ps/ps.h"

using namespace ps;
using clk = std::chrono::steady_clock;

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  const bool key_cache = argc > 6 && std::atoi(argv[6]) != 0;
  if (key_cache) CHECK_EQ(NumServers(), 1) << "a hashed key list goes to one server";
  if (IsServer()) {
    auto server = new KVServer<float>(0);
    KVServerDefaultHandle<float> h(key_cache);
    server->SetRequestHandle(h);
    const int id = PostOffice::Get()->my_id();
    RegisterExitCallback([server, h, id]() {
      uint64_t c[PSG_NCOUNTERS] = {};
      if (h.store()) device::Check(psg_store_counters(h.store(), c, PSG_NCOUNTERS), "psg_store_counters");
      std::printf("{\"server\": %d, \"fused\": %llu, \"ident\": %llu, \"notident\": %llu, \"ordered\": %llu, "
                  "\"runs\": %llu, \"run_frames\": %llu, \"strided_runs\": %llu, \"strided_frames\": %llu, \"strided_single\": %llu}\n",
                  id, (unsigned long long)c[0], (unsigned long long)c[1], (unsigned long long)c[2],
                  (unsigned long long)c[3], (unsigned long long)c[4], (unsigned long long)c[5],
                  (unsigned long long)c[PSG_CTR_STRIDED_RUNS], (unsigned long long)c[PSG_CTR_STRIDED_FRAMES],
                  (unsigned long long)c[PSG_CTR_STRIDED_SINGLE]);
      std::fflush(stdout);
      delete server;
    });
  }
  if (IsWorker()) {
    const long num = argc > 4 ? std::atol(argv[4]) : 1000000;
    const int repeat = argc > 5 ? std::atoi(argv[5]) : 20;
    const int layout = argc > 7 ? std::atoi(argv[7]) : 1;
    const bool pull_each = argc > 8 && std::atoi(argv[8]) != 0;
    const int rank = MyRank();
    const int dev = PostOffice::Get()->device();
    KVWorker<float> kv(0, 0);
    psg_stream s = device::ThreadStream();
    auto dkeys = SVector<Key>::OnDevice(num, dev);
    auto dvals = SVector<float>::OnDevice(num, dev);
    device::Check(psg_fill_keys_arith(dkeys.data(), num, layout == 0 ? (uint64_t)rank : 0, kMaxKey / num, s),
                  "fill keys");
    device::Check(psg_fill_synth(dvals.data(), num, PSG_F32, 7 + rank, 1, -1.0, 1.0, s), "fill vals");
    device::Check(psg_stream_sync(s), "sync");
    auto dout = SVector<float>::OnDevice(num, dev);
    kv.Wait(kv.ZPush(dkeys, dvals));
    kv.Wait(kv.ZPull(dkeys, &dout));
    SVector<Key> pkeys = dkeys;
    if (key_cache) {
      uint64_t hsh = 0;
      device::Check(psg_key_list_hash(dkeys.data(), num, &hsh, s), "psg_key_list_hash");
      pkeys = SVector<Key>::OnDevice(1, dev);
      device::CopySync(pkeys.data(), &hsh, sizeof(hsh), 0);
    }
    Barrier(0, kWorkerGroup);
    const char* out_path = std::getenv("PS_RUNS_OUT");
    auto dump = [&](const std::string& path) {
      std::vector<float> got(num);
      device::CopySync(got.data(), dout.data(), num * sizeof(float), 1);
      FILE* f = std::fopen(path.c_str(), "wb");
      CHECK(f) << "cannot write " << path;
      CHECK_EQ(std::fwrite(got.data(), sizeof(float), got.size(), f), got.size());
      std::fclose(f);
    };
    int last_pull_ts = -1;
    const auto t0 = clk::now();
    for (int r = 0; r < repeat; ++r) {
      kv.Wait(kv.ZPush(pkeys, dvals));
      if (pull_each) {
        last_pull_ts = kv.ZPull(dkeys, &dout);
        kv.Wait(last_pull_ts);
      }
    }
    const double push_ms = std::chrono::duration<double, std::milli>(clk::now() - t0).count() / repeat;
    if (pull_each && out_path) dump(std::string(out_path) + "." + std::to_string(rank) + ".last");
    Barrier(0, kWorkerGroup);
    if (rank == 0 || layout == 0) {
      kv.Wait(kv.ZPull(dkeys, &dout));
      if (out_path) dump(layout == 0 ? std::string(out_path) + "." + std::to_string(rank) : std::string(out_path));
    }
    std::printf("{\"rank\": %d, \"n\": %ld, \"workers\": %d, \"servers\": %d, \"key_cache\": %d, \"layout\": %d, "
                "\"push_ms\": %.4f, \"node\": %d, \"last_pull_ts\": %d}\n",
                rank, num, NumWorkers(), NumServers(), (int)key_cache, layout, push_ms, PostOffice::Get()->my_id(),
                last_pull_ts);
    std::fflush(stdout);
  }
  Finalize(0, true);
  return 0;
}
