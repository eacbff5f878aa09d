// kv_cluster_device.cpp — the KV API end to end on the GPU data path.
//
// Workers hold keys and values either in HBM (ZPush / ZPull on device
// SVectors: device slicer, frames read in place by the server kernels, pull
// replies merged by psg_merge) or in host std::vectors (Push / Pull: the
// worker stages them into HBM once the servers have said their handle takes
// HBM frames — the untimed first requests go as host frames — and copies the
// merged reply back).  The servers run
// KVServerDefaultHandle<float> (HBM store).  Checks the test_kv_app.cpp
// expectations (50 pushes -> 50 * vals, 50 push-pulls -> 100 * vals) and
// prints one JSON line of timings per worker:
//   {"rank":r,"n":N,"device_push_ms":..,"device_pull_ms":..,"device_pushpull_ms":..,
//    "host_push_ms":..,"host_pull_ms":..}
// With key_cache = 1 the server runs KVServerDefaultHandle<float>(true) and the
// timed requests carry ONE key, the hash of the list the untimed first
// request sent (the LR key-cache protocol, LRServer.h:127-142 / LRWorker.h:
// 214-219); one server only, as LR_ps.
// usage: kv_cluster_device [-ns S] [-nw W] [num_keys] [repeat] [key_cache]
#include <chrono>
#include <cstdio>
#include <vector>

#include "internal/device.h"
#include "ps/ps.h"

using namespace ps;
using clk = std::chrono::steady_clock;

static double ms_since(clk::time_point t0) {
  return std::chrono::duration<double, std::milli>(clk::now() - t0).count();
}

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  const bool key_cache = argc > 6 && std::atoi(argv[6]) != 0;
  if (key_cache) CHECK_EQ(NumServers(), 1) << "a hashed key list goes to one server";
  if (IsServer()) {
    auto server = new KVServer<float>(0);
    server->SetRequestHandle(KVServerDefaultHandle<float>(key_cache));
    RegisterExitCallback([server]() { delete server; });
  }
  if (IsWorker()) {
    const long num = argc > 4 ? std::atol(argv[4]) : 1000000;
    const int repeat = argc > 5 ? std::atoi(argv[5]) : 50;
    const int rank = MyRank();
    const int dev = PostOffice::Get()->device();
    KVWorker<float> kv(0, 0);
    psg_stream s = device::ThreadStream();

    // ---- HBM-resident keys / values (the device-resident data path)
    auto dkeys = SVector<Key>::OnDevice(num, dev);
    auto dvals = SVector<float>::OnDevice(num, dev);
    device::Check(psg_fill_keys_arith(dkeys.data(), num, rank, kMaxKey / num, s), "fill keys");
    device::Check(psg_fill_synth(dvals.data(), num, PSG_F32, 7 + rank, 0, 0.0, 1000.0, s), "fill vals");
    device::Check(psg_stream_sync(s), "sync");
    std::vector<float> hvals(num);
    device::CopySync(hvals.data(), dvals.data(), num * sizeof(float), 1);

    // one untimed Push (inserts the keys into the SORTED store) and Pull (warms
    // the HBM pools), then `repeat` timed requests of each
    auto dout = SVector<float>::OnDevice(num, dev);
    kv.Wait(kv.ZPush(dkeys, dvals));
    kv.Wait(kv.ZPull(dkeys, &dout));
    if (key_cache) {  // from now on the list is named by its hash
      uint64_t h = 0;
      device::Check(psg_key_list_hash(dkeys.data(), num, &h, s), "psg_key_list_hash");
      auto hk = SVector<Key>::OnDevice(1, dev);
      device::CopySync(hk.data(), &h, sizeof(h), 0);
      dkeys = hk;
    }
    auto t0 = clk::now();
    for (int r = 0; r < repeat; ++r) kv.Wait(kv.ZPush(dkeys, dvals));
    double dpush = ms_since(t0) / repeat;
    t0 = clk::now();
    for (int r = 0; r < repeat; ++r) kv.Wait(kv.ZPull(dkeys, &dout));
    double dpull = ms_since(t0) / repeat;
    std::vector<float> got(num);
    device::CopySync(got.data(), dout.data(), num * sizeof(float), 1);
    for (long i = 0; i < num; ++i) CHECK_EQ(got[i], hvals[i] * (repeat + 1)) << "device path, i=" << i;
    kv.Wait(kv.ZPushPull(dkeys, dvals, &dout));  // untimed, as the Push and Pull above
    t0 = clk::now();
    for (int r = 0; r < repeat; ++r) kv.Wait(kv.ZPushPull(dkeys, dvals, &dout));
    double dpushpull = ms_since(t0) / repeat;
    device::CopySync(got.data(), dout.data(), num * sizeof(float), 1);
    for (long i = 0; i < num; ++i)
      CHECK_EQ(got[i], hvals[i] * (2 * repeat + 2)) << "device push-pull, i=" << i;

    // ---- host std::vector keys / values (the reference's calling convention)
    std::vector<Key> hkeys(num);
    // fresh keys, disjoint from every worker's device-path keys (offset >= NumWorkers())
    for (long i = 0; i < num; ++i) hkeys[i] = kMaxKey / num * i + NumWorkers() + rank;
    std::vector<float> rets;
    kv.Wait(kv.Push(hkeys, hvals));
    kv.Wait(kv.Pull(hkeys, &rets));
    if (key_cache) hkeys = std::vector<Key>{detail::KeyListHash(hkeys.data(), hkeys.size())};
    // warm-up in the timed form (the hashed list names reply frames of a size
    // the pinned host pool has not seen yet)
    for (int w = 0; w < 3; ++w) {
      kv.Wait(kv.Push(hkeys, hvals));
      kv.Wait(kv.Pull(hkeys, &rets));
    }
    t0 = clk::now();
    for (int r = 0; r < repeat; ++r) kv.Wait(kv.Push(hkeys, hvals));
    double hpush = ms_since(t0) / repeat;
    t0 = clk::now();
    for (int r = 0; r < repeat; ++r) kv.Wait(kv.Pull(hkeys, &rets));
    double hpull = ms_since(t0) / repeat;
    for (long i = 0; i < num; ++i) CHECK_EQ(rets[i], hvals[i] * (repeat + 4)) << "host path, i=" << i;
    std::vector<float> outs;
    for (int r = 0; r < repeat; ++r) kv.Wait(kv.PushPull(hkeys, hvals, &outs));
    for (long i = 0; i < num; ++i)
      CHECK_EQ(outs[i], hvals[i] * (2 * repeat + 4)) << "host push-pull, i=" << i;

    std::printf("{\"rank\": %d, \"n\": %ld, \"servers\": %d, \"key_cache\": %d, \"device_push_ms\": %.4f, "
                "\"device_pull_ms\": %.4f, \"device_pushpull_ms\": %.4f, \"host_push_ms\": %.4f, "
                "\"host_pull_ms\": %.4f}\n",
                rank, num, NumServers(), (int)key_cache, dpush, dpull, dpushpull, hpush, hpull);
    std::fflush(stdout);
  }
  Finalize(0, true);
  return 0;
}
