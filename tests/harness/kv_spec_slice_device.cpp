// kv_spec_slice_device.cpp — unconfirmed slices (PS_SPEC_SLICE=1,
// KVWorker::Send / Refused) when the caller rewrites its HBM key list in place
// between requests, so that the bounds the slicer found last time are wrong:
// the servers refuse the slices that hold keys outside their ranges and the
// worker re-sends those keys sliced for real.  One worker, ns servers; the
// sequence (each request waited for):
//   K0 = kMaxKey / n * i:            Push(seed 7), Pull, Push(seed 8), Pull -> .p0
//   K1 = 1 + kMaxKey / 2 / n * i     (every key in server 0's half):
//                                    Push(seed 9), Pull -> .p1, Push(seed 10), Pull -> .p1b
//   K2 = kMaxKey / 2 + 5 + kMaxKey / 2 / n * i   (every key in the upper half):
//                                    Pull -> .p2, Push(seed 11), Pull -> .p2b
// Each Pull's values go to $PS_SPEC_OUT.<tag> (raw f32); the worker prints
// {"refused": ...} — how many slices its servers refused.  With one worker
// every key's additions come in program order, so the test replays the
// sequence through the oracle and compares every Pull bit for bit.
// usage: kv_spec_slice_device [-ns S] [-nw 1] [num_keys]
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "internal/device.h"
#include "ps/ps.h"

using namespace ps;

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  if (IsServer()) {
    auto server = new KVServer<float>(0);
    KVServerDefaultHandle<float> h;
    server->SetRequestHandle(h);
    RegisterExitCallback([server]() { delete server; });
  }
  if (IsWorker()) {
    CHECK_EQ(NumWorkers(), 1) << "one worker: its additions come in program order";
    const long num = argc > 4 ? std::atol(argv[4]) : 200000;
    const int dev = PostOffice::Get()->device();
    KVWorker<float> kv(0, 0);
    psg_stream s = device::ThreadStream();
    auto dkeys = SVector<Key>::OnDevice(num, dev);
    auto dvals = SVector<float>::OnDevice(num, dev);
    auto dout = SVector<float>::OnDevice(num, dev);
    const char* out_path = std::getenv("PS_SPEC_OUT");
    auto keys = [&](uint64_t first, uint64_t stride) {
      device::Check(psg_fill_keys_arith(dkeys.data(), num, first, stride, s), "fill keys");
      device::Check(psg_stream_sync(s), "sync");
    };
    auto push = [&](int seed) {
      device::Check(psg_fill_synth(dvals.data(), num, PSG_F32, seed, 1, -1.0, 1.0, s), "fill vals");
      device::Check(psg_stream_sync(s), "sync");
      kv.Wait(kv.ZPush(dkeys, dvals));
    };
    auto pull = [&](const char* tag) {
      kv.Wait(kv.ZPull(dkeys, &dout));
      if (!out_path) return;
      std::vector<float> got(num);
      device::CopySync(got.data(), dout.data(), num * sizeof(float), 1);
      const std::string path = std::string(out_path) + "." + tag;
      FILE* f = std::fopen(path.c_str(), "wb");
      CHECK(f) << "cannot write " << path;
      CHECK_EQ(std::fwrite(got.data(), sizeof(float), got.size(), f), got.size());
      std::fclose(f);
    };
    const uint64_t half = kMaxKey / 2;
    keys(0, kMaxKey / num);
    push(7);
    pull("p0a");
    push(8);
    pull("p0");
    keys(1, half / num);
    push(9);
    pull("p1");
    push(10);
    pull("p1b");
    keys(half + 5, half / num);
    pull("p2");
    push(11);
    pull("p2b");
    std::printf("{\"rank\": %d, \"n\": %ld, \"servers\": %d, \"refused\": %llu}\n", MyRank(), num, NumServers(),
                (unsigned long long)kv.refused_slices());
    std::fflush(stdout);
  }
  Finalize(0, true);
  return 0;
}
