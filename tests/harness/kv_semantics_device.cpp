// kv_semantics_device.cpp — reference semantics of the KV API that the fast
// paths must not bend, end to end through KVWorker / KVServer on the GPU data
// path (ns = 1, nw = 1; run by tests/test_dropin_gpu.py):
//
//  1. keys in any order, keys repeated (ZPush / ZPushPull / ZPull on HBM
//     SVectors; Push on host vectors, and PushPull / Pull on ascending host
//     vectors with repeats — the reference's pull merge, KVApp.h:683-686,
//     CHECK-fails on unsorted host keys): KVServerDefaultHandle's loop
//     (src/ps/KVApp.h:446-454) adds each occurrence in turn and answers each
//     with the running value — replayed here on a std::unordered_map, exactly;
//  2. the key cache of KVServerDefaultHandle<float>(true) keeps its own copy of
//     a list (LRServer.h:139 keeps the received copy): the worker rewrites its
//     key buffer in place after the first request, the store then inserts new
//     keys (so the cached list is re-resolved), and a hashed request must still
//     name the ORIGINAL keys;
//  3. a ZPull through a custom slicer that copies the values instead of slicing
//     them (KVWorker::set_slicer, KVApp.h:292-294) gets no direct-reply offer:
//     the reply is merged into the caller's output, which must hold the values.
// Exits non-zero on the first failed CHECK.
#include <algorithm>
#include <cstdio>
#include <random>
#include <unordered_map>
#include <vector>

#include "internal/device.h"
#include "ps/ps.h"

using namespace ps;

static std::vector<float> Replay(std::unordered_map<Key, float>& store, const std::vector<Key>& keys,
                                 const std::vector<float>& vals, bool push, bool pull) {
  std::vector<float> out(pull ? keys.size() : 0);
  for (size_t i = 0; i < keys.size(); ++i) {
    if (push) store[keys[i]] += vals[i];
    if (pull) out[i] = store[keys[i]];
  }
  return out;
}

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  CHECK_EQ(NumServers(), 1) << "ns = 1: the reference slices unsorted keys only for one server";
  if (IsServer()) {
    auto plain = new KVServer<float>(0);
    plain->SetRequestHandle(KVServerDefaultHandle<float>(false));
    auto cached = new KVServer<float>(1);
    cached->SetRequestHandle(KVServerDefaultHandle<float>(true));
    RegisterExitCallback([plain, cached]() {
      delete plain;
      delete cached;
    });
  }
  if (IsWorker()) {
    const int dev = PostOffice::Get()->device();
    psg_stream s = device::ThreadStream();
    std::mt19937_64 rng(17);
    auto to_dev = [&](const auto& v) {
      using T = typename std::decay_t<decltype(v)>::value_type;
      auto d = SVector<T>::OnDevice(v.size(), dev);
      device::CopySync(d.data(), v.data(), v.size() * sizeof(T), 0);
      return d;
    };
    auto to_host = [&](const SVector<float>& d) {
      std::vector<float> h(d.size());
      device::CopySync(h.data(), d.data(), d.size() * sizeof(float), 1);
      return h;
    };

    // ---- 1. out-of-order and repeated keys -----------------------------------
    {
      KVWorker<float> kv(0, 0);
      std::unordered_map<Key, float> ref;
      const size_t n = 300000;
      std::vector<Key> pool(40000);
      for (auto& k : pool) k = rng() >> 1;
      for (int round = 0; round < 4; ++round) {
        std::vector<Key> keys(n);
        for (auto& k : keys) k = pool[rng() % pool.size()];
        if (round & 1)
          for (size_t i = 0; i < n / 4; ++i) keys[i * 4] = pool[7];  // a hot key
        std::vector<float> vals(n);
        for (auto& v : vals) v = (float)(int)(rng() % 2001) / 8.0f - 125.0f;
        if (round < 2) {  // HBM frames
          auto dk = to_dev(keys);
          auto dv = to_dev(vals);
          kv.Wait(kv.ZPush(dk, dv));
          Replay(ref, keys, vals, true, false);
          auto dout = SVector<float>::OnDevice(n, dev);
          kv.Wait(kv.ZPushPull(dk, dv, &dout));
          auto exp = Replay(ref, keys, vals, true, true);
          auto got = to_host(dout);
          for (size_t i = 0; i < n; ++i) CHECK_EQ(got[i], exp[i]) << "HBM PushPull, round " << round << ", i=" << i;
          auto dout2 = SVector<float>::OnDevice(n, dev);
          kv.Wait(kv.ZPull(dk, &dout2));
          exp = Replay(ref, keys, vals, false, true);
          got = to_host(dout2);
          for (size_t i = 0; i < n; ++i) CHECK_EQ(got[i], exp[i]) << "HBM Pull, round " << round << ", i=" << i;
        } else {  // host vectors (staged into HBM once the server said it takes HBM frames)
          kv.Wait(kv.Push(keys, vals));
          Replay(ref, keys, vals, true, false);
          // a Pull's reply is matched to the request by FindRange over the
          // worker's host keys (KVApp.h:683-686), which needs them ascending:
          // the reference CHECK-fails on an unsorted host Pull, so these are
          // sorted — repeats kept
          std::sort(keys.begin(), keys.end());
          std::vector<float> outs;
          kv.Wait(kv.PushPull(keys, vals, &outs));
          auto exp = Replay(ref, keys, vals, true, true);
          for (size_t i = 0; i < n; ++i) CHECK_EQ(outs[i], exp[i]) << "host PushPull, round " << round << ", i=" << i;
          std::vector<float> pulled;
          kv.Wait(kv.Pull(keys, &pulled));
          exp = Replay(ref, keys, vals, false, true);
          for (size_t i = 0; i < n; ++i) CHECK_EQ(pulled[i], exp[i]) << "host Pull, round " << round << ", i=" << i;
        }
      }
      std::printf("out-of-order ok\n");
    }

    // ---- 2. the key cache keeps its own copy of a list -------------------------
    {
      KVWorker<float> kv(1, 0);
      const size_t n = 50000;
      std::vector<Key> a(n), b(n);
      for (size_t i = 0; i < n; ++i) {
        a[i] = (Key)i * 1000 + 1;
        b[i] = (Key)i * 1000 + 2;  // disjoint from a
      }
      std::vector<float> va(n, 1.5f), vb(n, 4.0f);
      auto buf = to_dev(a);  // the worker's key buffer
      auto dva = to_dev(va);
      kv.Wait(kv.ZPush(buf, dva));  // full list: cached under hash(a)
      uint64_t ha = detail::KeyListHash(a.data(), n);
      // the worker rewrites its buffer in place with list b and pushes it: a
      // full request again, whose absent keys the store inserts (every cached
      // list is then re-resolved from the cache's copy)
      device::CopySync(buf.data(), b.data(), n * sizeof(Key), 0);
      auto dvb = to_dev(vb);
      kv.Wait(kv.ZPush(buf, dvb));
      auto hk = to_dev(std::vector<Key>{ha});
      auto dout = SVector<float>::OnDevice(n, dev);
      kv.Wait(kv.ZPull(hk, &dout));
      auto got = to_host(dout);
      for (size_t i = 0; i < n; ++i) CHECK_EQ(got[i], 1.5f) << "hashed list a after the rewrite, i=" << i;
      kv.Wait(kv.ZPush(hk, dva));  // by hash, on the re-resolved slots
      kv.Wait(kv.ZPull(hk, &dout));
      got = to_host(dout);
      for (size_t i = 0; i < n; ++i) CHECK_EQ(got[i], 3.0f) << "hashed Push of list a, i=" << i;
      std::printf("key cache ok\n");
    }

    // ---- 3. a copying slicer gets no direct reply ------------------------------
    {
      KVWorker<float> kv(0, 1);
      const size_t n = 20000;
      std::vector<Key> keys(n);
      for (size_t i = 0; i < n; ++i) keys[i] = (Key)(i + 1) * 7919;
      std::vector<float> vals(n, 2.0f);
      auto dk = to_dev(keys);
      kv.Wait(kv.ZPush(dk, to_dev(vals)));
      kv.set_slicer([dev](KVPairs<float>& send, const std::vector<Range>&,
                          std::vector<std::pair<bool, KVPairs<float>>>* sliced) {
        sliced->assign(1, {true, KVPairs<float>()});
        auto& d = (*sliced)[0].second;
        d.keys = send.keys;
        if (send.vals.size()) {  // a copy of the values, not a slice of them
          d.vals = SVector<float>::OnDevice(send.vals.size(), dev);
          device::CopySync(d.vals.data(), send.vals.data(), send.vals.size() * sizeof(float), 2);
        }
        d.lens = send.lens;
      });
      auto dout = SVector<float>::OnDevice(n, dev);
      device::Check(psg_memset(dout.data(), 0, n * sizeof(float), s), "psg_memset");
      device::Check(psg_stream_sync(s), "psg_stream_sync");
      kv.Wait(kv.ZPull(dk, &dout));
      auto got = to_host(dout);
      // ZPull seeds its output with the request's own values only where the
      // reference would merge the reply: every value must be the store's
      std::unordered_map<Key, float> ref;
      auto exp = Replay(ref, keys, vals, true, true);
      for (size_t i = 0; i < n; ++i) CHECK_EQ(got[i], exp[i]) << "copying slicer, i=" << i;
      std::printf("custom slicer ok\n");
    }
  }
  Finalize(0, true);
  return 0;
}
