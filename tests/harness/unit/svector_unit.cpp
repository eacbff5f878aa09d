// svector_unit.cpp — SVector semantics the KV path relies on, following the
// reference's own unit tests (src/utility/test/SVector_test.cpp): copy from a
// std::vector, sharing copies, non-owning wraps, Slice aliasing and
// detach-on-growth (SliceTest, :411-462), resize/fill, reinterpreting views,
// FindRange.  Plain program (no PS node): exits non-zero on a failed CHECK.
#include <atomic>
#include <cstdio>
#include <cstdint>
#include <memory>
#include <thread>
#include <vector>

#include "ps/svector.h"

using ps::SVector;

int main() {
  {  // construction from std::vector copies; copies of SVector share
    std::vector<int> v{1, 2, 3};
    SVector<int> s(v);
    v[0] = 100;
    CHECK_EQ(s[0], 1);
    SVector<int> t = s;
    t[1] = 20;
    CHECK_EQ(s[1], 20);
    CHECK_EQ(s.data(), t.data());
  }
  {  // shared_ptr<vector>: shares the vector's storage
    auto sp = std::make_shared<std::vector<float>>(std::vector<float>{1.f, 2.f});
    SVector<float> s(sp);
    (*sp)[1] = 5.f;
    CHECK_EQ(s[1], 5.f);
  }
  {  // raw pointer, non-owning
    int raw[4] = {4, 3, 2, 1};
    SVector<int> s(raw, 4);
    raw[2] = 9;
    CHECK_EQ(s[2], 9);
    CHECK_EQ(s.size(), 4u);
  }
  {  // Slice aliases; growing the slice detaches it (SliceTest)
    SVector<int> s1{1, 2, 3, 4, 5};
    auto s2 = s1.Slice(2, 4);  // 3, 4
    CHECK_EQ(s2[0], 3);
    CHECK_EQ(s2[1], 4);
    s1[2] = -3;
    CHECK_EQ(s2[0], -3);
    s2[1] = -4;
    CHECK_EQ(s1[3], -4);
    s2.push_back(999);  // capacity of a slice == its size: reallocates
    CHECK_EQ(s2.size(), 3u);
    CHECK_EQ(s2[1], -4);
    CHECK_EQ(s2[2], 999);
    s2[0] = 7;
    CHECK_EQ(s1[2], -3);  // detached
    CHECK_EQ(s1[4], 5);
  }
  {  // growing the parent detaches it from its slices
    SVector<int> s1{1, 2, 3, 4};
    SVector<int> s2 = s1.Slice(1, s1.size());
    s2[1] = 30;
    CHECK_EQ(s1[2], 30);
    s1.push_back(5);
    CHECK_EQ(s1.size(), 5u);
    CHECK_EQ(s2.size(), 3u);
    s1[2] = 99;
    CHECK_EQ(s2[1], 30);
  }
  {  // resize fills new elements; shrink keeps the prefix
    SVector<float> s;
    s.resize(3, 1.5f);
    CHECK_EQ(s.size(), 3u);
    CHECK_EQ(s[2], 1.5f);
    s.resize(5);
    CHECK_EQ(s[4], 0.f);
    s.resize(2);
    CHECK_EQ(s.size(), 2u);
    CHECK_EQ(s[1], 1.5f);
  }
  {  // reinterpreting views share the bytes (Message::AddData frames)
    SVector<float> f{1.f, 2.f, 3.f};
    SVector<char> c(f);
    CHECK_EQ(c.size(), 12u);
    SVector<float> back(c);
    CHECK_EQ(back.size(), 3u);
    CHECK_EQ(back[2], 3.f);
    CHECK_EQ((void*)back.data(), (void*)f.data());
    bool threw = false;
    try {
      SVector<char> odd(5);
      SVector<float> bad(odd);  // 5 bytes are not whole floats
    } catch (const ps_log::PSError&) {
      threw = true;
    }
    CHECK(threw);
  }
  {  // FindRange (SVector.h:670-676)
    SVector<uint64_t> k{2, 4, 6, 8};
    ps::Range r = ps::FindRange<uint64_t>(k, 4, 8);
    CHECK_EQ(r.begin, 1u);
    CHECK_EQ(r.end, 3u);
  }
  {  // large copies go through the pooled multi-threaded HostCopy: contents
     // exact, from several threads at once, sizes not multiples of a part
    auto check_big = [](size_t n, uint32_t seed) {
      std::vector<uint32_t> v(n);
      for (size_t i = 0; i < n; ++i) v[i] = (uint32_t)(i * 2654435761u) ^ seed;
      SVector<uint32_t> s(v);
      for (size_t i = 0; i < n; ++i) CHECK_EQ(s[i], v[i]) << "at " << i;
    };
    check_big((size_t(24) << 20) / 4 + 12345, 7);
    std::vector<std::thread> ts;
    for (uint32_t t = 0; t < 4; ++t) ts.emplace_back([&, t] { for (int r = 0; r < 3; ++r) check_big((size_t(9) << 20) + 777 * t, t * 100 + r); });
    for (auto& t : ts) t.join();
  }
  {  // HostCopy stress: back-to-back jobs of varying sizes from 8 threads at
     // once (more callers than copy workers), every byte checked.  A worker
     // still leaving job k must never run a part of job k + 1, or a job could
     // return while one of its parts is still being copied.
    std::vector<std::thread> ts;
    std::atomic<int> bad{0};
    for (uint32_t t = 0; t < 8; ++t)
      ts.emplace_back([&, t] {
        for (int r = 0; r < 24; ++r) {
          const size_t n = (size_t(4) << 20) / 4 + (size_t)((t * 7919u + r * 104729u) % (3u << 20));
          std::vector<uint32_t> src(n), dst(n, 0xdeadbeefu);
          for (size_t i = 0; i < n; ++i) src[i] = (uint32_t)(i * 2246822519u) ^ (t << 24) ^ (uint32_t)r;
          ps::HostCopy(dst.data(), src.data(), n * 4);
          if (dst != src) bad.fetch_add(1);
        }
      });
    for (auto& t : ts) t.join();
    CHECK_EQ(bad.load(), 0) << "HostCopy returned before its copy was complete";
  }
  std::printf("svector ok\n");
  return 0;
}
