// shm_arena_unit.cpp — the process-mode frame arena (src/shm_pool.cc): frames
// carved from one pre-faulted shared-memory block never overlap while alive,
// freed ranges coalesce (a frame the size of the whole arena fits again once
// everything is freed), a frame the arena cannot hold gets a block of its own,
// every frame is found as (block name, offset), and a mapping of that name
// (what a peer process does) shows the frame's bytes.  Plain program (no PS
// node); PS_SHM_ARENA_MB sets the arena (this test runs it at 16 MiB).
#include <algorithm>
#include <cstdio>
#include <cstring>
#include <memory>
#include <random>
#include <string>
#include <vector>

#include "internal/shm_pool.h"
#include "ps/log.h"

using namespace ps;

namespace {
struct Frame {
  std::shared_ptr<void> p;
  size_t n;
  unsigned char tag;
};

void fill(const Frame& f) { std::memset(f.p.get(), f.tag, f.n); }

bool intact(const Frame& f) {
  const unsigned char* b = static_cast<const unsigned char*>(f.p.get());
  for (size_t i = 0; i < f.n; i += 4093)
    if (b[i] != f.tag) return false;
  return b[f.n - 1] == f.tag;
}
}  // namespace

int main() {
  shm::Enable(true);
  CHECK(shm::Enabled());
  const size_t MiB = size_t(1) << 20;
  std::mt19937 rng(7);
  std::vector<Frame> live;
  std::string arena_name;
  // churn: allocate and free frames of 1-5 MiB in random order, every live
  // frame keeps its bytes (no two live frames overlap)
  for (int round = 0; round < 400; ++round) {
    if (live.size() < 6 && (rng() % 3 != 0 || live.empty())) {
      Frame f;
      f.n = MiB + (rng() % (4 * MiB));
      f.p = shm::Alloc(f.n);
      CHECK(f.p) << "shm::Alloc failed";
      f.tag = (unsigned char)(1 + round % 250);
      fill(f);
      std::string name;
      uint64_t off = 0;
      CHECK(shm::Find(f.p.get(), f.n, &name, &off)) << "a frame must be found in its block";
      live.push_back(std::move(f));
    } else {
      const size_t i = rng() % live.size();
      CHECK(intact(live[i])) << "frame overwritten while alive";
      live.erase(live.begin() + (long)i);
    }
    for (const Frame& f : live) CHECK(intact(f)) << "frame overwritten while alive (round " << round << ")";
  }
  live.clear();
  // everything freed: the ranges coalesced, so one frame of the whole arena fits
  // in it (the same block name as a small frame's)
  {
    auto a = shm::Alloc(MiB);
    std::string small_name, whole_name;
    uint64_t off = 0, off2 = 0;
    CHECK(shm::Find(a.get(), MiB, &small_name, &off));
    a.reset();
    auto whole = shm::Alloc(16 * MiB);
    CHECK(whole);
    CHECK(shm::Find(whole.get(), 16 * MiB, &whole_name, &off2));
    CHECK_EQ(whole_name, small_name) << "the freed arena did not coalesce into one range";
    CHECK_EQ(off2, 0u);
    arena_name = whole_name;
    // while it is taken, another frame comes from a block of its own
    auto other = shm::Alloc(2 * MiB);
    CHECK(other);
    std::string other_name;
    CHECK(shm::Find(other.get(), 2 * MiB, &other_name, &off));
    CHECK(other_name != arena_name) << "a full arena must hand out a separate block";
    // a peer's view: map the arena by name and see a frame's bytes
    std::memset(whole.get(), 0x5a, 16 * MiB);
    size_t sz = 0;
    char* peer = shm::Map(arena_name, &sz);
    CHECK(peer) << "shm::Map of the arena failed";
    CHECK_GE(sz, 16 * MiB);
    CHECK_EQ((unsigned char)peer[12345], 0x5a);
    CHECK_EQ((unsigned char)peer[16 * MiB - 1], 0x5a);
  }
  // a frame larger than the arena: a block of its own
  {
    auto big = shm::Alloc(24 * MiB);
    CHECK(big);
    std::string name;
    uint64_t off = 0;
    CHECK(shm::Find(big.get(), 24 * MiB, &name, &off));
    CHECK(name != arena_name);
    CHECK_EQ(off, 0u);
  }
  shm::UnlinkAll();
  std::printf("shm arena ok\n");
  return 0;
}
