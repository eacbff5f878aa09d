// probe_host_faults.cpp — what first-touching fresh host memory costs on this
// host (the vector -> SVector copy of a cold Push into new pages, the Pull
// reply's resize): 120 MB written by 1..32 threads after each allocation
// form — malloc; 2 MiB-aligned + MADV_HUGEPAGE; mmap + MAP_POPULATE;
// MADV_POPULATE_WRITE split over the threads; and a recycled (already
// faulted) block.  Prints one line per (form, threads): allocation and touch
// times.  Diagnostics for DESIGN.md (configs[0]'s harness), not on any path.
#include <sys/mman.h>

#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif

using clk = std::chrono::steady_clock;
static double ms(clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); }

static void par(int nt, size_t bytes, void (*f)(char*, size_t), char* p) {
  std::vector<std::thread> th;
  const size_t chunk = (bytes / nt + 4095) & ~size_t(4095);
  for (int i = 0; i < nt; ++i) {
    const size_t off = chunk * i;
    if (off >= bytes) break;
    th.emplace_back(f, p + off, std::min(chunk, bytes - off));
  }
  for (auto& t : th) t.join();
}

int main() {
  const size_t bytes = size_t(120) << 20;
  std::vector<char> src(bytes, 3);
  const char* s = src.data();
  static const char* S;
  S = s;
  auto copy = [](char* p, size_t n) { std::memcpy(p, S + 0, n); };
  (void)copy;
  // a block faulted once and kept (what a pool hands out again)
  static char* kept = (char*)std::malloc(bytes);
  for (size_t i = 0; i < bytes; i += 4096) kept[i] = 1;
  for (int form = 0; form < 5; ++form) {
    for (int nt : {1, 4, 8, 16, 32}) {
      auto t0 = clk::now();
      char* p = nullptr;
      void* raw = nullptr;
      size_t maplen = 0;
      if (form == 0) {
        p = (char*)std::malloc(bytes);
      } else if (form == 1) {
        p = (char*)std::aligned_alloc(size_t(2) << 20, bytes);
        madvise(p, bytes, MADV_HUGEPAGE);
      } else if (form == 2) {
        maplen = bytes;
        raw = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE, -1, 0);
        p = (char*)raw;
      } else if (form == 3) {
        maplen = bytes;
        raw = mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
        p = (char*)raw;
        par(nt, bytes, [](char* q, size_t n) { (void)madvise(q, n, MADV_POPULATE_WRITE); }, p);
      } else {
        p = kept;  // recycled: already faulted
      }
      auto t1 = clk::now();
      par(nt, bytes, [](char* q, size_t n) { std::memcpy(q, S + (q - S) % 4096 * 0, n); }, p);
      auto t2 = clk::now();
      std::printf("form %-10s threads %2d: alloc %7.2f ms  copy 120 MB %7.2f ms\n",
                  form == 0 ? "malloc" : form == 1 ? "hugepage" : form == 2 ? "populate" : form == 3 ? "popwrite" : "recycled",
                  nt, ms(t0, t1), ms(t1, t2));
      if (maplen) munmap(raw, maplen);
      else if (p != kept) std::free(p);
    }
  }
  return 0;
}
