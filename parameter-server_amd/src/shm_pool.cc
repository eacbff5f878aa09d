// shm_pool.cc — host frames between processes as shared-memory mappings
// (internal/shm_pool.h).
#include "internal/shm_pool.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/statvfs.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <thread>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "internal/device.h"
#include "ps/log.h"

namespace ps {
namespace shm {

namespace {
constexpr size_t kMinBytes = size_t(1) << 20;

struct Block {
  std::string name;
  size_t size;
};

struct State {
  std::mutex mu;
  bool enabled = false;
  uint64_t seq = 0;
  std::map<uintptr_t, Block> own;                          // base -> block
  std::map<size_t, std::vector<void*>> free;               // pooled own blocks by size
  std::map<std::string, std::pair<char*, size_t>> mapped;  // peers' blocks
};
State& S() {
  static State* s = new State();  // never destroyed: blocks outlive static teardown
  return *s;
}

// size classes: 64 KiB steps up to 64 MiB, then 16 MiB steps (an 80 MB key
// frame took a 128 MiB block with power-of-two classes: 60 % more to zero)
size_t Round(size_t b) {
  if (b <= (size_t(64) << 20)) return (b + 65535) & ~size_t(65535);
  constexpr size_t kStep = size_t(16) << 20;
  return (b + kStep - 1) & ~(kStep - 1);
}

// Pin a block for DMA where this process drives a GPU — opt-in since round 5
// (PS_SHM_REGISTER=1): hipHostRegister of a fresh 120 MB frame cost the cold
// Push of test_kv_app_benchmark ~10-30 ms on each side (the writer's block,
// the reader's mapping), and a host frame between processes is no longer what
// a GPU copies from: workers stage into HBM themselves, and every host <-> HBM
// copy of the runtime goes through its own pinned staging blocks.
void Register(void* p, size_t n) {
  static const bool on = [] {
    const char* e = std::getenv("PS_SHM_REGISTER");
    return e && std::atoi(e) != 0;
  }();
  if (on && device::Count() > 0) (void)psg_host_register(p, n);
}
}  // namespace

namespace {
void StartArena();
}

void Enable(bool arena) {
  const char* e = std::getenv("PS_SHM_FRAMES");
  {
    std::lock_guard<std::mutex> lk(S().mu);
    if (S().enabled || (e && std::atoi(e) == 0)) return;
    S().enabled = true;
  }
  std::atexit([] { UnlinkAll(); });
  if (arena) StartArena();
}

bool Enabled() {
  std::lock_guard<std::mutex> lk(S().mu);
  return S().enabled;
}

// A block is one or more POSIX shared-memory segments of at most kSeg bytes,
// mapped back to back over one reserved address range; its name is
// "/psg.<pid>.<n>:<segments>:<segment bytes>" and segment k is
// "/psg.<pid>.<n>.<k>".  A fresh block's segments are reserved
// (posix_fallocate: the pages zeroed now, so /dev/shm running out fails here,
// not with SIGBUS at first touch) by several threads at once: tmpfs zeroes
// one file on one thread under its inode lock, and a fresh 128 MiB block in
// one file cost the cold Push of test_kv_app_benchmark ~15 ms in process mode
// (profiles/r5_dropin_after2.txt); in 8 MiB segments 9.8 ms, in 16 MiB ones
// 10.3-10.9 (profiles/r5_dropin_after3.txt).  PS_SHM_SEG_MB sets the segment
// size (default 8).
namespace {
size_t SegBytes() {
  static const size_t v = [] {
    const char* e = std::getenv("PS_SHM_SEG_MB");
    const long mb = e ? std::atol(e) : 8;
    return (size_t)(mb > 0 ? mb : 8) << 20;
  }();
  return v;
}

bool ParseName(const std::string& full, std::string* base, size_t* nseg, size_t* seg) {
  const size_t c1 = full.find(':');
  if (c1 == std::string::npos) return false;
  const size_t c2 = full.find(':', c1 + 1);
  if (c2 == std::string::npos) return false;
  *base = full.substr(0, c1);
  *nseg = (size_t)std::strtoull(full.c_str() + c1 + 1, nullptr, 10);
  *seg = (size_t)std::strtoull(full.c_str() + c2 + 1, nullptr, 10);
  return *nseg > 0 && *seg > 0;
}

// map segment k of a block at base + k * seg (creating and reserving it first
// when `create`)
bool MapSegment(const std::string& base_name, size_t k, size_t seg, size_t total, char* at, bool create,
                bool populate) {
  const std::string name = base_name + "." + std::to_string(k);
  const size_t len = std::min(seg, total - k * seg);
  int fd = create ? shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600) : shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) return false;
  if (create && (ftruncate(fd, (off_t)len) != 0 || posix_fallocate(fd, 0, (off_t)len) != 0)) {
    close(fd);
    return false;
  }
  void* q = mmap(at, len, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_FIXED | (populate ? MAP_POPULATE : 0), fd, 0);
  close(fd);
  return q == at;
}

void UnlinkBlock(const std::string& base_name, size_t nseg) {
  for (size_t k = 0; k < nseg; ++k) shm_unlink((base_name + "." + std::to_string(k)).c_str());
}

// a block of rb bytes over nseg segments; the segments are created on up to 8
// threads at once (`populate`: their page tables filled as well, for the arena)
char* MapBlock(const std::string& base_name, size_t rb, size_t nseg, size_t seg, bool create,
               bool populate = false) {
  void* v = mmap(nullptr, rb, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (v == MAP_FAILED) return nullptr;
  char* at = (char*)v;
  std::atomic<size_t> next{0};
  std::atomic<bool> ok{true};
  auto work = [&] {
    for (size_t k; (k = next.fetch_add(1)) < nseg;)
      if (!MapSegment(base_name, k, seg, rb, at + k * seg, create, populate)) ok = false;
  };
  const size_t nt = create ? std::min<size_t>(nseg, 8) : 1;
  std::vector<std::thread> th;
  for (size_t t = 1; t < nt; ++t) th.emplace_back(work);
  work();
  for (auto& t : th) t.join();
  if (!ok) {
    munmap(v, rb);
    if (create) UnlinkBlock(base_name, nseg);
    return nullptr;
  }
  return at;
}

// The arena: one block of PS_SHM_ARENA_MB (default 256) that a worker or
// server builds on a background thread when its van starts — segments
// reserved and their page tables filled (MAP_POPULATE) — and carves frames
// from, first fit, each frame a (arena name, offset) like any other.  A fresh
// block costs its first frame the page allocation and the write faults of
// every page (tmpfs: the cold 120 MB Push of test_kv_app_benchmark spent
// 9-10 ms of its 10 ms in the copy into a fresh block in process mode,
// profiles/r5_dropin_after3.txt); the arena pays that once, off the request
// path, while the application sets up.  A frame the arena cannot hold takes a
// block of its own as before.
struct Arena {
  std::mutex mu;
  bool started = false;
  std::atomic<bool> ready{false};  // the builder has published base / size / free
  std::atomic<bool> done{false};   // the builder has finished (built or not)
  char* base = nullptr;
  size_t size = 0;
  std::map<size_t, size_t> free;  // offset -> length, coalesced
};
Arena& A() {
  static Arena* a = new Arena();  // never destroyed, like State
  return *a;
}

// PS_SHM_ARENA_MB sets the size; by default 256 MiB, but never more than a
// 1/16 of what /dev/shm has free when the van starts (N workers and N servers
// on one host each build one: 2N arenas must leave room for the frames that do
// not fit them, and for the message rings).
size_t ArenaBytes() {
  const char* e = std::getenv("PS_SHM_ARENA_MB");
  if (e) {
    const long mb = std::atol(e);
    return mb > 0 ? (size_t)mb << 20 : 0;
  }
  size_t bytes = (size_t)256 << 20;
  struct statvfs fs;
  if (statvfs("/dev/shm", &fs) == 0) {
    const size_t cap = (size_t)fs.f_bavail * fs.f_frsize / 16;
    if (cap < bytes) bytes = cap & ~(((size_t)1 << 20) - 1);
  }
  return bytes >= ((size_t)16 << 20) ? bytes : 0;
}

void BuildArena(size_t bytes) {
  State& s = S();
  std::string base_name;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    base_name = "/psg." + std::to_string(getpid()) + "." + std::to_string(s.seq++);
  }
  const size_t seg = SegBytes();
  const size_t nseg = (bytes + seg - 1) / seg;
  const size_t rb = nseg * seg;
  char* p = MapBlock(base_name, rb, nseg, seg, true, true);
  if (!p) {  // no room in /dev/shm: every frame takes a block of its own
    A().done.store(true, std::memory_order_release);
    return;
  }
  Register(p, rb);
  {
    std::lock_guard<std::mutex> lk(s.mu);
    s.own[(uintptr_t)p] = Block{base_name + ":" + std::to_string(nseg) + ":" + std::to_string(seg), rb};
  }
  Arena& a = A();
  {
    std::lock_guard<std::mutex> lk(a.mu);
    a.base = p;
    a.size = rb;
    a.free[0] = rb;
  }
  a.ready.store(true, std::memory_order_release);
  a.done.store(true, std::memory_order_release);
}

// A frame from the arena, or nullptr — also while the arena is still being
// built: a request never waits for the builder (its frame takes a block of its
// own, as without an arena).
void* ArenaTake(size_t rb) {
  Arena& a = A();
  if (!a.ready.load(std::memory_order_acquire)) return nullptr;
  std::lock_guard<std::mutex> lk(a.mu);
  for (auto it = a.free.begin(); it != a.free.end(); ++it) {
    if (it->second < rb) continue;
    const size_t off = it->first, len = it->second;
    a.free.erase(it);
    if (len > rb) a.free[off + rb] = len - rb;
    return a.base + off;
  }
  return nullptr;
}

void ArenaGive(void* q, size_t rb) {
  Arena& a = A();
  std::lock_guard<std::mutex> lk(a.mu);
  size_t off = (size_t)((char*)q - a.base), len = rb;
  auto next = a.free.lower_bound(off);
  if (next != a.free.end() && off + len == next->first) {
    len += next->second;
    next = a.free.erase(next);
  }
  if (next != a.free.begin()) {
    auto prev = std::prev(next);
    if (prev->first + prev->second == off) {
      off = prev->first;
      len += prev->second;
      a.free.erase(prev);
    }
  }
  a.free[off] = len;
}

void StartArena() {
  const size_t bytes = ArenaBytes();
  if (!bytes) return;
  Arena& a = A();
  std::lock_guard<std::mutex> lk(a.mu);
  if (a.started) return;
  std::thread(BuildArena, bytes).detach();  // the arena lives as long as the process
  a.started = true;
}
}  // namespace

std::shared_ptr<void> Alloc(size_t bytes) {
  if (bytes < kMinBytes || !Enabled()) return nullptr;
  const size_t rb = Round(bytes);
  if (void* q = ArenaTake(rb)) return std::shared_ptr<void>(q, [rb](void* r) { ArenaGive(r, rb); });
  State& s = S();
  void* p = nullptr;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    auto& fl = s.free[rb];
    if (!fl.empty()) {
      p = fl.back();
      fl.pop_back();
    }
  }
  if (!p) {
    std::string base_name;
    {
      std::lock_guard<std::mutex> lk(s.mu);
      base_name = "/psg." + std::to_string(getpid()) + "." + std::to_string(s.seq++);
    }
    const size_t seg = SegBytes();
    const size_t nseg = (rb + seg - 1) / seg;
    p = MapBlock(base_name, rb, nseg, seg, true);
    if (!p) return nullptr;
    Register(p, rb);
    std::lock_guard<std::mutex> lk(s.mu);
    s.own[(uintptr_t)p] = Block{base_name + ":" + std::to_string(nseg) + ":" + std::to_string(seg), rb};
  }
  return std::shared_ptr<void>(p, [rb](void* q) {
    std::lock_guard<std::mutex> lk(S().mu);
    S().free[rb].push_back(q);
  });
}

bool Find(const void* p, size_t n, std::string* name, uint64_t* offset) {
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  auto it = s.own.upper_bound((uintptr_t)p);
  if (it == s.own.begin()) return false;
  --it;
  const uintptr_t base = it->first;
  if ((uintptr_t)p + n > base + it->second.size) return false;
  *name = it->second.name;
  *offset = (uint64_t)((uintptr_t)p - base);
  return true;
}

char* Map(const std::string& name, size_t* size) {
  State& s = S();
  {
    std::lock_guard<std::mutex> lk(s.mu);
    auto it = s.mapped.find(name);
    if (it != s.mapped.end()) {
      *size = it->second.second;
      return it->second.first;
    }
  }
  std::string base_name;
  size_t nseg = 0, seg = 0;
  if (!ParseName(name, &base_name, &nseg, &seg)) return nullptr;
  // the block's size: its segments, the last one possibly shorter
  const std::string last = base_name + "." + std::to_string(nseg - 1);
  int fd = shm_open(last.c_str(), O_RDONLY, 0600);
  if (fd < 0) return nullptr;
  struct stat st;
  const bool got = fstat(fd, &st) == 0;
  close(fd);
  if (!got) return nullptr;
  const size_t n = (nseg - 1) * seg + (size_t)st.st_size;
  char* p = MapBlock(base_name, n, nseg, seg, false);
  if (!p) return nullptr;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    auto ins = s.mapped.emplace(name, std::make_pair(p, n));
    if (!ins.second) {  // mapped by a racing reader meanwhile: keep one
      munmap(p, n);
      *size = ins.first->second.second;
      return ins.first->second.first;
    }
  }
  Register(p, n);
  *size = n;
  return p;
}

void UnlinkAll() {
  {
    Arena& a = A();  // a builder still creating segments would leave names behind
    bool started;
    {
      std::lock_guard<std::mutex> lk(a.mu);
      started = a.started;
    }
    while (started && !a.done.load(std::memory_order_acquire)) std::this_thread::yield();
  }
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  for (auto& kv : s.own) {
    std::string base_name;
    size_t nseg = 0, seg = 0;
    if (ParseName(kv.second.name, &base_name, &nseg, &seg)) UnlinkBlock(base_name, nseg);
  }
}

void UnlinkOf(int pid) {
  const std::string prefix = "psg." + std::to_string(pid) + ".";
  DIR* d = opendir("/dev/shm");
  if (!d) return;
  while (dirent* e = readdir(d))
    if (std::strncmp(e->d_name, prefix.c_str(), prefix.size()) == 0)
      shm_unlink(("/" + std::string(e->d_name)).c_str());
  closedir(d);
}

}  // namespace shm
}  // namespace ps
