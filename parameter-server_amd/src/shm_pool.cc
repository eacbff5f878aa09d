// shm_pool.cc — host frames between processes as shared-memory mappings
// (internal/shm_pool.h).
#include "internal/shm_pool.h"

#include <dirent.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

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

size_t Round(size_t b) {
  if (b <= (size_t(64) << 20)) return (b + 65535) & ~size_t(65535);
  size_t r = size_t(64) << 20;
  while (r < b) r <<= 1;
  return r;
}

// pin for DMA where this process drives a GPU (best effort: unpinned still works)
void Register(void* p, size_t n) {
  if (device::Count() > 0) (void)psg_host_register(p, n);
}
}  // namespace

void Enable() {
  const char* e = std::getenv("PS_SHM_FRAMES");
  std::lock_guard<std::mutex> lk(S().mu);
  if (S().enabled || (e && std::atoi(e) == 0)) return;
  S().enabled = true;
  std::atexit([] { UnlinkAll(); });
}

bool Enabled() {
  std::lock_guard<std::mutex> lk(S().mu);
  return S().enabled;
}

std::shared_ptr<void> Alloc(size_t bytes) {
  if (bytes < kMinBytes || !Enabled()) return nullptr;
  const size_t rb = Round(bytes);
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
    std::string name;
    {
      std::lock_guard<std::mutex> lk(s.mu);
      name = "/psg." + std::to_string(getpid()) + "." + std::to_string(s.seq++);
    }
    int fd = shm_open(name.c_str(), O_CREAT | O_EXCL | O_RDWR, 0600);
    if (fd < 0) return nullptr;
    // reserve the pages now: a /dev/shm too small for the block fails here
    // instead of with SIGBUS on first touch
    if (ftruncate(fd, (off_t)rb) != 0 || posix_fallocate(fd, 0, (off_t)rb) != 0) {
      close(fd);
      shm_unlink(name.c_str());
      return nullptr;
    }
    p = mmap(nullptr, rb, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    close(fd);
    if (p == MAP_FAILED) {
      shm_unlink(name.c_str());
      return nullptr;
    }
    Register(p, rb);
    std::lock_guard<std::mutex> lk(s.mu);
    s.own[(uintptr_t)p] = Block{name, rb};
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
  int fd = shm_open(name.c_str(), O_RDWR, 0600);
  if (fd < 0) return nullptr;
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return nullptr;
  }
  const size_t n = (size_t)st.st_size;
  void* p = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) return nullptr;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    auto ins = s.mapped.emplace(name, std::make_pair((char*)p, n));
    if (!ins.second) {  // mapped by a racing reader meanwhile: keep one
      munmap(p, n);
      *size = ins.first->second.second;
      return ins.first->second.first;
    }
  }
  Register(p, n);
  *size = n;
  return (char*)p;
}

void UnlinkAll() {
  State& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  for (auto& kv : s.own) shm_unlink(kv.second.name.c_str());
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
