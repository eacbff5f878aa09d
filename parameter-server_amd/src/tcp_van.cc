// tcp_van.cc — process mode: one node per OS process, the way tests/local.py
// runs the reference (local.py:87-114: argv = {prog, config.json, log, role}),
// a TCP Van between the processes, and a launcher that does local.py's job.
//
// Control plane (the reference's Van.cpp:182-443, re-designed for one host):
//   * every server / worker binds a listening socket and sends ADD_NODE to the
//     scheduler at PS_SCHEDULER_URI:PS_SCHEDULER_PORT;
//   * once PS_NUM_SERVER + PS_NUM_WORKER nodes registered, the scheduler orders
//     them as Van.cpp:333-336 does (hostname descending, port ascending), gives
//     server / worker ranks in that order and sends every node the table;
//   * BARRIER requests go to the scheduler, which releases a group once all its
//     members arrived (for customer c > 0: the members on which customer c
//     started — the in-process rule of cluster::Barrier);
//   * a failed CHECK anywhere is broadcast (ABORT), and a peer that disconnects
//     without TERMINATE aborts the job, so no process waits forever.
// Data plane:
//   * host frames are written to the socket (the ZMQ frames of
//     ZMQVan.cpp:147-248);
//   * HBM frames are not copied: the sender ships the hipIpc handle and offset
//     of the frame (psg_ipc_export_range) and keeps the frame alive; the
//     receiver maps the allocation once (psg_ipc_open, cached) and wraps the
//     bytes as an HBM SVector whose last reference sends RELEASE_FRAME back.
//     The server's kernel then reads a worker's keys / values in place — over
//     xGMI when the worker runs on another GPU.  Frames for a node without a
//     GPU or on another host are staged through host memory.
#include <arpa/inet.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <signal.h>
#include <spawn.h>
#include <fcntl.h>
#include <poll.h>
#include <sys/mman.h>
#include <sys/socket.h>
#include <dirent.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <sys/wait.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <chrono>
#include <cstdio>
#include <csignal>
#include <execinfo.h>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <random>
#include <set>
#include <thread>
#include <unordered_map>

#include "internal/Env.h"
#include "internal/PostOffice.h"
#include "internal/stage_time.h"
#include "internal/customer.h"
#include "internal/device.h"
#include "internal/shm_pool.h"

extern char** environ;

namespace ps {

namespace {

constexpr uint32_t kMagic = 0x31475350;  // "PSG1"
constexpr int kHandleBytes = 64;         // sizeof(hipIpcMemHandle_t)

// ---- socket helpers -----------------------------------------------------------
bool WriteAll(int fd, const void* buf, size_t n) {
  const char* p = static_cast<const char*>(buf);
  while (n) {
    ssize_t w = ::send(fd, p, n, MSG_NOSIGNAL);
    if (w < 0 && errno == EINTR) continue;
    if (w <= 0) return false;
    p += w;
    n -= (size_t)w;
  }
  return true;
}

bool ReadAll(int fd, void* buf, size_t n) {
  char* p = static_cast<char*>(buf);
  while (n) {
    ssize_t r = ::recv(fd, p, n, 0);
    if (r < 0 && errno == EINTR) continue;
    if (r <= 0) return false;
    p += r;
    n -= (size_t)r;
  }
  return true;
}

// A connection's reader takes what the socket holds in one recv and serves the
// message's small pieces (header, meta, frame descriptors) from it: one system
// call per message instead of three per frame.  Payloads larger than the
// buffer bypass it.
struct SockReader {
  int fd;
  std::vector<char> buf = std::vector<char>(64 << 10);
  size_t pos = 0, end = 0;
  explicit SockReader(int f) : fd(f) {}
  bool empty() const { return pos == end; }
  bool read(void* out, size_t n) {
    char* p = static_cast<char*>(out);
    const size_t have = std::min(n, end - pos);
    std::memcpy(p, buf.data() + pos, have);
    pos += have;
    p += have;
    n -= have;
    if (!n) return true;
    if (n >= buf.size()) return ReadAll(fd, p, n);
    pos = end = 0;
    while (end < n) {
      ssize_t r = ::recv(fd, buf.data() + end, buf.size() - end, 0);
      if (r < 0 && errno == EINTR) continue;
      if (r <= 0) return false;
      end += (size_t)r;
    }
    std::memcpy(p, buf.data(), n);
    pos = n;
    return true;
  }
};

// ---- shared-memory byte pipe (processes of one host) ---------------------------
// A connection between two processes of one host carries its message bytes
// through a single-producer single-consumer ring in shared memory instead of
// the socket: a request round trip crosses two connections, and a loopback
// TCP hop (two system calls and the stack) costs more than the rest of a small
// request.  The socket stays open beside it: its first bytes name the ring
// (kHello), a reader that found the ring empty for PS_SPIN_US blocks in poll()
// on the socket and the writer rings it (one doorbell byte) only then, and the
// socket's close is how either side learns the other is gone.  PS_SHM_RING=0
// keeps every byte on the socket.
constexpr uint32_t kHello = 0x48475350;  // "PSGH": first bytes of a connection
constexpr uint64_t kRingBytes = 1 << 20;

struct RingHdr {
  std::atomic<uint64_t> head;  // bytes written (writer)
  char pad0[56];
  std::atomic<uint64_t> tail;  // bytes read (reader)
  char pad1[56];
  std::atomic<uint32_t> sleeping;  // the reader waits on the socket for a doorbell
  char pad2[60];
  uint64_t cap;
};
constexpr size_t kRingHdrBytes = 4096;

bool PeerGone(int fd) {  // the peer closed a connection it never writes to
  char c;
  const ssize_t r = ::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
  return r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR);
}

struct Ring {
  RingHdr* h = nullptr;
  char* data = nullptr;
  size_t map_bytes = 0;
  std::string name;
  bool owner = false;
  ~Ring() {
    if (h) ::munmap(h, map_bytes);
    if (owner) ::shm_unlink(name.c_str());  // (gone already once the reader mapped it)
  }
  static std::unique_ptr<Ring> Map(const std::string& name, bool create) {
    const int fd = ::shm_open(name.c_str(), create ? (O_CREAT | O_EXCL | O_RDWR) : O_RDWR, 0600);
    if (fd < 0) return nullptr;
    const size_t bytes = kRingHdrBytes + kRingBytes;
    // the pages reserved now (posix_fallocate): a /dev/shm too small for the
    // ring fails here, and the connection keeps to its socket, instead of a
    // SIGBUS in the first write that touches a page tmpfs cannot supply
    if (create && (::ftruncate(fd, (off_t)bytes) != 0 || ::posix_fallocate(fd, 0, (off_t)bytes) != 0)) {
      ::close(fd);
      ::shm_unlink(name.c_str());
      return nullptr;
    }
    struct stat st;
    if (::fstat(fd, &st) != 0 || (size_t)st.st_size != bytes) {
      ::close(fd);
      if (create) ::shm_unlink(name.c_str());
      return nullptr;
    }
    void* p = ::mmap(nullptr, bytes, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
    ::close(fd);
    if (p == MAP_FAILED) {
      if (create) ::shm_unlink(name.c_str());
      return nullptr;
    }
    auto r = std::make_unique<Ring>();
    r->h = static_cast<RingHdr*>(p);
    r->data = static_cast<char*>(p) + kRingHdrBytes;
    r->map_bytes = bytes;
    r->name = name;
    r->owner = create;
    if (create) {
      new (&r->h->head) std::atomic<uint64_t>(0);
      new (&r->h->tail) std::atomic<uint64_t>(0);
      new (&r->h->sleeping) std::atomic<uint32_t>(0);
      r->h->cap = kRingBytes;
    } else {
      ::shm_unlink(name.c_str());  // both sides hold it now: nothing left to clean up
    }
    return r;
  }
  // writer (under the connection's mutex): false once the peer is gone
  bool Write(int fd, const void* buf, size_t n) {
    const char* p = static_cast<const char*>(buf);
    const uint64_t cap = h->cap;
    while (n) {
      const uint64_t hd = h->head.load(std::memory_order_relaxed);
      const uint64_t room = cap - (hd - h->tail.load(std::memory_order_acquire));
      if (room == 0) {
        if (!WaitRoom(fd)) return false;
        continue;
      }
      const size_t k = (size_t)std::min<uint64_t>(n, room);
      const size_t off = (size_t)(hd % cap), first = std::min(k, (size_t)cap - off);
      std::memcpy(data + off, p, first);
      std::memcpy(data, p + first, k - first);
      h->head.store(hd + k, std::memory_order_seq_cst);
      if (h->sleeping.load(std::memory_order_seq_cst)) {
        const char bell = 0;
        const ssize_t w = ::send(fd, &bell, 1, MSG_NOSIGNAL | MSG_DONTWAIT);
        if (w < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR) return false;
      }
      p += k;
      n -= k;
    }
    return true;
  }
  bool WaitRoom(int fd) {
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0;; ++i) {
      if (h->head.load(std::memory_order_relaxed) - h->tail.load(std::memory_order_acquire) < h->cap) return true;
      if (i < 256) {
        __builtin_ia32_pause();
        continue;
      }
      if (cluster::Aborted() || ((i & 63) == 0 && PeerGone(fd))) return false;
      if (std::chrono::steady_clock::now() - t0 > std::chrono::seconds(600)) return false;
      std::this_thread::sleep_for(std::chrono::microseconds(20));
    }
  }
  // reader: n bytes, waiting as long as the peer lives; false once it closed
  // the socket with nothing left in the ring
  bool Read(int fd, void* out, size_t n) {
    char* p = static_cast<char*>(out);
    const uint64_t cap = h->cap;
    while (n) {
      const uint64_t tl = h->tail.load(std::memory_order_relaxed);
      const uint64_t avail = h->head.load(std::memory_order_acquire) - tl;
      if (avail == 0) {
        if (!WaitData(fd)) return false;
        continue;
      }
      const size_t k = (size_t)std::min<uint64_t>(n, avail);
      const size_t off = (size_t)(tl % cap), first = std::min(k, (size_t)cap - off);
      std::memcpy(p, data + off, first);
      std::memcpy(p + first, data, k - first);
      h->tail.store(tl + k, std::memory_order_release);
      p += k;
      n -= k;
    }
    return true;
  }
  bool has_data() const {
    return h->head.load(std::memory_order_acquire) != h->tail.load(std::memory_order_relaxed);
  }
  bool WaitData(int fd) {
    const int us = SpinMicros();
    const auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; us > 0; ++i) {
      if (has_data()) return true;
      if ((i & 7) == 7 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(us)) break;
      __builtin_ia32_pause();
    }
    while (true) {
      h->sleeping.store(1, std::memory_order_seq_cst);
      if (h->head.load(std::memory_order_seq_cst) != h->tail.load(std::memory_order_relaxed)) {
        h->sleeping.store(0, std::memory_order_relaxed);
        return true;
      }
      pollfd pfd{fd, POLLIN, 0};
      const int pr = ::poll(&pfd, 1, 100);
      h->sleeping.store(0, std::memory_order_relaxed);
      if (pr < 0 && errno != EINTR) return has_data();
      if (pr > 0) {
        char bells[256];
        const ssize_t r = ::recv(fd, bells, sizeof(bells), MSG_DONTWAIT);
        if (r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR))
          return has_data();  // closed: what is left in the ring is still read
      }
      if (has_data()) return true;
    }
  }
};

// The reader's answer to a connection's ring (ReadLoop), read by the writer
// before its first message (Connect): 1 — 'Y', the ring carries the bytes; 0 —
// an explicit 'N' (the reader could not map it), every byte on the socket; -1
// — the socket closed, failed or gave no answer in PS_RING_ACK_MS (default
// 10 s).  Only 'N' may fall back to the socket: a reader that maps the ring
// after the writer gave up would read only the ring and take the socket's
// bytes for doorbells, so -1 fails the connection instead.
// PS_RING_ACK_DELAY_MS delays the reader's answer (fault injection, tests).
constexpr char kRingYes = 'Y', kRingNo = 'N';
int RingAccepted(int fd) {
  static const int limit_ms = [] {
    const char* e = std::getenv("PS_RING_ACK_MS");
    const int v = e ? std::atoi(e) : 0;
    return v > 0 ? v : 10000;
  }();
  pollfd pfd{fd, POLLIN, 0};
  for (int waited = 0; waited < limit_ms; waited += 100) {
    const int pr = ::poll(&pfd, 1, 100);
    if (pr < 0 && errno != EINTR) return -1;
    if (pr > 0) {
      char a = 0;
      const ssize_t r = ::recv(fd, &a, 1, 0);
      if (r != 1) return -1;
      return a == kRingYes ? 1 : a == kRingNo ? 0 : -1;
    }
  }
  errno = ETIMEDOUT;
  return -1;
}
int RingAckDelayMs() {
  static const int v = [] {
    const char* e = std::getenv("PS_RING_ACK_DELAY_MS");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

bool RingEnabled() {
  static const bool on = [] {
    const char* e = std::getenv("PS_SHM_RING");
    return !(e && std::atoi(e) == 0);
  }();
  return on;
}

// Before a connection's reader blocks in recv for the next message, poll the
// socket for up to PS_SPIN_US (default 250 us, the spin of the request queues,
// internal/customer.h): a request round trip crosses the socket twice, and a
// blocked reader's wake-up costs more than a loopback hop.
void SpinUntilReadable(int fd) {
  const int us = SpinMicros();
  if (us <= 0) return;
  const auto t0 = std::chrono::steady_clock::now();
  char c;
  for (int i = 0;; ++i) {
    const ssize_t r = ::recv(fd, &c, 1, MSG_PEEK | MSG_DONTWAIT);
    if (r > 0 || r == 0 || (r < 0 && errno != EAGAIN && errno != EWOULDBLOCK && errno != EINTR)) return;
    if ((i & 7) == 7 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(us)) return;
    __builtin_ia32_pause();
  }
}

void Tune(int fd) {
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  int buf = 8 << 20;
  setsockopt(fd, SOL_SOCKET, SO_SNDBUF, &buf, sizeof(buf));
  setsockopt(fd, SOL_SOCKET, SO_RCVBUF, &buf, sizeof(buf));
}

bool Resolve(const std::string& host, int port, sockaddr_in* sa) {
  std::memset(sa, 0, sizeof(*sa));
  sa->sin_family = AF_INET;
  sa->sin_port = htons((uint16_t)port);
  if (inet_pton(AF_INET, host.c_str(), &sa->sin_addr) == 1) return true;
  addrinfo hints{}, *res = nullptr;
  hints.ai_family = AF_INET;
  if (getaddrinfo(host.c_str(), nullptr, &hints, &res) != 0 || !res) return false;
  sa->sin_addr = reinterpret_cast<sockaddr_in*>(res->ai_addr)->sin_addr;
  freeaddrinfo(res);
  return true;
}

// ---- message codec ------------------------------------------------------------
struct Writer {
  std::string b;
  template <typename T>
  void pod(const T& v) {
    b.append(reinterpret_cast<const char*>(&v), sizeof(T));
  }
  void str(const std::string& s) {
    pod<uint32_t>((uint32_t)s.size());
    b.append(s);
  }
};

struct Reader {
  const char* p;
  const char* e;
  template <typename T>
  T pod() {
    CHECK(p + sizeof(T) <= e) << "truncated message";
    T v;
    std::memcpy(&v, p, sizeof(T));
    p += sizeof(T);
    return v;
  }
  std::string str() {
    const uint32_t n = pod<uint32_t>();
    CHECK(p + n <= e) << "truncated message";
    std::string s(p, n);
    p += n;
    return s;
  }
};

void PutNode(Writer& w, const Node& n) {
  w.pod<int32_t>(n.role);
  w.pod<int32_t>(n.id);
  w.pod<int32_t>(n.customer_id);
  w.str(n.hostname);
  w.pod<int32_t>(n.port);
  w.pod<uint8_t>(n.is_recovered);
  w.pod<uint8_t>(n.gpu);
}

Node GetNode(Reader& r) {
  Node n;
  n.role = (Node::Role)r.pod<int32_t>();
  n.id = r.pod<int32_t>();
  n.customer_id = r.pod<int32_t>();
  n.hostname = r.str();
  n.port = r.pod<int32_t>();
  n.is_recovered = r.pod<uint8_t>() != 0;
  n.gpu = r.pod<uint8_t>() != 0;
  return n;
}

void PutMeta(Writer& w, const Meta& m) {
  w.pod<int32_t>(m.head);
  w.pod<int32_t>(m.app_id);
  w.pod<int32_t>(m.customer_id);
  w.pod<int32_t>(m.timestamp);
  w.pod<int32_t>(m.sender);
  w.pod<int32_t>(m.receiver);
  w.pod<uint8_t>((uint8_t)(m.request | (m.push << 1) | (m.pull << 2) | (m.simple_app << 3) | (m.hbm_handle << 4) |
                           (m.direct_reply << 5) | (m.spec_slice << 6) | (m.refused << 7)));
  w.str(m.body);
  w.pod<uint32_t>((uint32_t)m.data_type.size());
  for (DataType t : m.data_type) w.pod<int32_t>((int32_t)t);
  w.pod<int32_t>(m.control.cmd);
  w.pod<uint32_t>((uint32_t)m.control.nodes.size());
  for (const Node& n : m.control.nodes) PutNode(w, n);
  w.pod<int32_t>(m.control.barrier_group);
  w.pod<uint64_t>(m.control.msg_sig);
  w.pod<int32_t>(m.data_size);
  w.pod<int32_t>(m.priority);
}

Meta GetMeta(Reader& r) {
  Meta m;
  m.head = r.pod<int32_t>();
  m.app_id = r.pod<int32_t>();
  m.customer_id = r.pod<int32_t>();
  m.timestamp = r.pod<int32_t>();
  m.sender = r.pod<int32_t>();
  m.receiver = r.pod<int32_t>();
  const uint8_t f = r.pod<uint8_t>();
  m.request = f & 1;
  m.push = (f >> 1) & 1;
  m.pull = (f >> 2) & 1;
  m.simple_app = (f >> 3) & 1;
  m.hbm_handle = (f >> 4) & 1;
  m.direct_reply = (f >> 5) & 1;
  m.spec_slice = (f >> 6) & 1;
  m.refused = (f >> 7) & 1;
  m.body = r.str();
  const uint32_t nt = r.pod<uint32_t>();
  for (uint32_t i = 0; i < nt; ++i) m.data_type.push_back((DataType)r.pod<int32_t>());
  m.control.cmd = (Control::Command)r.pod<int32_t>();
  const uint32_t nn = r.pod<uint32_t>();
  for (uint32_t i = 0; i < nn; ++i) m.control.nodes.push_back(GetNode(r));
  m.control.barrier_group = r.pod<int32_t>();
  m.control.msg_sig = r.pod<uint64_t>();
  m.data_size = r.pod<int32_t>();
  m.priority = r.pod<int32_t>();
  return m;
}

struct WireHeader {
  uint32_t magic;
  uint32_t meta_bytes;
  uint32_t nframes;
  uint32_t reserved;
};

// kPeerFrame: a slice of an HBM frame the RECEIVER sent earlier and this node
// mapped (a reply that echoes the request's keys, KVApp.h:449-455): sent back
// as (token, offset) and resolved to the receiver's own array.
// kShmFrame: a host frame in one of the sender's shared-memory blocks
// (internal/shm_pool.h), sent as (block name, offset) and mapped in place.
enum FrameKind : uint8_t { kHostFrame = 0, kIpcFrame = 1, kPeerFrame = 2, kShmFrame = 3 };

struct ShmFrame {
  char name[48];
  uint64_t offset;
  uint64_t token;
};

struct PeerFrame {
  uint64_t token;
  uint64_t offset;
};

struct IpcFrame {  // follows the frame's kind + size for kIpcFrame
  char handle[kHandleBytes];
  uint64_t offset;
  uint64_t token;
  int32_t device;
};

// HBM frames of peers mapped into this process: the views (so a reply can
// point back into its receiver's own array) and the RELEASE_FRAME queue their
// last references fill.  Shared with the views' deleters, so it outlives the Van.
struct FrameRegistry {
  struct View {
    uintptr_t end;
    int owner;
    uint64_t token;
  };
  std::mutex mu;
  std::condition_variable cv;
  std::map<uintptr_t, View> views;          // start -> view
  std::vector<std::pair<int, uint64_t>> q;  // (owner node id, token) to release
  bool closed = false;
  void Add(const char* p, uint64_t bytes, int owner, uint64_t token) {
    std::lock_guard<std::mutex> lk(mu);
    views[(uintptr_t)p] = View{(uintptr_t)p + bytes, owner, token};
  }
  void Release(const char* p, int owner, uint64_t token) {
    {
      std::lock_guard<std::mutex> lk(mu);
      views.erase((uintptr_t)p);
      if (closed) return;
      q.emplace_back(owner, token);
    }
    cv.notify_one();
  }
  /* the mapped view of `owner` containing [p, p + bytes), if any */
  bool Find(const char* p, uint64_t bytes, int owner, PeerFrame* out) {
    std::lock_guard<std::mutex> lk(mu);
    auto it = views.upper_bound((uintptr_t)p);
    if (it == views.begin()) return false;
    --it;
    const View& v = it->second;
    if (v.owner != owner || (uintptr_t)p + bytes > v.end) return false;
    out->token = v.token;
    out->offset = (uint64_t)((uintptr_t)p - it->first);
    return true;
  }
};

struct Conn {
  int fd = -1;
  std::mutex mu;               // one writer at a time
  std::unique_ptr<Ring> ring;  // the message bytes' path when the peer shares this host
  bool Put(const void* p, size_t n) { return ring ? ring->Write(fd, p, n) : WriteAll(fd, p, n); }
  ~Conn() {
    ring.reset();
    if (fd >= 0) ::close(fd);
  }
};

class TcpVan : public Van {
 public:
  explicit TcpVan(PostOffice* po) : Van(po), rel_(std::make_shared<FrameRegistry>()) {}
  ~TcpVan() override { Stop(); }

  void Start(int customer_id) override;
  void Stop() override;
  bool Barrier(int customer_id, int group) override;
  void NoteStarted(int customer_id) override;
  void NotifyAbort(const std::string& why) override;
  bool GroupBroadcast(int group, const std::string& mine, std::string* out) override;

 protected:
  int SendMsg(const Message& msg) override;

 private:
  void Listen(const std::string& host, int port);
  void AcceptLoop();
  void ReadLoop(int fd);
  void ReleaseLoop();
  void Dispatch(Message& msg);
  void OnAddNode(const Message& msg);
  void OnBarrier(const Message& msg);
  void OnGroupBroadcast(const Message& msg);
  std::shared_ptr<Conn> Connect(int id);
  std::string last_connect_error_;  // the stage and errno of the last Connect that failed (peers_mu_)
  std::string LastConnectError() {
    std::lock_guard<std::mutex> lk(peers_mu_);
    return last_connect_error_;
  }
  int Encode(const Message& msg, const Node& to, std::string* head, std::vector<SVector<char>>* host_frames);
  SVector<char> MapFrame(int sender, const IpcFrame& f, uint64_t bytes);
  SVector<char> MapShmFrame(int sender, const ShmFrame& f, uint64_t bytes);
  void SendControl(int to, Control::Command cmd, int group = 0, int customer_id = 0, const std::string& body = "");
  bool Abandoned() const { return cluster::Aborted(); }

  bool is_scheduler_ = false;
  std::string my_host_;
  int listen_fd_ = -1;
  std::atomic<bool> stopping_{false};
  std::thread accept_thread_, release_thread_;
  std::mutex readers_mu_;
  std::vector<std::thread> readers_;
  std::vector<int> reader_fds_;

  std::mutex peers_mu_;
  std::map<int, Node> nodes_;                    // id -> address (scheduler: from the config)
  std::map<int, std::shared_ptr<Conn>> conns_;  // id -> outgoing connection
  std::set<int> terminated_;                    // peers that said goodbye

  std::mutex reg_mu_;
  std::condition_variable reg_cv_;
  bool registered_ = false;
  std::vector<Node> joined_;  // scheduler: ADD_NODE requests so far

  std::mutex bar_mu_;
  std::condition_variable bar_cv_;
  std::map<std::pair<int, int>, uint64_t> bar_gen_;  // (group, customer) -> releases seen
  std::map<std::pair<int, int>, int> bar_count_;     // scheduler: arrivals
  std::map<int, std::set<int>> started_;             // scheduler: customer -> node ids
  struct Bcast {
    uint64_t gen = 0;    // results seen (node side)
    int arrived = 0;     // scheduler side
    std::string root_bytes, result;
  };
  std::map<int, Bcast> bcasts_;  // group -> rendezvous

  std::mutex frames_mu_;
  uint64_t next_token_ = 1;
  std::unordered_map<uint64_t, SVector<char>> inflight_;  // frames peers have mapped
  std::map<std::pair<int, std::string>, char*> mapped_;   // (owner, handle) -> base
  std::shared_ptr<FrameRegistry> rel_;
  std::atomic<bool> abort_sent_{false};
  bool started_van_ = false;
  std::atomic<uint64_t> sent_kind_[4] = {};  // frames sent per FrameKind (PS_VAN_STATS=1 prints them)
};

// ---------------------------------------------------------------------------
void TcpVan::Listen(const std::string& host, int port) {
  listen_fd_ = ::socket(AF_INET, SOCK_STREAM, 0);
  CHECK_GE(listen_fd_, 0) << "socket: " << std::strerror(errno);
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  sockaddr_in sa;
  CHECK(Resolve(host, port, &sa)) << "cannot resolve " << host;
  CHECK_EQ(::bind(listen_fd_, (sockaddr*)&sa, sizeof(sa)), 0)
      << "bind " << host << ":" << port << ": " << std::strerror(errno);
  CHECK_EQ(::listen(listen_fd_, 128), 0) << "listen: " << std::strerror(errno);
  socklen_t len = sizeof(sa);
  getsockname(listen_fd_, (sockaddr*)&sa, &len);
  my_node_.hostname = host;
  my_node_.port = ntohs(sa.sin_port);
  accept_thread_ = std::thread([this] { AcceptLoop(); });
}

void TcpVan::AcceptLoop() {
  while (!stopping_) {
    int fd = ::accept(listen_fd_, nullptr, nullptr);
    if (fd < 0) {
      if (errno == EINTR) continue;
      return;  // listening socket shut down
    }
    Tune(fd);
    std::lock_guard<std::mutex> lk(readers_mu_);
    reader_fds_.push_back(fd);
    readers_.emplace_back([this, fd] { ReadLoop(fd); });
  }
}

void TcpVan::Start(int customer_id) {
  (void)customer_id;
  if (started_van_) return;
  started_van_ = true;
  is_scheduler_ = po_->is_scheduler();
  my_host_ = Environment::GetOrDefault("PS_NODE_HOST", "127.0.0.1");
  const std::string sched_host = Environment::GetOrDefault("PS_SCHEDULER_URI", "127.0.0.1");
  const int sched_port = Environment::GetIntOrDefault("PS_SCHEDULER_PORT", 8000);
  const int timeout_s = Environment::GetIntOrDefault("PS_REGISTER_TIMEOUT", 120);
  Node sched;
  sched.role = Node::SCHEDULER;
  sched.id = kScheduler;
  sched.hostname = sched_host;
  sched.port = sched_port;
  {
    std::lock_guard<std::mutex> lk(peers_mu_);
    nodes_[kScheduler] = sched;
  }
  release_thread_ = std::thread([this] { ReleaseLoop(); });
  const auto deadline = std::chrono::steady_clock::now() + std::chrono::seconds(timeout_s);
  if (is_scheduler_) {
    my_node_ = sched;
    Listen(sched_host, sched_port);
    const size_t expect = (size_t)(po_->num_servers() + po_->num_workers());
    std::vector<Node> joined;
    {
      std::unique_lock<std::mutex> lk(reg_mu_);
      CHECK(reg_cv_.wait_until(lk, deadline, [&] { return joined_.size() >= expect || Abandoned(); }))
          << "scheduler: " << joined_.size() << " of " << expect << " nodes registered in " << timeout_s << " s";
      joined = joined_;
    }
    CHECK(!Abandoned()) << "job aborted during registration: " << cluster::AbortReason();
    // ranks in address order (Van.cpp:333-336)
    std::sort(joined.begin(), joined.end(), [](const Node& a, const Node& b) {
      int c = a.hostname.compare(b.hostname);
      return c != 0 ? c > 0 : a.port < b.port;
    });
    int ns = 0, nw = 0;
    for (Node& n : joined) n.id = n.role == Node::SERVER ? PostOffice::ServerRankToID(ns++) : PostOffice::WorkerRankToID(nw++);
    CHECK_EQ(ns, po_->num_servers()) << "registered servers";
    CHECK_EQ(nw, po_->num_workers()) << "registered workers";
    joined.push_back(my_node_);
    {
      std::lock_guard<std::mutex> lk(peers_mu_);
      for (const Node& n : joined) nodes_[n.id] = n;
    }
    Message table;
    table.meta.control.cmd = Control::ADD_NODE;
    table.meta.control.nodes = joined;
    for (const Node& n : joined) {
      if (n.id == kScheduler) continue;
      table.meta.receiver = n.id;
      table.meta.timestamp = GetAvailableTimestamp();
      Send(table);
    }
    std::lock_guard<std::mutex> lk(reg_mu_);
    registered_ = true;
  } else {
    Listen(my_host_, 0);
    my_node_.role = po_->role();
    my_node_.id = Node::kEmpty;
    my_node_.gpu = device::Count() > 0;
    // the scheduler may start after us (local.py starts them in order, but
    // nothing waits): retry the first connection until the deadline
    std::shared_ptr<Conn> c;
    auto next_note = std::chrono::steady_clock::now() + std::chrono::seconds(5);
    while (!(c = Connect(kScheduler))) {
      CHECK(std::chrono::steady_clock::now() < deadline)
          << "cannot reach the scheduler at " << sched_host << ":" << sched_port << " (" << LastConnectError() << ")";
      if (std::chrono::steady_clock::now() > next_note) {
        LOG(WARNING) << "still connecting to the scheduler: " << LastConnectError();
        next_note += std::chrono::seconds(5);
      }
      std::this_thread::sleep_for(std::chrono::milliseconds(50));
    }
    Message join;
    join.meta.control.cmd = Control::ADD_NODE;
    join.meta.request = true;
    join.meta.receiver = kScheduler;
    join.meta.control.nodes.push_back(my_node_);
    CHECK_NE(SendMsg(join), -1) << "ADD_NODE to the scheduler failed";
    std::unique_lock<std::mutex> lk(reg_mu_);
    CHECK(reg_cv_.wait_until(lk, deadline, [&] { return registered_ || Abandoned(); }))
        << "no node table from the scheduler in " << timeout_s << " s";
    CHECK(!Abandoned()) << "job aborted during registration: " << cluster::AbortReason();
  }
  ready_ = true;
}

void TcpVan::OnAddNode(const Message& msg) {
  if (msg.meta.request) {  // at the scheduler
    CHECK(is_scheduler_) << "ADD_NODE request at a non-scheduler";
    CHECK_EQ(msg.meta.control.nodes.size(), (size_t)1);
    std::lock_guard<std::mutex> lk(reg_mu_);
    joined_.push_back(msg.meta.control.nodes[0]);
    reg_cv_.notify_all();
    return;
  }
  // the node table (Van.cpp:420-443)
  int my_rank = -1;
  {
    std::lock_guard<std::mutex> lk(peers_mu_);
    for (const Node& n : msg.meta.control.nodes) {
      nodes_[n.id] = n;
      if (n.hostname == my_node_.hostname && n.port == my_node_.port) {
        my_node_.id = n.id;
        my_rank = PostOffice::IDToRank(n.id);
      }
    }
  }
  CHECK_GE(my_rank, 0) << "this node is missing from the scheduler's table";
  const int ndev = device::Count();
  po_->SetIdentity(my_rank, ndev > 0 ? my_rank % ndev : -1);
  std::lock_guard<std::mutex> lk(reg_mu_);
  registered_ = true;
  reg_cv_.notify_all();
}

void TcpVan::OnBarrier(const Message& msg) {
  const int group = msg.meta.control.barrier_group;
  const int cid = msg.meta.customer_id;
  const auto key = std::make_pair(group, cid);
  if (!msg.meta.request) {  // release
    std::lock_guard<std::mutex> lk(bar_mu_);
    ++bar_gen_[key];
    bar_cv_.notify_all();
    return;
  }
  CHECK(is_scheduler_) << "BARRIER request at a non-scheduler";
  std::vector<int> release;
  {
    std::lock_guard<std::mutex> lk(bar_mu_);
    const auto& ids = po_->GetNodeIDs(group);
    int participants = (int)ids.size();
    if (cid != 0) {
      participants = 0;
      for (int id : ids) participants += started_[cid].count(id) ? 1 : 0;
      participants = std::max(participants, 1);
    }
    if (++bar_count_[key] < participants) return;
    bar_count_[key] = 0;
    for (int id : ids)
      if (cid == 0 || started_[cid].count(id)) release.push_back(id);
    if (release.empty()) release.push_back(msg.meta.sender);
  }
  // the scheduler's own release last: once it returns from the barrier it may
  // stop its Van, and every other member must have its release by then
  std::stable_partition(release.begin(), release.end(), [](int id) { return id != kScheduler; });
  for (int id : release) SendControl(id, Control::BARRIER, group, cid);
}

void TcpVan::OnGroupBroadcast(const Message& msg) {
  const int group = msg.meta.control.barrier_group;
  if (!msg.meta.request) {  // the root's bytes, from the scheduler
    std::lock_guard<std::mutex> lk(bar_mu_);
    Bcast& b = bcasts_[group];
    b.result = msg.meta.body;
    ++b.gen;
    bar_cv_.notify_all();
    return;
  }
  CHECK(is_scheduler_) << "GROUP_BCAST request at a non-scheduler";
  std::vector<int> members;
  std::string bytes;
  {
    std::lock_guard<std::mutex> lk(bar_mu_);
    const auto& ids = po_->GetNodeIDs(group);
    Bcast& b = bcasts_[group];
    if (msg.meta.control.msg_sig) b.root_bytes = msg.meta.body;  // from the root
    if (++b.arrived < (int)ids.size()) return;
    b.arrived = 0;
    bytes = b.root_bytes;
    members.assign(ids.begin(), ids.end());
  }
  std::stable_partition(members.begin(), members.end(), [](int id) { return id != kScheduler; });
  for (int id : members) {
    Message m;
    m.meta.control.cmd = Control::GROUP_BCAST;
    m.meta.control.barrier_group = group;
    m.meta.body = bytes;
    m.meta.receiver = id;
    m.meta.request = false;
    m.meta.sender = my_node_.id;
    CHECK_NE(SendMsg(m), -1) << "group broadcast to node " << id << " failed";
  }
}

bool TcpVan::GroupBroadcast(int group, const std::string& mine, std::string* out) {
  const auto& ids = po_->GetNodeIDs(group);
  const bool root = my_node_.id == *std::min_element(ids.begin(), ids.end());
  uint64_t gen;
  {
    std::lock_guard<std::mutex> lk(bar_mu_);
    gen = bcasts_[group].gen;
  }
  Message req;
  req.meta.request = true;
  req.meta.control.cmd = Control::GROUP_BCAST;
  req.meta.control.barrier_group = group;
  req.meta.control.msg_sig = root ? 1 : 0;
  if (root) req.meta.body = mine;
  req.meta.receiver = kScheduler;
  req.meta.timestamp = GetAvailableTimestamp();
  Send(req);
  std::unique_lock<std::mutex> lk(bar_mu_);
  while (bcasts_[group].gen == gen) {
    bar_cv_.wait_for(lk, std::chrono::milliseconds(100));
    if (Abandoned()) {
      lk.unlock();
      LOG(FATAL) << "group broadcast abandoned: " << cluster::AbortReason();
    }
  }
  *out = bcasts_[group].result;
  return true;
}

bool TcpVan::Barrier(int customer_id, int group) {
  const auto key = std::make_pair(group, customer_id);
  uint64_t gen;
  {
    std::lock_guard<std::mutex> lk(bar_mu_);
    gen = bar_gen_[key];
  }
  Message req;
  req.meta.request = true;
  req.meta.control.cmd = Control::BARRIER;
  req.meta.control.barrier_group = group;
  req.meta.customer_id = customer_id;
  req.meta.receiver = kScheduler;
  req.meta.timestamp = GetAvailableTimestamp();
  Send(req);
  std::unique_lock<std::mutex> lk(bar_mu_);
  while (bar_gen_[key] == gen) {
    bar_cv_.wait_for(lk, std::chrono::milliseconds(100));
    if (Abandoned()) {
      lk.unlock();
      LOG(FATAL) << "barrier abandoned: " << cluster::AbortReason();
    }
  }
  return true;
}

void TcpVan::NoteStarted(int customer_id) {
  if (is_scheduler_) {
    std::lock_guard<std::mutex> lk(bar_mu_);
    started_[customer_id].insert(kScheduler);
    return;
  }
  SendControl(kScheduler, Control::STARTED, 0, customer_id);
}

void TcpVan::NotifyAbort(const std::string& why) {
  if (abort_sent_.exchange(true)) return;
  if (!started_van_) return;
  if (is_scheduler_) {
    std::vector<int> ids;
    {
      std::lock_guard<std::mutex> lk(peers_mu_);
      for (auto& kv : nodes_)
        if (kv.first != kScheduler) ids.push_back(kv.first);
    }
    for (int id : ids) SendControl(id, Control::ABORT, 0, 0, why);
  } else {
    SendControl(kScheduler, Control::ABORT, 0, 0, why);
  }
}

void TcpVan::SendControl(int to, Control::Command cmd, int group, int customer_id, const std::string& body) {
  Message m;
  m.meta.control.cmd = cmd;
  m.meta.control.barrier_group = group;
  m.meta.customer_id = customer_id;
  m.meta.body = body;
  m.meta.receiver = to;
  m.meta.request = false;
  m.meta.sender = my_node_.id;
  const int rc = SendMsg(m);
  // control traffic to a peer that already left (a late RELEASE_FRAME, an
  // ABORT racing an exit) is not an error
  if (rc < 0 && cmd != Control::RELEASE_FRAME && cmd != Control::ABORT && cmd != Control::TERMINATE && !stopping_)
    LOG(FATAL) << "control message to node " << to << " failed";
}

// ---------------------------------------------------------------------------
std::shared_ptr<Conn> TcpVan::Connect(int id) {
  Node n;
  {
    std::lock_guard<std::mutex> lk(peers_mu_);
    auto it = conns_.find(id);
    if (it != conns_.end()) return it->second;
    auto nt = nodes_.find(id);
    if (nt == nodes_.end()) return nullptr;
    n = nt->second;
  }
  sockaddr_in sa;
  auto failed = [&](const char* stage) {
    std::string why = std::string(stage) + " " + n.hostname + ":" + std::to_string(n.port) + ": " + std::strerror(errno);
    std::lock_guard<std::mutex> lk(peers_mu_);
    last_connect_error_ = std::move(why);
    return nullptr;
  };
  if (!Resolve(n.hostname, n.port, &sa)) return failed("resolve");
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return failed("socket");
  if (::connect(fd, (sockaddr*)&sa, sizeof(sa)) != 0) {
    const int e = errno;
    ::close(fd);
    errno = e;
    return failed("connect");
  }
  Tune(fd);
  auto c = std::make_shared<Conn>();
  c->fd = fd;
  // the connection's first bytes: kHello and the name of its ring (empty: the
  // socket carries everything)
  std::string name;
  if (RingEnabled() && n.hostname == my_node_.hostname) {
    static std::atomic<uint64_t> seq{0};
    name = "/psgring." + std::to_string(::getpid()) + "." + std::to_string(my_node_.id) + "." + std::to_string(id) +
           "." + std::to_string(seq++);
    c->ring = Ring::Map(name, true);
    if (!c->ring) name.clear();
  }
  const uint32_t hello[2] = {kHello, (uint32_t)name.size()};
  if (!WriteAll(fd, hello, sizeof(hello)) || (name.size() && !WriteAll(fd, name.data(), name.size())))
    return failed("hello to");  // (c closes fd)
  if (c->ring) {
    const int acc = RingAccepted(fd);
    if (acc < 0) return failed("ring answer from");  // no answer: fail, never guess (c closes fd)
    if (acc == 0) c->ring.reset();  // the reader could not map it: the socket carries all
  }
  std::lock_guard<std::mutex> lk(peers_mu_);
  auto ins = conns_.emplace(id, c);
  return ins.first->second;  // a racing connect to the same peer: keep one
}

int TcpVan::Encode(const Message& msg, const Node& to, std::string* head,
                   std::vector<SVector<char>>* host_frames) {
  Writer meta;
  PutMeta(meta, msg.meta);
  Writer frames;
  int64_t bytes = 0;  // frames may exceed 2 GiB (a 1 B-element f16 Push)
  const bool same_host = to.hostname == my_node_.hostname;
  const bool can_map = to.gpu && same_host;
  for (const SVector<char>& f : msg.data) {
    PeerFrame pf;
    if (f.size() && rel_->Find(f.data(), f.size(), to.id, &pf)) {
      ++sent_kind_[kPeerFrame];
      frames.pod<uint8_t>(kPeerFrame);
      frames.pod<uint64_t>(f.size());
      frames.pod(pf);
      bytes += (int64_t)sizeof(pf);
      continue;
    }
    if (f.on_device() && f.size() && can_map) {
      IpcFrame d;
      std::memset(&d, 0, sizeof(d));
      if (psg_ipc_export_range(f.data(), d.handle, &d.offset) == PSG_OK) {
        d.device = f.device();
        {
          std::lock_guard<std::mutex> lk(frames_mu_);
          d.token = next_token_++;
          inflight_[d.token] = f;
        }
        ++sent_kind_[kIpcFrame];
        frames.pod<uint8_t>(kIpcFrame);
        frames.pod<uint64_t>(f.size());
        frames.pod(d);
        bytes += (int64_t)sizeof(d);
        continue;
      }
      LOG(WARNING) << "hipIpc export of an HBM frame failed (" << psg_last_error() << "); sending its bytes";
    }
    ShmFrame sf;
    std::string sname;
    if (!f.on_device() && f.size() && same_host && shm::Find(f.data(), f.size(), &sname, &sf.offset) &&
        sname.size() < sizeof(sf.name)) {
      std::memset(sf.name, 0, sizeof(sf.name));
      std::memcpy(sf.name, sname.data(), sname.size());
      {
        std::lock_guard<std::mutex> lk(frames_mu_);
        sf.token = next_token_++;
        inflight_[sf.token] = f;
      }
      ++sent_kind_[kShmFrame];
      frames.pod<uint8_t>(kShmFrame);
      frames.pod<uint64_t>(f.size());
      frames.pod(sf);
      bytes += (int64_t)sizeof(sf);
      continue;
    }
    SVector<char> h = f;
    if (f.on_device() && f.size()) {
      h = SVector<char>::Uninitialized(f.size());
      device::CopySync(h.data(), f.data(), f.size(), 1);
    }
    if (h.size()) ++sent_kind_[kHostFrame];
    frames.pod<uint8_t>(kHostFrame);
    frames.pod<uint64_t>(h.size());
    host_frames->push_back(h);
    bytes += (int64_t)h.size();
  }
  WireHeader wh{kMagic, (uint32_t)meta.b.size(), (uint32_t)msg.data.size(), 0};
  head->assign(reinterpret_cast<const char*>(&wh), sizeof(wh));
  head->append(meta.b);
  head->append(frames.b);
  bytes += (int64_t)head->size();
  return bytes > INT32_MAX ? INT32_MAX : (int)bytes;  // Van::SendMsg reports an int
}

int TcpVan::SendMsg(const Message& msg) {
  stage::Scope t_send(msg.meta.control.cmd == Control::EMPTY ? "van.send" : "van.send.control", msg.meta.data_size);
  const int to = msg.meta.receiver;
  if (to == my_node_.id && my_node_.id != Node::kEmpty) {  // to itself: no socket
    Message m = msg;
    Dispatch(m);
    return (int)sizeof(Meta) + msg.meta.data_size;
  }
  // a connection whose ring got no answer in time is closed (Connect): try a
  // fresh one twice more before the message fails
  std::shared_ptr<Conn> c;
  for (int attempt = 0; attempt < 3 && !(c = Connect(to)); ++attempt) {
    const std::string why = LastConnectError();
    if (why.rfind("ring answer", 0) != 0) break;  // not a ring answer (a peer that left): no retry
    LOG(WARNING) << "connection to node " << to << " failed: " << why;
  }
  if (!c) return -1;
  Node dst;
  {
    std::lock_guard<std::mutex> lk(peers_mu_);
    dst = nodes_[to];
  }
  std::string head;
  std::vector<SVector<char>> host;
  const int bytes = Encode(msg, dst, &head, &host);
  std::lock_guard<std::mutex> lk(c->mu);
  // frame descriptors precede the host frame payloads, in frame order
  if (!c->Put(head.data(), head.size())) return -1;
  for (const SVector<char>& h : host)
    if (h.size() && !c->Put(h.data(), h.size())) return -1;
  return bytes;
}

SVector<char> TcpVan::MapFrame(int sender, const IpcFrame& f, uint64_t bytes) {
  const int dev = po_->device();
  CHECK_GE(dev, 0) << "an HBM frame reached a node without a GPU";
  device::Use(dev);
  const auto key = std::make_pair(sender, std::string(f.handle, kHandleBytes));
  char* base = nullptr;
  {
    std::lock_guard<std::mutex> lk(frames_mu_);
    auto it = mapped_.find(key);
    if (it != mapped_.end()) base = it->second;
  }
  if (!base) {
    void* p = nullptr;
    device::Check(psg_ipc_open(f.handle, &p), "psg_ipc_open (HBM frame of a peer process)");
    base = static_cast<char*>(p);
    std::lock_guard<std::mutex> lk(frames_mu_);
    mapped_.emplace(key, base);  // kept for the process lifetime (pooled blocks recur)
  }
  std::shared_ptr<FrameRegistry> reg = rel_;
  const uint64_t token = f.token;
  char* view = base + f.offset;
  reg->Add(view, bytes, sender, token);
  return SVector<char>(view, bytes, [reg, sender, token](char* p) { reg->Release(p, sender, token); }, f.device);
}

SVector<char> TcpVan::MapShmFrame(int sender, const ShmFrame& f, uint64_t bytes) {
  size_t size = 0;
  char* base = shm::Map(std::string(f.name, strnlen(f.name, sizeof(f.name))), &size);
  CHECK(base) << "cannot map the shared-memory frame " << f.name << " of node " << sender;
  CHECK_LE(f.offset + bytes, size) << "shared-memory frame outside its block";
  std::shared_ptr<FrameRegistry> reg = rel_;
  const uint64_t token = f.token;
  char* view = base + f.offset;
  reg->Add(view, bytes, sender, token);  // a reply may echo it back
  return SVector<char>(view, bytes, [reg, sender, token](char* p) { reg->Release(p, sender, token); });
}

void TcpVan::ReadLoop(int fd) {
  SockReader sock(fd);
  // the connection's hello: the name of the writer's ring, if any
  std::unique_ptr<Ring> ring;
  {
    uint32_t hello[2];
    if (!sock.read(hello, sizeof(hello)) || hello[0] != kHello || hello[1] > 255) {
      LOG(ERROR) << "connection without a hello; closing it";
      return;
    }
    if (hello[1]) {
      std::string name(hello[1], '\0');
      if (!sock.read(&name[0], name.size())) return;
      // PS_SHM_RING_REFUSE=1 (fault injection, tests): every ring refused
      static const bool refuse = [] {
        const char* e = std::getenv("PS_SHM_RING_REFUSE");
        return e && std::atoi(e) != 0;
      }();
      if (!refuse) ring = Ring::Map(name, false);
      // the answer the writer waits for before its first message: 'Y' the ring
      // carries the bytes, 'N' the socket does (a ring this process cannot map
      // — another /dev/shm behind the same hostname, or no room in it)
      const char ack = ring ? kRingYes : kRingNo;
      if (RingAckDelayMs() > 0) std::this_thread::sleep_for(std::chrono::milliseconds(RingAckDelayMs()));
      if (!WriteAll(fd, &ack, 1)) return;
    }
  }
  struct Source {
    SockReader& sock;
    Ring* ring;
    int fd;
    bool read(void* out, size_t n) { return ring ? ring->Read(fd, out, n) : sock.read(out, n); }
  } rd{sock, ring.get(), fd};
  int peer = Node::kEmpty;
  bool said_goodbye = false;
  while (true) {
    WireHeader wh;
    if (!ring && sock.empty()) SpinUntilReadable(fd);
    if (!rd.read(&wh, sizeof(wh))) break;
    if (wh.magic != kMagic) {
      LOG(ERROR) << "bad frame header from node " << peer << "; closing the connection";
      break;
    }
    std::string mb(wh.meta_bytes, '\0');
    if (!rd.read(&mb[0], mb.size())) break;
    stage::Scope t_recv("van.recv");
    Message msg;
    try {
      Reader r{mb.data(), mb.data() + mb.size()};
      msg.meta = GetMeta(r);
      peer = msg.meta.sender;
      struct Pending {
        uint8_t kind;
        uint64_t bytes;
        IpcFrame ipc;
        PeerFrame peer;
        ShmFrame shm;
      };
      std::vector<Pending> descs(wh.nframes);
      bool ok = true;
      for (auto& d : descs) {
        ok = ok && rd.read(&d.kind, 1) && rd.read(&d.bytes, 8);
        if (ok && d.kind == kIpcFrame) ok = rd.read(&d.ipc, sizeof(d.ipc));
        if (ok && d.kind == kPeerFrame) ok = rd.read(&d.peer, sizeof(d.peer));
        if (ok && d.kind == kShmFrame) ok = rd.read(&d.shm, sizeof(d.shm));
      }
      if (!ok) break;
      for (auto& d : descs) {
        if (d.kind == kHostFrame) {
          SVector<char> h = SVector<char>::Uninitialized(d.bytes);
          if (d.bytes && !rd.read(h.data(), d.bytes)) {
            ok = false;
            break;
          }
          msg.data.push_back(h);
        } else if (d.kind == kPeerFrame) {  // our own frame, echoed
          SVector<char> own;
          {
            std::lock_guard<std::mutex> lk(frames_mu_);
            auto it = inflight_.find(d.peer.token);
            CHECK(it != inflight_.end()) << "node " << peer << " echoed an HBM frame no longer in flight";
            own = it->second;
          }
          msg.data.push_back(own.Slice(d.peer.offset, d.peer.offset + d.bytes));
        } else if (d.kind == kShmFrame) {
          msg.data.push_back(MapShmFrame(peer, d.shm, d.bytes));
        } else {
          msg.data.push_back(MapFrame(peer, d.ipc, d.bytes));
        }
      }
      if (!ok) break;
      if (msg.meta.control.cmd == Control::TERMINATE) said_goodbye = true;
      Dispatch(msg);
    } catch (const std::exception& e) {
      cluster::Abort(std::string("receive from node ") + std::to_string(peer) + ": " + e.what());
    }
  }
  if (!said_goodbye && !stopping_ && !cluster::Aborted() && peer != Node::kEmpty) {
    bool known_gone;
    {
      std::lock_guard<std::mutex> lk(peers_mu_);
      known_gone = terminated_.count(peer) > 0;
    }
    if (!known_gone) cluster::Abort("node " + std::to_string(peer) + " disconnected");
  }
}

void TcpVan::Dispatch(Message& msg) {
  switch (msg.meta.control.cmd) {
    case Control::EMPTY:
      CHECK_NE(msg.meta.app_id, Meta::kEmpty);
      cluster::DeliverTo(po_, msg);
      return;
    case Control::ADD_NODE: OnAddNode(msg); return;
    case Control::BARRIER: OnBarrier(msg); return;
    case Control::GROUP_BCAST: OnGroupBroadcast(msg); return;
    case Control::STARTED: {
      std::lock_guard<std::mutex> lk(bar_mu_);
      started_[msg.meta.customer_id].insert(msg.meta.sender);
      return;
    }
    case Control::RELEASE_FRAME: {
      Reader r{msg.meta.body.data(), msg.meta.body.data() + msg.meta.body.size()};
      std::vector<SVector<char>> drop;  // released outside the lock
      std::lock_guard<std::mutex> lk(frames_mu_);
      while (r.p < r.e) {
        auto it = inflight_.find(r.pod<uint64_t>());
        if (it != inflight_.end()) {
          drop.push_back(std::move(it->second));
          inflight_.erase(it);
        }
      }
      return;
    }
    case Control::ABORT: {
      const std::string why = msg.meta.body;
      if (is_scheduler_) {
        abort_sent_ = false;  // forward it to everyone else
        NotifyAbort(why);
      }
      abort_sent_ = true;
      cluster::Abort(why);
      return;
    }
    case Control::TERMINATE: {
      std::lock_guard<std::mutex> lk(peers_mu_);
      terminated_.insert(msg.meta.sender);
      return;
    }
    default: return;  // ACK / HEARTBEAT: not used in one host
  }
}

void TcpVan::ReleaseLoop() {
  std::shared_ptr<FrameRegistry> rq = rel_;
  while (true) {
    std::vector<std::pair<int, uint64_t>> batch;
    {
      std::unique_lock<std::mutex> lk(rq->mu);
      rq->cv.wait(lk, [&] { return rq->closed || !rq->q.empty(); });
      if (rq->q.empty() && rq->closed) return;
      batch.swap(rq->q);
    }
    std::map<int, Writer> by_owner;
    for (auto& t : batch) by_owner[t.first].pod<uint64_t>(t.second);
    for (auto& kv : by_owner) SendControl(kv.first, Control::RELEASE_FRAME, 0, 0, kv.second.b);
  }
}

void TcpVan::Stop() {
  if (!started_van_ || stopping_.exchange(true)) return;
  ready_ = false;
  if (const char* e = std::getenv("PS_VAN_STATS"); e && std::atoi(e) != 0)
    std::fprintf(stderr, "van stats node %d: frames sent host=%llu hbm-ipc=%llu echoed=%llu shm=%llu\n",
                 my_node_.id, (unsigned long long)sent_kind_[kHostFrame].load(),
                 (unsigned long long)sent_kind_[kIpcFrame].load(), (unsigned long long)sent_kind_[kPeerFrame].load(),
                 (unsigned long long)sent_kind_[kShmFrame].load());
  {
    std::lock_guard<std::mutex> lk(rel_->mu);
    rel_->closed = true;
  }
  rel_->cv.notify_all();
  if (release_thread_.joinable()) release_thread_.join();
  std::map<int, std::shared_ptr<Conn>> conns;
  {
    std::lock_guard<std::mutex> lk(peers_mu_);
    conns.swap(conns_);
  }
  for (auto& kv : conns) {  // goodbye: the peer's reader then expects the close
    Message bye;
    bye.meta.control.cmd = Control::TERMINATE;
    bye.meta.sender = my_node_.id;
    std::string head;
    std::vector<SVector<char>> host;
    Encode(bye, Node(), &head, &host);
    std::lock_guard<std::mutex> lk(kv.second->mu);
    kv.second->Put(head.data(), head.size());
    ::shutdown(kv.second->fd, SHUT_RDWR);
  }
  if (listen_fd_ >= 0) {
    ::shutdown(listen_fd_, SHUT_RDWR);
    ::close(listen_fd_);
  }
  if (accept_thread_.joinable()) accept_thread_.join();
  std::vector<std::thread> readers;
  {
    std::lock_guard<std::mutex> lk(readers_mu_);
    for (int fd : reader_fds_) ::shutdown(fd, SHUT_RDWR);
    readers.swap(readers_);
  }
  for (auto& t : readers) t.join();
  {
    std::lock_guard<std::mutex> lk(readers_mu_);
    for (int fd : reader_fds_) ::close(fd);
    reader_fds_.clear();
  }
  {
    std::lock_guard<std::mutex> lk(frames_mu_);
    inflight_.clear();
  }
  shm::UnlinkAll();  // peers have mapped what they use; names go, mappings stay
}

// ---------------------------------------------------------------------------
PostOffice* g_node = nullptr;

Node::Role ParseRole(const std::string& r) {
  if (r == "scheduler") return Node::SCHEDULER;
  if (r == "server") return Node::SERVER;
  return Node::WORKER;
}

bool IsRole(const char* s) {
  return s && (!std::strcmp(s, "scheduler") || !std::strcmp(s, "server") || !std::strcmp(s, "worker"));
}

}  // namespace

Van* NewTcpVan(PostOffice* po) { return new TcpVan(po); }

namespace proc {

bool Active() { return g_node != nullptr; }
PostOffice* Node() { return g_node; }

const char* RoleOf(int argc, char** argv) {
  if (argc >= 4 && IsRole(argv[3])) return argv[3];
  const char* env = std::getenv("PS_ROLE");
  if (IsRole(env) && argc >= 2 && argc <= 3) return env;
  return nullptr;
}

// A node process that faults prints where (addresses; addr2line resolves
// them against the binary) before it dies, so a crash in a multi-process job
// names its frame instead of surfacing only as "node N disconnected".
static void FatalSignal(int sig) {
  char msg[64];
  const int n = std::snprintf(msg, sizeof(msg), "[node %d] fatal signal %d; backtrace:\n", (int)getpid(), sig);
  if (n > 0) (void)!::write(2, msg, (size_t)n);
  void* frames[48];
  const int k = ::backtrace(frames, 48);
  ::backtrace_symbols_fd(frames, k, 2);
  ::signal(sig, SIG_DFL);
  ::raise(sig);
}

// A node asked where it is (SIGQUIT: the launcher's job deadline, or a person)
// prints the stack of EVERY thread: the receiving thread signals each thread
// of the process (/proc/self/task) with SIGUSR2, whose handler prints its own
// backtrace under a spin lock, one thread at a time; then the process goes on.
static std::atomic<int> g_dump_lock{0};
static void DumpOwnStack(int) {
  while (g_dump_lock.exchange(1, std::memory_order_acquire)) {
  }
  // "[thread <tid>]:" formatted by hand (no stdio in a handler)
  char msg[40] = "[thread ";
  int n = 8;
  char digits[12];
  int nd = 0;
  for (long t = (long)::syscall(SYS_gettid); t > 0 && nd < 12; t /= 10) digits[nd++] = (char)('0' + t % 10);
  while (nd > 0) msg[n++] = digits[--nd];
  msg[n++] = ']';
  msg[n++] = ':';
  msg[n++] = '\n';
  (void)!::write(2, msg, (size_t)n);
  void* frames[48];
  const int k = ::backtrace(frames, 48);
  ::backtrace_symbols_fd(frames, k, 2);
  g_dump_lock.store(0, std::memory_order_release);
}
// Lists the threads with raw open / getdents64 / close system calls (no
// opendir / readdir: they allocate, and the interrupted thread may hold the
// malloc lock), and parses each name by hand.
static void DumpAllStacks(int) {
  static const char kHead[] = "[node] SIGQUIT: stacks of every thread follow\n";
  (void)!::write(2, kHead, sizeof(kHead) - 1);
  const int fd = (int)::syscall(SYS_open, "/proc/self/task", O_RDONLY | O_DIRECTORY);
  if (fd < 0) return;
  alignas(8) char buf[4096];
  const int pid = (int)::syscall(SYS_getpid);
  for (;;) {
    const long got = ::syscall(SYS_getdents64, fd, buf, sizeof(buf));
    if (got <= 0) break;
    for (long off = 0; off < got;) {
      // struct linux_dirent64: ino 8, off 8, reclen 2, type 1, name
      unsigned short reclen;
      std::memcpy(&reclen, buf + off + 16, sizeof(reclen));
      const char* name = buf + off + 19;
      int tid = 0;
      bool digits = *name != '\0';
      for (const char* c = name; *c; ++c) {
        if (*c < '0' || *c > '9') {
          digits = false;
          break;
        }
        tid = tid * 10 + (*c - '0');
      }
      if (digits && tid > 0) ::syscall(SYS_tgkill, pid, tid, SIGUSR2);
      off += reclen;
    }
  }
  ::syscall(SYS_close, fd);
}

int RunNode(const std::function<int(int, char**)>& node_main, int argc, char** argv) {
  const char* role = RoleOf(argc, argv);
  CHECK(role) << "process mode needs a role (argv[3] or PS_ROLE)";
  for (int sig : {SIGSEGV, SIGBUS, SIGFPE, SIGILL}) ::signal(sig, FatalSignal);
  // the stack dump only when the job has a deadline (the launcher's
  // PS_JOB_TIMEOUT_S) or PS_STACK_DUMP=1 asks for it: otherwise a drop-in
  // application's own SIGQUIT / SIGUSR2 handlers stay as it set them
  const char* jt = std::getenv("PS_JOB_TIMEOUT_S");
  const char* sd = std::getenv("PS_STACK_DUMP");
  if ((jt && std::atoi(jt) > 0) || (sd && std::atoi(sd) != 0)) {
    void* warm[2];
    (void)::backtrace(warm, 2);  // loads libgcc's unwinder now, not inside a handler
    ::signal(SIGUSR2, DumpOwnStack);
    ::signal(SIGQUIT, DumpAllStacks);
  }
  ReadLocalConfigToEnv(argv[1]);
  const Node::Role r = ParseRole(role);
  shm::Enable(r != Node::SCHEDULER);  // the scheduler sends no large frames
  const int ns = Environment::GetIntOrDefault("PS_NUM_SERVER", 1);
  const int nw = Environment::GetIntOrDefault("PS_NUM_WORKER", 1);
  g_node = new PostOffice(r, r == Node::SCHEDULER ? 0 : -1, ns, nw, -1, "tcp");
  g_node->BindThread();
  int rc = 0;
  try {
    rc = node_main(argc, argv);
  } catch (const std::exception& e) {
    rc = 1;
    cluster::Abort(std::string(role) + ": " + e.what());
  }
  if (cluster::Aborted()) rc = rc ? rc : 1;
  g_node->van()->Stop();
  // the node (and its Van's mapped frames) stays until exit: a program may still
  // hold SVectors or a KVServer whose teardown runs in static destructors
  return rc;
}

// A port for the scheduler that no node of the job can be handed: every
// server and worker listens on a kernel-chosen ephemeral port, so a port
// taken from the ephemeral range (bind to 0, then close) could go to one of
// them before the scheduler binds it — the job then fails with "ADD_NODE
// request at a non-scheduler" or "Address already in use" (seen about once in
// 20 launches with six jobs at a time).  So pick a free port BELOW the
// ephemeral range (/proc/sys/net/ipv4/ip_local_port_range); only a process
// that binds that very port explicitly could still collide.
static int SchedulerPort() {
  int eph_lo = 32768;
  if (FILE* f = std::fopen("/proc/sys/net/ipv4/ip_local_port_range", "r")) {
    int lo = 0, hi = 0;
    if (std::fscanf(f, "%d %d", &lo, &hi) == 2 && lo > 0) eph_lo = lo;
    std::fclose(f);
  }
  auto bindable = [](int port) {
    int fd = ::socket(AF_INET, SOCK_STREAM, 0);
    if (fd < 0) return false;
    sockaddr_in sa;
    Resolve("127.0.0.1", port, &sa);
    const bool ok = ::bind(fd, (sockaddr*)&sa, sizeof(sa)) == 0;
    ::close(fd);
    return ok;
  };
  const int base = 10000;
  if (eph_lo - base >= 1000) {
    std::mt19937 rng((uint32_t)getpid() ^ (uint32_t)std::chrono::steady_clock::now().time_since_epoch().count());
    for (int tries = 0; tries < 200; ++tries) {
      const int p = base + (int)(rng() % (uint32_t)(eph_lo - base));
      if (bindable(p)) return p;
    }
  }
  // no room below the ephemeral range: a kernel-chosen port (the old race)
  int fd = ::socket(AF_INET, SOCK_STREAM, 0);
  sockaddr_in sa;
  Resolve("127.0.0.1", 0, &sa);
  CHECK_EQ(::bind(fd, (sockaddr*)&sa, sizeof(sa)), 0);
  socklen_t len = sizeof(sa);
  getsockname(fd, (sockaddr*)&sa, &len);
  ::close(fd);
  return ntohs(sa.sin_port);
}

int Launch(int num_servers, int num_workers, int argc, char** argv) {
  CHECK_GT(num_servers, 0);
  CHECK_GT(num_workers, 0);
  const int port = SchedulerPort();
  const char* tmp = std::getenv("TMPDIR");
  std::string dir = std::string(tmp && *tmp ? tmp : "/tmp") + "/ps_procs_XXXXXX";
  std::vector<char> dbuf(dir.begin(), dir.end());
  dbuf.push_back(0);
  CHECK(mkdtemp(dbuf.data())) << "mkdtemp " << dir;
  dir = dbuf.data();
  // per-role config files as local.py writes them (local.py:61-85), each
  // written once, completely, before any node starts: rewriting a role's file
  // for every node of that role truncated it under a node already reading it,
  // which then fell back to the default PS_SCHEDULER_PORT (8000) and retried
  // a port nobody listens on until the job timed out (the hang
  // test_dropin_connection_processes[2-3] showed about once in 4-50 launches)
  auto cfg_path = [&](const char* role) { return dir + "/config_" + role + ".json"; };
  for (const char* role : {"scheduler", "server", "worker"}) {
    const std::string path = cfg_path(role), tmp_path = path + ".tmp";
    {
      std::ofstream f(tmp_path);
      f << "{\n  \"PS_NUM_SERVER\": " << num_servers << ",\n  \"PS_NUM_WORKER\": " << num_workers
        << ",\n  \"PS_ROLE\": \"" << role << "\",\n  \"PS_SCHEDULER_URI\": \"127.0.0.1\",\n"
        << "  \"PS_SCHEDULER_PORT\": " << port << ",\n  \"PS_VAN_TYPE\": \"tcp\"\n}\n";
      CHECK(f.good()) << "writing " << tmp_path;
    }
    CHECK_EQ(std::rename(tmp_path.c_str(), path.c_str()), 0) << "rename " << tmp_path;
  }
  char exe[4096];
  ssize_t n = readlink("/proc/self/exe", exe, sizeof(exe) - 1);
  CHECK_GT(n, 0) << "readlink /proc/self/exe";
  exe[n] = 0;
  std::vector<pid_t> pids;
  std::vector<std::string> logs;
  auto spawn = [&](const char* role, int i) {
    std::vector<std::string> args = {argv[0], cfg_path(role), dir + "/log_" + role + std::to_string(i) + ".txt", role};
    for (int k = 1; k < argc; ++k) args.push_back(argv[k]);
    std::vector<char*> av;
    for (auto& a : args) av.push_back(&a[0]);
    av.push_back(nullptr);
    pid_t pid;
    int rc = posix_spawn(&pid, exe, nullptr, nullptr, av.data(), environ);
    CHECK_EQ(rc, 0) << "posix_spawn " << exe << ": " << std::strerror(rc);
    pids.push_back(pid);
    logs.push_back(args[2]);
  };
  spawn("scheduler", 0);
  for (int i = 0; i < num_servers; ++i) spawn("server", i);
  for (int i = 0; i < num_workers; ++i) spawn("worker", i);
  // wait; once a node failed, give the others (which get the ABORT) 30 s.
  // PS_JOB_TIMEOUT_S: a job still running then is hung — every node prints
  // the stacks of all its threads (SIGQUIT, DumpAllStacks), then all are killed
  int rc = 0;
  size_t left = pids.size();
  std::vector<char> reaped(pids.size(), 0);  // waitpid has returned it: never signal that pid again
  auto failed_at = std::chrono::steady_clock::time_point::max();
  const int job_timeout_s = Environment::GetIntOrDefault("PS_JOB_TIMEOUT_S", 0);
  auto job_deadline = job_timeout_s > 0 ? std::chrono::steady_clock::now() + std::chrono::seconds(job_timeout_s)
                                              : std::chrono::steady_clock::time_point::max();
  while (left) {
    if (std::chrono::steady_clock::now() > job_deadline) {
      std::fprintf(stderr, "[launcher] job still running after PS_JOB_TIMEOUT_S=%d s: stacks of every node follow\n",
                   job_timeout_s);
      for (size_t k = 0; k < pids.size(); ++k) {  // one node at a time: their dumps share stderr
        if (reaped[k]) continue;  // (its pid may belong to another process by now)
        kill(pids[k], SIGQUIT);
        std::this_thread::sleep_for(std::chrono::milliseconds(500));
      }
      for (size_t k = 0; k < pids.size(); ++k)
        if (!reaped[k]) kill(pids[k], SIGKILL);
      rc = 124;
      failed_at = std::chrono::steady_clock::time_point::max();
      job_deadline = std::chrono::steady_clock::time_point::max();
    }
    int status = 0;
    pid_t p = waitpid(-1, &status, WNOHANG);
    if (p > 0) {
      --left;
      const bool bad = !WIFEXITED(status) || WEXITSTATUS(status) != 0;
      size_t k = 0;
      while (k < pids.size() && pids[k] != p) ++k;
      if (k < reaped.size()) reaped[k] = 1;
      if (WIFSIGNALED(status)) {
        std::fprintf(stderr, "[launcher] node process %d (%s) killed by signal %d\n", (int)p,
                     k < logs.size() ? logs[k].c_str() : "?", WTERMSIG(status));
      }
      if (bad && !rc) {
        rc = 1;
        failed_at = std::chrono::steady_clock::now();
      }
      continue;
    }
    if (p < 0 && errno != EINTR) break;
    if (rc && std::chrono::steady_clock::now() - failed_at > std::chrono::seconds(30)) {
      for (size_t k = 0; k < pids.size(); ++k)
        if (!reaped[k]) kill(pids[k], SIGKILL);
      failed_at = std::chrono::steady_clock::time_point::max();
    }
    std::this_thread::sleep_for(std::chrono::milliseconds(5));
  }
  for (pid_t q : pids) shm::UnlinkOf((int)q);  // what a crashed node left in /dev/shm
  for (const char* r : {"scheduler", "server", "worker"}) std::remove((dir + "/config_" + r + ".json").c_str());
  if (!std::getenv("PS_KEEP_LOGS")) {
    for (auto& l : logs) std::remove(l.c_str());
    rmdir(dir.c_str());
  }
  return rc;
}

}  // namespace proc
}  // namespace ps
