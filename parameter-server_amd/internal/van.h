// internal/van.h — the transport seam (reference src/internal/Van.h:25-111).
//
// The reference's Van moves protobuf-framed ZeroMQ multipart messages between
// processes (ZMQVan.cpp:147-248).  On one MI355X node this runtime keeps every
// node of the job in one process, one thread per node, so a Van hands the
// Message — frames included, host or HBM, zero-copy — straight to the
// receiver's Customer queue.  HBM frames stay where they are: the receiving
// node's kernels read them over xGMI (peer access is enabled between all GPUs
// at start-up).  Selected by PS_VAN_TYPE ("local", the default).
#pragma once
#include <atomic>
#include <memory>
#include <string>

#include "internal/message.h"

namespace ps {

class PostOffice;

class Van {
 public:
  static Van* Create(const std::string& type, PostOffice* po);
  virtual ~Van() = default;

  virtual void Start(int customer_id);
  virtual void Stop();
  /* send a message; fills meta.sender; returns bytes sent (Van.cpp:170-179) */
  int Send(const Message& msg);
  const Node& my_node() const { return my_node_; }
  bool IsReady() const { return ready_.load(); }
  int GetAvailableTimestamp() { return timestamp_++; }

  /* Process mode (one node per process, src/tcp_van.cc): the barrier runs
   * through the scheduler (Van.cpp:187-220) and returns true; the local Van
   * returns false and the in-process cluster barrier is used. */
  virtual bool Barrier(int customer_id, int group) {
    (void)customer_id;
    (void)group;
    return false;
  }
  /* a customer of this node called Start (the scheduler counts customer-c
   * barriers over the nodes where customer c exists) */
  virtual void NoteStarted(int customer_id) { (void)customer_id; }
  /* tell the other processes the job failed (their waiters then throw) */
  virtual void NotifyAbort(const std::string& why) { (void)why; }
  /* process mode: every node of `group` calls it; all get the bytes the
   * group's root (its lowest node id) passed.  Returns false on the local Van. */
  virtual bool GroupBroadcast(int group, const std::string& mine, std::string* out) {
    (void)group;
    (void)mine;
    (void)out;
    return false;
  }
  uint64_t send_bytes() const { return send_bytes_.load(); }
  uint64_t receive_bytes() const { return receive_bytes_.load(); }
  void CountReceived(uint64_t b) { receive_bytes_ += b; }

 protected:
  explicit Van(PostOffice* po);
  /* deliver to the receiver; returns bytes or -1 */
  virtual int SendMsg(const Message& msg) = 0;

  PostOffice* po_;
  Node my_node_;
  std::atomic<bool> ready_{false};
  std::atomic<int> timestamp_{0};
  std::atomic<uint64_t> send_bytes_{0};
  std::atomic<uint64_t> receive_bytes_{0};

  friend class PostOffice;
};

/* the process-mode Van (src/tcp_van.cc) */
Van* NewTcpVan(PostOffice* po);

}  // namespace ps
