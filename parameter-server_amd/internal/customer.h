// internal/customer.h — per-app receive thread and request tracker (reference
// src/internal/Customer.{h,cpp}, ThreadsafePQueue.h).
//
// One receive thread per app object runs the app's handle for every incoming
// message in priority order (FIFO among equal priorities — the reference's
// `<=` comparator is not a strict weak ordering), then,
// for a response, bumps the request tracker (the handle runs BEFORE the bump,
// Customer.cpp:58-67, which KVWorker::OnReceive relies on).
#pragma once
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <functional>
#include <memory>
#include <mutex>
#include <queue>
#include <thread>
#include <vector>

#include "internal/message.h"

namespace ps {

class PostOffice;

/* Spin up to PS_SPIN_US microseconds (default 250) for `ready` before the
 * caller blocks on its condition variable: a request's round trip crosses
 * three thread hand-offs (worker -> server queue, server -> worker queue,
 * worker receive thread -> waiting caller) and a futex wake-up costs more
 * than the GPU work of a small request.  The bound covers a keyed request's
 * device time (~50 us at 10 M keys): a waiter that stops spinning before the
 * reply arrives pays the wake-up on top (tests/harness/kv_latency_host.cpp,
 * LAT_WORK_US=50: 56 us per request at 250 against 69 at 50 in one process,
 * 61 against 109 across two). */
int SpinMicros();
template <typename Pred>
bool SpinFor(Pred ready) {
  const int us = SpinMicros();
  if (us <= 0) return ready();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0;; ++i) {
    if (ready()) return true;
    if ((i & 63) == 63 && std::chrono::steady_clock::now() - t0 > std::chrono::microseconds(us)) return false;
    __builtin_ia32_pause();
  }
}

class ThreadsafePQueue {
 public:
  void Push(Message msg) {
    {
      std::lock_guard<std::mutex> lk(mu_);
      msg.meta.seq = next_seq_++;
      queue_.push(std::move(msg));
      size_.store(queue_.size(), std::memory_order_release);
    }
    cv_.notify_one();
  }
  /* the message WaitAndPop would return next, popped only when take(it) says
   * so; never waits (a server draining a run of queued Pushes) */
  template <typename Pred>
  bool PopIf(Pred take, Message* out, bool* refused = nullptr) {
    if (refused) *refused = false;
    if (size_.load(std::memory_order_acquire) == 0) return false;
    std::lock_guard<std::mutex> lk(mu_);
    if (queue_.empty()) return false;
    if (!take(queue_.top())) {
      if (refused) *refused = true;  // the head is there and may not be taken
      return false;
    }
    *out = queue_.top();
    queue_.pop();
    size_.store(queue_.size(), std::memory_order_release);
    return true;
  }
  size_t Size() const { return size_.load(std::memory_order_acquire); }
  Message WaitAndPop() {
    SpinFor([this] { return size_.load(std::memory_order_acquire) > 0; });
    std::unique_lock<std::mutex> lk(mu_);
    cv_.wait(lk, [this] { return !queue_.empty(); });
    Message m = queue_.top();
    queue_.pop();
    size_.store(queue_.size(), std::memory_order_release);
    return m;
  }

 private:
  struct Cmp {
    bool operator()(const Message& a, const Message& b) const {
      if (a.meta.priority != b.meta.priority) return a.meta.priority < b.meta.priority;
      return a.meta.seq > b.meta.seq;
    }
  };
  std::mutex mu_;
  std::condition_variable cv_;
  std::atomic<size_t> size_{0};
  uint64_t next_seq_ = 0;
  std::priority_queue<Message, std::vector<Message>, Cmp> queue_;
};

class Customer {
 public:
  using ReceiveHandle = std::function<void(const Message& received)>;

  Customer(int app_id, int customer_id, const ReceiveHandle& handle);
  ~Customer();
  Customer(const Customer&) = delete;
  Customer& operator=(const Customer&) = delete;

  /* new request to `receiver` (a node id or group): tracker entry expects one
   * response per node (Customer.cpp:22-27) */
  int NewRequest(int receiver);
  void WaitRequest(int request_id);
  int GetResponse(int request_id);
  void AddResponse(int request_id, int cnt = 1);
  /* cnt more responses to wait for (a request re-sent in pieces) */
  void ExpectMore(int request_id, int cnt);
  int NumExpected(int request_id);
  /* called by the Van for every data message to this customer */
  void OnReceive(const Message& received) { receive_queue_.Push(received); }
  /* From the receive thread's handle: take the next queued message if take(it)
   * — exactly the one the thread would handle next, so the order of handling
   * is unchanged (a KVServer serving a run of queued Pushes in one pass). */
  template <typename Pred>
  bool TakeQueued(Pred take, Message* out, bool* refused = nullptr) {
    return receive_queue_.PopIf(take, out, refused);
  }
  /* messages waiting in the receive queue (a hint: it may change at once) */
  size_t Queued() const { return receive_queue_.Size(); }

  int app_id() const { return app_id_; }
  int customer_id() const { return customer_id_; }
  PostOffice* post_office() const { return po_; }

 private:
  void ReceiveThread();

  int app_id_;
  int customer_id_;
  PostOffice* po_;
  ReceiveHandle receive_handle_;
  ThreadsafePQueue receive_queue_;
  std::unique_ptr<std::thread> receive_thread_;
  // tracker_[ts] = (expected responses, received responses)
  std::vector<std::pair<int, int>> tracker_;
  std::condition_variable tracker_cond_;
  std::mutex tracker_mu_;
  std::atomic<uint64_t> completions_{0};  // requests completed so far (spin target)
};

}  // namespace ps
