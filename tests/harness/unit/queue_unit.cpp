// queue_unit.cpp — the receive queue's conditional pop, which a KVServer's
// gather window relies on (repo:internal/customer.h ThreadsafePQueue::PopIf;
// ps/kv_app.h KVServer::OnReceive): an empty queue is not a refusal, a head
// the predicate rejects is, and a message pushed while a consumer polls is
// taken by a later poll rather than ending the poll as a refusal.  Messages
// come out in priority, then arrival, order (Customer.cpp:52-70's queue).
// Plain program (no PS node): exits non-zero on a failed CHECK.
#include <atomic>
#include <cstdio>
#include <thread>

#include "internal/customer.h"

using ps::Message;
using ps::ThreadsafePQueue;

static Message Msg(int sender, int prio = 0) {
  Message m;
  m.meta.sender = sender;
  m.meta.priority = prio;
  return m;
}

int main() {
  ThreadsafePQueue q;
  Message out;
  bool refused = true;
  auto any = [](const Message&) { return true; };
  auto none = [](const Message&) { return false; };
  // empty: nothing taken, and no refusal
  CHECK(!q.PopIf(any, &out, &refused));
  CHECK(!refused);
  // a head the predicate rejects: a refusal, and the message stays
  q.Push(Msg(9));
  CHECK(!q.PopIf(none, &out, &refused));
  CHECK(refused);
  CHECK_EQ(q.Size(), 1u);
  CHECK(q.PopIf(any, &out, &refused));
  CHECK(!refused);
  CHECK_EQ(out.meta.sender, 9);
  CHECK_EQ(q.Size(), 0u);
  // priority first, then arrival
  q.Push(Msg(1));
  q.Push(Msg(2, 5));
  q.Push(Msg(3));
  int order[3];
  for (int i = 0; i < 3; ++i) {
    CHECK(q.PopIf(any, &out));
    order[i] = out.meta.sender;
  }
  CHECK_EQ(order[0], 2);
  CHECK_EQ(order[1], 1);
  CHECK_EQ(order[2], 3);
  // a producer pushing while a consumer polls: every poll that takes nothing
  // is an empty queue (never a refusal), and every message is taken
  constexpr int kMsgs = 20000;
  std::atomic<bool> go{false};
  std::thread producer([&] {
    while (!go.load()) {
    }
    for (int i = 0; i < kMsgs; ++i) q.Push(Msg(i));
  });
  go = true;
  int taken = 0, last = -1;
  while (taken < kMsgs) {
    bool r = true;
    if (q.PopIf(any, &out, &r)) {
      CHECK_GT(out.meta.sender, last);
      last = out.meta.sender;
      ++taken;
    } else {
      CHECK(!r) << "an accepting predicate was reported as a refusal";
    }
  }
  producer.join();
  CHECK_EQ(q.Size(), 0u);
  std::printf("queue ok\n");
  return 0;
}
