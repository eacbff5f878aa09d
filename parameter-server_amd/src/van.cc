// van.cc — Van base (reference src/internal/Van.cpp:23-179) and the local Van.
#include "internal/van.h"

#include "internal/PostOffice.h"

namespace ps {

namespace {
// Hands messages to the receiver node's Customer in this process: frames are
// shared, never copied (host or HBM).
class LocalVan : public Van {
 public:
  explicit LocalVan(PostOffice* po) : Van(po) {}

 protected:
  int SendMsg(const Message& msg) override {
    cluster::Deliver(msg);
    return (int)sizeof(Meta) + msg.meta.data_size;
  }
};
}  // namespace

Van* Van::Create(const std::string& type, PostOffice* po) {
  if (type == "local" || type.empty()) return new LocalVan(po);
  if (type == "tcp") return NewTcpVan(po);
  LOG(FATAL) << "PS_VAN_TYPE \"" << type << "\" is not available: \"local\" (every node a thread of "
             << "one process) or \"tcp\" (one node per process)";
  return nullptr;
}

Van::Van(PostOffice* po) : po_(po) {
  my_node_.role = po->role();
  my_node_.id = po->my_id();
}

void Van::Start(int customer_id) {
  (void)customer_id;
  ready_ = true;
}

void Van::Stop() { ready_ = false; }

int Van::Send(const Message& msg) {
  Message m = msg;
  m.meta.sender = my_node_.id;
  int n = SendMsg(m);
  CHECK_NE(n, -1) << "send failed: " << m.DebugString();
  send_bytes_ += (uint64_t)n;
  return n;
}

}  // namespace ps
