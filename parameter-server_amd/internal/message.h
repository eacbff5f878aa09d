// internal/message.h — the in-memory message (reference src/internal/Message.h,
// Node.h).  Frame 0 = keys, 1 = vals, 2 = lens for a KV request
// (KVApp.h:610-616); frames may be host or HBM arrays (SVector::device()).
#pragma once
#include <climits>
#include <cstdint>
#include <sstream>
#include <string>
#include <vector>

#include "ps/svector.h"

namespace ps {

enum class DataType { CHAR, INT8, INT16, INT32, INT64, UINT8, UINT16, UINT32, UINT64, FLOAT, DOUBLE, HALF, OTHER };

template <typename V>
constexpr DataType GetDataType() {
  if constexpr (std::is_same<V, char>::value) return DataType::CHAR;
  else if constexpr (std::is_same<V, int8_t>::value) return DataType::INT8;
  else if constexpr (std::is_same<V, int16_t>::value) return DataType::INT16;
  else if constexpr (std::is_same<V, int32_t>::value) return DataType::INT32;
  else if constexpr (std::is_same<V, int64_t>::value) return DataType::INT64;
  else if constexpr (std::is_same<V, uint8_t>::value) return DataType::UINT8;
  else if constexpr (std::is_same<V, uint16_t>::value) return DataType::UINT16;
  else if constexpr (std::is_same<V, uint32_t>::value) return DataType::UINT32;
  else if constexpr (std::is_same<V, uint64_t>::value) return DataType::UINT64;
  else if constexpr (std::is_same<V, float>::value) return DataType::FLOAT;
  else if constexpr (std::is_same<V, double>::value) return DataType::DOUBLE;
  else return DataType::OTHER;
}

struct Node {
  enum Role { SERVER, WORKER, SCHEDULER };
  static constexpr int kEmpty = INT_MAX;
  Role role = SCHEDULER;
  int id = kEmpty;
  int customer_id = 0;
  std::string hostname = "local";
  int port = 0;
  bool is_recovered = false;
  bool gpu = false;  // process mode: the node can map HBM frames (it sees a GPU)
  std::string DebugString() const {
    std::ostringstream os;
    os << (role == SERVER ? "server" : role == WORKER ? "worker" : "scheduler") << "[" << id << "]";
    return os.str();
  }
};

struct Control {
  // STARTED / RELEASE_FRAME / ABORT / GROUP_BCAST are this runtime's own
  // (process mode, src/tcp_van.cc): a customer started; an HBM frame a peer
  // mapped is no longer referenced; the job failed; a group rendezvous (the
  // RCCL unique id of ps::CreateComm).
  enum Command { EMPTY, TERMINATE, ADD_NODE, BARRIER, ACK, HEARTBEAT, STARTED, RELEASE_FRAME, ABORT,
                 GROUP_BCAST };
  Command cmd = EMPTY;
  std::vector<Node> nodes;
  int barrier_group = 0;
  uint64_t msg_sig = 0;
  bool IsEmpty() const { return cmd == EMPTY; }
};

struct Meta {
  static constexpr int kEmpty = INT_MAX;
  int head = kEmpty;           // KVMeta::cmd
  int app_id = kEmpty;
  int customer_id = kEmpty;
  int timestamp = kEmpty;      // request id
  int sender = kEmpty;
  int receiver = kEmpty;
  bool request = false;
  bool push = false;
  bool pull = false;
  bool simple_app = false;
  bool hbm_handle = false;     // a reply from a server whose handle takes HBM frames
  // request: a Pull whose frame 1 is the caller's HBM output slice (the server
  // may write the values there); reply: it did, and carries no values
  bool direct_reply = false;
  // request: its slice bounds are the worker's hint from the last slice of
  // this key array, not confirmed (the servers' own checks confirm them);
  // reply: the server's handle checks every slice it is sent (may be sent one)
  bool spec_slice = false;
  // reply: a speculative slice this server refused (a key outside its range;
  // nothing applied) — the worker re-sends its keys sliced for real
  bool refused = false;
  std::string body;
  std::vector<DataType> data_type;
  Control control;
  int data_size = 0;
  int priority = 0;
  uint64_t seq = 0;            // arrival order, FIFO tie-break of the priority queue
};

struct Message {
  Meta meta;
  std::vector<SVector<char>> data;

  /* zero-copy: the frame shares the array's storage (Message.h:221-229) */
  template <typename V>
  void AddData(const SVector<V>& val) {
    CHECK_EQ(data.size(), meta.data_type.size());
    meta.data_type.push_back(GetDataType<V>());
    SVector<char> bytes(val);
    meta.data_size += static_cast<int>(bytes.size());
    data.push_back(bytes);
  }
  std::string DebugString() const {
    std::ostringstream os;
    os << "msg{ts=" << meta.timestamp << " " << meta.sender << "->" << meta.receiver
       << (meta.request ? " req" : " resp") << (meta.push ? " push" : "") << (meta.pull ? " pull" : "")
       << " frames=" << data.size() << "}";
    return os.str();
  }
};

}  // namespace ps
