// internal/PostOffice.h — per-node roles, groups, key ranges, customers and
// barriers (reference src/internal/PostOffice.{h,cpp}).
//
// One PostOffice per node.  All nodes of a job live in one process (see
// internal/van.h); PostOffice::Get() returns the calling thread's node.  A
// node's threads are bound by the cluster launcher (ps::RunLocalCluster), by
// the Customer threads it creates, and — for threads a harness spawns itself
// (test_my.cpp, test_kv_app_multi_workers.cpp) — by the argv it passes to
// ps::Start, which identifies the node the thread belongs to.
#pragma once
#include <condition_variable>
#include <functional>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "internal/customer.h"
#include "internal/message.h"
#include "internal/van.h"
#include "ps/base.h"
#include "ps/range.h"

namespace ps {

class PostOffice {
 public:
  /* the calling thread's node (CHECK-fails on a thread bound to no node) */
  static PostOffice* Get();
  static PostOffice* GetIfBound();

  /* van_type: PS_VAN_TYPE when null ("local" by default) */
  PostOffice(Node::Role role, int rank, int num_servers, int num_workers, int device,
             const char* van_type = nullptr);
  ~PostOffice();

  void Start(int customer_id, const char* config_filename, const char* log_filename,
             bool need_barrier = true);
  void Finalize(int customer_id, bool need_barrier = true);

  void AddCustomer(Customer* customer);
  void RemoveCustomer(Customer* customer);
  /* waits up to timeout_in_sec for the customer to be created (PostOffice.cpp:138-152) */
  Customer* GetCustomer(int app_id, int customer_id, int timeout_in_sec = 0);

  /* node ids of a node id or a group (PostOffice.cpp:50-73) */
  const std::vector<int>& GetNodeIDs(int node_id) const;
  /* [kMaxKey/ns*i, kMaxKey/ns*(i+1)), last ends at kMaxKey (PostOffice.cpp:211-221) */
  const std::vector<Range>& GetServerRanges();

  void RegisterExitCallback(const std::function<void()>& cb) { exit_callback_ = cb; }
  void Barrier(int customer_id, int node_group);
  /* Every node of node_group calls it (like a barrier); each gets the bytes
   * the group's root — its lowest node id — passed as `mine`.  The control
   * plane's rendezvous for state a group shares, e.g. an RCCL unique id
   * (ps::CreateComm). */
  std::string GroupBroadcast(int node_group, const std::string& mine);

  static int ServerRankToID(int rank) { return rank * 2 + 8; }
  static int WorkerRankToID(int rank) { return rank * 2 + 9; }
  static int IDToRank(int id) { return std::max((id - 8) / 2, 0); }

  int num_workers() const { return num_workers_; }
  int num_servers() const { return num_servers_; }
  bool is_worker() const { return role_ == Node::WORKER; }
  bool is_server() const { return role_ == Node::SERVER; }
  bool is_scheduler() const { return role_ == Node::SCHEDULER; }
  bool is_recovered() const { return false; }
  int my_rank() const { return rank_; }
  int my_id() const { return id_; }
  Node::Role role() const { return role_; }
  /* GPU this node's kernels run on; -1 without a GPU */
  int device() const { return device_; }
  Van* van() const { return van_.get(); }
  bool verbose() const { return verbose_; }
  /* heartbeats are not needed in one process: nothing is ever dead */
  std::vector<int> GetDeadNodes(int t = 60) { (void)t; return {}; }
  /* set the calling thread's node (and its GPU) */
  void BindThread();
  /* process mode: the rank the scheduler assigned and the GPU it implies */
  void SetIdentity(int rank, int device);

 private:
  Node::Role role_;
  int rank_, id_;
  int num_servers_, num_workers_;
  int device_;
  bool verbose_ = false;
  std::unique_ptr<Van> van_;
  std::mutex start_mu_;
  int start_stage_ = 0;
  std::set<int> finalized_;  // customers (other than 0) past Finalize
  std::condition_variable finalize_cv_;
  std::map<int, std::vector<int>> node_ids_;
  std::mutex ranges_mu_;
  std::vector<Range> server_key_ranges_;
  std::mutex customers_mu_;
  std::condition_variable customers_cv_;
  std::unordered_map<int, std::unordered_map<int, Customer*>> customers_;
  std::function<void()> exit_callback_;
};

/* Run a job of one scheduler, num_servers servers and num_workers workers in
 * this process, each node a thread calling node_main(argc, argv) with
 * argv = {argv[0], <config.json>, <log file>, <role>, argv[1..]} — the command
 * line tests/local.py gives each process (local.py:96-114).  Returns 0 when
 * every node returned 0. */
int RunLocalCluster(int num_servers, int num_workers,
                    const std::function<int(int, char**)>& node_main, int argc, char** argv);

namespace cluster {
/* node of id (nullptr when none) */
PostOffice* NodeById(int id);
/* node whose launcher argv is argv (threads a harness spawns) */
PostOffice* NodeByArgv(char** argv);
/* barrier of (group, customer_id) across the group's nodes */
void Barrier(PostOffice* po, int customer_id, int group);
void NoteStarted(PostOffice* po, int customer_id);
std::string GroupBroadcast(PostOffice* po, int group, const std::string& mine);
void Deliver(const Message& msg);
/* hand msg to the right customer of node dst (Van.cpp:246-257) */
void DeliverTo(PostOffice* dst, const Message& msg);
/* wake every waiter with an error after a node failed */
void Abort(const std::string& why);
bool Aborted();
std::string AbortReason();
bool Configured();
}  // namespace cluster

/* Process mode: one node per OS process, as tests/local.py launches the
 * reference (local.py:87-114: argv = {prog, config.json, log, role}).  Nodes
 * find each other through the scheduler (PS_SCHEDULER_URI / _PORT) over TCP;
 * host frames travel on the socket, HBM frames as hipIpc handles that the
 * receiver maps in place (src/tcp_van.cc). */
namespace proc {
/* this process runs one node (RunNode) */
bool Active();
PostOffice* Node();
/* the role named by argv[3] or PS_ROLE ("scheduler" / "server" / "worker"), or
 * nullptr when this is not a process-mode launch */
const char* RoleOf(int argc, char** argv);
/* run node_main as the one node of this process */
int RunNode(const std::function<int(int, char**)>& node_main, int argc, char** argv);
/* local.py's job in C++: start one scheduler, num_servers servers and
 * num_workers workers of this executable as separate processes and wait */
int Launch(int num_servers, int num_workers, int argc, char** argv);
}  // namespace proc

}  // namespace ps
