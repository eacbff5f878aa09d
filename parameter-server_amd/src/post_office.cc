// post_office.cc — PostOffice (reference src/internal/PostOffice.cpp), the
// in-process cluster (node table, barrier, delivery) and RunLocalCluster.
#include "internal/PostOffice.h"

#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <memory>
#include <thread>

#include "internal/Env.h"
#include "internal/device.h"

namespace ps {

namespace {
thread_local PostOffice* t_node = nullptr;

struct ClusterState {
  std::mutex mu;
  std::condition_variable cv;
  std::map<int, std::unique_ptr<PostOffice>> nodes;  // id -> node
  std::map<char**, PostOffice*> by_argv;
  struct Bar {
    uint64_t gen = 0;
    int arrived = 0;
  };
  std::map<std::pair<int, int>, Bar> bars;  // (group, customer_id)
  struct Bcast {
    uint64_t gen = 0;
    int arrived = 0;
    std::string root_bytes, result;
  };
  std::map<int, Bcast> bcasts;  // group -> rendezvous
  std::map<int, std::set<int>> started;     // node id -> customer ids that called Start
  bool configured = false;
  bool env_loaded = false;
  std::atomic<bool> aborted{false};
  std::string why;
};
ClusterState& S() {
  static ClusterState* s = new ClusterState();
  return *s;
}
}  // namespace

// ---------------------------------------------------------------------------
namespace cluster {

PostOffice* NodeById(int id) {
  ClusterState& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  auto it = s.nodes.find(id);
  return it == s.nodes.end() ? nullptr : it->second.get();
}

PostOffice* NodeByArgv(char** argv) {
  ClusterState& s = S();
  std::lock_guard<std::mutex> lk(s.mu);
  auto it = s.by_argv.find(argv);
  return it == s.by_argv.end() ? nullptr : it->second;
}

bool Configured() { return S().configured; }
bool Aborted() { return S().aborted.load(); }
std::string AbortReason() {
  std::lock_guard<std::mutex> lk(S().mu);
  return S().why;
}

void Abort(const std::string& why) {
  ClusterState& s = S();
  {
    std::lock_guard<std::mutex> lk(s.mu);
    if (!s.aborted) s.why = why;
    s.aborted = true;
  }
  s.cv.notify_all();
  LOG(ERROR) << "job aborted: " << why;
  if (proc::Active()) proc::Node()->van()->NotifyAbort(why);
}

void NoteStarted(PostOffice* po, int customer_id) {
  {
    std::lock_guard<std::mutex> lk(S().mu);
    S().started[po->my_id()].insert(customer_id);
  }
  po->van()->NoteStarted(customer_id);
}

// Barrier per (group, customer_id): customer 0 of every node in the group
// takes part in a customer-0 barrier; a barrier of customer c > 0 waits for
// the nodes of the group on which customer c has started (the reference's
// per-customer barrier_done_ flags, PostOffice.cpp:154-200).
void Barrier(PostOffice* po, int customer_id, int group) {
  const auto& ids = po->GetNodeIDs(group);
  if (ids.size() <= 1) return;
  if (po->van()->Barrier(customer_id, group)) return;  // process mode: via the scheduler
  ClusterState& s = S();
  std::unique_lock<std::mutex> lk(s.mu);
  int participants = (int)ids.size();
  if (customer_id != 0) {
    participants = 0;
    for (int id : ids) participants += s.started[id].count(customer_id) ? 1 : 0;
    participants = std::max(participants, 1);
  }
  auto& b = s.bars[{group, customer_id}];
  const uint64_t gen = b.gen;
  if (++b.arrived >= participants) {
    b.arrived = 0;
    ++b.gen;
    s.cv.notify_all();
    return;
  }
  while (b.gen == gen) {
    s.cv.wait_for(lk, std::chrono::milliseconds(100));
    if (s.aborted) {
      std::string why = s.why;
      lk.unlock();
      LOG(FATAL) << "barrier abandoned: " << why;
    }
  }
}

std::string GroupBroadcast(PostOffice* po, int group, const std::string& mine) {
  const auto& ids = po->GetNodeIDs(group);
  const int root = *std::min_element(ids.begin(), ids.end());
  if (ids.size() <= 1) return mine;
  std::string out;
  if (po->van()->GroupBroadcast(group, mine, &out)) return out;  // process mode
  ClusterState& s = S();
  std::unique_lock<std::mutex> lk(s.mu);
  auto& b = s.bcasts[group];
  if (po->my_id() == root) b.root_bytes = mine;
  const uint64_t gen = b.gen;
  if (++b.arrived >= (int)ids.size()) {
    b.arrived = 0;
    b.result = b.root_bytes;
    ++b.gen;
    s.cv.notify_all();
    return b.result;
  }
  while (b.gen == gen) {
    s.cv.wait_for(lk, std::chrono::milliseconds(100));
    if (s.aborted) {
      std::string why = s.why;
      lk.unlock();
      LOG(FATAL) << "group broadcast abandoned: " << why;
    }
  }
  return b.result;
}

void Deliver(const Message& msg) {
  PostOffice* dst = NodeById(msg.meta.receiver);
  CHECK(dst) << "no node with id " << msg.meta.receiver;
  DeliverTo(dst, msg);
}

void DeliverTo(PostOffice* dst, const Message& msg) {
  // only workers run several customers per app (Van.cpp:246-257)
  const int cid = dst->is_worker() ? msg.meta.customer_id : msg.meta.app_id;
  Customer* c = dst->GetCustomer(msg.meta.app_id, cid, 5);
  CHECK(c) << "Cannot find customer with app_id: " << msg.meta.app_id << ", customer_id: " << cid
           << " after waiting for 5s";
  dst->van()->CountReceived((uint64_t)msg.meta.data_size);
  c->OnReceive(msg);
}

}  // namespace cluster

// ---------------------------------------------------------------------------
PostOffice* PostOffice::GetIfBound() { return t_node ? t_node : (proc::Active() ? proc::Node() : nullptr); }

PostOffice* PostOffice::Get() {
  if (!t_node && proc::Active()) return proc::Node();  // one node per process
  if (!t_node)
    LOG(FATAL) << "this thread belongs to no PS node: run the program under a ps launcher "
                  "(ps::RunLocalCluster / ps_launch)";
  return t_node;
}

PostOffice::PostOffice(Node::Role role, int rank, int num_servers, int num_workers, int device,
                       const char* van_type)
    : role_(role), rank_(rank), num_servers_(num_servers), num_workers_(num_workers), device_(device) {
  id_ = role == Node::SCHEDULER ? kScheduler
        : rank < 0              ? Node::kEmpty  // process mode: assigned by the scheduler
        : role == Node::SERVER  ? ServerRankToID(rank)
                                : WorkerRankToID(rank);
  // group -> node ids (PostOffice.cpp:50-73)
  for (int i = 0; i < num_servers_; ++i) {
    int id = ServerRankToID(i);
    for (int g : {id, kServerGroup, kServerGroup + kScheduler, kServerGroup + kWorkerGroup,
                  kServerGroup + kWorkerGroup + kScheduler})
      node_ids_[g].push_back(id);
  }
  for (int i = 0; i < num_workers_; ++i) {
    int id = WorkerRankToID(i);
    for (int g : {id, kWorkerGroup, kWorkerGroup + kScheduler, kWorkerGroup + kServerGroup,
                  kWorkerGroup + kServerGroup + kScheduler})
      node_ids_[g].push_back(id);
  }
  for (int g : {kScheduler, kScheduler + kServerGroup, kScheduler + kWorkerGroup,
                kScheduler + kServerGroup + kWorkerGroup})
    node_ids_[g].push_back(kScheduler);
  const char* vt = van_type ? van_type : std::getenv("PS_VAN_TYPE");
  van_.reset(Van::Create(vt ? vt : "local", this));
}

void PostOffice::SetIdentity(int rank, int device) {
  rank_ = rank;
  id_ = role_ == Node::SCHEDULER ? kScheduler : role_ == Node::SERVER ? ServerRankToID(rank) : WorkerRankToID(rank);
  device_ = device;
}

PostOffice::~PostOffice() {
  if (van_) van_->Stop();
}

void PostOffice::BindThread() {
  t_node = this;
  device::Use(device_);
}

void PostOffice::Start(int customer_id, const char* config_filename, const char* log_filename,
                       bool need_barrier) {
  {
    std::lock_guard<std::mutex> lk(start_mu_);
    if (start_stage_ == 0) {
      ps_log::InitLogging(log_filename);
      {
        std::lock_guard<std::mutex> clk(S().mu);
        if (!S().env_loaded && config_filename) {
          S().env_loaded = true;
          ReadLocalConfigToEnv(config_filename);
        }
      }
      verbose_ = Environment::GetIntOrDefault("PS_VERBOSE", 0) > 0;
      van_->Start(customer_id);
      start_stage_ = 1;
    }
  }
  BindThread();  // process mode: the GPU is known only after registration
  cluster::NoteStarted(this, customer_id);
  if (need_barrier) Barrier(customer_id, kAllNodes);
}

void PostOffice::Finalize(int customer_id, bool need_barrier) {
  if (customer_id == 0) {
    // customer 0 tears the node down (PostOffice.cpp:99-112): first let every
    // other customer this node started finish its own Finalize
    std::unique_lock<std::mutex> lk(start_mu_);
    while (true) {
      std::set<int> started;
      {
        std::lock_guard<std::mutex> clk(S().mu);
        started = S().started[id_];
      }
      bool all = true;
      for (int c : started)
        if (c != 0 && !finalized_.count(c)) all = false;
      if (all) break;
      finalize_cv_.wait_for(lk, std::chrono::milliseconds(50));
      if (cluster::Aborted()) break;
    }
  }
  if (need_barrier) Barrier(customer_id, kAllNodes);
  if (customer_id != 0) {
    std::lock_guard<std::mutex> lk(start_mu_);
    finalized_.insert(customer_id);
    finalize_cv_.notify_all();
  } else {
    if (exit_callback_) {
      auto cb = exit_callback_;
      exit_callback_ = nullptr;
      cb();
    }
    van_->Stop();
  }
}

void PostOffice::AddCustomer(Customer* customer) {
  std::lock_guard<std::mutex> lk(customers_mu_);
  int app_id = customer->app_id(), cid = customer->customer_id();
  CHECK_EQ(customers_[app_id].count(cid), (size_t)0) << "customer_id " << cid << " already exists";
  customers_[app_id][cid] = customer;
  customers_cv_.notify_all();
}

void PostOffice::RemoveCustomer(Customer* customer) {
  std::lock_guard<std::mutex> lk(customers_mu_);
  int app_id = customer->app_id();
  customers_[app_id].erase(customer->customer_id());
  if (customers_[app_id].empty()) customers_.erase(app_id);
}

Customer* PostOffice::GetCustomer(int app_id, int customer_id, int timeout_in_sec) {
  std::unique_lock<std::mutex> lk(customers_mu_);
  auto find = [&]() -> Customer* {
    auto it = customers_.find(app_id);
    if (it == customers_.end()) return nullptr;
    auto jt = it->second.find(customer_id);
    return jt == it->second.end() ? nullptr : jt->second;
  };
  Customer* c = find();
  if (!c && timeout_in_sec > 0) {
    customers_cv_.wait_for(lk, std::chrono::seconds(timeout_in_sec), [&] { return (c = find()) != nullptr; });
  }
  return c;
}

const std::vector<int>& PostOffice::GetNodeIDs(int node_id) const {
  auto it = node_ids_.find(node_id);
  CHECK(it != node_ids_.end()) << "node " << node_id << " doesn't exist";
  return it->second;
}

const std::vector<Range>& PostOffice::GetServerRanges() {
  std::lock_guard<std::mutex> lk(ranges_mu_);
  if (server_key_ranges_.empty()) {
    for (int i = 0; i < num_servers_; ++i) {
      Key b = kMaxKey / num_servers_ * i;
      Key e = i != num_servers_ - 1 ? kMaxKey / num_servers_ * (i + 1) : kMaxKey;
      server_key_ranges_.emplace_back(b, e);
    }
  }
  return server_key_ranges_;
}

std::string PostOffice::GroupBroadcast(int node_group, const std::string& mine) {
  return cluster::GroupBroadcast(this, node_group, mine);
}

void PostOffice::Barrier(int customer_id, int node_group) {
  switch (role_) {
    case Node::SERVER: CHECK(node_group & kServerGroup); break;
    case Node::WORKER: CHECK(node_group & kWorkerGroup); break;
    case Node::SCHEDULER: CHECK(node_group & kScheduler); break;
  }
  cluster::Barrier(this, customer_id, node_group);
}

// ---------------------------------------------------------------------------
int RunLocalCluster(int num_servers, int num_workers, const std::function<int(int, char**)>& node_main,
                    int argc, char** argv) {
  CHECK_GT(num_servers, 0);
  CHECK_GT(num_workers, 0);
  ClusterState& s = S();
  {
    std::lock_guard<std::mutex> lk(s.mu);
    CHECK(!s.configured) << "one local cluster per process at a time";
    s.configured = true;
    s.aborted = false;
    s.why.clear();
    s.env_loaded = false;
    s.bars.clear();
    s.bcasts.clear();
    s.started.clear();
    s.by_argv.clear();
  }
  const int ndev = device::Count();
  if (ndev > 1) device::EnableAllPeerAccess();
  auto dev_of = [ndev](int rank) { return ndev > 0 ? rank % ndev : -1; };

  // per-role config files, as tests/local.py writes them (local.py:61-85)
  const char* tmp = std::getenv("TMPDIR");
  std::string dir = std::string(tmp && *tmp ? tmp : "/tmp") + "/ps_local_XXXXXX";
  std::vector<char> dbuf(dir.begin(), dir.end());
  dbuf.push_back(0);
  CHECK(mkdtemp(dbuf.data())) << "mkdtemp " << dir;
  dir = dbuf.data();
  auto write_cfg = [&](const char* role) {
    std::string path = dir + "/config_" + role + ".json";
    std::ofstream f(path);
    f << "{\n  \"PS_NUM_SERVER\": " << num_servers << ",\n  \"PS_NUM_WORKER\": " << num_workers
      << ",\n  \"PS_ROLE\": \"" << role << "\",\n  \"PS_SCHEDULER_URI\": \"127.0.0.1\",\n"
      << "  \"PS_SCHEDULER_PORT\": 8000,\n  \"PS_VAN_TYPE\": \"local\"\n}\n";
    return path;
  };

  struct NodeRun {
    PostOffice* po;
    std::vector<std::string> args;
    std::vector<char*> argv;
    int rc = 0;
  };
  std::vector<std::unique_ptr<NodeRun>> runs;
  auto add = [&](Node::Role role, int rank) {
    auto po = std::make_unique<PostOffice>(role, rank, num_servers, num_workers,
                                           role == Node::SCHEDULER ? (ndev ? 0 : -1) : dev_of(rank));
    auto r = std::make_unique<NodeRun>();
    r->po = po.get();
    const char* rname = role == Node::SCHEDULER ? "scheduler" : role == Node::SERVER ? "server" : "worker";
    r->args = {argv[0], write_cfg(rname), dir + "/log_" + rname + std::to_string(rank) + ".txt", rname};
    for (int i = 1; i < argc; ++i) r->args.push_back(argv[i]);
    for (auto& a : r->args) r->argv.push_back(&a[0]);
    r->argv.push_back(nullptr);
    std::lock_guard<std::mutex> lk(s.mu);
    s.by_argv[r->argv.data()] = r->po;
    s.nodes[po->my_id()] = std::move(po);
    runs.push_back(std::move(r));
  };
  add(Node::SCHEDULER, 0);
  for (int i = 0; i < num_servers; ++i) add(Node::SERVER, i);
  for (int i = 0; i < num_workers; ++i) add(Node::WORKER, i);

  std::vector<std::thread> threads;
  for (auto& r : runs) {
    NodeRun* rp = r.get();
    threads.emplace_back([rp, &node_main] {
      rp->po->BindThread();
      try {
        rp->rc = node_main((int)rp->args.size(), rp->argv.data());
      } catch (const std::exception& e) {
        rp->rc = 1;
        cluster::Abort(std::string(e.what()));
      }
    });
  }
  for (auto& t : threads) t.join();
  int rc = 0;
  for (auto& r : runs) rc = rc || r->rc;
  if (s.aborted) rc = 1;
  {
    std::lock_guard<std::mutex> lk(s.mu);
    s.by_argv.clear();
  }
  {
    std::map<int, std::unique_ptr<PostOffice>> nodes;
    {
      std::lock_guard<std::mutex> lk(s.mu);
      nodes.swap(s.nodes);
    }
    nodes.clear();
  }
  for (const char* f : {"config_scheduler.json", "config_server.json", "config_worker.json"})
    std::remove((dir + "/" + f).c_str());
  if (!std::getenv("PS_KEEP_LOGS")) {
    for (auto& r : runs) std::remove(r->args[2].c_str());
    rmdir(dir.c_str());
  }
  std::lock_guard<std::mutex> lk(s.mu);
  s.configured = false;
  return rc;
}

}  // namespace ps
