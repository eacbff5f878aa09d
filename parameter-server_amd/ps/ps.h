// ps/ps.h — the one header a PS program includes (reference src/ps/PS.h:24-125).
#pragma once
#include <cstdlib>
#include <functional>
#include <iostream>

#include "internal/Env.h"
#include "internal/PostOffice.h"
#include "ps/base.h"
#include "ps/kv_app.h"
#include "ps/simple_app.h"

namespace ps {

/* Start the system; blocks until every node started (PS.h:34-36). */
inline void Start(int customer_id, const char* config_filename, const char* log_filename = nullptr) {
  PostOffice::Get()->Start(customer_id, config_filename, log_filename, true);
}

/* argv = {program, config, [log], ...} (PS.h:38-53).  A thread the program
 * spawned itself is bound to its node by this argv (internal/PostOffice.h). */
inline void Start(int customer_id, int argc, char* argv[]) {
  if (argc < 2) {
    std::cout << "param error:\n"
              << "usage: " << argv[0] << " config_filename [log_filename] [args...]\n";
    std::exit(0);
  }
  if (!PostOffice::GetIfBound()) {
    PostOffice* po = cluster::NodeByArgv(argv);
    CHECK(po) << "ps::Start on a thread of no node: run the program under a ps launcher "
                 "(ps::RunLocalCluster / ps_launch)";
    po->BindThread();
  }
  ps::Start(customer_id, argv[1], argc > 2 ? argv[2] : nullptr);
}

/* Start without the closing barrier (PS.h:61-63). */
inline void StartAsync(int customer_id, const char* config_filename, const char* log_filename = nullptr) {
  PostOffice::Get()->Start(customer_id, config_filename, log_filename, false);
}

/* Leave the system; with need_barrier, wait for every node (PS.h:71-73). */
inline void Finalize(int customer_id, bool need_barrier = true) {
  PostOffice::Get()->Finalize(customer_id, need_barrier);
}

inline void Barrier(int customer_id, int group_id) { PostOffice::Get()->Barrier(customer_id, group_id); }
inline void RegisterExitCallback(const std::function<void()>& cb) { PostOffice::Get()->RegisterExitCallback(cb); }
inline int NumWorkers() { return PostOffice::Get()->num_workers(); }
inline int NumServers() { return PostOffice::Get()->num_servers(); }
inline bool IsWorker() { return PostOffice::Get()->is_worker(); }
inline bool IsServer() { return PostOffice::Get()->is_server(); }
inline bool IsScheduler() { return PostOffice::Get()->is_scheduler(); }
inline int MyRank() { return PostOffice::Get()->my_rank(); }

}  // namespace ps
