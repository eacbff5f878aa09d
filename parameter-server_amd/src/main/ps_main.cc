// ps_main.cc — the launcher: links under a PS program whose main() symbol
// was renamed ps_user_main in its object file (objcopy --redefine-sym
// main=ps_user_main; see PS_BUILD in the Makefile).  Three ways to run:
//
//   ./prog config.json log.txt <role> [args]   one node of a multi-process job,
//        exactly the command line tests/local.py gives a node (local.py:87-114);
//        the nodes meet at the scheduler over TCP (src/tcp_van.cc)
//   ./prog -ns N -nw M -procs [args]           this launcher does local.py's job:
//        one scheduler, N servers and M workers as separate processes
//   ./prog [-ns N] [-nw M] [args]              every node a thread of this
//        process, frames handed over zero-copy (ps::RunLocalCluster)
//
// Defaults: PS_NUM_SERVER / PS_NUM_WORKER from the environment, else 1 / 1.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "internal/PostOffice.h"

// the program's own main(), renamed: an unmangled symbol, so C linkage here
extern "C" int ps_user_main(int argc, char** argv);

int main(int argc, char** argv) {
  if (ps::proc::RoleOf(argc, argv)) return ps::proc::RunNode(ps_user_main, argc, argv);
  const char* es = std::getenv("PS_NUM_SERVER");
  const char* ew = std::getenv("PS_NUM_WORKER");
  int ns = es ? std::atoi(es) : 1;
  int nw = ew ? std::atoi(ew) : 1;
  bool procs = false;
  std::vector<char*> rest{argv[0]};
  for (int i = 1; i < argc; ++i) {
    if ((!std::strcmp(argv[i], "-ns") || !std::strcmp(argv[i], "--num-servers")) && i + 1 < argc)
      ns = std::atoi(argv[++i]);
    else if ((!std::strcmp(argv[i], "-nw") || !std::strcmp(argv[i], "--num-workers")) && i + 1 < argc)
      nw = std::atoi(argv[++i]);
    else if (!std::strcmp(argv[i], "-procs") || !std::strcmp(argv[i], "--processes"))
      procs = true;
    else
      rest.push_back(argv[i]);
  }
  rest.push_back(nullptr);
  if (procs) return ps::proc::Launch(ns, nw, (int)rest.size() - 1, rest.data());
  return ps::RunLocalCluster(ns, nw, ps_user_main, (int)rest.size() - 1, rest.data());
}
