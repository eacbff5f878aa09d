// ps_main.cc — the local launcher: links under a PS program whose main() was
// compiled as ps_user_main (-Dmain=ps_user_main) and runs one scheduler,
// -ns servers and -nw workers of it as node threads of this process, each
// with the argv tests/local.py gives a node process (local.py:96-114).
//   ./prog [-ns N] [-nw M] [program args...]
// Defaults: PS_NUM_SERVER / PS_NUM_WORKER from the environment, else 1 / 1.
#include <cstdlib>
#include <cstring>
#include <vector>

#include "internal/PostOffice.h"

int ps_user_main(int argc, char** argv);

int main(int argc, char** argv) {
  const char* es = std::getenv("PS_NUM_SERVER");
  const char* ew = std::getenv("PS_NUM_WORKER");
  int ns = es ? std::atoi(es) : 1;
  int nw = ew ? std::atoi(ew) : 1;
  std::vector<char*> rest{argv[0]};
  for (int i = 1; i < argc; ++i) {
    if ((!std::strcmp(argv[i], "-ns") || !std::strcmp(argv[i], "--num-servers")) && i + 1 < argc)
      ns = std::atoi(argv[++i]);
    else if ((!std::strcmp(argv[i], "-nw") || !std::strcmp(argv[i], "--num-workers")) && i + 1 < argc)
      nw = std::atoi(argv[++i]);
    else
      rest.push_back(argv[i]);
  }
  rest.push_back(nullptr);
  return ps::RunLocalCluster(ns, nw, ps_user_main, (int)rest.size() - 1, rest.data());
}
