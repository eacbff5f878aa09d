// crash_node.cpp — failure handling of process mode: after the start barrier,
// worker 0 dies without a goodbye (std::_Exit, like a crash); every other
// process must notice the dropped connection, abort its waits and exit
// non-zero instead of hanging in the final barrier.
// usage: crash_node -ns S -nw W -procs
#include <cstdlib>

#include "ps/ps.h"

using namespace ps;

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  if (IsWorker() && MyRank() == 0) std::_Exit(3);
  Finalize(0, true);
  return 0;
}
