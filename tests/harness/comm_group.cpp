// comm_group.cpp — the control plane's group rendezvous and the RCCL
// communicator built on it (PostOffice::GroupBroadcast, device::CreateComm),
// in thread mode and in process mode (-procs).
//   every node: broadcasts over three groups, checks it got the root's bytes
//   with "comm" (GPU): the servers build an RCCL communicator through the
//   scheduler and run a BSP dense Push + Pull over it (psg_comm_push / _pull)
// usage: comm_group [-ns S] [-nw W] [-procs] [comm]
#include <cstdio>
#include <cstring>
#include <vector>

#include "internal/device.h"
#include "ps/ps.h"

using namespace ps;

int main(int argc, char* argv[]) {
  Start(0, argc, argv);
  const int me = PostOffice::Get()->my_id();
  for (int round = 0; round < 3; ++round) {
    for (int group : {kServerGroup + kWorkerGroup, kWorkerGroup, kAllNodes}) {
      const auto& ids = PostOffice::Get()->GetNodeIDs(group);
      bool member = false;
      int root = ids[0];
      for (int id : ids) {
        member = member || id == me;
        root = std::min(root, id);
      }
      if (!member) continue;
      const std::string mine = "root " + std::to_string(me) + " round " + std::to_string(round);
      const std::string got = PostOffice::Get()->GroupBroadcast(group, mine);
      CHECK_EQ(got, "root " + std::to_string(root) + " round " + std::to_string(round)) << "group " << group;
    }
  }
  bool comm = false;
  for (int i = 4; i < argc; ++i) comm = comm || !std::strcmp(argv[i], "comm");
  if (comm && IsServer()) {
    psg_comm* c = device::CreateComm(kServerGroup);
    int rank = -1, n = 0;
    device::Check(psg_comm_rank(c, &rank, &n), "psg_comm_rank");
    CHECK_EQ(n, NumServers());
    const uint64_t len = 1 << 20, blk = len / n;
    psg_stream s = device::ThreadStream();
    psg_store* shard = nullptr;
    device::Check(psg_store_create(PSG_STORE_DENSE, PSG_F32, rank * blk, (rank + 1) * blk, blk, &shard), "store");
    auto vals = SVector<float>::OnDevice(len, PostOffice::Get()->device());
    auto out = SVector<float>::OnDevice(len, PostOffice::Get()->device());
    auto scratch = SVector<float>::OnDevice(blk, PostOffice::Get()->device());
    device::Check(psg_fill_synth(vals.data(), len, PSG_F32, 7 + rank, 0, 0.0, 100.0, s), "fill");
    for (int r = 0; r < 2; ++r)
      device::Check(psg_comm_push(c, shard, vals.data(), len, scratch.data(), s), "psg_comm_push");
    device::Check(psg_comm_pull(c, shard, out.data(), len, s), "psg_comm_pull");
    device::Check(psg_stream_sync(s), "sync");
    // every server pushed its own synth vector twice: out = 2 * sum_w vals_w
    std::vector<float> got(len), mine(len), expect(len, 0.f);
    device::CopySync(got.data(), out.data(), len * 4, 1);
    auto tmp = SVector<float>::OnDevice(len, PostOffice::Get()->device());
    for (int w = 0; w < n; ++w) {
      device::Check(psg_fill_synth(tmp.data(), len, PSG_F32, 7 + w, 0, 0.0, 100.0, s), "fill");
      device::CopySync(mine.data(), tmp.data(), len * 4, 1);
      for (uint64_t i = 0; i < len; ++i) expect[i] += mine[i];
    }
    for (uint64_t i = 0; i < len; ++i) CHECK_EQ(got[i], 2 * expect[i]) << "i=" << i;
    psg_store_destroy(shard);
    psg_comm_destroy(c);
    std::printf("comm ok (server %d of %d)\n", rank, n);
  }
  std::printf("bcast ok %d\n", me);
  std::fflush(stdout);
  Finalize(0, true);
  return 0;
}
