// internal/device.h — the host runtime's side of the psg C-ABI: GPU binding,
// per-thread streams, the HBM pool behind SVector::OnDevice, and the device
// forms of the slicer and the pull merge.  Every GPU operation goes through
// include/psg.h; a failed call throws ps_log::PSError with psg_last_error().
#pragma once
#include <cstdint>
#include <memory>
#include <vector>

#include "../../include/psg.h"
#include "ps/range.h"

namespace ps {
namespace device {

/* GPUs visible to this process (0 when none / no driver) */
int Count();
/* throw PSError(what + psg_last_error()) when rc != PSG_OK */
void Check(int rc, const char* what);
/* bind the calling thread to GPU dev (no-op for dev < 0) */
void Use(int dev);
/* the calling thread's stream on its current GPU (created on first use) */
psg_stream ThreadStream();
/* pooled HBM allocation (also declared in ps/svector.h) */
std::shared_ptr<void> Alloc(size_t bytes, int dev);
/* let every GPU read every other GPU's HBM (xGMI) */
void EnableAllPeerAccess();
/* kind: 0 H2D, 1 D2H, 2 D2D, 3 default; synchronises the thread stream */
void CopySync(void* dst, const void* src, size_t bytes, int kind = 3);

/* Pipelined copies between a pageable host array and HBM: chunks go through
 * two pinned staging blocks of the calling thread, so the host copy of chunk
 * c + 1 (HostCopy, several threads) runs while chunk c is on PCIe.  Return
 * when the data has landed.  Used for the host-vector forms of KVWorker's
 * Push / Pull / PushPull on a node with a GPU. */
void StageToDevice(void* dst_dev, const void* src_host, size_t bytes);
void StageToHost(void* dst_host, const void* src_dev, size_t bytes);

/* DefaultSlicer positions for a device key array (psg_slice) */
void SliceKeys(const uint64_t* keys, size_t n, const int* lens, size_t num_vals,
               const std::vector<Range>& ranges, std::vector<uint64_t>* key_pos,
               std::vector<uint64_t>* val_pos);
/* psg_merge on the thread stream, then synchronise */
void Merge(std::vector<psg_segment>* segs, int elem_size, void* dst, uint64_t dst_count);

/* An RCCL communicator (psg_comm) over the nodes of a ps group (kServerGroup,
 * kWorkerGroup, ...): this node's rank is its position in
 * PostOffice::GetNodeIDs(group).  The group's root (lowest node id) makes the
 * RCCL unique id and the control plane hands it to every member
 * (PostOffice::GroupBroadcast: through the scheduler in process mode).
 * Collective: every member calls it; one GPU per member. */
psg_comm* CreateComm(int group);

/* psg dtype of a value type (-1 if the store does not support it) */
template <typename V>
constexpr int DType() {
  if constexpr (std::is_same<V, float>::value) return PSG_F32;
  else if constexpr (std::is_same<V, double>::value) return PSG_F64;
  else return -1;
}

}  // namespace device
}  // namespace ps
