// internal/shm_pool.h — host frames between processes as shared-memory mappings.
//
// In process mode (src/tcp_van.cc) a large host array (>= 1 MiB: the key /
// value frames of a Push, the values of a Pull reply) is allocated from POSIX
// shared-memory blocks instead of the heap.  A frame that lies in such a block
// is sent to a peer on the same host as (block name, offset) and the peer maps
// the block (once, cached): the frame crosses no socket and no copy, the way
// HBM frames travel as hipIpc mappings.  (PS_SHM_REGISTER=1 also registers
// every block with HIP for DMA; off by default since round 5, shm_pool.cc.)
//
// Frames are carved from a per-process arena built in the background at start
// (below); a frame it cannot hold gets a block of its own.
// A block is segments of at most 8 MiB ("/psg.<pid>.<n>.<k>") mapped back to
// back; its name "/psg.<pid>.<n>:<segments>:<segment bytes>" says how to map
// it.  The owner unlinks its names when its Van stops (and at exit); the
// -procs launcher removes what a crashed node left.  A block that /dev/shm
// cannot hold is not created (posix_fallocate per segment): the array then
// comes from the heap and travels on the socket.
#pragma once
#include <cstddef>
#include <cstdint>
#include <memory>
#include <string>

namespace ps {
namespace shm {

/* switch the pool on for this process (process mode; PS_SHM_FRAMES=0 keeps it
   off); `arena`: build the pre-faulted frame arena in the background
   (PS_SHM_ARENA_MB, default 256; 0 = none) — workers and servers */
void Enable(bool arena = false);
bool Enabled();
/* a pooled shared-memory block of >= bytes, or nullptr (pool off / small / no room) */
std::shared_ptr<void> Alloc(size_t bytes);
/* this process's block holding [p, p + n): its name and p's offset in it */
bool Find(const void* p, size_t n, std::string* name, uint64_t* offset);
/* map a peer's block (cached for the process lifetime); nullptr on failure */
char* Map(const std::string& name, size_t* size);
/* remove this process's block names (mappings stay valid) */
void UnlinkAll();
/* remove the names a process left behind (the launcher, after a crash) */
void UnlinkOf(int pid);

}  // namespace shm
}  // namespace ps
