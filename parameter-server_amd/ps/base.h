// ps/base.h — node groups and the key type (reference src/ps/Base.h:12-26).
#pragma once
#include <cstdint>
#include <limits>

namespace ps {

/* node id of the scheduler */
static constexpr int kScheduler = 1;
/* group ids, combinable with + or | */
static constexpr int kServerGroup = 2;
static constexpr int kWorkerGroup = 4;
static constexpr int kAllNodes = kScheduler + kServerGroup + kWorkerGroup;

/* the key type and the largest key; server ranges partition [0, kMaxKey) */
using Key = uint64_t;
static constexpr Key kMaxKey = std::numeric_limits<Key>::max();

}  // namespace ps
