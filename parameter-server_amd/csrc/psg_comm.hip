// psg_comm.hip — the multi-GPU BSP data path: one server shard per GPU, RCCL
// over xGMI in place of the ZMQ data frames of Van::Send / ZMQVan::SendMsg
// (src/internal/Van.cpp:170-179, src/internal/ZMQVan.cpp:147-196).
//
// With nw = ns = nranks and every worker pushing its full dense vector in the
// same step (BSP, LRServer SYNC_MODE=0, tests/src/LRServer.h:151-178), the
// nw x ns point-to-point messages of a Push collapse into one reduce-scatter:
// rank r receives sum_w vals_w[block r] and adds it into its store shard with
// the dense accumulate kernel.  A Pull is the all-gather of the shards, which
// also performs the merge of KVApp.h:713-720 (blocks land in key order).
//
// psg_comm_push_pull pipelines the two over buckets: bucket b's reduce (to
// each owner) + accumulate runs on the caller's stream and communicator 0
// while bucket b-1's broadcast (from each owner) runs on a side stream and
// communicator 1, so the two directions of every xGMI link carry traffic at
// once.  Two communicators keep the two streams' collectives independent.
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <thread>
#include <vector>

#include "psg_internal.h"

struct psg_comm {
  ncclComm_t comm[2];
  int rank, nranks, device;
  bool force;  // run the collectives even with one rank (testing)
  void* scratch;
  size_t scratch_bytes;
  hipStream_t side;
  std::vector<hipEvent_t> ev;  // per-bucket "accumulated" events
  hipEvent_t side_done;
  bool aborted;  // psg_comm_sync timed out and aborted the communicators
};

namespace psg {

static int nccl_fail(ncclResult_t r, const char* what) {
  set_error("%s failed: %s", what, ncclGetErrorString(r));
  return PSG_ERR_COMM;
}

#define PSG_NCCL(call)                                       \
  do {                                                       \
    ncclResult_t r_ = (call);                                \
    if (r_ != ncclSuccess) return psg::nccl_fail(r_, #call); \
  } while (0)

static bool nccl_type(int dtype, ncclDataType_t* t) {
  switch (dtype) {
    case PSG_F32: *t = ncclFloat32; return true;
    case PSG_F64: *t = ncclFloat64; return true;
    case PSG_F16: *t = ncclFloat16; return true;
    case PSG_BF16: *t = ncclBfloat16; return true;
    default: return false;
  }
}

static int check_shard(psg_comm* c, psg_store* s, uint64_t n_total, uint64_t* blk) {
  PSG_REQUIRE(c && s, PSG_ERR_INVALID, "psg_comm: null comm or store");
  PSG_REQUIRE(!c->aborted, PSG_ERR_COMM, "psg_comm: the communicators were aborted (psg_comm_sync timed out)");
  PSG_REQUIRE(s->kind == PSG_STORE_DENSE, PSG_ERR_INVALID, "psg_comm: shard must be a DENSE store");
  PSG_REQUIRE(n_total % (uint64_t)c->nranks == 0, PSG_ERR_INVALID,
              "psg_comm: n_total %llu not divisible by %d ranks", (unsigned long long)n_total,
              c->nranks);
  *blk = n_total / (uint64_t)c->nranks;
  PSG_REQUIRE(s->capacity >= *blk, PSG_ERR_RANGE, "psg_comm: shard holds %llu slots, block is %llu",
              (unsigned long long)s->capacity, (unsigned long long)*blk);
  return PSG_OK;
}

static int ensure_scratch(psg_comm* c, size_t bytes) {
  if (c->scratch_bytes >= bytes) return PSG_OK;
  if (c->scratch) PSG_HIP(hipFree(c->scratch));
  c->scratch = nullptr;
  c->scratch_bytes = 0;
  PSG_HIP(hipMalloc(&c->scratch, bytes));
  c->scratch_bytes = bytes;
  return PSG_OK;
}

}  // namespace psg

using namespace psg;

extern "C" {

// Two unique ids: one communicator per direction of psg_comm_push_pull.
constexpr int kCommIds = 2;

int psg_comm_id_bytes(void) { return kCommIds * (int)sizeof(ncclUniqueId); }

int psg_comm_get_id(void* id_host) {
  PSG_REQUIRE(id_host, PSG_ERR_INVALID, "psg_comm_get_id: null out");
  for (int k = 0; k < kCommIds; ++k) {
    ncclUniqueId id;
    PSG_NCCL(ncclGetUniqueId(&id));
    memcpy((char*)id_host + k * sizeof(id), &id, sizeof(id));
  }
  return PSG_OK;
}

}  // extern "C"

namespace psg {

// Seconds a communicator's rendezvous may take (PSG_COMM_TIMEOUT_S, default 90).
static double comm_timeout_s() {
  const char* e = getenv("PSG_COMM_TIMEOUT_S");
  const double v = e ? atof(e) : 0.0;
  return v > 0 ? v : 90.0;
}

// ncclCommInitRank blocks until every rank of the communicator has joined, and
// RCCL has no deadline of its own: one rank that never arrives (it died before
// init, or runs another job) would hang every other rank for good.  (RCCL
// 2.27's non-blocking config did not help here: ncclCommInitRankConfig with
// blocking = 0 still blocked in the rendezvous, measured on MI355X with a rank
// missing.)  So the two inits run on a helper thread and the caller waits for
// them against a deadline.  On a timeout psg_comm_init fails with PSG_ERR_COMM
// on this rank — every rank of such a job fails the same way within the
// deadline — so the caller can fall back (bench.py: the xGMI kernels, agreed by
// all ranks) or exit with a message instead of hanging.  The helper thread is
// then abandoned inside RCCL: it owns everything it touches (the job below),
// and if its peers do turn up later it leaves the communicators it made unused.
struct CommInitJob {
  ncclUniqueId ids[kCommIds];
  int nranks = 0, rank = 0, device = 0;
  ncclComm_t comm[kCommIds] = {};
  ncclResult_t r = ncclSuccess;
  hipError_t e = hipSuccess;
  bool done = false;
  std::mutex mu;
  std::condition_variable cv;
};

static void comm_init_thread(std::shared_ptr<CommInitJob> j) {
  ncclResult_t r = ncclSuccess;
  hipError_t e = hipSetDevice(j->device);  // HIP's current device is per thread
  ncclComm_t comm[kCommIds] = {};
  if (e == hipSuccess) {
    for (int k = 0; k < kCommIds && r == ncclSuccess; ++k) r = ncclCommInitRank(&comm[k], j->nranks, j->ids[k], j->rank);
    if (r != ncclSuccess)
      for (int k = 0; k < kCommIds; ++k)
        if (comm[k]) (void)ncclCommDestroy(comm[k]);
  }
  std::lock_guard<std::mutex> lk(j->mu);
  j->r = r;
  j->e = e;
  for (int k = 0; k < kCommIds; ++k) j->comm[k] = r == ncclSuccess ? comm[k] : nullptr;
  j->done = true;
  j->cv.notify_all();
}

}  // namespace psg

extern "C" {

int psg_comm_init(const void* id_host, int nranks, int rank, psg_comm** out) {
  PSG_REQUIRE(id_host && out && nranks > 0 && rank >= 0 && rank < nranks, PSG_ERR_INVALID,
              "psg_comm_init: bad arguments");
  *out = nullptr;
  auto job = std::make_shared<CommInitJob>();
  for (int k = 0; k < kCommIds; ++k) memcpy(&job->ids[k], (const char*)id_host + k * sizeof(ncclUniqueId), sizeof(ncclUniqueId));
  job->nranks = nranks;
  job->rank = rank;
  PSG_HIP(hipGetDevice(&job->device));
  const double timeout_s = comm_timeout_s();
  std::thread(comm_init_thread, job).detach();
  {
    std::unique_lock<std::mutex> lk(job->mu);
    const bool done = job->cv.wait_for(lk, std::chrono::microseconds((int64_t)(timeout_s * 1e6)), [&] { return job->done; });
    PSG_REQUIRE(done, PSG_ERR_COMM,
                "psg_comm_init: the RCCL rendezvous of %d ranks (this is rank %d) did not complete within %.0f s "
                "(PSG_COMM_TIMEOUT_S): a rank did not join",
                nranks, rank, timeout_s);
  }
  if (job->e != hipSuccess) return hip_fail(job->e, "psg_comm_init: hipSetDevice", __FILE__, __LINE__);
  if (job->r != ncclSuccess) return nccl_fail(job->r, "ncclCommInitRank");
  psg_comm* c = new psg_comm();
  c->rank = rank;
  c->nranks = nranks;
  const char* f = getenv("PSG_COMM_FORCE_COLLECTIVE");
  c->force = f && atoi(f) != 0;
  c->device = job->device;
  for (int k = 0; k < kCommIds; ++k) c->comm[k] = job->comm[k];
  hipError_t e = hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking);
  if (e == hipSuccess) e = hipEventCreateWithFlags(&c->side_done, hipEventDisableTiming);
  if (e != hipSuccess) {
    psg_comm_destroy(c);
    return hip_fail(e, "psg_comm_init stream", __FILE__, __LINE__);
  }
  *out = c;
  return PSG_OK;
}

int psg_comm_destroy(psg_comm* c) {
  if (!c) return PSG_OK;
  if (c->side) (void)hipStreamSynchronize(c->side);
  for (hipEvent_t e : c->ev) (void)hipEventDestroy(e);
  if (c->side_done) (void)hipEventDestroy(c->side_done);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->scratch) (void)hipFree(c->scratch);
  for (int k = 0; k < 2; ++k)
    if (c->comm[k]) ncclCommDestroy(c->comm[k]);
  delete c;
  return PSG_OK;
}

int psg_comm_sync(psg_comm* c, psg_stream stream, double timeout_s) {
  PSG_REQUIRE(c, PSG_ERR_INVALID, "psg_comm_sync: null comm");
  PSG_REQUIRE(!c->aborted, PSG_ERR_COMM, "psg_comm_sync: the communicators were aborted");
  const double limit_s = timeout_s > 0 ? timeout_s : comm_timeout_s();  // 0: the default
  const auto deadline = std::chrono::steady_clock::now() +
                        std::chrono::microseconds((int64_t)(limit_s * 1e6));
  hipStream_t sts[2] = {(hipStream_t)stream, c->side};
  for (hipStream_t st : sts) {
    for (;;) {
      const hipError_t q = hipStreamQuery(st);
      if (q == hipSuccess) break;
      if (q != hipErrorNotReady) return hip_fail(q, "psg_comm_sync", __FILE__, __LINE__);
      if (std::chrono::steady_clock::now() > deadline) {
        // a collective that cannot complete (a peer gone, a transport that
        // never connected): abort the communicators, whose kernels then leave
        // their wait loops, and report it instead of hanging
        for (int k = 0; k < kCommIds; ++k)
          if (c->comm[k]) (void)ncclCommAbort(c->comm[k]);
        for (int k = 0; k < kCommIds; ++k) c->comm[k] = nullptr;
        c->aborted = true;
        set_error("psg_comm_sync: the collectives did not complete within %.0f s; communicators aborted", limit_s);
        return PSG_ERR_COMM;
      }
      std::this_thread::sleep_for(std::chrono::microseconds(100));
    }
  }
  return PSG_OK;
}

int psg_comm_abort(psg_comm* c) {
  PSG_REQUIRE(c, PSG_ERR_INVALID, "psg_comm_abort: null comm");
  for (int k = 0; k < kCommIds; ++k)
    if (c->comm[k]) (void)ncclCommAbort(c->comm[k]);
  for (int k = 0; k < kCommIds; ++k) c->comm[k] = nullptr;
  c->aborted = true;
  return PSG_OK;
}

int psg_comm_rank(psg_comm* c, int* rank, int* nranks) {
  PSG_REQUIRE(c, PSG_ERR_INVALID, "psg_comm_rank: null comm");
  if (rank) *rank = c->rank;
  if (nranks) *nranks = c->nranks;
  return PSG_OK;
}

int psg_comm_push(psg_comm* c, psg_store* shard, const void* vals, uint64_t n_total, void* scratch,
                  psg_stream stream) {
  uint64_t blk = 0;
  PSG_TRY(check_shard(c, shard, n_total, &blk));
  if (blk == 0) return PSG_OK;
  PSG_REQUIRE(vals, PSG_ERR_INVALID, "psg_comm_push: null vals");
  hipStream_t st = (hipStream_t)stream;
  if (c->nranks == 1 && !c->force)  // a one-rank reduce-scatter is the identity
    return dense_request(shard->dtype, PSG_PUSH, shard->vals, vals, nullptr, blk, st);
  ncclDataType_t t;
  PSG_REQUIRE(nccl_type(shard->dtype, &t), PSG_ERR_UNSUPPORTED, "psg_comm_push: dtype %d", shard->dtype);
  if (!scratch) {
    PSG_TRY(ensure_scratch(c, blk * shard->esize));
    scratch = c->scratch;
  }
  PSG_NCCL(ncclReduceScatter(vals, scratch, blk, t, ncclSum, c->comm[0], st));
  return dense_request(shard->dtype, PSG_PUSH, shard->vals, scratch, nullptr, blk, st);
}

// LR BSP Push over RCCL: the reduce-scatter of every rank's gradient vector,
// then the fused apply on this rank's weight shard (the merge buffer of
// LRServer.h:158-160 is the reduce-scatter output; no merge store, no clear).
int psg_comm_lr_push(psg_comm* c, psg_store* weights, const float* grads, uint64_t n_total, float lr,
                     psg_adam* adam, int iteration, void* scratch, psg_stream stream) {
  uint64_t blk = 0;
  PSG_TRY(check_shard(c, weights, n_total, &blk));
  if (blk == 0) return PSG_OK;
  PSG_REQUIRE(grads, PSG_ERR_INVALID, "psg_comm_lr_push: null grads");
  PSG_REQUIRE(weights->dtype == PSG_F32, PSG_ERR_UNSUPPORTED, "psg_comm_lr_push: f32 weights only");
  hipStream_t st = (hipStream_t)stream;
  const float* merged = grads;  // one rank: its own gradient block is the merge
  if (c->nranks > 1 || c->force) {
    if (!scratch) {
      PSG_TRY(ensure_scratch(c, blk * sizeof(float)));
      scratch = c->scratch;
    }
    PSG_NCCL(ncclReduceScatter(grads, scratch, blk, ncclFloat32, ncclSum, c->comm[0], st));
    merged = (const float*)scratch;
  } else {
    merged = grads + (uint64_t)c->rank * blk;
  }
  const float* g[1] = {merged};
  return lr_apply_sum(weights, 0, g, 1, 1, blk, lr, adam, 0, iteration, st);
}

int psg_comm_pull(psg_comm* c, psg_store* shard, void* out, uint64_t n_total, psg_stream stream) {
  uint64_t blk = 0;
  PSG_TRY(check_shard(c, shard, n_total, &blk));
  if (blk == 0) return PSG_OK;
  PSG_REQUIRE(out, PSG_ERR_INVALID, "psg_comm_pull: null out");
  hipStream_t st = (hipStream_t)stream;
  if (c->nranks == 1 && !c->force)
    return dense_request(shard->dtype, PSG_PULL, shard->vals, nullptr, out, blk, st);
  ncclDataType_t t;
  PSG_REQUIRE(nccl_type(shard->dtype, &t), PSG_ERR_UNSUPPORTED, "psg_comm_pull: dtype %d", shard->dtype);
  PSG_NCCL(ncclAllGather(shard->vals, out, blk, t, c->comm[0], st));
  return PSG_OK;
}

int psg_comm_push_pull(psg_comm* c, psg_store* shard, const void* vals, void* out, uint64_t n_total,
                       int nbuckets, psg_stream stream) {
  uint64_t blk = 0;
  PSG_TRY(check_shard(c, shard, n_total, &blk));
  if (blk == 0) return PSG_OK;
  PSG_REQUIRE(vals && out, PSG_ERR_INVALID, "psg_comm_push_pull: null buffer");
  hipStream_t st = (hipStream_t)stream;
  if (nbuckets <= 1 || (c->nranks == 1 && !c->force)) {
    PSG_TRY(psg_comm_push(c, shard, vals, n_total, nullptr, stream));
    return psg_comm_pull(c, shard, out, n_total, stream);
  }
  ncclDataType_t t;
  PSG_REQUIRE(nccl_type(shard->dtype, &t), PSG_ERR_UNSUPPORTED, "psg_comm_push_pull: dtype %d",
              shard->dtype);
  const int es = shard->esize;
  std::vector<uint64_t> boff((size_t)nbuckets), bcnt((size_t)nbuckets);
  int nb = 0;
  PSG_TRY(psg_comm_bucket_plan(blk, nbuckets, boff.data(), bcnt.data(), nbuckets, &nb));
  PSG_TRY(ensure_scratch(c, blk * es));
  while ((int)c->ev.size() < nb) {
    hipEvent_t e;
    PSG_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    c->ev.push_back(e);
  }
  // the side stream must not start a bucket's broadcast before the caller's
  // earlier work on the output buffer is done
  PSG_HIP(hipEventRecord(c->side_done, st));
  PSG_HIP(hipStreamWaitEvent(c->side, c->side_done, 0));
  const char* in = (const char*)vals;
  char* o = (char*)out;
  char* sv = (char*)shard->vals;
  char* sc = (char*)c->scratch;
  for (int b = 0; b < nb; ++b) {
    const uint64_t off = boff[b], cnt = bcnt[b];
    // Push of bucket b: every rank's chunk b reduced to its owner, then accumulated
    PSG_NCCL(ncclGroupStart());
    for (int r = 0; r < c->nranks; ++r) {
      const char* src = in + ((uint64_t)r * blk + off) * es;
      PSG_NCCL(ncclReduce(src, sc + off * es, cnt, t, ncclSum, r, c->comm[0], st));
    }
    PSG_NCCL(ncclGroupEnd());
    PSG_TRY(dense_request(shard->dtype, PSG_PUSH, sv + off * es, sc + off * es, nullptr, cnt, st));
    PSG_HIP(hipEventRecord(c->ev[b], st));
    // Pull of bucket b on the side stream: each owner broadcasts its updated chunk
    PSG_HIP(hipStreamWaitEvent(c->side, c->ev[b], 0));
    PSG_NCCL(ncclGroupStart());
    for (int r = 0; r < c->nranks; ++r) {
      char* dst = o + ((uint64_t)r * blk + off) * es;
      PSG_NCCL(ncclBroadcast(sv + off * es, dst, cnt, t, r, c->comm[1], c->side));
    }
    PSG_NCCL(ncclGroupEnd());
  }
  PSG_HIP(hipEventRecord(c->side_done, c->side));
  PSG_HIP(hipStreamWaitEvent(st, c->side_done, 0));
  return PSG_OK;
}

int psg_comm_bucket_plan(uint64_t blk, int nbuckets, uint64_t* offs, uint64_t* cnts, int cap, int* nb_out) {
  PSG_REQUIRE(offs && cnts && nb_out && nbuckets >= 1, PSG_ERR_INVALID, "psg_comm_bucket_plan: bad arguments");
  *nb_out = 0;
  if (blk == 0) return PSG_OK;
  // bucket b covers [b*chunk, min((b+1)*chunk, blk)) of every rank's block;
  // chunks are multiples of 64 elements so vector kernels stay aligned
  uint64_t chunk = (blk + (uint64_t)nbuckets - 1) / (uint64_t)nbuckets;
  chunk = (chunk + 63) / 64 * 64;
  const int nb = (int)((blk + chunk - 1) / chunk);
  PSG_REQUIRE(nb <= cap, PSG_ERR_INVALID, "psg_comm_bucket_plan: %d buckets, room for %d", nb, cap);
  for (int b = 0; b < nb; ++b) {
    offs[b] = (uint64_t)b * chunk;
    cnts[b] = offs[b] + chunk <= blk ? chunk : blk - offs[b];
  }
  *nb_out = nb;
  return PSG_OK;
}

// ---- keyed BSP (configs[3], LR_ps): every rank pushes values for the SAME
// sorted key array, cut by psg_slice into per-server segments key_pos[r] ..
// key_pos[r+1].  Push: segment r of every rank is reduced to rank r, which
// applies it to its store with the keyed handle; Pull: every owner reads its
// segment and broadcasts it into place.
int psg_comm_keyed_plan(const uint64_t* kp, int nranks, uint64_t n, uint64_t* maxseg) {
  PSG_REQUIRE(kp && maxseg && nranks >= 1, PSG_ERR_INVALID, "psg_comm keyed: null argument");
  PSG_REQUIRE(kp[0] == 0 && kp[nranks] == n, PSG_ERR_INVALID,
              "psg_comm keyed: key_pos must cover [0, n) (%llu..%llu vs %llu)",
              (unsigned long long)kp[0], (unsigned long long)kp[nranks], (unsigned long long)n);
  *maxseg = 0;
  for (int r = 0; r < nranks; ++r) {
    PSG_REQUIRE(kp[r] <= kp[r + 1], PSG_ERR_INVALID, "psg_comm keyed: key_pos not ascending");
    if (kp[r + 1] - kp[r] > *maxseg) *maxseg = kp[r + 1] - kp[r];
  }
  return PSG_OK;
}

static int keyed_args(psg_comm* c, psg_store* s, const uint64_t* keys, uint64_t n,
                      const uint64_t* kp, uint64_t* maxseg) {
  PSG_REQUIRE(c && s && kp, PSG_ERR_INVALID, "psg_comm keyed: null argument");
  PSG_REQUIRE(!c->aborted, PSG_ERR_COMM, "psg_comm: the communicators were aborted (psg_comm_sync timed out)");
  PSG_REQUIRE(n == 0 || keys, PSG_ERR_INVALID, "psg_comm keyed: null keys");
  return psg_comm_keyed_plan(kp, c->nranks, n, maxseg);
}

int psg_comm_push_keyed(psg_comm* c, psg_store* shard, const uint64_t* keys, const void* vals,
                        uint64_t n, const uint64_t* key_pos_host, psg_stream stream) {
  uint64_t maxseg = 0;
  PSG_TRY(keyed_args(c, shard, keys, n, key_pos_host, &maxseg));
  if (n == 0) return PSG_OK;
  PSG_REQUIRE(vals, PSG_ERR_INVALID, "psg_comm_push_keyed: null vals");
  const int me = c->rank, es = shard->esize;
  const uint64_t* kp = key_pos_host;
  const uint64_t mine = kp[me + 1] - kp[me];
  if (c->nranks == 1 && !c->force)
    return psg_store_handle(shard, PSG_PUSH, keys, 0, vals, nullptr, n, stream);
  hipStream_t st = (hipStream_t)stream;
  ncclDataType_t t;
  PSG_REQUIRE(nccl_type(shard->dtype, &t), PSG_ERR_UNSUPPORTED, "psg_comm_push_keyed: dtype %d",
              shard->dtype);
  PSG_TRY(ensure_scratch(c, (maxseg ? maxseg : 1) * es));
  PSG_NCCL(ncclGroupStart());
  for (int r = 0; r < c->nranks; ++r) {
    const uint64_t cnt = kp[r + 1] - kp[r];
    if (cnt) PSG_NCCL(ncclReduce((const char*)vals + kp[r] * es, c->scratch, cnt, t, ncclSum, r, c->comm[0], st));
  }
  PSG_NCCL(ncclGroupEnd());
  if (!mine) return PSG_OK;
  return psg_store_handle(shard, PSG_PUSH, keys + kp[me], 0, c->scratch, nullptr, mine, stream);
}

int psg_comm_pull_keyed(psg_comm* c, psg_store* shard, const uint64_t* keys, void* out, uint64_t n,
                        const uint64_t* key_pos_host, psg_stream stream) {
  uint64_t maxseg = 0;
  PSG_TRY(keyed_args(c, shard, keys, n, key_pos_host, &maxseg));
  if (n == 0) return PSG_OK;
  PSG_REQUIRE(out, PSG_ERR_INVALID, "psg_comm_pull_keyed: null out");
  const int me = c->rank, es = shard->esize;
  const uint64_t* kp = key_pos_host;
  const uint64_t mine = kp[me + 1] - kp[me];
  if (mine)
    PSG_TRY(psg_store_handle(shard, PSG_PULL, keys + kp[me], 0, nullptr, (char*)out + kp[me] * es, mine,
                             stream));
  if (c->nranks == 1 && !c->force) return PSG_OK;
  hipStream_t st = (hipStream_t)stream;
  ncclDataType_t t;
  PSG_REQUIRE(nccl_type(shard->dtype, &t), PSG_ERR_UNSUPPORTED, "psg_comm_pull_keyed: dtype %d",
              shard->dtype);
  PSG_NCCL(ncclGroupStart());
  for (int r = 0; r < c->nranks; ++r) {
    const uint64_t cnt = kp[r + 1] - kp[r];
    char* p = (char*)out + kp[r] * es;
    if (cnt) PSG_NCCL(ncclBroadcast(p, p, cnt, t, r, c->comm[0], st));
  }
  PSG_NCCL(ncclGroupEnd());
  return PSG_OK;
}

}  // extern "C"
