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
#include <rccl/rccl.h>

#include <cstring>

#include "psg_internal.h"

struct psg_comm {
  ncclComm_t comm;
  int rank, nranks, device;
  void* scratch;
  size_t scratch_bytes;
};

namespace psg {

static int nccl_fail(ncclResult_t r, const char* what) {
  set_error("%s failed: %s", what, ncclGetErrorString(r));
  return PSG_ERR_COMM;
}

#define PSG_NCCL(call)                                   \
  do {                                                   \
    ncclResult_t r_ = (call);                            \
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
  PSG_REQUIRE(s->kind == PSG_STORE_DENSE, PSG_ERR_INVALID, "psg_comm: shard must be a DENSE store");
  PSG_REQUIRE(n_total % (uint64_t)c->nranks == 0, PSG_ERR_INVALID,
              "psg_comm: n_total %llu not divisible by %d ranks", (unsigned long long)n_total,
              c->nranks);
  *blk = n_total / (uint64_t)c->nranks;
  PSG_REQUIRE(s->capacity >= *blk, PSG_ERR_RANGE, "psg_comm: shard holds %llu slots, block is %llu",
              (unsigned long long)s->capacity, (unsigned long long)*blk);
  return PSG_OK;
}

}  // namespace psg

using namespace psg;

extern "C" {

int psg_comm_id_bytes(void) { return (int)sizeof(ncclUniqueId); }

int psg_comm_get_id(void* id_host) {
  PSG_REQUIRE(id_host, PSG_ERR_INVALID, "psg_comm_get_id: null out");
  ncclUniqueId id;
  PSG_NCCL(ncclGetUniqueId(&id));
  memcpy(id_host, &id, sizeof(id));
  return PSG_OK;
}

int psg_comm_init(const void* id_host, int nranks, int rank, psg_comm** out) {
  PSG_REQUIRE(id_host && out && nranks > 0 && rank >= 0 && rank < nranks, PSG_ERR_INVALID,
              "psg_comm_init: bad arguments");
  *out = nullptr;
  ncclUniqueId id;
  memcpy(&id, id_host, sizeof(id));
  psg_comm* c = new psg_comm();
  memset(c, 0, sizeof(*c));
  c->rank = rank;
  c->nranks = nranks;
  (void)hipGetDevice(&c->device);
  ncclResult_t r = ncclCommInitRank(&c->comm, nranks, id, rank);
  if (r != ncclSuccess) {
    delete c;
    return nccl_fail(r, "ncclCommInitRank");
  }
  *out = c;
  return PSG_OK;
}

int psg_comm_destroy(psg_comm* c) {
  if (!c) return PSG_OK;
  if (c->scratch) (void)hipFree(c->scratch);
  if (c->comm) ncclCommDestroy(c->comm);
  delete c;
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
  if (c->nranks == 1)  // a one-rank reduce-scatter is the identity
    return dense_request(shard->dtype, PSG_PUSH, shard->vals, vals, nullptr, blk, st);
  ncclDataType_t t;
  PSG_REQUIRE(nccl_type(shard->dtype, &t), PSG_ERR_UNSUPPORTED, "psg_comm_push: dtype %d", shard->dtype);
  const size_t bytes = blk * shard->esize;
  if (!scratch) {
    if (c->scratch_bytes < bytes) {
      if (c->scratch) PSG_HIP(hipFree(c->scratch));
      c->scratch = nullptr;
      c->scratch_bytes = 0;
      PSG_HIP(hipMalloc(&c->scratch, bytes));
      c->scratch_bytes = bytes;
    }
    scratch = c->scratch;
  }
  PSG_NCCL(ncclReduceScatter(vals, scratch, blk, t, ncclSum, c->comm, st));
  return dense_request(shard->dtype, PSG_PUSH, shard->vals, scratch, nullptr, blk, st);
}

int psg_comm_pull(psg_comm* c, psg_store* shard, void* out, uint64_t n_total, psg_stream stream) {
  uint64_t blk = 0;
  PSG_TRY(check_shard(c, shard, n_total, &blk));
  if (blk == 0) return PSG_OK;
  PSG_REQUIRE(out, PSG_ERR_INVALID, "psg_comm_pull: null out");
  hipStream_t st = (hipStream_t)stream;
  if (c->nranks == 1)
    return dense_request(shard->dtype, PSG_PULL, shard->vals, nullptr, out, blk, st);
  ncclDataType_t t;
  PSG_REQUIRE(nccl_type(shard->dtype, &t), PSG_ERR_UNSUPPORTED, "psg_comm_pull: dtype %d", shard->dtype);
  PSG_NCCL(ncclAllGather(shard->vals, out, blk, t, c->comm, st));
  return PSG_OK;
}

}  // extern "C"
