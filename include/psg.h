/*
 * psg.h — C-ABI of the MI355X parameter-server value store and data path.
 *
 * This is the drop-in boundary between the C++ host runtime (the ps::KVWorker /
 * ps::KVServer mirror under parameter-server_amd/ps/) and the HIP kernels for
 * gfx950 in parameter-server_amd/csrc/.  Every entry point is plain C: raw
 * pointers, sizes and an int status.  No exception crosses it, no torch type
 * appears in it.  The detail of a failure is in psg_last_error() (per thread).
 *
 * Reference interfaces each group replaces (paths relative to the reference
 * repository SovietPower/Parameter-Server):
 *
 *   psg_store_*      the server-side value store `std::unordered_map<Key,V> store`
 *                    of KVServerDefaultHandle            src/ps/KVApp.h:433-458
 *   psg_store_handle the per-request accumulate loop
 *                    `store[key] += vals[i]; res.vals[i] = store[key]`
 *                                                        src/ps/KVApp.h:446-454
 *   psg_server_ranges PostOffice::GetServerRanges        src/internal/PostOffice.cpp:211-221
 *   psg_slice        KVWorker<V>::DefaultSlicer           src/ps/KVApp.h:515-574
 *   psg_merge        the AddPullCB merge lambda           src/ps/KVApp.h:673-726
 *   psg_comm_*       the ZMQ data path of Van::Send / ZMQVan::SendMsg / ReceiveMsg
 *                    (src/internal/Van.cpp:170-179, src/internal/ZMQVan.cpp:147-248)
 *                    for the BSP case: Push = reduce-scatter + accumulate,
 *                    Pull = all-gather, over RCCL / xGMI
 *   psg_lr_apply     LRServer::RequestHandle sync-mode apply (SGD / Adam)
 *                                                        tests/src/LRServer.h:151-189,
 *                                                        tests/src/Adam.h:28-34
 *
 * Conventions
 *   - All data pointers passed to compute entry points are DEVICE pointers
 *     (hipMalloc'd, or psg_malloc'd) unless the parameter name ends in _host.
 *   - Work is stream-ordered on the given stream (NULL = the legacy default
 *     stream).  An entry point that must return a host value (psg_slice,
 *     psg_store_resolve with insert) synchronises that stream itself and says so.
 *   - The store owns its device memory.  Buffers passed in stay owned by the
 *     caller and must stay valid until the stream has executed the work.
 *   - One store per server shard; calls on one store must be serialised by the
 *     caller (the reference runs ReqHandle on a single Customer thread,
 *     src/internal/Customer.cpp:52-70).
 */
#ifndef PSG_H_
#define PSG_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PSG_ABI_VERSION 1

/* ---- status codes ------------------------------------------------------ */
enum {
  PSG_OK = 0,
  PSG_ERR_INVALID = 1,     /* bad argument (a reference CHECK would have thrown) */
  PSG_ERR_HIP = 2,         /* HIP runtime error */
  PSG_ERR_OOM = 3,         /* device allocation failed */
  PSG_ERR_RANGE = 4,       /* key outside the store's range / capacity */
  PSG_ERR_COMM = 5,        /* RCCL error */
  PSG_ERR_UNSUPPORTED = 6  /* dtype / kind combination not built */
};

/* ---- value types (Message.h DataType has no half; f16/bf16 are ours) --- */
enum { PSG_F32 = 0, PSG_F64 = 1, PSG_F16 = 2, PSG_BF16 = 3 };

/* ---- store kinds ------------------------------------------------------- */
enum {
  /* Slots cover keys [key_begin, key_begin + capacity) contiguously: key k lives
   * at slot k - key_begin.  The layout of configs 2, 3 and 5 (dense vectors). */
  PSG_STORE_DENSE = 0,
  /* Arbitrary uint64 keys in [key_begin, key_end), kept as a sorted key array
   * plus a value array in HBM.  A key is inserted on first touch with value 0,
   * exactly like unordered_map::operator[] (KVApp.h:449, 452). */
  PSG_STORE_SORTED = 1
};

/* ---- request flags (KVMeta::push / KVMeta::pull, KVApp.h:42-57) --------- */
enum { PSG_PUSH = 1, PSG_PULL = 2 };

typedef struct psg_store psg_store;
typedef struct psg_comm psg_comm;
typedef void* psg_stream; /* a hipStream_t */
typedef void* psg_event;  /* a hipEvent_t */

/* ======================================================================== */
/* Runtime                                                                   */
/* ======================================================================== */
int psg_abi_version(void);
/* Message of the last failed call on this thread ("" if none). */
const char* psg_last_error(void);
int psg_device_count(int* n);
/* Bind the calling thread to a GPU (hipSetDevice). */
int psg_set_device(int device);
int psg_get_device(int* device);
/* The PCI bus id of `device` ("0000:05:00.0", hipDeviceGetPCIBusId) into buf
 * (len bytes, NUL-terminated).  No reference counterpart: a multi-GPU job
 * records which physical GPU each rank ran on (bench.py), and refuses two
 * ranks on one GPU. */
int psg_device_pci_bus_id(int device, char* buf, int len);
int psg_device_sync(void);
/* Let kernels on `device` read/write `peer`'s HBM over xGMI (idempotent). */
int psg_enable_peer_access(int device, int peer);

int psg_malloc(void** dptr, size_t bytes);
int psg_free(void* dptr);
int psg_host_alloc(void** hptr, size_t bytes); /* pinned host memory */
int psg_host_free(void* hptr);
int psg_host_register(void* hptr, size_t bytes); /* pin a caller's heap range */
int psg_host_unregister(void* hptr);
/* kind: 0 = H2D, 1 = D2H, 2 = D2D, 3 = default (unified addressing) */
int psg_memcpy(void* dst, const void* src, size_t bytes, int kind, psg_stream stream);
int psg_memset(void* dptr, int value, size_t bytes, psg_stream stream);
/* A plain 16-B-per-lane streaming copy (non-temporal loads and stores, grid
 * stride) of `bytes` (a multiple of 16, both pointers 16-B aligned), with
 * `unroll` vectors per lane in flight (1, 2, 4 or 8) at `blocks_per_cu`
 * 256-thread blocks per CU (1..16): the HBM copy ceiling a Pull — whose traffic
 * is exactly a copy's, read the store, write the reply — is measured against in
 * the same process (bench.py).  Not on any request path. */
int psg_copy(void* dst, const void* src, uint64_t bytes, int unroll, int blocks_per_cu, psg_stream stream);

int psg_stream_create(psg_stream* stream);
/* A stream of high priority (priority != 0: the device's greatest,
 * hipStreamCreateWithPriority) or of the default one.  A worker's small
 * kernels (the slicer, the merge) go on one, so that a server's long store
 * kernels sharing the process's hardware queues do not hold them back (no
 * reference counterpart: the reference slices on the host). */
int psg_stream_create_priority(psg_stream* stream, int priority);
int psg_stream_destroy(psg_stream stream);
int psg_stream_sync(psg_stream stream);
int psg_event_create(psg_event* ev);
/* An event for timing only (bench.py's markers): its record skips the
   system-scope release fence (hipEventDisableSystemFence), so a marker between
   two launches does not write back and invalidate the caches — the cost that
   made an event-timed launch read ~2 us longer than rocprof's kernel time.
   Elapsed times are valid once the stream has been synchronised; do not use
   it to hand data to the host or another device. */
int psg_event_create_timing(psg_event* ev);
int psg_event_destroy(psg_event ev);
int psg_event_record(psg_event ev, psg_stream stream);
int psg_event_sync(psg_event ev);
int psg_event_elapsed_ms(psg_event start, psg_event stop, float* ms);
/* later work on `stream` waits for `ev` (recorded on another stream) */
int psg_stream_wait_event(psg_stream stream, psg_event ev);

/* Seeded synthetic data generated on the device: element i of the output is a
 * pure function of (seed, i), so the CPU oracle regenerates it bit-exactly
 * (oracle/ps_oracle.cpp: oracle_synth).
 *   mode 0: integer-valued  floor(u * span) + lo        (exact float sums)
 *   mode 1: real-valued     lo + u * (hi - lo)
 * with u = (splitmix64(seed + i) >> 40) * 2^-24 in [0, 1). */
int psg_fill_synth(void* dptr, uint64_t n, int dtype, uint64_t seed, int mode,
                   double lo, double hi, psg_stream stream);
/* keys[i] = base + i * step (the test_kv_app_benchmark key layout
 * `kMaxKey / num * i + rank`, tests/test_kv_app_benchmark.cpp:47-52). */
int psg_fill_keys_arith(uint64_t* keys, uint64_t n, uint64_t base, uint64_t step,
                        psg_stream stream);
/* Position-keyed checksum of a device range (nbytes % 8 == 0, 8-B aligned):
 * sum over 64-bit words i of splitmix64(w_i ^ i * 0x9e3779b97f4a7c15), mod
 * 2^64.  Synchronises `stream`.  Used to verify an exchange end to end (the
 * xGMI pull against the owners' shards) without moving the data to the host.
 * No reference counterpart: test/verification support. */
int psg_checksum(const void* dptr, uint64_t nbytes, uint64_t* sum_host, psg_stream stream);
/* Closed-form check of a pulled vector of integer-valued synthetic pushes:
 * counts i < n with got[i] != scale * sum_{w < nseeds} synth(seed0 + w, i + offset)
 * (psg_fill_synth mode 0 over [lo, hi), summed in double).  *first_bad_host
 * (may be NULL) gets the smallest mismatching index, or UINT64_MAX.
 * Synchronises `stream`.  No reference counterpart: it checks a whole
 * multi-GPU Pull — every rank's block — on the device (bench.py, tests). */
int psg_verify_synth_sum(const void* dptr, uint64_t n, int dtype, uint64_t seed0, int nseeds,
                         uint64_t offset, double lo, double hi, double scale,
                         uint64_t* mismatches_host, uint64_t* first_bad_host, psg_stream stream);

/* ======================================================================== */
/* Server-side value store  (KVServerDefaultHandle::store, KVApp.h:457)      */
/* ======================================================================== */
typedef struct psg_store_info {
  int kind;
  int dtype;
  uint64_t key_begin;  /* owned key range [key_begin, key_end) */
  uint64_t key_end;
  uint64_t size;       /* keys currently present (dense: = capacity) */
  uint64_t capacity;   /* slots allocated */
  void* vals;          /* device pointer to the value array (slot order) */
  uint64_t* keys;      /* device pointer to the sorted key array (SORTED), else NULL */
} psg_store_info;

int psg_store_create(int kind, int dtype, uint64_t key_begin, uint64_t key_end,
                     uint64_t capacity, psg_store** out);
int psg_store_destroy(psg_store* s);
int psg_store_get_info(psg_store* s, psg_store_info* info);
/* Zero every value (DENSE) / drop every key (SORTED). */
int psg_store_clear(psg_store* s, psg_stream stream);
/* How a SORTED store served its keyed requests so far (diagnostics and tests;
 * no reference counterpart): out[PSG_CTR_FUSED] requests on the validated
 * resolve-and-apply kernels, [PSG_CTR_IDENT] sent as identity requests (a key
 * list covering stretches of the store, at slots known from its cached
 * windows: no validation pass, no search), [PSG_CTR_NOTIDENT] of those that
 * were not and ran again on the general path, [PSG_CTR_ORDERED] on the
 * order-preserving path (keys out of order or repeated).  Waits for the
 * requests in flight.  Writes min(n, PSG_NCOUNTERS) counters, zero past them. */
#define PSG_CTR_FUSED 0
#define PSG_CTR_IDENT 1
#define PSG_CTR_NOTIDENT 2
#define PSG_CTR_ORDERED 3
/* runs of queued Pushes served in one pass (psg_store_push_frames,
 * psg_store_push_slots_frames), and the requests those runs held */
#define PSG_CTR_RUNS 4
#define PSG_CTR_RUN_FRAMES 5
/* fused Pushes whose validation pass also resolved their tiles (coded tiles:
 * the apply then reads no request keys and stages no window for a tile whose
 * keys are all in the store) */
#define PSG_CTR_CODED 6
/* of those, Pushes whose stretch and coded tiles went to the lean apply
 * (k_tile_apply), and those of them that met a general tile and had it applied
 * by a follow-up on the general path */
#define PSG_CTR_LEAN 7
#define PSG_CTR_LEAN_PARTIAL 8
/* runs of queued requests on interleaved key lists served in one pass
 * (psg_store_run, PSG_RUN_STRIDED), and the requests those runs held */
#define PSG_CTR_STRIDED_RUNS 9
#define PSG_CTR_STRIDED_FRAMES 10
/* lean Pushes validated against their list's verified copy (k_list_check: the
 * list as a learning request of this K validated it), and those that were not
 * that list after all and ran again with the full validation */
#define PSG_CTR_LISTS 11
#define PSG_CTR_NOTLIST 12
/* requests served on their own as a strided pass (psg_store_run, k = 1: a list
 * whose place in a learnt interleaved layout the store knows) */
#define PSG_CTR_STRIDED_SINGLE 13
#define PSG_NCOUNTERS 14
int psg_store_counters(psg_store* s, uint64_t* out, int n);

/* One request, KVServerDefaultHandle::operator() (KVApp.h:435-456):
 *   for i < n:  if (flags & PSG_PUSH) store[key_i] += vals[i];
 *               if (flags & PSG_PULL) out[i] = store[key_i];   (post-update)
 * keys == NULL means the consecutive keys first_key, first_key + 1, ...
 * (dense request: no key array travels).  Keys may come in any order and may
 * repeat, as the reference's loop allows: each occurrence adds in arrival
 * order and a PushPull answers each occurrence with the running value.
 * Strictly ascending keys (the KVPairs contract, KVApp.h:23) take the fused
 * streaming kernels; any other request takes the order-preserving path (a
 * stable device sort by slot, then one lane per key walking its occurrences),
 * with the same result bit for bit.  An absent key is inserted with 0
 * (operator[], KVApp.h:449/452).  A key outside the store's range (a DENSE
 * store: outside [key_begin, key_begin + capacity)) fails the request
 * (PSG_ERR_RANGE) and leaves the store unchanged; out is then unspecified.
 * vals/out are device arrays of n elements of the store's dtype.
 * A keyed request (SORTED store, or DENSE with keys) returns once the request
 * is complete: its keys and vals are no longer read — the caller may reuse
 * them — and a Pull's reply is in memory, readable by any agent (a copy
 * engine, the host, another stream) without synchronising `stream`.  Its last
 * store writes may still be in flight: work that reads the store must be
 * ordered after it on `stream`.  (On the steady SORTED path it waits for the
 * completion word its own kernel writes, which also carries the request's
 * flags, and for a Pull for an event recorded behind the kernel, polled —
 * not for the stream itself.)  The store
 * remembers the LDS windows of the last few key arrays it saw (by device
 * pointer and n) and verifies them per tile, so a caller may rewrite a key
 * array in place between requests. */
int psg_store_handle(psg_store* s, int flags, const uint64_t* keys,
                     uint64_t first_key, const void* vals, void* out, uint64_t n,
                     psg_stream stream);

/* The same request without waiting for it (the server answering a stream of
 * requests, KVServer::Process, KVApp.h:462-489): a fused keyed request on a
 * populated SORTED store is launched and *ticket names it; every other request
 * completes before the call returns (*ticket = 0).  Requests of one store run
 * in call order.  keys / vals / out must stay untouched until the ticket is
 * waited for.  A request that needs the host (absent keys to insert, keys out
 * of order) raises a device word that makes every request launched after it
 * write nothing; the wait that reaps it inserts the keys, clears the word and
 * replays those requests, in order — the store sees exactly the call sequence.
 * psg_store_wait(s, t) completes every request up to ticket t (0: all) and
 * returns the first failure of those not reported yet; when it returns, the
 * replies of the Pulls reaped so far are in memory (it synchronises their
 * stream once, rather than each request waiting for its own).  Every other
 * store call
 * completes the requests in flight first.
 * It can block: the first request of a key list sent as an identity request
 * after K's generation changed (any insert, a clear) is a trial, reaped —
 * with any replay it needs — before the call returns, so no request is
 * launched behind a verdict not yet known; growing a key list's window cache
 * also waits for the requests in flight. */
int psg_store_handle_async(psg_store* s, int flags, const uint64_t* keys,
                           uint64_t first_key, const void* vals, void* out, uint64_t n,
                           psg_stream stream, uint64_t* ticket);
int psg_store_wait(psg_store* s, uint64_t ticket);

/* A run of k Push requests on ONE key list, queued one behind the other at a
 * server (the reference's KVServer drains its queue one message at a time,
 * src/internal/Customer.cpp:52-70, and applies each with `store[key] +=
 * vals[i]`, src/ps/KVApp.h:446-454).  The result is bit for bit that of
 *     for j < k:  psg_store_handle(s, PSG_PUSH, keys_host[j], first_key,
 *                                  vals_host[j], NULL, n, stream)
 * — each key's frames added in order j = 0, 1, ..., every add rounded to the
 * store's dtype as k requests round — but when the lists are one list, the
 * store is read and written once for the k frames: 8 + 4k B per f32 key
 * instead of 12k, plus reading each list once to know that it is the same
 * (8 B per list).  keys_host: k device key arrays of n keys (pointers may
 * differ: each worker's own frame), or NULL for a dense run on a DENSE store
 * (consecutive keys from first_key).  vals_host: k device value arrays.
 * 1 <= k <= 16.  On a SORTED store one pass serves lists that are a stretch
 * of the store's keys, or, failing that, lists equal to list 0 whose keys are
 * all present, in range and ascending; any other run — lists that differ,
 * absent keys, keys out of order — is served request by request, exactly as
 * k psg_store_handle calls (a request that fails stops the run there and
 * returns its status).  *fused_host (may be NULL) = 1 when one pass served the
 * run.  Returns as psg_store_handle does: the frames are no longer read (a
 * dense run on a DENSE store: stream-ordered, like a dense request).
 * PSG_FRAMES=0 serves every run request by request (A/B). */
int psg_store_push_frames(psg_store* s, const uint64_t* const* keys_host, uint64_t first_key,
                          const void* const* vals_host, int k, uint64_t n, psg_stream stream,
                          int* fused_host);

/* A run of k requests queued one behind the other at a server — Pushes, Pulls
 * and PushPulls, each on its own key list — served with the result of
 *     for j < k:  psg_store_handle(s, ops[j], keys[j], 0, vals[j], outs[j],
 *                                  ns[j], stream)
 * (the reference's receive thread takes queued messages one at a time,
 * src/internal/Customer.cpp:52-70, and serves each with its own loop,
 * src/ps/KVApp.h:446-454).  Two layouts are served in one pass:
 *   PSG_RUN_SAME_LIST  every request a Push on one list (nw workers of a BSP
 *                      round): as psg_store_push_frames, each key's values
 *                      added in order j = 0, 1, ...;
 *   PSG_RUN_STRIDED    the lists are distinct phases of one period P <= 64 of
 *                      the store's keys, keys[j][i] == K[D + p_j + P i] — the
 *                      reference benchmark's layout `kMaxKey / num * i + rank`
 *                      (tests/test_kv_app_benchmark.cpp:47-52) at nw workers,
 *                      P = nw.  Such lists are pairwise disjoint: every store
 *                      value is touched by at most one request, so the order
 *                      of the run changes no result, and one pass over the
 *                      slots they span serves them: 28 B per pushed and 24 per
 *                      pulled f32 key (request and store keys 16, values),
 *                      against 8 P + 8 P of store lines per key for each
 *                      request on its own.
 * Any other run — lists that overlap or differ in layout, absent keys, keys out
 * of order — is served request by request, exactly as the k calls (a request
 * that fails stops the run there and returns its status).  Every key is
 * checked before any value is written: a run a pass rejects leaves the store
 * as it found it.  keys[j], vals[j] (Push), outs[j] (Pull): device arrays of
 * ns[j] elements; 1 <= k <= 16.  *served (may be NULL) = PSG_RUN_*.  Returns
 * as psg_store_handle does: every key and value array is no longer read and
 * every Pull's reply is in memory.  k = 1: a request whose list this store
 * has seen in a strided run (its first key's slot and period known, at this
 * K generation) takes the strided pass on its own — its phase's slots of the
 * rows, against the general path's windows and search — else it is
 * psg_store_handle.  PSG_RUNS_STRIDED=0 never tries the strided pass (A/B). */
#define PSG_RUN_ONE_BY_ONE 0
#define PSG_RUN_SAME_LIST 1
#define PSG_RUN_STRIDED 2
int psg_store_run(psg_store* s, int k, const int* ops, const uint64_t* const* keys, const uint64_t* ns,
                  const void* const* vals, void* const* outs, psg_stream stream, int* served);
/* psg_store_run with a status per request (status: k ints): a request whose
 * key lies outside the store's range is refused on its own (status
 * PSG_ERR_RANGE, nothing of it applied) and the others are served, in order.
 * Returns PSG_OK when every request was served or refused that way; any other
 * failure stops the run (the failing request and those after it carry its
 * code).  The server's answer to a worker's unconfirmed slice
 * (KVWorker::Send, Meta::spec_slice): a wrong one is refused, not applied. */
int psg_store_run_status(psg_store* s, int k, const int* ops, const uint64_t* const* keys, const uint64_t* ns,
                         const void* const* vals, void* const* outs, psg_stream stream, int* served,
                         int* status);
/* A SORTED store's key range from now on (psg_store_create's key_begin /
 * key_end): a request key outside it rejects the request, on every path (the
 * strided pass checks it too).  The default handle narrows it to the server's
 * own range while it serves unconfirmed slices, then widens it again. */
int psg_store_set_key_range(psg_store* s, uint64_t key_begin, uint64_t key_end);

/* The stable device radix sort of the order-preserving path (psg_sort.hip),
 * exported for its parity tests: sorts (keys[i], vals[i]) by bits [0, bits) of
 * the key, equal keys keeping their order.  In place; synchronises `stream`
 * (its scratch is allocated before and freed after). */
int psg_sort_pairs_u64(uint64_t* keys, uint32_t* vals, uint64_t n, int bits, psg_stream stream);

/* Slot cache (LR USE_KEY_CACHING, tests/src/LRServer.h:127-142): resolve a key
 * list to slot indices once, then run requests by slot.  insert != 0 inserts
 * absent keys (value 0) and synchronises the stream; insert == 0 writes
 * UINT32_MAX for absent keys.  Slots stay valid until the next insert.  A
 * slot list names each key once: its keys must be strictly ascending
 * (PSG_ERR_INVALID otherwise), since the slot kernels update a slot from one
 * lane. */
int psg_store_resolve(psg_store* s, const uint64_t* keys, uint64_t n, int insert,
                      uint32_t* slots, psg_stream stream);
int psg_store_handle_slots(psg_store* s, int flags, const uint32_t* slots,
                           const void* vals, void* out, uint64_t n,
                           psg_stream stream);
/* A slot list that is a stretch of the store — slots[i] == slots[0] + i for
 * every i, as when a cached key list covers its range of the store (an LR
 * worker sending every feature, tests/src/LRServer.h:144) — needs no slot
 * stream: *first = slots[0] then, else UINT64_MAX.  Synchronises `stream`.
 * psg_store_handle_stretch is then psg_store_handle_slots on the slots
 * [first, first + n): store[first + i] += vals[i] and / or out[i] =
 * store[first + i], a plain stream (12 B / f32 key for a Push instead of 16,
 * 8 for a Pull instead of 12).  Slots stay valid until the next insert. */
int psg_store_slots_stretch(psg_store* s, const uint32_t* slots, uint64_t n, uint64_t* first,
                            psg_stream stream);
int psg_store_handle_stretch(psg_store* s, int flags, uint64_t first, const void* vals, void* out,
                             uint64_t n, psg_stream stream);
/* A run of k Pushes on one cached list (LR key caching names it by its hash,
 * tests/src/LRServer.h:127-142): psg_store_handle_slots(PSG_PUSH) with
 * vals_host[0], then vals_host[1], ... in one pass — slot 4 + store 8 + 4k B
 * per f32 key; slots == NULL: psg_store_handle_stretch on [first, first + n),
 * 8 + 4k.  Bit for bit the k requests in order.  Stream-ordered, like them
 * (psg_store_sync before answering).  1 <= k <= 16. */
int psg_store_push_slots_frames(psg_store* s, const uint32_t* slots, uint64_t first,
                                const void* const* vals_host, int k, uint64_t n, psg_stream stream);
/* Return once everything enqueued on `stream` so far has run, its writes
 * visible to any agent (a slot or stretch request's values no longer read, its
 * Pull reply in memory for a copy engine, the host or another process): an
 * event recorded behind that work and polled with hipEventQuery — what
 * psg_store_handle does for its own Pull replies — instead of a sleeping
 * stream wait; after 2 ms it falls back to hipEventSynchronize
 * (PSG_SYNC_POLL=0: hipStreamSynchronize always).  Lets a server answer a
 * cached-list request as soon as its kernel ends (KVServer::Response,
 * KVApp.h:491-513). */
int psg_store_sync(psg_store* s, psg_stream stream);

/* The hash a key list is cached under in LR key caching (the std::hash
 * specialisation of tests/src/LRServer.h:11-29, which LRWorker.h:214-219 also
 * computes): n XOR the XOR of splitmix64(keys[i]).  Device keys; synchronises
 * `stream`.  Lets a server cache a list that arrives as an HBM frame. */
int psg_key_list_hash(const uint64_t* keys, uint64_t n, uint64_t* hash_host, psg_stream stream);

/* Copy the store to host memory (checkpoint, LRServer::SaveModel analogue,
 * tests/src/LRServer.h:107-115).  keys_host may be NULL for a DENSE store;
 * both arrays must hold info.size elements.  Synchronous. */
int psg_store_dump(psg_store* s, uint64_t* keys_host, void* vals_host);

/* ======================================================================== */
/* Worker side: key-range slicing and pull merge                              */
/* ======================================================================== */
/* Server i owns [kMaxKey/ns*i, kMaxKey/ns*(i+1)), the last one ends at kMaxKey
 * (PostOffice::GetServerRanges, PostOffice.cpp:211-221).  Host only. */
int psg_server_ranges(int num_servers, uint64_t* begins_host, uint64_t* ends_host);

/* DefaultSlicer (KVApp.h:515-574) on a device key array:
 *   key_pos[0] = lower_bound(keys, begins[0]);
 *   key_pos[i+1] = lower_bound(keys, ends[i])            (i < ns)
 * and the value bounds of each slice:
 *   lens == NULL:  val_pos[i] = key_pos[i] * (num_vals / n)   (CHECKs divisibility)
 *   lens != NULL:  val_pos[i] = val_pos[0] + sum(lens[key_pos[0] .. key_pos[i]))
 *                  (the running sum of KVApp.h:565-569; val_pos[0] = 0).
 * key_pos_host / val_pos_host hold ns + 1 entries (val_pos_host may be NULL).
 * Fails (PSG_ERR_INVALID) when key_pos[ns] != n, i.e. a key lies at or above
 * the last range's end (the CHECK at KVApp.h:544).  Returns once the bounds
 * are known: the bound kernels write them, tagged, straight into pinned host
 * memory, so a request costs no copy launch and no stream synchronisation
 * (with lens, the per-slice sums still come back by a copy and a sync). */
int psg_slice(const uint64_t* keys, uint64_t n, const int* lens, uint64_t num_vals,
              int num_servers, const uint64_t* begins_host,
              const uint64_t* ends_host, uint64_t* key_pos_host,
              uint64_t* val_pos_host, psg_stream stream);

/* The bounds psg_slice found at its last slice of this key array (same
 * pointer, n, server count and first range) on this thread, without reading
 * the keys: *found = 1 and key_pos_host (ns + 1 entries) filled, else
 * *found = 0.  A worker may send these slices unconfirmed when every server
 * checks each key against its own range (a wrong bound puts some key outside
 * its server's range, and that server refuses the request). */
int psg_slice_hint(const uint64_t* keys, uint64_t n, int num_servers, uint64_t begin0, uint64_t* key_pos_host,
                   int* found);

/* One pull reply (KVPairs from one server, KVApp.h:631-637). */
typedef struct psg_segment {
  const void* vals;    /* device pointer */
  uint64_t count;      /* elements in vals */
  uint64_t first_key;  /* keys.front() of the reply, the sort key */
} psg_segment;

/* The AddPullCB merge (KVApp.h:680-720): order the replies by first key and
 * concatenate their values into dst (dst_count elements of elem_size bytes),
 * in one batched-copy kernel.  Fails if the counts do not add up to dst_count
 * (the "lost some servers?" CHECK, KVApp.h:691, 701). */
int psg_merge(psg_segment* segs_host, int nsegs, int elem_size, void* dst,
              uint64_t dst_count, psg_stream stream);

/* ======================================================================== */
/* Multi-GPU BSP data path over RCCL / xGMI (one server shard per GPU)        */
/* ======================================================================== */
/* Bytes of the opaque id rank 0 creates and every rank passes to init (two
 * RCCL unique ids: one communicator per direction of psg_comm_push_pull).
 * PSG_COMM_FORCE_COLLECTIVE=1 makes a one-rank comm run the collectives
 * anyway (they degenerate to copies) so the RCCL calls can be tested on one GPU.
 * psg_comm_init never waits for a missing rank for good: the RCCL inits run on
 * a helper thread, waited for against PSG_COMM_TIMEOUT_S (default 90 s); when
 * a rank does not join, init fails with PSG_ERR_COMM on every rank that did
 * (the reference's Van waits for ADD_NODE the same way, Van.cpp:320-442, but
 * without a deadline). */
int psg_comm_id_bytes(void);
int psg_comm_get_id(void* id_host);
int psg_comm_init(const void* id_host, int nranks, int rank, psg_comm** out);

/* Host-only plans of the exchanges (no GPU needed): the offsets the RCCL
 * paths use, exported so the multi-rank CPU rehearsal (tests/test_dist.py)
 * drives its gloo collectives with the very same numbers.
 * psg_comm_bucket_plan: the buckets of psg_comm_push_pull over a block of blk
 * elements — bucket b covers [offs[b], offs[b] + cnts[b]) of every rank's
 * block; chunks are multiples of 64 elements.  *nb_out = the bucket count
 * (<= cap, else PSG_ERR_INVALID).
 * psg_comm_keyed_plan: checks key_pos[nranks+1] as psg_comm_push_keyed /
 * _pull_keyed do (key_pos[0] = 0, key_pos[nranks] = n, ascending) and returns
 * the longest segment (the reduce scratch the owner needs). */
int psg_comm_bucket_plan(uint64_t blk, int nbuckets, uint64_t* offs, uint64_t* cnts, int cap, int* nb_out);
int psg_comm_keyed_plan(const uint64_t* key_pos_host, int nranks, uint64_t n, uint64_t* maxseg);
int psg_comm_destroy(psg_comm* c);
int psg_comm_rank(psg_comm* c, int* rank, int* nranks);
/* Wait for the collectives queued on `stream` (and the comm's side stream) for
 * at most timeout_s (<= 0: PSG_COMM_TIMEOUT_S).  On a timeout the communicators
 * are aborted (their kernels leave their wait loops), every later collective
 * call on c fails with PSG_ERR_COMM, and so does this one: a caller that runs
 * a first collective under it can fall back instead of hanging. */
int psg_comm_sync(psg_comm* c, psg_stream stream, double timeout_s);
/* Abort the communicators now (every rank of a job that gives up on RCCL
 * together calls it); later collective calls on c fail with PSG_ERR_COMM. */
int psg_comm_abort(psg_comm* c);

/* BSP Push of a dense vector: every rank contributes its worker's full vector
 * vals[n_total]; rank r's DENSE store `shard` owns the contiguous block
 * [r * n_total / nranks, (r + 1) * n_total / nranks) (n_total % nranks == 0).
 * shard += sum over ranks of vals[block r] — a reduce-scatter then the
 * accumulate kernel.  `scratch` is a device buffer of n_total / nranks elements
 * (NULL: the comm keeps one).  Equivalent to nranks KVWorker::Push calls
 * arriving at each KVServerDefaultHandle (KVApp.h:449). */
int psg_comm_push(psg_comm* c, psg_store* shard, const void* vals, uint64_t n_total,
                  void* scratch, psg_stream stream);
/* BSP Pull: out[n_total] on every rank = concatenation of every rank's shard,
 * an all-gather (KVApp.h:452 + the merge of KVApp.h:713-720). */
int psg_comm_pull(psg_comm* c, psg_store* shard, void* out, uint64_t n_total,
                  psg_stream stream);
/* Push then Pull of the same vector, pipelined over nbuckets: bucket b's
 * reduce-to-owner + accumulate (stream, communicator 0) overlaps bucket b-1's
 * broadcast-from-owner (side stream, communicator 1), so both directions of
 * the xGMI links carry traffic.  Same result as psg_comm_push + psg_comm_pull;
 * nbuckets <= 1 is exactly those two calls.  Complete on `stream` on return. */
int psg_comm_push_pull(psg_comm* c, psg_store* shard, const void* vals, void* out,
                       uint64_t n_total, int nbuckets, psg_stream stream);

/* Keyed BSP Push / Pull (configs[3], LR_ps): every rank passes the SAME sorted
 * key array keys[n] (device) and its values; key_pos_host[nranks+1] are the
 * psg_slice bounds of the server ranges (key_pos[0] = 0, key_pos[nranks] = n).
 * Push: segment r of every rank's vals is reduced to rank r and applied to its
 * store (SORTED or DENSE) with psg_store_handle — the nranks x nranks Push
 * messages of KVWorker::Send (KVApp.h:596-618) as one grouped RCCL reduce.
 * Pull: each owner reads its segment into out[key_pos[r]..] and broadcasts
 * it, which also does the merge of KVApp.h:713-720. */
int psg_comm_push_keyed(psg_comm* c, psg_store* shard, const uint64_t* keys, const void* vals,
                        uint64_t n, const uint64_t* key_pos_host, psg_stream stream);
int psg_comm_pull_keyed(psg_comm* c, psg_store* shard, const uint64_t* keys, void* out,
                        uint64_t n, const uint64_t* key_pos_host, psg_stream stream);

/* ---- one-shot xGMI exchange (no RCCL) -------------------------------------
 * Every rank maps its peers' request vectors and store shards (hipIpc handles
 * the caller exchanges: psg_ipc_export on the owner, psg_ipc_open on the
 * others) and reads all peers in ONE kernel, so the 7 xGMI links of an MI355X
 * carry traffic together and the reduction is fused with the accumulate.
 * Ordering between ranks is the caller's (psg_node_barrier after each phase). */
typedef struct psg_xgmi psg_xgmi;
typedef struct psg_barrier psg_barrier;
int psg_ipc_handle_bytes(void);
int psg_ipc_export(const void* dptr, void* handle_out);   /* dptr: start of an allocation */
/* the same for a pointer anywhere inside an allocation: the handle of the
 * allocation and dptr's byte offset in it (the process-mode Van ships HBM
 * frames — slices of pooled blocks — this way: parameter-server_amd/src/tcp_van.cc) */
int psg_ipc_export_range(const void* dptr, void* handle_out, uint64_t* offset_out);
int psg_ipc_open(const void* handle, void** dptr_out);
int psg_ipc_close(void* dptr);
/* peer_vals[r] / peer_stores[r]: rank r's request vector (n_total values) and
 * DENSE shard value array, as pointers valid in this process. */
int psg_xgmi_create(int nranks, int rank, void* const* peer_vals, void* const* peer_stores,
                    psg_xgmi** out);
int psg_xgmi_destroy(psg_xgmi* x);
/* shard += sum over ranks w (in rank order) of vals_w[block r] */
int psg_xgmi_push(psg_xgmi* x, psg_store* shard, uint64_t n_total, psg_stream stream);
/* out[w * blk ...] = shard of rank w, for every w */
int psg_xgmi_pull(psg_xgmi* x, psg_store* shard, void* out, uint64_t n_total, psg_stream stream);
/* The same on elements [off, off + cnt) of every block (16-B multiples): the
 * chunks of a double-buffered step, where the Pull of chunk c (one stream)
 * runs while the Push of chunk c + 1 (another stream) is in flight —
 * configs[4]'s "Push/Pull double-buffered on HIP streams".  The caller orders
 * the ranks per chunk (psg_node_barrier after every rank's Push of chunk c). */
int psg_xgmi_push_range(psg_xgmi* x, psg_store* shard, uint64_t n_total, uint64_t off,
                        uint64_t cnt, psg_stream stream);
int psg_xgmi_pull_range(psg_xgmi* x, psg_store* shard, void* out, uint64_t n_total,
                        uint64_t off, uint64_t cnt, psg_stream stream);
/* The Pull as writes (egress) instead of reads (ingress).  psg_xgmi_set_outs
 * registers every rank's Pull output buffer (n_total values, mapped here;
 * this rank's own at [rank]).  psg_xgmi_pull_write_range then copies this
 * rank's shard elements [off, off + cnt) into out_w[rank * blk + off ...] of
 * every rank w: the all-gather pushed out over the links while the Push
 * (psg_xgmi_push*, which reads its peers) uses the other direction of each
 * full-duplex link.  It needs only this rank's own Push of that range to be
 * complete (stream order): no barrier between the phases.  A rank's output
 * is complete once every rank's writes are: the caller synchronises its
 * stream and passes a psg_node_barrier before any rank reads its output, and
 * before the next step's writes. */
int psg_xgmi_set_outs(psg_xgmi* x, void* const* peer_outs);
int psg_xgmi_pull_write_range(psg_xgmi* x, psg_store* shard, uint64_t n_total, uint64_t off,
                              uint64_t cnt, psg_stream stream);
int psg_xgmi_pull_write(psg_xgmi* x, psg_store* shard, uint64_t n_total, psg_stream stream);
/* Keyed exchange on cached slots (configs[3] with LR key caching): every rank
 * pushes values for the SAME key list; [seg_off, seg_off + seg_n) is the
 * psg_slice segment of this rank's shard, and `slots` its psg_store_resolve
 * slots in this rank's SORTED store (registered as this rank's store array).
 *   push: store[slots[i]] += vals_0[seg_off + i] + ... + vals_{N-1}[...]
 *         (rank order: the N Push requests in arrival order 0..N-1)
 *   pull: out[seg_off_w + i] = store_w[slots_w[i]] for every rank w
 * peer_slots[w] is rank w's slot array mapped here (hipIpc).  The stores
 * must not insert keys while mapped (an insert moves the value array). */
int psg_xgmi_push_slots(psg_xgmi* x, psg_store* shard, const uint32_t* slots, uint64_t seg_off,
                        uint64_t seg_n, psg_stream stream);
int psg_xgmi_pull_slots(psg_xgmi* x, psg_store* shard, const uint32_t* const* peer_slots,
                        const uint64_t* seg_off_host, const uint64_t* seg_n_host, void* out,
                        psg_stream stream);
/* The keyed Pull as writes (outputs registered with psg_xgmi_set_outs): rank r
 * writes store[slots[i]] into out_w[seg_off + i] of every rank w.  Needs only
 * this rank's own push_slots to be complete; one barrier per step, as for
 * psg_xgmi_pull_write. */
int psg_xgmi_pull_write_slots(psg_xgmi* x, psg_store* shard, const uint32_t* slots, uint64_t seg_off,
                              uint64_t seg_n, psg_stream stream);
/* Host barrier of the ranks of one node over a POSIX shared-memory page. */
int psg_node_barrier_create(const char* name, int nranks, int rank, psg_barrier** out);
int psg_node_barrier_wait(psg_barrier* b, double timeout_s);
int psg_node_barrier_destroy(psg_barrier* b);

/* ======================================================================== */
/* LR server apply                                             */
/* ======================================================================== */
typedef struct psg_adam psg_adam;
/* Adam state (m, v as double, Adam.h:14-18, 40-41) for n features. */
int psg_adam_create(uint64_t n, double learning_rate, double beta1, double beta2,
                    double epsilon, psg_adam** out);
int psg_adam_destroy(psg_adam* a);
/* weight[i] = (float)((double)weight[i] - g), with g = (double)(lr * merged[i])
 * (an f32 product, as `double grad = learning_rate_ * merge_buf_.vals[i]`),
 * then g = adam(g, i, iteration) when adam != NULL (LRServer.h:171-177,
 * Adam.h:28-34); merged is f32, weights are the f32 DENSE store's slots
 * [0, n).  Bit-identical to the reference's operation order. */
int psg_lr_apply(psg_store* weights, const float* merged, uint64_t n, float lr,
                 psg_adam* adam, int iteration, psg_stream stream);
/* The BSP round of LRServer::RequestHandle fused into ONE pass:
 *   s_i = from_zero ? ((0 + g_0[i]) + g_1[i]) + ... : (g_0[i] + g_1[i]) + ...
 * (f32 adds in the order given — the arrival order of `merge_buf_.vals[i] +=
 * req_data.vals[i]`, LRServer.h:158-160; from_zero = 1 for sync mode's merge
 * buffer, 0 for async mode's single push, LRServer.h:179-189), then the
 * update of psg_lr_apply on s_i.  No merge buffer is written or cleared.
 * grads_host: 1..16 device pointers to n floats each. */
int psg_lr_apply_sum(psg_store* weights, const float* const* grads_host, int ngrads,
                     int from_zero, uint64_t n, float lr, psg_adam* adam, int iteration,
                     psg_stream stream);
/* Measurement only (no reference counterpart): psg_lr_apply_sum's Adam pass
 * (from_zero) with its loads and stores unchanged and a copy's arithmetic in
 * place of the update (m += s, v -= s, w += s) — the rate this box moves the
 * Adam apply's byte mix (4 B per frame + weight 8 + f64 moments 32 per
 * feature), the ceiling bench.py --workload lr compares the apply with.  It
 * scribbles on the weights and moments. */
int psg_lr_mix_copy(psg_store* weights, const float* const* grads_host, int ngrads, uint64_t n, psg_adam* adam,
                    psg_stream stream);
/* Multi-GPU LR BSP Push (nw = ns = nranks, weights = rank r's f32 DENSE shard
 * of n_total / nranks features, adam = that shard's state):
 *   psg_comm_lr_push  reduce-scatter of every rank's grads[n_total] (RCCL; its
 *                     summation order, so 1e-6 relative against the reference)
 *                     into scratch (NULL: the comm's), then the fused apply;
 *   psg_xgmi_lr_push  ONE kernel reading block r of every rank's registered
 *                     request vector (the gradients) over xGMI, merged from 0 in
 *                     rank order and applied (bit-exact against the reference
 *                     replaying the pushes in rank order).
 * Pull of the model is psg_comm_pull / psg_xgmi_pull. */
int psg_comm_lr_push(psg_comm* c, psg_store* weights, const float* grads, uint64_t n_total,
                     float lr, psg_adam* adam, int iteration, void* scratch, psg_stream stream);
int psg_xgmi_lr_push(psg_xgmi* x, psg_store* weights, uint64_t n_total, float lr,
                     psg_adam* adam, int iteration, psg_stream stream);

#ifdef __cplusplus
}
#endif
#endif /* PSG_H_ */
