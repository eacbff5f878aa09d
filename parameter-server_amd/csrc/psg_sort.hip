// psg_sort.hip — a stable device radix sort for the requests the fast keyed
// path cannot take: keys in any order, keys repeated (KVServerDefaultHandle
// walks such a request in arrival order, src/ps/KVApp.h:446-454, so every
// occurrence of a key adds to the store in turn and a PushPull returns the
// running value).  The store sorts (store slot, request position) pairs by slot
// — stable, so each key's occurrences stay in arrival order — and the absent
// keys of such a request (sorted and made unique before the store merges them
// in).
//
// LSD radix sort, 8-bit digits, one tile of 4096 items per 256-thread block:
//   k_rs_hist     digit histogram of every tile -> counts[digit][tile]
//   k_rs_scan     per digit, exclusive scan over the tiles; digit totals
//   k_rs_scatter  every tile ranks its items stably inside the tile (16 rounds
//                 of 256 items in position order; a wave finds the lanes that
//                 share its digit with 8 ballots), reorders them by digit in
//                 LDS, and writes each digit's run to its global place:
//                 consecutive lanes -> consecutive addresses within a run.
// Byte/integer work bound by HBM: per pass the keys are read twice and written
// once (and the values read and written once).
#include "psg_internal.h"

namespace psg {

namespace {

constexpr int kRsBlock = 256;
constexpr int kRsRounds = 16;
constexpr int kRsTile = kRsBlock * kRsRounds;  // 4096 items per block
constexpr int kRsWaves = kRsBlock / 64;

// the digit of a pass: 8 bits at `shift`, fewer in a last pass that ends at
// the requested bit count (dmask)
template <typename K>
__device__ __forceinline__ uint32_t digit_of(K k, int shift, uint32_t dmask) {
  return (uint32_t)(k >> shift) & dmask;
}

template <typename K>
__global__ __launch_bounds__(kRsBlock) void k_rs_hist(const K* __restrict__ keys, uint64_t n, int shift,
                                                      uint32_t dmask, uint32_t* __restrict__ counts,
                                                      uint64_t ntiles) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * kRsTile;
#pragma unroll 4
  for (int r = 0; r < kRsRounds; ++r) {
    const uint64_t i = t0 + (uint64_t)r * kRsBlock + threadIdx.x;
    if (i < n) atomicAdd(&h[digit_of(keys[i], shift, dmask)], 1u);
  }
  __syncthreads();
  counts[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// exclusive scan over 256 lanes of a block (4 waves)
__device__ __forceinline__ uint32_t rs_block_scan(uint32_t v, uint32_t* total, uint32_t* wsum) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = __shfl_up(x, d, 64);
    if (lane >= d) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  uint32_t off = 0, tot = 0;
#pragma unroll
  for (int k = 0; k < kRsWaves; ++k) {
    if (k < w) off += wsum[k];
    tot += wsum[k];
  }
  __syncthreads();
  *total = tot;
  return off + x - v;
}

// one block per digit: counts[d][0..ntiles) -> exclusive prefix; dtot[d] = total
__global__ __launch_bounds__(kRsBlock) void k_rs_scan(uint32_t* __restrict__ counts, uint64_t ntiles,
                                                      uint32_t* __restrict__ dtot) {
  __shared__ uint32_t wsum[kRsWaves];
  uint32_t* c = counts + (uint64_t)blockIdx.x * ntiles;
  uint32_t carry = 0;
  for (uint64_t b = 0; b < ntiles; b += kRsBlock) {
    const uint64_t i = b + threadIdx.x;
    const uint32_t v = i < ntiles ? c[i] : 0u;
    uint32_t tot;
    const uint32_t ex = rs_block_scan(v, &tot, wsum);
    if (i < ntiles) c[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) dtot[blockIdx.x] = carry;
}

template <typename K, bool IOTA>
__global__ __launch_bounds__(kRsBlock) void k_rs_scatter(const K* __restrict__ kin, const uint32_t* __restrict__ vin,
                                                         K* __restrict__ kout, uint32_t* __restrict__ vout,
                                                         uint64_t n, int shift, uint32_t dmask,
                                                         const uint32_t* __restrict__ counts,
                                                         const uint32_t* __restrict__ dtot, uint64_t ntiles) {
  __shared__ K sK[kRsTile];
  __shared__ uint32_t sV[kRsTile];
  __shared__ uint32_t gbase[256], lstart[256], running[256];
  __shared__ uint32_t wcnt[kRsWaves][256];
  __shared__ uint32_t wsum[kRsWaves];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint64_t tile = blockIdx.x, t0 = tile * kRsTile;
  {
    // global start of digit tid = sum of the smaller digits' totals; this
    // tile's place in it = the scanned count of the earlier tiles
    uint32_t tot;
    const uint32_t ds = rs_block_scan(dtot[tid], &tot, wsum);
    gbase[tid] = ds + counts[(uint64_t)tid * ntiles + tile];
    running[tid] = 0;
#pragma unroll
    for (int w = 0; w < kRsWaves; ++w) wcnt[w][tid] = 0;
  }
  K key[kRsRounds];
  uint32_t val[kRsRounds], rank[kRsRounds];
#pragma unroll
  for (int r = 0; r < kRsRounds; ++r) {
    const uint64_t i = t0 + (uint64_t)r * kRsBlock + tid;
    key[r] = i < n ? kin[i] : (K)0;
    val[r] = IOTA ? (uint32_t)i : (i < n ? vin[i] : 0u);
  }
  __syncthreads();
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  // 16 rounds in position order: round r holds items t0 + r*256 + tid, so
  // (round, wave, lane) order is position order and every rank is stable
#pragma unroll
  for (int r = 0; r < kRsRounds; ++r) {
    const uint64_t i = t0 + (uint64_t)r * kRsBlock + tid;
    const bool valid = i < n;
    const uint32_t d = digit_of(key[r], shift, dmask);
    uint64_t peers = __ballot(valid);
#pragma unroll
    for (int b = 0; b < 8; ++b) {
      const uint64_t bb = __ballot((d >> b) & 1u);
      peers &= ((d >> b) & 1u) ? bb : ~bb;
    }
    const uint32_t in_wave = (uint32_t)__popcll(peers & lt);
    if (valid && in_wave == 0) wcnt[wv][d] = (uint32_t)__popcll(peers);
    __syncthreads();
    if (valid) {
      uint32_t before = running[d];
      for (int w = 0; w < wv; ++w) before += wcnt[w][d];
      rank[r] = before + in_wave;
    }
    __syncthreads();
    {
      uint32_t add = 0;
#pragma unroll
      for (int w = 0; w < kRsWaves; ++w) {
        add += wcnt[w][tid];
        wcnt[w][tid] = 0;
      }
      running[tid] += add;
    }
    __syncthreads();
  }
  {
    uint32_t tot;
    lstart[tid] = rs_block_scan(running[tid], &tot, wsum);
  }
  __syncthreads();
#pragma unroll
  for (int r = 0; r < kRsRounds; ++r) {
    const uint64_t i = t0 + (uint64_t)r * kRsBlock + tid;
    if (i < n) {
      const uint32_t p = lstart[digit_of(key[r], shift, dmask)] + rank[r];
      sK[p] = key[r];
      sV[p] = val[r];
    }
  }
  __syncthreads();
  const uint64_t tn = n - t0 < (uint64_t)kRsTile ? n - t0 : (uint64_t)kRsTile;
  for (uint32_t j = tid; j < tn; j += kRsBlock) {
    const K k = sK[j];
    const uint32_t d = digit_of(k, shift, dmask);
    const uint64_t g = (uint64_t)gbase[d] + (j - lstart[d]);
    kout[g] = k;
    vout[g] = sV[j];
  }
}

template <typename K>
int radix_sort_impl(K* keys, uint32_t* vals, uint64_t n, int bits, bool iota, K* keys_alt, uint32_t* vals_alt,
                    uint32_t* counts, uint32_t* dtot, hipStream_t st, int* result) {
  *result = 0;
  if (n == 0) return PSG_OK;
  PSG_REQUIRE(n <= 0xffffffffull, PSG_ERR_RANGE, "radix sort: more than 2^32-1 items");
  const uint64_t ntiles = (n + kRsTile - 1) / kRsTile;
  K* kb[2] = {keys, keys_alt};
  uint32_t* vb[2] = {vals, vals_alt};
  int cur = 0;
  const int passes = bits <= 0 ? 1 : (bits + 7) / 8;
  for (int p = 0; p < passes; ++p) {
    const int shift = 8 * p;
    const int dbits = bits - shift < 8 && bits > 0 ? bits - shift : 8;
    const uint32_t dmask = (1u << dbits) - 1u;
    k_rs_hist<K><<<(unsigned)ntiles, kRsBlock, 0, st>>>(kb[cur], n, shift, dmask, counts, ntiles);
    k_rs_scan<<<256, kRsBlock, 0, st>>>(counts, ntiles, dtot);
    if (p == 0 && iota)
      k_rs_scatter<K, true><<<(unsigned)ntiles, kRsBlock, 0, st>>>(kb[cur], nullptr, kb[cur ^ 1], vb[cur ^ 1], n,
                                                                    shift, dmask, counts, dtot, ntiles);
    else
      k_rs_scatter<K, false><<<(unsigned)ntiles, kRsBlock, 0, st>>>(kb[cur], vb[cur], kb[cur ^ 1], vb[cur ^ 1], n,
                                                                     shift, dmask, counts, dtot, ntiles);
    PSG_HIP(hipGetLastError());
    cur ^= 1;
  }
  *result = cur;
  return PSG_OK;
}

}  // namespace

uint64_t radix_counts_elems(uint64_t n) { return 256 * ((n + kRsTile - 1) / kRsTile) + 256; }

int radix_sort_u32(uint32_t* keys, uint32_t* vals, uint64_t n, int bits, bool iota, uint32_t* keys_alt,
                   uint32_t* vals_alt, uint32_t* counts, hipStream_t st, int* result) {
  const uint64_t ntiles = (n + kRsTile - 1) / kRsTile;
  return radix_sort_impl<uint32_t>(keys, vals, n, bits, iota, keys_alt, vals_alt, counts, counts + 256 * ntiles, st,
                                   result);
}

int radix_sort_u64(uint64_t* keys, uint32_t* vals, uint64_t n, int bits, bool iota, uint64_t* keys_alt,
                   uint32_t* vals_alt, uint32_t* counts, hipStream_t st, int* result) {
  const uint64_t ntiles = (n + kRsTile - 1) / kRsTile;
  return radix_sort_impl<uint64_t>(keys, vals, n, bits, iota, keys_alt, vals_alt, counts, counts + 256 * ntiles, st,
                                   result);
}

}  // namespace psg

using namespace psg;

extern "C" {

int psg_sort_pairs_u64(uint64_t* keys, uint32_t* vals, uint64_t n, int bits, psg_stream stream) {
  PSG_REQUIRE(n == 0 || (keys && vals), PSG_ERR_INVALID, "psg_sort_pairs_u64: null argument");
  PSG_REQUIRE(bits >= 1 && bits <= 64, PSG_ERR_INVALID, "psg_sort_pairs_u64: bits %d", bits);
  if (n == 0) return PSG_OK;
  hipStream_t st = (hipStream_t)stream;
  // scratch by plain allocations, freed once the stream has finished with
  // them: one intermittent wrong result of this export (vals half unwritten,
  // n = 17) came from a run whose scratch was stream-ordered on the legacy
  // null stream (hipMallocAsync / hipFreeAsync), the only thing about it no
  // other sort in the library shares
  uint64_t* ka = nullptr;
  uint32_t *va = nullptr, *counts = nullptr;
  int rc = PSG_OK;
  auto release = [&] {
    if (ka) (void)hipFree(ka);
    if (va) (void)hipFree(va);
    if (counts) (void)hipFree(counts);
  };
  if (hipMalloc((void**)&ka, n * sizeof(uint64_t)) != hipSuccess ||
      hipMalloc((void**)&va, n * sizeof(uint32_t)) != hipSuccess ||
      hipMalloc((void**)&counts, radix_counts_elems(n) * sizeof(uint32_t)) != hipSuccess) {
    release();
    return hip_fail(hipErrorOutOfMemory, "psg_sort_pairs_u64 scratch", __FILE__, __LINE__);
  }
  int res = 0;
  rc = radix_sort_u64(keys, vals, n, bits, false, ka, va, counts, st, &res);
  if (rc == PSG_OK && res == 1) {
    if (hipMemcpyAsync(keys, ka, n * sizeof(uint64_t), hipMemcpyDeviceToDevice, st) != hipSuccess ||
        hipMemcpyAsync(vals, va, n * sizeof(uint32_t), hipMemcpyDeviceToDevice, st) != hipSuccess)
      rc = hip_fail(hipGetLastError(), "psg_sort_pairs_u64 copy back", __FILE__, __LINE__);
  }
  const hipError_t se = hipStreamSynchronize(st);
  if (rc == PSG_OK && se != hipSuccess) rc = hip_fail(se, "psg_sort_pairs_u64 sync", __FILE__, __LINE__);
  release();
  return rc;
}

}  // extern "C"
