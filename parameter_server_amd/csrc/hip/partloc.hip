// Localisation by partition + per-bucket LDS dedup (key spaces of <= 32 bits).
//
// The reference's Localizer::countUniqIndex (src/util/localizer.h:69-108) sorts
// (key, position) pairs and run-length encodes them; remapIndex (:126-191)
// rebuilds the CSR with local column ids. A full LSD radix sort of the 2.56 M
// occurrences of a 65,536 x 39 minibatch costs 3 passes x 4 launches and is
// latency bound on MI355X. But the step only needs the UNIQUE keys in sorted
// order (about 1 in 11 occurrences here), every occurrence's unique id, and the
// occurrences grouped by key (CSC order) - the order of positions inside a key's
// group is free. So:
//
//   count    one pass over the raw keys: mix, LDS histogram of the top BB bits,
//            one global atomic per (tile, non-empty bucket)
//   scatter  recompute the tile histogram, reserve each bucket run with one global
//            atomic, write (mixed key, position) into its bucket (LDS rank)
//   dedup    one workgroup per bucket: LDS hash of the bucket's distinct keys with
//            occurrence counts (hot keys: one LDS atomic per wave-group of equal
//            keys, a 64-lane match-any built from ballots), then an LDS bitonic sort
//            of the distinct keys -> per-bucket sorted list + counts
//   emit     one workgroup per bucket: global unique base = prefix of the buckets'
//            distinct counts; rebuild the hash from the sorted list, per-key
//            cursors = occurrence offsets; every occurrence -> CSC slot, segment id,
//            local column; unique keys, segment starts, zeroed gradient buffers.
//
// 5 launches (incl. one memset) instead of 16. Mixed keys are a bijection of the
// raw ids, so distinct keys spread evenly over buckets; BB is chosen so a bucket
// averages <= HCAP / 1.6 occurrences, which bounds its distinct keys even when
// every key is distinct. A bucket whose distinct keys overflow the LDS hash sets
// *err (the caller raises); the output is then incomplete.
#include "common.cuh"

#include <stdexcept>
#include <string>

namespace psamd {

namespace pl {
constexpr int kTileThreads = 1024;
constexpr int kTileItems = 16;
constexpr int kTile = kTileThreads * kTileItems;  // 16384 occurrences per tile
constexpr int kMaxBB = 12;
constexpr int kMaxBuckets = 1 << kMaxBB;
constexpr int kBThreads = 512;  // dedup / emit workgroups
constexpr uint32_t kEmpty = 0xffffffffu;
}  // namespace pl
using namespace pl;

__device__ __forceinline__ uint32_t lhash(uint32_t k) {
  k ^= k >> 16;
  k *= 0x7feb352du;
  k ^= k >> 15;
  k *= 0x846ca68bu;
  k ^= k >> 16;
  return k;
}

// 64-lane match-any of an nbits-wide value: mask of the active lanes holding v.
__device__ __forceinline__ uint64_t match_any(uint32_t v, int nbits, uint64_t active) {
  uint64_t peers = active;
  for (int b = 0; b < nbits; ++b) {
    const bool bit = (v >> b) & 1u;
    const uint64_t bal = __ballot(bit);
    peers &= bit ? bal : ~bal;
  }
  return peers;
}

template <int kN>
__device__ __forceinline__ uint32_t block_excl_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
  constexpr int kW = kN / 64;
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t run = 0;
    for (int w = 0; w < kW; ++w) {
      const uint32_t t = lds[w];
      lds[w] = run;
      run += t;
    }
    lds[kW] = run;
  }
  __syncthreads();
  const uint32_t r = x - v + lds[wid];
  *total = lds[kW];
  __syncthreads();
  return r;
}

// Bucket b's start in the partitioned arrays: sum of totals[0:b) (each workgroup
// sums the few thousand L2-resident totals itself: no scan launch).
template <int kN>
__device__ __forceinline__ uint32_t prefix_of(const uint32_t* __restrict__ a, int b,
                                              uint32_t* lds) {
  uint32_t s = 0;
  for (int i = threadIdx.x; i < b; i += kN) s += a[i];
  uint32_t tot;
  block_excl_scan<kN>(s, lds, &tot);
  return tot;
}

// ------------------------------------------------------------------ count
__global__ void __launch_bounds__(kTileThreads)
pl_count_kernel(const uint64_t* __restrict__ raw, int64_t n, KeyMix m, int shift, int nbk,
                uint32_t* __restrict__ totals) {
  __shared__ uint32_t hist[kMaxBuckets];
  for (int d = threadIdx.x; d < nbk; d += kTileThreads) hist[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll 4
  for (int j = 0; j < kTileItems; ++j) {
    const int64_t i = base + (int64_t)j * kTileThreads + threadIdx.x;
    if (i < n) atomicAdd(&hist[(uint32_t)mix_key(raw[i], m) >> shift], 1u);
  }
  __syncthreads();
  for (int d = threadIdx.x; d < nbk; d += kTileThreads)
    if (hist[d]) atomicAdd(&totals[d], hist[d]);
}

// ---------------------------------------------------------------- scatter
__global__ void __launch_bounds__(kTileThreads)
pl_scatter_kernel(const uint64_t* __restrict__ raw, int64_t n, KeyMix m, int shift, int nbk,
                  const uint32_t* __restrict__ totals, uint32_t* __restrict__ cursors,
                  uint32_t* __restrict__ pk, int32_t* __restrict__ pv) {
  __shared__ uint32_t hist[kMaxBuckets];
  __shared__ uint32_t off[kMaxBuckets];
  __shared__ uint32_t lds[kTileThreads / 64 + 1];
  for (int d = threadIdx.x; d < nbk; d += kTileThreads) hist[d] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  uint32_t k[kTileItems];
#pragma unroll
  for (int j = 0; j < kTileItems; ++j) {
    const int64_t i = base + (int64_t)j * kTileThreads + threadIdx.x;
    k[j] = i < n ? (uint32_t)mix_key(raw[i], m) : 0u;
  }
#pragma unroll
  for (int j = 0; j < kTileItems; ++j) {
    const int64_t i = base + (int64_t)j * kTileThreads + threadIdx.x;
    if (i < n) atomicAdd(&hist[k[j] >> shift], 1u);
  }
  __syncthreads();
  // bucket starts: exclusive prefix of the global totals (kTileThreads digits per round)
  uint32_t carry = 0;
  for (int d0 = 0; d0 < nbk; d0 += kTileThreads) {
    const int d = d0 + threadIdx.x;
    const uint32_t t = d < nbk ? totals[d] : 0u;
    uint32_t tot;
    const uint32_t ex = block_excl_scan<kTileThreads>(t, lds, &tot);
    if (d < nbk) {
      const uint32_t h = hist[d];
      off[d] = h ? carry + ex + atomicAdd(&cursors[d], h) : 0u;
      hist[d] = 0;  // reused as the tile-local rank counter
    }
    carry += tot;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kTileItems; ++j) {
    const int64_t i = base + (int64_t)j * kTileThreads + threadIdx.x;
    if (i < n) {
      const uint32_t d = k[j] >> shift;
      const uint32_t q = off[d] + atomicAdd(&hist[d], 1u);
      if (in_range(q, n)) {
        pk[q] = k[j];
        pv[q] = (int32_t)i;
      }
    }
  }
}

// ------------------------------------------------------------------ dedup
// scratch[b * kH + j] = (local key << 32) | count of the bucket's j-th distinct key
// (ascending), dcount[b] = distinct keys of bucket b.
template <int kH>
__global__ void __launch_bounds__(kBThreads)
pl_dedup_kernel(const uint32_t* __restrict__ pk, int64_t n, int shift,
                const uint32_t* __restrict__ totals, uint64_t* __restrict__ scratch,
                uint32_t* __restrict__ dcount, int32_t* __restrict__ err) {
  constexpr int kHB = __builtin_ctz(kH);
  __shared__ uint64_t sbuf[kH];  // the hash (keys | counts) first, then the sort buffer
  uint32_t* hkey = reinterpret_cast<uint32_t*>(sbuf);
  uint32_t* hcnt = hkey + kH;
  __shared__ uint32_t lds[kBThreads / 64 + 1];
  const int b = blockIdx.x;
  const uint32_t lo = prefix_of<kBThreads>(totals, b, lds);
  const uint32_t hi = lo + totals[b];
  const uint32_t lmask = shift >= 32 ? 0xffffffffu : ((1u << shift) - 1u);
  for (int s = threadIdx.x; s < kH; s += kBThreads) {
    hkey[s] = kEmpty;
    hcnt[s] = 0;
  }
  __syncthreads();
  bool overflow = false;
  const int lane = threadIdx.x & 63;
  for (uint32_t i0 = lo + (threadIdx.x & ~63u); i0 < hi; i0 += kBThreads) {
    const uint32_t i = i0 + lane;
    const bool valid = i < hi && in_range(i, n);
    uint32_t slot = 0;
    bool ok = false;
    if (valid) {
      const uint32_t key = pk[i] & lmask;
      uint32_t h = lhash(key) & (kH - 1);
      for (int p = 0; p < kH; ++p) {
        const uint32_t cur = hkey[h];
        if (cur == key) { ok = true; break; }
        if (cur == kEmpty) {
          const uint32_t prev = atomicCAS(&hkey[h], kEmpty, key);
          if (prev == kEmpty || prev == key) { ok = true; break; }
        }
        h = (h + 1) & (kH - 1);
      }
      slot = h;
      overflow |= !ok;
    }
    const uint64_t act = __ballot(ok);
    const uint64_t peers = match_any(slot, kHB, act);
    if (ok && (peers & ((1ull << lane) - 1ull)) == 0ull)
      atomicAdd(&hcnt[slot], (uint32_t)__popcll(peers));
  }
  if (overflow) atomicOr(err, 1);
  __syncthreads();
  // compact the occupied entries, then sort them by key
  constexpr int kPer = kH / kBThreads;
  uint64_t ent[kPer];
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int s = threadIdx.x * kPer + q;
    ent[q] = hkey[s] != kEmpty ? (((uint64_t)hkey[s] << 32) | hcnt[s]) : ~0ull;
    c += ent[q] != ~0ull;
  }
  uint32_t D;
  uint32_t w = block_excl_scan<kBThreads>(c, lds, &D);  // (every hash read is done)
#pragma unroll
  for (int q = 0; q < kPer; ++q)
    if (ent[q] != ~0ull) sbuf[w++] = ent[q];
  int P = 2;
  while ((uint32_t)P < D) P <<= 1;
  for (int s = (int)D + threadIdx.x; s < P; s += kBThreads) sbuf[s] = ~0ull;
  __syncthreads();
  for (int kk = 2; kk <= P; kk <<= 1) {  // bitonic sort of sbuf[0:P)
    for (int j = kk >> 1; j > 0; j >>= 1) {
      for (int t = threadIdx.x; t < P / 2; t += kBThreads) {
        const int lo_i = ((t / j) * 2 * j) + (t % j);
        const int hi_i = lo_i + j;
        const bool up = (lo_i & kk) == 0;
        const uint64_t a = sbuf[lo_i], bb = sbuf[hi_i];
        if ((a > bb) == up) {
          sbuf[lo_i] = bb;
          sbuf[hi_i] = a;
        }
      }
      __syncthreads();
    }
  }
  for (uint32_t s = threadIdx.x; s < D; s += kBThreads) scratch[(int64_t)b * kH + s] = sbuf[s];
  if (threadIdx.x == 0) dcount[b] = D;
}

// ------------------------------------------------------------------- emit
template <int kH>
__global__ void __launch_bounds__(kBThreads)
pl_emit_kernel(const uint32_t* __restrict__ pk, const int32_t* __restrict__ pv, int64_t n,
               int shift, int nbk, const uint32_t* __restrict__ totals,
               const uint64_t* __restrict__ scratch, const uint32_t* __restrict__ dcount,
               int32_t* __restrict__ pos_s, int32_t* __restrict__ segid,
               uint64_t* __restrict__ uniq, int32_t* __restrict__ seg_start,
               int32_t* __restrict__ local_col, int32_t* __restrict__ n_uniq,
               float* __restrict__ zero_a, float* __restrict__ zero_b, int64_t u_cap) {
  constexpr int kHB = __builtin_ctz(kH);
  __shared__ uint32_t hkey[kH];
  __shared__ uint32_t hval[kH];  // sorted index j of the key
  __shared__ uint32_t cur[kH];   // per-key cursor: occurrence offset within the bucket
  __shared__ uint32_t lds[kBThreads / 64 + 1];
  const int b = blockIdx.x;
  const uint32_t lo = prefix_of<kBThreads>(totals, b, lds);
  const uint32_t hi = lo + totals[b];
  const uint32_t ubase = prefix_of<kBThreads>(dcount, b, lds);
  const uint32_t D = dcount[b] < (uint32_t)kH ? dcount[b] : (uint32_t)kH;
  const uint32_t lmask = shift >= 32 ? 0xffffffffu : ((1u << shift) - 1u);
  for (int s = threadIdx.x; s < kH; s += kBThreads) hkey[s] = kEmpty;
  // occurrence offsets of the sorted distinct keys (exclusive prefix of counts)
  constexpr int kPer = kH / kBThreads;
  uint64_t e[kPer];
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const uint32_t j = threadIdx.x * kPer + q;
    e[q] = j < D ? scratch[(int64_t)b * kH + j] : 0ull;
    c += (uint32_t)(e[q] & 0xffffffffull);
  }
  uint32_t tot;
  uint32_t run = block_excl_scan<kBThreads>(c, lds, &tot);  // (also orders the hkey reset)
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const uint32_t j = threadIdx.x * kPer + q;
    if (j < D) {
      const uint32_t key = (uint32_t)(e[q] >> 32);
      uint32_t h = lhash(key) & (kH - 1);
      for (int p = 0; p < kH; ++p) {
        if (atomicCAS(&hkey[h], kEmpty, key) == kEmpty) break;
        h = (h + 1) & (kH - 1);
      }
      hval[h] = j;
      cur[j] = run;
      const uint64_t u = (uint64_t)ubase + j;
      if (in_range((int64_t)u, u_cap)) {
        uniq[u] = ((uint64_t)b << shift) | key;
        seg_start[u] = (int32_t)(lo + run);
        if (zero_a) zero_a[u] = 0.f;
        if (zero_b) zero_b[u] = 0.f;
      }
      run += (uint32_t)(e[q] & 0xffffffffull);
    }
  }
  if (b == nbk - 1 && threadIdx.x == 0) {
    const uint32_t U = ubase + D;
    *n_uniq = (int32_t)U;
    if (in_range((int64_t)U, u_cap + 1)) seg_start[U] = (int32_t)n;
  }
  __syncthreads();
  const int lane = threadIdx.x & 63;
  for (uint32_t i0 = lo + (threadIdx.x & ~63u); i0 < hi; i0 += kBThreads) {
    const uint32_t i = i0 + lane;
    const bool valid = i < hi && in_range(i, n);
    uint32_t h = 0;
    bool ok = false;
    if (valid) {
      const uint32_t key = pk[i] & lmask;
      h = lhash(key) & (kH - 1);
      for (int p = 0; p < kH; ++p) {
        const uint32_t k2 = hkey[h];
        if (k2 == key) { ok = true; break; }
        if (k2 == kEmpty) break;
        h = (h + 1) & (kH - 1);
      }
    }
    const uint32_t j = ok ? hval[h] : 0u;
    const uint64_t act = __ballot(ok);
    const uint64_t peers = match_any(j, kHB, act);
    const uint64_t below = peers & ((1ull << lane) - 1ull);
    uint32_t rbase = 0;
    if (ok && below == 0ull) rbase = atomicAdd(&cur[j], (uint32_t)__popcll(peers));
    // the group leader's base to every lane of its group
    const int leader = ok ? (int)(__ffsll((long long)peers) - 1) : lane;
    rbase = __shfl(rbase, leader, 64);
    if (ok) {
      const uint32_t q = lo + rbase + (uint32_t)__popcll(below);
      const int32_t p = pv[i];
      const uint32_t u = ubase + j;
      if (in_range(q, n)) {
        pos_s[q] = p;
        segid[q] = (int32_t)(u + 1);
      }
      if (in_range(p, n)) local_col[p] = (int32_t)u;
    }
  }
}

// ---------------------------------------------------------------------------
struct PlGeom {
  int bb, nbk, shift, hcap;
  int64_t tiles;
};

static PlGeom pl_geom(int64_t n, int bits) {
  PlGeom g;
  // average bucket <= hcap / 1.6 occurrences: distinct keys fit even if all distinct
  int bb = 1;
  while (bb < kMaxBB && (n >> bb) > 1250) ++bb;
  g.hcap = (n >> bb) > 1250 ? 4096 : 2048;
  if (bb > bits) bb = bits;
  g.bb = bb;
  g.nbk = 1 << bb;
  g.shift = bits - bb;
  g.tiles = (n + kTile - 1) / kTile;
  return g;
}

size_t partloc_temp_bytes(int64_t n, int bits) {
  const PlGeom g = pl_geom(n, bits);
  return (size_t)kMaxBuckets * 4 * 3 + (size_t)n * 8 + (size_t)g.nbk * g.hcap * 8 + 256;
}

bool partloc_supported(int64_t n, int bits) {
  return bits >= 1 && bits <= 32 && n > 0 && n < (int64_t(1) << 31) &&
         (n >> kMaxBB) <= 2500;
}

void localize_part(const uint64_t* raw, int64_t n, KeyMix m, void* temp, size_t temp_bytes,
                   int32_t* pos_s, int32_t* segid, uint64_t* uniq, int32_t* seg_start,
                   int32_t* local_col, int32_t* n_uniq, float* zero_a, float* zero_b,
                   int32_t* err, int64_t u_cap, hipStream_t st) {
  if (n <= 0) return;
  if (!partloc_supported(n, m.bits)) throw std::runtime_error("localize_part: unsupported size");
  if (temp_bytes < partloc_temp_bytes(n, m.bits))
    throw std::runtime_error("localize_part: temp too small");
  const PlGeom g = pl_geom(n, m.bits);
  char* p = (char*)temp;
  uint32_t* totals = (uint32_t*)p;
  uint32_t* cursors = totals + kMaxBuckets;
  uint32_t* dcount = cursors + kMaxBuckets;
  p += (size_t)kMaxBuckets * 4 * 3;
  uint32_t* pk = (uint32_t*)p;
  p += (size_t)n * 4;
  int32_t* pv = (int32_t*)p;
  p += (size_t)n * 4;
  uint64_t* scratch = (uint64_t*)(((uintptr_t)p + 7) & ~(uintptr_t)7);
  fill_async<uint32_t>(totals, (int64_t)kMaxBuckets * 2, 0u, st);
  pl_count_kernel<<<(unsigned)g.tiles, kTileThreads, 0, st>>>(raw, n, m, g.shift, g.nbk, totals);
  PSAMD_HIP_CHECK(hipGetLastError());
  pl_scatter_kernel<<<(unsigned)g.tiles, kTileThreads, 0, st>>>(raw, n, m, g.shift, g.nbk, totals,
                                                                 cursors, pk, pv);
  PSAMD_HIP_CHECK(hipGetLastError());
  if (g.hcap == 2048) {
    pl_dedup_kernel<2048><<<g.nbk, kBThreads, 0, st>>>(pk, n, g.shift, totals, scratch, dcount,
                                                       err);
    PSAMD_HIP_CHECK(hipGetLastError());
    pl_emit_kernel<2048><<<g.nbk, kBThreads, 0, st>>>(pk, pv, n, g.shift, g.nbk, totals, scratch,
                                                      dcount, pos_s, segid, uniq, seg_start,
                                                      local_col, n_uniq, zero_a, zero_b, u_cap);
  } else {
    pl_dedup_kernel<4096><<<g.nbk, kBThreads, 0, st>>>(pk, n, g.shift, totals, scratch, dcount,
                                                       err);
    PSAMD_HIP_CHECK(hipGetLastError());
    pl_emit_kernel<4096><<<g.nbk, kBThreads, 0, st>>>(pk, pv, n, g.shift, g.nbk, totals, scratch,
                                                      dcount, pos_s, segid, uniq, seg_start,
                                                      local_col, n_uniq, zero_a, zero_b, u_cap);
  }
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
