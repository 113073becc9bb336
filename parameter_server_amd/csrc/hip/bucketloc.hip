// Bucketed localisation: one partition pass + per-bucket LDS presence bitmaps.
//
// Same outputs as localize32 (sort32.hip) for key spaces of <= 32 bits — sorted
// unique mixed keys, CSC order (pos_s / segid / seg_start) and the local column of
// every nnz — but without an LSD sort. Measured motivation (Criteo-shaped
// 65,536 x 39 keys over 10^9 features): three 10-bit LSD passes + RLE cost
// ~210 us, of which the digit scatters are latency bound (4 elements per
// digit per tile), while a minibatch holds only ~10% distinct keys.
//
//   K1 bl_hist      mix raw keys, LDS histogram of the top B key bits, one global
//                   atomic per (block, bucket)
//   K2 bl_scan      one block: bucket starts / cursors, reset of the look-back state
//   K3 bl_partition 8K-element tiles: LDS rank within (tile, bucket), one global
//                   cursor reservation per (tile, bucket), scatter (key, position)
//   K4 bl_bucket    one 1024-thread block per bucket (ticket order): an LDS
//                   presence bitmap over the remaining R = bits - B key bits (in
//                   2^18-bit sub-ranges) gives every key its rank among the
//                   bucket's distinct keys with a popcount — unique keys come out
//                   sorted with no comparison sort; the bucket's unique base is a
//                   decoupled look-back over earlier buckets; per-key counts +
//                   an LDS scan give seg_start, a second pass places positions.
//
// Hot keys (a Criteo integer slot value can occur in most rows) make a few
// buckets large and all their lanes hit the same LDS counter: the count/slot
// atomics are wave-aggregated on the first active lane's key (one ballot).
// Within one key's segment the order of positions is not deterministic (LDS
// atomics); everything else is. Heavy-bucket blocks stream their elements with
// 1024 threads and 4 independent loads per thread in flight.
#include "common.cuh"
#include <stdexcept>

namespace psamd {

namespace bl {
constexpr int kMaxBucketBits = 12;
constexpr int kMaxBuckets = 1 << kMaxBucketBits;
constexpr int kHistBlk = 512;
constexpr int kPartBlk = 1024;
constexpr int kPartItems = 8;
constexpr int kPartTile = kPartBlk * kPartItems;  // 8192 (313 tiles for 2.56M keys)
constexpr int kBkBlk = 1024;
constexpr int kBkWaves = kBkBlk / 64;
constexpr int kSubBits = 18;
constexpr int kWords = (1 << kSubBits) / 32;  // 8192 bitmap words = 32 KB
constexpr int kCntCap = 3584;                 // per-key counters per chunk (2 blocks/CU fit)
constexpr int kUnroll = 4;
constexpr unsigned long long kFlagAgg = 1ull << 32, kFlagIncl = 2ull << 32;
}  // namespace bl
using namespace bl;

namespace {

// Exclusive block scan of one u32 per thread (any multiple of 64 threads).
__device__ __forceinline__ uint32_t bl_excl_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
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
    for (int w = 0; w < nw; ++w) {
      const uint32_t t = lds[w];
      lds[w] = run;
      run += t;
    }
    lds[nw] = run;
  }
  __syncthreads();
  const uint32_t r = x - v + lds[wid];
  *total = lds[nw];
  __syncthreads();
  return r;
}

// atomicAdd(&cnt[idx], 1) for every active lane, returning the old value, with the
// lanes that share the first active lane's idx folded into one LDS atomic. Must
// be called by all lanes of the wave.
__device__ __forceinline__ uint32_t agg_inc(uint32_t* cnt, uint32_t idx, bool active) {
  const uint64_t act = __ballot(active);
  if (act == 0) return 0;
  const int lane = threadIdx.x & 63;
  const int lead = __ffsll((long long)act) - 1;
  const uint32_t lidx = __shfl(idx, lead, 64);
  const bool same = active && idx == lidx;
  const uint64_t sm = __ballot(same);
  uint32_t base = 0;
  if (lane == lead) base = atomicAdd(&cnt[lidx], (uint32_t)__popcll(sm));
  base = __shfl(base, lead, 64);
  if (same) return base + (uint32_t)__popcll(sm & ((1ull << lane) - 1ull));
  return active ? atomicAdd(&cnt[idx], 1u) : 0u;
}

__global__ void __launch_bounds__(kHistBlk) bl_hist_kernel(const uint64_t* __restrict__ raw,
                                                           int64_t n, KeyMix m, int R, int nbk,
                                                           uint32_t* __restrict__ count) {
  __shared__ uint32_t h[kMaxBuckets];
  for (int i = threadIdx.x; i < nbk; i += kHistBlk) h[i] = 0;
  __syncthreads();
  const int64_t stride = (int64_t)gridDim.x * kHistBlk;
  for (int64_t i = (int64_t)blockIdx.x * kHistBlk + threadIdx.x; i < n; i += stride) {
    const uint32_t k = (uint32_t)mix_key(raw[i], m);
    atomicAdd(&h[k >> R], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < nbk; i += kHistBlk)
    if (h[i]) atomicAdd(&count[i], h[i]);
}

// 1024 threads, nbk <= 4096 buckets (4 per thread).
__global__ void __launch_bounds__(1024) bl_scan_kernel(const uint32_t* __restrict__ count, int nbk,
                                                       uint32_t* __restrict__ start,
                                                       uint32_t* __restrict__ cursor,
                                                       unsigned long long* __restrict__ status,
                                                       uint32_t* __restrict__ ticket) {
  __shared__ uint32_t lds[17];
  const int t = threadIdx.x;
  uint32_t c[4], s = 0;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = t * 4 + j;
    c[j] = d < nbk ? count[d] : 0u;
    s += c[j];
  }
  uint32_t total;
  uint32_t run = bl_excl_scan(s, lds, &total);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int d = t * 4 + j;
    if (d < nbk) {
      start[d] = run;
      cursor[d] = run;
      status[d] = 0ull;
    }
    run += c[j];
  }
  if (t == 0) {
    start[nbk] = total;
    *ticket = 0u;
  }
}

__global__ void __launch_bounds__(kPartBlk) bl_partition_kernel(
    const uint64_t* __restrict__ raw, int64_t n, KeyMix m, int R, int nbk,
    uint32_t* __restrict__ cursor, uint32_t* __restrict__ kp, int32_t* __restrict__ pp) {
  __shared__ uint32_t cnt[kMaxBuckets];
  __shared__ uint32_t base[kMaxBuckets];
  const int t = threadIdx.x;
  const int64_t tb = (int64_t)blockIdx.x * kPartTile;
  for (int i = t; i < nbk; i += kPartBlk) cnt[i] = 0;
  __syncthreads();
  uint32_t k[kPartItems], r[kPartItems];
#pragma unroll
  for (int j = 0; j < kPartItems; ++j) {
    const int64_t i = tb + j * kPartBlk + t;
    if (i < n) {
      k[j] = (uint32_t)mix_key(raw[i], m);
      r[j] = atomicAdd(&cnt[k[j] >> R], 1u);
    }
  }
  __syncthreads();
#pragma unroll 4
  for (int d = t; d < nbk; d += kPartBlk) {
    const uint32_t c = cnt[d];
    base[d] = c ? atomicAdd(&cursor[d], c) : 0u;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kPartItems; ++j) {
    const int64_t i = tb + j * kPartBlk + t;
    if (i < n) {
      const uint32_t q = base[k[j] >> R] + r[j];
      if (q < (uint64_t)n) {
        kp[q] = k[j];
        pp[q] = (int32_t)i;
      }
    }
  }
}

struct BucketOut {
  uint64_t* uniq;
  int32_t* seg_start;
  int32_t* pos_s;
  int32_t* segid;
  int32_t* local_col;
  int32_t* n_uniq;
  float* za;
  float* zb;
  unsigned long long* dbg;  // optional per-bucket timestamps [nbk][5] (profiling)
};

__global__ void __launch_bounds__(kBkBlk) bl_bucket_kernel(
    const uint32_t* __restrict__ kp, const int32_t* __restrict__ pp,
    const uint32_t* __restrict__ start, int nbk, int R, int SUB, int nsub,
    uint32_t* __restrict__ ticket, unsigned long long* __restrict__ status, int64_t n,
    BucketOut o) {
  __shared__ uint32_t bm[kWords];
  __shared__ uint32_t wpre[kWords];
  __shared__ uint32_t cnt[kCntCap];
  __shared__ uint32_t red[kBkWaves + 1];
  __shared__ uint32_t sh_b;
  __shared__ uint32_t sh_prefix;
  const int t = threadIdx.x;
  if (t == 0) sh_b = atomicAdd(ticket, 1u);
  __syncthreads();
  const int b = (int)sh_b;
  if (b >= nbk) return;  // uniform: grid == nbk, never taken
  if (o.dbg && t == 0) o.dbg[b * 5 + 0] = wall_clock64();
  const uint32_t e0 = start[b], e1 = min(start[b + 1], (uint32_t)n);
  const uint32_t rem_mask = R == 0 ? 0u : (R >= 32 ? ~0u : ((1u << R) - 1u));
  const uint32_t sub_mask = SUB == 0 ? 0u : ((1u << SUB) - 1u);
  const int W = SUB >= 5 ? (1 << (SUB - 5)) : 1;
  const int wpt = (W + kBkBlk - 1) / kBkBlk;  // bitmap words per thread (contiguous)

  auto build_bitmap = [&](int s) {
    for (int w = t; w < W; w += kBkBlk) bm[w] = 0u;
    __syncthreads();
    for (uint32_t e = e0 + t; e < e1; e += kBkBlk) {
      const uint32_t rem = kp[e] & rem_mask;
      if ((int)(rem >> SUB) != s) continue;
      const uint32_t x = rem & sub_mask;
      const uint32_t bit = 1u << (x & 31);
      uint32_t* word = &bm[x >> 5];
      if (!(*word & bit)) atomicOr(word, bit);
    }
    __syncthreads();
  };

  // ---- phase A: distinct keys in the bucket (bitmap kept when nsub == 1)
  uint32_t Ub = 0;
  for (int s = 0; s < nsub; ++s) {
    build_bitmap(s);
    uint32_t c = 0;
    for (int q = 0; q < wpt; ++q) {
      const int w = t * wpt + q;
      if (w < W) c += (uint32_t)__popc(bm[w]);
    }
    uint32_t tot;
    bl_excl_scan(c, red, &tot);
    Ub += tot;
  }
  // ---- decoupled look-back over earlier buckets (ticket order == bucket order)
  if (o.dbg && t == 0) o.dbg[b * 5 + 1] = wall_clock64();
  if (t == 0) {
    __hip_atomic_store(&status[b], kFlagAgg | Ub, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
    unsigned long long excl = 0;
    for (int j = b - 1; j >= 0; --j) {
      unsigned long long s;
      do {
        s = __hip_atomic_load(&status[j], __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT);
      } while ((s >> 32) == 0ull);
      excl += s & 0xffffffffull;
      if ((s >> 32) == 2ull) break;
    }
    __hip_atomic_store(&status[b], kFlagIncl | (excl + Ub), __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_AGENT);
    sh_prefix = (uint32_t)excl;
    if (o.dbg) o.dbg[b * 5 + 2] = wall_clock64();
  }
  __syncthreads();
  uint32_t ubase = sh_prefix;
  uint32_t ebase = e0;

  for (int s = 0; s < nsub; ++s) {
    if (nsub > 1) build_bitmap(s);
    // per-word exclusive prefix of set bits
    uint32_t c = 0;
    for (int q = 0; q < wpt; ++q) {
      const int w = t * wpt + q;
      if (w < W) c += (uint32_t)__popc(bm[w]);
    }
    uint32_t Us;
    uint32_t run = bl_excl_scan(c, red, &Us);
    for (int q = 0; q < wpt; ++q) {
      const int w = t * wpt + q;
      if (w < W) {
        const uint32_t x = bm[w];
        wpre[w] = run;
        // unique keys of this word, in ascending order
        uint32_t y = x, r = run;
        while (y) {
          const int bit = __ffs(y) - 1;
          y &= y - 1u;
          const uint32_t u = ubase + r++;
          if (u < (uint64_t)n) {
            const uint64_t key = ((uint64_t)b << R) | ((uint64_t)s << SUB) |
                                 (uint64_t)((uint32_t)w * 32u + (uint32_t)bit);
            o.uniq[u] = key;
            if (o.za) o.za[u] = 0.f;
            if (o.zb) o.zb[u] = 0.f;
          }
        }
        run += (uint32_t)__popc(x);
      }
    }
    __syncthreads();
    for (uint32_t c0 = 0; c0 < Us; c0 += kCntCap) {
      const uint32_t cn = min((uint32_t)kCntCap, Us - c0);
      for (uint32_t i = t; i < cn; i += kBkBlk) cnt[i] = 0u;
      __syncthreads();
      // pass 1: counts per key + local columns
      for (uint32_t e = e0; e < e1; e += kBkBlk * kUnroll) {
        uint32_t kk[kUnroll];
        int32_t pq[kUnroll];
#pragma unroll
        for (int j = 0; j < kUnroll; ++j) {
          const uint32_t ei = e + j * kBkBlk + t;
          kk[j] = ei < e1 ? kp[ei] : ~0u;
          pq[j] = ei < e1 ? pp[ei] : -1;
        }
#pragma unroll
        for (int j = 0; j < kUnroll; ++j) {
          const uint32_t rem = kk[j] & rem_mask;
          bool act = pq[j] >= 0 && (int)(rem >> SUB) == s;
          uint32_t u = 0;
          if (act) {
            const uint32_t x = rem & sub_mask, w = x >> 5;
            u = wpre[w] + (uint32_t)__popc(bm[w] & ((1u << (x & 31)) - 1u));
            act = u >= c0 && u < c0 + cn;
          }
          agg_inc(cnt, u - c0, act);
          if (act && in_range(pq[j], n)) o.local_col[pq[j]] = (int32_t)(ubase + u);
        }
      }
      __syncthreads();
      // exclusive scan of the counts -> segment starts
      const int cpt = ((int)cn + kBkBlk - 1) / kBkBlk;
      uint32_t cs = 0;
      for (int q = 0; q < cpt; ++q) {
        const int i = t * cpt + q;
        if (i < (int)cn) cs += cnt[i];
      }
      uint32_t Ec;
      uint32_t cr = bl_excl_scan(cs, red, &Ec);
      for (int q = 0; q < cpt; ++q) {
        const int i = t * cpt + q;
        if (i < (int)cn) {
          const uint32_t v = cnt[i];
          cnt[i] = cr;
          const uint32_t u = ubase + c0 + i;
          if (u < (uint64_t)n) o.seg_start[u] = (int32_t)(ebase + cr);
          cr += v;
        }
      }
      __syncthreads();
      // pass 2: place positions in key order
      for (uint32_t e = e0; e < e1; e += kBkBlk * kUnroll) {
        uint32_t kk[kUnroll];
        int32_t pq[kUnroll];
#pragma unroll
        for (int j = 0; j < kUnroll; ++j) {
          const uint32_t ei = e + j * kBkBlk + t;
          kk[j] = ei < e1 ? kp[ei] : ~0u;
          pq[j] = ei < e1 ? pp[ei] : -1;
        }
#pragma unroll
        for (int j = 0; j < kUnroll; ++j) {
          const uint32_t rem = kk[j] & rem_mask;
          bool act = pq[j] >= 0 && (int)(rem >> SUB) == s;
          uint32_t u = 0;
          if (act) {
            const uint32_t x = rem & sub_mask, w = x >> 5;
            u = wpre[w] + (uint32_t)__popc(bm[w] & ((1u << (x & 31)) - 1u));
            act = u >= c0 && u < c0 + cn;
          }
          const uint32_t slot = agg_inc(cnt, u - c0, act);
          const uint32_t q = ebase + slot;
          if (act && q < (uint64_t)n) {
            o.pos_s[q] = pq[j];
            o.segid[q] = (int32_t)(ubase + u + 1);
          }
        }
      }
      __syncthreads();
      ebase += Ec;
    }
    ubase += Us;
  }
  if (o.dbg && t == 0) {
    o.dbg[b * 5 + 3] = wall_clock64();
    o.dbg[b * 5 + 4] = e1 - e0;
  }
  if (b == nbk - 1 && t == 0) {
    *o.n_uniq = (int32_t)ubase;
    if (ubase <= (uint64_t)n) o.seg_start[ubase] = (int32_t)n;
  }
}

inline int bucket_bits(int bits) { return bits < kMaxBucketBits ? bits : kMaxBucketBits; }

}  // namespace

// Workspace: count[4096] start[4097] cursor[4096] status[4096] u64, ticket, kp[n], pp[n].
size_t bucketloc_temp_bytes(int64_t n) {
  return (size_t)kMaxBuckets * 4 * 3 + 64 + (size_t)kMaxBuckets * 8 + 64 + (size_t)n * 8 + 256;
}

void localize_bucket(const uint64_t* raw, int64_t n, KeyMix m, void* temp, size_t temp_bytes,
                     int32_t* pos_s, int32_t* segid, uint64_t* uniq, int32_t* seg_start,
                     int32_t* local_col, int32_t* n_uniq, float* zero_a, float* zero_b,
                     unsigned long long* dbg, hipStream_t st) {
  if (n <= 0) return;
  if (m.bits > 32) throw std::runtime_error("localize_bucket needs key bits <= 32");
  if (n >= (int64_t)0x7fffffff) throw std::runtime_error("localize_bucket: n < 2^31");
  if (temp_bytes < bucketloc_temp_bytes(n))
    throw std::runtime_error("localize_bucket temp too small");
  const int B = bucket_bits(m.bits);
  const int nbk = 1 << B;
  const int R = m.bits - B;
  const int SUB = R < kSubBits ? R : kSubBits;
  const int nsub = 1 << (R - SUB);
  char* p = (char*)temp;
  uint32_t* count = (uint32_t*)p;
  p += (size_t)kMaxBuckets * 4;
  uint32_t* start = (uint32_t*)p;
  p += (size_t)kMaxBuckets * 4 + 64;
  uint32_t* cursor = (uint32_t*)p;
  p += (size_t)kMaxBuckets * 4;
  unsigned long long* status = (unsigned long long*)p;
  p += (size_t)kMaxBuckets * 8;
  uint32_t* ticket = (uint32_t*)p;
  p += 64;
  uint32_t* kp = (uint32_t*)p;
  p += (size_t)n * 4;
  int32_t* pp = (int32_t*)p;

  fill_async<uint32_t>(count, nbk, 0u, st);
  const int gh = grid_for(n, kHistBlk, 512);
  bl_hist_kernel<<<gh, kHistBlk, 0, st>>>(raw, n, m, R, nbk, count);
  PSAMD_HIP_CHECK(hipGetLastError());
  bl_scan_kernel<<<1, 1024, 0, st>>>(count, nbk, start, cursor, status, ticket);
  PSAMD_HIP_CHECK(hipGetLastError());
  const unsigned tiles = (unsigned)((n + kPartTile - 1) / kPartTile);
  bl_partition_kernel<<<tiles, kPartBlk, 0, st>>>(raw, n, m, R, nbk, cursor, kp, pp);
  PSAMD_HIP_CHECK(hipGetLastError());
  BucketOut o{uniq, seg_start, pos_s, segid, local_col, n_uniq, zero_a, zero_b, dbg};
  bl_bucket_kernel<<<(unsigned)nbk, kBkBlk, 0, st>>>(kp, pp, start, nbk, R, SUB, nsub, ticket,
                                                     status, n, o);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
