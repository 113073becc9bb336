// Sort-free minibatch localisation for key spaces of <= 32 bits.
//
// The reference's Localizer (src/util/localizer.h:69-191) sorts (key, pos) pairs
// and run-length encodes them; the radix-sort version of that is the biggest
// cost of a sparse-LR step on the GPU. Deduplication does not need an order:
// here a per-step scratch hash table (resident in the 256 MB Infinity Cache for
// minibatches of a few M keys) assigns compact ids.
//
//   A  insert   thread per nnz: mixed key -> linear probing in slots[C]; an
//               empty or stale slot is claimed with one 64-bit CAS of
//               (epoch << 32 | key). Outputs the slot and a "won" flag.
//   S  scan     exclusive scan of the won flags (chunk sums + per-chunk scan),
//               the scan kernel also publishes id -> (ids[slot], uniq[id]).
//   C  gather   local_col[i] = ids[slot[i]]; bumps the device epoch.
//
// Epoch tagging (epoch = *epoch_dev + 1, all slots start at epoch 0) means the
// table is never cleared; the epoch lives on the device so the whole step stays
// graph-capturable. Ids are dense in [0, U) and ordered by the position of the
// occurrence that claimed each key (which occurrence wins a race is not fixed).
//
// Backward without a CSC order: grad[local_col[i]] += coef[row(i)] through a
// per-block LDS accumulation cache (hot keys reach global memory once per
// block), fp32 atomics for the rest.
#include "common.cuh"

#include <stdexcept>

namespace psamd {

namespace hl {
constexpr int kBlk = 256;
constexpr int kChunk = 2048;  // scan chunk
}  // namespace hl
using namespace hl;

__device__ __forceinline__ uint32_t hl_hash(uint32_t k) {  // keys are already mixed
  return k * 0x9E3779B1u;
}

__global__ void __launch_bounds__(kBlk)
hl_insert_kernel(const uint64_t* __restrict__ raw, int64_t n, KeyMix m,
                 unsigned long long* __restrict__ slots, int64_t cap_mask,
                 const int64_t* __restrict__ epoch_dev, int32_t* __restrict__ slot_of,
                 uint32_t* __restrict__ won, uint32_t* __restrict__ mixed,
                 int32_t* __restrict__ err) {
  const uint64_t epoch = (uint64_t)(*epoch_dev + 1) & 0xffffffffull;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t k = (uint32_t)mix_key(raw[i], m);
    mixed[i] = k;
    const unsigned long long tag = (epoch << 32) | k;
    int64_t p = (int64_t)(hl_hash(k) & (uint32_t)cap_mask);
    uint32_t w = 0;
    int64_t probes = 0;
    while (true) {
      unsigned long long v = slots[p];
      if (v == tag) break;                      // already claimed this step
      if ((v >> 32) != epoch) {                 // empty / stale: try to claim
        const unsigned long long o = atomicCAS(&slots[p], v, tag);
        if (o == v) { w = 1; break; }
        if (o == tag) break;                    // lost to the same key
        continue;                               // lost to another key: re-read p
      }
      p = (p + 1) & cap_mask;
      if (++probes > cap_mask) { atomicExch(err, 1); break; }
    }
    slot_of[i] = (int32_t)p;
    won[i] = w;
  }
}

__device__ __forceinline__ uint32_t hl_block_excl_scan(uint32_t v, uint32_t* lds,
                                                       uint32_t* total) {
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
    for (int w = 0; w < nw; ++w) { const uint32_t t = lds[w]; lds[w] = run; run += t; }
    lds[nw] = run;
  }
  __syncthreads();
  const uint32_t r = x - v + lds[wid];
  *total = lds[nw];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(kBlk)
hl_chunk_sum_kernel(const uint32_t* __restrict__ won, int64_t n, uint32_t* __restrict__ part) {
  __shared__ uint32_t lds[kBlk / 64 + 1];
  const int64_t base = (int64_t)blockIdx.x * kChunk;
  uint32_t s = 0;
#pragma unroll
  for (int j = 0; j < kChunk / kBlk; ++j) {
    const int64_t i = base + j * kBlk + threadIdx.x;
    if (i < n) s += won[i];
  }
  uint32_t tot;
  hl_block_excl_scan(s, lds, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

// Scan of the won flags + publication of the new ids.
__global__ void __launch_bounds__(kBlk)
hl_assign_kernel(const uint32_t* __restrict__ won, const int32_t* __restrict__ slot_of,
                 const uint32_t* __restrict__ mixed, int64_t n, const uint32_t* __restrict__ part,
                 int64_t nchunks, int32_t* __restrict__ ids, int64_t cap,
                 uint64_t* __restrict__ uniq, int32_t* __restrict__ n_uniq,
                 float* __restrict__ zero_a) {
  __shared__ uint32_t lds[kBlk / 64 + 1];
  uint32_t pre = 0;
  for (int64_t c = threadIdx.x; c < (int64_t)blockIdx.x; c += kBlk) pre += part[c];
  uint32_t offset;
  hl_block_excl_scan(pre, lds, &offset);
  constexpr int kPer = kChunk / kBlk;  // 8 consecutive elements per thread
  const int64_t base = (int64_t)blockIdx.x * kChunk + threadIdx.x * kPer;
  uint32_t f[kPer], s = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    f[q] = (base + q < n) ? won[base + q] : 0u;
    s += f[q];
  }
  uint32_t tot;
  uint32_t run = hl_block_excl_scan(s, lds, &tot) + offset;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    if (f[q]) {
      const int32_t sl = slot_of[base + q];
      if (in_range(sl, cap)) ids[sl] = (int32_t)run;
      uniq[run] = mixed[base + q];
      if (zero_a) zero_a[run] = 0.f;
      ++run;
    }
  }
  if (blockIdx.x == nchunks - 1 && threadIdx.x == kBlk - 1) *n_uniq = (int32_t)run;
}

__global__ void __launch_bounds__(kBlk)
hl_gather_kernel(const int32_t* __restrict__ slot_of, int64_t n, const int32_t* __restrict__ ids,
                 int64_t cap, int32_t* __restrict__ local_col, int64_t* __restrict__ epoch_dev) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t sl = slot_of[i];
    local_col[i] = in_range(sl, cap) ? ids[sl] : -1;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) *epoch_dev += 1;  // epoch is read only by A
}

// grad[local_col[i]] += coef[row(i)] * (vals ? vals[i] : 1).
// Each block accumulates a contiguous chunk of nnz into a direct-mapped LDS cache
// of (id, partial) pairs; hot ids (small-cardinality slots) are absorbed in LDS
// and reach global memory once per block, colliding cold ids go straight to a
// global fp32 atomic. Coalesced reads, no order required.
constexpr int kCache = 4096;  // LDS entries (32 KB)
constexpr int kBwdChunk = 16384;  // nnz per block iteration

__global__ void __launch_bounds__(kBlk)
hl_backward_kernel(const int32_t* __restrict__ local_col, int64_t n, int width,
                   const int32_t* __restrict__ rows, const float* __restrict__ vals,
                   const float* __restrict__ coef, int64_t B, float* __restrict__ grad,
                   const int32_t* __restrict__ n_uniq, int64_t grad_cap) {
  __shared__ int32_t tag[kCache];
  __shared__ float part[kCache];
  const int64_t U = dev_len(n_uniq, grad_cap);
  for (int64_t c0 = (int64_t)blockIdx.x * kBwdChunk; c0 < n;
       c0 += (int64_t)gridDim.x * kBwdChunk) {
    for (int e = threadIdx.x; e < kCache; e += kBlk) { tag[e] = -1; part[e] = 0.f; }
    __syncthreads();
    const int64_t c1 = min(n, c0 + kBwdChunk);
    for (int64_t i = c0 + threadIdx.x; i < c1; i += kBlk) {
      const int32_t u = local_col[i];
      const int64_t r = rows ? (int64_t)rows[i] : (int64_t)((uint32_t)i / (uint32_t)width);
      if (!in_range(u, U) || !in_range(r, B)) continue;
      const float g = coef[r] * (vals ? vals[i] : 1.f);
      const int e = (int)(((uint32_t)u * 0x9E3779B1u) >> 20);  // 12-bit index
      int t = tag[e];
      if (t == -1) {
        const int o = atomicCAS(&tag[e], -1, u);
        t = (o == -1) ? u : o;
      }
      if (t == u) atomicAdd(&part[e], g);
      else atomicAdd(&grad[u], g);  // collision: bypass the cache
    }
    __syncthreads();
    for (int e = threadIdx.x; e < kCache; e += kBlk)
      if (tag[e] >= 0) atomicAdd(&grad[tag[e]], part[e]);
    __syncthreads();
  }
}

size_t hashloc_temp_bytes(int64_t n) {
  const int64_t chunks = (n + kChunk - 1) / kChunk;
  return (size_t)n * 12 + (size_t)chunks * 4 + 256;
}

void localize_hash(const uint64_t* raw, int64_t n, KeyMix m, unsigned long long* slots,
                   int32_t* ids, int64_t cap, int64_t* epoch_dev, void* temp, size_t temp_bytes,
                   uint64_t* uniq, int32_t* local_col, int32_t* n_uniq, float* zero_a,
                   int32_t* err, hipStream_t st) {
  if (n <= 0) return;
  if (m.bits > 32) throw std::runtime_error("localize_hash needs key bits <= 32");
  if ((cap & (cap - 1)) != 0 || cap < 2 * n) throw std::runtime_error("hash capacity");
  if (temp_bytes < hashloc_temp_bytes(n)) throw std::runtime_error("hashloc temp too small");
  char* p = (char*)temp;
  int32_t* slot_of = (int32_t*)p;
  p += (size_t)n * 4;
  uint32_t* won = (uint32_t*)p;
  p += (size_t)n * 4;
  uint32_t* mixed = (uint32_t*)p;
  p += (size_t)n * 4;
  uint32_t* part = (uint32_t*)p;
  const int64_t chunks = (n + kChunk - 1) / kChunk;
  hl_insert_kernel<<<grid_for(n, kBlk, 8192), kBlk, 0, st>>>(raw, n, m, slots, cap - 1, epoch_dev,
                                                              slot_of, won, mixed, err);
  PSAMD_HIP_CHECK(hipGetLastError());
  hl_chunk_sum_kernel<<<(unsigned)chunks, kBlk, 0, st>>>(won, n, part);
  PSAMD_HIP_CHECK(hipGetLastError());
  hl_assign_kernel<<<(unsigned)chunks, kBlk, 0, st>>>(won, slot_of, mixed, n, part, chunks, ids,
                                                      cap, uniq, n_uniq, zero_a);
  PSAMD_HIP_CHECK(hipGetLastError());
  hl_gather_kernel<<<grid_for(n, kBlk, 8192), kBlk, 0, st>>>(slot_of, n, ids, cap, local_col,
                                                              epoch_dev);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void hash_backward(const int32_t* local_col, int64_t n, int width, const int32_t* rows,
                   const float* vals, const float* coef, int64_t B, float* grad,
                   const int32_t* n_uniq, int64_t grad_cap, hipStream_t st) {
  if (n <= 0) return;
  const int64_t blocks = (n + kBwdChunk - 1) / kBwdChunk;
  hl_backward_kernel<<<(unsigned)(blocks < 2048 ? blocks : 2048), kBlk, 0, st>>>(
      local_col, n, width, rows, vals, coef, B, grad, n_uniq, grad_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// ----------------------------------------------------------- owner bucketing
// Multi-GPU exchanges need the unique keys grouped by owner shard. With
// sort-free ids they are in claim order, so they are bucketed (G <= 64):
//   count:   per-block LDS counts per owner -> one global atomic per (block, owner)
//   scatter: every block reserves its per-owner runs with one atomic per owner
//            on cursors that start at the owner offsets; keys_out[dst] = uniq[u],
//            perm[dst] = u. Order inside an owner's run is not fixed.
constexpr int kMaxOwners = 64;

__device__ __forceinline__ int owner_of_key(uint64_t x, const uint64_t* __restrict__ bounds,
                                            int G) {
  int lo = 0, hi = G;
  while (hi - lo > 1) {
    const int mid = (lo + hi) >> 1;
    if (bounds[mid] <= x) lo = mid; else hi = mid;
  }
  return lo;
}

__global__ void __launch_bounds__(kBlk)
ob_count_kernel(const uint64_t* __restrict__ uniq, const int32_t* __restrict__ n_uniq,
                int64_t n_host, const uint64_t* __restrict__ bounds, int G,
                unsigned long long* __restrict__ totals) {
  __shared__ uint32_t cnt[kMaxOwners];
  if (threadIdx.x < kMaxOwners) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t U = dev_len(n_uniq, n_host);
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < U;
       i += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[owner_of_key(uniq[i], bounds, G)], 1u);
  __syncthreads();
  if (threadIdx.x < G && cnt[threadIdx.x])
    atomicAdd(&totals[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
}

// totals[0:G] -> offsets[0:G+1] (exclusive) and cursors[0:G] = offsets[0:G]
__global__ void ob_offsets_kernel(const unsigned long long* __restrict__ totals, int G,
                                  int64_t* __restrict__ offsets,
                                  unsigned long long* __restrict__ cursors) {
  if (threadIdx.x != 0) return;
  unsigned long long run = 0;
  for (int g = 0; g < G; ++g) {
    offsets[g] = (int64_t)run;
    cursors[g] = run;
    run += totals[g];
  }
  offsets[G] = (int64_t)run;
}

__global__ void __launch_bounds__(kBlk)
ob_scatter_kernel(const uint64_t* __restrict__ uniq, const int32_t* __restrict__ n_uniq,
                  int64_t n_host, const uint64_t* __restrict__ bounds, int G,
                  unsigned long long* __restrict__ cursors, uint64_t* __restrict__ keys_out,
                  int32_t* __restrict__ perm) {
  __shared__ uint32_t cnt[kMaxOwners];
  __shared__ unsigned long long base[kMaxOwners];
  const int64_t U = dev_len(n_uniq, n_host);
  const int64_t per_block = (int64_t)blockDim.x * 16;
  for (int64_t b0 = (int64_t)blockIdx.x * per_block; b0 < U;
       b0 += (int64_t)gridDim.x * per_block) {
    if (threadIdx.x < kMaxOwners) cnt[threadIdx.x] = 0;
    __syncthreads();
    int own[16];
    uint32_t rk[16];
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int64_t i = b0 + j * blockDim.x + threadIdx.x;
      own[j] = -1;
      if (i < U) {
        own[j] = owner_of_key(uniq[i], bounds, G);
        rk[j] = atomicAdd(&cnt[own[j]], 1u);
      }
    }
    __syncthreads();
    if (threadIdx.x < G && cnt[threadIdx.x])
      base[threadIdx.x] = atomicAdd(&cursors[threadIdx.x], (unsigned long long)cnt[threadIdx.x]);
    __syncthreads();
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      if (own[j] < 0) continue;
      const int64_t i = b0 + j * blockDim.x + threadIdx.x;
      const int64_t dst = (int64_t)(base[own[j]] + rk[j]);
      if (in_range(dst, U)) {
        keys_out[dst] = uniq[i];
        perm[dst] = (int32_t)i;
      }
    }
    __syncthreads();
  }
}

void owner_bucket(const uint64_t* uniq, const int32_t* n_uniq, int64_t n_host,
                  const uint64_t* bounds, int G, void* temp, int64_t* offsets,
                  uint64_t* keys_out, int32_t* perm, hipStream_t st) {
  if (G > kMaxOwners) throw std::runtime_error("owner_bucket: at most 64 shards");
  unsigned long long* totals = (unsigned long long*)temp;
  unsigned long long* cursors = totals + kMaxOwners;
  fill_async<unsigned long long>(totals, kMaxOwners, 0ull, st);
  ob_count_kernel<<<grid_for(n_host, kBlk, 1024), kBlk, 0, st>>>(uniq, n_uniq, n_host, bounds, G,
                                                                  totals);
  PSAMD_HIP_CHECK(hipGetLastError());
  ob_offsets_kernel<<<1, 64, 0, st>>>(totals, G, offsets, cursors);
  PSAMD_HIP_CHECK(hipGetLastError());
  ob_scatter_kernel<<<grid_for(n_host, kBlk * 16, 1024), kBlk, 0, st>>>(
      uniq, n_uniq, n_host, bounds, G, cursors, keys_out, perm);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
