// CountMin sketch cells shared by the filter kernels (filters.hip) and the flat
// localiser's fused tail filter (tploc.hip).
//
// Reference CountMin<K, uint8> (src/util/countmin.h:8-48): k probes by double hashing of
// the 64->32 sketch hash (src/util/sketch.h:20-33), saturating uint8 counters (v_max 254,
// src/parameter/frequency_filter.h:17). Cells are bytes packed in 32-bit words and updated
// by a CAS on the word, so concurrent inserts of keys sharing a word lose nothing.
//
// Partitioned layout (the GPU trainers'): the sketch is 2^lgR regions of `rsize` cells
// (a multiple of 64: regions never share a line), and a key's k cells all lie in region
// (mixed key >> rshift), inside ONE 64-cell block of it (blocked CountMin: block h mod
// (rsize / 64), offsets o_j = (h2 + j * d2) mod 64 with d2 odd, from the double-hash step):
// a key touches one cache line of the 100 MB-class sketch instead of k. The flat localiser's bucket workgroups own whole key ranges,
// hence whole regions, so one workgroup can insert its keys and then query them after a
// workgroup barrier: every insert that can touch a key's cells came from the same
// workgroup (no grid-wide barrier between the reference's insertKeys and queryKeys).
// rshift >= 64: one region (the reference's global layout; CPU runtime apps).
#pragma once
#include "common.cuh"

namespace psamd {

__host__ __device__ __forceinline__ uint32_t sketch_hash(uint64_t key) {
  const uint32_t seed = 0xbc9f1d34u, m = 0xc6a4a793u;
  uint32_t h = seed ^ (8u * m);
  h += (uint32_t)key; h *= m; h ^= h >> 16;
  h += (uint32_t)(key >> 32); h *= m; h ^= h >> 16;
  return h;
}

struct CmArgs {
  uint32_t* cells;   // byte cells, as words
  uint64_t rsize;    // cells per region
  int rshift;        // region = key >> rshift (>= 64: one region)
  int k;             // probes
  uint32_t vmax;     // saturation
  int freq;          // keep keys whose estimate > freq
  int ncells32;      // every cell index < 2^32 (the batched forms' 32-bit indices)
};

__host__ __device__ __forceinline__ uint64_t cm_base(uint64_t key, int rshift, uint64_t rsize) {
  return rshift >= 64 ? 0ull : (key >> rshift) * rsize;
}

constexpr int kCmBlock = 64;  // cells of a block (partitioned layout)

// cell j of a key: the reference's double hashing over the whole table (rshift >= 64), or
// inside the key's block of its region (partitioned)
struct CmProbe {
  uint64_t base;  // first cell of the key's block (partitioned) or 0
  uint32_t h, delta, o, d2;
  __host__ __device__ __forceinline__ CmProbe(uint64_t key, int rshift, uint64_t rsize) {
    h = sketch_hash(key);
    delta = (h >> 17) | (h << 15);
    base = cm_base(key, rshift, rsize);
    o = delta & (kCmBlock - 1);
    d2 = ((delta >> 6) & (kCmBlock - 1)) | 1u;
    if (rshift < 64) base += (uint64_t)(h % (uint32_t)(rsize / kCmBlock)) * kCmBlock;
  }
  // the next cell (call k times)
  __host__ __device__ __forceinline__ uint64_t next(int rshift, uint64_t rsize) {
    uint64_t c;
    if (rshift >= 64) {
      c = h % rsize;
      h += delta;
    } else {
      c = base + o;
      o = (o + d2) & (kCmBlock - 1);
    }
    return c;
  }
};

__device__ __forceinline__ uint32_t sat_add_byte(uint32_t* table, uint64_t cell, uint32_t cnt,
                                                 uint32_t vmax) {
  uint32_t* word = table + (cell >> 2);
  const int sh = (int)(cell & 3) * 8;
  uint32_t old = __hip_atomic_load(word, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  while (true) {
    const uint32_t b = (old >> sh) & 0xffu;
    const uint32_t nb = (cnt > vmax - b) ? vmax : b + cnt;
    if (nb == b) return b;
    const uint32_t nw = (old & ~(0xffu << sh)) | (nb << sh);
    const uint32_t prev = atomicCAS(word, old, nw);
    if (prev == old) return nb;
    old = prev;
  }
}

__device__ __forceinline__ void cm_insert_key(const CmArgs& a, uint64_t key, uint32_t cnt) {
  if (cnt == 0) return;
  CmProbe p(key, a.rshift, a.rsize);
  for (int j = 0; j < a.k; ++j) sat_add_byte(a.cells, p.next(a.rshift, a.rsize), cnt, a.vmax);
}

// min over the key's cells (agent-scope loads: they see every insert that completed
// before, whatever this CU's L1 holds)
__device__ __forceinline__ uint32_t cm_query_key(const CmArgs& a, uint64_t key) {
  CmProbe p(key, a.rshift, a.rsize);
  uint32_t res = a.vmax;
  for (int j = 0; j < a.k; ++j) {
    const uint64_t c = p.next(a.rshift, a.rsize);
    const uint32_t w = __hip_atomic_load(a.cells + (c >> 2), __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT);
    const uint32_t v = (w >> ((c & 3) * 8)) & 0xffu;
    res = v < res ? v : res;
  }
  return res;
}

// Batched forms for a thread holding several keys (the flat localiser's fused filter):
// every cell's word load, then every CAS, are issued before any result is used, so a
// thread pays ~2 memory round trips for all its keys instead of 2 per probe (a dependent
// chain of 16 for 4 keys x 2 probes). A CAS that lost a race (another key on the same
// word) retries alone. Exactly kCmBatchK probes (the reference default k = 2; other k:
// the one-key forms). Word indices and region sizes are 32-bit (the caller checks).
constexpr int kCmBatchK = 2;

template <int kN>
__device__ __forceinline__ void cm_cells_batch(const CmArgs& a, const uint64_t (&key)[kN],
                                               uint32_t (&cell)[kN][kCmBatchK]) {
  const uint32_t rs = (uint32_t)a.rsize;  // (32-bit cell indices: the caller checks)
  const bool part = a.rshift < 64;
#pragma unroll
  for (int q = 0; q < kN; ++q) {
    uint32_t base = (uint32_t)cm_base(key[q], a.rshift, a.rsize);
    uint32_t h = sketch_hash(key[q]);
    const uint32_t delta = (h >> 17) | (h << 15);
    if (part) {  // (CmProbe, 32-bit)
      base += (h % (rs / kCmBlock)) * kCmBlock;
      const uint32_t d2 = ((delta >> 6) & (kCmBlock - 1)) | 1u;
      uint32_t o = delta & (kCmBlock - 1);
#pragma unroll
      for (int j = 0; j < kCmBatchK; ++j) {
        cell[q][j] = base + o;
        o = (o + d2) & (kCmBlock - 1);
      }
    } else {
#pragma unroll
      for (int j = 0; j < kCmBatchK; ++j) {
        cell[q][j] = base + h % rs;
        h += delta;
      }
    }
  }
}

template <int kN>
__device__ __forceinline__ void cm_insert_batch(const CmArgs& a, const uint64_t (&key)[kN],
                                                const uint32_t (&cnt)[kN], uint32_t valid) {
  uint32_t cell[kN][kCmBatchK], old[kN][kCmBatchK];
  cm_cells_batch<kN>(a, key, cell);
#pragma unroll
  for (int q = 0; q < kN; ++q)
#pragma unroll
    for (int j = 0; j < kCmBatchK; ++j)
      old[q][j] = ((valid >> q) & 1u) && cnt[q]
                      ? __hip_atomic_load(a.cells + (cell[q][j] >> 2), __ATOMIC_RELAXED,
                                          __HIP_MEMORY_SCOPE_AGENT)
                      : 0u;
  uint32_t lost = 0;  // bit q * K + j: that CAS lost a race
#pragma unroll
  for (int q = 0; q < kN; ++q)
#pragma unroll
    for (int j = 0; j < kCmBatchK; ++j)
      if (((valid >> q) & 1u) && cnt[q]) {
        const uint32_t sh = (cell[q][j] & 3u) * 8u;
        const uint32_t b = (old[q][j] >> sh) & 0xffu;
        const uint32_t nb = (cnt[q] > a.vmax - b) ? a.vmax : b + cnt[q];
        if (nb != b && atomicCAS(a.cells + (cell[q][j] >> 2), old[q][j],
                                 (old[q][j] & ~(0xffu << sh)) | (nb << sh)) != old[q][j])
          lost |= 1u << (q * kCmBatchK + j);
      }
#pragma unroll
  for (int q = 0; q < kN; ++q)
#pragma unroll
    for (int j = 0; j < kCmBatchK; ++j)
      if ((lost >> (q * kCmBatchK + j)) & 1u)
        sat_add_byte(a.cells, cell[q][j], cnt[q], a.vmax);  // (lost a race: retry alone)
}

// min over each key's cells, all loads in flight together
template <int kN>
__device__ __forceinline__ void cm_query_batch(const CmArgs& a, const uint64_t (&key)[kN],
                                               uint32_t valid, uint32_t (&res)[kN]) {
  uint32_t cell[kN][kCmBatchK], w[kN][kCmBatchK];
  cm_cells_batch<kN>(a, key, cell);
#pragma unroll
  for (int q = 0; q < kN; ++q)
#pragma unroll
    for (int j = 0; j < kCmBatchK; ++j)
      w[q][j] = (valid >> q) & 1u ? __hip_atomic_load(a.cells + (cell[q][j] >> 2),
                                                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                  : 0u;
#pragma unroll
  for (int q = 0; q < kN; ++q) {
    uint32_t r = a.vmax;
#pragma unroll
    for (int j = 0; j < kCmBatchK; ++j) {
      const uint32_t v = (w[q][j] >> ((cell[q][j] & 3u) * 8u)) & 0xffu;
      r = v < r ? v : r;
    }
    res[q] = r;
  }
}

}  // namespace psamd
