// Tile-deduplicating localisation (mixed key space <= 31 bits).
//
// Reference: Localizer::countUniqIndex / remapIndex (src/util/localizer.h:69-191)
// sort every (key, position) pair of a minibatch. Criteo-shaped minibatches are
// dominated by hot keys: of 65,536 x 39 = 2.55M keys only ~9% are distinct, and
// inside one tile of 4096 consecutive keys (105 rows) about half are repeats.
// So each 256-thread workgroup first collapses its tile in an LDS hash table
// (keys -> tile-local ids, CAS only on a miss), and the global radix sort + RLE
// (sort32.hip, sort_rle32_dev) then runs on the ~half-size set of tile-distinct
// keys; its first pass reads the ragged tiles directly, so no compaction pass.
//
//   tile_dedup      raw u64 -> mix -> LDS hash -> dkeys[b*4096 + r], dcnt[b],
//                   rep[i] (u16 tile-local id of position i), n_ent (atomic total)
//   sort_rle32_dev  (dkeys, fixed-stride id b*4096 + r) -> uniq, CSC order over
//                   entries, ent_uid[b*4096 + r] = unique id
//   tile_gather     local_col[i] = ent_uid[b*4096 + rep[i]]
// Backward (grad[u] = sum over positions of key u of coef[row] * val):
//   tile_bwd_accum  per tile, LDS float atomics into its distinct entries -> psum
//   tile_seg_reduce 64-lane segmented scan of psum over the sorted entries
#include "common.cuh"
#include <stdexcept>
#include <string>

namespace psamd {

namespace tl {
constexpr int kBlk = 256;
constexpr int kItems = 16;
constexpr int kTile = kBlk * kItems;  // 4096 (= the radix-sort tile of sort32.hip)
constexpr int kHash = 2 * kTile;      // load factor <= 0.5
constexpr uint32_t kEmpty = 0xffffffffu;
}  // namespace tl

size_t sort32_dev_temp_bytes(int64_t n_max);
void sort_rle32_dev(const uint32_t* keys_in, const int32_t* tile_cnt, int64_t n_max,
                    const int32_t* n_dev, int bits, int digit_bits, void* temp, size_t temp_bytes,
                    uint32_t* hs, int32_t* pos_s, int32_t* segid, uint64_t* uniq,
                    int32_t* seg_start, int32_t* ent_uid, int64_t p_cap, int32_t* n_uniq,
                    float* zero_a, hipStream_t st);

__device__ __forceinline__ uint32_t tl_hash(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__device__ __forceinline__ uint32_t tl_block_excl_scan(uint32_t v, uint32_t* lds, uint32_t* total) {
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
    for (int w = 0; w < tl::kBlk / 64; ++w) {
      const uint32_t t = lds[w];
      lds[w] = run;
      run += t;
    }
    lds[tl::kBlk / 64] = run;
  }
  __syncthreads();
  const uint32_t r = x - v + lds[wid];
  *total = lds[tl::kBlk / 64];
  __syncthreads();
  return r;
}

__global__ void __launch_bounds__(tl::kBlk)
tile_dedup_kernel(const uint64_t* __restrict__ raw, int64_t n, KeyMix m,
                  uint32_t* __restrict__ dkeys, int32_t* __restrict__ dcnt,
                  uint16_t* __restrict__ rep, int32_t* __restrict__ n_ent) {
  using namespace tl;
  __shared__ uint32_t hk[kHash];
  __shared__ uint16_t hid[kHash];
  __shared__ uint32_t lds[kBlk / 64 + 1];
  const int t = threadIdx.x;
  for (int i = t; i < kHash; i += kBlk) hk[i] = kEmpty;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  uint16_t sl[kItems];
  uint64_t kr[kItems];
#pragma unroll
  for (int j = 0; j < kItems; ++j) {  // all loads in flight before the LDS insert chain
    const int64_t i = base + j * kBlk + t;
    kr[j] = i < n ? raw[i] : 0ull;
  }
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int64_t i = base + j * kBlk + t;
    sl[j] = 0;
    if (i < n) {
      const uint32_t k = (uint32_t)mix_key(kr[j], m);
      uint32_t h = tl_hash(k) & (kHash - 1);
      for (int probe = 0; probe < kHash; ++probe) {  // <= kTile keys: always a free slot
        const uint32_t cur = hk[h];
        if (cur == k) break;
        if (cur == kEmpty) {
          const uint32_t prev = atomicCAS(&hk[h], kEmpty, k);
          if (prev == kEmpty || prev == k) break;
        }
        h = (h + 1) & (kHash - 1);
      }
      sl[j] = (uint16_t)h;
    }
  }
  __syncthreads();
  // compact the occupied slots; thread t owns slots t, t + 256, ... (consecutive
  // lanes -> consecutive banks; ids stay dense in [0, total), order is irrelevant)
  constexpr int kPer = kHash / kBlk;
  uint32_t c = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) c += hk[q * kBlk + t] != kEmpty;
  uint32_t total;
  uint32_t run = tl_block_excl_scan(c, lds, &total);
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int s = q * kBlk + t;
    const uint32_t k = hk[s];
    if (k != kEmpty) {
      hid[s] = (uint16_t)run;
      dkeys[base + run] = k;
      ++run;
    }
  }
  if (t == 0) {
    dcnt[blockIdx.x] = (int32_t)total;
    atomicAdd(n_ent, (int32_t)total);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int64_t i = base + j * kBlk + t;
    if (i < n) rep[i] = hid[sl[j]];
  }
}

__global__ void tile_gather_kernel(const uint16_t* __restrict__ rep,
                                   const int32_t* __restrict__ ent_uid, int64_t n,
                                   int32_t* __restrict__ local_col) {
  constexpr int kPer = 4;  // positions per thread, loads batched
  const int64_t i0 = (blockIdx.x * (int64_t)blockDim.x) * kPer + threadIdx.x;
  int64_t e[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = i0 + q * blockDim.x;
    e[q] = i < n ? (i / tl::kTile) * tl::kTile + rep[i] : -1;
  }
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    const int64_t i = i0 + q * blockDim.x;
    if (e[q] >= 0) local_col[i] = ent_uid[e[q]];
  }
}

__global__ void __launch_bounds__(tl::kBlk)
tile_bwd_accum_kernel(const uint16_t* __restrict__ rep, const int32_t* __restrict__ dcnt, int64_t n,
                      const int32_t* __restrict__ rows, int width, const float* __restrict__ vals,
                      const float* __restrict__ coef, int64_t B, float* __restrict__ psum) {
  using namespace tl;
  __shared__ float acc[kTile];
  const int t = threadIdx.x;
  for (int i = t; i < kTile; i += kBlk) acc[i] = 0.f;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
  float v[kItems];
  uint16_t e[kItems];
#pragma unroll
  for (int j = 0; j < kItems; ++j) {  // gather phase: all loads in flight
    const int64_t i = base + j * kBlk + t;
    v[j] = 0.f;
    e[j] = 0;
    if (i < n) {
      // positions < 2^31: 32-bit division (a 64-bit one is a ~150-instruction call)
      const int64_t r = rows ? (int64_t)rows[i] : (int64_t)((uint32_t)i / (uint32_t)width);
      e[j] = rep[i];
      if (in_range(r, B)) v[j] = coef[r] * (vals ? vals[i] : 1.f);
    }
  }
#pragma unroll
  for (int j = 0; j < kItems; ++j)
    if (v[j] != 0.f) atomicAdd(&acc[e[j]], v[j]);
  __syncthreads();
  const int cnt = min(kTile, max(0, dcnt[blockIdx.x]));
  for (int i = t; i < cnt; i += kBlk) psum[base + i] = acc[i];
}

// grad[segid - 1] = sum of psum[pos_s[i]] over the segment (64-lane segmented scan,
// one atomic per wave piece for segments that cross a wave boundary).
__global__ void __launch_bounds__(256)
tile_seg_reduce_kernel(const int32_t* __restrict__ pos_s, const int32_t* __restrict__ segid,
                       int64_t n_host, const int32_t* __restrict__ n_dev,
                       const float* __restrict__ psum, int64_t p_cap, float* __restrict__ grad,
                       int64_t grad_cap) {
  const int lane = threadIdx.x & 63;
  const int64_t n = dev_len(n_dev, n_host);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < n;
       i0 += stride) {
    const int64_t i = i0 + lane;
    const bool valid = i < n;
    int32_t s = -1;
    float v = 0.f;
    if (valid) {
      s = segid[i];
      const int32_t p = pos_s[i];
      if (in_range(p, p_cap)) v = psum[p];
    }
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float vo = __shfl_up(v, off, 64);
      const int32_t so = __shfl_up(s, off, 64);
      if (lane >= off && so == s) v += vo;
    }
    const int32_t s_next = __shfl_down(s, 1, 64);
    const int32_t s_lane0 = __shfl(s, 0, 64);
    int32_t prev_of_lane0 = -2;
    if (lane == 0 && i0 > 0) prev_of_lane0 = segid[i0 - 1];
    prev_of_lane0 = __shfl(prev_of_lane0, 0, 64);
    const bool tail = valid && (lane == 63 || s_next != s || i + 1 >= n);
    if (tail) {
      const bool starts_inside = (s != s_lane0) || (prev_of_lane0 != s);
      bool ends_inside = true;
      if (lane == 63 && i + 1 < n) ends_inside = segid[i + 1] != s;
      const int32_t u = s - 1;
      if (in_range(u, grad_cap)) {
        if (starts_inside && ends_inside) grad[u] = v;
        else atomicAdd(&grad[u], v);
      }
    }
  }
}

__global__ void tile_zero_kernel(int32_t* __restrict__ p) {
  if (threadIdx.x == 0) *p = 0;
}

// ---------------------------------------------------------------------------
int64_t tileloc_stride(int64_t n) { return ((n + tl::kTile - 1) / tl::kTile) * tl::kTile; }

size_t tileloc_sort_temp_bytes(int64_t n) { return sort32_dev_temp_bytes(tileloc_stride(n)); }

void localize_tile(const uint64_t* raw, int64_t n, KeyMix m, int digit_bits, uint32_t* dkeys,
                   int32_t* dcnt, uint16_t* rep, int32_t* n_ent, void* sort_temp,
                   size_t sort_temp_bytes, uint32_t* hs, int32_t* pos_s, int32_t* segid,
                   uint64_t* uniq, int32_t* seg_start, int32_t* ent_uid, int32_t* local_col,
                   int32_t* n_uniq, float* grad, hipStream_t st) {
  if (n <= 0) return;
  if (m.bits > 31) throw std::runtime_error("localize_tile needs key bits <= 31");
  const int64_t T = (n + tl::kTile - 1) / tl::kTile;
  const int64_t N = T * tl::kTile;
  // a kernel, not hipMemsetAsync: inside a captured graph a memset node may run on
  // a blit/SDMA path and add a cross-engine dependency to the localisation
  tile_zero_kernel<<<1, 64, 0, st>>>(n_ent);
  PSAMD_HIP_CHECK(hipGetLastError());
  tile_dedup_kernel<<<(unsigned)T, tl::kBlk, 0, st>>>(raw, n, m, dkeys, dcnt, rep, n_ent);
  PSAMD_HIP_CHECK(hipGetLastError());
  sort_rle32_dev(dkeys, dcnt, N, n_ent, m.bits, digit_bits, sort_temp, sort_temp_bytes, hs, pos_s,
                 segid, uniq, seg_start, ent_uid, N, n_uniq, grad, st);
  tile_gather_kernel<<<(unsigned)((n + 1023) / 1024), 256, 0, st>>>(rep, ent_uid, n, local_col);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void tile_backward(const uint16_t* rep, const int32_t* dcnt, int64_t n, const int32_t* rows,
                   int width, const float* vals, const float* coef, int64_t B, float* psum,
                   const int32_t* pos_s, const int32_t* segid, const int32_t* n_ent, float* grad,
                   int64_t grad_cap, hipStream_t st) {
  if (n <= 0) return;
  const int64_t T = (n + tl::kTile - 1) / tl::kTile;
  const int64_t N = T * tl::kTile;
  tile_bwd_accum_kernel<<<(unsigned)T, tl::kBlk, 0, st>>>(rep, dcnt, n, rows, width, vals, coef, B,
                                                         psum);
  PSAMD_HIP_CHECK(hipGetLastError());
  tile_seg_reduce_kernel<<<grid_for(N, 256, 8192), 256, 0, st>>>(pos_s, segid, N, n_ent, psum, N,
                                                                 grad, grad_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
