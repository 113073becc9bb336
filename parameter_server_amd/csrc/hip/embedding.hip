// Embedding-table (dense value block) kernels for the wide & deep model.
//
// A shard's table = the scalar KV table (32-B slots: key | wide w, z, n ...;
// csrc/hip/kv_table.hip) + a row block rows[capacity, D] (bf16) addressed by
// the SAME slot index, + a per-row AdaGrad accumulator and an init flag.
// D = 128 bf16 = 256 B = 16 lanes x 16 B: every kernel maps one key / row to a
// 16-lane group (4 groups per wave64) doing 16-byte vector loads and stores.
//
//   emb_init_rows    first touch of a slot -> deterministic N(0, s) row from its key
//   emb_gather_rows  rows[slot[i]] -> out[i]          (pull replies, G > 1)
//   emb_expand       X0[p] = src[idx[p]], p = b*S + s (the [B, S*D] MLP input)
//   emb_grad_reduce  dE[u] = sum of dX0 rows of u's occurrences (CSC order of the
//                    localiser, 64-entry runs per wavefront: no atomics, fp32
//                    accumulation, deterministic cross-run partials)
//   emb_update       row-wise AdaGrad: acc += mean(g^2); row -= lr g / sqrt(acc + eps)
//   wd_head          deep logit (h.w + b) + wide margin, logistic loss, metrics,
//                    AUC histogram, dL/dlogit, dh = coef w * relu'(h), db
//   colred_bf16      column reductions: dw = h^T coef, the last hidden layer's bias
//                    gradient, plain column sums (library-GEMM backend)
//   adam_update      fp32 master weights + bf16 copy for the GEMMs
#include "common.cuh"
#include "kv_slot.cuh"

#include <algorithm>
#include <cstdlib>

#include <hip/hip_bf16.h>

namespace psamd {

namespace {

constexpr int kGroup = 16;  // lanes per row

__device__ __forceinline__ float bf2f(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {  // round to nearest even, NaN kept
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}

__device__ __forceinline__ float group_sum(float v) {
#pragma unroll
  for (int o = kGroup / 2; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ---------------------------------------------------------------- init / gather
// deterministic N(0, scale) row of a key (16-lane group, lane l), then the init flag
__device__ __forceinline__ void init_row(uint16_t* __restrict__ rows, int64_t s, uint64_t key,
                                         int D, uint64_t seed, float scale, int l,
                                         uint8_t* __restrict__ inited) {
  for (int d = l; d < D; d += kGroup) {  // Box-Muller on a counter-based stream
    const uint64_t r = rng64(seed ^ key, (uint64_t)d);
    const float u1 = ((r >> 40) + 1) * (1.f / 16777217.f);
    const float u2 = ((r >> 16) & 0xffffff) * (1.f / 16777216.f);
    const float z = sqrtf(-2.f * logf(u1)) * cospif(2.f * u2);
    rows[s * D + d] = f2bf(z * scale);
  }
  __threadfence_block();
  if (l == 0) inited[s] = 1;  // racing duplicates write identical rows
}

__global__ void __launch_bounds__(256)
emb_init_rows_kernel(const int64_t* __restrict__ slot, const uint64_t* __restrict__ keys, int64_t n,
                     const int32_t* __restrict__ n_dev, int64_t cap, uint16_t* __restrict__ rows,
                     uint8_t* __restrict__ inited, int D, uint64_t seed, float scale) {
  // kIR keys per group per round, their slot and flag loads issued together at clamped
  // in-range addresses (one key per round was two dependent round trips per key)
  constexpr int kIR = 4;
  const int64_t nn = dev_len(n_dev, n);
  if (nn <= 0) return;
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  const int64_t stride = (int64_t)gridDim.x * (blockDim.x / kGroup);
  for (int64_t i0 = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; i0 < nn; i0 += kIR * stride) {
    int64_t sv[kIR];
#pragma unroll
    for (int q = 0; q < kIR; ++q) sv[q] = slot[min(i0 + q * stride, nn - 1)];
    uint8_t fv[kIR];
#pragma unroll
    for (int q = 0; q < kIR; ++q) fv[q] = inited[in_range(sv[q], cap) ? sv[q] : 0];
#pragma unroll
    for (int q = 0; q < kIR; ++q) {
      const int64_t i = i0 + q * stride;
      if (i < nn && in_range(sv[q], cap) && !fv[q])
        init_row(rows, sv[q], keys[i], D, seed, scale, l, inited);
    }
  }
}

__global__ void __launch_bounds__(256)
emb_gather_rows_kernel(const int64_t* __restrict__ slot, int64_t n_host,
                       const int32_t* __restrict__ n_dev, int64_t cap,
                       const uint16_t* __restrict__ rows, int D, uint16_t* __restrict__ out) {
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  const int vec = D / 8;  // 16-B vectors per row
  const int64_t n = dev_len(n_dev, n_host);
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; i < n;
       i += (int64_t)gridDim.x * (blockDim.x / kGroup)) {
    const int64_t s = slot[i];
    uint4* o = reinterpret_cast<uint4*>(out + i * D);
    if (!in_range(s, cap)) {
      for (int v = l; v < vec; v += kGroup) o[v] = make_uint4(0, 0, 0, 0);
      continue;
    }
    const uint4* r = reinterpret_cast<const uint4*>(rows + s * D);
    for (int v = l; v < vec; v += kGroup) o[v] = r[v];
  }
}

// X0[p, :] = src[idx ? idx[local_col[p]] : local_col[p], :]. Each 16-lane group moves
// kExpR rows per round with every load of the round in flight (local_col -> idx -> row
// is a three-deep dependent chain; one row per round ran at ~2.6 TB/s, 72 us for a
// 16,384 x 39 x 128 minibatch).
constexpr int kExpR = 4;

__global__ void __launch_bounds__(256)
emb_expand_kernel(const int32_t* __restrict__ local_col, int64_t nnz,
                  const int64_t* __restrict__ idx, int64_t idx_cap,
                  const uint16_t* __restrict__ src, int64_t src_rows, int D,
                  uint16_t* __restrict__ X0) {
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  const int vec = D / 8;
  const int64_t ng = (int64_t)gridDim.x * (blockDim.x / kGroup);
  for (int64_t p0 = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; p0 < nnz;
       p0 += kExpR * ng) {
    int64_t r[kExpR];
#pragma unroll
    for (int q = 0; q < kExpR; ++q) {
      const int64_t p = p0 + q * ng;
      r[q] = p < nnz ? (int64_t)local_col[p] : -1;
    }
    if (idx) {
#pragma unroll
      for (int q = 0; q < kExpR; ++q) r[q] = in_range(r[q], idx_cap) ? idx[r[q]] : -1;
    }
    for (int v = l; v < vec; v += kGroup) {
      uint4 x[kExpR];
#pragma unroll
      for (int q = 0; q < kExpR; ++q)
        x[q] = in_range(r[q], src_rows) ? reinterpret_cast<const uint4*>(src + r[q] * D)[v]
                                        : make_uint4(0, 0, 0, 0);
#pragma unroll
      for (int q = 0; q < kExpR; ++q) {
        const int64_t p = p0 + q * ng;
        if (p < nnz) reinterpret_cast<uint4*>(X0 + p * D)[v] = x[q];
      }
    }
  }
}

// dE[u, :] = sum_{k in [seg_start[u], seg_start[u+1])} dX0[pos_s[k], :]
// Short segments (<= kShortSeg occurrences): one 16-lane group per unique key,
// plain stores. Long segments (hot keys of small-cardinality slots, up to B
// occurrences) are zeroed by the first kernel and reduced by the second, which
// walks the CSC positions in runs of kRun per 16-lane group and adds each run's
// per-segment partial sum with fp32 atomics — a hot key is spread over
// B / kRun groups instead of serialising one.
constexpr int kShortSeg = 64;
constexpr int kRun = 64;

__global__ void __launch_bounds__(256)
emb_grad_reduce_kernel(const int32_t* __restrict__ pos_s, const int32_t* __restrict__ seg_start,
                       const int32_t* __restrict__ n_uniq, int64_t u_cap, int64_t nnz,
                       const uint16_t* __restrict__ dX0, int D, float* __restrict__ dE) {
  const int64_t U = dev_len(n_uniq, u_cap);
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  for (int64_t u = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; u < U;
       u += (int64_t)gridDim.x * (blockDim.x / kGroup)) {
    const int64_t a = seg_start[u], b = seg_start[u + 1];
    const bool lng = b - a > kShortSeg;  // long: zero here, summed by the run kernel
    for (int d0 = l * 8; d0 < D; d0 += kGroup * 8) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      for (int64_t k = lng ? b : a; k < b; ++k) {
        const int32_t p = pos_s[k];
        if (!in_range(p, nnz)) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(dX0 + (int64_t)p * D + d0);
        const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(h[j]);
      }
      float4* o = reinterpret_cast<float4*>(dE + u * D + d0);
      o[0] = make_float4(acc[0], acc[1], acc[2], acc[3]);
      o[1] = make_float4(acc[4], acc[5], acc[6], acc[7]);
    }
  }
}

__global__ void __launch_bounds__(256)
emb_grad_reduce_long_kernel(const int32_t* __restrict__ pos_s, const int32_t* __restrict__ segid,
                            const int32_t* __restrict__ seg_start, int64_t u_cap, int64_t nnz,
                            const uint16_t* __restrict__ dX0, int D, float* __restrict__ dE) {
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  const int64_t runs = (nnz + kRun - 1) / kRun;
  for (int64_t run = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; run < runs;
       run += (int64_t)gridDim.x * (blockDim.x / kGroup)) {
    const int64_t k0 = run * kRun, k1 = min(nnz, k0 + kRun);
    for (int d0 = l * 8; d0 < D; d0 += kGroup * 8) {
      float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      int64_t cur = -1;
      bool cur_long = false;
      for (int64_t k = k0; k < k1; ++k) {
        const int64_t u = (int64_t)segid[k] - 1;
        if (u != cur) {
          if (cur_long) {
#pragma unroll
            for (int j = 0; j < 8; ++j) atomicAdd(dE + cur * D + d0 + j, acc[j]);
          }
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] = 0.f;
          cur = u;
          cur_long = in_range(u, u_cap) && seg_start[u + 1] - seg_start[u] > kShortSeg;
        }
        if (!cur_long) continue;
        const int32_t p = pos_s[k];
        if (!in_range(p, nnz)) continue;
        const uint4 v = *reinterpret_cast<const uint4*>(dX0 + (int64_t)p * D + d0);
        const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(h[j]);
      }
      if (cur_long) {
#pragma unroll
        for (int j = 0; j < 8; ++j) atomicAdd(dE + cur * D + d0 + j, acc[j]);
      }
    }
  }
}

// D = 128 * C (the wide & deep width): one wavefront per run of kSegRun = 64
// consecutive CSC entries, lane l owning dims {c*128 + 2l, +1}. The wave first
// loads the run's positions / segment ids (one per lane) and then all 64 dX0
// rows (64 x C independent coalesced 256-B loads in flight per wave; the row
// index comes from a readlane, so the addresses are scalar + lane offset), and
// only then walks the entries in order, summing in registers and flushing at each
// segment end (scalar-uniform branches). A segment inside the run is stored to
// dE directly; a piece of a segment that crosses a run boundary goes to the run's
// partials (slot 0: continues from the left, slot 1: continues to the right) and
// emb_grad_cross_kernel adds them up in run order. No atomics, no zeroing, one
// pass over dX0, and the sums are deterministic. The 16-lane-group kernels above
// walked each segment with 3 dependent loads per entry (segid -> seg_start, pos
// -> row): latency bound (55 + 147 us for 639 k x 128 on MI355X).
constexpr int kSegRun = 64;

// gw != null (wide & deep): the wide gradient of the same segments rides along,
// gw[u] = sum of coef[row] over u's occurrences (row = position / width), summed in
// entry order like the rows (partials in partw[run * 2 + 0 / 1], added by the cross
// kernel): one pass for both, deterministic.
template <int C>
__global__ void __launch_bounds__(256)
emb_grad_seg_kernel(const int32_t* __restrict__ pos_s, const int32_t* __restrict__ segid,
                    const int32_t* __restrict__ seg_start, int64_t u_cap, int64_t nnz,
                    const uint32_t* __restrict__ dX0, float* __restrict__ dE,
                    float* __restrict__ part, const float* __restrict__ coef, int width,
                    float* __restrict__ gw, float* __restrict__ partw) {
  constexpr int D = 128 * C;
  const int lane = threadIdx.x & 63;
  const int64_t run = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t k0 = run * kSegRun;
  if (k0 >= nnz) return;  // wave-uniform
  const int64_t k = k0 + lane;
  const bool live = k < nnz;
  int32_t p = live ? pos_s[k] : 0;
  const bool take = live && in_range(p, nnz);
  if (!take) p = 0;
  const int32_t u = live ? segid[k] - 1 : -1;
  int32_t un = __shfl_down(u, 1, 64);
  if (lane == 63) un = k + 1 < nnz ? segid[k + 1] - 1 : -1;
  const bool fl = live && (un != u || lane == 63);
  int kind = 0;  // 1: whole segment in the run, 2: from the left, 3: to the right
  if (fl && in_range(u, u_cap)) {
    const int64_t a = seg_start[u], b = seg_start[u + 1];
    kind = a < k0 ? 2 : (b > k0 + kSegRun ? 3 : 1);
  }
  const uint64_t take_m = __ballot(take);
  const uint64_t fl_m = __ballot(fl);
  const float cw = gw && take ? coef[(uint32_t)p / (uint32_t)width] : 0.f;
  uint32_t v[kSegRun][C];
#pragma unroll
  for (int j = 0; j < kSegRun; ++j) {
    const int32_t pj = __builtin_amdgcn_readlane(p, j);
    const uint32_t* row = dX0 + (int64_t)pj * (D / 2);
#pragma unroll
    for (int c = 0; c < C; ++c) v[j][c] = row[c * 64 + lane];
  }
  float acc[2 * C];
#pragma unroll
  for (int c = 0; c < 2 * C; ++c) acc[c] = 0.f;
  float aw = 0.f;  // (wave-uniform)
#pragma unroll
  for (int j = 0; j < kSegRun; ++j) {
    const bool tj = (take_m >> j) & 1;
    aw += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cw), j));
#pragma unroll
    for (int c = 0; c < C; ++c) {
      const uint32_t w = tj ? v[j][c] : 0u;
      acc[2 * c] += bf2f((uint16_t)(w & 0xffffu));
      acc[2 * c + 1] += bf2f((uint16_t)(w >> 16));
    }
    if ((fl_m >> j) & 1) {
      const int kj = __builtin_amdgcn_readlane(kind, j);
      const int uj = __builtin_amdgcn_readlane(u, j);
      float* dst = kj == 1 ? dE + (int64_t)uj * D
                 : kj == 2 ? part + run * 2 * D
                 : kj == 3 ? part + run * 2 * D + D : nullptr;
      if (dst) {
#pragma unroll
        for (int c = 0; c < C; ++c)
          *reinterpret_cast<float2*>(dst + c * 128 + 2 * lane) =
              make_float2(acc[2 * c], acc[2 * c + 1]);
        if (gw && lane == 0) {
          float* dw = kj == 1 ? gw + uj : partw + run * 2 + (kj == 3);
          *dw = aw;
        }
      }
#pragma unroll
      for (int c = 0; c < 2 * C; ++c) acc[c] = 0.f;
      aw = 0.f;
    }
  }
}

// Segments crossing run boundaries: the run where segment u starts (its last
// piece continues to the right) sums its slot-1 partial and the slot-0 partials
// of the following runs up to the segment's end, in order.
// (A hot key's segment spans up to B / 64 runs: its partials are loaded kB at a time,
// clamped in range and unconditionally, so one wave has kB loads in flight instead of
// a round trip per run.)
template <int C, int kB>
__global__ void __launch_bounds__(256)
emb_grad_cross_kernel(const int32_t* __restrict__ segid, const int32_t* __restrict__ seg_start,
                      int64_t u_cap, int64_t nnz, const float* __restrict__ part,
                      float* __restrict__ dE, const float* __restrict__ partw,
                      float* __restrict__ gw) {
  constexpr int D = 128 * C;
  const int lane = threadIdx.x & 63;
  const int64_t run = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t k0 = run * kSegRun;
  if (k0 >= nnz) return;
  const int32_t u = segid[min(nnz, k0 + kSegRun) - 1] - 1;
  if (!in_range(u, u_cap)) return;
  const int64_t a = seg_start[u], b = seg_start[u + 1];
  if (a < k0 || b <= k0 + kSegRun) return;
  const int64_t re = (b - 1) / kSegRun;
  float acc[2 * C];
#pragma unroll
  for (int c = 0; c < C; ++c) {
    const float2 x = *reinterpret_cast<const float2*>(part + run * 2 * D + D + c * 128 + 2 * lane);
    acc[2 * c] = x.x;
    acc[2 * c + 1] = x.y;
  }
  float aw = gw ? partw[run * 2 + 1] : 0.f;
  if (kB == 1) {  // (one run per iteration, the compiler's unroll)
#pragma unroll 8
    for (int64_t r = run + 1; r <= re; ++r) {
#pragma unroll
      for (int c = 0; c < C; ++c) {
        const float2 x = *reinterpret_cast<const float2*>(part + r * 2 * D + c * 128 + 2 * lane);
        acc[2 * c] += x.x;
        acc[2 * c + 1] += x.y;
      }
      if (gw) aw += partw[r * 2];
    }
  } else
  for (int64_t r0 = run + 1; r0 <= re; r0 += kB) {
    float2 x[kB][C];
    float xw[kB];
#pragma unroll
    for (int q = 0; q < kB; ++q) {
      const int64_t r = r0 + q <= re ? r0 + q : re;
#pragma unroll
      for (int c = 0; c < C; ++c)
        x[q][c] = *reinterpret_cast<const float2*>(part + r * 2 * D + c * 128 + 2 * lane);
      xw[q] = gw ? partw[r * 2] : 0.f;
    }
#pragma unroll
    for (int q = 0; q < kB; ++q) {
      if (r0 + q > re) break;
#pragma unroll
      for (int c = 0; c < C; ++c) {
        acc[2 * c] += x[q][c].x;
        acc[2 * c + 1] += x[q][c].y;
      }
      aw += xw[q];
    }
  }
#pragma unroll
  for (int c = 0; c < C; ++c)
    *reinterpret_cast<float2*>(dE + (int64_t)u * D + c * 128 + 2 * lane) =
        make_float2(acc[2 * c], acc[2 * c + 1]);
  if (gw && lane == 0) gw[u] = aw;
}

// Narrow rows (D = 8 .. 64, the FM factors): the same 64-entry runs, but lane =
// entry: each lane loads its own D-wide row (D / 8 16-B loads), a segmented
// inclusive scan over the wave (6 DPP steps per dim; segments are contiguous,
// so "same segment id at distance off" is the segment test) leaves each
// segment's run-local sum in its last lane, which stores it (kind 1) or parks it
// in the run partials (kinds 2 / 3) exactly like emb_grad_seg_kernel.
template <int D>
__global__ void __launch_bounds__(256)
emb_grad_lane_kernel(const int32_t* __restrict__ pos_s, const int32_t* __restrict__ segid,
                     const int32_t* __restrict__ seg_start, int64_t u_cap, int64_t nnz,
                     const uint16_t* __restrict__ dX0, float* __restrict__ dE,
                     float* __restrict__ part) {
  const int lane = threadIdx.x & 63;
  const int64_t run = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t k0 = run * kSegRun;
  if (k0 >= nnz) return;
  const int64_t k = k0 + lane;
  const bool live = k < nnz;
  const int32_t p = live ? pos_s[k] : 0;
  const bool take = live && in_range(p, nnz);
  const int32_t u = live ? segid[k] - 1 : -1;
  float x[D];
  const uint4* row = reinterpret_cast<const uint4*>(dX0 + (int64_t)(take ? p : 0) * D);
#pragma unroll
  for (int v = 0; v < D / 8; ++v) {
    const uint4 w = row[v];
    const uint16_t* h = reinterpret_cast<const uint16_t*>(&w);
#pragma unroll
    for (int j = 0; j < 8; ++j) x[v * 8 + j] = take ? bf2f(h[j]) : 0.f;
  }
  // segmented inclusive scan on DPP (VALU lane moves, no LDS bpermute): row_shr 1/2/4/8
  // inside each 16-lane row, then row_bcast:15 / :31 carry row ends into later rows
  seg_scan_step<0x111, 0xf>(u, x);
  seg_scan_step<0x112, 0xf>(u, x);
  seg_scan_step<0x114, 0xf>(u, x);
  seg_scan_step<0x118, 0xf>(u, x);
  seg_scan_step<0x142, 0xa>(u, x);
  seg_scan_step<0x143, 0xc>(u, x);
  int32_t un = __shfl_down(u, 1, 64);
  if (lane == 63) un = k + 1 < nnz ? segid[k + 1] - 1 : -1;
  if (!live || (un == u && lane != 63) || !in_range(u, u_cap)) return;
  const int64_t a = seg_start[u], b = seg_start[u + 1];
  float* dst = a < k0 ? part + run * 2 * D
             : (b > k0 + kSegRun ? part + run * 2 * D + D : dE + (int64_t)u * D);
#pragma unroll
  for (int v = 0; v < D / 4; ++v)
    reinterpret_cast<float4*>(dst)[v] =
        make_float4(x[4 * v], x[4 * v + 1], x[4 * v + 2], x[4 * v + 3]);
}

// emb_grad_cross_kernel for narrow rows: lane d < D sums dim d.
template <int D>
__global__ void __launch_bounds__(256)
emb_grad_cross_narrow_kernel(const int32_t* __restrict__ segid,
                             const int32_t* __restrict__ seg_start, int64_t u_cap, int64_t nnz,
                             const float* __restrict__ part, float* __restrict__ dE) {
  const int lane = threadIdx.x & 63;
  const int64_t run = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
  const int64_t k0 = run * kSegRun;
  if (k0 >= nnz || lane >= D) return;
  const int32_t u = segid[min(nnz, k0 + kSegRun) - 1] - 1;
  if (!in_range(u, u_cap)) return;
  const int64_t a = seg_start[u], b = seg_start[u + 1];
  if (a < k0 || b <= k0 + kSegRun) return;
  const int64_t re = (b - 1) / kSegRun;
  float acc = part[run * 2 * D + D + lane];
#pragma unroll 8
  for (int64_t r = run + 1; r <= re; ++r) acc += part[r * 2 * D + lane];
  dE[(int64_t)u * D + lane] = acc;
}

// ------------------------------------------- padded exchange (G > 1, sync-free)
// The embedding models' pull / push over the sparse-LR padded exchange layout
// (exchange.hip): every peer gets a fixed row of C keys with the live count in
// the row header, so sizes never travel to the host. Records of a peer chunk:
// [C x D bf16 rows | C fp32 wide values] (Q = C*D/2 + C words), one equal-split
// all-to-all each way; the owner serves all G rows in one launch per kernel.

// owner: first touch of the pulled keys' rows (the KV resolve inserted them)
__global__ void __launch_bounds__(256)
emb_init_rows_padded_kernel(const int32_t* __restrict__ recv, int64_t H, int64_t C, int kw,
                            const int64_t* __restrict__ slot, int64_t cap,
                            uint16_t* __restrict__ rows, uint8_t* __restrict__ inited, int D,
                            uint64_t seed, float scale) {
  const int sidx = blockIdx.y;
  const int32_t* row = recv + (int64_t)sidx * H;
  const int64_t n = dev_len(row, C);
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; i < n;
       i += (int64_t)gridDim.x * (blockDim.x / kGroup)) {
    const int64_t s = slot[(int64_t)sidx * C + i];
    if (!in_range(s, cap) || inited[s]) continue;
    const uint64_t key = kw == 1 ? (uint64_t)(uint32_t)row[4 + i]
                                 : reinterpret_cast<const uint64_t*>(row + 4)[i];
    init_row(rows, s, key, D, seed, scale, l, inited);
  }
}

// owner: [row | w] records of every pulled key, chunk per source row
__global__ void __launch_bounds__(256)
emb_gather_records_kernel(const int32_t* __restrict__ recv, int64_t H, int64_t C,
                          const int64_t* __restrict__ slot, const float* __restrict__ w,
                          int64_t cap, const uint16_t* __restrict__ rows, int D,
                          int32_t* __restrict__ out) {
  const int sidx = blockIdx.y;
  const int64_t n = dev_len(recv + (int64_t)sidx * H, C);
  const int64_t Q = C * (D / 2) + C;
  uint16_t* orows = reinterpret_cast<uint16_t*>(out + (int64_t)sidx * Q);
  float* ow = reinterpret_cast<float*>(out + (int64_t)sidx * Q + C * (D / 2));
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  const int vec = D / 8;
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; i < n;
       i += (int64_t)gridDim.x * (blockDim.x / kGroup)) {
    const int64_t s = slot[(int64_t)sidx * C + i];
    uint4* o = reinterpret_cast<uint4*>(orows + i * D);
    if (in_range(s, cap)) {
      const uint4* src = reinterpret_cast<const uint4*>(rows + s * D);
      for (int v = l; v < vec; v += kGroup) o[v] = src[v];
    } else {
      for (int v = l; v < vec; v += kGroup) o[v] = make_uint4(0, 0, 0, 0);
    }
    if (l == 0) ow[i] = w[(int64_t)sidx * C + i];
  }
}

__device__ __forceinline__ int owner_of(const int64_t* __restrict__ off, int G, int64_t u) {
  int lo = 0, hi = G - 1;  // largest p with off[p] <= u
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (off[mid] <= u) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// worker: records back -> rows_u [U, D] bf16 and w_u [U] in unique-key order
// (keys past a full row C came back as nothing: zero rows, counted in ovf on pack)
__global__ void __launch_bounds__(256)
emb_unpack_records_kernel(const int32_t* __restrict__ in, int64_t C, int G,
                          const int64_t* __restrict__ off, const int32_t* __restrict__ n_uniq,
                          int64_t u_cap, int D, uint16_t* __restrict__ rows_u,
                          float* __restrict__ w_u) {
  const int64_t U = dev_len(n_uniq, u_cap);
  const int64_t Q = C * (D / 2) + C;
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  const int vec = D / 8;
  for (int64_t u = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; u < U;
       u += (int64_t)gridDim.x * (blockDim.x / kGroup)) {
    const int p = owner_of(off, G, u);
    const int64_t j = u - off[p];
    uint4* o = reinterpret_cast<uint4*>(rows_u + u * D);
    if (j < C) {
      const uint4* src = reinterpret_cast<const uint4*>(in + (int64_t)p * Q) + j * vec;
      for (int v = l; v < vec; v += kGroup) o[v] = src[v];
      if (l == 0) w_u[u] = reinterpret_cast<const float*>(in + (int64_t)p * Q + C * (D / 2))[j];
    } else {
      for (int v = l; v < vec; v += kGroup) o[v] = make_uint4(0, 0, 0, 0);
      if (l == 0) w_u[u] = 0.f;
    }
  }
}

// worker: [dE bf16 | wide gradient] of every unique key into its owner's chunk
__global__ void __launch_bounds__(256)
emb_pack_grads_kernel(const float* __restrict__ dE, const float* __restrict__ g_wide,
                      const int64_t* __restrict__ off, const int32_t* __restrict__ n_uniq,
                      int64_t u_cap, int64_t C, int G, int D, int32_t* __restrict__ out) {
  const int64_t U = dev_len(n_uniq, u_cap);
  const int64_t Q = C * (D / 2) + C;
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  for (int64_t u = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; u < U;
       u += (int64_t)gridDim.x * (blockDim.x / kGroup)) {
    const int p = owner_of(off, G, u);
    const int64_t j = u - off[p];
    if (j >= C) continue;
    uint16_t* orow = reinterpret_cast<uint16_t*>(out + (int64_t)p * Q) + j * D;
    for (int d0 = l * 8; d0 < D; d0 += kGroup * 8) {
      const float4 a = *reinterpret_cast<const float4*>(dE + u * D + d0);
      const float4 b = *reinterpret_cast<const float4*>(dE + u * D + d0 + 4);
      uint4 o;
      uint16_t* h = reinterpret_cast<uint16_t*>(&o);
      h[0] = f2bf(a.x); h[1] = f2bf(a.y); h[2] = f2bf(a.z); h[3] = f2bf(a.w);
      h[4] = f2bf(b.x); h[5] = f2bf(b.y); h[6] = f2bf(b.z); h[7] = f2bf(b.w);
      *reinterpret_cast<uint4*>(orow + d0) = o;
    }
    if (l == 0) reinterpret_cast<float*>(out + (int64_t)p * Q + C * (D / 2))[j] = g_wide[u];
  }
}

// Row-wise AdaGrad (one accumulator per row, DLRM-style) on bf16 rows, fp32 math.
// kWide (wide & deep, one shard): the first lane of each key's group also applies the
// key's wide gradient to its table slot (the same slot index: rows and slots are one
// table), so the slot's optimizer update overlaps the row's loads instead of running
// as a second pass over the keys (kv_update_kernel; same update, same stats).
template <bool kWide>
__global__ void __launch_bounds__(256)
emb_update_kernel(const int64_t* __restrict__ slot, int64_t n, const int32_t* __restrict__ n_dev,
                  int64_t cap, const float* __restrict__ grad, const uint16_t* __restrict__ grad16,
                  uint16_t* __restrict__ rows, float* __restrict__ acc, int D, float lr,
                  float eps, Slot* __restrict__ slots, const float* __restrict__ gwide,
                  UpdateParams up, double* __restrict__ stats, int acc_stripes) {
  const int64_t nn = dev_len(n_dev, n);
  const int g = threadIdx.x / kGroup, l = threadIdx.x % kGroup;
  double dnnz = 0, wsum = 0, dsum = 0;
  for (int64_t i = (int64_t)blockIdx.x * (blockDim.x / kGroup) + g; i < nn;
       i += (int64_t)gridDim.x * (blockDim.x / kGroup)) {
    const int64_t s = slot[i];
    const bool ok = in_range(s, cap);
    float gv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    float sq = 0.f;
    const int d0 = l * 8;  // D == 128: one 8-element chunk per lane
    if (ok && d0 < D) {
      if (grad) {
        const float4* p = reinterpret_cast<const float4*>(grad + i * D + d0);
        const float4 x = p[0], y = p[1];
        gv[0] = x.x; gv[1] = x.y; gv[2] = x.z; gv[3] = x.w;
        gv[4] = y.x; gv[5] = y.y; gv[6] = y.z; gv[7] = y.w;
      } else {
        const uint4 v = *reinterpret_cast<const uint4*>(grad16 + i * D + d0);
        const uint16_t* h = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
        for (int j = 0; j < 8; ++j) gv[j] = bf2f(h[j]);
      }
#pragma unroll
      for (int j = 0; j < 8; ++j) sq += gv[j] * gv[j];
    }
    float gw = 0.f;
    if (kWide && l == 0 && ok) gw = gwide[i] * up.grad_scale;
    sq = group_sum(sq);
    if (!ok) continue;
    if (kWide && l == 0 && gw == gw) {  // (NaN mark = filtered entry)
      Slot sl = slots[s];
      const float w_old = apply_update(sl, gw, up);
      slots[s] = sl;
      dnnz += (double)((sl.w != 0.f) - (w_old != 0.f));
      wsum += (double)sl.w * sl.w;
      const double d = (double)sl.w - w_old;
      dsum += d * d;
    }
    float a = acc[s] + sq / D;
    if (l == 0) acc[s] = a;
    const float step = lr / (sqrtf(a) + eps);
    if (d0 < D) {
      uint4* rp = reinterpret_cast<uint4*>(rows + s * D + d0);
      uint4 v = *rp;
      uint16_t* h = reinterpret_cast<uint16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) h[j] = f2bf(bf2f(h[j]) - step * gv[j]);
      *rp = v;
    }
  }
  if (kWide && stats) {  // per-wave DPP sums, lane 63 adds (as kv_update_kernel)
    const double a = wave_sum_dpp(dnnz), b = wave_sum_dpp(wsum), c = wave_sum_dpp(dsum);
    if ((threadIdx.x & 63) == 63) {
      double* st = acc_stripe(stats, acc_stripes);
      if (a != 0) atomicAdd(&st[0], a);
      if (b != 0) atomicAdd(&st[1], b);
      if (c != 0) atomicAdd(&st[2], c);
    }
  }
}

// ---------------------------------------------------------------- head
// A wave per example (h [B, H] bf16, H <= 512, w [H] fp32): logit, loss,
// metrics, AUC bin, coef, dh. Per-row work only: every load of a row is issued
// at once (H / 64 h values + the S wide weights per lane), 4 examples per wave
// and B / 16 blocks (the previous 256-block version walked 16 examples per wave
// and did the dw reduction in LDS atomics: 71 us at B = 16384).
// The column reductions (dw = h^T coef, db of the last hidden layer) run after it
// in colred_bf16_kernel.
__global__ void __launch_bounds__(256)
wd_head_kernel(const uint16_t* __restrict__ h, int64_t B, int H, const float* __restrict__ w,
               const float* __restrict__ b, const float* __restrict__ wide_w, int64_t wide_cap,
               const int32_t* __restrict__ local_col, int S, const float* __restrict__ labels,
               float* __restrict__ coef_out, uint16_t* __restrict__ dh, float* __restrict__ db,
               double* __restrict__ metrics, uint32_t* __restrict__ hist, int nbins,
               int acc_stripes) {
  const int lane = threadIdx.x & 63;
  double loss_acc = 0, corr = 0, cnt = 0, dbsum = 0;
  for (int64_t r = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < B;
       r += (int64_t)gridDim.x * (blockDim.x >> 6)) {
    // loads at clamped in-range indices, issued together, then selects (a guarded load
    // per element compiled to a branch + s_waitcnt each: serialised round trips)
    float hv[8], wv[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = lane + 64 * q;
      const int kc = k < H ? k : 0;
      hv[q] = bf2f(h[r * H + kc]);
      wv[q] = w[kc];
    }
    float m = 0.f;
    if (S > 0) {  // (S = 0: no wide part, local_col / wide_w may be null)
      const int32_t c = local_col[r * S + (lane < S ? lane : 0)];
      const float wc = wide_w[in_range(c, wide_cap) ? c : 0];
      if (lane < S && in_range(c, wide_cap)) m = wc;
    }
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = lane + 64 * q;
      if (k >= H) hv[q] = 0.f;
      m += k < H ? hv[q] * wv[q] : 0.f;
    }
    m = wave_allsum(m) + b[0];
    const float y = labels[r] > 0.f ? 1.f : -1.f;
    const float ym = y * m;
    const float coef = -y / (1.f + expf(ym));
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const int k = lane + 64 * q;
      if (k < H) dh[r * H + k] = f2bf(hv[q] > 0.f ? coef * wv[q] : 0.f);
    }
    if (lane == 0) {
      coef_out[r] = coef;
      loss_acc += ym > 0 ? log1pf(expf(-ym)) : -ym + log1pf(expf(ym));
      corr += ((y > 0.f) == (m > 0.f)) ? 1.0 : 0.0;
      cnt += 1.0;
      dbsum += coef;
      const float p = 1.f / (1.f + expf(-m));
      const float pb = p == p ? fminf(fmaxf(p * nbins, 0.f), (float)(nbins - 1)) : 0.f;
      atomicAdd(&hist[(y > 0.f ? nbins : 0) + (int)pb], 1u);
    }
  }
  // per-wave DPP sums, lane 63 adds (no barriers)
  const double a = wave_sum_dpp(loss_acc), c = wave_sum_dpp(corr), n = wave_sum_dpp(cnt);
  const double d = wave_sum_dpp(dbsum);
  if ((threadIdx.x & 63) == 63 && n > 0) {
    double* mt = acc_stripe(metrics, acc_stripes);
    atomicAdd(&mt[0], a);
    atomicAdd(&mt[1], c);
    atomicAdd(&mt[2], n);
    atomicAdd(&mt[5], d);  // db of the head, folded into db by wd_head_db_kernel
  }
}

// out[n] += sum_r s_r x[r, n]  and  out_pos[n] += g[n] sum_r s_r [x[r, n] > 0]
// (bf16 x [B, N], N % 8 == 0; s = 1 when null). A block covers 8 * tpr columns
// (tpr threads per row, 16-B loads) and kColredRows rows, 256 / tpr rows per
// pass; per-block partials meet in LDS, one fp32 atomic per column and block.
// Used for the head's dw = h^T coef and last-layer db = w * sum coef [h > 0], and
// as the stand-alone column sum (bias gradient of the library-GEMM backend).
constexpr int kColredRows = 128;

__global__ void __launch_bounds__(256)
colred_bf16_kernel(const uint16_t* __restrict__ x, int64_t B, int N, int tpr,
                   const float* __restrict__ s, float* __restrict__ out,
                   const float* __restrict__ g, float* __restrict__ out_pos) {
  __shared__ float red[2][256 * 8];
  const int t = threadIdx.x, cl = t % tpr, rg = t / tpr, nrg = 256 / tpr;
  const int n0 = blockIdx.x * tpr * 8 + cl * 8;
  const int64_t r0 = (int64_t)blockIdx.y * kColredRows, r1 = min(B, r0 + kColredRows);
  float a[8], c[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) a[j] = c[j] = 0.f;
  if (n0 < N) {
#pragma unroll 4
    for (int64_t r = r0 + rg; r < r1; r += nrg) {
      const uint4 v = *reinterpret_cast<const uint4*>(x + r * N + n0);
      const float sr = s ? s[r] : 1.f;
      const uint16_t* hv = reinterpret_cast<const uint16_t*>(&v);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xv = bf2f(hv[j]);
        a[j] += sr * xv;
        c[j] += xv > 0.f ? sr : 0.f;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    red[0][rg * tpr * 8 + cl * 8 + j] = a[j];
    red[1][rg * tpr * 8 + cl * 8 + j] = c[j];
  }
  __syncthreads();
  for (int i = t; i < tpr * 8; i += 256) {
    const int n = blockIdx.x * tpr * 8 + i;
    if (n >= N) continue;
    float sa = 0.f, sc = 0.f;
    for (int q = 0; q < nrg; ++q) {
      sa += red[0][q * tpr * 8 + i];
      sc += red[1][q * tpr * 8 + i];
    }
    unsafeAtomicAdd(out + n, sa);
    if (out_pos) unsafeAtomicAdd(out_pos + n, g[n] * sc);
  }
}

// db (head bias) += the striped coef sums the head kernel left in metrics[5]
__global__ void __launch_bounds__(64)
wd_head_db_kernel(double* __restrict__ metrics, int acc_stripes, float* __restrict__ db) {
  double d = 0;  // one stripe per lane (acc_stripes <= 64)
  if ((int)threadIdx.x < acc_stripes) {
    d = metrics[threadIdx.x * kAccStride + 5];
    metrics[threadIdx.x * kAccStride + 5] = 0;
  }
  for (int off = 32; off > 0; off >>= 1) d += __shfl_xor(d, off, 64);
  if (threadIdx.x == 0) db[0] += (float)d;
}

// Adam with fp32 master weights; writes the bf16 copy used by the GEMMs. With a device
// step clock (step_dev: steps completed so far, advanced later in the step by the AUC
// epilogue) the bias corrections come from it, so a captured step replays correctly.
__global__ void __launch_bounds__(256)
adam_update_kernel(float* __restrict__ p, float* __restrict__ g, float* __restrict__ m,
                   float* __restrict__ v, int64_t n, float lr, float b1, float b2, float eps,
                   float bc1, float bc2, float gscale, uint16_t* __restrict__ p16,
                   const int64_t* __restrict__ step_dev, int zero_grad) {
  if (step_dev) {
    const float s = (float)(step_dev[0] + 1);
    bc1 = 1.f - exp2f(s * log2f(b1));
    bc2 = 1.f - exp2f(s * log2f(b2));
  }
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * gscale;
    if (zero_grad) g[i] = 0.f;  // leave the next step's accumulators zeroed (no fill pass)
    const float mi = b1 * m[i] + (1.f - b1) * gi;
    const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float pi = p[i] - lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
    p[i] = pi;
    if (p16) p16[i] = f2bf(pi);
  }
}

}  // namespace

void emb_init_rows(const int64_t* slot, const uint64_t* keys, int64_t n, const int32_t* n_dev,
                   int64_t cap, void* rows, uint8_t* inited, int D, uint64_t seed, float scale,
                   hipStream_t st) {
  if (n <= 0) return;
  emb_init_rows_kernel<<<grid_for(n, 16, 4096), 256, 0, st>>>(
      slot, keys, n, n_dev, cap, reinterpret_cast<uint16_t*>(rows), inited, D, seed, scale);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void emb_gather_rows(const int64_t* slot, int64_t n, const int32_t* n_dev, int64_t cap,
                     const void* rows, int D, void* out, hipStream_t st) {
  if (n <= 0) return;
  emb_gather_rows_kernel<<<grid_for(n, 16, 8192), 256, 0, st>>>(
      slot, n, n_dev, cap, reinterpret_cast<const uint16_t*>(rows), D,
      reinterpret_cast<uint16_t*>(out));
  PSAMD_HIP_CHECK(hipGetLastError());
}

void emb_expand(const int32_t* local_col, int64_t nnz, const int64_t* idx, int64_t idx_cap,
                const void* src, int64_t src_rows, int D, void* X0, hipStream_t st) {
  if (nnz <= 0) return;
  emb_expand_kernel<<<grid_for(nnz, 16 * kExpR, 8192), 256, 0, st>>>(
      local_col, nnz, idx, idx_cap, reinterpret_cast<const uint16_t*>(src), src_rows, D,
      reinterpret_cast<uint16_t*>(X0));
  PSAMD_HIP_CHECK(hipGetLastError());
}

static bool seg_path(int D) {
  return D == 8 || D == 16 || D == 32 || D == 64 || D == 128 || D == 256;
}

// (+ 2 wide partials per run when the wide gradient rides along: wide_ok(D))
int64_t emb_grad_part_floats(int64_t nnz, int D) {
  return seg_path(D) ? ((nnz + kSegRun - 1) / kSegRun) * 2 * (D + 1) : 0;
}
bool emb_grad_wide_ok(int D) { return D == 128 || D == 256; }
// PSAMD_CROSS_BATCH=1: the cross kernel loads kB runs' partials per iteration (A/B)
static bool cross_batched() {
  static const bool on = [] {
    const char* e = getenv("PSAMD_CROSS_BATCH");
    return e && e[0] == '1';
  }();
  return on;
}

void emb_grad_reduce(const int32_t* pos_s, const int32_t* segid, const int32_t* seg_start,
                     const int32_t* n_uniq, int64_t u_cap, int64_t nnz, const void* dX0, int D,
                     float* dE, float* part, const float* coef, int width, float* gw,
                     hipStream_t st) {
  if (u_cap <= 0 || nnz <= 0) return;
  if (gw && !(part && emb_grad_wide_ok(D) && coef && width > 0))
    throw std::runtime_error("emb_grad_reduce: the wide gradient rides along only with D = 128 / 256");
  float* partw = part ? part + ((nnz + kSegRun - 1) / kSegRun) * 2 * D : nullptr;
  if (part && seg_path(D)) {
    const int64_t runs = (nnz + kSegRun - 1) / kSegRun;
    const dim3 grid((unsigned)((runs + 3) / 4));
    const uint32_t* x = reinterpret_cast<const uint32_t*>(dX0);
    const uint16_t* x16 = reinterpret_cast<const uint16_t*>(dX0);
#define PSAMD_NARROW(DD)                                                                    \
  emb_grad_lane_kernel<DD><<<grid, 256, 0, st>>>(pos_s, segid, seg_start, u_cap, nnz, x16, dE, \
                                                 part);                                      \
  PSAMD_HIP_CHECK(hipGetLastError());                                                       \
  emb_grad_cross_narrow_kernel<DD><<<grid, 256, 0, st>>>(segid, seg_start, u_cap, nnz, part, dE)
    if (D == 8) {
      PSAMD_NARROW(8);
    } else if (D == 16) {
      PSAMD_NARROW(16);
    } else if (D == 32) {
      PSAMD_NARROW(32);
    } else if (D == 64) {
      PSAMD_NARROW(64);
    } else if (D == 128) {
      emb_grad_seg_kernel<1><<<grid, 256, 0, st>>>(pos_s, segid, seg_start, u_cap, nnz, x, dE, part,
                                                    coef, width, gw, partw);
      PSAMD_HIP_CHECK(hipGetLastError());
      if (cross_batched())
        emb_grad_cross_kernel<1, 16><<<grid, 256, 0, st>>>(segid, seg_start, u_cap, nnz, part, dE,
                                                           partw, gw);
      else
        emb_grad_cross_kernel<1, 1><<<grid, 256, 0, st>>>(segid, seg_start, u_cap, nnz, part, dE,
                                                          partw, gw);
    } else {
      emb_grad_seg_kernel<2><<<grid, 256, 0, st>>>(pos_s, segid, seg_start, u_cap, nnz, x, dE, part,
                                                    coef, width, gw, partw);
      PSAMD_HIP_CHECK(hipGetLastError());
      if (cross_batched())
        emb_grad_cross_kernel<2, 8><<<grid, 256, 0, st>>>(segid, seg_start, u_cap, nnz, part, dE,
                                                          partw, gw);
      else
        emb_grad_cross_kernel<2, 1><<<grid, 256, 0, st>>>(segid, seg_start, u_cap, nnz, part, dE,
                                                          partw, gw);
    }
#undef PSAMD_NARROW
    PSAMD_HIP_CHECK(hipGetLastError());
    return;
  }
  emb_grad_reduce_kernel<<<grid_for(u_cap, 16, 8192), 256, 0, st>>>(
      pos_s, seg_start, n_uniq, u_cap, nnz, reinterpret_cast<const uint16_t*>(dX0), D, dE);
  PSAMD_HIP_CHECK(hipGetLastError());
  emb_grad_reduce_long_kernel<<<grid_for((nnz + kRun - 1) / kRun, 16, 8192), 256, 0, st>>>(
      pos_s, segid, seg_start, u_cap, nnz, reinterpret_cast<const uint16_t*>(dX0), D, dE);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void emb_update(const int64_t* slot, int64_t n, const int32_t* n_dev, int64_t cap,
                const float* grad, const void* grad16, void* rows, float* acc, int D, float lr,
                float eps, void* slots, const float* gwide, const int* wide_rule,
                const float* wide_hyper, double* stats, int acc_stripes, hipStream_t st) {
  if (n <= 0) return;
  if (slots) {
    const UpdateParams p{wide_rule[0], wide_rule[1], wide_hyper[0], wide_hyper[1], wide_hyper[2],
                         wide_hyper[3], wide_hyper[4], wide_hyper[5]};
    emb_update_kernel<true><<<grid_for(n, 16, 8192), 256, 0, st>>>(
        slot, n, n_dev, cap, grad, reinterpret_cast<const uint16_t*>(grad16),
        reinterpret_cast<uint16_t*>(rows), acc, D, lr, eps, (Slot*)slots, gwide, p, stats,
        acc_stripes);
  } else {
    emb_update_kernel<false><<<grid_for(n, 16, 8192), 256, 0, st>>>(
        slot, n, n_dev, cap, grad, reinterpret_cast<const uint16_t*>(grad16),
        reinterpret_cast<uint16_t*>(rows), acc, D, lr, eps, nullptr, nullptr, UpdateParams{},
        nullptr, 1);
  }
  PSAMD_HIP_CHECK(hipGetLastError());
}

void colred_bf16(const void* x, int64_t B, int N, const float* s, float* out, const float* g,
                 float* out_pos, hipStream_t st);

void wd_head(const void* h, int64_t B, int H, const float* w, const float* b, const float* wide_w,
             int64_t wide_cap, const int32_t* local_col, int S, const float* labels,
             float* coef, void* dh, float* dw, float* db, float* db_h, double* metrics,
             uint32_t* hist, int nbins, int acc_stripes, hipStream_t st) {
  if (B <= 0) return;
  // 4 examples per wave: 4 x fewer blocks ending in the 4 striped metric atomics
  wd_head_kernel<<<(unsigned)std::min<int64_t>((B + 15) / 16, 65535), 256, 0, st>>>(
      reinterpret_cast<const uint16_t*>(h), B, H, w, b, wide_w, wide_cap, local_col, S, labels,
      coef, reinterpret_cast<uint16_t*>(dh), db, metrics, hist, nbins, acc_stripes);
  PSAMD_HIP_CHECK(hipGetLastError());
  wd_head_db_kernel<<<1, 64, 0, st>>>(metrics, acc_stripes, db);
  PSAMD_HIP_CHECK(hipGetLastError());
  colred_bf16(h, B, H, coef, dw, db_h ? w : nullptr, db_h, st);
}

void colred_bf16(const void* x, int64_t B, int N, const float* s, float* out, const float* g,
                 float* out_pos, hipStream_t st) {
  if (N <= 0 || B <= 0) return;
  int tpr = 64;
  while (tpr > 1 && tpr * 8 >= 2 * N) tpr >>= 1;  // 8 * tpr >= N > 4 * tpr (or 64)
  const dim3 grid((unsigned)((N + 8 * tpr - 1) / (8 * tpr)),
                  (unsigned)((B + kColredRows - 1) / kColredRows));
  colred_bf16_kernel<<<grid, 256, 0, st>>>(reinterpret_cast<const uint16_t*>(x), B, N, tpr, s,
                                           out, g, out_pos);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void adam_update(float* p, float* g, float* m, float* v, int64_t n, float lr, float b1,
                 float b2, float eps, float bc1, float bc2, float gscale, void* p16,
                 const int64_t* step_dev, bool zero_grad, hipStream_t st) {
  if (n <= 0) return;
  adam_update_kernel<<<grid_for(n, 256, 4096), 256, 0, st>>>(
      p, g, m, v, n, lr, b1, b2, eps, bc1, bc2, gscale, reinterpret_cast<uint16_t*>(p16),
      step_dev, zero_grad ? 1 : 0);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void emb_padded_serve(const int32_t* recv, int64_t H, int64_t C, int kw, int G,
                      const int64_t* slot, const float* w, int64_t cap, void* rows,
                      uint8_t* inited, int D, uint64_t seed, float scale, int32_t* out,
                      hipStream_t st) {
  if (C <= 0 || G <= 0) return;
  const dim3 grid((unsigned)std::min<int64_t>((C + 15) / 16, 2048), (unsigned)G);
  auto r = reinterpret_cast<uint16_t*>(rows);
  emb_init_rows_padded_kernel<<<grid, 256, 0, st>>>(recv, H, C, kw, slot, cap, r, inited, D,
                                                    seed, scale);
  PSAMD_HIP_CHECK(hipGetLastError());
  emb_gather_records_kernel<<<grid, 256, 0, st>>>(recv, H, C, slot, w, cap, r, D, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void emb_unpack_records(const int32_t* in, int64_t C, int G, const int64_t* off,
                        const int32_t* n_uniq, int64_t u_cap, int D, void* rows_u, float* w_u,
                        hipStream_t st) {
  if (u_cap <= 0) return;
  emb_unpack_records_kernel<<<grid_for(u_cap, 16, 8192), 256, 0, st>>>(
      in, C, G, off, n_uniq, u_cap, D, reinterpret_cast<uint16_t*>(rows_u), w_u);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void emb_pack_grads(const float* dE, const float* g_wide, const int64_t* off,
                    const int32_t* n_uniq, int64_t u_cap, int64_t C, int G, int D, int32_t* out,
                    hipStream_t st) {
  if (u_cap <= 0) return;
  emb_pack_grads_kernel<<<grid_for(u_cap, 16, 8192), 256, 0, st>>>(dE, g_wide, off, n_uniq,
                                                                   u_cap, C, G, D, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
