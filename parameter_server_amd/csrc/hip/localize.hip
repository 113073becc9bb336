// Minibatch key localisation on the GPU.
//
// Reference: Localizer::countUniqIndex (src/util/localizer.h:69-108) sorts
// (key, pos) pairs with a thread-recursive merge sort and run-length encodes
// them; remapIndex (:126-191) merge-joins against a key dictionary and emits a
// CSR with uint32 local column ids. Here:
//   1. mix:    h = mix(key) (bijection, see common.cuh), pos = iota
//   2. sort:   rocPRIM/hipCUB LSD radix sort of (h, pos) over only the `bits`
//              significant bits of the mixed key space (30 bits for 10^9
//              features => 4 digit passes instead of 8)
//   3. RLE:    head flags -> inclusive scan -> scatter: unique keys (sorted,
//              hence already grouped by owner shard for range partitioning),
//              segment starts, per-nnz local column, per-sorted-element segment
//   4. split:  owner boundaries by binary search (K14, sliceKeyOrderedMsg,
//              src/system/message.h:120-159)
#include "common.cuh"
#include <hipcub/hipcub.hpp>
#include <stdexcept>
#include <string>

namespace psamd {

__global__ void mix_iota_kernel(const uint64_t* __restrict__ keys, int64_t n, KeyMix m,
                                uint64_t* __restrict__ h, int32_t* __restrict__ pos) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    h[i] = mix_key(keys[i], m);
    pos[i] = (int32_t)i;
  }
}

__global__ void mix_kernel(const uint64_t* __restrict__ keys, int64_t n, KeyMix m,
                           uint64_t* __restrict__ h, int inverse) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    h[i] = inverse ? unmix_key(keys[i], m) : mix_key(keys[i], m);
  }
}

__global__ void head_flags_kernel(const uint64_t* __restrict__ hs, int64_t n,
                                  int32_t* __restrict__ flags) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    flags[i] = (i == 0 || hs[i] != hs[i - 1]) ? 1 : 0;
  }
}

// segid[i] is the 1-based inclusive scan of head flags.
__global__ void rle_scatter_kernel(const uint64_t* __restrict__ hs,
                                   const int32_t* __restrict__ pos_s,
                                   const int32_t* __restrict__ segid, int64_t n,
                                   uint64_t* __restrict__ uniq, int32_t* __restrict__ seg_start,
                                   int32_t* __restrict__ local_col, int32_t* __restrict__ n_uniq,
                                   float* __restrict__ zero_a, float* __restrict__ zero_b) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t s = segid[i] - 1;
    const int32_t p = pos_s[i];
    if (!in_range(s, n)) continue;  // corrupted scan/sort output: never write OOB
    if (in_range(p, n)) local_col[p] = s;
    const bool head = (i == 0) || (segid[i - 1] != segid[i]);
    if (head) {
      uniq[s] = hs[i];
      seg_start[s] = (int32_t)i;
      if (zero_a) zero_a[s] = 0.f;
      if (zero_b) zero_b[s] = 0.f;
    }
    if (i == n - 1) {
      *n_uniq = s + 1;
      seg_start[s + 1] = (int32_t)n;
    }
  }
}

// counts[u] = min(seg length, sat) as uint8 (CountMin input, reference uses uint8 counts:
// src/util/localizer.h:95-105).
__global__ void seg_counts_kernel(const int32_t* __restrict__ seg_start,
                                  const int32_t* __restrict__ n_uniq, int64_t cap,
                                  uint8_t* __restrict__ counts, int sat) {
  const int64_t u_n = dev_len(n_uniq, cap);
  for (int64_t u = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; u < u_n;
       u += (int64_t)gridDim.x * blockDim.x) {
    int c = seg_start[u + 1] - seg_start[u];
    counts[u] = (uint8_t)(c > sat ? sat : c);
  }
}

// offsets[g] = lower_bound(uniq[0:U], bounds[g]) for g in [0, G]; offsets[G] = U.
// One workgroup per bound, 256-ary search: each round the 256 threads probe 256 evenly
// spaced keys of the interval at once and __syncthreads_count narrows it 256-fold, so
// U = 234 K takes 3 rounds of one memory latency each instead of the 18 dependent
// loads of a one-thread binary search (7.4 us -> the launch floor at 8 peers).
constexpr int kSplitThr = 256;
__global__ void __launch_bounds__(kSplitThr)
owner_split_kernel(const uint64_t* __restrict__ uniq, const int32_t* __restrict__ n_uniq,
                   int64_t n_host, const uint64_t* __restrict__ bounds, int G,
                   int64_t* __restrict__ offsets) {
  const int g = blockIdx.x, t = threadIdx.x;
  const int64_t U = dev_len(n_uniq, n_host);
  if (g == 0 || g == G) {
    if (t == 0) offsets[g] = g == 0 ? 0 : U;
    return;
  }
  const uint64_t b = bounds[g];
  int64_t lo = 0, hi = U;  // the answer lies in [lo, hi]
  while (hi - lo > kSplitThr) {
    const int64_t step = (hi - lo + kSplitThr - 1) / kSplitThr;
    const int64_t i = lo + t * step;
    // predicate uniq[i] < b is a true prefix over the probes (uniq is sorted)
    const int c = __syncthreads_count(i < hi && uniq[i] < b);
    if (c == 0) { hi = lo; break; }
    const int64_t nlo = lo + (int64_t)(c - 1) * step + 1;
    hi = min(hi, lo + (int64_t)c * step);
    lo = nlo;
  }
  const int64_t i = lo + t;
  const int c = __syncthreads_count(i < hi && uniq[i] < b);
  if (t == 0) offsets[g] = lo + c;
}

// Owner of each key for unsorted key lists (range partition of mixed space).
__global__ void owner_of_kernel(const uint64_t* __restrict__ h, int64_t n,
                                const uint64_t* __restrict__ bounds, int G,
                                int32_t* __restrict__ owner) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint64_t x = h[i];
    int lo = 0, hi = G;  // find last g with bounds[g] <= x
    while (hi - lo > 1) {
      int mid = (lo + hi) >> 1;
      if (bounds[mid] <= x) lo = mid; else hi = mid;
    }
    owner[i] = lo;
  }
}

// ---------------------------------------------------------------------------
void mix_iota(const uint64_t* keys, int64_t n, KeyMix m, uint64_t* h, int32_t* pos,
              hipStream_t st) {
  mix_iota_kernel<<<grid_for(n, 256), 256, 0, st>>>(keys, n, m, h, pos);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void mix_keys(const uint64_t* keys, int64_t n, KeyMix m, uint64_t* h, bool inverse,
              hipStream_t st) {
  mix_kernel<<<grid_for(n, 256), 256, 0, st>>>(keys, n, m, h, inverse ? 1 : 0);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// rocPRIM reference path (kept for A/B benchmarking; not used by the trainer).
size_t rocprim_sort_temp_bytes(int64_t n, int end_bit) {
  size_t bytes = 0;
  PSAMD_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(
      nullptr, bytes, (const uint64_t*)nullptr, (uint64_t*)nullptr, (const int32_t*)nullptr,
      (int32_t*)nullptr, (int)n, 0, end_bit, (hipStream_t)0));
  return bytes;
}

void rocprim_sort_pairs(void* temp, size_t temp_bytes, const uint64_t* k_in, uint64_t* k_out,
                        const int32_t* v_in, int32_t* v_out, int64_t n, int end_bit,
                        hipStream_t st) {
  PSAMD_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, k_in, k_out, v_in, v_out,
                                                     (int)n, 0, end_bit, st));
}

size_t scan_i32_temp_bytes(int64_t n);
void scan_i32(const int32_t* in, int32_t* out, int64_t n, void* temp, bool inclusive,
              hipStream_t st);

size_t scan_temp_bytes(int64_t n) { return scan_i32_temp_bytes(n); }

void inclusive_scan_i32(void* temp, size_t temp_bytes, const int32_t* in, int32_t* out,
                        int64_t n, hipStream_t st) {
  if (temp_bytes < scan_i32_temp_bytes(n)) throw std::runtime_error("scan temp too small");
  scan_i32(in, out, n, temp, true, st);
}

void rle(const uint64_t* hs, const int32_t* pos_s, int64_t n, int32_t* flags, int32_t* segid,
         void* scan_temp, size_t scan_bytes, uint64_t* uniq, int32_t* seg_start,
         int32_t* local_col, int32_t* n_uniq, float* zero_a, float* zero_b, hipStream_t st) {
  head_flags_kernel<<<grid_for(n, 256), 256, 0, st>>>(hs, n, flags);
  PSAMD_HIP_CHECK(hipGetLastError());
  inclusive_scan_i32(scan_temp, scan_bytes, flags, segid, n, st);
  rle_scatter_kernel<<<grid_for(n, 256), 256, 0, st>>>(hs, pos_s, segid, n, uniq, seg_start,
                                                        local_col, n_uniq, zero_a, zero_b);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void seg_counts(const int32_t* seg_start, const int32_t* n_uniq, int64_t cap, uint8_t* counts,
                int sat, hipStream_t st) {
  seg_counts_kernel<<<grid_for(cap, 256), 256, 0, st>>>(seg_start, n_uniq, cap, counts, sat);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void owner_split(const uint64_t* uniq, const int32_t* n_uniq, int64_t n_host,
                 const uint64_t* bounds, int G, int64_t* offsets, hipStream_t st) {
  owner_split_kernel<<<G + 1, kSplitThr, 0, st>>>(uniq, n_uniq, n_host, bounds, G,
                                                             offsets);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void owner_of(const uint64_t* h, int64_t n, const uint64_t* bounds, int G, int32_t* owner,
              hipStream_t st) {
  owner_of_kernel<<<grid_for(n, 256), 256, 0, st>>>(h, n, bounds, G, owner);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
