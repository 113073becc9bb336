// Device-wide scan and stable LSD radix sort (hand-written, wave64 / LDS-tiled).
//
// Scan: reduce-then-scan over 2048-element tiles (256 threads x 8 items): tile
// sums -> one-block scan of the tile sums -> per-tile scan with its offset.
// Three launches, no inter-workgroup spinning, so it is safe under any dispatch
// order and inside HIP graphs.
//
// Radix sort (keys u64, values i32, bits [0, end_bit)): 6-bit digits. Per pass:
//   1. radix_hist:    per-tile digit histogram -> hist[digit * num_tiles + tile]
//                     (digit-major, so an exclusive scan of the flat array IS the
//                     global output offset of every (digit, tile) run)
//   2. exclusive scan of hist
//   3. radix_scatter: stable tile-local ranking with per-thread u16 digit counters
//                     in LDS ([64 digits][256 threads] = 32 KB) + a raking block
//                     scan over them; the tile is reordered in LDS and written out
//                     digit-run contiguous (coalesced stores).
// Every global index is bounds-checked.
#include "common.cuh"
#include <stdexcept>
#include <string>

namespace psamd {

constexpr int kBlk = 256;
constexpr int kItems = 8;
constexpr int kTile = kBlk * kItems;  // 2048
constexpr int kRadixBits = 6;
constexpr int kRadix = 1 << kRadixBits;  // 64

// Exclusive scan of one value per thread over a 256-thread block; returns the
// exclusive prefix, *total = block sum. lds must hold >= 4 + 1 words.
template <typename T>
__device__ __forceinline__ T block_exclusive_scan(T v, T* lds, T* total) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  T x = v;
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    T y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  if (lane == 63) lds[wid] = x;
  __syncthreads();
  if (threadIdx.x == 0) {
    T run = 0;
    for (int w = 0; w < kBlk / 64; ++w) {
      T t = lds[w];
      lds[w] = run;
      run += t;
    }
    lds[kBlk / 64] = run;
  }
  __syncthreads();
  const T res = x - v + lds[wid];
  *total = lds[kBlk / 64];
  __syncthreads();
  return res;
}

// ------------------------------------------------------------------- scan
template <typename T>
__global__ void __launch_bounds__(kBlk) scan_reduce_kernel(const T* __restrict__ in, int64_t n,
                                                           T* __restrict__ partials) {
  __shared__ T lds[8];
  const int64_t base = (int64_t)blockIdx.x * kTile;
  T s = 0;
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int64_t i = base + j * kBlk + threadIdx.x;
    if (i < n) s += in[i];
  }
  T tot;
  block_exclusive_scan<T>(s, lds, &tot);
  if (threadIdx.x == 0) partials[blockIdx.x] = tot;
}

// One block scans all tile partials (exclusive), carrying across 256-chunks.
template <typename T>
__global__ void __launch_bounds__(kBlk) scan_partials_kernel(T* __restrict__ partials,
                                                             int64_t num_tiles) {
  __shared__ T lds[8];
  T carry = 0;
  for (int64_t c = 0; c < num_tiles; c += kBlk) {
    const int64_t i = c + threadIdx.x;
    const T v = i < num_tiles ? partials[i] : (T)0;
    T tot;
    const T ex = block_exclusive_scan<T>(v, lds, &tot);
    if (i < num_tiles) partials[i] = ex + carry;
    carry += tot;
  }
}

template <typename T, bool kInclusive>
__global__ void __launch_bounds__(kBlk) scan_down_kernel(const T* __restrict__ in, int64_t n,
                                                         const T* __restrict__ partials,
                                                         T* __restrict__ out) {
  __shared__ T tile[kTile];
  __shared__ T lds[8];
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll
  for (int j = 0; j < kItems; ++j) {  // striped, coalesced
    const int64_t i = base + j * kBlk + threadIdx.x;
    tile[j * kBlk + threadIdx.x] = i < n ? in[i] : (T)0;
  }
  __syncthreads();
  T v[kItems];
  T s = 0;
#pragma unroll
  for (int j = 0; j < kItems; ++j) {  // blocked: thread owns 8 consecutive items
    v[j] = tile[threadIdx.x * kItems + j];
    s += v[j];
  }
  T tot;
  T run = block_exclusive_scan<T>(s, lds, &tot) + partials[blockIdx.x];
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const T x = v[j];
    tile[threadIdx.x * kItems + j] = kInclusive ? run + x : run;
    run += x;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int64_t i = base + j * kBlk + threadIdx.x;
    if (i < n) out[i] = tile[j * kBlk + threadIdx.x];
  }
}

template <typename T>
void device_scan(const T* in, T* out, int64_t n, T* partials, bool inclusive, hipStream_t st) {
  if (n <= 0) return;
  const int64_t tiles = (n + kTile - 1) / kTile;
  scan_reduce_kernel<T><<<(unsigned)tiles, kBlk, 0, st>>>(in, n, partials);
  scan_partials_kernel<T><<<1, kBlk, 0, st>>>(partials, tiles);
  if (inclusive)
    scan_down_kernel<T, true><<<(unsigned)tiles, kBlk, 0, st>>>(in, n, partials, out);
  else
    scan_down_kernel<T, false><<<(unsigned)tiles, kBlk, 0, st>>>(in, n, partials, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

// ------------------------------------------------------------------- sort
__global__ void __launch_bounds__(kBlk) radix_hist_kernel(const uint64_t* __restrict__ keys,
                                                          int64_t n, int shift,
                                                          uint32_t* __restrict__ hist,
                                                          int64_t num_tiles) {
  __shared__ uint32_t cnt[kRadix];
  if (threadIdx.x < kRadix) cnt[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = (int64_t)blockIdx.x * kTile;
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int64_t i = base + j * kBlk + threadIdx.x;
    if (i < n) atomicAdd(&cnt[(keys[i] >> shift) & (kRadix - 1)], 1u);
  }
  __syncthreads();
  if (threadIdx.x < kRadix) hist[(int64_t)threadIdx.x * num_tiles + blockIdx.x] = cnt[threadIdx.x];
}

__global__ void __launch_bounds__(kBlk) radix_scatter_kernel(
    const uint64_t* __restrict__ keys_in, const int32_t* __restrict__ vals_in,
    uint64_t* __restrict__ keys_out, int32_t* __restrict__ vals_out, int64_t n, int shift,
    const uint32_t* __restrict__ offs, int64_t num_tiles) {
  __shared__ uint64_t skeys[kTile];
  __shared__ int32_t svals[kTile];
  __shared__ uint16_t ctr[kRadix * kBlk];  // [digit][thread], 32 KB
  __shared__ uint32_t part[kBlk];
  __shared__ uint32_t lds[8];
  __shared__ uint32_t dstart[kRadix];
  const int t = threadIdx.x;
  const int64_t base = (int64_t)blockIdx.x * kTile;
  const int tile_n = (int)min((int64_t)kTile, n - base);

  for (int f = t; f < kRadix * kBlk; f += kBlk) ctr[f] = 0;
#pragma unroll
  for (int j = 0; j < kItems; ++j) {  // striped coalesced load in original order
    const int li = j * kBlk + t;
    if (li < tile_n) {
      skeys[li] = keys_in[base + li];
      svals[li] = vals_in[base + li];
    }
  }
  __syncthreads();
  // blocked ownership: thread t holds tile items [t*8, t*8+8) (original order)
  uint64_t k[kItems];
  int32_t v[kItems];
  uint16_t local[kItems];
  int d[kItems];
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int li = t * kItems + j;
    if (li < tile_n) {
      k[j] = skeys[li];
      v[j] = svals[li];
      d[j] = (int)((k[j] >> shift) & (kRadix - 1));
      local[j] = ctr[d[j] * kBlk + t]++;
    } else {
      d[j] = -1;
    }
  }
  __syncthreads();
  // raking exclusive scan over ctr in (digit, thread) order: thread t owns flat
  // range [t*64, t*64+64) (kRadix*kBlk / kBlk = 64 counters each).
  constexpr int kPer = kRadix * kBlk / kBlk;
  uint32_t s = 0;
  for (int q = 0; q < kPer; ++q) s += ctr[t * kPer + q];
  uint32_t tot;
  uint32_t run = block_exclusive_scan<uint32_t>(s, lds, &tot);
  for (int q = 0; q < kPer; ++q) {
    const uint32_t c = ctr[t * kPer + q];
    ctr[t * kPer + q] = (uint16_t)run;
    run += c;
  }
  __syncthreads();
  if (t < kRadix) dstart[t] = ctr[t * kBlk];  // tile-local start of digit t
  __syncthreads();
  // reorder the tile in LDS by (digit, original order)
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    if (d[j] >= 0) {
      const int r = (int)ctr[d[j] * kBlk + t] + local[j];
      if (r < kTile) {
        skeys[r] = k[j];
        svals[r] = v[j];
      }
    }
  }
  __syncthreads();
  // digit-run contiguous, coalesced write-out
#pragma unroll
  for (int j = 0; j < kItems; ++j) {
    const int li = j * kBlk + t;
    if (li < tile_n) {
      const uint64_t key = skeys[li];
      const int dg = (int)((key >> shift) & (kRadix - 1));
      const int64_t g = (int64_t)offs[(int64_t)dg * num_tiles + blockIdx.x] + (li - (int)dstart[dg]);
      if (in_range(g, n)) {
        keys_out[g] = key;
        vals_out[g] = svals[li];
      }
    }
  }
  (void)part;
}

__global__ void copy_pairs_kernel(const uint64_t* __restrict__ ki, const int32_t* __restrict__ vi,
                                  uint64_t* __restrict__ ko, int32_t* __restrict__ vo, int64_t n) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    ko[i] = ki[i];
    vo[i] = vi[i];
  }
}

// Workspace layout (bytes): [keys_tmp n*8][vals_tmp n*4 (pad 8)][hist R*T*4][partials]
size_t radix_sort_temp_bytes(int64_t n) {
  const int64_t tiles = (n + kTile - 1) / kTile;
  const int64_t hist = (int64_t)kRadix * tiles;
  const int64_t ptiles = (hist + kTile - 1) / kTile;
  size_t b = (size_t)n * 8 + ((size_t)n * 4 + 7) / 8 * 8 + (size_t)hist * 4 + (size_t)ptiles * 4 + 64;
  return b;
}

void radix_sort_pairs(void* temp, size_t temp_bytes, const uint64_t* k_in, uint64_t* k_out,
                      const int32_t* v_in, int32_t* v_out, int64_t n, int end_bit,
                      hipStream_t st) {
  if (n <= 0) return;
  if (temp_bytes < radix_sort_temp_bytes(n)) throw std::runtime_error("radix sort temp too small");
  const int64_t tiles = (n + kTile - 1) / kTile;
  const int64_t hist_n = (int64_t)kRadix * tiles;
  char* p = (char*)temp;
  uint64_t* kt = (uint64_t*)p;
  p += (size_t)n * 8;
  int32_t* vt = (int32_t*)p;
  p += ((size_t)n * 4 + 7) / 8 * 8;
  uint32_t* hist = (uint32_t*)p;
  p += (size_t)hist_n * 4;
  uint32_t* partials = (uint32_t*)p;
  const int passes = (end_bit + kRadixBits - 1) / kRadixBits;
  // ping-pong so that the last pass lands in k_out / v_out
  const uint64_t* src_k = k_in;
  const int32_t* src_v = v_in;
  for (int pass = 0; pass < passes; ++pass) {
    const bool to_out = ((passes - 1 - pass) % 2) == 0;
    uint64_t* dk = to_out ? k_out : kt;
    int32_t* dv = to_out ? v_out : vt;
    const int shift = pass * kRadixBits;
    radix_hist_kernel<<<(unsigned)tiles, kBlk, 0, st>>>(src_k, n, shift, hist, tiles);
    PSAMD_HIP_CHECK(hipGetLastError());
    device_scan<uint32_t>(hist, hist, hist_n, partials, false, st);
    radix_scatter_kernel<<<(unsigned)tiles, kBlk, 0, st>>>(src_k, src_v, dk, dv, n, shift, hist,
                                                           tiles);
    PSAMD_HIP_CHECK(hipGetLastError());
    src_k = dk;
    src_v = dv;
  }
  if (passes == 0) {
    copy_pairs_kernel<<<grid_for(n, 256), 256, 0, st>>>(k_in, v_in, k_out, v_out, n);
    PSAMD_HIP_CHECK(hipGetLastError());
  }
}

size_t scan_i32_temp_bytes(int64_t n) { return (size_t)((n + kTile - 1) / kTile) * 4 + 64; }

void scan_i32(const int32_t* in, int32_t* out, int64_t n, void* temp, bool inclusive,
              hipStream_t st) {
  device_scan<int32_t>(in, out, n, (int32_t*)temp, inclusive, st);
}

}  // namespace psamd
