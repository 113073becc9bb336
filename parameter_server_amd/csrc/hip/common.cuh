// Shared device helpers for the parameter-server HIP kernels (gfx950 / CDNA4).
//
// Design notes (MI355X-first):
//  * wave64 everywhere: block sizes are multiples of 64, cross-lane reductions
//    use 64-lane shuffles, ballots are 64-bit.
//  * all sparse kernels are HBM/latency bound; they use grid-stride loops with
//    grids capped at ~8 blocks per CU (256 CUs) and read their valid length from
//    a device counter when the host does not know it (graph-capturable steps).
//  * keys are 64-bit; the "mixed" key space is a bijection of the raw key space
//    so that deduplication on mixed keys == deduplication on raw keys, and range
//    partitioning on mixed keys balances shards even for small integer ids
//    (reference partitions raw keys by range: src/system/postmaster.cc:17-31).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace psamd {

constexpr uint64_t kEmptyKey = ~0ull;
constexpr int kWave = 64;

#define PSAMD_HIP_CHECK(expr)                                                   \
  do {                                                                          \
    hipError_t _e = (expr);                                                     \
    if (_e != hipSuccess) {                                                     \
      throw std::runtime_error(std::string("HIP error ") + hipGetErrorString(_e) + \
                               " at " __FILE__ ":" + std::to_string(__LINE__)); \
    }                                                                           \
  } while (0)

// ---------------------------------------------------------------------------
// 64-bit finaliser (murmur3 fmix64) — used for table slot placement.
__host__ __device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// Bijective key mixer on [0, 2^bits): two rounds of (odd multiply mod 2^bits,
// xorshift by s >= bits/2). xorshift by s >= bits/2 is an involution, and an odd
// multiply is invertible mod 2^bits, so unmix() exists (host computes inverses).
struct KeyMix {
  uint64_t mask;   // 2^bits - 1 (all ones for bits == 64)
  uint64_t a, b;   // odd multipliers (mod 2^bits)
  uint64_t ai, bi; // their inverses mod 2^bits
  int s;           // shift, >= ceil(bits/2)
  int bits;
};

__host__ __device__ __forceinline__ uint64_t mix_key(uint64_t x, const KeyMix& m) {
  x = (x * m.a) & m.mask;
  x ^= x >> m.s;
  x = (x * m.b) & m.mask;
  x ^= x >> m.s;
  return x;
}

// mix_key for bits <= 32 in 32-bit arithmetic (the same value: products mod 2^bits only
// see the factors' low bits)
__host__ __device__ __forceinline__ uint32_t mix_key32(uint64_t x64, const KeyMix& m) {
  const uint32_t mask = (uint32_t)m.mask;
  uint32_t x = ((uint32_t)x64 * (uint32_t)m.a) & mask;
  x ^= x >> m.s;
  x = (x * (uint32_t)m.b) & mask;
  x ^= x >> m.s;
  return x;
}

__host__ __device__ __forceinline__ uint64_t unmix_key(uint64_t x, const KeyMix& m) {
  x ^= x >> m.s;
  x = (x * m.bi) & m.mask;
  x ^= x >> m.s;
  x = (x * m.ai) & m.mask;
  return x;
}

// Grid helpers ---------------------------------------------------------------
inline int grid_for(int64_t n, int block, int max_blocks = 2048) {
  int64_t g = (n + block - 1) / block;
  if (g < 1) g = 1;
  if (g > max_blocks) g = max_blocks;
  return (int)g;
}

// Valid length: from a device counter if given (clamped to the host capacity so a
// corrupted counter can never drive an out-of-bounds access), else the host n.
__device__ __forceinline__ int64_t dev_len(const int32_t* n_dev, int64_t n_host) {
  if (!n_dev) return n_host;
  const int64_t d = (int64_t)(*n_dev);
  return d < 0 ? 0 : (d > n_host ? n_host : d);
}

// Contended accumulators (loss / accuracy / optimizer stats): device-scope atomics
// on ONE address serialise (measured on MI355X: 512 blocks x 3 double atomics cost
// ~19 us of a 33 us forward kernel). A buffer of >= 64 x 16 doubles is used as 64
// stripes on separate 128-B lines, block b adding into stripe b % 64; the host sums
// the stripes. Smaller buffers (acc_stripes == 1) keep the single-address layout.
constexpr int kAccStripes = 64;
constexpr int kAccStride = 16;
__device__ __forceinline__ double* acc_stripe(double* base, int acc_stripes) {
  return base + (int64_t)(blockIdx.x % acc_stripes) * kAccStride;
}

// Index guard for gathered / scattered indices.
__device__ __forceinline__ bool in_range(int64_t i, int64_t cap) {
  return (uint64_t)i < (uint64_t)cap;
}

// One step of a wave-wide segmented inclusive scan over DPP lane moves (GFX9 DPP
// controls: 0x110 + n = row_shr:n, 0x142 = row_bcast:15, 0x143 = row_bcast:31). Lanes
// the move does not write (no source lane, or a row outside ROW_MASK) keep the "old"
// operand: segment id -2 (never equal) and value 0.
template <int CTRL, int ROW_MASK, int D>
__device__ __forceinline__ void seg_scan_step(int32_t u, float (&x)[D]) {
  const int32_t uo = __builtin_amdgcn_update_dpp(-2, u, CTRL, ROW_MASK, 0xf, false);
  const bool add = uo == u;
#pragma unroll
  for (int d = 0; d < D; ++d) {
    const float y = __int_as_float(
        __builtin_amdgcn_update_dpp(0, __float_as_int(x[d]), CTRL, ROW_MASK, 0xf, false));
    x[d] += add ? y : 0.f;
  }
}

// Sum over the wave by DPP lane moves (inclusive scan: the total lands in lane 63), no
// ds_bpermute / LDS: row_shr 1/2/4/8, then row_bcast:15 / :31 (rows outside the mask,
// and lanes without a source, take the "old" operand 0).
template <int CTRL, int ROW_MASK>
__device__ __forceinline__ double dpp_f64(double v) {
  const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, ROW_MASK, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, ROW_MASK, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_sum_dpp(double v) {
  v += dpp_f64<0x111, 0xf>(v);
  v += dpp_f64<0x112, 0xf>(v);
  v += dpp_f64<0x114, 0xf>(v);
  v += dpp_f64<0x118, 0xf>(v);
  v += dpp_f64<0x142, 0xa>(v);
  v += dpp_f64<0x143, 0xc>(v);
  return v;  // lane 63
}

// Wave-level reductions (64 lanes) -------------------------------------------
template <typename T>
__device__ __forceinline__ T wave_sum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
  return v;
}

// Sum over the wave, result in EVERY lane (xor butterfly; wave_sum is lane 0 only).
template <typename T>
__device__ __forceinline__ T wave_allsum(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_max(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T o = __shfl_down(v, off, 64);
    v = o > v ? o : v;
  }
  return v;
}

template <typename T>
__device__ __forceinline__ T wave_min(T v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    T o = __shfl_down(v, off, 64);
    v = o < v ? o : v;
  }
  return v;
}

// Block reduction of a double, result valid in thread 0. Block size <= 1024.
__device__ __forceinline__ double block_sum_f64(double v, double* lds /*[16]*/) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  if (lane == 0) lds[wid] = v;
  __syncthreads();
  double r = 0;
  if (threadIdx.x == 0) {
    const int nw = (blockDim.x + 63) >> 6;
    for (int i = 0; i < nw; ++i) r += lds[i];
  }
  __syncthreads();
  return r;
}

// Counter-based RNG (splitmix64 of (seed, index)) — deterministic per element.
__host__ __device__ __forceinline__ uint64_t rng64(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9e3779b97f4a7c15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
__host__ __device__ __forceinline__ float u01(uint64_t r) {  // (0,1]
  return ((float)(r >> 40) + 1.0f) * (1.0f / 16777216.0f);
}

// Device fill by a kernel, never hipMemsetAsync: inside a captured HIP graph a memset
// node can run on a blit/SDMA engine outside the stream order the kernels around it
// see (measured: a scratch table reset by a memset node was not reset on replay).
template <typename T>
__global__ void fill_kernel(T* __restrict__ p, int64_t n, T v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    p[i] = v;
}

template <typename T>
inline void fill_async(T* p, int64_t n, T v, hipStream_t st) {
  if (n <= 0) return;
  fill_kernel<T><<<grid_for(n, 256, 4096), 256, 0, st>>>(p, n, v);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
