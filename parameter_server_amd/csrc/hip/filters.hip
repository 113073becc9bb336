// Tail-feature filter (CountMin) and message-filter kernels.
//
// CountMin: reference CountMin<K,uint8> (src/util/countmin.h:8-48) with the
// murmur-style 64->32 sketch hash (src/util/sketch.h:20-33), k <= 30 probes by
// double hashing, saturating uint8 counters (v_max 254 from
// src/parameter/frequency_filter.h:17). Here the byte counters live in HBM and
// are updated with a 32-bit CAS loop on the containing word, so concurrent
// inserts of different keys that share a word never lose an increment.
//
// FixingFloat (reference src/filter/fixing_float.h:44-95): min/max reduce, then
// quantise to `nbytes` fixed point with stochastic rounding. The reference adds an
// independent random bit (biased); here rounding up happens with probability equal
// to the fractional part (unbiased), using a counter-based RNG per element.
//
// Key signature (reference KeyCachingFilter: crc32c of the first <= 2048 key
// bytes, src/filter/key_caching.h:18,43): a whole-array, position-dependent
// 64-bit hash computed on device so the key list never leaves HBM.
#include "common.cuh"
#include "countmin.cuh"
#include <stdexcept>
#include <string>

namespace psamd {

__global__ void cm_insert_kernel(CmArgs a, const uint64_t* __restrict__ keys,
                                 const uint8_t* __restrict__ counts, int64_t n_host,
                                 const int32_t* __restrict__ n_dev) {
  const int64_t n = dev_len(n_dev, n_host);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    cm_insert_key(a, keys[i], counts ? counts[i] : 1u);
}

// Tail-filter insert of a localised minibatch (reference MinibatchReader::read,
// src/learner/sgd.h:140-146): count of unique key i = its occurrences
// seg_start[i+1] - seg_start[i], saturated to a byte; device unique count.
__global__ void cm_insert_seg_kernel(CmArgs a, const uint64_t* __restrict__ keys,
                                     const int32_t* __restrict__ seg_start, int64_t n_host,
                                     const int32_t* __restrict__ n_dev) {
  const int64_t n = dev_len(n_dev, n_host);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t occ = seg_start[i + 1] - seg_start[i];
    cm_insert_key(a, keys[i], occ <= 0 ? 0u : (occ > 255 ? 255u : (uint32_t)occ));
  }
}

// keep[i] = (min count > freq) ; also returns the min count.
__global__ void cm_query_kernel(CmArgs a, const uint64_t* __restrict__ keys, int64_t n_host,
                                const int32_t* __restrict__ n_dev, int32_t* __restrict__ keep,
                                uint8_t* __restrict__ out_count) {
  const int64_t n = dev_len(n_dev, n_host);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const uint32_t res = cm_query_key(a, keys[i]);
    if (keep) keep[i] = (int)res > a.freq ? 1 : 0;
    if (out_count) out_count[i] = (uint8_t)res;
  }
}

// Compaction of kept entries given keep flags and their inclusive scan.
__global__ void compact_kept_kernel(const int32_t* __restrict__ keep,
                                    const int32_t* __restrict__ incl, int64_t n_host,
                                    const int32_t* __restrict__ n_dev,
                                    int32_t* __restrict__ kept_idx, int32_t* __restrict__ n_kept,
                                    int32_t* __restrict__ remap,
                                    const uint64_t* __restrict__ keys_in,
                                    uint64_t* __restrict__ keys_out) {
  const int64_t n = dev_len(n_dev, n_host);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const int32_t dst = incl[i] - 1;
    if (keep[i] && in_range(dst, n_host)) {
      kept_idx[dst] = (int32_t)i;
      if (keys_out) keys_out[dst] = keys_in[i];
    }
    if (remap) remap[i] = keep[i] ? dst : -1;
    if (i == n - 1) *n_kept = incl[i];
  }
  if (n == 0 && blockIdx.x == 0 && threadIdx.x == 0) *n_kept = 0;
}

// ---------------------------------------------------------------------------
__global__ void minmax_kernel(const float* __restrict__ x, int64_t n, float* __restrict__ mm) {
  float lo = 3.4e38f, hi = -3.4e38f;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    const float v = x[i];
    if (v == v) { lo = fminf(lo, v); hi = fmaxf(hi, v); }
  }
  lo = wave_min(lo);
  hi = wave_max(hi);
  if ((threadIdx.x & 63) == 0) {
    // order-preserving int mapping for float atomics min/max
    int ilo = __float_as_int(lo), ihi = __float_as_int(hi);
    ilo = ilo >= 0 ? ilo : ilo ^ 0x7fffffff;
    ihi = ihi >= 0 ? ihi : ihi ^ 0x7fffffff;
    atomicMin((int*)&mm[0], ilo);
    atomicMax((int*)&mm[1], ihi);
  }
}

__device__ __forceinline__ int ord_int(float f) {
  const int b = __float_as_int(f);
  return b >= 0 ? b : b ^ 0x7fffffff;
}

__global__ void minmax_init_kernel(float* __restrict__ mm) {
  ((int*)mm)[0] = ord_int(3.4e38f);
  ((int*)mm)[1] = ord_int(-3.4e38f);
}

__global__ void minmax_finish_kernel(float* __restrict__ mm, float eps) {
  int a = __float_as_int(mm[0]), b = __float_as_int(mm[1]);
  a = a >= 0 ? a : a ^ 0x7fffffff;
  b = b >= 0 ? b : b ^ 0x7fffffff;
  mm[0] = __int_as_float(a);
  mm[1] = __int_as_float(b) + eps;  // reference: max + 1e-6 to avoid max == min
}

__global__ void ff_encode_kernel(const float* __restrict__ x, int64_t n,
                                 const float* __restrict__ mm, int nbytes, uint64_t seed,
                                 uint8_t* __restrict__ out) {
  const float lo = mm[0], hi = mm[1];
  const double bin = (double)hi - (double)lo;
  const double ratio = (double)((1ull << (8 * nbytes)) - 2ull);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    float v = x[i];
    v = v > hi ? hi : (v < lo ? lo : v);
    const double t = ((double)v - lo) / bin * ratio;
    const double f = floor(t);
    const double u = (double)u01(rng64(seed, (uint64_t)i)) - 1e-12;
    uint64_t r = (uint64_t)f + ((t - f) > u ? 1ull : 0ull);
    for (int j = 0; j < nbytes; ++j) { out[i * nbytes + j] = (uint8_t)(r & 0xff); r >>= 8; }
  }
}

__global__ void ff_decode_kernel(const uint8_t* __restrict__ code, int64_t n,
                                 const float* __restrict__ mm, int nbytes,
                                 float* __restrict__ out) {
  const float lo = mm[0], hi = mm[1];
  const double bin = (double)hi - (double)lo;
  const double ratio = (double)((1ull << (8 * nbytes)) - 2ull);
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    uint64_t r = 0;
    for (int j = 0; j < nbytes; ++j) r |= (uint64_t)code[i * nbytes + j] << (8 * j);
    out[i] = (float)((double)r / ratio * bin + lo);
  }
}

__global__ void key_signature_kernel(const uint64_t* __restrict__ keys, int64_t n,
                                     unsigned long long* __restrict__ sig) {
  unsigned long long acc = 0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x) {
    acc += fmix64(keys[i] ^ fmix64((uint64_t)i + 0x9e3779b97f4a7c15ull));
  }
  acc = wave_sum(acc);
  if ((threadIdx.x & 63) == 0 && acc) atomicAdd(sig, acc);
}

// ---------------------------------------------------------------------------
// (rsize: cells per region; rshift >= 64: one region of rsize cells)
void cm_insert(uint32_t* table, uint64_t rsize, int rshift, int k, uint32_t vmax,
               const uint64_t* keys, const uint8_t* counts, int64_t n, const int32_t* n_dev,
               hipStream_t st) {
  const CmArgs a{table, rsize, rshift, k, vmax, 0, 0};
  cm_insert_kernel<<<grid_for(n, 256), 256, 0, st>>>(a, keys, counts, n, n_dev);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void cm_query(const uint32_t* table, uint64_t rsize, int rshift, int k, uint32_t vmax,
              const uint64_t* keys, int64_t n, const int32_t* n_dev, int freq, int32_t* keep,
              uint8_t* out_count, hipStream_t st) {
  const CmArgs a{const_cast<uint32_t*>(table), rsize, rshift, k, vmax, freq, 0};
  cm_query_kernel<<<grid_for(n, 256), 256, 0, st>>>(a, keys, n, n_dev, keep, out_count);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void cm_insert_seg(uint32_t* table, uint64_t rsize, int rshift, int k, uint32_t vmax,
                   const uint64_t* keys, const int32_t* seg_start, int64_t n, const int32_t* n_dev,
                   hipStream_t st) {
  const CmArgs a{table, rsize, rshift, k, vmax, 0, 0};
  cm_insert_seg_kernel<<<grid_for(n, 256), 256, 0, st>>>(a, keys, seg_start, n, n_dev);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void compact_kept(const int32_t* keep, const int32_t* incl, int64_t n, const int32_t* n_dev,
                  int32_t* kept_idx, int32_t* n_kept, int32_t* remap, const uint64_t* keys_in,
                  uint64_t* keys_out, hipStream_t st) {
  compact_kept_kernel<<<grid_for(n, 256), 256, 0, st>>>(keep, incl, n, n_dev, kept_idx, n_kept,
                                                        remap, keys_in, keys_out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void ff_minmax(const float* x, int64_t n, float* mm, hipStream_t st) {
  minmax_init_kernel<<<1, 1, 0, st>>>(mm);
  PSAMD_HIP_CHECK(hipGetLastError());
  minmax_kernel<<<grid_for(n, 256), 256, 0, st>>>(x, n, mm);
  PSAMD_HIP_CHECK(hipGetLastError());
  minmax_finish_kernel<<<1, 1, 0, st>>>(mm, 1e-6f);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void ff_encode(const float* x, int64_t n, const float* mm, int nbytes, uint64_t seed,
               uint8_t* out, hipStream_t st) {
  ff_encode_kernel<<<grid_for(n, 256), 256, 0, st>>>(x, n, mm, nbytes, seed, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void ff_decode(const uint8_t* code, int64_t n, const float* mm, int nbytes, float* out,
               hipStream_t st) {
  ff_decode_kernel<<<grid_for(n, 256), 256, 0, st>>>(code, n, mm, nbytes, out);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void key_signature(const uint64_t* keys, int64_t n, unsigned long long* sig, hipStream_t st) {
  fill_async<unsigned long long>(sig, 1, 0ull, st);
  key_signature_kernel<<<grid_for(n, 256, 1024), 256, 0, st>>>(keys, n, sig);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
