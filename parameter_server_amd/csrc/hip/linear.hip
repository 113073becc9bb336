// Fused sparse linear-model kernels on localized minibatches.
//
// Reference hot loops (CPU, Eigen + thread pool):
//   Xw = X*w           SparseMatrix::times        src/util/sparse_matrix.h:73-107
//   loss/tau/objective LogitLoss::evaluate/compute src/app/linear_method/loss.h:75-97
//   grad = X^T(-y*tau) SparseMatrix::transTimes   src/util/matrix.h:57-59
//   AUC / accuracy     Evaluation::auc/accuracy   src/util/evaluation.h:22-63
// Here the forward pass computes Xw, the loss, dL/d(Xw), accuracy and a
// bucketed-AUC histogram in ONE launch (lane per example, w_local is the small
// pulled vector and stays L2 resident). The backward pass needs no atomics for
// segments that live inside a wavefront: it walks the key-sorted order from
// localisation (that order IS the CSC layout, so no CSR->CSC transpose,
// reference alterStorage sparse_matrix.h:186-241, is ever materialised) and
// does a 64-lane segmented scan; only segments that cross a wave boundary
// issue one float atomic per wave piece.
#include "common.cuh"
#include "loss.cuh"
#include <stdexcept>
#include <string>

namespace psamd {

// Loss, dL/dm, accuracy and AUC bin of one example with margin m (lane-group leader).
__device__ __forceinline__ void fwd_row_epilogue(int64_t r, float m, const float* __restrict__ labels,
                                                 int loss_type, float* __restrict__ xw_out,
                                                 float* __restrict__ coef_out,
                                                 float* __restrict__ coef2_out, uint32_t* lhist,
                                                 int nbins, double& loss_acc, double& corr_acc,
                                                 double& cnt) {
  float loss, coef, coef2;
  loss_terms(m, labels[r], loss_type, loss, coef, coef2);
  if (xw_out) xw_out[r] = m;
  coef_out[r] = coef;
  if (coef2_out) coef2_out[r] = coef2;
  loss_acc += loss;
  corr_acc += ((labels[r] > 0.f) == (m > 0.f)) ? 1.0 : 0.0;  // evaluation.h:55-57
  cnt += 1.0;
  if (lhist) atomicAdd(&lhist[auc_bin(m, labels[r], nbins)], 1u);
}

template <bool kHasRowPtr, int kLPR>
__global__ void __launch_bounds__(256)
linear_fwd_kernel(const int64_t* __restrict__ row_ptr, int64_t B, int width,
                  const int32_t* __restrict__ local_col, const float* __restrict__ vals,
                  const float* __restrict__ w_local, int64_t w_cap,
                  const float* __restrict__ labels,
                  int loss_type, float* __restrict__ xw_out, float* __restrict__ coef_out,
                  float* __restrict__ coef2_out, double* __restrict__ metrics,
                  uint32_t* __restrict__ hist, int nbins, int acc_stripes, int hist_stripes) {
  // kLPR lanes cooperate on one example (strided over its nnz, then a shuffle
  // reduction), so B = 65536 rows launch 8x more waves than lane-per-row.
  extern __shared__ uint32_t lhist[];  // [2*nbins] when hist != nullptr
  if (hist) {
    for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x) lhist[i] = 0;
    __syncthreads();
  }
  uint32_t* lh = hist ? lhist : nullptr;
  const int sub = threadIdx.x % kLPR;
  double loss_acc = 0, corr_acc = 0, cnt = 0;
  const int64_t groups_per_grid = ((int64_t)gridDim.x * blockDim.x) / kLPR;
  const int64_t g0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kLPR;
  constexpr int kRows = 4, kPer = 8;  // fixed-width fast path: 4 rows x <= 8 nnz per lane
  if (!kHasRowPtr && width <= kLPR * kPer) {
    // every load of kRows rows is issued before any gather and every gather before
    // the reductions: 2 dependent memory latencies per kRows rows, not 2 per row
    for (int64_t r0 = g0; r0 < ((B + groups_per_grid * kRows - 1) / (groups_per_grid * kRows)) *
                                   groups_per_grid * kRows;
         r0 += groups_per_grid * kRows) {
      int32_t c[kRows][kPer];
      float xv[kRows][kPer];
#pragma unroll
      for (int q = 0; q < kRows; ++q) {
        const int64_t r = r0 + q * groups_per_grid;
#pragma unroll
        for (int j = 0; j < kPer; ++j) {
          const int k = j * kLPR + sub;
          const bool ok = r < B && k < width;
          c[q][j] = ok ? local_col[r * width + k] : -1;
          xv[q][j] = (ok && vals) ? vals[r * width + k] : 1.f;
        }
      }
      float m[kRows];
#pragma unroll
      for (int q = 0; q < kRows; ++q) {
        m[q] = 0.f;
#pragma unroll
        for (int j = 0; j < kPer; ++j)
          if (in_range(c[q][j], w_cap)) m[q] += w_local[c[q][j]] * xv[q][j];
#pragma unroll
        for (int off = kLPR / 2; off > 0; off >>= 1) m[q] += __shfl_xor(m[q], off, 64);
      }
      if (sub == 0) {
#pragma unroll
        for (int q = 0; q < kRows; ++q) {
          const int64_t r = r0 + q * groups_per_grid;
          if (r < B)
            fwd_row_epilogue(r, m[q], labels, loss_type, xw_out, coef_out, coef2_out, lh, nbins,
                             loss_acc, corr_acc, cnt);
        }
      }
    }
  } else {
    for (int64_t r = g0; r < ((B + groups_per_grid - 1) / groups_per_grid) * groups_per_grid;
         r += groups_per_grid) {
      const bool row_ok = r < B;
      int64_t b = 0, e = 0;
      if (row_ok) {
        if (kHasRowPtr) { b = row_ptr[r]; e = row_ptr[r + 1]; }
        else { b = r * width; e = b + width; }
      }
      float m = 0.f;
      for (int64_t k = b + sub; k < e; k += kLPR) {
        const int32_t c = local_col[k];
        if (in_range(c, w_cap)) m += vals ? w_local[c] * vals[k] : w_local[c];
      }
#pragma unroll
      for (int off = kLPR / 2; off > 0; off >>= 1) m += __shfl_xor(m, off, 64);
      if (!row_ok || sub != 0) continue;
      fwd_row_epilogue(r, m, labels, loss_type, xw_out, coef_out, coef2_out, lh, nbins, loss_acc,
                       corr_acc, cnt);
    }
  }
  if (metrics) {  // per-wave DPP sums, lane 63 adds (no barriers)
    const double a = wave_sum_dpp(loss_acc), c = wave_sum_dpp(corr_acc), n = wave_sum_dpp(cnt);
    if ((threadIdx.x & 63) == 63 && n > 0) {
      double* mt = acc_stripe(metrics, acc_stripes);
      atomicAdd(&mt[0], a);
      atomicAdd(&mt[1], c);
      atomicAdd(&mt[2], n);
    }
  }
  if (hist) {  // flush into stripe blockIdx % hist_stripes (popular bins are contended)
    __syncthreads();
    uint32_t* hs = hist + (int64_t)(blockIdx.x % hist_stripes) * 2 * nbins;
    for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x)
      if (lhist[i]) atomicAdd(&hs[i], lhist[i]);
  }
}

// grad[u] = sum_{i in seg u} coef[row(pos_s[i])] * val[pos_s[i]]   (and hess with val^2)
__global__ void __launch_bounds__(256)
linear_bwd_kernel(const int32_t* __restrict__ pos_s, const int32_t* __restrict__ segid,
                  int64_t n, const int32_t* __restrict__ rows, int width,
                  const float* __restrict__ vals, const float* __restrict__ coef, int64_t B,
                  const float* __restrict__ coef2, float* __restrict__ grad,
                  float* __restrict__ hess, int64_t grad_cap) {
  const int lane = threadIdx.x & 63;
  // One element per lane; each wavefront is one segmented-scan unit.
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i0 = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); i0 < n;
       i0 += stride) {
    const int64_t i = i0 + lane;
    const bool valid = i < n;
    int32_t s = -1;
    float v = 0.f, v2 = 0.f;
    if (valid) {
      s = segid[i];
      const int32_t p = pos_s[i];
      if (in_range(p, n)) {
        const int32_t r = rows ? rows[p] : (int32_t)((uint32_t)p / (uint32_t)width);
        if (in_range(r, B)) {
          const float x = vals ? vals[p] : 1.f;
          v = coef[r] * x;
          if (hess) v2 = coef2[r] * x * x;
        }
      }
    }
    // segmented inclusive scan (Hillis-Steele) over 64 lanes
#pragma unroll
    for (int off = 1; off < 64; off <<= 1) {
      const float vo = __shfl_up(v, off, 64);
      const float v2o = __shfl_up(v2, off, 64);
      const int32_t so = __shfl_up(s, off, 64);
      if (lane >= off && so == s) { v += vo; v2 += v2o; }
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
      if (!in_range(u, grad_cap)) {
        // corrupted segment id: drop (never write out of bounds)
      } else if (starts_inside && ends_inside) {
        grad[u] = v;
        if (hess) hess[u] = v2;
      } else {
        atomicAdd(&grad[u], v);
        if (hess) atomicAdd(&hess[u], v2);
      }
    }
  }
}

// Bucketed AUC of one minibatch from its histogram (auc_hist_block, loss.cuh).
__global__ void auc_from_hist_kernel(uint32_t* __restrict__ hist, int nbins, int hist_stripes,
                                     double* __restrict__ metrics,
                                     int64_t* __restrict__ step_counter) {
  auc_hist_block(hist, nbins, hist_stripes, metrics, step_counter);
}

// Expand a CSR row pointer into a per-nnz row index (COO rows).
__global__ void csr_rows_kernel(const int64_t* __restrict__ row_ptr, int64_t B,
                                int32_t* __restrict__ rows) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < B;
       r += (int64_t)gridDim.x * blockDim.x) {
    for (int64_t k = row_ptr[r]; k < row_ptr[r + 1]; ++k) rows[k] = (int32_t)r;
  }
}

// ---------------------------------------------------------------------------
// Criteo-shaped synthetic minibatch: 13 integer slots (log-bucketised counts) + 26
// categorical slots with per-slot cardinalities and power-law ids, hashed into
// [0, num_features). Labels from a planted sparse logistic model shared by every
// seed (the ranks of a data-parallel job sample rows of ONE ground truth).
//
// Cost model (the generator runs inside every timed step): 32-bit hashes only (a
// 64-bit multiply is 4 VALU ops on CDNA), the power-law inverse CDF on the native
// v_log_f32 / v_exp_f32, the planted weights from a 256-entry Gaussian quantile table
// instead of Box-Muller (no log / sqrt / cos, no divergent branch), and the key hash
// a 32-bit bijection + multiply-shift range reduction when num_features <= 2^32.
// ops/synthetic.py holds the bit-for-bit CPU reference (numpy f32 log2 / exp2 may
// differ from the hardware approximations in the last ulp for a few keys).
__constant__ uint32_t c_cards[26];
__constant__ float c_gauss[256];  // 0.6 * Phi^-1((i + 0.5) / 256)

__host__ __device__ __forceinline__ uint32_t gen_mix32(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}
// uniform bits of (global row, stream s)
__device__ __forceinline__ uint32_t gen_row_bits(uint64_t gr, uint32_t s) {
  return gen_mix32((uint32_t)gr ^ gen_mix32((uint32_t)(gr >> 32) ^ s));
}
__device__ __forceinline__ float gen_u01(uint32_t x) {  // (0, 1]
  return (float)((x >> 8) + 1u) * (1.0f / 16777216.0f);
}
__device__ __forceinline__ float gen_planted(uint64_t key) {  // ~20 % of keys carry signal
  const uint32_t h = gen_mix32((uint32_t)key ^ gen_mix32((uint32_t)(key >> 32) ^ 0x5bd1e995u));
  return (h & 0xffu) < 51u ? c_gauss[h >> 24] : 0.f;
}

// h % N without a 64-bit division: Barrett reduction with m = floor((2^64 - 1) / N);
// q = umulhi(h, m) undershoots floor(h / N) by at most 2 -> <= 2 corrections. Exact.
__device__ __forceinline__ uint64_t mod_barrett(uint64_t h, uint64_t N, uint64_t m) {
  uint64_t r = h - __umul64hi(h, m) * N;
  if (r >= N) r -= N;
  if (r >= N) r -= N;
  return r;
}

// uniform u -> feature id of slot j -> key. Integer slots: a heavy-tailed count
// x = e^(12u) - 1 log2-bucketised, floor(2 log2(1 + x)) = floor(u * 24 log2 e).
// Categorical slots: power-law id x = (cm1 u + 1)^(1 / (1 - alpha)) - 1, cm1 =
// C_j^(1 - alpha) - 1. (j is wave-uniform at every call site: no divergence.)
template <bool kWide>
__device__ __forceinline__ uint64_t gen_key(float u, int j, uint64_t num_features, uint64_t nf_m,
                                            float inv_oma, float cm1) {
  uint32_t id;
  if (j < 13) {
    id = (uint32_t)(u * 34.62468098f);
  } else {
    const float x = __builtin_amdgcn_exp2f(inv_oma * __builtin_amdgcn_logf(cm1 * u + 1.f));
    const uint32_t v = (uint32_t)x;
    id = v >= 1u ? v - 1u : 0u;
  }
  if (!kWide)  // bijective 32-bit hash per slot, multiply-shift into [0, N), N <= 2^32
    return ((uint64_t)gen_mix32(id + 0x9e3779b9u * (uint32_t)(j + 1)) * num_features) >> 32;
  return mod_barrett(fmix64(((uint64_t)(j + 1) << 48) ^ id), num_features, nf_m);
}

// 64 rows per block, one per lane; 6 waves, wave w generating a fixed run of slots of
// every row (integer slots 0-6 / 7-12 in waves 0-1, categorical 13-19 / 20-25 / 26-32 /
// 33-38 in waves 2-5: the slot index is wave-uniform, so the integer and power-law
// branches never diverge). (Round 3 used 3 waves of 13 slots: 12 waves per CU and 13
// sequential samples per lane, 11 us per 65,536-row minibatch.) Keys and the planted
// weight of every (row, slot) are staged in LDS; the keys leave as one contiguous
// 64 x 39 x 8 B run, and lane r of wave 0 sums row r's planted weights in the
// original order (three sequential 13-slot sums, then -1.2 + s0 + s1 + s2: bitwise the
// labels of the 3-wave kernel) and draws the label.
constexpr int kGenRows = 64;
constexpr int kGenThreads = 384;
__device__ __forceinline__ void gen_slot_range(int w, int& j0, int& j1) {
  // w = 0..5 -> [0, 7) [7, 13) [13, 20) [20, 26) [26, 33) [33, 39)
  j0 = (w >> 1) * 13 + (w & 1) * 7;
  j1 = (w & 1) ? ((w >> 1) + 1) * 13 : j0 + 7;
}
template <bool kWide>
__global__ void __launch_bounds__(kGenThreads)
criteo_gen_kernel(uint64_t seed, int64_t row0, const int64_t* __restrict__ row0_dev,
                  int64_t row_scale, int64_t B, uint64_t num_features, uint64_t nf_m,
                  float alpha, uint64_t* __restrict__ keys, float* __restrict__ labels,
                  int64_t* __restrict__ row0_out) {
  __shared__ uint64_t sk[kGenRows * 39];
  __shared__ float sp[kGenRows * 39];
  __shared__ float s_cm1[26];
  __shared__ uint32_t s_seed[40];  // per-slot streams + the label stream
  // (an L2-coherent vector load, not a scalar-cache load: the counter is advanced on the
  // device between graph replays)
  int64_t cursor = 0;
  if (row0_dev) {
    cursor = __hip_atomic_load(row0_dev, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    row0 += cursor * row_scale;
  }
  const int t = threadIdx.x, lane = t & 63;
  // row0_out: the cursor of the NEXT launch, in a second word (ping-pong: the launch
  // after this one reads row0_out and writes this launch's row0_dev), written by one
  // lane: no block reads what another writes within a launch, no atomics. (A completion
  // counter on one address, bumped by each of the 1024 blocks, serialised them: 21 -> 55
  // us per launch in the pipelined 8-peer step, profiles/r5_gen_cursor.log.)
  if (row0_out && blockIdx.x == 0 && t == 0) row0_out[0] = cursor + 1;
  const int g = __builtin_amdgcn_readfirstlane(t >> 6);
  int j0, j1;
  gen_slot_range(g, j0, j1);
  const float oma = 1.f - alpha, inv_oma = 1.f / oma;
  if (t < 26) s_cm1[t] = powf((float)c_cards[t], oma) - 1.f;
  if (t < 40)
    s_seed[t] = gen_mix32((uint32_t)seed ^
                          gen_mix32((uint32_t)(seed >> 32) + 0x9e3779b9u * (uint32_t)(t + 1)));
  __syncthreads();
  for (int64_t rb = (int64_t)blockIdx.x * kGenRows; rb < B; rb += (int64_t)gridDim.x * kGenRows) {
    const int64_t r = rb + lane;
    const uint64_t gr = (uint64_t)(row0 + r);
    if (r < B) {
#pragma unroll
      for (int jj = 0; jj < 7; ++jj) {  // (fixed trip count: the 6-7 samples interleave)
        const int j = j0 + jj;
        if (j >= j1) break;
        const float u = gen_u01(gen_row_bits(gr, s_seed[j]));
        const uint64_t key = gen_key<kWide>(u, j, num_features, nf_m, inv_oma,
                                            j >= 13 ? s_cm1[j - 13] : 0.f);
        sk[lane * 39 + j] = key;
        sp[lane * 39 + j] = gen_planted(key);
      }
    }
    __syncthreads();
    const int nrow = (int)min<int64_t>(kGenRows, B - rb);
    for (int i = t; i < nrow * 39; i += kGenThreads) keys[rb * 39 + i] = sk[i];
    if (g == 0 && r < B) {
      float spw[3];
#pragma unroll
      for (int q = 0; q < 3; ++q) {
        float pw = 0.f;
        for (int jj = 0; jj < 13; ++jj) pw += sp[lane * 39 + q * 13 + jj];
        spw[q] = pw;
      }
      const float logit = -1.2f + spw[0] + spw[1] + spw[2];
      const float p = 1.f / (1.f + __expf(-logit));
      labels[r] = gen_u01(gen_row_bits(gr, s_seed[39])) < p ? 1.f : -1.f;
    }
    __syncthreads();
  }
}

// ---------------------------------------------------------------------------
void linear_fwd(const int64_t* row_ptr, int64_t B, int width, const int32_t* local_col,
                const float* vals, const float* w_local, int64_t w_cap, const float* labels,
                int loss_type,
                float* xw, float* coef, float* coef2, double* metrics, uint32_t* hist, int nbins,
                int acc_stripes, int hist_stripes, hipStream_t st) {
  const size_t lds = hist ? (size_t)2 * nbins * sizeof(uint32_t) : 0;
  constexpr int kLPR = 8;
  // cap the grid: each block zeroes and scans a 2*nbins LDS histogram (measured: a
  // 2048-block grid makes that the bottleneck, 90 us vs 37 us at 512 blocks)
  const int g = grid_for(B * kLPR, 256, 512);
  if (row_ptr)
    linear_fwd_kernel<true, kLPR><<<g, 256, lds, st>>>(row_ptr, B, width, local_col, vals, w_local,
                                                 w_cap, labels, loss_type, xw, coef, coef2, metrics,
                                                 hist, nbins, acc_stripes, hist_stripes);
  else
    linear_fwd_kernel<false, kLPR><<<g, 256, lds, st>>>(row_ptr, B, width, local_col, vals, w_local,
                                                  w_cap, labels, loss_type, xw, coef, coef2, metrics,
                                                  hist, nbins, acc_stripes, hist_stripes);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void linear_bwd(const int32_t* pos_s, const int32_t* segid, int64_t n, const int32_t* rows,
                int width, const float* vals, const float* coef, int64_t B, const float* coef2,
                float* grad, float* hess, int64_t grad_cap, hipStream_t st) {
  linear_bwd_kernel<<<grid_for(n, 256, 8192), 256, 0, st>>>(pos_s, segid, n, rows, width, vals,
                                                            coef, B, coef2, grad, hess, grad_cap);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void auc_from_hist(uint32_t* hist, int nbins, int hist_stripes, double* metrics,
                   int64_t* step_counter, hipStream_t st) {
  auc_from_hist_kernel<<<1, 256, 0, st>>>(hist, nbins, hist_stripes, metrics, step_counter);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void csr_rows(const int64_t* row_ptr, int64_t B, int32_t* rows, hipStream_t st) {
  csr_rows_kernel<<<grid_for(B, 256), 256, 0, st>>>(row_ptr, B, rows);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void criteo_set_tables(const uint32_t* cards26, const float* gauss256) {
  PSAMD_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_cards), cards26, 26 * sizeof(uint32_t)));
  PSAMD_HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(c_gauss), gauss256, 256 * sizeof(float)));
}

void criteo_gen(uint64_t seed, int64_t row0, const int64_t* row0_dev, int64_t row_scale,
                int64_t B, uint64_t num_features, float alpha, uint64_t* keys, float* labels,
                int64_t* row0_out, hipStream_t st) {
  const int64_t blocks = (B + kGenRows - 1) / kGenRows;
  const uint64_t nf_m = ~0ull / num_features;
  const unsigned grid = (unsigned)(blocks < 65535 ? blocks : 65535);
  if (num_features <= (1ull << 32))
    criteo_gen_kernel<false><<<grid, kGenThreads, 0, st>>>(seed, row0, row0_dev, row_scale, B,
                                                           num_features, nf_m, alpha, keys, labels,
                                                           row0_dev ? row0_out : nullptr);
  else
    criteo_gen_kernel<true><<<grid, kGenThreads, 0, st>>>(seed, row0, row0_dev, row_scale, B,
                                                          num_features, nf_m, alpha, keys, labels,
                                                          row0_dev ? row0_out : nullptr);
  PSAMD_HIP_CHECK(hipGetLastError());
}

__global__ void add_i64_kernel(int64_t* p, int64_t v) { *p += v; }

void add_i64(int64_t* p, int64_t v, hipStream_t st) {
  add_i64_kernel<<<1, 1, 0, st>>>(p, v);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
