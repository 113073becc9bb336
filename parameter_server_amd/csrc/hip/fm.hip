// Factorization machine forward + backward (one wavefront per example).
//
// Reference: src/app/factor_machine/ (fm_worker.h, fm.m). The reference FM is an
// unfinished sketch (not in the Makefile); fm.m gives the model it aims at:
//   py = x.w + 1/2 sum_f [ (sum_i x_i v_if)^2 - sum_i x_i^2 v_if^2 ]
//   p  = -y / (1 + exp(y py))              (logistic loss)
//   gv_i = p * (x_i s_f - x_i^2 v_if),  s_f = sum_j x_j v_jf
// (fm.m adds the x^2 v^2 term in the prediction; its gradient uses the standard
// minus sign, which is what is implemented here.)
//
// Inputs are the expanded embedding rows X0 [B*S, D] (bf16, rows of the pulled
// unique keys) and the pulled wide weights; x_i = vals ? vals[i] : 1. Per example:
// lanes own features f = lane, lane + 64 (D <= 128), loop over the S positions to
// build s_f and q_f = sum x^2 v^2; the wide margin is a 64-lane reduction. Outputs:
// coef[b] = p (for the wide-weight gradient), dX0[b*S+i, f] = p (x_i s_f - x_i^2 v_if)
// (bf16, reduced per unique key by emb_grad_reduce), loss / accuracy / AUC histogram.
#include "common.cuh"

#include <algorithm>
#include <stdexcept>

namespace psamd {

namespace {
__device__ __forceinline__ float bf16_to_f32(uint16_t h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ uint16_t f32_to_bf16(float f) {  // round to nearest even
  const uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);
  return (uint16_t)((u + 0x7fffu + ((u >> 16) & 1u)) >> 16);
}
}  // namespace

__global__ void __launch_bounds__(256)
fm_fwd_bwd_kernel(const uint16_t* __restrict__ X0, const float* __restrict__ vals, int64_t B,
                  int S, int D, const int32_t* __restrict__ local_col,
                  const float* __restrict__ w_local, int64_t w_cap,
                  const float* __restrict__ labels, float* __restrict__ coef_out,
                  uint16_t* __restrict__ dX0, double* __restrict__ metrics,
                  uint32_t* __restrict__ hist, int nbins, int acc_stripes) {
  extern __shared__ uint32_t lhist[];  // [2*nbins]
  for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x) lhist[i] = 0;
  __syncthreads();
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
  double loss_acc = 0, corr_acc = 0, cnt = 0;
  for (int64_t b = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6); b < B;
       b += waves) {
    const int64_t p0 = b * S;
    float s0 = 0.f, s1 = 0.f, q0 = 0.f, q1 = 0.f;
    const int f0 = lane, f1 = lane + 64;
    for (int i = 0; i < S; ++i) {
      const float x = vals ? vals[p0 + i] : 1.f;
      const uint16_t* row = X0 + (p0 + i) * D;
      if (f0 < D) {
        const float v = bf16_to_f32(row[f0]) * x;
        s0 += v;
        q0 += v * v;
      }
      if (f1 < D) {
        const float v = bf16_to_f32(row[f1]) * x;
        s1 += v;
        q1 += v * v;
      }
    }
    float part = 0.5f * (s0 * s0 - q0 + s1 * s1 - q1);
    if (lane < S) {
      const int32_t c = local_col[p0 + lane];
      const float x = vals ? vals[p0 + lane] : 1.f;
      if (in_range(c, w_cap)) part += w_local[c] * x;
    }
    const float m = wave_allsum(part);
    const float y = labels[b] > 0.f ? 1.f : -1.f;
    const float ym = y * m;
    const float tau = 1.f / (1.f + expf(ym));
    const float coef = -y * tau;
    if (lane == 0) {
      coef_out[b] = coef;
      loss_acc += ym > 20.f ? expf(-ym) : (ym < -20.f ? -ym : log1pf(expf(-ym)));
      corr_acc += ((y > 0.f) == (m > 0.f)) ? 1.0 : 0.0;
      cnt += 1.0;
      if (hist) {
        const float pr = 1.f / (1.f + expf(-m));
        const float pb = pr == pr ? fminf(fmaxf(pr * nbins, 0.f), (float)(nbins - 1)) : 0.f;
        atomicAdd(&lhist[(y > 0.f ? nbins : 0) + (int)pb], 1u);
      }
    }
    for (int i = 0; i < S; ++i) {
      const float x = vals ? vals[p0 + i] : 1.f;
      const uint16_t* row = X0 + (p0 + i) * D;
      uint16_t* drow = dX0 + (p0 + i) * D;
      if (f0 < D) drow[f0] = f32_to_bf16(coef * (x * s0 - x * x * bf16_to_f32(row[f0])));
      if (f1 < D) drow[f1] = f32_to_bf16(coef * (x * s1 - x * x * bf16_to_f32(row[f1])));
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
  if (hist) {
    __syncthreads();
    for (int i = threadIdx.x; i < 2 * nbins; i += blockDim.x)
      if (lhist[i]) atomicAdd(&hist[i], lhist[i]);
  }
}

// Narrow factors (D <= 32, S <= 64): lane = position. Each lane loads its own
// D-wide row with D / 8 16-B loads (the kernel above walks the S positions
// serially with 2-byte loads on D of 64 lanes: latency bound, 94 us at
// B = 16384, S = 39, D = 16), s_f comes from D butterfly sums, and each lane
// writes its own dX0 row with 16-B stores. 4 examples per wave; the AUC
// histogram goes straight to global (one atomic per example, no per-block
// LDS histogram to clear and flush).
//
// Gather mode (X0 == nullptr): the rows are read straight from the embedding store,
// row = rows[idx ? idx[local_col[p]] : local_col[p]], so the [B*S, D] expansion is
// never written and re-read (emb_expand 121 us + its re-read, B = 65536, D = 16).
//
// s_f = sum over the wave of x v_f for all D features: a transpose-reduce butterfly
// (each xor stage hands half of the remaining features to the partner lane, so
// D/2 + D/4 + ... + 1 shuffles, then plain xor sums for the last stages) leaves the
// total of feature f in lane bfly_lane(f); readlane broadcasts it as a wave-uniform
// value. D = 16: 17 shuffles instead of 16 full 6-stage all-sums (96).
template <int D>
__device__ __forceinline__ int bfly_lane(int f) {
  // stage k (offset 32 >> k) decides feature bit (log2(D) - 1 - k)
  int l = 0;
#pragma unroll
  for (int k = 0, n = D; n > 1; ++k, n >>= 1)
    if (f & (n >> 1)) l |= 32 >> k;
  return l;
}

template <int D>
__device__ __forceinline__ void wave_sum_vec(float (&v)[D], float (&s)[D]) {
  const int lane = threadIdx.x & 63;
  float w[D];
#pragma unroll
  for (int j = 0; j < D; ++j) w[j] = v[j];
  int off = 32;
#pragma unroll
  for (int n = D; n > 1; n >>= 1, off >>= 1) {
    const bool hi = lane & off;
#pragma unroll
    for (int j = 0; j < n / 2; ++j) {
      const float keep = hi ? w[j + n / 2] : w[j];
      const float send = hi ? w[j] : w[j + n / 2];
      w[j] = keep + __shfl_xor(send, off, 64);
    }
  }
  float t = w[0];
  for (; off > 0; off >>= 1) t += __shfl_xor(t, off, 64);
  const int ti = __float_as_int(t);
#pragma unroll
  for (int f = 0; f < D; ++f) s[f] = __int_as_float(__builtin_amdgcn_readlane(ti, bfly_lane<D>(f)));
}

template <int D>
__global__ void __launch_bounds__(256)
fm_rows_kernel(const uint16_t* __restrict__ X0, const uint16_t* __restrict__ rows,
               const int64_t* __restrict__ idx, int64_t idx_cap, int64_t rows_cap,
               const float* __restrict__ vals, int64_t B, int S,
               const int32_t* __restrict__ local_col, const float* __restrict__ w_local,
               int64_t w_cap, const float* __restrict__ labels, float* __restrict__ coef_out,
               uint16_t* __restrict__ dX0, double* __restrict__ metrics,
               uint32_t* __restrict__ hist, int nbins, int acc_stripes) {
  const int lane = threadIdx.x & 63;
  const int64_t waves = (int64_t)gridDim.x * (blockDim.x / 64);
  double loss_acc = 0, corr_acc = 0, cnt = 0;
  for (int64_t b = blockIdx.x * (int64_t)(blockDim.x / 64) + (threadIdx.x >> 6); b < B;
       b += waves) {
    const int64_t p = b * S + lane;
    const bool on = lane < S;
    const float x = on ? (vals ? vals[p] : 1.f) : 0.f;
    const int32_t col = on ? local_col[p] : -1;
    const uint16_t* src = nullptr;
    if (X0) {
      if (on) src = X0 + p * D;
    } else if (on) {
      int64_t r = col;
      if (idx) r = in_range(r, idx_cap) ? idx[r] : -1;
      if (in_range(r, rows_cap)) src = rows + r * D;  // unresolved key: zero row
    }
    float v[D];
#pragma unroll
    for (int c = 0; c < D / 8; ++c) {
      uint4 w = make_uint4(0, 0, 0, 0);
      if (src) w = reinterpret_cast<const uint4*>(src)[c];
      const uint16_t* h = reinterpret_cast<const uint16_t*>(&w);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[c * 8 + j] = bf16_to_f32(h[j]);
    }
    float part = 0.f;
    if (on && in_range(col, w_cap)) part = w_local[col] * x;
    float xv[D], s[D], s2 = 0.f;
#pragma unroll
    for (int f = 0; f < D; ++f) {
      xv[f] = x * v[f];
      part -= 0.5f * xv[f] * xv[f];
    }
    wave_sum_vec<D>(xv, s);
#pragma unroll
    for (int f = 0; f < D; ++f) s2 += s[f] * s[f];
    const float m = wave_allsum(part) + 0.5f * s2;
    const float y = labels[b] > 0.f ? 1.f : -1.f;
    const float ym = y * m;
    const float coef = -y / (1.f + expf(ym));
    if (on) {
#pragma unroll
      for (int c = 0; c < D / 8; ++c) {
        uint4 o;
        uint16_t* h = reinterpret_cast<uint16_t*>(&o);
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int f = c * 8 + j;
          h[j] = f32_to_bf16(coef * (x * s[f] - x * x * v[f]));
        }
        reinterpret_cast<uint4*>(dX0 + p * D)[c] = o;
      }
    }
    if (lane == 0) {
      coef_out[b] = coef;
      loss_acc += ym > 20.f ? expf(-ym) : (ym < -20.f ? -ym : log1pf(expf(-ym)));
      corr_acc += ((y > 0.f) == (m > 0.f)) ? 1.0 : 0.0;
      cnt += 1.0;
      if (hist) {
        const float pr = 1.f / (1.f + expf(-m));
        const float pb = pr == pr ? fminf(fmaxf(pr * nbins, 0.f), (float)(nbins - 1)) : 0.f;
        atomicAdd(&hist[(y > 0.f ? nbins : 0) + (int)pb], 1u);
      }
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
}

// dE[u, :] += lambda * v_u (L2 on the factors, once per unique key and step, as fm.m);
// v_u = rows[idx ? idx[u] : u] (bf16).
__global__ void fm_l2_kernel(float* __restrict__ dE, const uint16_t* __restrict__ rows,
                             const int64_t* __restrict__ idx, int64_t rows_cap,
                             const int32_t* __restrict__ n_dev, int64_t u_cap, int D,
                             float lambda) {
  const int64_t n = dev_len(n_dev, u_cap) * D;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < n;
       e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t u = e / D;
    const int f = (int)(e - u * D);
    const int64_t r = idx ? idx[u] : u;
    if (in_range(r, rows_cap)) dE[e] += lambda * bf16_to_f32(rows[r * D + f]);
  }
}

// X0 [B*S, D] expanded rows, or X0 == nullptr and rows [rows_cap, D] gathered through
// local_col (and idx [idx_cap] if given); the gather form needs S <= 64, D in {8, 16, 32}.
void fm_fwd_bwd(const void* X0, const void* rows, const int64_t* idx, int64_t idx_cap,
                int64_t rows_cap, const float* vals, int64_t B, int S, int D,
                const int32_t* local_col, const float* w_local, int64_t w_cap, const float* labels,
                float* coef, void* dX0, double* metrics, uint32_t* hist, int nbins,
                int acc_stripes, hipStream_t st) {
  if (S <= 64 && (D == 8 || D == 16 || D == 32)) {
    const unsigned g = (unsigned)std::min<int64_t>((B + 15) / 16, 1 << 20);
#define PSAMD_FM(DD)                                                                          \
  fm_rows_kernel<DD><<<g, 256, 0, st>>>((const uint16_t*)X0, (const uint16_t*)rows, idx, idx_cap, \
                                        rows_cap, vals, B, S, local_col, w_local, w_cap, labels, \
                                        coef, (uint16_t*)dX0, metrics, hist, hist ? nbins : 0,  \
                                        acc_stripes)
    if (D == 8) PSAMD_FM(8);
    else if (D == 16) PSAMD_FM(16);
    else PSAMD_FM(32);
#undef PSAMD_FM
    PSAMD_HIP_CHECK(hipGetLastError());
    return;
  }
  if (!X0) throw std::runtime_error("fm_fwd_bwd: row gather needs S <= 64, D in {8, 16, 32}");
  const int g = grid_for(B * 64, 256, 4096);
  fm_fwd_bwd_kernel<<<g, 256, hist ? 2 * nbins * sizeof(uint32_t) : 0, st>>>(
      (const uint16_t*)X0, vals, B, S, D, local_col, w_local, w_cap, labels, coef,
      (uint16_t*)dX0, metrics, hist, hist ? nbins : 0, acc_stripes);
  PSAMD_HIP_CHECK(hipGetLastError());
}

void fm_l2(float* dE, const void* rows, const int64_t* idx, int64_t rows_cap, const int32_t* n_dev,
           int64_t u_cap, int D, float lambda, hipStream_t st) {
  fm_l2_kernel<<<grid_for(u_cap * D, 256, 4096), 256, 0, st>>>(dE, (const uint16_t*)rows, idx,
                                                               rows_cap, n_dev, u_cap, D, lambda);
  PSAMD_HIP_CHECK(hipGetLastError());
}

}  // namespace psamd
