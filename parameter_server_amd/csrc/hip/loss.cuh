// Per-example loss terms shared by the linear-model forward kernels (linear.hip,
// tploc.hip). Reference: LogitLoss / SquareHingeLoss ... (src/app/linear_method/loss.h:75-97).
#pragma once
#include "common.cuh"

namespace psamd {

enum LossType : int { kSquare = 1, kLogit = 2, kHinge = 3, kSquareHinge = 4 };

__device__ __forceinline__ float softplus(float x) {
  return x > 20.f ? x : (x < -20.f ? expf(x) : log1pf(expf(x)));
}

// loss(m), dL/dm and d2L/dm2 of one example with margin m and label `label`.
__device__ __forceinline__ void loss_terms(float m, float label, int loss_type, float& loss,
                                           float& coef, float& coef2) {
  const float y = label > 0.f ? 1.f : -1.f;
  const float ym = y * m;
  switch (loss_type) {
    case kSquare: {
      const float d = m - label;
      loss = 0.5f * d * d; coef = d; coef2 = 1.f;
      break;
    }
    case kHinge:
      loss = fmaxf(0.f, 1.f - ym); coef = ym < 1.f ? -y : 0.f; coef2 = 0.f;
      break;
    case kSquareHinge: {
      const float h = fmaxf(0.f, 1.f - ym);
      loss = h * h; coef = -2.f * y * h; coef2 = ym < 1.f ? 2.f : 0.f;
      break;
    }
    default: {  // logit: tau = 1/(1+exp(y m))
      loss = softplus(-ym);
      const float tau = 1.f / (1.f + expf(ym));
      coef = -y * tau; coef2 = tau * (1.f - tau);
      break;
    }
  }
}

// Bucketed-AUC bin of an example (positives in the upper half of the histogram).
__device__ __forceinline__ int auc_bin(float m, float label, int nbins) {
  const float p = 1.f / (1.f + expf(-m));
  const float pb = p == p ? fminf(fmaxf(p * nbins, 0.f), (float)(nbins - 1)) : 0.f;
  return (label > 0.f ? nbins : 0) + (int)pb;
}

// Bucketed AUC of one minibatch from its histogram; metrics[3] += auc, metrics[4] += 1.
// Resets the histogram (so the next step starts clean inside a captured graph).
// Run by ONE whole 256-thread block (auc_from_hist_kernel, or block 0 of the KV update
// that follows the fused forward: one launch less per step).
// kBatch: stripes loaded per round (2 halves the dependent round trips for +16 VGPRs in
// this block; measured neutral in tpf_step / tpf_pack_grads, gpurun r6z: 1 everywhere)
template <int kBatch = 1>
__device__ __forceinline__ void auc_hist_block(uint32_t* __restrict__ hist, int nbins,
                                               int hist_stripes, double* __restrict__ metrics,
                                               int64_t* __restrict__ step_counter) {
  // Exact integer AUC: 2 * area = sum_b pos_b * (2 * neg_below_b + neg_b) fits u64
  // (counts <= 2^32). Thread t owns the contiguous bins [t*kPer, t*kPer + kPer) of
  // every stripe; the stripe loads go in batches of kBatch (one memory latency per
  // batch), the stripes are zeroed for the next graph-replayed step, and the
  // cross-thread prefix is a wave-shuffle scan + 4-wave combine. kBatch = 1 keeps this
  // epilogue at 16 VGPRs of loads: with all 8 stripes in flight (128 VGPRs) it set the
  // register count of the whole kernel it is folded into (kv_update 126 VGPRs + 16
  // spilled, 4 waves per SIMD for every block, not just block 0; now 58, 8 waves). The
  // 1-GPU step did not change measurably (A/B on one box, 3 runs each: 0.1301 vs 0.1288
  // ms, within run-to-run noise): the update is bound by its random slot lines.
  constexpr int kPer = 8;  // nbins == 256 * kPer (AUC_BINS = 2048), checked on the host
  constexpr int kMaxStripes = 8;
  __shared__ unsigned long long s_w[3][4];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;  // blockDim.x == 256
  const int lo = t * kPer;
  uint32_t nb[kPer], pb[kPer];
#pragma unroll
  for (int q = 0; q < kPer; ++q) nb[q] = pb[q] = 0;
#pragma unroll 1
  for (int s0 = 0; s0 < kMaxStripes && s0 < hist_stripes; s0 += kBatch) {
    uint4 ln[kBatch][2], lp[kBatch][2];
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int sp = s0 + b;
      if (sp < hist_stripes) {
        const uint4* hn = reinterpret_cast<const uint4*>(hist + (int64_t)sp * 2 * nbins + lo);
        const uint4* hp =
            reinterpret_cast<const uint4*>(hist + (int64_t)sp * 2 * nbins + nbins + lo);
        ln[b][0] = hn[0]; ln[b][1] = hn[1];
        lp[b][0] = hp[0]; lp[b][1] = hp[1];
      }
    }
#pragma unroll
    for (int b = 0; b < kBatch; ++b) {
      const int sp = s0 + b;
      if (sp < hist_stripes) {
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          nb[4 * h + 0] += ln[b][h].x; nb[4 * h + 1] += ln[b][h].y;
          nb[4 * h + 2] += ln[b][h].z; nb[4 * h + 3] += ln[b][h].w;
          pb[4 * h + 0] += lp[b][h].x; pb[4 * h + 1] += lp[b][h].y;
          pb[4 * h + 2] += lp[b][h].z; pb[4 * h + 3] += lp[b][h].w;
        }
        uint4* zn = reinterpret_cast<uint4*>(hist + (int64_t)sp * 2 * nbins + lo);
        uint4* zp = reinterpret_cast<uint4*>(hist + (int64_t)sp * 2 * nbins + nbins + lo);
        const uint4 z = make_uint4(0, 0, 0, 0);
        zn[0] = z; zn[1] = z; zp[0] = z; zp[1] = z;
      }
    }
  }
  unsigned long long neg = 0, pos = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) { neg += nb[q]; pos += pb[q]; }
  unsigned long long x = neg;  // inclusive wave scan of negatives
#pragma unroll
  for (int off = 1; off < 64; off <<= 1) {
    const unsigned long long y = __shfl_up(x, off, 64);
    if (lane >= off) x += y;
  }
  const unsigned long long wpos = wave_sum(pos);
  if (lane == 63) s_w[0][w] = x;
  if (lane == 0) s_w[1][w] = wpos;
  __syncthreads();
  unsigned long long before = 0, Ntot = 0, Ptot = 0;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    if (q < w) before += s_w[0][q];
    Ntot += s_w[0][q];
    Ptot += s_w[1][q];
  }
  unsigned long long below = before + x - neg, area2 = 0;
#pragma unroll
  for (int q = 0; q < kPer; ++q) {
    area2 += (unsigned long long)pb[q] * (2 * below + nb[q]);
    below += nb[q];
  }
  area2 = wave_sum(area2);
  if (lane == 0) s_w[2][w] = area2;
  __syncthreads();
  if (t == 0) {
    const unsigned long long A2 = s_w[2][0] + s_w[2][1] + s_w[2][2] + s_w[2][3];
    if (Ptot > 0 && Ntot > 0) {
      metrics[3] += 0.5 * (double)A2 / ((double)Ptot * (double)Ntot);
      metrics[4] += 1.0;
    }
    if (step_counter) *step_counter += 1;  // device step clock (graph-replay safe)
  }
}

}  // namespace psamd
