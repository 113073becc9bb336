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

}  // namespace psamd
