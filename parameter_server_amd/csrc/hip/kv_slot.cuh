// KV slot layout and the per-key device primitives shared by the table kernels
// (kv_table.hip) and the one-sided peer exchange (p2p.hip): probe / insert with
// ordered or hashed home slots, and the optimizer update of one slot.
#pragma once
#include "common.cuh"

namespace psamd {

struct alignas(32) Slot {
  uint64_t key;
  float w, z, n, acc;
  uint32_t cnt, flags;
};
static_assert(sizeof(Slot) == 32, "slot must be 32 bytes");

enum InitType : int { kInitZero = 0, kInitConstant = 1, kInitGaussian = 2, kInitUniform = 3 };
enum Algo : int { kSGD = 0, kAdaGrad = 1, kFTRL = 2 };
enum LrType : int { kLrConstant = 1, kLrDecay = 2 };

struct UpdateParams {
  int algo;
  int lr_type;
  float alpha, beta;
  float l1, l2;
  float grad_scale;  // multiply incoming gradient (e.g. 1/minibatch)
  float max_delta;   // optional clip of |w_new - w_old| (<=0: off)
};

__device__ __forceinline__ float init_value(uint64_t key, int init_type, float v, float s,
                                            uint64_t seed) {
  switch (init_type) {
    case kInitConstant: return v;
    case kInitGaussian: {
      uint64_t r1 = rng64(seed, key * 2), r2 = rng64(seed, key * 2 + 1);
      float u1 = u01(r1), u2 = u01(r2);
      return v + s * sqrtf(-2.f * logf(u1)) * cosf(6.283185307f * u2);
    }
    case kInitUniform: return v + s * (2.f * u01(rng64(seed, key)) - 1.f);
    default: return 0.f;
  }
}

// Home slot: hashed (fmix64) for arbitrary keys, or ORDERED for a shard that owns
// the mixed-key range [base, base + span): home = ((key - base) * m) >> (64 - log2 cap)
// with m = floor((2^64 - 1) / span). Mixed keys are uniform, so the ordered map is as
// balanced as hashing, and a localiser's sorted unique keys then visit the table in
// increasing address order (TLB- and DRAM-page-friendly on a 64 GB table).
__device__ __forceinline__ uint64_t home_slot(uint64_t h, uint64_t mask, uint64_t base,
                                              uint64_t m, int shr) {
  return m ? ((h - base) * m) >> shr : (fmix64(h) & mask);
}

// Partition of a key in an ordered-home shard: the top lgP bits of its home
// position, so partitions are contiguous, equally wide key ranges and a sorted
// key list splits into P consecutive runs (owner push apply, kv_apply_part).
__device__ __forceinline__ int key_part(uint64_t h, uint64_t base, uint64_t m, int lgP) {
  if (lgP == 0) return 0;
  return (int)(((h - base) * m) >> (64 - lgP));
}

// flags bit 1: the slot's non-zero initial weight is published. An inserter claims the
// slot by CAS on the key and only then writes the weight, so a reader that finds the key
// (another lane of the launch, or a peer's one-sided lookup over xGMI, p2p.hip) may run
// ahead of that store: it takes the weight only once the flag is set (release / acquire
// at system scope) and otherwise the init value itself, which is what the inserter
// writes. Zero init needs no flag (the slot's weight starts at 0). (Bit 0: the
// aggregated push's "touched" mark, kv_table.hip.)
constexpr uint32_t kSlotInit = 2u;

__device__ __forceinline__ float published_w(Slot* s, uint64_t h, int init_type, float init_v,
                                             float init_s, uint64_t seed) {
  if (init_type == kInitZero) return s->w;
  const uint32_t f = __hip_atomic_load(&s->flags, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
  return (f & kSlotInit) ? s->w : init_value(h, init_type, init_v, init_s, seed);
}

__device__ __forceinline__ void publish_init(Slot* s, float w) {
  s->w = w;
  __hip_atomic_fetch_or(&s->flags, kSlotInit, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// Probe for one key; insert it if asked. Returns the slot index (-1: absent or
// table full) and the weight through *w.
__device__ __forceinline__ int64_t resolve_key(Slot* __restrict__ slots, uint64_t mask,
                                               uint64_t home_base, uint64_t home_m, int home_shr,
                                               uint64_t h, int insert, int init_type,
                                               float init_v, float init_s, uint64_t seed,
                                               float* w, int* ins) {
  uint64_t idx = home_slot(h, mask, home_base, home_m, home_shr) & mask;
  *w = 0.f;
  for (uint64_t probe = 0; probe <= mask; ++probe) {
    uint64_t k = slots[idx].key;
    if (k == h) {
      *w = published_w(&slots[idx], h, init_type, init_v, init_s, seed);
      return (int64_t)idx;
    }
    if (k == kEmptyKey) {
      if (!insert) return -1;
      unsigned long long prev = atomicCAS((unsigned long long*)&slots[idx].key,
                                          (unsigned long long)kEmptyKey, (unsigned long long)h);
      if (prev == kEmptyKey) {
        if (init_type != kInitZero) {
          *w = init_value(h, init_type, init_v, init_s, seed);
          publish_init(&slots[idx], *w);
        }
        ++*ins;
        return (int64_t)idx;
      }
      if (prev == h) {
        *w = published_w(&slots[idx], h, init_type, init_v, init_s, seed);
        return (int64_t)idx;
      }
    }
    idx = (idx + 1) & mask;
  }
  return -1;
}

__device__ __forceinline__ float soft_threshold_prox(float zz, float eta, float l1, float l2) {
  // argmin_w 1/(2 eta) (w - zz)^2 + l1 |w| + l2/2 ... (reference ElasticNet::proximal,
  // src/app/linear_method/penalty.h:38-43): shrink by l1*eta, scale by 1/(1+l2*eta).
  const float leta = l1 * eta;
  if (zz <= leta && zz >= -leta) return 0.f;
  return (zz > 0.f ? zz - leta : zz + leta) / (1.f + l2 * eta);
}

__device__ __forceinline__ float apply_update(Slot& s, float g, const UpdateParams& p) {
  const float w_old = s.w;
  float w_new;
  if (p.algo == kFTRL) {
    // FTRL-proximal (reference FTRLEntry::get, async_sgd.h:107-119).
    const float n_new = sqrtf(s.n * s.n + g * g);
    const float sigma = (n_new - s.n) / p.alpha;
    s.z += g - sigma * w_old;
    s.n = n_new;
    const float eta = p.lr_type == kLrConstant ? p.alpha : p.alpha / (n_new + p.beta);
    w_new = soft_threshold_prox(-s.z * eta, eta, p.l1, p.l2);
  } else if (p.algo == kAdaGrad) {
    // Proximal AdaGrad (the reference leaves this as a TODO, async_sgd.h:73-79).
    s.n += g * g;
    const float eta = p.alpha / (p.beta + sqrtf(s.n));
    w_new = soft_threshold_prox(w_old - eta * g, eta, p.l1, p.l2);
  } else {
    // Proximal SGD with per-key step count (reference stub: async_sgd.h:89-94).
    s.cnt += 1;
    const float eta = p.lr_type == kLrConstant ? p.alpha
                                                : p.alpha / (p.beta + sqrtf((float)s.cnt));
    w_new = soft_threshold_prox(w_old - eta * g, eta, p.l1, p.l2);
  }
  if (p.max_delta > 0.f) {
    const float d = w_new - w_old;
    if (d > p.max_delta) w_new = w_old + p.max_delta;
    if (d < -p.max_delta) w_new = w_old - p.max_delta;
  }
  s.w = w_new;
  return w_old;
}

}  // namespace psamd
