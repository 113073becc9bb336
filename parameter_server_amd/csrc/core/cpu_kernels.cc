#include "cpu_kernels.h"

#include <algorithm>
#include <cmath>
#include <stdexcept>

namespace pscore {

uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

static uint64_t inv_mod64(uint64_t a) {
  uint64_t x = a;
  for (int i = 0; i < 6; ++i) x *= 2 - a * x;
  return x;
}

KeyMix make_keymix(int bits) {
  if (bits < 2 || bits > 64) throw std::invalid_argument("key bits must be in [2, 64]");
  KeyMix m;
  m.bits = bits;
  m.mask = bits == 64 ? ~0ull : ((1ull << bits) - 1);
  m.a = (0xbf58476d1ce4e5b9ull & m.mask) | 1;
  m.b = (0x94d049bb133111ebull & m.mask) | 1;
  m.ai = inv_mod64(m.a) & m.mask;
  m.bi = inv_mod64(m.b) & m.mask;
  m.s = (bits + 1) / 2;
  return m;
}

uint64_t mix_key(uint64_t x, const KeyMix& m) {
  x = (x * m.a) & m.mask;
  x ^= x >> m.s;
  x = (x * m.b) & m.mask;
  x ^= x >> m.s;
  return x;
}

uint64_t unmix_key(uint64_t x, const KeyMix& m) {
  x ^= x >> m.s;
  x = (x * m.bi) & m.mask;
  x ^= x >> m.s;
  x = (x * m.ai) & m.mask;
  return x;
}

uint64_t rng64(uint64_t seed, uint64_t idx) {
  uint64_t z = seed + 0x9e3779b97f4a7c15ull * (idx + 1);
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}

static float u01(uint64_t r) { return ((float)(r >> 40) + 1.0f) * (1.0f / 16777216.0f); }

float init_value(uint64_t key, int init_type, float v, float s, uint64_t seed) {
  switch (init_type) {
    case 1: return v;
    case 2: {
      float u1 = u01(rng64(seed, key * 2)), u2 = u01(rng64(seed, key * 2 + 1));
      return v + s * std::sqrt(-2.f * std::log(u1)) * std::cos(6.283185307f * u2);
    }
    case 3: return v + s * (2.f * u01(rng64(seed, key)) - 1.f);
    default: return 0.f;
  }
}

void kv_init(Slot* slots, int64_t cap) {
  for (int64_t i = 0; i < cap; ++i) {
    slots[i] = Slot{kEmptyKey, 0.f, 0.f, 0.f, 0.f, 0u, 0u};
  }
}

int64_t kv_resolve(Slot* slots, int64_t cap, const uint64_t* keys, int64_t n, int64_t* out_slot,
                   float* out_w, bool insert, int init_type, float init_v, float init_s,
                   uint64_t seed, bool* full, uint64_t home_base, uint64_t home_m) {
  const uint64_t mask = (uint64_t)cap - 1;
  int lg = 0;
  while ((1ll << lg) < cap) ++lg;
  int64_t inserted = 0;
  for (int64_t i = 0; i < n; ++i) {
    const uint64_t h = keys[i];
    // home slot: hashed, or ordered for a shard's key range (kv_table.hip home_slot)
    uint64_t idx = (home_m ? ((h - home_base) * home_m) >> (64 - lg) : fmix64(h)) & mask;
    int64_t found = -1;
    for (uint64_t p = 0; p <= mask; ++p) {
      Slot& s = slots[idx];
      if (s.key == h) { found = (int64_t)idx; break; }
      if (s.key == kEmptyKey) {
        if (!insert) break;
        s.key = h;
        if (init_type != 0) s.w = init_value(h, init_type, init_v, init_s, seed);
        ++inserted;
        found = (int64_t)idx;
        break;
      }
      idx = (idx + 1) & mask;
    }
    if (found < 0 && insert && full) *full = true;
    out_slot[i] = found;
    if (out_w) out_w[i] = found >= 0 ? slots[found].w : 0.f;
  }
  return inserted;
}

void kv_gather(const Slot* slots, const int64_t* idx, int64_t n, float* out, int field) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = idx[i];
    out[i] = s >= 0 ? (&slots[s].w)[field] : 0.f;
  }
}

void kv_set(Slot* slots, const int64_t* idx, int64_t n, const float* w, const float* z,
            const float* nn) {
  for (int64_t i = 0; i < n; ++i) {
    const int64_t s = idx[i];
    if (s < 0) continue;
    if (w) slots[s].w = w[i];
    if (z) slots[s].z = z[i];
    if (nn) slots[s].n = nn[i];
  }
}

static float prox(float zz, float eta, float l1, float l2) {
  const float leta = l1 * eta;
  if (zz <= leta && zz >= -leta) return 0.f;
  return (zz > 0.f ? zz - leta : zz + leta) / (1.f + l2 * eta);
}

void kv_update(Slot* slots, const int64_t* idx, const float* grad, int64_t n,
               const UpdateParams& p, double* stats) {
  double dnnz = 0, wsum = 0, dsum = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t si = idx[i];
    if (si < 0) continue;
    const float g = grad[i] * p.grad_scale;
    if (g != g) continue;
    Slot& s = slots[si];
    const float w_old = s.w;
    float w_new;
    if (p.algo == 2) {
      const float n_new = std::sqrt(s.n * s.n + g * g);
      const float sigma = (n_new - s.n) / p.alpha;
      s.z += g - sigma * w_old;
      s.n = n_new;
      const float eta = p.lr_type == 1 ? p.alpha : p.alpha / (n_new + p.beta);
      w_new = prox(-s.z * eta, eta, p.l1, p.l2);
    } else if (p.algo == 1) {
      s.n += g * g;
      const float eta = p.alpha / (p.beta + std::sqrt(s.n));
      w_new = prox(w_old - eta * g, eta, p.l1, p.l2);
    } else {
      s.cnt += 1;
      const float eta = p.lr_type == 1 ? p.alpha : p.alpha / (p.beta + std::sqrt((float)s.cnt));
      w_new = prox(w_old - eta * g, eta, p.l1, p.l2);
    }
    if (p.max_delta > 0.f) {
      const float d = w_new - w_old;
      if (d > p.max_delta) w_new = w_old + p.max_delta;
      if (d < -p.max_delta) w_new = w_old - p.max_delta;
    }
    s.w = w_new;
    dnnz += (double)((w_new != 0.f) - (w_old != 0.f));
    wsum += (double)w_new * w_new;
    const double d = (double)w_new - w_old;
    dsum += d * d;
  }
  if (stats) {
    stats[0] += dnnz;
    stats[1] += wsum;
    stats[2] += dsum;
  }
}

void kv_census(const Slot* slots, int64_t cap, int64_t* occ, int64_t* nnz) {
  int64_t o = 0, z = 0;
  for (int64_t i = 0; i < cap; ++i) {
    if (slots[i].key != kEmptyKey) {
      ++o;
      z += slots[i].w != 0.f;
    }
  }
  *occ = o;
  *nnz = z;
}

uint32_t sketch_hash(uint64_t key) {
  const uint32_t seed = 0xbc9f1d34u, m = 0xc6a4a793u;
  uint32_t h = seed ^ (8u * m);
  h += (uint32_t)key; h *= m; h ^= h >> 16;
  h += (uint32_t)(key >> 32); h *= m; h ^= h >> 16;
  return h;
}

void cm_insert(uint8_t* cells, uint64_t n_cells, int k, uint32_t vmax, const uint64_t* keys,
               const uint8_t* counts, int64_t n) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t h = sketch_hash(keys[i]);
    const uint32_t delta = (h >> 17) | (h << 15);
    const uint32_t c = counts ? counts[i] : 1u;
    for (int j = 0; j < k; ++j) {
      uint8_t& v = cells[h % n_cells];
      v = (uint8_t)(c > vmax - v ? vmax : v + c);
      h += delta;
    }
  }
}

void cm_query(const uint8_t* cells, uint64_t n_cells, int k, uint32_t vmax, const uint64_t* keys,
              int64_t n, int freq, int32_t* keep, uint8_t* out_count) {
  for (int64_t i = 0; i < n; ++i) {
    uint32_t h = sketch_hash(keys[i]);
    const uint32_t delta = (h >> 17) | (h << 15);
    uint32_t res = vmax;
    for (int j = 0; j < k; ++j) {
      res = std::min<uint32_t>(res, cells[h % n_cells]);
      h += delta;
    }
    if (keep) keep[i] = (int)res > freq;
    if (out_count) out_count[i] = (uint8_t)res;
  }
}

}  // namespace pscore
