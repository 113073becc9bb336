// CPU reference implementations of the device kernels.
//
// Same data layouts as the HIP kernels (32-byte KV slots, byte CountMin
// cells, mixed key space) so a table can be moved between host and device
// memory verbatim and the two paths can be checked against each other.
#pragma once
#include <cstddef>
#include <cstdint>

namespace pscore {

constexpr uint64_t kEmptyKey = ~0ull;

struct KeyMix {
  uint64_t mask, a, b, ai, bi;
  int s, bits;
};
KeyMix make_keymix(int bits);
uint64_t mix_key(uint64_t x, const KeyMix& m);
uint64_t unmix_key(uint64_t x, const KeyMix& m);
uint64_t fmix64(uint64_t k);

struct Slot {
  uint64_t key;
  float w, z, n, acc;
  uint32_t cnt, flags;
};
static_assert(sizeof(Slot) == 32, "slot must be 32 bytes");

struct UpdateParams {
  int algo;  // 0 sgd, 1 adagrad, 2 ftrl
  int lr_type;
  float alpha, beta, l1, l2, grad_scale, max_delta;
};

void kv_init(Slot* slots, int64_t cap);
// returns number of inserted keys; -1 in out_slot for missing / full
int64_t kv_resolve(Slot* slots, int64_t cap, const uint64_t* keys, int64_t n, int64_t* out_slot,
                   float* out_w, bool insert, int init_type, float init_v, float init_s,
                   uint64_t seed, bool* full, uint64_t home_base = 0, uint64_t home_m = 0);
void kv_gather(const Slot* slots, const int64_t* idx, int64_t n, float* out, int field);
void kv_set(Slot* slots, const int64_t* idx, int64_t n, const float* w, const float* z,
            const float* nn);
void kv_update(Slot* slots, const int64_t* idx, const float* grad, int64_t n,
               const UpdateParams& p, double* stats);
void kv_census(const Slot* slots, int64_t cap, int64_t* occ, int64_t* nnz);

uint32_t sketch_hash(uint64_t key);
void cm_insert(uint8_t* cells, uint64_t n_cells, int k, uint32_t vmax, const uint64_t* keys,
               const uint8_t* counts, int64_t n);
void cm_query(const uint8_t* cells, uint64_t n_cells, int k, uint32_t vmax, const uint64_t* keys,
              int64_t n, int freq, int32_t* keep, uint8_t* out_count);

float init_value(uint64_t key, int init_type, float v, float s, uint64_t seed);
uint64_t rng64(uint64_t seed, uint64_t idx);

}  // namespace pscore
