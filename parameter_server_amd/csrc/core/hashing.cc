#include "hashing.h"

#include <cstring>

namespace pscore {

namespace {
struct Crc32cTable {
  uint32_t t[8][256];
  Crc32cTable() {
    const uint32_t poly = 0x82F63B78u;  // reflected Castagnoli polynomial
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? (c >> 1) ^ poly : (c >> 1);
      t[0][i] = c;
    }
    for (int s = 1; s < 8; ++s)
      for (uint32_t i = 0; i < 256; ++i) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xff];
  }
};
const Crc32cTable& crc_table() {
  static const Crc32cTable tab;
  return tab;
}

inline uint32_t rotl32(uint32_t x, int r) { return (x << r) | (x >> (32 - r)); }
inline uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
inline uint32_t fmix32(uint32_t h) {
  h ^= h >> 16; h *= 0x85ebca6bu; h ^= h >> 13; h *= 0xc2b2ae35u; h ^= h >> 16;
  return h;
}
inline uint64_t fmix64(uint64_t k) {
  k ^= k >> 33; k *= 0xff51afd7ed558ccdull; k ^= k >> 33; k *= 0xc4ceb9fe1a85ec53ull; k ^= k >> 33;
  return k;
}
}  // namespace

// Slicing-by-8 table-driven CRC32C.
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n) {
  const auto& T = crc_table().t;
  const uint8_t* p = static_cast<const uint8_t*>(data);
  uint32_t c = ~crc;
  while (n >= 8) {
    uint64_t v;
    std::memcpy(&v, p, 8);
    const uint32_t lo = (uint32_t)v ^ c, hi = (uint32_t)(v >> 32);
    c = T[7][lo & 0xff] ^ T[6][(lo >> 8) & 0xff] ^ T[5][(lo >> 16) & 0xff] ^ T[4][lo >> 24] ^
        T[3][hi & 0xff] ^ T[2][(hi >> 8) & 0xff] ^ T[1][(hi >> 16) & 0xff] ^ T[0][hi >> 24];
    p += 8;
    n -= 8;
  }
  while (n--) c = (c >> 8) ^ T[0][(c ^ *p++) & 0xff];
  return ~c;
}

uint32_t murmur3_32(const void* key, size_t len, uint32_t seed) {
  const uint8_t* data = static_cast<const uint8_t*>(key);
  const size_t nblocks = len / 4;
  uint32_t h = seed;
  const uint32_t c1 = 0xcc9e2d51u, c2 = 0x1b873593u;
  for (size_t i = 0; i < nblocks; ++i) {
    uint32_t k;
    std::memcpy(&k, data + 4 * i, 4);
    k *= c1; k = rotl32(k, 15); k *= c2;
    h ^= k; h = rotl32(h, 13); h = h * 5 + 0xe6546b64u;
  }
  const uint8_t* tail = data + nblocks * 4;
  uint32_t k = 0;
  switch (len & 3) {
    case 3: k ^= (uint32_t)tail[2] << 16; [[fallthrough]];
    case 2: k ^= (uint32_t)tail[1] << 8; [[fallthrough]];
    case 1: k ^= tail[0]; k *= c1; k = rotl32(k, 15); k *= c2; h ^= k;
  }
  h ^= (uint32_t)len;
  return fmix32(h);
}

void murmur3_x64_128(const void* key, size_t len, uint32_t seed, uint64_t out[2]) {
  const uint8_t* data = static_cast<const uint8_t*>(key);
  const size_t nblocks = len / 16;
  uint64_t h1 = seed, h2 = seed;
  const uint64_t c1 = 0x87c37b91114253d5ull, c2 = 0x4cf5ad432745937full;
  for (size_t i = 0; i < nblocks; ++i) {
    uint64_t k1, k2;
    std::memcpy(&k1, data + 16 * i, 8);
    std::memcpy(&k2, data + 16 * i + 8, 8);
    k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
    h1 = rotl64(h1, 27); h1 += h2; h1 = h1 * 5 + 0x52dce729;
    k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
    h2 = rotl64(h2, 31); h2 += h1; h2 = h2 * 5 + 0x38495ab5;
  }
  const uint8_t* tail = data + nblocks * 16;
  uint64_t k1 = 0, k2 = 0;
  switch (len & 15) {
    case 15: k2 ^= (uint64_t)tail[14] << 48; [[fallthrough]];
    case 14: k2 ^= (uint64_t)tail[13] << 40; [[fallthrough]];
    case 13: k2 ^= (uint64_t)tail[12] << 32; [[fallthrough]];
    case 12: k2 ^= (uint64_t)tail[11] << 24; [[fallthrough]];
    case 11: k2 ^= (uint64_t)tail[10] << 16; [[fallthrough]];
    case 10: k2 ^= (uint64_t)tail[9] << 8; [[fallthrough]];
    case 9: k2 ^= (uint64_t)tail[8]; k2 *= c2; k2 = rotl64(k2, 33); k2 *= c1; h2 ^= k2;
      [[fallthrough]];
    case 8: k1 ^= (uint64_t)tail[7] << 56; [[fallthrough]];
    case 7: k1 ^= (uint64_t)tail[6] << 48; [[fallthrough]];
    case 6: k1 ^= (uint64_t)tail[5] << 40; [[fallthrough]];
    case 5: k1 ^= (uint64_t)tail[4] << 32; [[fallthrough]];
    case 4: k1 ^= (uint64_t)tail[3] << 24; [[fallthrough]];
    case 3: k1 ^= (uint64_t)tail[2] << 16; [[fallthrough]];
    case 2: k1 ^= (uint64_t)tail[1] << 8; [[fallthrough]];
    case 1: k1 ^= (uint64_t)tail[0]; k1 *= c1; k1 = rotl64(k1, 31); k1 *= c2; h1 ^= k1;
  }
  h1 ^= (uint64_t)len; h2 ^= (uint64_t)len;
  h1 += h2; h2 += h1;
  h1 = fmix64(h1); h2 = fmix64(h2);
  h1 += h2; h2 += h1;
  out[0] = h1;
  out[1] = h2;
}

}  // namespace pscore
