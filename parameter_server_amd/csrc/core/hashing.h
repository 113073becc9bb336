// crc32c (Castagnoli) and MurmurHash3 (x86_32, x64_128).
// Reference uses crc32c for KeyCaching signatures (src/filter/key_caching.h:43)
// and MurmurHash3 for the TERAFEA --shuffle_fea_id option (text_parser.cc:160-164).
#pragma once
#include <cstddef>
#include <cstdint>

namespace pscore {
uint32_t crc32c_extend(uint32_t crc, const void* data, size_t n);
inline uint32_t crc32c(const void* data, size_t n) { return crc32c_extend(0, data, n); }
uint32_t murmur3_32(const void* key, size_t len, uint32_t seed);
void murmur3_x64_128(const void* key, size_t len, uint32_t seed, uint64_t out[2]);
}  // namespace pscore
