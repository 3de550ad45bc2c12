// XXH64 (the zstd frame content checksum, RFC 8878 3.1.1) for one wave: lanes 0-3 are the four
// accumulators over the 32-byte stripes, the tail runs uniform. Shared by the zstd decoder (checksum
// check) and encoder (checksum write).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace zgpu {
namespace xxh {

__device__ __forceinline__ uint32_t U(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t U64(uint64_t x) {
  return (uint64_t)U((uint32_t)x) | ((uint64_t)U((uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ int lane_id() { return __lane_id(); }

constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl64(acc, 31);
  return acc * P1;
}
__device__ __forceinline__ uint64_t ld64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= (uint64_t)__builtin_nontemporal_load(p + i) << (8 * i);
  return v;
}
__device__ inline uint64_t xxh64(const uint8_t *p, uint64_t len) {
  const int lane = lane_id();
  uint64_t h;
  uint64_t off = 0;
  if (len >= 32) {
    uint64_t v = lane == 0 ? P1 + P2 : lane == 1 ? P2 : lane == 2 ? 0 : 0 - P1;
    const uint64_t nst = len / 32;
    if (lane < 4)
      for (uint64_t s = 0; s < nst; s++) v = xround(v, ld64(p + s * 32 + lane * 8));
    auto rl = [&](int l) -> uint64_t {
      return (uint64_t)U(__builtin_amdgcn_readlane((uint32_t)v, l)) |
             ((uint64_t)U(__builtin_amdgcn_readlane((uint32_t)(v >> 32), l)) << 32);
    };
    const uint64_t v1 = rl(0), v2 = rl(1), v3 = rl(2), v4 = rl(3);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    const uint64_t vs[4] = {v1, v2, v3, v4};
    for (int k = 0; k < 4; k++) {
      h ^= xround(0, vs[k]);
      h = h * P1 + P4;
    }
    off = nst * 32;
  } else {
    h = P5;
  }
  h += len;
  while (off + 8 <= len) {
    h ^= xround(0, U64(ld64(p + off)));
    h = rotl64(h, 27) * P1 + P4;
    off += 8;
  }
  if (off + 4 <= len) {
    uint64_t w = 0;
    for (int i = 0; i < 4; i++) w |= (uint64_t)U(__builtin_nontemporal_load(p + off + i)) << (8 * i);
    h ^= w * P1;
    h = rotl64(h, 23) * P2 + P3;
    off += 4;
  }
  while (off < len) {
    h ^= (uint64_t)U(__builtin_nontemporal_load(p + off)) * P5;
    h = rotl64(h, 11) * P1;
    off++;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

}  // namespace xxh
using xxh::xxh64;
}  // namespace zgpu
