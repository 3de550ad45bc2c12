// Small device helpers shared by the gfx950 copy kernels (scatter.hip, encode.hip).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace zgpu {

// reverse each `comp`-byte component of a 32-bit word (bytes codec, non-native endianness)
__device__ __forceinline__ uint32_t swap_word(uint32_t x, uint32_t comp) {
  if (comp == 4) return __builtin_bswap32(x);
  if (comp == 2) return ((x >> 8) & 0x00FF00FFu) | ((x << 8) & 0xFF00FF00u);
  return x;
}

__device__ __forceinline__ uint4 swap_vec(uint4 v, uint32_t comp) {
  if (comp == 8) return make_uint4(__builtin_bswap32(v.y), __builtin_bswap32(v.x),
                                   __builtin_bswap32(v.w), __builtin_bswap32(v.z));
  return make_uint4(swap_word(v.x, comp), swap_word(v.y, comp), swap_word(v.z, comp),
                    swap_word(v.w, comp));
}

// 16-B non-temporal global load / store (streaming data touched once: no L2 retention)
typedef unsigned int zg_v4u __attribute__((ext_vector_type(4)));
__device__ __forceinline__ uint4 nt_load16(const void *p) {
  const zg_v4u x = __builtin_nontemporal_load((const zg_v4u *)p);
  return make_uint4(x.x, x.y, x.z, x.w);
}
__device__ __forceinline__ void nt_store16(void *p, uint4 v) {
  const zg_v4u x = {v.x, v.y, v.z, v.w};
  __builtin_nontemporal_store(x, (zg_v4u *)p);
}

}  // namespace zgpu
