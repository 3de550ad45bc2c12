// Standalone numcodecs.shuffle decode (zarrs/src/array/codec/bytes_to_bytes/shuffle/shuffle_codec.rs:109-129)
// for chains where the shuffle does not sit directly above the bytes codec (otherwise it is fused
// into the scatter stage). dec[j*es + i] = enc[i*count + j]; length must divide by elementsize.
#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "launch.hpp"

namespace zgpu {

__global__ __launch_bounds__(256) void k_unshuffle(ZgItem *items, uint32_t *status, uint8_t *dst,
                                                   uint64_t slot_bytes, uint32_t es) {
  const uint32_t i = blockIdx.y;
  const ZgItem it = items[i];
  if (status[i] || (it.flags & ZG_ITEM_FILL)) return;
  if (it.len % es || it.len > slot_bytes) {
    if (blockIdx.x == 0 && threadIdx.x == 0) status[i] = it.len % es ? ZG_SHUFFLE_LENGTH : ZG_DECODED_SIZE_MISMATCH;
    return;
  }
  const uint64_t count = it.len / es;
  const uint8_t *src = (const uint8_t *)it.src;
  uint8_t *o = dst + (uint64_t)i * slot_bytes;
  // each thread produces whole elements so the writes are contiguous per lane
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < count;
       j += (uint64_t)gridDim.x * blockDim.x)
    for (uint32_t b = 0; b < es; b++) o[j * es + b] = src[(uint64_t)b * count + j];
}

__global__ void k_point_to_slots(ZgItem *items, const uint32_t *status, uint32_t n, uint8_t *dst,
                                 uint64_t slot_bytes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || status[i] || (items[i].flags & ZG_ITEM_FILL)) return;
  items[i].src = (uint64_t)(dst + (uint64_t)i * slot_bytes);
}

hipError_t launch_unshuffle(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                            uint32_t elementsize, hipStream_t s) {
  if (!n_items) return hipSuccess;
  const uint64_t want = (slot_bytes / elementsize + 255) / 256 + 1;
  const uint32_t gx = (uint32_t)(want < 64 ? want : 64);
  hipLaunchKernelGGL(k_unshuffle, dim3(gx, n_items), dim3(256), 0, s, items, status, dst, slot_bytes, elementsize);
  // lengths are unchanged; only the source pointer moves to the slot
  hipLaunchKernelGGL(k_point_to_slots, dim3((n_items + 255) / 256), dim3(256), 0, s, items, status, n_items, dst,
                     slot_bytes);
  return hipGetLastError();
}

}  // namespace zgpu
