// zstd frame decode (RFC 8878) — placeholder until the device decoder lands: marks items UNSUPPORTED.
#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "launch.hpp"

namespace zgpu {

__global__ void k_zstd_unsupported(const ZgItem *items, uint32_t *status, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !status[i] && !(items[i].flags & ZG_ITEM_FILL)) status[i] = ZG_UNSUPPORTED;
}

hipError_t launch_zstd(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                       hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_zstd_unsupported, dim3((n_items + 255) / 256), dim3(256), 0, s, items, status, n_items);
  return hipGetLastError();
}

}  // namespace zgpu
