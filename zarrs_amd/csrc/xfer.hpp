// Host <-> device transfers of the decode call (the PCIe-inclusive path).
//
// Encoded chunks that start in host memory reach HBM in one of two ways:
//  * pinned (page-locked / hipHostRegister'ed) buffers: DMA straight from the caller's memory --
//    the chunks are sorted by address and touching/overlapping ranges are merged, so chunks that sit
//    back to back in one buffer (a read shard, a packed batch) cost ONE hipMemcpyAsync;
//  * pageable buffers: copied by a pool of host threads into two pinned staging slabs, each slab's
//    H2D overlapping the fill of the other.
// Decoded output bound for host memory takes the same two routes in reverse.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <vector>

namespace zgpu {

struct HostRange {
  const uint8_t *src;  // host source
  uint64_t len;
  uint64_t dev_off;    // byte offset in the device staging buffer
};

// true if p lies in page-locked host memory the GPU can DMA from directly
bool host_is_pinned(const void *p);

// memcpy of many (dst, src, n) pieces on up to `threads` host threads
void parallel_memcpy(const std::vector<uint8_t *> &dst, const std::vector<const uint8_t *> &src,
                     const std::vector<uint64_t> &len, int threads);

// Copy host ranges into dev (at their dev_off) on stream s. pinned_ok: every range is in pinned
// memory (direct DMA); else staged through `stage` (2 slabs of slab_bytes pinned memory).
// Returns after all copies are enqueued AND the staging slabs are free again (synchronises s when
// staging was used).
hipError_t h2d_ranges(uint8_t *dev, const std::vector<HostRange> &ranges, bool pinned_ok, uint8_t *stage,
                      uint64_t slab_bytes, int threads, hipStream_t s);

// dst (host) <- src (device), n bytes: direct if dst is pinned, else staged. Synchronises s.
hipError_t d2h_bytes(uint8_t *dst, const uint8_t *src, uint64_t n, uint8_t *stage, uint64_t slab_bytes,
                     int threads, hipStream_t s);
// dst (device) <- src (host), n bytes, same policy. Synchronises s when staged.
hipError_t h2d_bytes(uint8_t *dst, const uint8_t *src, uint64_t n, uint8_t *stage, uint64_t slab_bytes,
                     int threads, hipStream_t s);

int host_copy_threads();

}  // namespace zgpu
