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

// A box [start, start+shape) of a C-order array (array_shape, elements of es bytes) as a sequence of
// contiguous byte runs in C order of the box: run k covers bytes [k*run_bytes, (k+1)*run_bytes) of
// the box's compact (C-order, shape) layout and lies at byte offset offset(k) of the array. Trailing
// axes the box spans whole are folded into the run (the array itself is one run).
struct BoxRuns {
  uint32_t outer = 0;                  // axes enumerated run by run
  uint64_t shape[8] = {0};             // their extents
  uint64_t stride[8] = {0};            // their array strides (bytes)
  uint64_t base = 0;                   // array byte offset of the box origin
  uint64_t run_bytes = 0, n_runs = 0;  // n_runs * run_bytes = box bytes
  uint64_t offset(uint64_t k) const;
};
BoxRuns box_runs(uint32_t nd, const uint64_t *array_shape, const uint64_t *start, const uint64_t *shape, uint32_t es);
bool box_is_whole(uint32_t nd, const uint64_t *array_shape, const uint64_t *start, const uint64_t *shape);

// Copy the bytes [lo, hi) of a box's compact layout between `compact` (holding those bytes at
// compact[0 .. hi-lo)) and the array at `array`: to_array = true scatters into the array, false
// gathers from it. Runs are split over up to `threads` host threads.
void copy_box_runs(const BoxRuns &R, uint8_t *array, uint8_t *compact, uint64_t lo, uint64_t hi, bool to_array,
                   int threads);

// host array box <- device compact box (D2H through the pinned slabs, rows placed by host threads),
// and the reverse; both synchronise s.
hipError_t d2h_box(const BoxRuns &R, uint8_t *host_array, const uint8_t *dev_compact, uint8_t *stage,
                   uint64_t slab_bytes, int threads, hipStream_t s);
hipError_t h2d_box(const BoxRuns &R, uint8_t *dev_compact, const uint8_t *host_array, uint8_t *stage,
                   uint64_t slab_bytes, int threads, hipStream_t s);

}  // namespace zgpu
