// Multi-GPU array reads from ONE process over the C ABI (north_star: "a batch is
// partitioned across the 8 GPUs of one node ... only for the final gather when a requested array
// subset spans GPUs").
//
// Reference: zarrs decodes the chunks a subset touches in one rayon loop
// (zarrs/src/array/array_read_ops_common.rs:173-176); chunks are independent, so the loop is cut into
// one contiguous range per GPU here. The cut is along axis 0 of the chunk grid: each device's chunks
// cover a run of whole output rows, which is ONE contiguous byte range of the C-order output, so:
//   * host output: every device decodes its range (host-resident encoded chunks, uploaded over its
//     own PCIe link) and writes its rows straight into place — no gather at all;
//   * device output (on chains[0]'s device): device 0 decodes into place, the others decode into a
//     scratch slab in their own HBM and copy it peer-to-peer over xGMI (one copy per device, the only
//     exchange the path has).
// A multi-process deployment (one rank per GPU) does the same cut in zarrs_amd/distributed.py with an
// RCCL gather; this entry is what a single-process Rust caller binds.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zgpu.h"
#include "chain.hpp"
#include "internal.hpp"

using namespace zgpu;

namespace {

struct Part {
  uint64_t row0 = 0, rows = 0;  // output rows (axis 0 of the subset) of this device
  int rc = ZGPU_OK;
  std::string err;
};

}  // namespace

int zgpu_retrieve_array_subset_multi(zgpu_chain *const *chains, uint32_t n_dev, uint32_t nd,
                                     const uint64_t *array_shape, const uint64_t *chunk_shape,
                                     const void *const *chunk_ptrs, const uint64_t *chunk_lens,
                                     const uint64_t *sel_start, const uint64_t *sel_shape, void *out, uint32_t flags) {
  try {
    if (!chains || n_dev == 0 || !array_shape || !chunk_shape || !chunk_ptrs || !chunk_lens || !sel_start ||
        !sel_shape || !out)
      return set_last_error(ZGPU_INVALID_ARGUMENT, "NULL argument");
    if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_last_error(ZGPU_INVALID_ARGUMENT, "ndim out of range");
    if (flags & ZGPU_ENC_DEVICE)
      return set_last_error(ZGPU_INVALID_ARGUMENT, "multi-device reads take host-resident encoded chunks");
    for (uint32_t d = 0; d < n_dev; d++)
      if (!chains[d]) return set_last_error(ZGPU_INVALID_ARGUMENT, "NULL chain");
    const uint32_t es = chain_model(chains[0]).es;
    for (uint32_t d = 1; d < n_dev; d++)
      if (chain_model(chains[d]).es != es) return set_last_error(ZGPU_INVALID_ARGUMENT, "chains of different data types");
    for (uint32_t k = 0; k < nd; k++) {
      if (chunk_shape[k] == 0) return set_last_error(ZGPU_INVALID_ARGUMENT, "zero chunk extent");
      if (sel_start[k] + sel_shape[k] > array_shape[k])
        return set_last_error(ZGPU_INVALID_ARGUMENT, "subset out of the array bounds");
      if (sel_shape[k] == 0) return ZGPU_OK;
    }
    uint64_t row_elems = 1;
    for (uint32_t k = 1; k < nd; k++) row_elems *= sel_shape[k];
    const uint64_t row_bytes = row_elems * es;
    // chunk rows of the subset along axis 0, cut into n_dev contiguous groups
    const uint64_t c0 = sel_start[0] / chunk_shape[0];
    const uint64_t c1 = (sel_start[0] + sel_shape[0] - 1) / chunk_shape[0] + 1;
    const uint64_t ncr = c1 - c0;
    std::vector<Part> parts(n_dev);
    for (uint32_t d = 0; d < n_dev; d++) {
      const uint64_t a = c0 + ncr * d / n_dev, b = c0 + ncr * (d + 1) / n_dev;
      if (a == b) continue;
      const uint64_t r0 = std::max(sel_start[0], a * chunk_shape[0]);
      const uint64_t r1 = std::min(sel_start[0] + sel_shape[0], b * chunk_shape[0]);
      parts[d].row0 = r0 - sel_start[0];
      parts[d].rows = r1 - r0;
    }
    const bool dev_out = (flags & ZGPU_OUT_DEVICE) != 0;
    const int out_dev = ctx_device(chain_ctx(chains[0]));
    // runs on its own host thread per device: every failure (HIP, allocation, exceptions) is recorded
    // in the device's Part, never thrown across the thread boundary
    auto work = [&](uint32_t d) {
      Part &P = parts[d];
      if (!P.rows) return;
      zgpu_ctx *C = chain_ctx(chains[d]);
      void *scratch = nullptr;
      try {
        std::vector<uint64_t> s(sel_start, sel_start + nd), n(sel_shape, sel_shape + nd);
        s[0] = sel_start[0] + P.row0;
        n[0] = P.rows;
        uint8_t *dst = (uint8_t *)out + P.row0 * row_bytes;
        const int dev = ctx_device(C);
        if (dev_out && d != 0) {  // decode into a slab of this device's HBM, then one peer copy
          // a stream-ordered allocation on the context's copy stream (not the context's grow-only
          // pool: a large read would otherwise keep rows * row_bytes of every secondary device reserved
          // for the context's lifetime; not hipMalloc/hipFree either: hipFree synchronises the whole
          // device, stalling the other lanes' decodes there)
          hipError_t e = hipSetDevice(dev);
          hipStream_t cs = e == hipSuccess ? ctx_copy_stream(C) : nullptr;
          if (e == hipSuccess && !cs) e = hipErrorInvalidValue;
          if (e == hipSuccess) e = hipMallocAsync(&scratch, std::max<uint64_t>(P.rows * row_bytes, 1), cs);
          if (e == hipSuccess) e = hipStreamSynchronize(cs);  // the decode runs on another stream
          if (e != hipSuccess) {
            (void)hipGetLastError();
            scratch = nullptr;
            P.rc = ZGPU_HIP_ERROR;
            P.err = std::string("allocation of the device slab failed: ") + hipGetErrorString(e);
            return;
          }
          dst = (uint8_t *)scratch;
        }
        P.rc = zgpu_retrieve_array_subset(chains[d], nd, array_shape, chunk_shape, chunk_ptrs, chunk_lens, s.data(),
                                          n.data(), dst, flags, nullptr);
        if (P.rc) P.err = zgpu_last_error(nullptr);
        if (scratch && !P.rc) {
          hipError_t e = hipSetDevice(dev);
          // the direct xGMI path for the copy below; without peer access the runtime still copies
          // (staged), so a refusal is not an error
          if (e == hipSuccess && dev != out_dev && hipDeviceEnablePeerAccess(out_dev, 0) != hipSuccess)
            (void)hipGetLastError();
          hipStream_t st = e == hipSuccess ? ctx_copy_stream(C) : nullptr;
          if (e == hipSuccess && !st) e = hipErrorInvalidValue;
          if (e == hipSuccess)
            e = hipMemcpyPeerAsync((uint8_t *)out + P.row0 * row_bytes, out_dev, scratch, dev, P.rows * row_bytes, st);
          if (e == hipSuccess) e = hipStreamSynchronize(st);
          if (e != hipSuccess) {
            P.rc = ZGPU_HIP_ERROR;
            P.err = std::string("peer copy: ") + hipGetErrorString(e);
          }
        }
      } catch (const std::exception &e) {
        P.rc = ZGPU_HIP_ERROR;
        P.err = e.what();
      } catch (...) {
        P.rc = ZGPU_HIP_ERROR;
        P.err = "unknown exception";
      }
      if (scratch && hipSetDevice(ctx_device(C)) == hipSuccess) {
        // ordered after the peer copy (synchronised above). After a failure the decode may still have
        // kernels writing the slab on its lane stream: wait for the device before the pool reuses it
        if (P.rc) (void)hipDeviceSynchronize();
        hipStream_t cs = ctx_copy_stream(C);
        if (!cs || hipFreeAsync(scratch, cs) != hipSuccess) (void)hipGetLastError();
      }
    };
    std::vector<std::thread> threads;
    for (uint32_t d = 1; d < n_dev; d++)
      if (parts[d].rows) threads.emplace_back(work, d);
    work(0);
    for (std::thread &t : threads) t.join();
    for (uint32_t d = 0; d < n_dev; d++)  // zarrs' try_for_each: the first failure in chunk order
      if (parts[d].rc) return set_last_error(parts[d].rc, "device " + std::to_string(d) + ": " + parts[d].err);
    return ZGPU_OK;
  } catch (const std::exception &e) {
    return set_last_error(ZGPU_HIP_ERROR, e.what());
  }
}
