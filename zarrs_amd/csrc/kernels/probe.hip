// Decoded-size hints of whole-shard bytes->bytes stages (a compressor applied to a shard after
// sharding_indexed, codec_chain.rs:192-229 composes it like any other bytes->bytes codec): one thread
// per item reads what the encoded stream says about its decoded size, so the host can size the
// decode slots before the stage runs.
//   gzip : ISIZE of the trailer (RFC 1952 §2.3.1; mod 2^32, and only the last member's -- a hint,
//          the host retries an overflowing item with a larger slot)
//   zstd : ZSTD_decompressBound (zstd_codec.rs:118 takes Decompressor::upper_bound): per frame the
//          Frame_Content_Size when present, else the sum of its block bounds (raw / RLE: the block
//          size; compressed: min(window size, 128 KiB)); skippable frames count 0
//   blosc: nbytes of the blosc header (blosc_codec_via_blosc_src.rs reads it the same way)
#include <hip/hip_runtime.h>

#include "launch.hpp"

namespace zgpu {

namespace {

__device__ inline uint32_t rd_le(const uint8_t *p, int n) {
  uint32_t v = 0;
  for (int b = 0; b < n; b++) v |= (uint32_t)p[b] << (8 * b);
  return v;
}

__device__ uint64_t zstd_bound(const uint8_t *p, uint64_t len) {
  uint64_t pos = 0, total = 0;
  while (pos + 4 <= len) {
    const uint32_t magic = rd_le(p + pos, 4);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (pos + 8 > len) return 0;
      pos += 8 + (uint64_t)rd_le(p + pos + 4, 4);
      continue;
    }
    if (magic != 0xFD2FB528u || pos + 5 > len) return 0;
    const uint8_t fhd = p[pos + 4];
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, cksum = (fhd >> 2) & 1, did = fhd & 3;
    uint64_t q = pos + 5;
    uint64_t window = 0;
    if (!single) {
      if (q + 1 > len) return 0;
      const uint8_t wd = p[q++];
      const uint64_t base = 1ull << (10 + (wd >> 3));
      window = base + (base >> 3) * (wd & 7);
    }
    q += did == 0 ? 0 : did == 1 ? 1 : did == 2 ? 2 : 4;
    const uint32_t fcs_bytes = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
    if (q + fcs_bytes > len) return 0;
    bool have_fcs = fcs_bytes > 0;
    uint64_t fcs = 0;
    if (fcs_bytes == 8) fcs = rd_le(p + q, 4) | (uint64_t)rd_le(p + q + 4, 4) << 32;
    else if (fcs_bytes) fcs = rd_le(p + q, fcs_bytes) + (fcs_bytes == 2 ? 256 : 0);
    q += fcs_bytes;
    if (single) window = fcs;
    const uint64_t blk_max = window < (128u << 10) ? window : (128u << 10);
    uint64_t sum = 0;
    for (;;) {  // block headers
      if (q + 3 > len) return 0;
      const uint32_t bh = rd_le(p + q, 3);
      const uint32_t last = bh & 1, type = (bh >> 1) & 3, size = bh >> 3;
      q += 3;
      if (type == 0) { sum += size; q += size; }
      else if (type == 1) { sum += size; q += 1; }
      else if (type == 2) { sum += blk_max; q += size; }
      else return 0;
      if (last) break;
    }
    q += cksum ? 4 : 0;
    total += have_fcs ? fcs : sum;
    pos = q;
  }
  return total;
}

__global__ void k_size_hint(const ZgItem *items, const uint32_t *status, uint32_t n, uint32_t kind, uint64_t *hint) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ZgItem it = items[i];
  uint64_t h = 0;
  if (!status[i] && !(it.flags & ZG_ITEM_FILL) && it.src) {
    const uint8_t *p = (const uint8_t *)it.src;
    if (kind == SIZE_HINT_GZIP) h = it.len >= 18 ? rd_le(p + it.len - 4, 4) : 0;
    else if (kind == SIZE_HINT_ZSTD) h = zstd_bound(p, it.len);
    else if (kind == SIZE_HINT_BLOSC) h = it.len >= 16 ? rd_le(p + 4, 4) : 0;
  }
  hint[i] = h;
}

}  // namespace

hipError_t launch_size_hint(const ZgItem *items, const uint32_t *status, uint32_t n, uint32_t kind, uint64_t *hint,
                            hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_size_hint, dim3((n + 255) / 256), dim3(256), 0, s, items, status, n, kind, hint);
  return hipGetLastError();
}

}  // namespace zgpu
