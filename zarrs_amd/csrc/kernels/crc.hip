// Checksums and shard-index resolution for gfx950.
//
//   crc32c stage   zarrs/src/array/codec/bytes_to_bytes/crc32c/crc32c_codec.rs:108-158
//                  (4-byte LE checksum at End/Start; verify only on the full-decode path and when
//                  validate_checksums; the partial path strips: strip_suffix_partial_decoder.rs:39-62)
//   shard index    zarrs/src/array/codec/array_to_bytes/sharding.rs:156-235 and
//                  sharding/sharding_codec.rs:1262-1298 (index chain bytes{endian}+crc32c, decoded
//                  and verified on both paths), :617-707 (empty entry = (u64::MAX, u64::MAX) -> fill;
//                  offset+size > shard length -> "out-of-bounds" error)
//
// Parallel CRC (crc.hpp): one workgroup per byte range, slice-by-4 segments merged by crc32_combine.
#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "crc.hpp"
#include "launch.hpp"

namespace zgpu {

__global__ __launch_bounds__(CRC_THREADS) void k_crc32c_strip(ZgItem *items, uint32_t *status, int at_start,
                                                              int verify) {
  __shared__ CrcTables T;
  __shared__ uint64_t s_len[CRC_THREADS / 64];
  __shared__ uint32_t s_crc[CRC_THREADS / 64];
  const uint32_t i = blockIdx.x;
  ZgItem it = items[i];
  if (status[i] || (it.flags & ZG_ITEM_FILL)) return;
  if (it.len < 4) {
    if (threadIdx.x == 0) status[i] = ZG_CRC_INPUT_TOO_SHORT;
    return;
  }
  const uint8_t *base = (const uint8_t *)it.src;
  const uint8_t *data = at_start ? base + 4 : base;
  const uint8_t *stored = at_start ? base : base + it.len - 4;
  const uint64_t n = it.len - 4;
  if (verify && !(it.flags & ZG_ITEM_PARTIAL)) {
    build_tables(T, POLY_CRC32C);
    const uint32_t c = wg_crc(data, n, T, POLY_CRC32C, s_len, s_crc);
    if (threadIdx.x == 0) {
      const uint32_t s = stored[0] | stored[1] << 8 | stored[2] << 16 | (uint32_t)stored[3] << 24;
      if (s != c) {
        status[i] = ZG_INVALID_CHECKSUM;
        return;
      }
    }
  }
  if (threadIdx.x == 0) {
    items[i].src = (uint64_t)data;
    items[i].len = n;
  }
}

// The trailing crc32c of C3's inner chain verified beside the one-wave k_gzip (which strips the 4 bytes
// itself, crc_tail 3) on a side stream: reads a snapshot of the items and statuses taken before the
// fork (k_gzip rewrites both), writes only bad[i]. k_crc32c_merge, after the join, makes a failed
// checksum the item's status whatever k_gzip reported (the chain decodes crc32c first,
// crc32c_codec.rs:108-141).
__global__ __launch_bounds__(CRC_THREADS) void k_crc32c_check(const ZgItem *items, const uint32_t *status,
                                                              uint32_t *bad) {
  __shared__ CrcTables T;
  __shared__ uint64_t s_len[CRC_THREADS / 64];
  __shared__ uint32_t s_crc[CRC_THREADS / 64];
  const uint32_t i = blockIdx.x;
  const ZgItem it = items[i];
  if (threadIdx.x == 0) bad[i] = 0;
  if (status[i] || (it.flags & (ZG_ITEM_FILL | ZG_ITEM_PARTIAL)) || it.len < 4) return;
  const uint8_t *data = (const uint8_t *)it.src;
  const uint8_t *stored = data + it.len - 4;
  build_tables(T, POLY_CRC32C);
  const uint32_t c = wg_crc(data, it.len - 4, T, POLY_CRC32C, s_len, s_crc);
  if (threadIdx.x == 0) {
    const uint32_t st = stored[0] | stored[1] << 8 | stored[2] << 16 | (uint32_t)stored[3] << 24;
    bad[i] = st != c;
  }
}

__global__ void k_crc32c_merge(uint32_t *status, const uint32_t *bad, uint32_t n) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && bad[i]) status[i] = ZG_INVALID_CHECKSUM;
}

hipError_t launch_crc32c_check(const ZgItem *items, const uint32_t *status, uint32_t *bad, uint32_t n_items,
                               hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_crc32c_check, dim3(n_items), dim3(CRC_THREADS), 0, s, items, status, bad);
  return hipGetLastError();
}

hipError_t launch_crc32c_merge(uint32_t *status, const uint32_t *bad, uint32_t n_items, hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_crc32c_merge, dim3((n_items + 255) / 256), dim3(256), 0, s, status, bad, n_items);
  return hipGetLastError();
}

hipError_t launch_crc32c_strip(ZgItem *items, uint32_t *status, uint32_t n_items, int at_start, int verify,
                               hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_crc32c_strip, dim3(n_items), dim3(CRC_THREADS), 0, s, items, status, at_start, verify);
  return hipGetLastError();
}

// ------------------------------- Adler-32 (zlib trailer) ---------------------------------------
// RFC 1950: s1 = 1 + sum b_j, s2 = sum of the running s1 = n + sum (n - j) b_j (mod 65521). Both sums
// are linear in the bytes, so the threads take coalesced 4-byte words in any order (byte j adds b to A
// and (n - j) b to B), reduce their residues every 4096 words, and the workgroup adds them.
__global__ __launch_bounds__(CRC_THREADS) void k_adler32_check(const ZgItem *items, uint32_t *status,
                                                               const uint32_t *kind, const uint2 *aux) {
  constexpr uint32_t M = 65521;
  __shared__ uint32_t s1s[CRC_THREADS], s2s[CRC_THREADS];
  const uint32_t i = blockIdx.x, t = threadIdx.x;
  if (kind[i] != BL_KIND_ZLIB || status[i] != 0) return;
  const ZgItem it = items[i];
  const uint8_t *p = (const uint8_t *)it.src;
  const uint64_t n = it.len;
  uint64_t A = 0, B = 0;
  uint32_t cnt = 0;
  for (uint64_t j0 = 4ull * t; j0 < n; j0 += 4ull * CRC_THREADS) {
    uint32_t w;
    if (j0 + 4 <= n) {
      __builtin_memcpy(&w, p + j0, 4);  // unaligned dword (gfx950 runs in unaligned mode)
    } else {
      w = 0;
      for (uint32_t k = 0; j0 + k < n; k++) w |= (uint32_t)p[j0 + k] << (8 * k);
    }
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {  // bytes past n are 0 and add nothing
      const uint32_t b = (w >> (8 * k)) & 0xffu;
      A += b;
      B += (n - j0 - k) * b;  // blosc streams are < 2^31 bytes
    }
    if (++cnt == 4096) {  // B < 4096 * 4 * 2^32 * 255 < 2^56 between reductions
      A %= M;
      B %= M;
      cnt = 0;
    }
  }
  s1s[t] = (uint32_t)(A % M);
  s2s[t] = (uint32_t)(B % M);
  __syncthreads();
  if (t == 0) {
    uint64_t s1 = 1, s2 = n % M;
    for (uint32_t k = 0; k < CRC_THREADS; k++) {
      s1 += s1s[k];
      s2 += s2s[k];
    }
    const uint32_t adler = (uint32_t)((s2 % M) << 16) | (uint32_t)(s1 % M);
    if (adler != aux[i].x) status[i] = ZG_CORRUPT_STREAM;
  }
}

hipError_t launch_adler32_check(const ZgItem *subs, uint32_t *sub_status, const uint32_t *sub_kind, uint32_t n_sub,
                                const uint2 *aux, hipStream_t s) {
  if (!n_sub) return hipSuccess;
  hipLaunchKernelGGL(k_adler32_check, dim3(n_sub), dim3(CRC_THREADS), 0, s, subs, sub_status, sub_kind, aux);
  return hipGetLastError();
}

// ------------------------------- shard index --------------------------------------------------
__global__ __launch_bounds__(CRC_THREADS) void k_shard_index(const ZgShard *shards, ZgIndexSpec spec,
                                                             uint64_t *index, uint32_t *shard_status, int keep_err) {
  __shared__ CrcTables T;
  __shared__ uint64_t s_len[CRC_THREADS / 64];
  __shared__ uint32_t s_crc[CRC_THREADS / 64];
  const uint32_t sh = blockIdx.x;
  if (keep_err && shard_status[sh]) return;
  const ZgShard S = shards[sh];
  uint64_t *dst = index + (uint64_t)sh * spec.n_inner * 2;
  if (S.ptr == 0) {  // missing shard: every inner chunk is empty (fill)
    for (uint64_t k = threadIdx.x; k < spec.n_inner * 2; k += blockDim.x) dst[k] = ~0ull;
    if (threadIdx.x == 0) shard_status[sh] = 0;
    return;
  }
  if (S.len < spec.index_bytes) {
    if (threadIdx.x == 0) shard_status[sh] = ZG_SHARD_TOO_SMALL;
    return;
  }
  const uint8_t *p = (const uint8_t *)S.ptr + (spec.at_start ? 0 : S.len - spec.index_bytes);
  uint64_t n = spec.index_bytes;
  if (spec.n_crc && spec.verify) build_tables(T, POLY_CRC32C);
  for (int k = (int)spec.n_crc - 1; k >= 0; k--) {  // b2b decode in reverse
    const uint8_t *data = spec.crc_at_start[k] ? p + 4 : p;
    const uint8_t *stored = spec.crc_at_start[k] ? p : p + n - 4;
    if (spec.verify) {
      const uint32_t c = wg_crc(data, n - 4, T, POLY_CRC32C, s_len, s_crc);
      const uint32_t sv = stored[0] | stored[1] << 8 | stored[2] << 16 | (uint32_t)stored[3] << 24;
      if (c != sv) {
        if (threadIdx.x == 0) shard_status[sh] = ZG_INVALID_CHECKSUM;
        return;
      }
    }
    p = data;
    n -= 4;
  }
  for (uint64_t k = threadIdx.x; k < spec.n_inner * 2; k += blockDim.x) {
    const uint8_t *q = p + k * 8;
    uint64_t v = 0;
    for (int b = 0; b < 8; b++) v |= (uint64_t)q[b] << (8 * (spec.big_endian ? 7 - b : b));
    dst[k] = v;
  }
  if (threadIdx.x == 0) shard_status[sh] = 0;
}

hipError_t launch_shard_index(const ZgShard *shards, uint32_t n_shards, const ZgIndexSpec &spec,
                              uint64_t *index, uint32_t *shard_status, int keep_err, hipStream_t s) {
  if (!n_shards) return hipSuccess;
  hipLaunchKernelGGL(k_shard_index, dim3(n_shards), dim3(CRC_THREADS), 0, s, shards, spec, index, shard_status,
                     keep_err);
  return hipGetLastError();
}

__global__ void k_mid_shards(const ZgItem *mids, const uint32_t *mid_status, uint32_t n, ZgShard *shards,
                             uint32_t *shard_status) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const ZgItem m = mids[i];
  const uint32_t st = mid_status[i];
  shard_status[i] = st;
  shards[i] = (st || (m.flags & ZG_ITEM_FILL)) ? ZgShard{0, 0} : ZgShard{m.src, m.len};
}

hipError_t launch_mid_shards(const ZgItem *mids, const uint32_t *mid_status, uint32_t n, ZgShard *shards,
                             uint32_t *shard_status, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_mid_shards, dim3((n + 255) / 256), dim3(256), 0, s, mids, mid_status, n, shards, shard_status);
  return hipGetLastError();
}

__global__ void k_item_resolve(ZgItem *items, uint32_t *status, uint32_t n_items, const ZgShard *shards,
                               const uint64_t *index, const uint32_t *shard_status, uint64_t n_inner,
                               unsigned long long *enc_bytes) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_items) return;
  ZgItem it = items[i];
  if (!(it.flags & ZG_ITEM_SHARDED)) return;
  const uint32_t ss = shard_status[it.shard];
  if (ss) {
    status[i] = ss;
    return;
  }
  const ZgShard S = shards[it.shard];
  const uint64_t off = index[((uint64_t)it.shard * n_inner + it.inner) * 2];
  const uint64_t size = index[((uint64_t)it.shard * n_inner + it.inner) * 2 + 1];
  if (off == ~0ull && size == ~0ull) {
    items[i].flags = it.flags | ZG_ITEM_FILL;
    return;
  }
  if (off > S.len || size > S.len - off) {
    status[i] = ZG_SHARD_INDEX_OOB;
    return;
  }
  items[i].src = S.ptr + off;
  items[i].len = size;
  atomicAdd(enc_bytes, (unsigned long long)size);
}

hipError_t launch_item_resolve(ZgItem *items, uint32_t *status, uint32_t n_items, const ZgShard *shards,
                               const uint64_t *index, const uint32_t *shard_status, uint64_t n_inner,
                               unsigned long long *enc_bytes, hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_item_resolve, dim3((n_items + 255) / 256), dim3(256), 0, s, items, status, n_items,
                     shards, index, shard_status, n_inner, enc_bytes);
  return hipGetLastError();
}


// ------------------------------- crc32c encode (write path) -----------------------------------
// CodecChain::encode of a crc32c codec (crc32c_codec.rs:88-106): checksum of the bytes so far,
// 4 bytes LE appended (End) or prepended (Start). Chunk c's bytes are dsts[c] + [lo, lo + len).
__global__ __launch_bounds__(CRC_THREADS) void k_crc32c_encode(const uint64_t *dsts, uint64_t lo, uint64_t len,
                                                               int at_start) {
  __shared__ CrcTables T;
  __shared__ uint64_t s_len[CRC_THREADS / 64];
  __shared__ uint32_t s_crc[CRC_THREADS / 64];
  if (!dsts[blockIdx.x]) return;  // a shard whose layout failed (variable-length encode)
  uint8_t *p = (uint8_t *)dsts[blockIdx.x] + lo;
  build_tables(T, POLY_CRC32C);
  const uint32_t c = wg_crc(p, len, T, POLY_CRC32C, s_len, s_crc);
  if (threadIdx.x < 4) {
    uint8_t *w = at_start ? p - 4 : p + len;
    w[threadIdx.x] = (uint8_t)(c >> (8 * threadIdx.x));
  }
}

hipError_t launch_crc32c_encode(const uint64_t *dsts, uint32_t n, uint64_t lo, uint64_t len, int at_start,
                                hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_crc32c_encode, dim3(n), dim3(CRC_THREADS), 0, s, dsts, lo, len, at_start);
  return hipGetLastError();
}

}  // namespace zgpu
