// Variable-length stages of the write path (chains with a compressor): per-item crc32c appended /
// prepended in place, the final copy of each encoded chunk into its caller-given destination, and
// the sharding_indexed layout over inner chunks of variable encoded length
// (ShardingCodecBound::encode_bounded, sharding_codec.rs:924-1085, SubchunkWriteOrder::C).
//
// Items ({src, len}, common.hpp) point into scratch slots whose layout leaves room around the
// bytes: crc32c codecs at the start move src back by 4 (headroom in front), at the end write past len.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../common.hpp"
#include "crc.hpp"
#include "launch.hpp"

namespace zgpu {

// crc32c (Crc32cCodec::encode, crc32c_codec.rs:88-98) of every item's bytes, one workgroup per item
__global__ __launch_bounds__(CRC_THREADS) void k_crc32c_items(ZgItem *items, const uint32_t *status, int at_start) {
  __shared__ CrcTables T;
  __shared__ uint64_t s_len[CRC_THREADS / 64];
  __shared__ uint32_t s_crc[CRC_THREADS / 64];
  const uint32_t i = blockIdx.x;
  if (status[i]) return;
  const ZgItem it = items[i];
  uint8_t *p = (uint8_t *)it.src;
  build_tables(T, POLY_CRC32C);
  const uint32_t c = wg_crc(p, it.len, T, POLY_CRC32C, s_len, s_crc);
  if (threadIdx.x < 4) {
    uint8_t *w = at_start ? p - 4 : p + it.len;
    w[threadIdx.x] = (uint8_t)(c >> (8 * threadIdx.x));
  }
  if (threadIdx.x == 0) {
    items[i].src = at_start ? it.src - 4 : it.src;
    items[i].len = it.len + 4;
  }
}

// every item's encoded bytes into dst[i] (capacity cap[i]); lens[i] = its length
__global__ __launch_bounds__(256) void k_encode_place(const ZgItem *items, uint32_t *status, const uint64_t *dst,
                                                      const uint64_t *cap, uint64_t *lens) {
  const uint32_t i = blockIdx.x;
  if (status[i]) return;
  const ZgItem it = items[i];
  if (it.len > cap[i]) {
    if (threadIdx.x == 0) status[i] = ZG_DECODED_SIZE_MISMATCH;
    return;
  }
  const uint8_t *s = (const uint8_t *)it.src;
  uint8_t *d = (uint8_t *)dst[i];
  if (threadIdx.x == 0) lens[i] = it.len;
  if (((uintptr_t)s & 3) == ((uintptr_t)d & 3)) {  // same alignment: bytes to the word boundary, then words
    const uint64_t head = std::min<uint64_t>(it.len, (4 - ((uintptr_t)s & 3)) & 3);
    if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
    const uint64_t nw = (it.len - head) / 4;
    const uint32_t *s4 = (const uint32_t *)(s + head);
    uint32_t *d4 = (uint32_t *)(d + head);
    for (uint64_t k = threadIdx.x; k < nw; k += 256) d4[k] = s4[k];
    for (uint64_t k = head + 4 * nw + threadIdx.x; k < it.len; k += 256) d[k] = s[k];
  } else {
    for (uint64_t k = threadIdx.x; k < it.len; k += 256) d[k] = s[k];
  }
}

// One workgroup per shard: C-order prefix sum of the present inner chunks' encoded lengths (an inner
// chunk equal to the fill value everywhere is omitted: nonfill 0), index entries (offset, nbytes)
// written raw (index bytes codec endianness) at the index position; the shard length and the position
// of its encoded index (for the index crc32c launches) returned. A failed inner chunk fails its shard.
__global__ __launch_bounds__(256) void k_shard_layout_var(const uint32_t *__restrict__ nonfill,
                                                          const ZgItem *__restrict__ items,
                                                          const uint32_t *__restrict__ item_status,
                                                          ZgShardLayoutArgs Lo, const uint64_t *__restrict__ shard_dst,
                                                          uint64_t *__restrict__ inner_off, uint64_t *__restrict__ index_ptr,
                                                          uint64_t *__restrict__ shard_len,
                                                          uint32_t *__restrict__ shard_status) {
  __shared__ uint64_t s_base, s_wsum[4];
  __shared__ uint32_t s_bad;
  const uint64_t sh = blockIdx.x, n = Lo.n_inner;
  const uint32_t *nf = nonfill + sh * n;
  uint64_t *off = inner_off + sh * n;
  const uint64_t body0 = Lo.at_start ? Lo.index_bytes : 0;
  if (threadIdx.x == 0) {
    s_base = 0;
    s_bad = 0;
  }
  __syncthreads();
  for (uint64_t k0 = 0; k0 < n; k0 += 256) {
    const uint64_t k = k0 + threadIdx.x;
    uint64_t f = 0;
    if (k < n && nf[k]) {
      if (item_status[sh * n + k]) atomicOr(&s_bad, 1u);
      f = items[sh * n + k].len;
    }
    uint64_t incl = f;
    const uint32_t lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t u = __shfl_up((unsigned long long)incl, o, 64);
      if ((int)lane >= o) incl += u;
    }
    if (lane == 63) s_wsum[threadIdx.x / 64] = incl;
    __syncthreads();
    uint64_t before = s_base;
    for (uint32_t w = 0; w < threadIdx.x / 64; w++) before += s_wsum[w];
    before += incl - f;
    if (k < n) off[k] = (k < n && nf[k]) ? body0 + before : ~0ull;
    __syncthreads();
    if (threadIdx.x == 0) s_base += s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
    __syncthreads();
  }
  const uint64_t body = s_base;
  const uint64_t idx0 = Lo.at_start ? 0 : body0 + body;  // encoded index position in the shard
  const uint64_t total = body0 + body + (Lo.at_start ? 0 : Lo.index_bytes);
  if (s_bad || total > Lo.E_pitch) {  // E_pitch: the destination capacity of a shard
    if (threadIdx.x == 0) {
      shard_status[sh] = s_bad ? 1u : ZG_DECODED_SIZE_MISMATCH;
      index_ptr[sh] = 0;
      shard_len[sh] = 0;
    }
    for (uint64_t k = threadIdx.x; k < n; k += 256) off[k] = ~0ull;
    return;
  }
  uint8_t *raw = (uint8_t *)shard_dst[sh] + idx0 + Lo.pre;
  for (uint64_t q = threadIdx.x; q < 2 * n; q += 256) {
    const uint64_t o = off[q / 2];
    const uint64_t v = o == ~0ull ? ~0ull : (q & 1 ? items[sh * n + q / 2].len : o);
#pragma unroll
    for (int b = 0; b < 8; b++) raw[q * 8 + b] = (uint8_t)(v >> (8 * (Lo.big_endian ? 7 - b : b)));
  }
  if (threadIdx.x == 0) {
    shard_status[sh] = 0;
    index_ptr[sh] = shard_dst[sh] + idx0;
    shard_len[sh] = total;
  }
}

// the present inner chunks from their slots to their shard offsets: a workgroup per inner chunk
__global__ __launch_bounds__(256) void k_shard_copy_var(const ZgItem *__restrict__ items, uint64_t n_inner,
                                                        const uint64_t *__restrict__ shard_dst,
                                                        const uint64_t *__restrict__ inner_off) {
  const uint64_t g = blockIdx.x, sh = g / n_inner;
  const uint64_t o = inner_off[g];
  if (o == ~0ull) return;
  const ZgItem it = items[g];
  const uint8_t *s = (const uint8_t *)it.src;
  uint8_t *d = (uint8_t *)shard_dst[sh] + o;
  if (((uintptr_t)s & 3) == ((uintptr_t)d & 3)) {
    const uint64_t head = std::min<uint64_t>(it.len, (4 - ((uintptr_t)s & 3)) & 3);
    if (threadIdx.x < head) d[threadIdx.x] = s[threadIdx.x];
    const uint64_t nw = (it.len - head) / 4;
    const uint32_t *s4 = (const uint32_t *)(s + head);
    uint32_t *d4 = (uint32_t *)(d + head);
    for (uint64_t k = threadIdx.x; k < nw; k += 256) d4[k] = s4[k];
    for (uint64_t k = head + 4 * nw + threadIdx.x; k < it.len; k += 256) d[k] = s[k];
  } else {
    for (uint64_t k = threadIdx.x; k < it.len; k += 256) d[k] = s[k];
  }
}

hipError_t launch_crc32c_items(ZgItem *items, const uint32_t *status, uint32_t n, int at_start, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_crc32c_items, dim3(n), dim3(CRC_THREADS), 0, s, items, status, at_start);
  return hipGetLastError();
}

hipError_t launch_encode_place(const ZgItem *items, uint32_t *status, const uint64_t *dst, const uint64_t *cap,
                               uint64_t *lens, uint32_t n, hipStream_t s) {
  if (!n) return hipSuccess;
  hipLaunchKernelGGL(k_encode_place, dim3(n), dim3(256), 0, s, items, status, dst, cap, lens);
  return hipGetLastError();
}

hipError_t launch_fill_check(const uint64_t *starts, const uint8_t *array, const ZgEncode &inner, uint32_t n_chunks,
                             uint32_t *nonfill, hipStream_t s);

hipError_t launch_shard_encode_var(const uint64_t *starts, const uint8_t *array, const ZgEncode &inner,
                                   uint32_t n_chunks, uint32_t *nonfill, const ZgItem *items,
                                   const uint32_t *item_status, const ZgShardLayoutArgs &A, const uint64_t *shard_dst,
                                   uint64_t *inner_off, uint64_t *index_ptr, uint64_t *shard_len,
                                   uint32_t *shard_status, uint32_t n_shards, hipStream_t s) {
  if (!n_chunks) return hipSuccess;
  hipError_t e = launch_fill_check(starts, array, inner, n_chunks, nonfill, s);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k_shard_layout_var, dim3(n_shards), dim3(256), 0, s, nonfill, items, item_status, A, shard_dst,
                     inner_off, index_ptr, shard_len, shard_status);
  hipLaunchKernelGGL(k_shard_copy_var, dim3(n_chunks), dim3(256), 0, s, items, A.n_inner, shard_dst, inner_off);
  return hipGetLastError();
}

}  // namespace zgpu
