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
// Parallel CRC: one workgroup per byte range. Each thread checksums a contiguous segment with
// slice-by-4 tables held in LDS; the 256 partial CRCs are merged with the GF(2) shift operator
// crc(A||B) = crc(A) * x^(8|B|) mod P  xor  crc(B) (the zlib crc32_combine identity), using a
// table of x^(2^k) mod P, in a log2(256)-deep shuffle/LDS tree.
#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "launch.hpp"

namespace zgpu {

constexpr uint32_t POLY_CRC32C = 0x82F63B78u;  // reflected Castagnoli (crc32c crate)
constexpr uint32_t POLY_CRC32 = 0xEDB88320u;   // reflected IEEE (gzip trailer, RFC 1952)
constexpr int CRC_THREADS = 256;

struct CrcTables {
  uint32_t t[4][256];  // slice-by-4
  uint32_t x2n[32];    // x^(2^k) mod P
};

__device__ __forceinline__ uint32_t multmodp(uint32_t a, uint32_t b, uint32_t poly) {
  uint32_t m = 1u << 31, p = 0;
  for (;;) {
    if (a & m) {
      p ^= b;
      if ((a & (m - 1)) == 0) break;
    }
    m >>= 1;
    b = (b & 1) ? (b >> 1) ^ poly : b >> 1;
  }
  return p;
}

// x^(8*len) mod P
__device__ __forceinline__ uint32_t x8nmodp(uint64_t len, const uint32_t *x2n, uint32_t poly) {
  uint32_t p = 1u << 31;
  uint32_t k = 3;
  while (len) {
    if (len & 1) p = multmodp(x2n[k & 31], p, poly);
    len >>= 1;
    k++;
  }
  return p;
}

__device__ __forceinline__ uint32_t crc_combine(uint32_t c1, uint32_t c2, uint64_t len2, const uint32_t *x2n,
                                                uint32_t poly) {
  if (len2 == 0) return c1;
  return multmodp(x8nmodp(len2, x2n, poly), c1, poly) ^ c2;
}

__device__ void build_tables(CrcTables &T, uint32_t poly) {
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
    T.t[0][i] = c;
  }
  __syncthreads();
  for (uint32_t i = threadIdx.x; i < 256; i += blockDim.x) {
    uint32_t c = T.t[0][i];
    for (int s = 1; s < 4; s++) {
      c = (c >> 8) ^ T.t[0][c & 0xff];
      T.t[s][i] = c;
    }
  }
  if (threadIdx.x == 0) {
    uint32_t p = 1u << 30;  // x^1
    T.x2n[0] = p;
    for (int n = 1; n < 32; n++) T.x2n[n] = p = multmodp(p, p, poly);
  }
  __syncthreads();
}

// Standard CRC (init/xorout 0xFFFFFFFF) of a short segment.
__device__ __forceinline__ uint32_t crc_segment(const uint8_t *p, uint64_t n, const CrcTables &T) {
  uint32_t c = 0xFFFFFFFFu;
  while (n && ((uintptr_t)p & 3)) {
    c = (c >> 8) ^ T.t[0][(c ^ *p++) & 0xff];
    n--;
  }
  while (n >= 16) {
    const uint4 v = *(const uint4 *)p;
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t x = c ^ w[k];
      c = T.t[3][x & 0xff] ^ T.t[2][(x >> 8) & 0xff] ^ T.t[1][(x >> 16) & 0xff] ^ T.t[0][x >> 24];
    }
    p += 16;
    n -= 16;
  }
  while (n >= 4) {
    const uint32_t x = c ^ *(const uint32_t *)p;
    c = T.t[3][x & 0xff] ^ T.t[2][(x >> 8) & 0xff] ^ T.t[1][(x >> 16) & 0xff] ^ T.t[0][x >> 24];
    p += 4;
    n -= 4;
  }
  while (n--) c = (c >> 8) ^ T.t[0][(c ^ *p++) & 0xff];
  return ~c;
}

// Workgroup-wide CRC of p[0..n): every thread returns the same value.
__device__ uint32_t wg_crc(const uint8_t *p, uint64_t n, const CrcTables &T, uint32_t poly, uint64_t *s_len,
                           uint32_t *s_crc) {
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  // segments aligned to 16 bytes so the inner loop runs on 16-B loads
  uint64_t seg = (n + nt - 1) / nt;
  seg = (seg + 15) & ~(uint64_t)15;
  const uint64_t b0 = min<uint64_t>((uint64_t)tid * seg, n), b1 = min<uint64_t>(b0 + seg, n);
  uint32_t c = crc_segment(p + b0, b1 - b0, T);
  uint64_t l = b1 - b0;
  // tree merge: lane pairs within the wave, then waves through LDS
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t c2 = __shfl_down(c, off, 64);
    const uint64_t l2 = __shfl_down(l, off, 64);
    if ((tid & 63) % (2 * off) == 0 && (tid & 63) + off < 64) {
      c = crc_combine(c, c2, l2, T.x2n, poly);
      l += l2;
    }
  }
  const uint32_t nw = nt / 64;
  if ((tid & 63) == 0) {
    s_crc[tid / 64] = c;
    s_len[tid / 64] = l;
  }
  __syncthreads();
  if (tid == 0) {
    uint32_t acc = s_crc[0];
    for (uint32_t w = 1; w < nw; w++) acc = crc_combine(acc, s_crc[w], s_len[w], T.x2n, poly);
    s_crc[0] = acc;
  }
  __syncthreads();
  const uint32_t r = s_crc[0];
  __syncthreads();
  return r;
}

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

hipError_t launch_crc32c_strip(ZgItem *items, uint32_t *status, uint32_t n_items, int at_start, int verify,
                               hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_crc32c_strip, dim3(n_items), dim3(CRC_THREADS), 0, s, items, status, at_start, verify);
  return hipGetLastError();
}

// ------------------------------- gzip trailer check ------------------------------------------
// aux[i] = {crc32 from the trailer, ISIZE from the trailer}
__global__ __launch_bounds__(CRC_THREADS) void k_crc32_check(const ZgItem *items, uint32_t *status,
                                                             const uint2 *aux) {
  __shared__ CrcTables T;
  __shared__ uint64_t s_len[CRC_THREADS / 64];
  __shared__ uint32_t s_crc[CRC_THREADS / 64];
  const uint32_t i = blockIdx.x;
  const ZgItem it = items[i];
  if (status[i] || (it.flags & ZG_ITEM_FILL)) return;
  build_tables(T, POLY_CRC32);
  const uint32_t c = wg_crc((const uint8_t *)it.src, it.len, T, POLY_CRC32, s_len, s_crc);
  if (threadIdx.x == 0) {
    const uint2 a = aux[i];
    if (a.x != c || a.y != (uint32_t)it.len) status[i] = ZG_CORRUPT_STREAM;
  }
}

hipError_t launch_crc32_check(const ZgItem *items, uint32_t *status, uint32_t n_items, const uint2 *aux,
                              hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_crc32_check, dim3(n_items), dim3(CRC_THREADS), 0, s, items, status, aux);
  return hipGetLastError();
}

// ------------------------------- Adler-32 (zlib trailer) ---------------------------------------
// RFC 1950: s1 = 1 + sum b_j, s2 = sum of the running s1 = n + sum (n - j) b_j (mod 65521). Each
// thread runs the serial recurrence over one contiguous segment [a, e) (A = sum b, B = sum (e - j) b),
// reducing every NMAX bytes as zlib does; segments combine as s1 += A, s2 += B + (n - e) A.
__global__ __launch_bounds__(CRC_THREADS) void k_adler32_check(const ZgItem *items, uint32_t *status,
                                                               const uint32_t *kind, const uint2 *aux) {
  constexpr uint32_t M = 65521, NMAX = 5552;
  __shared__ uint32_t s1s[CRC_THREADS], s2s[CRC_THREADS];
  const uint32_t i = blockIdx.x, t = threadIdx.x;
  if (kind[i] != BL_KIND_ZLIB || status[i] != 0) return;
  const ZgItem it = items[i];
  const uint8_t *p = (const uint8_t *)it.src;
  const uint64_t n = it.len, L = (n + CRC_THREADS - 1) / CRC_THREADS;
  const uint64_t a = min<uint64_t>((uint64_t)t * L, n), e = min<uint64_t>(a + L, n);
  uint32_t A = 0, B = 0;
  for (uint64_t j = a; j < e;) {
    const uint64_t k = min<uint64_t>(e, j + NMAX);
    for (; j < k; j++) {
      A += p[j];
      B += A;
    }
    A %= M;
    B %= M;
  }
  s1s[t] = A;
  s2s[t] = (uint32_t)((B + (uint64_t)((n - e) % M) * A) % M);
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
                                                             uint64_t *index, uint32_t *shard_status) {
  __shared__ CrcTables T;
  __shared__ uint64_t s_len[CRC_THREADS / 64];
  __shared__ uint32_t s_crc[CRC_THREADS / 64];
  const uint32_t sh = blockIdx.x;
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
                              uint64_t *index, uint32_t *shard_status, hipStream_t s) {
  if (!n_shards) return hipSuccess;
  hipLaunchKernelGGL(k_shard_index, dim3(n_shards), dim3(CRC_THREADS), 0, s, shards, spec, index, shard_status);
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
