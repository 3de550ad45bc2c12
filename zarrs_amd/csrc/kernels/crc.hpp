// CRC-32 / CRC-32C helpers shared by crc.hip and inflate.hip (the gzip trailer check runs at the
// end of k_gzip). Parallel CRC: each thread checksums a contiguous segment with slice-by-4 tables
// held in LDS; the partial CRCs are merged with the GF(2) shift operator
// crc(A||B) = crc(A) * x^(8|B|) mod P  xor  crc(B) (the zlib crc32_combine identity), using a table
// of x^(2^k) mod P, in a log2(threads)-deep shuffle/LDS tree.
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>

namespace zgpu {

constexpr uint32_t POLY_CRC32C = 0x82F63B78u;  // reflected Castagnoli (crc32c crate)
constexpr uint32_t POLY_CRC32 = 0xEDB88320u;   // reflected IEEE (gzip trailer, RFC 1952)
constexpr int CRC_THREADS = 256;

static __constant__ uint32_t c_x2n_crc32c[32] = {
    0x40000000u, 0x20000000u, 0x08000000u, 0x00800000u, 0x00008000u, 0x82F63B78u, 0x6EA2D55Cu, 0x18B8EA18u,
    0x510AC59Au, 0xB82BE955u, 0xB8FDB1E7u, 0x88E56F72u, 0x74C360A4u, 0xE4172B16u, 0x0D65762Au, 0x35D73A62u,
    0x28461564u, 0xBF455269u, 0xE2EA32DCu, 0xFE7740E6u, 0xF946610Bu, 0x3C204F8Fu, 0x538586E3u, 0x59726915u,
    0x734D5309u, 0xBC1AC763u, 0x7D0722CCu, 0xD289CABEu, 0xE94CA9BCu, 0x05B74F3Fu, 0xA51E1F42u, 0x40000000u};
static __constant__ uint32_t c_x2n_crc32[32] = {
    0x40000000u, 0x20000000u, 0x08000000u, 0x00800000u, 0x00008000u, 0xEDB88320u, 0xB1E6B092u, 0xA06A2517u,
    0xED627DAEu, 0x88D14467u, 0xD7BBFE6Au, 0xEC447F11u, 0x8E7EA170u, 0x6427800Eu, 0x4D47BAE0u, 0x09FE548Fu,
    0x83852D0Fu, 0x30362F1Au, 0x7B5A9CC3u, 0x31FEC169u, 0x9FEC022Au, 0x6C8DEDC4u, 0x15D6874Du, 0x5FDE7A4Eu,
    0xBAD90E37u, 0x2E4E5EEFu, 0x4EABA214u, 0xA8A472C0u, 0x429A969Eu, 0x148D302Au, 0xC40BA6D0u, 0xC4E22C3Cu};

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

__device__ inline void build_tables(CrcTables &T, uint32_t poly) {
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
  // x^(2^k) mod P: precomputed (zlib's x2n_table for the IEEE polynomial; the same recurrence,
  // p(0) = x^1, p(k+1) = p(k)^2 mod P, for Castagnoli) — thread 0 used to square 31 times per workgroup
  if (threadIdx.x < 32) T.x2n[threadIdx.x] = poly == POLY_CRC32C ? c_x2n_crc32c[threadIdx.x] : c_x2n_crc32[threadIdx.x];
  __syncthreads();
}

// The running (pre-inversion) CRC state c advanced over p[0..n): crc_segment = ~crc_run(~0, ...), and
// a segment split into pieces is one run over them.
__device__ __forceinline__ uint32_t crc_run(uint32_t c, const uint8_t *p, uint64_t n, const CrcTables &T) {
  while (n && ((uintptr_t)p & 3)) {
    c = (c >> 8) ^ T.t[0][(c ^ *p++) & 0xff];
    n--;
  }
  // 16-B vectors, the next two already in flight while one is folded in (a lane's segment is a
  // serial chain: without the prefetch every vector waits a full memory round trip)
  auto fold = [&](const uint4 v) {
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
    for (int k = 0; k < 4; k++) {
      const uint32_t x = c ^ w[k];
      c = T.t[3][x & 0xff] ^ T.t[2][(x >> 8) & 0xff] ^ T.t[1][(x >> 16) & 0xff] ^ T.t[0][x >> 24];
    }
  };
  if (n >= 16) {
    const uint64_t nv = n >> 4;
    uint4 v0 = *(const uint4 *)p, v1 = nv > 1 ? *(const uint4 *)(p + 16) : v0;
    for (uint64_t k = 0; k < nv; k++) {
      const uint4 v2 = k + 2 < nv ? *(const uint4 *)(p + 16 * (k + 2)) : v1;
      fold(v0);
      v0 = v1;
      v1 = v2;
    }
    p += 16 * nv;
    n -= 16 * nv;
  }
  while (n >= 4) {
    const uint32_t x = c ^ *(const uint32_t *)p;
    c = T.t[3][x & 0xff] ^ T.t[2][(x >> 8) & 0xff] ^ T.t[1][(x >> 16) & 0xff] ^ T.t[0][x >> 24];
    p += 4;
    n -= 4;
  }
  while (n--) c = (c >> 8) ^ T.t[0][(c ^ *p++) & 0xff];
  return c;
}

// Standard CRC (init/xorout 0xFFFFFFFF) of a short segment.
__device__ __forceinline__ uint32_t crc_segment(const uint8_t *p, uint64_t n, const CrcTables &T) {
  return ~crc_run(0xFFFFFFFFu, p, n, T);
}

// Workgroup-wide merge of each thread's CRC c of its contiguous segment of l bytes (segments in thread
// order): every thread returns the CRC of the concatenation.
__device__ inline uint32_t wg_crc_merge(uint32_t c, uint64_t l, const CrcTables &T, uint32_t poly, uint64_t *s_len,
                                        uint32_t *s_crc) {
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
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

// Workgroup-wide CRC of p[0..n): every thread returns the same value.
__device__ inline uint32_t wg_crc(const uint8_t *p, uint64_t n, const CrcTables &T, uint32_t poly, uint64_t *s_len,
                                  uint32_t *s_crc) {
  const uint32_t tid = threadIdx.x, nt = blockDim.x;
  // segments aligned to 16 bytes so the inner loop runs on 16-B loads
  uint64_t seg = (n + nt - 1) / nt;
  seg = (seg + 15) & ~(uint64_t)15;
  const uint64_t b0 = min<uint64_t>((uint64_t)tid * seg, n), b1 = min<uint64_t>(b0 + seg, n);
  return wg_crc_merge(crc_segment(p + b0, b1 - b0, T), b1 - b0, T, poly, s_len, s_crc);
}

}  // namespace zgpu
