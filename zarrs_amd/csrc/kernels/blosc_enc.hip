// blosc (c-blosc 1.x frame, format 2) ENCODER on gfx950: the write half of the blosc codec
// (BloscCodec::encode, zarrs/src/array/codec/bytes_to_bytes/blosc/blosc_codec_via_blosc_src.rs:113-128
// -> blosc_compress_bytes, blosc_via_blosc_src.rs:64-96 -> c-blosc's blosc_compress_ctx). The frames
// are read by any c-blosc 1.x decoder and by k_blosc_*; their bytes are not c-blosc's (block size,
// block splitting and the LZ parse are encoder choices the format leaves open).
//
//   k_blosc_shuf_enc   one workgroup per (item, block): byte shuffle (shuffle.c shuffle_generic) or
//                      bitshuffle (bshuf_trans_bit_elem; blocks whose element count is not a multiple
//                      of 8 stay as they are, format 2) of the block into the staging buffer
//   k_lz4_encode       one wave per stream: an LZ4 block, a blosclz or a snappy stream (greedy LZ77, 64
//                      positions a step, 4-byte hash candidates in LDS, 64 / 72 KiB window; the last 5
//                      bytes literals and no match starting in the last 12, as the LZ4 block format
//                      requires and blosclz's decoder needs: it must end on a literal run), emitted
//                      only when smaller than the stream
//   zstd streams       k_zstd_encode_seg + k_zstd_frame over the stream table (zstd_enc.hip)
//   zlib streams       k_gzip_encode in its zlib mode over the stream table (deflate_enc.hip)
//   k_blosc_layout_enc one thread per item: every stream's offset in the frame (stored streams
//                      where compression did not help), a memcpyed frame when nothing is gained
//   k_blosc_write_enc  one workgroup per stream: its {csize, payload} (the header and a block's
//                      bstarts entry by the first streams)
#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "launch.hpp"

namespace zgpu {
namespace {

constexpr uint32_t LZ4E_HBITS = 12, LZ4E_HSIZE = 1u << LZ4E_HBITS;
constexpr uint32_t LZ4E_CAP1 = 32;        // per-lane match search; longer chosen matches: the wave
constexpr uint32_t LZ4E_MAXOFF = 65535;   // 2-byte offsets
constexpr uint32_t BLZ_MAXOFF = 8191 + 65536;  // blosclz: 13-bit near distances, 16-bit far ones above 8191
constexpr uint32_t LZ4E_LAST = 5;         // LASTLITERALS
constexpr uint32_t LZ4E_MFLIMIT = 12;     // no match starts in the last 12 bytes

__device__ __forceinline__ uint32_t ld4u(const uint8_t *p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t lo = w[0];
  const uint32_t hi = sh ? w[1] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

// ZstdCodec::encoded_representation's bound (chain.cpp zstd_bound)
inline uint64_t zbound(uint64_t n) { return n + 4 + 14 + 4 + 3 * ((n + 999) / 1000); }

__device__ __forceinline__ uint32_t lz4_extra(uint32_t v) { return v >= 15 ? (v - 15) / 255 + 1 : 0u; }

// blosclz (c-blosc blosclz.c, the FastLZ level-2 format): literal runs of 1..32 bytes behind a
// control byte run-1; a match: control (len-2) << 5 | distance-1 >> 8 (len 3..8; 7 << 5 and 255-terminated
// extension bytes for longer ones), then the distance's low byte; distances above 8191 use the
// reserved low byte 255 under high bits 31 and two big-endian bytes of distance - 8192.
__device__ __forceinline__ uint32_t blz_match_size(uint32_t L, uint32_t dist) {
  const uint32_t ext = L - 2 < 7 ? 0u : (L - 9) / 255 + 1;
  return 1 + ext + 1 + (dist - 1 >= 8191 ? 2u : 0u);
}

// snappy (google/snappy format_description.txt, c-blosc's snappy_wrap_compress = snappy::RawCompress):
// a varint of the stream's length, then elements: a literal (tag 00, length - 1 in the tag below 60,
// else in 1..4 following bytes) and copies of at most 64 bytes (tag 01: length 4..11, offset < 2048,
// two bytes; tag 10: length 1..64, a 2-byte offset); longer matches are several copies.
constexpr int FMT_LZ4 = 0, FMT_BLZ = 1, FMT_SNAPPY = 2;
__device__ __forceinline__ uint32_t sn_varint_size(uint32_t v) {
  uint32_t n = 1;
  while (v >= 128) {
    v >>= 7;
    n++;
  }
  return n;
}
__device__ __forceinline__ uint32_t sn_lit_size(uint32_t ll) {
  if (!ll) return 0;
  const uint32_t n = ll - 1;
  return 1 + (n < 60 ? 0u : n < 256 ? 1u : n < 65536 ? 2u : n < (1u << 24) ? 3u : 4u) + ll;
}
__device__ __forceinline__ uint32_t sn_copy_piece(uint32_t L) { return L > 64 ? (L - 64 >= 4 ? 64u : 60u) : L; }
__device__ __forceinline__ uint32_t sn_match_size(uint32_t L, uint32_t off) {
  uint32_t n = 0;
  while (L) {
    const uint32_t c = sn_copy_piece(L);
    n += (c >= 4 && c <= 11 && off < 2048) ? 2u : 3u;
    L -= c;
  }
  return n;
}

// stream s of an item: (offset in the item, length)
__device__ __forceinline__ void stream_range(const BloscEnc &E, uint32_t s, uint64_t &off, uint32_t &len) {
  const uint32_t nfull = (uint32_t)(E.nbytes / E.bs);
  if (s < nfull * E.nsplit) {
    const uint32_t b = s / E.nsplit, j = s % E.nsplit;
    const uint32_t ne = (uint32_t)(E.bs / E.nsplit);
    off = (uint64_t)b * E.bs + (uint64_t)j * ne;
    len = ne;
  } else {
    off = (uint64_t)nfull * E.bs;
    len = (uint32_t)(E.nbytes - off);
  }
}

__global__ __launch_bounds__(256) void k_blosc_shuf_enc(const ZgItem *items, const uint32_t *status,
                                                        uint32_t n_items, BloscEnc E, uint8_t *staging) {
  const uint32_t item = blockIdx.x / E.nblk, b = blockIdx.x % E.nblk;
  if (item >= n_items || status[item]) return;
  const uint8_t *in = (const uint8_t *)items[item].src + (uint64_t)b * E.bs;
  uint8_t *out = staging + (uint64_t)item * E.nbytes + (uint64_t)b * E.bs;
  const uint64_t b0 = (uint64_t)b * E.bs;
  const uint32_t bsize = (uint32_t)min<uint64_t>(E.bs, E.nbytes - b0), ts = E.ts;
  if (E.shuffle == 1 && ts > 1) {  // shuffled[i * neb + j] = in[j * ts + i]
    const uint32_t neb = bsize / ts, body = neb * ts;
    for (uint32_t q = threadIdx.x; q < bsize; q += 256) {
      uint8_t v;
      if (q < body) {
        const uint32_t i = q / neb, j = q - i * neb;
        v = in[(uint64_t)j * ts + i];
      } else {
        v = in[q];
      }
      out[q] = v;
    }
  } else if (E.shuffle == 2 && bsize >= ts) {
    // bit-row r = b*8 + k holds bit k of byte b of every element; element count a multiple of 8
    // A thread takes 8 elements (8 ts contiguous input bytes) and per byte b transposes the 8x8 bit
    // matrix (rows: the elements' byte b) into column byte g of bit-rows 8b..8b+7 (coalesced stores)
    const uint32_t size = bsize / ts, n8 = (size % 8) ? 0u : size, body = n8 * ts, rb = n8 / 8;
    for (uint32_t g = threadIdx.x; g < rb; g += 256) {
      const uint8_t *e = in + 8ull * g * ts;
      for (uint32_t bb = 0; bb < ts; bb++) {
        uint64_t x = 0;
#pragma unroll
        for (uint32_t m = 0; m < 8; m++) x |= (uint64_t)e[m * ts + bb] << (8 * m);
        uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
        x ^= t ^ (t << 7);
        t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
        x ^= t ^ (t << 14);
        t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
        x ^= t ^ (t << 28);  // byte k: bit k of the 8 elements' byte bb
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) out[(uint64_t)(8 * bb + k) * rb + g] = (uint8_t)(x >> (8 * k));
      }
    }
    for (uint32_t q = body + threadIdx.x; q < bsize; q += 256) out[q] = in[q];
  } else {
    for (uint32_t q = threadIdx.x; q < bsize; q += 256) out[q] = in[q];
  }
}

struct Lz4Smem {
  uint32_t head[LZ4E_HSIZE];
  uint32_t tot;
};

// One LZ4 block, blosclz stream or snappy stream per stream (FMT): out_len[s] = compressed length, or
// ~0 when it would not be smaller (stored). scratch per wave: 3 u32 per possible sequence (match
// start, length, offset).
template <int FMT>
__global__ __launch_bounds__(64) void k_lz4_encode(const uint32_t *status, uint32_t n_items, BloscEnc E,
                                                   const uint8_t *staging, uint8_t *outs, uint64_t out_pitch,
                                                   uint32_t *out_len, uint32_t *scratch, uint64_t seq_cap) {
  __shared__ Lz4Smem S;
  const uint32_t lane = threadIdx.x;
  uint32_t *ms = scratch + (uint64_t)blockIdx.x * seq_cap * 3;
  uint32_t *ml = ms + seq_cap, *mo = ml + seq_cap;
  const uint64_t n_streams = (uint64_t)n_items * E.spi;
  for (uint64_t sg = blockIdx.x; sg < n_streams; sg += gridDim.x) {
    const uint32_t item = (uint32_t)(sg / E.spi), si = (uint32_t)(sg % E.spi);
    if (status[item]) continue;
    uint64_t off;
    uint32_t m;
    stream_range(E, si, off, m);
    const uint8_t *in = staging + (uint64_t)item * E.nbytes + off;
    for (uint32_t k = lane; k < LZ4E_HSIZE; k += 64) S.head[k] = 0;
    __syncthreads();
    // ---- greedy LZ77 parse, 64 positions a step
    uint32_t ns = 0, skip = 0;
    const uint32_t mlast = m > LZ4E_MFLIMIT ? m - LZ4E_MFLIMIT : 0u;  // a match starts before this
    for (uint32_t base = 0; base < mlast; base += 64) {
      if (skip >= base + 64) continue;
      const uint32_t p = base + lane;
      const bool hv = p + 4 <= m;
      const uint32_t w4 = hv ? ld4u(in + p) : 0u;
      const uint32_t h = (w4 * 0x9E3779B1u) >> (32 - LZ4E_HBITS);
      const uint32_t hvv = hv ? S.head[h] : 0u;
      __syncthreads();
      if (hv) S.head[h] = p + 1;
      uint32_t mlen = 0, cand = 0;
      if (hvv && p >= skip && p < mlast) {
        cand = hvv - 1;
        if (p - cand <= (FMT == FMT_BLZ ? BLZ_MAXOFF : LZ4E_MAXOFF) && ld4u(in + cand) == w4) {
          const uint32_t lim = min(LZ4E_CAP1, m - LZ4E_LAST - p);
          uint32_t k = 4;
          while (k < lim && in[p + k] == in[cand + k]) k++;
          mlen = k >= 4 && k <= lim ? k : 0u;
        }
      }
      const uint32_t lim = min(64u, mlast - base);
      const uint64_t M = __ballot(mlen >= 4);
      uint32_t pos = skip > base ? skip - base : 0;
      while (pos < lim) {
        const uint64_t rest = M >> pos;
        if (!rest) {
          pos = lim;
          break;
        }
        const uint32_t mi = pos + (uint32_t)__builtin_ctzll(rest);
        if (mi >= lim) {
          pos = lim;
          break;
        }
        uint32_t L = (uint32_t)__builtin_amdgcn_readlane((int)mlen, (int)mi);
        const uint32_t cnd = (uint32_t)__builtin_amdgcn_readlane((int)cand, (int)mi);
        const uint32_t pm = base + mi;
        const uint32_t mlim = m - LZ4E_LAST - pm;
        if (L == LZ4E_CAP1 && mlim > LZ4E_CAP1) {  // the wave extends a long match
          for (uint32_t k0 = LZ4E_CAP1;; k0 += 64) {
            const uint32_t k = k0 + lane;
            const bool mis = k < mlim && in[pm + k] != in[cnd + k];
            const uint64_t bm = __ballot(mis);
            if (bm) {
              L = k0 + (uint32_t)__builtin_ctzll(bm);
              break;
            }
            if (k0 + 64 >= mlim) {
              L = mlim;
              break;
            }
          }
        }
        if (lane == 0) {
          ms[ns] = pm;
          ml[ns] = L;
          mo[ns] = pm - cnd;
        }
        ns++;
        pos = mi + L;
      }
      skip = base + pos;
    }
    __syncthreads();
    // ---- sizes: sequence k's literals run from the previous match's end to its start; a last
    // sequence of literals only
    auto seq_size = [&](uint32_t k, uint32_t &lit0, uint32_t &ll) -> uint32_t {
      lit0 = k ? ms[k - 1] + ml[k - 1] : 0u;
      ll = (k == ns ? m : ms[k]) - lit0;
      if (FMT == FMT_BLZ) return (ll + 31) / 32 + ll + (k == ns ? 0u : blz_match_size(ml[k], mo[k]));
      if (FMT == FMT_SNAPPY) return sn_lit_size(ll) + (k == ns ? 0u : sn_match_size(ml[k], mo[k]));
      if (k == ns) return 1 + lz4_extra(ll) + ll;
      return 1 + lz4_extra(ll) + ll + 2 + lz4_extra(ml[k] - 4);
    };
    const uint32_t pre = FMT == FMT_SNAPPY ? sn_varint_size(m) : 0u;  // snappy: the length preamble
    uint32_t total = 0;
    for (uint32_t k = lane; k <= ns; k += 64) {
      uint32_t a, b;
      total += seq_size(k, a, b);
    }
    for (int o = 32; o; o >>= 1) total += __shfl_xor(total, o, 64);
    total += pre;
    if (total >= m) {  // stored
      if (lane == 0) out_len[sg] = 0xFFFFFFFFu;
      continue;
    }
    uint8_t *out = outs + sg * out_pitch;
    uint32_t obase = pre;
    if (FMT == FMT_SNAPPY && lane == 0) {
      uint32_t v = m, q = 0;
      for (; v >= 128; v >>= 7) out[q++] = (uint8_t)(v | 128);
      out[q] = (uint8_t)v;
    }
    for (uint32_t c0 = 0; c0 <= ns; c0 += 64) {
      const uint32_t k = c0 + lane;
      uint32_t sz = 0, lit0 = 0, ll = 0;
      if (k <= ns) sz = seq_size(k, lit0, ll);
      uint32_t incl = sz;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if ((int)lane >= o) incl += u;
      }
      const uint32_t tot = __shfl(incl, 63, 64);
      if (FMT == FMT_SNAPPY && k <= ns) {
        uint8_t *o = out + obase + incl - sz;
        if (ll) {
          const uint32_t n = ll - 1;
          if (n < 60) {
            *o++ = (uint8_t)(n << 2);
          } else {
            const uint32_t nb = n < 256 ? 1u : n < 65536 ? 2u : n < (1u << 24) ? 3u : 4u;
            *o++ = (uint8_t)((59 + nb) << 2);
            for (uint32_t q = 0; q < nb; q++) *o++ = (uint8_t)(n >> (8 * q));
          }
          for (uint32_t q = 0; q < ll; q++) o[q] = in[lit0 + q];
          o += ll;
        }
        if (k < ns) {
          uint32_t L = ml[k];
          const uint32_t of = mo[k];
          while (L) {
            const uint32_t c = sn_copy_piece(L);
            if (c >= 4 && c <= 11 && of < 2048) {
              *o++ = (uint8_t)(1u | ((c - 4) << 2) | ((of >> 8) << 5));
              *o++ = (uint8_t)of;
            } else {
              *o++ = (uint8_t)(2u | ((c - 1) << 2));
              *o++ = (uint8_t)of;
              *o++ = (uint8_t)(of >> 8);
            }
            L -= c;
          }
        }
      } else if (FMT == FMT_BLZ && k <= ns) {
        uint8_t *o = out + obase + incl - sz;
        for (uint32_t q = 0; q < ll; q += 32) {  // literal runs of <= 32 bytes
          const uint32_t r = min(32u, ll - q);
          *o++ = (uint8_t)(r - 1);
          for (uint32_t t = 0; t < r; t++) o[t] = in[lit0 + q + t];
          o += r;
        }
        if (k < ns) {
          const uint32_t L = ml[k], d = mo[k] - 1;
          const bool far = d >= 8191;
          const uint32_t hi = far ? 31u : d >> 8;
          if (L - 2 < 7) {
            *o++ = (uint8_t)(((L - 2) << 5) | hi);
          } else {
            *o++ = (uint8_t)((7u << 5) | hi);
            uint32_t r = L - 9;
            for (; r >= 255; r -= 255) *o++ = 255;
            *o++ = (uint8_t)r;
          }
          if (far) {
            const uint32_t f = mo[k] - 8192;
            *o++ = 255;
            *o++ = (uint8_t)(f >> 8);
            *o++ = (uint8_t)f;
          } else {
            *o++ = (uint8_t)d;
          }
        }
      } else if (k <= ns) {
        uint8_t *o = out + obase + incl - sz;
        const uint32_t mm = k < ns ? ml[k] - 4 : 0u;
        *o++ = (uint8_t)((min(ll, 15u) << 4) | (k < ns ? min(mm, 15u) : 0u));
        if (ll >= 15) {
          uint32_t r = ll - 15;
          for (; r >= 255; r -= 255) *o++ = 255;
          *o++ = (uint8_t)r;
        }
        for (uint32_t q = 0; q < ll; q++) o[q] = in[lit0 + q];
        o += ll;
        if (k < ns) {
          const uint32_t of = mo[k];
          *o++ = (uint8_t)of;
          *o++ = (uint8_t)(of >> 8);
          if (mm >= 15) {
            uint32_t r = mm - 15;
            for (; r >= 255; r -= 255) *o++ = 255;
            *o++ = (uint8_t)r;
          }
        }
      }
      obase += tot;
    }
    if (lane == 0) out_len[sg] = total;
    __syncthreads();
  }
}

}  // namespace

// one thread per item: stream offsets in the frame; stored streams; a memcpyed frame when the
// compressed one would not be smaller than nbytes + 16 (c-blosc's "destination too small" fallback)
__global__ void k_blosc_layout_enc(const uint32_t *status, uint32_t n_items, BloscEnc E, const uint32_t *clen,
                                   uint64_t *soff, uint64_t *ftot) {
  const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= n_items || status[item]) return;
  uint64_t p = 16 + 4ull * E.nblk;
  for (uint32_t s = 0; s < E.spi; s++) {
    uint64_t off;
    uint32_t len;
    stream_range(E, s, off, len);
    const uint32_t c = clen[(uint64_t)item * E.spi + s];
    soff[(uint64_t)item * E.spi + s] = p;
    p += 4 + ((c == 0xFFFFFFFFu || c >= len) ? len : c);
  }
  ftot[item] = p > E.nbytes + 16 ? (E.nbytes + 16) | (1ull << 63) : p;  // bit 63: memcpyed
}

// one workgroup per stream: {csize, payload}; the first stream of a block writes its bstarts entry,
// stream 0 the header; a memcpyed frame: each stream copies its range of the unshuffled input
__global__ __launch_bounds__(256) void k_blosc_write_enc(const ZgItem *items, const uint32_t *status,
                                                         uint32_t n_items, BloscEnc E, const uint8_t *staging,
                                                         const uint8_t *cdata, uint64_t cpitch,
                                                         const uint64_t *cptr, const uint32_t *clen,
                                                         const uint64_t *soff, const uint64_t *ftot,
                                                         uint8_t *slots, uint64_t slot_bytes) {
  const uint64_t sg = blockIdx.x;
  const uint32_t item = (uint32_t)(sg / E.spi), si = (uint32_t)(sg % E.spi);
  if (item >= n_items || status[item]) return;
  uint8_t *fr = slots + (uint64_t)item * slot_bytes + BLE_HDR;
  const uint64_t ft = ftot[item];
  const bool memcpyed = ft >> 63;
  const uint64_t total = ft & ~(1ull << 63);
  uint64_t off;
  uint32_t len;
  stream_range(E, si, off, len);
  if (si == 0 && threadIdx.x < 16) {
    const uint32_t flags = (E.shuffle == 1 ? 0x1u : E.shuffle == 2 ? 0x4u : 0u) | (memcpyed ? 0x2u : 0u) |
                           (E.nsplit == 1 ? 0x10u : 0u) | (E.comp << 5);
    const uint32_t v = threadIdx.x;
    uint8_t b;
    if (v == 0) b = 2;                       // BLOSC_VERSION_FORMAT
    else if (v == 1) b = 1;                  // the compressor's format version
    else if (v == 2) b = (uint8_t)flags;
    else if (v == 3) b = (uint8_t)E.ts;
    else if (v < 8) b = (uint8_t)(E.nbytes >> (8 * (v - 4)));
    else if (v < 12) b = (uint8_t)(E.bs >> (8 * (v - 8)));
    else b = (uint8_t)(total >> (8 * (v - 12)));
    fr[v] = b;
  }
  if (memcpyed) {
    const uint8_t *src = (const uint8_t *)items[item].src + off;
    for (uint32_t q = threadIdx.x; q < len; q += 256) fr[16 + off + q] = src[q];
    return;
  }
  const uint64_t p = soff[sg];
  const uint32_t nfull = (uint32_t)(E.nbytes / E.bs);
  const bool first_of_block = si >= nfull * E.nsplit || si % E.nsplit == 0;
  if (first_of_block && threadIdx.x < 4) {
    const uint32_t b = si < nfull * E.nsplit ? si / E.nsplit : nfull;
    fr[16 + 4 * b + threadIdx.x] = (uint8_t)(p >> (8 * threadIdx.x));
  }
  const uint32_t c = clen[sg];
  const bool stored = c == 0xFFFFFFFFu || c >= len;
  const uint32_t cs = stored ? len : c;
  if (threadIdx.x < 4) fr[p + threadIdx.x] = (uint8_t)(cs >> (8 * threadIdx.x));
  const uint8_t *src = stored ? staging + (uint64_t)item * E.nbytes + off
                              : (cptr ? (const uint8_t *)cptr[sg] : cdata + sg * cpitch);
  for (uint32_t q = threadIdx.x; q < cs; q += 256) fr[p + 4 + q] = src[q];
}

__global__ void k_blosc_items_enc(ZgItem *items, const uint32_t *status, uint32_t n_items, BloscEnc E,
                                  const uint64_t *ftot, uint8_t *slots, uint64_t slot_bytes) {
  const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= n_items || status[item]) return;
  uint8_t *fr = slots + (uint64_t)item * slot_bytes + BLE_HDR;
  if (E.spi == 0) {  // an empty input: a header-only memcpyed frame
    const uint8_t h[16] = {2, 1, (uint8_t)(0x2u | (E.comp << 5)), (uint8_t)E.ts, 0, 0, 0, 0,
                           (uint8_t)E.bs, (uint8_t)(E.bs >> 8), (uint8_t)(E.bs >> 16), (uint8_t)(E.bs >> 24), 16, 0, 0, 0};
    for (int k = 0; k < 16; k++) fr[k] = h[k];
  }
  items[item].src = (uint64_t)fr;
  items[item].len = ftot[item] & ~(1ull << 63);
}

// zstd streams: the stream table as items for the zstd encoder, and its lengths back
__global__ void k_blosc_zitems(const uint32_t *status, uint32_t n_items, BloscEnc E, const uint8_t *staging,
                               ZgItem *zitems, uint32_t *zstatus) {
  const uint64_t sg = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (sg >= (uint64_t)n_items * E.spi) return;
  const uint32_t item = (uint32_t)(sg / E.spi), si = (uint32_t)(sg % E.spi);
  uint64_t off;
  uint32_t len;
  stream_range(E, si, off, len);
  zitems[sg] = ZgItem{(uint64_t)(staging + (uint64_t)item * E.nbytes + off), len, (uint32_t)sg, 0, 0, 0};
  zstatus[sg] = status[item] ? 1u : 0u;
}
__global__ void k_blosc_zlens(const ZgItem *zitems, const uint32_t *zstatus, uint64_t n, uint64_t *cptr,
                              uint32_t *clen) {
  const uint64_t sg = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (sg >= n) return;
  const bool ok = zstatus[sg] == 0;
  cptr[sg] = ok ? zitems[sg].src : 0;
  clen[sg] = ok ? (uint32_t)min<uint64_t>(zitems[sg].len, 0xFFFFFFFEull) : 0xFFFFFFFFu;
}

// a zlib stream's slot: the member offset, the stream and deflate's worst case (stored blocks: 5 bytes
// per block of at most 16384 symbols), the trailer
static uint64_t zlib_pitch(uint64_t n) { return (GZE_HDR + n + 5 * (n / 1024 + 2) + 64 + 255) & ~255ull; }

BloscEnc blosc_enc_params(uint32_t comp, uint32_t shuffle, uint32_t ts, uint64_t nbytes, uint64_t blocksize) {
  BloscEnc E{};
  E.comp = comp;
  E.ts = ts ? ts : 1;
  E.shuffle = (shuffle == 1 && E.ts > 1) || shuffle == 2 ? shuffle : 0u;
  E.nbytes = nbytes;
  // block size: the codec's, else 128 KiB (c-blosc's compute_blocksize lands between 32 KiB and
  // 256 KiB for typical levels); a multiple of the type size, at most nbytes
  uint64_t bs = blocksize ? blocksize : (128u << 10);
  bs = std::max<uint64_t>(E.ts, bs - bs % E.ts);
  if (nbytes && bs > nbytes) bs = nbytes;
  if (!bs) bs = E.ts;
  E.bs = bs;
  E.nblk = (uint32_t)(nbytes ? (nbytes + bs - 1) / bs : 0);
  // split the byte-shuffled planes into streams of their own (c-blosc's forward-compatible rule for
  // its LZ compressors); zstd streams stay whole
  E.nsplit = (E.shuffle == 1 && (comp == BL_COMP_LZ4 || comp == BL_COMP_BLOSCLZ || comp == BL_COMP_SNAPPY) &&
              E.ts <= 16 && bs % E.ts == 0)
                 ? E.ts : 1u;
  const uint32_t nfull = (uint32_t)(nbytes / bs);
  E.spi = nfull * E.nsplit + ((nbytes % bs) ? 1u : 0u);
  E.ne_max = std::max<uint64_t>(bs / E.nsplit, nbytes % bs);
  return E;
}

uint64_t blosc_encode_scratch(const BloscEnc &E, uint32_t n_items) {
  const uint64_t ns = (uint64_t)n_items * E.spi;
  uint64_t b = (uint64_t)n_items * E.nbytes + 256;      // staging
  b += ns * (8 + 8 + 4 + 4) + 1024;                       // soff, cptr, clen, zstatus
  b += (uint64_t)n_items * 8 + 256;                       // ftot
  if (E.comp == BL_COMP_LZ4 || E.comp == BL_COMP_BLOSCLZ || E.comp == BL_COMP_SNAPPY) {
    const uint64_t grid = std::min<uint64_t>(std::max<uint64_t>(ns, 1), (uint64_t)device_cu_count() * 8);
    b += ns * ((E.ne_max + 255) & ~255ull);                // compressed streams
    b += grid * (E.ne_max / 4 + 2) * 12 + 256;             // sequence records
  } else if (E.comp == BL_COMP_ZLIB) {
    b += ns * zlib_pitch(E.ne_max) + ns * sizeof(ZgItem) + 256;
    b += (uint64_t)gzip_encode_grid((uint32_t)std::max<uint64_t>(ns, 1)) * GZE_BLK_SYMS * 4 + 256;
  } else {
    const uint64_t zp = ((ZE_HDR + zbound(E.ne_max) + 64 + 255) & ~255ull);
    b += ns * zp + ns * sizeof(ZgItem) + 256;
    b += zstd_encode_scratch((uint32_t)ns, E.ne_max);
  }
  return b;
}

hipError_t launch_blosc_encode(ZgItem *items, uint32_t *status, uint32_t n_items, const BloscEnc &E, uint8_t *slots,
                               uint64_t slot_bytes, uint8_t *scratch, int zlevel, hipStream_t s) {
  if (!n_items) return hipSuccess;
  const uint64_t ns = (uint64_t)n_items * E.spi;
  uint8_t *p = scratch;
  auto take = [&](uint64_t bytes) {
    uint8_t *r = p;
    p += (bytes + 255) & ~255ull;
    return r;
  };
  uint8_t *staging = take((uint64_t)n_items * E.nbytes);
  uint64_t *soff = (uint64_t *)take(ns * 8);
  uint64_t *cptr = (uint64_t *)take(ns * 8);
  uint32_t *clen = (uint32_t *)take(ns * 4);
  uint32_t *zstatus = (uint32_t *)take(ns * 4);
  uint64_t *ftot = (uint64_t *)take((uint64_t)n_items * 8);
  if (E.nblk)
    hipLaunchKernelGGL(k_blosc_shuf_enc, dim3(n_items * E.nblk), dim3(256), 0, s, items, status, n_items, E, staging);
  const uint8_t *cdata = nullptr;
  uint64_t cpitch = 0;
  const uint64_t *cp = nullptr;
  if (ns && (E.comp == BL_COMP_LZ4 || E.comp == BL_COMP_BLOSCLZ || E.comp == BL_COMP_SNAPPY)) {
    cpitch = (E.ne_max + 255) & ~255ull;
    uint8_t *outs = take(ns * cpitch);
    const uint32_t grid = (uint32_t)std::min<uint64_t>(ns, (uint64_t)device_cu_count() * 8);
    const uint64_t seq_cap = E.ne_max / 4 + 2;
    uint32_t *seqs = (uint32_t *)take((uint64_t)grid * seq_cap * 12);
    if (E.comp == BL_COMP_BLOSCLZ)
      hipLaunchKernelGGL(k_lz4_encode<FMT_BLZ>, dim3(grid), dim3(64), 0, s, status, n_items, E, staging, outs,
                         cpitch, clen, seqs, seq_cap);
    else if (E.comp == BL_COMP_SNAPPY)
      hipLaunchKernelGGL(k_lz4_encode<FMT_SNAPPY>, dim3(grid), dim3(64), 0, s, status, n_items, E, staging, outs,
                         cpitch, clen, seqs, seq_cap);
    else
      hipLaunchKernelGGL(k_lz4_encode<FMT_LZ4>, dim3(grid), dim3(64), 0, s, status, n_items, E, staging, outs,
                         cpitch, clen, seqs, seq_cap);
    cdata = outs;
  } else if (ns && E.comp == BL_COMP_ZLIB) {
    const uint64_t zp = zlib_pitch(E.ne_max);
    uint8_t *zslots = take(ns * zp);
    ZgItem *zitems = (ZgItem *)take(ns * sizeof(ZgItem));
    uint32_t *sym = (uint32_t *)take((uint64_t)gzip_encode_grid((uint32_t)ns) * GZE_BLK_SYMS * 4);
    hipLaunchKernelGGL(k_blosc_zitems, dim3((uint32_t)((ns + 255) / 256)), dim3(256), 0, s, status, n_items, E,
                       staging, zitems, zstatus);
    hipError_t e = launch_gzip_encode(zitems, zstatus, (uint32_t)ns, zslots, zp, sym, zlevel, s, true);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_blosc_zlens, dim3((uint32_t)((ns + 255) / 256)), dim3(256), 0, s, zitems, zstatus, ns, cptr,
                       clen);
    cp = cptr;
  } else if (ns) {
    const uint64_t zp = ((ZE_HDR + zbound(E.ne_max) + 64 + 255) & ~255ull);
    uint8_t *zslots = take(ns * zp);
    ZgItem *zitems = (ZgItem *)take(ns * sizeof(ZgItem));
    uint8_t *zscr = take(zstd_encode_scratch((uint32_t)ns, E.ne_max));
    hipLaunchKernelGGL(k_blosc_zitems, dim3((uint32_t)((ns + 255) / 256)), dim3(256), 0, s, status, n_items, E,
                       staging, zitems, zstatus);
    hipError_t e = launch_zstd_encode(zitems, zstatus, (uint32_t)ns, E.ne_max, zslots, zp, zscr, 0, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_blosc_zlens, dim3((uint32_t)((ns + 255) / 256)), dim3(256), 0, s, zitems, zstatus, ns, cptr,
                       clen);
    cp = cptr;
  }
  hipLaunchKernelGGL(k_blosc_layout_enc, dim3((n_items + 255) / 256), dim3(256), 0, s, status, n_items, E, clen, soff,
                     ftot);
  if (ns)
    hipLaunchKernelGGL(k_blosc_write_enc, dim3((uint32_t)ns), dim3(256), 0, s, items, status, n_items, E, staging,
                       cdata, cpitch, cp, clen, soff, ftot, slots, slot_bytes);
  hipLaunchKernelGGL(k_blosc_items_enc, dim3((n_items + 255) / 256), dim3(256), 0, s, items, status, n_items, E,
                     ftot, slots, slot_bytes);
  return hipGetLastError();
}

}  // namespace zgpu
