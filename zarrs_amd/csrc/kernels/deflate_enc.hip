// gzip (RFC 1952 / DEFLATE RFC 1951) ENCODER on gfx950: the write half of the gzip codec
// (GzipCodec::encode, zarrs/src/array/codec/bytes_to_bytes/gzip/gzip_codec.rs:96-107, flate2's
// GzEncoder). The output is a valid gzip member any inflater decodes (zlib, flate2, k_gzip); its bytes
// are not flate2's (LZ77 parsing and block splitting are encoder choices: gzip_codec.rs:126-128).
//
// One 64-lane wave encodes one item (a persistent grid loops over the items):
//   1. CRC-32 (IEEE) of the input for the trailer: 64 lane segments with slice-by-4 LDS tables,
//      merged by crc32_combine (crc.hpp)
//   2. LZ77, 64 positions per step: every lane hashes the 4 bytes at its position, reads the
//      hash bucket (u16 positions in LDS, filled by the earlier steps) and extends a candidate match
//      (aligned dword loads + v_alignbyte, up to 258 bytes, 32 KiB window); the greedy parse of the
//      step is a scalar walk over the ballot of match-starting lanes (one step per match, runs of
//      literals in one mask operation); the chosen symbols are written to the wave's symbol scratch
//      (u32 records) and counted into LDS histograms
//   3. per DEFLATE block (<= 16384 symbols): length-limited Huffman codes for the literal/length and
//      distance alphabets (frequency ranks computed lane-parallel, then the two-queue Huffman merge
//      and zlib's overflow repair of the bit-length counts), the run-length-coded code lengths with
//      their own code, then every 64 symbols' bit strings placed by a wave prefix sum of their
//      lengths and OR-ed into an LDS word buffer that is flushed to HBM in coalesced words; a block
//      the dynamic code would not shrink is written stored (BTYPE 00)
//   4. the trailer (CRC-32, ISIZE)
// The member is written at slot + GZE_HDR (the bit stream then starts word-aligned); the headroom in
// front of it takes crc32c codecs located at the start.
#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "crc.hpp"
#include "huff.hpp"
#include "launch.hpp"

namespace zgpu {
namespace {

constexpr uint32_t GZE_HBITS = 12, GZE_HSIZE = 1u << GZE_HBITS;
constexpr uint32_t GZE_BB = 256;      // bit staging words
constexpr uint32_t GZE_FLUSH = GZE_BB - 104;  // flush once this many words are full
constexpr uint32_t GZE_WINDOW = 32768, GZE_MAXMATCH = 258;

struct GzeSmem {
  union {
    uint16_t head[GZE_HSIZE];  // hash -> (position + 1) mod 2^16, 0 = empty
    CrcTables crc;             // the input CRC runs before the LZ77 pass
  };
  uint32_t lfreq[288], dfreq[32], cfreq[20];
  uint32_t lcode[288], dcode[32], ccode[20];  // bit-reversed code | length << 16
  uint8_t llen[288], dlen[32], clen[20];
  HuffScratch hs;  // huff_lengths
  uint32_t blc[16], next[16];
  uint16_t rle[320];
  uint32_t bits[GZE_BB + 4];
  uint64_t s_len[1];
  uint32_t s_crc[1], nrle;
};

#define WSYNC() __syncthreads()

// order of the code length code lengths in a dynamic block header (RFC 1951 3.2.7)
__constant__ uint8_t c_clen_perm[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

__device__ __forceinline__ uint32_t ld4(const uint8_t *p) {
  // 4 bytes at any address from aligned dwords (a word holding one valid byte is always mapped)
  const uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t lo = w[0];
  const uint32_t hi = sh ? w[1] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}

__device__ __forceinline__ uint32_t rev_bits(uint32_t c, uint32_t n) { return n ? __builtin_bitreverse32(c) >> (32 - n) : 0u; }

// length - 3 -> literal/length code, extra bit count, extra value (RFC 1951 3.2.5)
__device__ __forceinline__ void len_sym(uint32_t x, uint32_t &code, uint32_t &eb, uint32_t &ev) {
  if (x < 8) {
    code = 257 + x, eb = 0, ev = 0;
  } else if (x == 255) {
    code = 285, eb = 0, ev = 0;
  } else {
    const uint32_t nb = 31 - __clz(x);
    eb = nb - 2;
    code = 257 + 4 * (nb - 1) + ((x >> eb) & 3);
    ev = x & ((1u << eb) - 1);
  }
}
// distance - 1 -> distance code, extra bit count, extra value
__device__ __forceinline__ void dist_sym(uint32_t x, uint32_t &code, uint32_t &eb, uint32_t &ev) {
  if (x < 4) {
    code = x, eb = 0, ev = 0;
  } else {
    const uint32_t nb = 31 - __clz(x);
    eb = nb - 1;
    code = 2 * nb + ((x >> eb) & 1);
    ev = x & ((1u << eb) - 1);
  }
}
__device__ __forceinline__ uint32_t len_extra(uint32_t c) { return (c >= 265 && c < 285) ? (c - 261) / 4 : 0u; }
__device__ __forceinline__ uint32_t dist_extra(uint32_t c) { return c < 4 ? 0u : (c - 2) / 2; }

__device__ __forceinline__ uint32_t wave_sum(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ uint32_t wave_max(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v = max(v, (uint32_t)__shfl_xor(v, o, 64));
  return v;
}

// canonical codes (RFC 1951 3.2.2), stored bit-reversed | length << 16
__device__ void huff_codes(GzeSmem &S, const uint8_t *lens, uint32_t n, uint32_t *codes) {
  if (threadIdx.x == 0) {
    for (uint32_t b = 0; b < 16; b++) S.blc[b] = 0;
    for (uint32_t s = 0; s < n; s++) S.blc[lens[s]]++;
    S.blc[0] = 0;
    uint32_t code = 0;
    for (uint32_t b = 1; b < 16; b++) {
      code = (code + S.blc[b - 1]) << 1;
      S.next[b] = code;
    }
    for (uint32_t s = 0; s < n; s++) {
      const uint32_t L = lens[s];
      codes[s] = L ? (rev_bits(S.next[L]++, L) | (L << 16)) : 0u;
    }
  }
  WSYNC();
}

// zlib trees.c scan_tree / send_tree run-length coding of one code-length sequence into S.rle
// (symbol | extra value << 8), counting S.cfreq. Lane 0 (serial, <= 316 lengths).
__device__ void rle_lengths(GzeSmem &S, const uint8_t *lens, uint32_t n) {
  uint32_t &cnt = S.nrle;
  int prevlen = -1, nextlen = lens[0];
  uint32_t count = 0, max_count = 7, min_count = 4;
  if (nextlen == 0) max_count = 138, min_count = 3;
  auto emit = [&](uint32_t sym, uint32_t ex) {
    S.rle[cnt++] = (uint16_t)(sym | (ex << 8));
    S.cfreq[sym]++;
  };
  for (uint32_t i = 0; i < n; i++) {
    const int curlen = nextlen;
    nextlen = i + 1 < n ? lens[i + 1] : 0xffff;
    if (++count < max_count && curlen == nextlen) continue;
    if (count < min_count) {
      for (uint32_t k = 0; k < count; k++) emit((uint32_t)curlen, 0);
    } else if (curlen != 0) {
      if (curlen != prevlen) {
        emit((uint32_t)curlen, 0);
        count--;
      }
      emit(16, count - 3);
    } else if (count <= 10) {
      emit(17, count - 3);
    } else {
      emit(18, count - 11);
    }
    count = 0;
    prevlen = curlen;
    if (nextlen == 0) max_count = 138, min_count = 3;
    else if (curlen == nextlen) max_count = 6, min_count = 3;
    else max_count = 7, min_count = 4;
  }
}

struct BitOut {
  uint32_t bitpos;  // bits in S.bits
  uint32_t outw;    // words already flushed
  uint32_t *out32;  // the stream's first word in HBM
  uint32_t cap_w;   // words the slot holds for the stream
  uint32_t ovf;     // 1: the slot would overflow (nothing more is written)
};

// lane 0 appends v (n <= 32 bits) at the bit position (all lanes keep the same bitpos)
__device__ __forceinline__ void put(GzeSmem &S, BitOut &B, uint32_t v, uint32_t n) {
  if (threadIdx.x == 0 && n) {
    const uint32_t w = B.bitpos >> 5, sh = B.bitpos & 31;
    const uint64_t t = (uint64_t)v << sh;
    S.bits[w] |= (uint32_t)t;
    if (sh + n > 32) S.bits[w + 1] |= (uint32_t)(t >> 32);
  }
  B.bitpos += n;
}

// full words (all words with `all`) to HBM; the partial word moves to the front
__device__ void flush(GzeSmem &S, BitOut &B, bool all) {
  WSYNC();
  const uint32_t F = all ? (B.bitpos + 31) >> 5 : B.bitpos >> 5;
  if (B.outw + F > B.cap_w) B.ovf = 1;
  if (!B.ovf)
    for (uint32_t k = threadIdx.x; k < F; k += 64) B.out32[B.outw + k] = S.bits[k];
  WSYNC();
  const uint32_t keep = (!all && (B.bitpos & 31)) ? S.bits[F] : 0u;
  WSYNC();
  for (uint32_t k = threadIdx.x; k < GZE_BB + 4; k += 64) S.bits[k] = 0;
  WSYNC();
  if (threadIdx.x == 0) S.bits[0] = keep;
  WSYNC();
  B.outw += F;
  B.bitpos -= all ? B.bitpos : 32 * F;
}

__device__ __forceinline__ void maybe_flush(GzeSmem &S, BitOut &B) {
  if ((B.bitpos >> 5) >= GZE_FLUSH) flush(S, B, false);
}

// stored blocks (BTYPE 00) for in[b0, b1)
__device__ void emit_stored(GzeSmem &S, BitOut &B, const uint8_t *in, uint32_t b0, uint32_t b1, bool final) {
  uint32_t p = b0;
  do {
    const uint32_t len = min(b1 - p, 65535u);
    const bool last = p + len >= b1;
    maybe_flush(S, B);
    put(S, B, (final && last) ? 1u : 0u, 1);
    put(S, B, 0, 2);
    B.bitpos = (B.bitpos + 7) & ~7u;
    put(S, B, len, 16);
    put(S, B, len ^ 0xFFFFu, 16);
    WSYNC();
    for (uint32_t k0 = 0; k0 < len; k0 += 256) {
      maybe_flush(S, B);
      for (uint32_t k = k0 + threadIdx.x; k < min(len, k0 + 256); k += 64) {
        const uint32_t o = B.bitpos + 8 * (k - k0);
        atomicOr(&S.bits[o >> 5], (uint32_t)in[p + k] << (o & 31));
      }
      WSYNC();
      B.bitpos += 8 * min(256u, len - k0);
    }
    p += len;
  } while (p < b1);
}

// One DEFLATE block: symbols syms[0..nsym) covering in[b0, b1); S.lfreq / S.dfreq hold their counts.
__device__ void emit_block(GzeSmem &S, BitOut &B, const uint32_t *syms, uint32_t nsym, const uint8_t *in, uint32_t b0,
                           uint32_t b1, bool final) {
  const uint32_t lane = threadIdx.x;
  if (lane == 0) S.lfreq[256] += 1;  // end of block
  WSYNC();
  huff_lengths(S.hs, S.lfreq, 286, 15, S.llen);
  huff_lengths(S.hs, S.dfreq, 30, 15, S.dlen);
  huff_codes(S, S.llen, 286, S.lcode);
  huff_codes(S, S.dlen, 30, S.dcode);
  uint32_t hl = 0, hd = 0;
  for (uint32_t s = lane; s < 286; s += 64)
    if (S.llen[s]) hl = max(hl, s + 1);
  for (uint32_t s = lane; s < 30; s += 64)
    if (S.dlen[s]) hd = max(hd, s + 1);
  const uint32_t hlit = max(257u, wave_max(hl)), hdist = max(1u, wave_max(hd));
  for (uint32_t s = lane; s < 20; s += 64) S.cfreq[s] = 0;
  WSYNC();
  if (lane == 0) {
    S.nrle = 0;
    rle_lengths(S, S.llen, hlit);
    rle_lengths(S, S.dlen, hdist);
  }
  WSYNC();
  huff_lengths(S.hs, S.cfreq, 19, 7, S.clen);
  huff_codes(S, S.clen, 19, S.ccode);
  uint32_t hclen = 4;
  for (uint32_t i = 0; i < 19; i++)
    if (S.clen[c_clen_perm[i]]) hclen = max(hclen, i + 1);
  // sizes: dynamic block vs stored
  uint32_t bits = 0;  // < 2^32: a block holds <= 16384 symbols of <= 48 bits
  for (uint32_t s = lane; s < 286; s += 64) bits += S.lfreq[s] * (S.llen[s] + len_extra(s));
  for (uint32_t s = lane; s < 30; s += 64) bits += S.dfreq[s] * (S.dlen[s] + dist_extra(s));
  for (uint32_t k = lane; k < S.nrle; k += 64) {
    const uint32_t sym = S.rle[k] & 0xff;
    bits += S.clen[sym] + (sym == 16 ? 2 : sym == 17 ? 3 : sym == 18 ? 7 : 0);
  }
  bits = wave_sum(bits) + 17 + 3 * hclen;
  const uint64_t raw = b1 - b0;
  const uint64_t stored = 8 * raw + 42 * ((raw + 65534) / 65535 + (raw == 0));
  if (bits > stored) {
    emit_stored(S, B, in, b0, b1, final);
  } else {
    maybe_flush(S, B);
    put(S, B, final ? 1u : 0u, 1);
    put(S, B, 2, 2);
    put(S, B, hlit - 257, 5);
    put(S, B, hdist - 1, 5);
    put(S, B, hclen - 4, 4);
    for (uint32_t i = 0; i < hclen; i++) put(S, B, S.clen[c_clen_perm[i]], 3);
    for (uint32_t k = 0; k < S.nrle; k++) {
      if ((k & 63) == 0) maybe_flush(S, B);
      const uint32_t r = S.rle[k], sym = r & 0xff, ex = r >> 8;
      put(S, B, S.ccode[sym] & 0xFFFF, S.ccode[sym] >> 16);
      if (sym >= 16) put(S, B, ex, sym == 16 ? 2 : sym == 17 ? 3 : 7);
    }
    WSYNC();
    // symbols, 64 at a time: bit strings placed by a wave prefix sum of their lengths
    for (uint32_t k0 = 0; k0 < nsym; k0 += 64) {
      maybe_flush(S, B);
      const uint32_t k = k0 + lane;
      uint64_t v = 0;
      uint32_t nb = 0;
      if (k < nsym) {
        const uint32_t rec = syms[k];
        if (!(rec >> 31)) {
          const uint32_t c = S.lcode[rec & 0xff];
          v = c & 0xFFFF;
          nb = c >> 16;
        } else {
          uint32_t lc, le, lv, dc, de, dv;
          len_sym(rec & 0xff, lc, le, lv);
          dist_sym((rec >> 8) & 0x7FFF, dc, de, dv);
          const uint32_t l = S.lcode[lc], d = S.dcode[dc];
          const uint32_t ln = l >> 16, dn = d >> 16;
          v = (uint64_t)(l & 0xFFFF) | ((uint64_t)lv << ln) | ((uint64_t)(d & 0xFFFF) << (ln + le)) |
              ((uint64_t)dv << (ln + le + dn));
          nb = ln + le + dn + de;
        }
      }
      uint32_t incl = nb;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if ((int)lane >= o) incl += u;
      }
      const uint32_t o = B.bitpos + incl - nb;
      if (nb) {
        const uint32_t w = o >> 5, sh = o & 31;
        const uint64_t t = v << sh;
        atomicOr(&S.bits[w], (uint32_t)t);
        if ((uint32_t)(t >> 32)) atomicOr(&S.bits[w + 1], (uint32_t)(t >> 32));
        if (sh && (uint32_t)(v >> (64 - sh))) atomicOr(&S.bits[w + 2], (uint32_t)(v >> (64 - sh)));
      }
      B.bitpos += __shfl(incl, 63, 64);
      WSYNC();
    }
    put(S, B, S.lcode[256] & 0xFFFF, S.lcode[256] >> 16);
    WSYNC();
  }
  for (uint32_t s = lane; s < 288; s += 64) S.lfreq[s] = 0;
  if (lane < 32) S.dfreq[lane] = 0;
  WSYNC();
}

}  // namespace

// Adler-32 (RFC 1950) of in[0, n) on one wave: byte j adds b to s1 and (n - j) b to s2, so the lanes
// sum coalesced dwords in any order and the wave adds their residues (s1 = 1 + sum, s2 = n + sum).
__device__ uint32_t wave_adler32(const uint8_t *in, uint32_t n) {
  constexpr uint32_t M = 65521;
  const uint32_t lane = threadIdx.x;
  uint64_t A = 0, Bs = 0;
  uint32_t it = 0;
  for (uint32_t base = 0; base < n; base += 256) {
    const uint32_t j0 = base + 4 * lane;
    if (j0 < n) {
      const uint32_t w = j0 + 4 <= n ? ld4(in + j0) : 0u;
#pragma unroll
      for (uint32_t k = 0; k < 4; k++) {
        const uint32_t j = j0 + k;
        const uint32_t b = j0 + 4 <= n ? (w >> (8 * k)) & 0xff : (j < n ? in[j] : 0u);
        A += b;
        Bs += (uint64_t)(n - j) * b;
      }
    }
    if (++it == 4096) {  // per lane <= 16384 bytes between reductions: Bs < 2^53
      A %= M;
      Bs %= M;
      it = 0;
    }
  }
  uint32_t a = (uint32_t)(A % M), b = (uint32_t)(Bs % M);
#pragma unroll
  for (int o = 32; o; o >>= 1) {
    a += __shfl_xor(a, o, 64);
    b += __shfl_xor(b, o, 64);
  }
  const uint32_t s1 = (1u + a) % M, s2 = (n % M + b) % M;
  return (s2 << 16) | s1;
}

// items[i] {src,len} -> a gzip member in slot i at GZE_HDR; items rewritten to it. sym: grid * 16384
// u32 symbol records (one block's worth per wave). xfl: the header's XFL byte (flate2: 4 for level <= 1,
// 2 for level >= 9, else 0). zhdr != 0: a zlib stream (RFC 1950) instead, CMF FLG = zhdr, at slot i +
// GZE_HDR + 8 (the same bit stream position), with the Adler-32 trailer (blosc's zlib streams).
__global__ __launch_bounds__(64) void k_gzip_encode(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *slots,
                                                    uint64_t slot_bytes, uint32_t *sym_scratch, uint32_t xfl,
                                                    uint32_t zhdr) {
  __shared__ GzeSmem S;
  const uint32_t lane = threadIdx.x;
  uint32_t *syms = sym_scratch + (uint64_t)blockIdx.x * GZE_BLK_SYMS;
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    if (status[item]) continue;
    const ZgItem it = items[item];
    uint8_t *slot = slots + (uint64_t)item * slot_bytes;
    if (it.len >= 0x7FFFFFFFull) {
      if (lane == 0) status[item] = ZG_UNSUPPORTED;
      continue;
    }
    const uint8_t *in = (const uint8_t *)it.src;
    const uint32_t n = (uint32_t)it.len;
    // 1. CRC-32 of the input (tables in the hash table's space), or Adler-32 for zlib
    uint32_t crc;
    if (zhdr) {
      crc = wave_adler32(in, n);
    } else {
      build_tables(S.crc, POLY_CRC32);
      crc = wg_crc(in, n, S.crc, POLY_CRC32, S.s_len, S.s_crc);
    }
    WSYNC();
    for (uint32_t k = lane; k < GZE_HSIZE / 2; k += 64) ((uint32_t *)S.head)[k] = 0;
    for (uint32_t s = lane; s < 288; s += 64) S.lfreq[s] = 0;
    if (lane < 32) S.dfreq[lane] = 0;
    for (uint32_t k = lane; k < GZE_BB + 4; k += 64) S.bits[k] = 0;
    if (zhdr) {
      if (lane < 2) slot[GZE_HDR + 8 + lane] = (uint8_t)(lane == 0 ? zhdr >> 8 : zhdr);
    } else if (lane < 10)  // ID1 ID2 CM=deflate FLG=0 MTIME=0 XFL OS=255 (flate2's GzBuilder defaults)
      slot[GZE_HDR + lane] = lane == 0 ? 0x1f : lane == 1 ? 0x8b : lane == 2 ? 8 : lane == 8 ? (uint8_t)xfl : lane == 9 ? 255 : 0;
    WSYNC();
    BitOut B{0, 0, (uint32_t *)(slot + GZE_HDR + 10), (uint32_t)((slot_bytes - GZE_HDR - 10) / 4), 0};
    // 2. LZ77 in steps of 64 positions, symbols per block into syms[]
    uint32_t skip = 0, nsym = 0, blk0 = 0;
    for (uint32_t base = 0; base < n; base += 64) {
      if (skip >= base + 64) continue;
      const uint32_t p = base + lane;
      const bool hv = p + 4 <= n;
      uint32_t w4 = 0;
      if (hv) w4 = ld4(in + p);
      else if (p < n) w4 = in[p];
      const uint32_t h = (w4 * 0x9E3779B1u) >> (32 - GZE_HBITS);
      const uint32_t hvv = hv ? S.head[h] : 0u;
      WSYNC();
      if (hv && ((p + 1) & 0xFFFF)) S.head[h] = (uint16_t)(p + 1);
      uint32_t mlen = 0, dist = 0;
      if (hvv && p >= skip) {
        uint32_t cand = (p & ~0xFFFFu) | (hvv - 1);
        bool ok = true;
        if (cand >= p) {
          ok = p >= 65536u;
          cand -= 65536u;
        }
        if (ok && p - cand <= GZE_WINDOW && ld4(in + cand) == w4) {
          const uint32_t lim = min(GZE_MAXMATCH, n - p);
          uint32_t k = 4;
          bool done = false;
          while (k + 4 <= lim) {
            const uint32_t x = ld4(in + p + k) ^ ld4(in + cand + k);
            if (x) {
              k += (uint32_t)__builtin_ctz(x) >> 3;
              done = true;
              break;
            }
            k += 4;
          }
          if (!done)
            while (k < lim && in[p + k] == in[cand + k]) k++;
          mlen = k;
          dist = p - cand;
        }
      }
      // greedy parse of the step: a scalar walk over the match-starting lanes
      const uint32_t lim = min(64u, n - base);
      const uint64_t M = __ballot(mlen >= 4);
      uint64_t chosen = 0;
      uint32_t pos = skip > base ? skip - base : 0;
      while (pos < lim) {
        const uint64_t rest = M >> pos;
        uint32_t m = rest ? pos + (uint32_t)__builtin_ctzll(rest) : lim;
        if (m > lim) m = lim;
        chosen |= ((m >= 64 ? ~0ull : ((1ull << m) - 1)) & ~((1ull << pos) - 1));
        if (m >= lim) {
          pos = lim;
          break;
        }
        chosen |= 1ull << m;
        pos = m + (uint32_t)__builtin_amdgcn_readlane((int)mlen, (int)m);
      }
      skip = base + pos;
      if ((chosen >> lane) & 1) {
        const uint32_t idx = nsym + (uint32_t)__builtin_popcountll(chosen & ((1ull << lane) - 1));
        if (mlen >= 4) {
          syms[idx] = 0x80000000u | (mlen - 3) | ((dist - 1) << 8);
          uint32_t lc, le, lv, dc, de, dv;
          len_sym(mlen - 3, lc, le, lv);
          dist_sym(dist - 1, dc, de, dv);
          atomicAdd(&S.lfreq[lc], 1u);
          atomicAdd(&S.dfreq[dc], 1u);
        } else {
          syms[idx] = w4 & 0xff;
          atomicAdd(&S.lfreq[w4 & 0xff], 1u);
        }
      }
      nsym += (uint32_t)__builtin_popcountll(chosen);
      if (nsym > GZE_BLK_SYMS - 64) {
        WSYNC();
        emit_block(S, B, syms, nsym, in, blk0, skip, false);
        blk0 = skip;
        nsym = 0;
      }
    }
    WSYNC();
    if (nsym) {
      emit_block(S, B, syms, nsym, in, blk0, n, true);
    } else {  // an empty final block (fixed Huffman: the end-of-block code alone)
      maybe_flush(S, B);
      put(S, B, 1, 1);
      put(S, B, 1, 2);
      put(S, B, 0, 7);
    }
    // 4. trailer: CRC-32 and ISIZE, or the big-endian Adler-32; byte-aligned
    maybe_flush(S, B);
    B.bitpos = (B.bitpos + 7) & ~7u;
    if (zhdr) {
      put(S, B, __builtin_bswap32(crc), 32);
    } else {
      put(S, B, crc, 32);
      put(S, B, n, 32);
    }
    const uint64_t total_bits = (uint64_t)B.outw * 32 + B.bitpos;
    flush(S, B, true);
    if (lane == 0) {
      if (B.ovf) {
        status[item] = ZG_DECODED_SIZE_MISMATCH;
      } else {
        items[item].src = (uint64_t)(slot + GZE_HDR + (zhdr ? 8 : 0));
        items[item].len = (zhdr ? 2 : 10) + total_bits / 8;
      }
    }
    WSYNC();
  }
}

uint32_t gzip_encode_grid(uint32_t n_items) {
  return (uint32_t)std::min<uint64_t>(n_items, (uint64_t)device_cu_count() * 8);
}

hipError_t launch_gzip_encode(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *slots, uint64_t slot_bytes,
                              uint32_t *sym_scratch, int level, hipStream_t s, bool zlib) {
  if (!n_items) return hipSuccess;
  const uint32_t xfl = level <= 1 ? 4u : level >= 9 ? 2u : 0u;
  uint32_t zhdr = 0;
  if (zlib) {  // CMF 0x78 (deflate, 32 KiB window), FLEVEL as zlib's deflate sets it, FCHECK
    const uint32_t flevel = level < 0 ? 2u : level < 2 ? 0u : level < 6 ? 1u : level == 6 ? 2u : 3u;
    zhdr = 0x7800u | (flevel << 6);
    zhdr |= (31u - zhdr % 31u) % 31u;
  }
  hipLaunchKernelGGL(k_gzip_encode, dim3(gzip_encode_grid(n_items)), dim3(64), 0, s, items, status, n_items, slots,
                     slot_bytes, sym_scratch, xfl, zhdr);
  return hipGetLastError();
}

}  // namespace zgpu
