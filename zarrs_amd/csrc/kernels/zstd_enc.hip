// zstd (RFC 8878) frame ENCODER on gfx950: the write half of the zstd codec (ZstdCodec::encode,
// zarrs/src/array/codec/bytes_to_bytes/zstd/zstd_codec.rs:100-111, zstd::bulk::Compressor). The output
// is one single-segment frame any zstd decoder reads (libzstd, zstd-sys, k_zstd*); its bytes are not
// libzstd's (match finding and block splitting are encoder choices).
//
// One 64-lane wave encodes one item, in superblocks of 64 zstd blocks of ZE_BLK input bytes:
//   1. LZ77 over the superblock, 64 positions per step (the gzip encoder's scheme, deflate_enc.hip):
//      per lane a 4-byte hash bucket candidate (u32 positions: the window is the whole frame, offsets
//      below 2^29) and a match of up to 32 bytes; the greedy parse is a scalar walk over the ballot of match-starting lanes, and a chosen
//      match that reached 32 bytes is extended by the whole wave (64 x 4 bytes per step). Matches never
//      cross a block end. Chosen literals go to the block's literal scratch, matches to its sequence
//      scratch (literal length, match length, offset), counted per block.
//   2. one lane per block: the block's sequences FSE-coded with the predefined distributions
//      (Symbol_Compression_Modes 0: no table descriptions), the tANS state chain walked backwards from
//      the last sequence as the format requires, into the lane's bitstream scratch; the block size from
//      its raw literals section, sequences section and bitstream (a raw block when that is not smaller).
//   3. the blocks' sizes prefix-summed over the wave, each lane writes its block (header, literals,
//      sequences) at its offset; the frame header first, the XXH64 content checksum last when the
//      codec asks for one.
#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "launch.hpp"
#include "xxh.hpp"

namespace zgpu {
namespace {

constexpr uint32_t ZE_BLK = 4096;            // input bytes per zstd block
constexpr uint32_t ZE_NB = 64;               // blocks per superblock (one per lane in phase 2)
constexpr uint32_t ZE_SB = ZE_BLK * ZE_NB;   // superblock input bytes
constexpr uint32_t ZE_SEQ = ZE_BLK / 4;      // sequences per block at most (matches >= 4 bytes)
constexpr uint32_t ZE_BITW = 2048;           // bitstream scratch words per block (61 bits x 1024 seqs)
constexpr uint32_t ZE_HBITS = 12, ZE_HSIZE = 1u << ZE_HBITS;
constexpr uint32_t ZE_MAXOFF = (1u << 29) - 4;  // offset + 3 within the predefined OF table (codes <= 28)
constexpr uint32_t ZE_CAP1 = 32;             // per-lane match search; longer chosen matches: the wave
constexpr uint64_t ZE_SCRATCH = (uint64_t)ZE_SB + (uint64_t)ZE_NB * ZE_SEQ * 8 + (uint64_t)ZE_NB * ZE_BITW * 4;

__constant__ int16_t c_ll_norm[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                      2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t c_ml_norm[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                      1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                      1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t c_of_norm[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                      1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ uint32_t c_llb[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,
                                   12, 13, 14, 15, 16, 18, 20,  22,  24,  28,  32,   40,
                                   48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t c_llx[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                  1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t c_mlb[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,   15,   16,
                                   17, 18, 19, 20, 21, 22, 23, 24, 25, 26,  27,  28,   29,   30,
                                   31, 32, 33, 34, 35, 37, 39, 41, 43, 47,  51,  59,   67,   83,
                                   99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t c_mlx[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                  0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                  2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

// one predefined FSE table, decoding view (state -> symbol, next-state base, bits) plus the encoding
// lookup (symbol, next state -> state) and each symbol's initial state
template <uint32_t LOG, uint32_t NSYM>
struct PreTab {
  uint8_t sym[1u << LOG];
  uint8_t nb[1u << LOG];
  uint16_t base[1u << LOG];
  uint8_t enc[NSYM][1u << LOG];
  uint8_t first[NSYM];
};

struct ZeSmem {
  uint32_t head[ZE_HSIZE];  // hash -> position + 1 of the last 4-byte string with that hash, 0 = empty
  PreTab<6, 36> ll;
  PreTab<6, 53> ml;
  PreTab<5, 29> of;
  uint32_t nlit[ZE_NB], nseq[ZE_NB];
  uint32_t next[64];
};

#define WSYNC() __syncthreads()

__device__ __forceinline__ uint32_t ld4(const uint8_t *p) {
  const uintptr_t a = (uintptr_t)p;
  const uint32_t *w = (const uint32_t *)(a & ~(uintptr_t)3);
  const uint32_t sh = (uint32_t)(a & 3);
  const uint32_t lo = w[0];
  const uint32_t hi = sh ? w[1] : 0u;
  return __builtin_amdgcn_alignbyte(hi, lo, sh);
}
__device__ __forceinline__ uint32_t highbit(uint32_t v) { return 31 - __builtin_clz(v); }

// FSE_buildDTable's spread and state table for a predefined distribution, then the encoding view
template <uint32_t LOG, uint32_t NSYM>
__device__ void build_pre(PreTab<LOG, NSYM> &T, const int16_t *norm, uint32_t *next) {
  constexpr uint32_t size = 1u << LOG, mask = size - 1;
  const uint32_t lane = threadIdx.x;
  if (lane == 0) {
    uint32_t high = size - 1;
    for (uint32_t s = 0; s < NSYM; s++)
      if (norm[s] == -1) T.sym[high--] = (uint8_t)s;
    const uint32_t step = (size >> 1) + (size >> 3) + 3;
    uint32_t pos = 0;
    for (uint32_t s = 0; s < NSYM; s++)
      for (int32_t i = 0; i < norm[s]; i++) {
        T.sym[pos] = (uint8_t)s;
        do {
          pos = (pos + step) & mask;
        } while (pos > high);
      }
    for (uint32_t s = 0; s < NSYM; s++) next[s] = norm[s] == -1 ? 1u : (uint32_t)norm[s];
    for (uint32_t u = 0; u < size; u++) {  // states of a symbol in increasing table position
      const uint32_t s = T.sym[u];
      const uint32_t nx = next[s]++;
      const uint32_t nb = LOG - highbit(nx);
      T.nb[u] = (uint8_t)nb;
      T.base[u] = (uint16_t)((nx << nb) - size);
    }
    for (uint32_t s = 0; s < NSYM; s++) T.first[s] = 0xFF;
    for (uint32_t u = size; u-- > 0;) T.first[T.sym[u]] = (uint8_t)u;
  }
  WSYNC();
  // encoding: state u (symbol s) is reached from every next state in [base, base + 2^nb)
  if (lane < size) {
    const uint32_t s = T.sym[lane], b = T.base[lane], n = 1u << T.nb[lane];
    for (uint32_t x = b; x < b + n; x++) T.enc[s][x] = (uint8_t)lane;
  }
  WSYNC();
}

__device__ __forceinline__ uint32_t ll_code(uint32_t ll) {
  if (ll < 16) return ll;
  if (ll >= 64) return highbit(ll) + 19;
  // 16..63: codes 16..24
  return ll < 24 ? 16 + ((ll - 16) >> 1) : ll < 32 ? 20 + ((ll - 24) >> 2) : ll < 48 ? 22 + ((ll - 32) >> 3) : 24;
}
__device__ __forceinline__ uint32_t ml_code(uint32_t ml) {
  const uint32_t b = ml - 3;
  if (b < 32) return b;
  if (b >= 128) return highbit(b) + 36;
  // 32..127: codes 32..42
  return b < 40 ? 32 + ((b - 32) >> 1) : b < 48 ? 36 + ((b - 40) >> 2) : b < 64 ? 38 + ((b - 48) >> 3)
         : b < 96 ? 40 + ((b - 64) >> 4) : 42;
}

struct BitW {  // one lane's forward bit writer into its word scratch
  uint64_t acc;
  uint32_t n, nw;
  uint32_t *w;
  __device__ __forceinline__ void put(uint32_t v, uint32_t k) {
    acc |= (uint64_t)v << n;
    n += k;
    if (n >= 32) {
      w[nw++] = (uint32_t)acc;
      acc >>= 32;
      n -= 32;
    }
  }
};

// block b of the superblock: the sequences' FSE bitstream (predefined tables) into the lane's words;
// returns its byte length
__device__ uint32_t encode_seqs(ZeSmem &S, const uint64_t *seqs, uint32_t nseq, uint32_t *words) {
  BitW W{0, 0, 0, words};
  auto codes = [&](uint64_t r, uint32_t &llc, uint32_t &mlc, uint32_t &ofc, uint32_t &ll, uint32_t &ml,
                   uint32_t &ob) {
    ll = (uint32_t)(r & 0xFFFF);
    ml = (uint32_t)((r >> 16) & 0xFFFF);
    ob = (uint32_t)(r >> 32) + 3;  // Offset_Value of a new offset
    llc = ll_code(ll);
    mlc = ml_code(ml);
    ofc = highbit(ob);
  };
  uint32_t llc, mlc, ofc, ll, ml, ob;
  codes(seqs[nseq - 1], llc, mlc, ofc, ll, ml, ob);
  uint32_t xl = S.ll.first[llc], xm = S.ml.first[mlc], xo = S.of.first[ofc];
  W.put(ll - c_llb[llc], c_llx[llc]);
  W.put(ml - c_mlb[mlc], c_mlx[mlc]);
  W.put(ob - (1u << ofc), ofc);
  for (int32_t k = (int32_t)nseq - 2; k >= 0; k--) {
    codes(seqs[k], llc, mlc, ofc, ll, ml, ob);
    // FSE_encodeSymbol: offsets, match lengths, literal lengths (the decoder updates LL, ML, OF)
    {
      const uint32_t u = S.of.enc[ofc][xo];
      W.put(xo - S.of.base[u], S.of.nb[u]);
      xo = u;
    }
    {
      const uint32_t u = S.ml.enc[mlc][xm];
      W.put(xm - S.ml.base[u], S.ml.nb[u]);
      xm = u;
    }
    {
      const uint32_t u = S.ll.enc[llc][xl];
      W.put(xl - S.ll.base[u], S.ll.nb[u]);
      xl = u;
    }
    W.put(ll - c_llb[llc], c_llx[llc]);
    W.put(ml - c_mlb[mlc], c_mlx[mlc]);
    W.put(ob - (1u << ofc), ofc);
  }
  // initial states (read first: LL, OF, ML), then the end mark
  W.put(xm, 6);
  W.put(xo, 5);
  W.put(xl, 6);
  W.put(1, 1);
  const uint32_t bytes = W.nw * 4 + (W.n + 7) / 8;
  if (W.n) W.w[W.nw] = (uint32_t)W.acc;
  return bytes;
}

}  // namespace

// items[i] {src,len} -> one zstd frame in slot i at ZE_HDR (headroom for crc32c codecs at the start);
// items rewritten to it. scratch: zstd_encode_grid(n) * zstd_encode_scratch() bytes.
__global__ __launch_bounds__(64) void k_zstd_encode(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *slots,
                                                    uint64_t slot_bytes, uint8_t *scratch, uint32_t checksum) {
  __shared__ ZeSmem S;
  const uint32_t lane = threadIdx.x;
  uint8_t *scr = scratch + (uint64_t)blockIdx.x * ZE_SCRATCH;
  uint8_t *lits = scr;                                                      // ZE_SB bytes
  uint64_t *seqs = (uint64_t *)(scr + ZE_SB);                               // ZE_NB * ZE_SEQ
  uint32_t *bits = (uint32_t *)(scr + ZE_SB + (uint64_t)ZE_NB * ZE_SEQ * 8);  // ZE_NB * ZE_BITW
  build_pre(S.ll, c_ll_norm, S.next);
  build_pre(S.ml, c_ml_norm, S.next);
  build_pre(S.of, c_of_norm, S.next);
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    if (status[item]) continue;
    const ZgItem it = items[item];
    if (it.len >= 0xFFFFFFF0ull) {
      if (lane == 0) status[item] = ZG_UNSUPPORTED;
      continue;
    }
    const uint8_t *in = (const uint8_t *)it.src;
    const uint32_t n = (uint32_t)it.len;
    uint8_t *out = slots + (uint64_t)item * slot_bytes + ZE_HDR;
    const uint64_t cap = slot_bytes - ZE_HDR - 8;
    for (uint32_t k = lane; k < ZE_HSIZE; k += 64) S.head[k] = 0;
    // frame header: magic, descriptor (single segment, content size, checksum flag), content size
    const uint32_t fcs_flag = n <= 255 ? 0u : n <= 65535 + 256 ? 1u : 2u;
    const uint32_t fcs_len = fcs_flag == 0 ? 1 : fcs_flag == 1 ? 2 : 4;
    const uint32_t fcs_val = fcs_flag == 1 ? n - 256 : n;
    if (lane < 5 + fcs_len) {
      uint8_t b;
      if (lane < 4) b = (uint8_t)(0xFD2FB528u >> (8 * lane));
      else if (lane == 4) b = (uint8_t)((fcs_flag << 6) | (1u << 5) | (checksum ? 4u : 0u));
      else b = (uint8_t)(fcs_val >> (8 * (lane - 5)));
      out[lane] = b;
    }
    uint64_t op = 5 + fcs_len;
    bool ovf = false;
    WSYNC();
    uint32_t skip = 0;
    for (uint32_t sb0 = 0; sb0 < n || (n == 0 && sb0 == 0); sb0 += ZE_SB) {
      const uint32_t sb_len = min(ZE_SB, n - sb0);
      const uint32_t nblk = n ? (sb_len + ZE_BLK - 1) / ZE_BLK : 1;
      // ---- 1. LZ77 over the superblock's blocks
      for (uint32_t b = 0; b < nblk; b++) {
        const uint32_t b0 = sb0 + b * ZE_BLK, b1 = min(b0 + ZE_BLK, n);
        uint32_t nl = 0, ns = 0, carry = 0;  // literals / sequences so far; literals since the last match
        uint8_t *blit = lits + b * ZE_BLK;
        uint64_t *bseq = seqs + b * ZE_SEQ;
        for (uint32_t base = b0; base < b1; base += 64) {
          if (skip >= base + 64) continue;
          const uint32_t p = base + lane;
          const bool hv = p + 4 <= n;
          uint32_t w4 = 0;
          if (hv) w4 = ld4(in + p);
          else if (p < n) w4 = in[p];
          const uint32_t h = (w4 * 0x9E3779B1u) >> (32 - ZE_HBITS);
          const uint32_t hvv = hv ? S.head[h] : 0u;
          WSYNC();
          if (hv) S.head[h] = p + 1;
          uint32_t mlen = 0, cand = 0;
          if (hvv && p >= skip && p + 4 <= b1) {
            cand = hvv - 1;  // < p; the window is the whole frame (single segment)
            if (p - cand <= ZE_MAXOFF && ld4(in + cand) == w4) {
              const uint32_t lim = min(ZE_CAP1, b1 - p);
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
            }
          }
          // greedy parse: scalar walk over the match-starting lanes; a match that reached the lane
          // search's cap is extended by the whole wave
          const uint32_t lim = min(64u, b1 - base);
          const uint64_t M = __ballot(mlen >= 4);
          uint64_t chosen = 0, cm = 0;
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
            cm |= 1ull << m;
            uint32_t L = (uint32_t)__builtin_amdgcn_readlane((int)mlen, (int)m);
            const uint32_t pm = base + m;
            if (L == ZE_CAP1 && b1 - pm > ZE_CAP1) {
              const uint32_t cnd = (uint32_t)__builtin_amdgcn_readlane((int)cand, (int)m);
              const uint32_t mlim = b1 - pm;
              for (uint32_t k0 = ZE_CAP1;; k0 += 256) {
                const uint32_t k = k0 + 4 * lane;
                uint32_t mis = 0xFFFFFFFFu;  // first mismatching offset this lane sees
                if (k < mlim) {
                  if (k + 4 <= mlim) {
                    const uint32_t x = ld4(in + pm + k) ^ ld4(in + cnd + k);
                    if (x) mis = k + ((uint32_t)__builtin_ctz(x) >> 3);
                  } else {
                    for (uint32_t q = k; q < mlim; q++)
                      if (in[pm + q] != in[cnd + q]) {
                        mis = q;
                        break;
                      }
                  }
                }
                const uint64_t bm = __ballot(mis != 0xFFFFFFFFu);
                if (bm) {
                  L = (uint32_t)__builtin_amdgcn_readlane((int)mis, (int)__builtin_ctzll(bm));
                  break;
                }
                if (k0 + 256 >= mlim) {
                  L = mlim;
                  break;
                }
              }
              if (lane == m) mlen = L;
            }
            pos = m + L;
          }
          skip = base + pos;
          const uint64_t lm = chosen & ~cm;
          const uint64_t lt = (1ull << lane) - 1;
          if ((lm >> lane) & 1) blit[nl + (uint32_t)__builtin_popcountll(lm & lt)] = (uint8_t)w4;
          if ((cm >> lane) & 1) {
            const uint64_t pmk = cm & lt;
            const uint32_t before = (uint32_t)__builtin_popcountll(lm & lt);
            uint32_t ll;
            if (pmk) {
              const uint32_t prev = 63 - (uint32_t)__builtin_clzll(pmk);
              ll = before - (uint32_t)__builtin_popcountll(lm & ((1ull << prev) - 1));
            } else {
              ll = carry + before;
            }
            bseq[ns + (uint32_t)__builtin_popcountll(pmk)] =
                (uint64_t)ll | ((uint64_t)mlen << 16) | ((uint64_t)(p - cand) << 32);
          }
          if (cm) {
            const uint32_t last = 63 - (uint32_t)__builtin_clzll(cm);
            carry = (uint32_t)__builtin_popcountll(lm >> last);
          } else {
            carry += (uint32_t)__builtin_popcountll(lm);
          }
          nl += (uint32_t)__builtin_popcountll(lm);
          ns += (uint32_t)__builtin_popcountll(cm);
        }
        if (lane == 0) {
          S.nlit[b] = nl;
          S.nseq[b] = ns;
        }
      }
      WSYNC();
      // ---- 2. one lane per block: sequences bitstream and the block's size
      uint32_t bsz = 0, kind = 0, nbytes = 0, nl = 0, ns = 0, blen = 0;
      if (lane < nblk) {
        const uint32_t b0 = sb0 + lane * ZE_BLK;
        blen = n ? min(ZE_BLK, n - b0) : 0;
        nl = S.nlit[lane];
        ns = S.nseq[lane];
        nbytes = ns ? encode_seqs(S, seqs + lane * ZE_SEQ, ns, bits + lane * ZE_BITW) : 0;
        const uint32_t shdr = ns == 0 ? 1 : ns < 128 ? 2 : ns < 0x7F00 ? 3 : 4;  // count (+ modes)
        const uint32_t content = 3 + nl + shdr + nbytes;
        kind = (ns && content < blen) ? 2u : 0u;  // compressed, else raw
        bsz = 3 + (kind == 2 ? content : blen);
      }
      uint32_t incl = bsz;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t u = __shfl_up(incl, o, 64);
        if ((int)lane >= o) incl += u;
      }
      const uint32_t total = __shfl(incl, 63, 64);
      if (op + total > cap) ovf = true;
      // ---- 3. every lane writes its block
      if (!ovf && lane < nblk) {
        uint8_t *o = out + op + (incl - bsz);
        const bool last = sb0 + ZE_SB >= n && lane == nblk - 1;
        const uint32_t bs = bsz - 3;
        const uint32_t hdr = (last ? 1u : 0u) | (kind << 1) | (bs << 3);
        o[0] = (uint8_t)hdr;
        o[1] = (uint8_t)(hdr >> 8);
        o[2] = (uint8_t)(hdr >> 16);
        o += 3;
        if (kind == 0) {
          const uint8_t *src = in + sb0 + lane * ZE_BLK;
          for (uint32_t q = 0; q < blen; q++) o[q] = src[q];
        } else {
          // raw literals section, 3-byte header (Size_Format 11: 20-bit Regenerated_Size)
          o[0] = (uint8_t)((3u << 2) | ((nl & 0xF) << 4));
          o[1] = (uint8_t)(nl >> 4);
          o[2] = (uint8_t)(nl >> 12);
          o += 3;
          const uint8_t *bl = lits + lane * ZE_BLK;
          for (uint32_t q = 0; q < nl; q++) o[q] = bl[q];
          o += nl;
          // sequences section: count, Symbol_Compression_Modes = 0 (predefined LL / OF / ML)
          if (ns < 128) {
            *o++ = (uint8_t)ns;
          } else if (ns < 0x7F00) {
            *o++ = (uint8_t)((ns >> 8) + 128);
            *o++ = (uint8_t)ns;
          } else {
            *o++ = 0xFF;
            *o++ = (uint8_t)(ns - 0x7F00);
            *o++ = (uint8_t)((ns - 0x7F00) >> 8);
          }
          *o++ = 0;
          const uint8_t *bw = (const uint8_t *)(bits + lane * ZE_BITW);
          for (uint32_t q = 0; q < nbytes; q++) o[q] = bw[q];
        }
      }
      op += total;
      WSYNC();
      if (n == 0) break;
    }
    if (checksum && !ovf) {
      const uint64_t h = xxh64(in, n);
      if (lane < 4) out[op + lane] = (uint8_t)(h >> (8 * lane));
      op += 4;
    }
    if (lane == 0) {
      if (ovf) {
        status[item] = ZG_DECODED_SIZE_MISMATCH;
      } else {
        items[item].src = (uint64_t)out;
        items[item].len = op;
      }
    }
    WSYNC();
  }
}

uint64_t zstd_encode_scratch() { return ZE_SCRATCH; }

uint32_t zstd_encode_grid(uint32_t n_items) {
  return (uint32_t)std::min<uint64_t>(n_items, (uint64_t)device_cu_count() * 4);
}

hipError_t launch_zstd_encode(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *slots, uint64_t slot_bytes,
                              uint8_t *scratch, int checksum, hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_zstd_encode, dim3(zstd_encode_grid(n_items)), dim3(64), 0, s, items, status, n_items, slots,
                     slot_bytes, scratch, checksum ? 1u : 0u);
  return hipGetLastError();
}

}  // namespace zgpu
