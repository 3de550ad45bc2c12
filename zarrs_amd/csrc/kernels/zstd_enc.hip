// zstd (RFC 8878) frame ENCODER on gfx950: the write half of the zstd codec (ZstdCodec::encode,
// zarrs/src/array/codec/bytes_to_bytes/zstd/zstd_codec.rs:100-111, zstd::bulk::Compressor). The output
// is one single-segment frame any zstd decoder reads (libzstd, zstd-sys, k_zstd*); its bytes are not
// libzstd's (match finding, block splitting and entropy tables are encoder choices).
//
// One 64-lane wave encodes one item, in superblocks of ZE_NB zstd blocks of ZE_BLK (64 KiB) input:
//   1. LZ77 over the superblock, 64 positions per step (the gzip encoder's scheme, deflate_enc.hip):
//      per lane a 4-byte hash bucket candidate (u32 positions: the window is the whole frame, offsets
//      below 2^29) and a match of up to 32 bytes; the greedy parse is a scalar walk over the ballot of
//      match-starting lanes, and a chosen match that reached 32 bytes is extended by the whole wave
//      (64 x 4 bytes per step). Matches never cross a block end. Chosen literals go to the block's
//      literal scratch, matches to its sequence scratch (literal length, match length, offset).
//   2. one lane per block: the block's sequences FSE-coded with the predefined distributions
//      (Symbol_Compression_Modes 0: no table descriptions), the tANS state chain walked backwards from
//      the last sequence as the format requires, into the lane's bitstream scratch.
//   3. the wave writes the blocks in order: each block's literals become a Huffman-compressed
//      literals section (RFC 8878 3.1.1.3.1 / 4.2.1: a length-limited code from the block's
//      histogram, its tree description as FSE-compressed or 4-bit weights, 1 or 4 streams placed
//      by a wave prefix sum of the code lengths through an LDS bit ring), an RLE section (one distinct
//      byte) or raw literals, whichever is smallest; the block is written compressed (literals +
//      sequences) or raw, whichever is smaller. The frame header first, the XXH64 content checksum
//      last when the codec asks for one. 64 KiB blocks keep the decoder's per-block work (k_zstd_*:
//      one Huffman table, one block record per block) to the libzstd frames' order of magnitude.
// The literal-section format is pinned on the CPU by tests/zstd_huf_model.py (a Python restatement
// of these steps whose frames libzstd decodes).
#include <hip/hip_runtime.h>

#include "../common.hpp"
#include "huff.hpp"
#include "launch.hpp"
#include "xxh.hpp"

namespace zgpu {
namespace {

constexpr uint32_t ZE_BLK = 65536;           // input bytes per zstd block
constexpr uint32_t ZE_NB = 8;                // blocks per superblock (one per lane in phase 2)
constexpr uint32_t ZE_SB = ZE_BLK * ZE_NB;   // superblock input bytes
constexpr uint32_t ZE_SEQ = ZE_BLK / 4;      // sequences per block at most (matches >= 4 bytes)
constexpr uint32_t ZE_BITW = ZE_SEQ * 77 / 32 + 16;  // bitstream scratch words per block (<= 77 bits a sequence)
constexpr uint32_t ZE_HBITS = 12, ZE_HSIZE = 1u << ZE_HBITS;
constexpr uint32_t ZE_MAXOFF = (1u << 29) - 4;  // offset + 3 within the predefined OF table (codes <= 28)
constexpr uint32_t ZE_CAP1 = 32;             // per-lane match search; longer chosen matches: the wave
constexpr uint64_t ZE_SCRATCH = (uint64_t)ZE_SB + (uint64_t)ZE_NB * ZE_SEQ * 8 + (uint64_t)ZE_NB * ZE_BITW * 4;
constexpr uint32_t HUF_MAXBITS = 11;         // Max_Number_of_Bits of a literals code (RFC 8878 4.2.1)
constexpr uint32_t HUF_WLOG = 6;             // accuracy log of the FSE-compressed weights
constexpr uint32_t HR_WORDS = 512;           // LDS bit ring of a Huffman stream being written (>= 1024 x 11 bits)

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
  uint32_t nlit[ZE_NB], nseq[ZE_NB], sbytes[ZE_NB];
  uint32_t next[64];
  // the literals section of the block being written
  uint32_t hfreq[256];
  uint32_t sfreq[4][256];  // per literal stream (4-stream sections)
  uint8_t hlen[256];
  uint16_t hcode[256];
  HuffScratch hs;
  uint32_t ring[HR_WORDS];
  uint8_t hdesc[136];  // tree description (<= 1 + 128 bytes)
  uint8_t wts[256];    // Huffman weights (tree description input)
  uint32_t hmisc[8];
  // FSE table of the weights (accuracy log 6, <= 13 symbols)
  uint8_t wsym[64], wnb[64];
  uint16_t wbase[64];
  uint8_t wenc[13][64];
  uint8_t wfirst[13];
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

struct BW8 {  // lane-serial forward bit writer into bytes, LSB first (k <= 24 bits a call)
  uint8_t *out;
  uint32_t n;
  uint64_t acc;
  uint32_t nb;
  __device__ void put(uint32_t v, uint32_t k) {
    acc |= (uint64_t)(v & ((1u << k) - 1u)) << nb;
    nb += k;
    while (nb >= 8) {
      out[n++] = (uint8_t)acc;
      acc >>= 8;
      nb -= 8;
    }
  }
  __device__ void close() {
    if (nb) out[n++] = (uint8_t)acc;
    acc = 0;
    nb = 0;
  }
  __device__ void close_backward() {  // end mark of a backward-read stream: a 1 bit, zero padding
    put(1, 1);
    close();
  }
};

// Normalised weight counts summing to 2^HUF_WLOG, every present symbol >= 1 (tests/zstd_huf_model.py
// fse_normalize)
__device__ void w_normalize(const uint32_t *counts, uint32_t nsym, int32_t *norm) {
  uint32_t total = 0;
  for (uint32_t s = 0; s < nsym; s++) total += counts[s];
  int32_t sum = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    norm[s] = counts[s] ? max(1, (int32_t)((counts[s] << HUF_WLOG) / total)) : 0;
    sum += norm[s];
  }
  int32_t diff = (1 << HUF_WLOG) - sum;
  while (diff) {
    int32_t best = -1;
    for (uint32_t t = 0; t < nsym; t++)
      if ((diff > 0 || norm[t] > 1) && (best < 0 || norm[t] > norm[best])) best = (int32_t)t;
    if (diff > 0) {
      norm[best] += diff;
      diff = 0;
    } else {
      const int32_t take = min(-diff, norm[best] - 1);
      norm[best] -= take;
      diff += take;
    }
  }
}

// FSE table description (RFC 8878 4.1.1; libzstd FSE_writeNCount; the model's fse_write_ncount)
__device__ void w_ncount(const int32_t *norm, uint32_t nsym, BW8 &w) {
  w.put(HUF_WLOG - 5, 4);
  int32_t remaining = (1 << HUF_WLOG) + 1, threshold = 1 << HUF_WLOG, nbits = HUF_WLOG + 1;
  uint32_t s = 0;
  bool prev0 = false;
  while (s < nsym && remaining > 1) {
    if (prev0) {
      uint32_t start = s;
      while (s < nsym && norm[s] == 0) s++;
      while (s >= start + 3) {
        start += 3;
        w.put(3, 2);
      }
      w.put(s - start, 2);
    }
    int32_t count = norm[s++];
    const int32_t mx = (2 * threshold - 1) - remaining;
    remaining -= count;
    count += 1;
    if (count >= threshold) count += mx;
    w.put((uint32_t)count, (uint32_t)(nbits - (count < mx ? 1 : 0)));
    prev0 = count == 1;
    while (remaining < threshold) {
      nbits--;
      threshold >>= 1;
    }
  }
  w.close();
}

// Huffman tree description of the code in S.hlen (lane 0; RFC 8878 4.2.1, libzstd HUF_writeCTable;
// the model's huf_description): weights maxb + 1 - len of symbols 0..max_sym-1 (max_sym's is
// implied), FSE-compressed when that is smaller, else 4-bit weights when max_sym <= 128. Returns the
// description's length in S.hdesc, 0 when neither form applies.
__device__ uint32_t huf_desc(ZeSmem &S, uint32_t maxb, uint32_t max_sym) {
  uint32_t counts[13];
  for (uint32_t k = 0; k < 13; k++) counts[k] = 0;
  for (uint32_t s = 0; s < max_sym; s++) {
    const uint32_t w = S.hlen[s] ? maxb + 1 - S.hlen[s] : 0u;
    S.wts[s] = (uint8_t)w;
    counts[w]++;
  }
  uint32_t distinct = 0, mxc = 0, last = 0;
  for (uint32_t k = 0; k < 13; k++)
    if (counts[k]) {
      distinct++;
      mxc = max(mxc, counts[k]);
      last = k;
    }
  if (distinct > 1 && mxc < max_sym) {
    int32_t norm[13];
    const uint32_t nsym = last + 1;
    w_normalize(counts, nsym, norm);
    BW8 w{S.hdesc + 1, 0, 0, 0};
    w_ncount(norm, nsym, w);
    // the weights' FSE table (FSE_buildDTable's spread) and its encoding view
    constexpr uint32_t size = 1u << HUF_WLOG, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
    uint32_t pos = 0, nxt[13];
    for (uint32_t s = 0; s < nsym; s++) {
      for (int32_t i = 0; i < norm[s]; i++) {
        S.wsym[pos] = (uint8_t)s;
        pos = (pos + step) & mask;
      }
      nxt[s] = (uint32_t)norm[s];
    }
    for (uint32_t u = 0; u < size; u++) {
      const uint32_t x = nxt[S.wsym[u]]++;
      const uint32_t nb = HUF_WLOG - (31 - __builtin_clz(x));
      S.wnb[u] = (uint8_t)nb;
      S.wbase[u] = (uint16_t)((x << nb) - size);
    }
    for (uint32_t u = size; u-- > 0;) S.wfirst[S.wsym[u]] = (uint8_t)u;
    for (uint32_t u = 0; u < size; u++)
      for (uint32_t x = S.wbase[u]; x < S.wbase[u] + (1u << S.wnb[u]); x++) S.wenc[S.wsym[u]][x] = (uint8_t)u;
    // two interleaved states (even / odd positions), the last two weights' states first
    const uint32_t N = max_sym;
    uint32_t X[2];
    X[(N - 1) & 1] = S.wfirst[S.wts[N - 1]];
    X[(N - 2) & 1] = S.wfirst[S.wts[N - 2]];
    for (int32_t k = (int32_t)N - 3; k >= 0; k--) {
      const uint32_t st = (uint32_t)k & 1u;
      const uint32_t u = S.wenc[S.wts[k]][X[st]];
      w.put(X[st] - S.wbase[u], S.wnb[u]);
      X[st] = u;
    }
    w.put(X[1], HUF_WLOG);
    w.put(X[0], HUF_WLOG);
    w.close_backward();
    const uint32_t comp = w.n;
    if (comp > 1 && comp < max_sym / 2 && comp < 128) {
      S.hdesc[0] = (uint8_t)comp;
      return comp + 1;
    }
  }
  if (max_sym <= 128) {
    S.hdesc[0] = (uint8_t)(127 + max_sym);
    for (uint32_t i = 0; i < max_sym; i += 2)
      S.hdesc[1 + i / 2] = (uint8_t)((S.wts[i] << 4) | (i + 1 < max_sym ? S.wts[i + 1] : 0u));
    return 1 + (max_sym + 1) / 2;
  }
  return 0;
}

// 16 bytes per lane per step, loads issued before use (byte loads of one step are independent, so
// they are in flight together instead of one L2 round trip per byte)
__device__ __forceinline__ void wave_copy(uint8_t *dst, const uint8_t *src, uint32_t n) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t q0 = 16 * lane; q0 < n; q0 += 1024) {
    uint8_t t[16];
#pragma unroll
    for (int k = 0; k < 16; k++) t[k] = q0 + k < n ? src[q0 + k] : 0;
#pragma unroll
    for (int k = 0; k < 16; k++)
      if (q0 + k < n) dst[q0 + k] = t[k];
  }
}

// One Huffman stream of the literals L[a, e) into dst, whose byte length is bits / 8 + 1: written
// last literal first (the backward reader meets L[a] first). Steps of 1024 codes: lane t takes 16
// consecutive write positions (one batch of byte loads), a wave prefix sum of the lanes' bit totals
// places them, and each lane ORs its 16 codes into an LDS bit ring whose complete bytes go out after
// every step.
__device__ void huf_emit(ZeSmem &S, const uint8_t *L, uint32_t a, uint32_t e, uint8_t *dst) {
  const uint32_t lane = threadIdx.x;
  for (uint32_t k = lane; k < HR_WORDS; k += 64) S.ring[k] = 0;
  WSYNC();
  uint32_t base = 0, flushed = 0, cleared = 0;
  const uint32_t m = e - a;
  for (uint32_t c0 = 0; c0 < m; c0 += 1024) {
    const uint32_t i0 = c0 + 16 * lane;  // write positions i0 .. i0 + 15: literals e-1-i
    uint8_t v[16];
#pragma unroll
    for (int k = 0; k < 16; k++) v[k] = i0 + k < m ? L[e - 1 - (i0 + k)] : 0;
    uint32_t mine = 0;
#pragma unroll
    for (int k = 0; k < 16; k++) mine += i0 + k < m ? S.hlen[v[k]] : 0u;
    uint32_t incl = mine;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if ((int)lane >= o) incl += u;
    }
    const uint32_t tot = __shfl(incl, 63, 64);
    uint32_t off = base + incl - mine;
#pragma unroll
    for (int k = 0; k < 16; k++) {
      if (i0 + k < m) {
        const uint32_t len = S.hlen[v[k]], code = S.hcode[v[k]];
        const uint32_t w = (off >> 5) % HR_WORDS, sh = off & 31;
        atomicOr(&S.ring[w], code << sh);
        if (sh + len > 32) atomicOr(&S.ring[(w + 1) % HR_WORDS], code >> (32 - sh));
        off += len;
      }
    }
    base += tot;
    WSYNC();
    const uint32_t upto = base >> 3;  // complete bytes
    for (uint32_t q = flushed + lane; q < upto; q += 64) dst[q] = (uint8_t)(S.ring[(q >> 2) % HR_WORDS] >> (8 * (q & 3)));
    flushed = upto;
    WSYNC();
    for (uint32_t wd = cleared + lane; wd < (upto >> 2); wd += 64) S.ring[wd % HR_WORDS] = 0;
    cleared = upto >> 2;
    WSYNC();
  }
  if (lane == 0) atomicOr(&S.ring[(base >> 5) % HR_WORDS], 1u << (base & 31));  // end mark
  WSYNC();
  const uint32_t end = (base >> 3) + 1;
  for (uint32_t q = flushed + lane; q < end; q += 64) dst[q] = (uint8_t)(S.ring[(q >> 2) % HR_WORDS] >> (8 * (q & 3)));
  WSYNC();
}

}  // namespace

// Segment-parallel frame encode. An item is cut into segments of ZE_SEG input bytes (whole blocks);
// every (item, segment) unit is one wave's work, so a few large chunks still fill the GPU. A
// segment's blocks are independent of the other segments' encoding: every block carries its own
// Huffman table and new offsets (no repeat codes), and its matches may reach back before the
// segment (the input is all resident; the hash table is warmed up with the ZE_WARM bytes before it).
//   k_zstd_encode_seg : unit u -> its blocks in unit scratch u (seg_len[u], ~0 on overflow)
//   k_zstd_xxh        : XXH64 of each item (checksum chains only), before the items are rewritten
//   k_zstd_frame      : unit u -> frame header (segment 0), its blocks copied after the previous
//                       segments' bytes, the checksum and the frame length (last segment)
//   k_zstd_items      : the items rewritten to the frames (after every unit has read its item)
constexpr uint32_t ZE_SEG = 2 * ZE_SB;                      // 1 MiB input per unit
// a segment's blocks at most (raw blocks: the input + 3 bytes a block), for items of at most max_len
__host__ __device__ inline uint64_t ze_segcap(uint64_t max_len) {
  const uint64_t seg = max_len < ZE_SEG ? max_len : ZE_SEG;
  return ((seg + ((seg + ZE_BLK - 1) / ZE_BLK + 1) * 3 + 256) + 255) & ~255ull;
}
constexpr uint32_t ZE_WARM = 16384;

__global__ __launch_bounds__(64) void k_zstd_encode_seg(const ZgItem *items, const uint32_t *status,
                                                        uint32_t n_items, uint32_t ups, uint8_t *scratch,
                                                        uint8_t *segout, uint32_t *seg_len, uint64_t segcap) {
  __shared__ ZeSmem S;
  const uint32_t lane = threadIdx.x;
  uint8_t *scr = scratch + (uint64_t)blockIdx.x * ZE_SCRATCH;
  uint8_t *lits = scr;                                                      // ZE_SB bytes
  uint64_t *seqs = (uint64_t *)(scr + ZE_SB);                               // ZE_NB * ZE_SEQ
  uint32_t *bits = (uint32_t *)(scr + ZE_SB + (uint64_t)ZE_NB * ZE_SEQ * 8);  // ZE_NB * ZE_BITW
  build_pre(S.ll, c_ll_norm, S.next);
  build_pre(S.ml, c_ml_norm, S.next);
  build_pre(S.of, c_of_norm, S.next);
  const uint64_t n_units = (uint64_t)n_items * ups;
  for (uint64_t u = blockIdx.x; u < n_units; u += gridDim.x) {
    const uint32_t item = (uint32_t)(u / ups), seg = (uint32_t)(u % ups);
    if (status[item]) continue;
    const ZgItem it = items[item];
    if (it.len >= 0xFFFFFFF0ull) continue;  // k_zstd_frame reports it
    const uint8_t *in = (const uint8_t *)it.src;
    const uint32_t n = (uint32_t)it.len;
    const uint32_t s0 = seg * ZE_SEG;
    if (s0 >= n && !(n == 0 && seg == 0)) continue;
    const uint32_t s1 = min(n, s0 + ZE_SEG);
    uint8_t *out = segout + u * segcap;
    const uint64_t cap = segcap;
    for (uint32_t k = lane; k < ZE_HSIZE; k += 64) S.head[k] = 0;
    WSYNC();
    // warm-up: the positions of the ZE_WARM bytes before the segment enter the hash table, in order
    for (uint32_t p0 = s0 > ZE_WARM ? s0 - ZE_WARM : 0u; p0 < s0; p0 += 64) {
      const uint32_t p = p0 + lane;
      if (p < s0 && p + 4 <= n) {
        const uint32_t h = (ld4(in + p) * 0x9E3779B1u) >> (32 - ZE_HBITS);
        S.head[h] = p + 1;
      }
      WSYNC();
    }
    uint64_t op = 0;
    bool ovf = false;
    uint32_t skip = s0;
    for (uint32_t sb0 = s0; sb0 < s1 || (s1 == s0 && sb0 == s0); sb0 += ZE_SB) {
      const uint32_t sb_len = min(ZE_SB, s1 - sb0);
      const uint32_t nblk = s1 > s0 ? (sb_len + ZE_BLK - 1) / ZE_BLK : 1;
      // ---- 1. LZ77 over the superblock's blocks
      for (uint32_t b = 0; b < nblk; b++) {
        const uint32_t b0 = sb0 + b * ZE_BLK, b1 = min(b0 + ZE_BLK, s1);
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
              const uint32_t mlim = min(b1 - pm, 65535u);  // a sequence record holds 16-bit lengths
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
      // ---- 2. one lane per block: the sequences' FSE bitstream
      if (lane < nblk) {
        const uint32_t ns = S.nseq[lane];
        S.sbytes[lane] = ns ? encode_seqs(S, seqs + lane * ZE_SEQ, ns, bits + lane * ZE_BITW) : 0u;
      }
      WSYNC();
      // ---- 3. the wave writes the blocks in order: literals section (Huffman / RLE / raw), sequences
      for (uint32_t b = 0; b < nblk && !ovf; b++) {
        const uint32_t b0 = sb0 + b * ZE_BLK;
        const uint32_t blen = s1 > s0 ? min(ZE_BLK, s1 - b0) : 0u;
        const uint32_t nl = S.nlit[b], ns = S.nseq[b], sbyt = S.sbytes[b];
        const uint8_t *L = lits + b * ZE_BLK;
        const bool last = s1 == n && sb0 + ZE_SB >= s1 && b == nblk - 1;
        // histograms per literal stream (4-stream cut at seg4) and of the block
        const uint32_t seg4 = (nl + 3) / 4;
        for (uint32_t k = lane; k < 4 * 256; k += 64) (&S.sfreq[0][0])[k] = 0;
        WSYNC();
        for (uint32_t q0 = 16 * lane; q0 < nl; q0 += 1024) {
          uint8_t v[16];
#pragma unroll
          for (int k = 0; k < 16; k++) v[k] = q0 + k < nl ? L[q0 + k] : 0;
#pragma unroll
          for (int k = 0; k < 16; k++) {
            const uint32_t q = q0 + k;
            if (q < nl) atomicAdd(&S.sfreq[(q >= seg4) + (q >= 2 * seg4) + (q >= 3 * seg4)][v[k]], 1u);
          }
        }
        WSYNC();
        uint32_t used = 0;
        for (uint32_t k = lane; k < 256; k += 64) {
          S.hfreq[k] = S.sfreq[0][k] + S.sfreq[1][k] + S.sfreq[2][k] + S.sfreq[3][k];
          used += S.hfreq[k] ? 1u : 0u;
        }
        used = huff_wave_sum(used);
        const uint32_t rh = nl <= 31 ? 1u : nl <= 4095 ? 2u : 3u;  // raw / RLE header (Size_Format)
        uint32_t lsec = rh + nl, ltype = 0;
        if (used == 1) {
          lsec = rh + 1;
          ltype = 1;
        }
        uint32_t dl = 0, nstr = 0, comp = 0, hh = 0, sf = 0, sb4[4] = {0, 0, 0, 0};
#ifdef ZE_NO_HUF
        if (false) {
#else
        if (used >= 2) {
#endif
          huff_lengths(S.hs, S.hfreq, 256, HUF_MAXBITS, S.hlen);
          if (lane == 0) {
            uint32_t maxb = 0, max_sym = 0;
            for (uint32_t v = 0; v < 256; v++)
              if (S.hlen[v]) {
                maxb = max(maxb, (uint32_t)S.hlen[v]);
                max_sym = v;
              }
            S.hmisc[0] = huf_desc(S, maxb, max_sym);
            uint32_t val = 0;  // prefix codes: from the longest length up, in symbol order
            for (uint32_t len = maxb; len >= 1; len--) {
              for (uint32_t v = 0; v < 256; v++)
                if (S.hlen[v] == len) S.hcode[v] = (uint16_t)val++;
              val >>= 1;
            }
          }
          WSYNC();
          dl = S.hmisc[0];
          if (dl) {
            // stream bit counts from the stream histograms
            uint32_t bs[4] = {0, 0, 0, 0};
            for (uint32_t k = lane; k < 256; k += 64)
              for (uint32_t t = 0; t < 4; t++) bs[t] += S.sfreq[t][k] * S.hlen[k];
            for (uint32_t t = 0; t < 4; t++) bs[t] = huff_wave_sum(bs[t]);
            nstr = 1;
            sb4[0] = (bs[0] + bs[1] + bs[2] + bs[3]) / 8 + 1;
            comp = dl + sb4[0];
            if (nl > 1023 || comp > 1023) {
              nstr = 4;
              comp = dl + 6;
              for (uint32_t t = 0; t < 4; t++) {
                sb4[t] = bs[t] / 8 + 1;
                comp += sb4[t];
              }
            }
            sf = nstr == 1 ? 0u : (nl <= 1023 && comp <= 1023) ? 1u : (nl <= 16383 && comp <= 16383) ? 2u : 3u;
            hh = sf <= 1 ? 3u : sf == 2 ? 4u : 5u;
            if (hh + comp < lsec) {
              lsec = hh + comp;
              ltype = 2;
            }
          }
        }
        const uint32_t shdr = ns == 0 ? 1u : ns < 128 ? 2u : ns < 0x7F00 ? 3u : 4u;
        const uint32_t content = lsec + shdr + sbyt;
        const bool cmp = content < blen;
        const uint32_t bsz = 3 + (cmp ? content : blen);
        if (op + bsz > cap) {
          ovf = true;
          break;
        }
        uint8_t *o = out + op;
#ifdef ZE_DEBUG
        if (lane == 0)
          printf("blk %u nl %u ns %u sbyt %u used %u lsec %u ltype %u content %u bsz %u op %llu cmp %d\n", b, nl, ns,
                 sbyt, used, lsec, ltype, content, bsz, (unsigned long long)op, (int)cmp);
#endif
        if (lane == 0) {
          const uint32_t hdr = (last ? 1u : 0u) | ((cmp ? 2u : 0u) << 1) | ((cmp ? content : blen) << 3);
          o[0] = (uint8_t)hdr;
          o[1] = (uint8_t)(hdr >> 8);
          o[2] = (uint8_t)(hdr >> 16);
        }
        o += 3;
        if (!cmp) {
          wave_copy(o, in + b0, blen);
        } else {
          if (ltype < 2) {  // raw / RLE literals
            if (lane == 0) {
              const uint32_t h = rh == 1 ? (ltype | (nl << 3)) : rh == 2 ? (ltype | (1u << 2) | (nl << 4))
                                                                       : (ltype | (3u << 2) | (nl << 4));
              for (uint32_t k = 0; k < rh; k++) o[k] = (uint8_t)(h >> (8 * k));
              if (ltype == 1) o[rh] = L[0];
            }
            if (ltype == 0) wave_copy(o + rh, L, nl);
          } else {  // Huffman: header, tree description, jump table, streams
            if (lane == 0) {
              const uint64_t h = 2u | (sf << 2) | ((uint64_t)nl << 4) |
                                 ((uint64_t)comp << (sf <= 1 ? 14 : sf == 2 ? 18 : 22));
              for (uint32_t k = 0; k < hh; k++) o[k] = (uint8_t)(h >> (8 * k));
              if (nstr == 4)
                for (uint32_t t = 0; t < 3; t++) {
                  o[hh + dl + 2 * t] = (uint8_t)sb4[t];
                  o[hh + dl + 2 * t + 1] = (uint8_t)(sb4[t] >> 8);
                }
            }
            for (uint32_t q = lane; q < dl; q += 64) o[hh + q] = S.hdesc[q];
            uint8_t *st = o + hh + dl + (nstr == 4 ? 6 : 0);
            const uint32_t seg = nstr == 4 ? (nl + 3) / 4 : nl;
            for (uint32_t t = 0; t < nstr; t++) {
              huf_emit(S, L, min(nl, t * seg), min(nl, (t + 1) * seg), st);
              st += sb4[t];
            }
          }
          uint8_t *q8 = o + lsec;
          if (lane == 0) {  // Number_of_Sequences, Symbol_Compression_Modes = 0 (predefined LL / OF / ML)
            if (ns < 128) {
              q8[0] = (uint8_t)ns;
            } else if (ns < 0x7F00) {
              q8[0] = (uint8_t)((ns >> 8) + 128);
              q8[1] = (uint8_t)ns;
            } else {
              q8[0] = 0xFF;
              q8[1] = (uint8_t)(ns - 0x7F00);
              q8[2] = (uint8_t)((ns - 0x7F00) >> 8);
            }
            if (ns) q8[shdr - 1] = 0;
          }
          wave_copy(q8 + shdr, (const uint8_t *)(bits + b * ZE_BITW), sbyt);
        }
        op += bsz;
        WSYNC();
      }
      if (ovf || s1 == s0) break;
    }
    if (lane == 0) seg_len[u] = ovf ? 0xFFFFFFFFu : (uint32_t)op;
    WSYNC();
  }
}

__global__ __launch_bounds__(64) void k_zstd_xxh(const ZgItem *items, const uint32_t *status, uint32_t n_items,
                                                 uint64_t *hash) {
  for (uint32_t item = blockIdx.x; item < n_items; item += gridDim.x) {
    if (status[item]) continue;
    const ZgItem it = items[item];
    const uint64_t h = xxh64((const uint8_t *)it.src, it.len);
    if (threadIdx.x == 0) hash[item] = h;
  }
}

__global__ __launch_bounds__(64) void k_zstd_frame(ZgItem *items, uint32_t *status, uint32_t n_items, uint32_t ups,
                                                   uint8_t *slots, uint64_t slot_bytes, const uint8_t *segout,
                                                   const uint32_t *seg_len, const uint64_t *hash, uint32_t checksum,
                                                   uint64_t *ftot, uint64_t segcap) {
  const uint32_t lane = threadIdx.x;
  const uint64_t u = blockIdx.x;
  const uint32_t item = (uint32_t)(u / ups), seg = (uint32_t)(u % ups);
  if (status[item]) return;
  const ZgItem it = items[item];
  if (it.len >= 0xFFFFFFF0ull) {
    if (seg == 0 && lane == 0) status[item] = ZG_UNSUPPORTED;
    return;
  }
  const uint32_t n = (uint32_t)it.len;
  const uint32_t nseg = n ? (n + ZE_SEG - 1) / ZE_SEG : 1u;
  if (seg >= nseg) return;
  // frame header: magic, descriptor (single segment, content size, checksum flag), content size
  const uint32_t fcs_flag = n <= 255 ? 0u : n <= 65535 + 256 ? 1u : 2u;
  const uint32_t fcs_len = fcs_flag == 0 ? 1 : fcs_flag == 1 ? 2 : 4;
  const uint32_t fcs_val = fcs_flag == 1 ? n - 256 : n;
  uint64_t before = 5 + fcs_len, total = 5 + fcs_len;
  bool ovf = false;
  for (uint32_t k = 0; k < nseg; k++) {
    const uint32_t l = seg_len[(uint64_t)item * ups + k];
    if (l == 0xFFFFFFFFu) ovf = true;
    if (k < seg) before += l;
    total += l;
  }
  if (checksum) total += 4;
  const uint64_t cap = slot_bytes - ZE_HDR - 8;
  if (ovf || total > cap) {
    if (seg == 0 && lane == 0) status[item] = ZG_DECODED_SIZE_MISMATCH;
    return;
  }
  uint8_t *out = slots + (uint64_t)item * slot_bytes + ZE_HDR;
  if (seg == 0 && lane < 5 + fcs_len) {
    uint8_t b;
    if (lane < 4) b = (uint8_t)(0xFD2FB528u >> (8 * lane));
    else if (lane == 4) b = (uint8_t)((fcs_flag << 6) | (1u << 5) | (checksum ? 4u : 0u));
    else b = (uint8_t)(fcs_val >> (8 * (lane - 5)));
    out[lane] = b;
  }
  wave_copy(out + before, segout + u * segcap, seg_len[u]);
  if (seg == nseg - 1 && lane == 0) {
    if (checksum) {
      const uint64_t h = hash[item];
      for (int k = 0; k < 4; k++) out[total - 4 + k] = (uint8_t)(h >> (8 * k));
    }
    ftot[item] = total;  // the items are rewritten by k_zstd_items: the other segments still read them
  }
}

__global__ void k_zstd_items(ZgItem *items, const uint32_t *status, uint32_t n_items, uint8_t *slots,
                             uint64_t slot_bytes, const uint64_t *ftot) {
  const uint32_t item = blockIdx.x * blockDim.x + threadIdx.x;
  if (item >= n_items || status[item]) return;
  items[item].src = (uint64_t)(slots + (uint64_t)item * slot_bytes + ZE_HDR);
  items[item].len = ftot[item];
}

uint64_t zstd_encode_scratch(uint32_t n_items, uint64_t max_len) {
  const uint64_t units = (uint64_t)n_items * ((max_len + ZE_SEG - 1) / ZE_SEG + (max_len == 0 ? 1 : 0));
  const uint64_t grid = std::min<uint64_t>(std::max<uint64_t>(units, 1), (uint64_t)device_cu_count() * 4);
  return grid * ZE_SCRATCH + units * ze_segcap(max_len) + units * 4 + (uint64_t)n_items * 16 + 256;
}

hipError_t launch_zstd_encode(ZgItem *items, uint32_t *status, uint32_t n_items, uint64_t max_len, uint8_t *slots,
                              uint64_t slot_bytes, uint8_t *scratch, int checksum, hipStream_t s) {
  if (!n_items) return hipSuccess;
  const uint32_t ups = (uint32_t)((max_len + ZE_SEG - 1) / ZE_SEG + (max_len == 0 ? 1 : 0));
  const uint64_t units = (uint64_t)n_items * ups;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(units, (uint64_t)device_cu_count() * 4);
  const uint64_t segcap = ze_segcap(max_len);
  uint8_t *segout = scratch + (uint64_t)grid * ZE_SCRATCH;
  uint32_t *seg_len = (uint32_t *)(segout + units * segcap);
  uint64_t *hash = (uint64_t *)(((uintptr_t)(seg_len + units) + 7) & ~(uintptr_t)7);
  hipLaunchKernelGGL(k_zstd_encode_seg, dim3(grid), dim3(64), 0, s, items, status, n_items, ups, scratch, segout,
                     seg_len, segcap);
  if (checksum)
    hipLaunchKernelGGL(k_zstd_xxh, dim3(std::min<uint32_t>(n_items, device_cu_count() * 4)), dim3(64), 0, s, items,
                       status, n_items, hash);
  uint64_t *ftot = hash + n_items;
  hipLaunchKernelGGL(k_zstd_frame, dim3((uint32_t)units), dim3(64), 0, s, items, status, n_items, ups, slots,
                     slot_bytes, segout, seg_len, hash, checksum ? 1u : 0u, ftot, segcap);
  hipLaunchKernelGGL(k_zstd_items, dim3((n_items + 255) / 256), dim3(256), 0, s, items, status, n_items, slots,
                     slot_bytes, ftot);
  return hipGetLastError();
}

}  // namespace zgpu
