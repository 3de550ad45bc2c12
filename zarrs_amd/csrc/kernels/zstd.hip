// zstd frame decode (RFC 8878) for gfx950.
//
// Reference behaviour restated: zarrs/src/array/codec/bytes_to_bytes/zstd/zstd_codec.rs:113-130 —
// `zstd::bulk::decompress(encoded, ZSTD_decompressBound(encoded))` (zstd 0.13 / zstd-sys, libzstd
// 1.5): every frame of the input is decoded and the outputs concatenated; skippable frames are
// skipped; a frame's content checksum (XXH64, low 32 bits) is verified when present; dictionaries
// are not configured. Any error -> io::Error -> CodecError::IOError (ZG_CORRUPT_STREAM).
//
// Design (one 64-lane wavefront = one workgroup = one zstd item):
//  * Headers, FSE tables and the sequence bitstream are decoded by wave-uniform code (values in
//    SGPRs via readfirstlane); the backward bitstream is read through two 256-byte register windows.
//  * Huffman literals: the 4 streams are decoded by 4 lanes in parallel, each with its own backward
//    bit container, from an LDS decoding table (<= 11 bits); literals land in a per-item scratch.
//  * Sequences are decoded in batches of up to 64 (one per lane), then executed like the inflate
//    kernel: a wave scan places them, all literal runs of the batch are copied at once, each match is
//    copied by all lanes (out[p+i] = out[p-o+(i mod o)]), through a 16 KiB LDS ring of recent output;
//    older match sources are read back from the flushed output (zstd windows exceed the ring).
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../common.hpp"
#include "launch.hpp"

namespace zgpu {

#ifdef ZG_PROFILE
// lab builds only (tools/lab/zstd_lab.cpp): k_zstd_exec per-phase shader-clock totals
__device__ unsigned long long g_zprof[8];
#define ZP_DECL uint64_t zp_acc[8] = {0, 0, 0, 0, 0, 0, 0, 0}
#define ZP_T(v) const uint64_t v = clock64()
#define ZP_ADD(slot, t0) zp_acc[slot] += clock64() - (t0)
#define ZP_FLUSH do { if (__lane_id() == 0) for (int k_ = 0; k_ < 8; k_++) atomicAdd(&g_zprof[k_], (unsigned long long)zp_acc[k_]); } while (0)
#else
#define ZP_DECL
#define ZP_T(v)
#define ZP_ADD(slot, t0)
#define ZP_FLUSH
#endif

namespace {

constexpr int ZRING = 16384, ZRMASK = ZRING - 1;
constexpr int ZBATCH = 4096;         // max output span of one sequence batch
constexpr uint32_t ZBIG = 2048;      // sequences with a longer run are executed alone, chunked
constexpr uint32_t BLOCK_MAX = 131072;
constexpr uint32_t MAX_HUF_LOG = 12;
// per-item decode mode chosen by k_zstd_scan
constexpr uint32_t ZMODE_PARALLEL = 0, ZMODE_SERIAL = 1, ZMODE_SKIP = 2;

struct Fse {  // FSE decoding table entry
  uint16_t base;
  uint8_t sym;
  uint8_t nb;
};

struct ZSmem {
  uint8_t ring[ZRING];
  uint16_t huf[1 << MAX_HUF_LOG];  // (nb << 8) | sym
  Fse ll[512], ml[512], of[256], wt[64];
  int16_t norm[64];
  uint8_t weights[256];
  uint16_t hsorted[256];
  uint32_t pfx_lit[64], pfx_out[64];
  uint32_t tmp[32];
};

__constant__ int16_t c_ll_def[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                     2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
__constant__ int16_t c_ml_def[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
__constant__ int16_t c_of_def[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                     1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
__constant__ uint32_t c_ll_base[36] = {0,  1,  2,  3,  4,  5,  6,   7,   8,   9,   10,   11,
                                       12, 13, 14, 15, 16, 18, 20,  22,  24,  28,  32,   40,
                                       48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
__constant__ uint8_t c_ll_bits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,  0,  1,  1,
                                      1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
__constant__ uint32_t c_ml_base[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,   15,   16,
                                       17, 18, 19, 20, 21, 22, 23, 24, 25, 26,  27,  28,   29,   30,
                                       31, 32, 33, 34, 35, 37, 39, 41, 43, 47,  51,  59,   67,   83,
                                       99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
__constant__ uint8_t c_ml_bits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                      0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1,
                                      2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

__device__ __forceinline__ uint32_t U(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t U64(uint64_t x) {
  return (uint64_t)U((uint32_t)x) | ((uint64_t)U((uint32_t)(x >> 32)) << 32);
}
__device__ __forceinline__ int lane_id() { return __lane_id(); }
__device__ __forceinline__ uint32_t highbit(uint32_t v) { return 31 - __builtin_clz(v); }  // v > 0

// ---- uniform forward byte access (headers) ----
struct In {
  const uint8_t *p;
  uint64_t n;
  __device__ __forceinline__ uint32_t b(uint64_t i) const { return i < n ? U(p[i]) : 0u; }
  __device__ __forceinline__ uint32_t le16(uint64_t i) const { return b(i) | (b(i + 1) << 8); }
  __device__ __forceinline__ uint32_t le24(uint64_t i) const { return le16(i) | (b(i + 2) << 16); }
  __device__ __forceinline__ uint32_t le32(uint64_t i) const { return le24(i) | (b(i + 3) << 24); }
};

// ---- uniform backward bit reader over [lo, hi) bytes of the item input ----
// Bits are numbered as in a little-endian integer of the aligned item buffer; the stream's data
// bits are [lo_bit, top) where top is just below the padding marker of byte hi-1.
struct BitsBack {
  const uint32_t *words;  // aligned item base
  uint32_t nwords;
  int32_t wb;             // first word of the current window (wcur covers [wb, wb+64))
  uint32_t wcur, wprev;   // wprev covers [wb-64, wb)
  int64_t cur;            // next unread bit is cur-1
  int64_t lo_bit;
};

__device__ __forceinline__ uint32_t ldw(const BitsBack &R, int32_t k) {
  return (k >= 0 && (uint32_t)k < R.nwords) ? R.words[k] : 0u;
}
__device__ __forceinline__ uint32_t wget(const BitsBack &R, int32_t k) {
  const int32_t d = k - R.wb;
  if (d >= 0) return U(__builtin_amdgcn_readlane(R.wcur, d & 63));
  return U(__builtin_amdgcn_readlane(R.wprev, (d + 64) & 63));
}
// returns false if the last byte carries no padding marker
__device__ bool bb_init(BitsBack &R, const uint8_t *item, uint64_t item_len, uint64_t lo, uint64_t hi) {
  const uintptr_t mis = (uintptr_t)item & 3;
  R.words = (const uint32_t *)((uintptr_t)item - mis);
  R.nwords = (uint32_t)((item_len + mis + 3) / 4);
  const uint32_t last = hi > lo ? U(item[hi - 1]) : 0u;
  if (last == 0) return false;
  R.cur = (int64_t)(hi - 1 + mis) * 8 + highbit(last);
  R.lo_bit = (int64_t)(lo + mis) * 8;
  const int32_t kt = (int32_t)((R.cur >> 5));
  R.wb = kt - 62;
  R.wcur = ldw(R, R.wb + lane_id());
  R.wprev = ldw(R, R.wb - 64 + lane_id());
  return true;
}
// read n <= 32 bits (bits below lo_bit read as zero)
__device__ __forceinline__ uint32_t bb_read(BitsBack &R, uint32_t n) {
  if (n == 0) return 0;
  const int64_t lo = R.cur - n;
  R.cur = lo;
  if (lo + (int64_t)n <= R.lo_bit) return 0;
  const int64_t lo_c = lo < 0 ? 0 : lo;
  const int32_t k = (int32_t)(lo_c >> 5);
  const uint64_t w = (uint64_t)wget(R, k) | ((uint64_t)wget(R, k + 1) << 32);
  uint64_t v = w >> (lo_c & 31);
  uint32_t r = (uint32_t)(v & ((n == 32) ? 0xFFFFFFFFull : ((1ull << n) - 1)));
  if (lo < R.lo_bit) {  // clear the bits that lie below the stream start
    const int64_t z = R.lo_bit - lo;
    r = z >= 32 ? 0u : (r & ~((1u << z) - 1));
  }
  if (k < R.wb - 16) {  // slide the window pair down, prefetching the next lower window
    R.wb -= 64;
    R.wcur = R.wprev;
    R.wprev = ldw(R, R.wb - 64 + lane_id());
  }
  return r;
}
__device__ __forceinline__ bool bb_exact_end(const BitsBack &R) { return R.cur == R.lo_bit; }
__device__ __forceinline__ bool bb_overflow(const BitsBack &R) { return R.cur < R.lo_bit; }

// ---- FSE ----
// Parse an FSE table description (FSE_readNCount semantics). Returns bytes consumed, 0 on error.
__device__ uint32_t read_ncount(const In &I, uint64_t off, uint64_t avail, int16_t *norm, uint32_t max_sym,
                                uint32_t max_log, uint32_t &acc_log, uint32_t &nsym) {
  uint64_t bit = 0;
  auto peek32 = [&](uint64_t b) -> uint32_t {
    const uint64_t byte = off + (b >> 3);
    const uint64_t w = (uint64_t)I.le32(byte) | ((uint64_t)I.b(byte + 4) << 32);
    return (uint32_t)(w >> (b & 7));
  };
  uint32_t bs = peek32(0);
  acc_log = (bs & 15) + 5;
  if (acc_log > max_log) return 0;
  bit = 4;
  int remaining = (1 << acc_log) + 1;
  int threshold = 1 << acc_log;
  int nbBits = acc_log + 1;
  uint32_t s = 0;
  bool prev0 = false;
  for (uint32_t k = 0; k <= max_sym; k++) norm[k] = 0;
  while (remaining > 1 && s <= max_sym) {
    if (prev0) {
      uint32_t rep;
      for (;;) {
        rep = peek32(bit) & 3;
        bit += 2;
        if (rep != 3) break;
        s += 3;
        if (s > max_sym) return 0;
      }
      s += rep;
      if (s > max_sym) return 0;
    }
    bs = peek32(bit);
    const int maxv = (2 * threshold - 1) - remaining;
    int count;
    if ((int)(bs & (threshold - 1)) < maxv) {
      count = bs & (threshold - 1);
      bit += nbBits - 1;
    } else {
      count = bs & (2 * threshold - 1);
      if (count >= threshold) count -= maxv;
      bit += nbBits;
    }
    count--;
    remaining -= count < 0 ? -count : count;
    if (s > max_sym) return 0;
    norm[s++] = (int16_t)count;
    prev0 = (count == 0);
    if (remaining < threshold) {
      if (remaining <= 1) break;
      nbBits = (int)highbit((uint32_t)remaining) + 1;
      threshold = 1 << (nbBits - 1);
    }
  }
  if (remaining != 1 || s == 0) return 0;
  nsym = s;
  const uint64_t bytes = (bit + 7) >> 3;
  if (bytes > avail) return 0;
  return (uint32_t)bytes;
}

// Build an FSE decoding table from normalized counts (FSE_buildDTable).
__device__ void build_fse(Fse *T, const int16_t *norm, uint32_t nsym, uint32_t acc_log, uint32_t *tmp) {
  const uint32_t size = 1u << acc_log, mask = size - 1;
  const int lane = lane_id();
  // low-probability (-1) symbols at the top, then spread the others
  uint32_t high = size - 1;
  for (uint32_t s = 0; s < nsym; s++) {
    if (U((uint32_t)(int32_t)norm[s]) == 0xFFFFFFFFu) {
      if (lane == 0) {
        T[high].sym = (uint8_t)s;
      }
      high--;
    }
  }
  const uint32_t step = (size >> 1) + (size >> 3) + 3;
  uint32_t pos = 0;
  for (uint32_t s = 0; s < nsym; s++) {
    const int32_t c = (int32_t)U((uint32_t)(int32_t)norm[s]);
    for (int32_t i = 0; i < c; i++) {
      if (lane == 0) T[pos].sym = (uint8_t)s;
      do {
        pos = (pos + step) & mask;
      } while (pos > high);
    }
  }
  __syncthreads();
  // state info: lane s owns symbol s (nsym <= 64); symbols' next-state counters start at norm[s]
  // (1 for -1 symbols) and advance in increasing table position.
  uint32_t next = 0;
  if (lane < (int)nsym) {
    const int32_t c = norm[lane];
    next = c == -1 ? 1u : (uint32_t)c;
  }
  for (uint32_t u = 0; u < size; u++) {
    const uint32_t s = T[u].sym;
    if ((uint32_t)lane == s) {
      const uint32_t nb = acc_log - highbit(next);
      T[u].nb = (uint8_t)nb;
      T[u].base = (uint16_t)((next << nb) - size);
      next++;
    }
  }
  __syncthreads();
  (void)tmp;
}

__device__ void build_fse_rle(Fse *T, uint32_t sym) {
  if (lane_id() == 0) {
    T[0].sym = (uint8_t)sym;
    T[0].nb = 0;
    T[0].base = 0;
  }
  __syncthreads();
}

__device__ void build_fse_default(Fse *T, const int16_t *def, uint32_t nsym, uint32_t acc_log, int16_t *norm,
                                  uint32_t *tmp) {
  for (uint32_t s = lane_id(); s < nsym; s += 64) norm[s] = def[s];
  __syncthreads();
  build_fse(T, norm, nsym, acc_log, tmp);
}

// ---- Huffman (literals) ----
// Parse the tree description and build the decoding table. Returns bytes consumed, 0 on error.
template <class SM>
__device__ uint32_t read_huffman(const In &I, uint64_t off, uint64_t avail, SM &S, uint32_t &table_log,
                                 const uint8_t *item, uint64_t item_len) {
  const int lane = lane_id();
  if (avail < 1) return 0;
  const uint32_t hb = I.b(off);
  uint32_t nw = 0, used = 0;
  if (hb >= 128) {
    nw = hb - 127;
    used = 1 + (nw + 1) / 2;
    if (used > avail) return 0;
    for (uint32_t n = lane; n < nw; n += 64) {
      const uint32_t byte = item[off + 1 + n / 2];
      S.weights[n] = (uint8_t)((n & 1) ? (byte & 15) : (byte >> 4));
    }
    __syncthreads();
  } else {
    used = 1 + hb;
    if (used > avail || hb == 0) return 0;
    uint32_t acc, ns;
    const uint32_t h = read_ncount(I, off + 1, hb, S.norm, 15, 6, acc, ns);
    if (!h) return 0;
    __syncthreads();
    build_fse(S.wt, S.norm, ns, acc, S.tmp);
    BitsBack R;
    if (!bb_init(R, item, item_len, off + 1 + h, off + 1 + hb)) return 0;
    uint32_t s1 = bb_read(R, acc), s2 = bb_read(R, acc);
    // FSE_decompress tail semantics: alternate states until the stream overflows
    for (;;) {
      if (nw > 253) return 0;
      {
        const Fse e = S.wt[s1];
        const uint32_t sym = U(e.sym), nb = U(e.nb), base = U(e.base);
        if (lane == 0) S.weights[nw] = (uint8_t)sym;
        nw++;
        s1 = base + bb_read(R, nb);
      }
      if (bb_overflow(R)) {
        if (lane == 0) S.weights[nw] = U(S.wt[s2].sym);
        nw++;
        break;
      }
      {
        const Fse e = S.wt[s2];
        const uint32_t sym = U(e.sym), nb = U(e.nb), base = U(e.base);
        if (lane == 0) S.weights[nw] = (uint8_t)sym;
        nw++;
        s2 = base + bb_read(R, nb);
      }
      if (bb_overflow(R)) {
        if (lane == 0) S.weights[nw] = U(S.wt[s1].sym);
        nw++;
        break;
      }
    }
    __syncthreads();
  }
  // weights -> table log, implied last weight
  if (lane < 16) S.tmp[lane] = 0;
  __syncthreads();
  uint32_t wsum = 0;
  for (uint32_t n0 = 0; n0 < nw; n0 += 64) {
    const uint32_t n = n0 + lane;
    const uint32_t w = n < nw ? S.weights[n] : 0u;
    if (__ballot(w > MAX_HUF_LOG) != 0) return 0;
    uint32_t contrib = w ? (1u << w) >> 1 : 0u;
    for (int o = 32; o >= 1; o >>= 1) contrib += __shfl_xor(contrib, o, 64);
    wsum += U(contrib);
  }
  if (wsum == 0) return 0;
  const uint32_t tl = highbit(wsum) + 1;
  if (tl > MAX_HUF_LOG) return 0;
  const uint32_t rest = (1u << tl) - wsum;
  if (rest == 0 || (rest & (rest - 1))) return 0;
  const uint32_t last_w = highbit(rest) + 1;
  if (lane == 0) S.weights[nw] = (uint8_t)last_w;
  __syncthreads();
  const uint32_t nsym = nw + 1;
  // rank counts
  for (uint32_t n = lane; n < nsym; n += 64) {
    const uint32_t w = S.weights[n];
    if (w) atomicAdd(&S.tmp[w], 1u);
  }
  __syncthreads();
  uint32_t cnt[13];
  for (int w = 0; w < 13; w++) cnt[w] = w < 16 ? U(S.tmp[w]) : 0u;
  if (cnt[1] < 2 || (cnt[1] & 1)) return 0;
  uint32_t start[13], sbase[13];
  {
    uint32_t next = 0, sb = 0;
    for (uint32_t w = 1; w <= tl; w++) {
      start[w] = next;
      next += cnt[w] << (w - 1);
      sbase[w] = sb;
      sb += cnt[w];
    }
  }
  // symbols grouped by weight, ascending symbol order (ballot ranks)
  {
    uint32_t b[13];
    for (uint32_t w = 1; w <= tl; w++) b[w] = sbase[w];
    for (uint32_t n0 = 0; n0 < nsym; n0 += 64) {
      const uint32_t n = n0 + lane;
      const uint32_t w = n < nsym ? S.weights[n] : 0u;
      for (uint32_t W = 1; W <= tl; W++) {
        const uint64_t m = __ballot(w == W);
        if (w == W) S.hsorted[b[W] + __builtin_popcountll(m & ((1ull << lane) - 1))] = (uint16_t)n;
        b[W] += __builtin_popcountll(m);
      }
    }
  }
  __syncthreads();
  // fill: entries of weight class W occupy [start[W], start[W] + cnt[W] * 2^(W-1))
  const uint32_t size = 1u << tl;
  for (uint32_t e = lane; e < size; e += 64) {
    uint32_t W = 1;
    while (W < tl && e >= start[W + 1]) W++;
    const uint32_t len = 1u << (W - 1);
    const uint32_t sym = S.hsorted[sbase[W] + (e - start[W]) / len];
    S.huf[e] = (uint16_t)(((tl + 1 - W) << 8) | sym);
  }
  __syncthreads();
  table_log = tl;
  return used;
}

// Per-lane backward reader for one Huffman literal stream: c64 holds words [ck, ck+2) of the aligned
// item buffer; the next two lower words are prefetched so a step down never waits on memory.
struct LaneBits {
  const uint32_t *words;
  uint32_t nwords;
  int64_t cur, lo_bit;
  int32_t ck;
  uint64_t c64;
  uint32_t nx1, nx2;  // words ck-1, ck-2
};

__device__ __forceinline__ uint32_t lw(const LaneBits &L, int32_t k) {
  return (k >= 0 && (uint32_t)k < L.nwords) ? L.words[k] : 0u;
}
__device__ __forceinline__ void lane_bits_init(LaneBits &L) {
  L.ck = (int32_t)((L.cur - 1) >> 5) - 1;
  if (L.ck < 0) L.ck = 0;
  L.c64 = (uint64_t)lw(L, L.ck) | ((uint64_t)lw(L, L.ck + 1) << 32);
  L.nx1 = lw(L, L.ck - 1);
  L.nx2 = lw(L, L.ck - 2);
}
// bits [cur-n, cur) as an integer (MSB = bit cur-1), zeros below lo_bit; n <= 12
__device__ __forceinline__ uint32_t lane_peek(LaneBits &L, uint32_t n) {
  int64_t lo = L.cur - n;
  uint32_t shift_up = 0;
  if (lo < L.lo_bit) {
    const int64_t have = L.cur - L.lo_bit;
    if (have <= 0) return 0;
    shift_up = (uint32_t)(n - have);
    n = (uint32_t)have;
    lo = L.lo_bit;
  }
  const int32_t k = (int32_t)(lo >> 5);
  while (k < L.ck) {  // step the 64-bit container down one word
    L.c64 = (L.c64 << 32) | L.nx1;
    L.ck--;
    L.nx1 = L.nx2;
    L.nx2 = lw(L, L.ck - 2);
  }
  const uint32_t v = (uint32_t)(L.c64 >> (lo - (int64_t)L.ck * 32)) & ((1u << n) - 1);
  return v << shift_up;
}

// ---- XXH64 (content checksum), 4 lanes = the 4 accumulators ----
constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                   P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
__device__ __forceinline__ uint64_t rotl64(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
__device__ __forceinline__ uint64_t xround(uint64_t acc, uint64_t in) {
  acc += in * P2;
  acc = rotl64(acc, 31);
  return acc * P1;
}
__device__ __forceinline__ uint64_t ld64(const uint8_t *p) {
  uint64_t v = 0;
  for (int i = 0; i < 8; i++) v |= (uint64_t)__builtin_nontemporal_load(p + i) << (8 * i);
  return v;
}
__device__ uint64_t xxh64(const uint8_t *p, uint64_t len) {
  const int lane = lane_id();
  uint64_t h;
  uint64_t off = 0;
  if (len >= 32) {
    uint64_t v = lane == 0 ? P1 + P2 : lane == 1 ? P2 : lane == 2 ? 0 : 0 - P1;
    const uint64_t nst = len / 32;
    if (lane < 4)
      for (uint64_t s = 0; s < nst; s++) v = xround(v, ld64(p + s * 32 + lane * 8));
    auto rl = [&](int l) -> uint64_t {
      return (uint64_t)U(__builtin_amdgcn_readlane((uint32_t)v, l)) |
             ((uint64_t)U(__builtin_amdgcn_readlane((uint32_t)(v >> 32), l)) << 32);
    };
    const uint64_t v1 = rl(0), v2 = rl(1), v3 = rl(2), v4 = rl(3);
    h = rotl64(v1, 1) + rotl64(v2, 7) + rotl64(v3, 12) + rotl64(v4, 18);
    const uint64_t vs[4] = {v1, v2, v3, v4};
    for (int k = 0; k < 4; k++) {
      h ^= xround(0, vs[k]);
      h = h * P1 + P4;
    }
    off = nst * 32;
  } else {
    h = P5;
  }
  h += len;
  while (off + 8 <= len) {
    h ^= xround(0, U64(ld64(p + off)));
    h = rotl64(h, 27) * P1 + P4;
    off += 8;
  }
  if (off + 4 <= len) {
    uint64_t w = 0;
    for (int i = 0; i < 4; i++) w |= (uint64_t)U(__builtin_nontemporal_load(p + off + i)) << (8 * i);
    h ^= w * P1;
    h = rotl64(h, 23) * P2 + P3;
    off += 4;
  }
  while (off < len) {
    h ^= (uint64_t)U(__builtin_nontemporal_load(p + off)) * P5;
    h = rotl64(h, 11) * P1;
    off++;
  }
  h ^= h >> 33;
  h *= P2;
  h ^= h >> 29;
  h *= P3;
  h ^= h >> 32;
  return h;
}

// ---- output engine: LDS ring + flush to the item slot ----
struct Out {
  uint8_t *out;
  uint64_t cap;
  uint64_t pos;      // bytes produced
  uint64_t flushed;  // bytes in the slot
  bool dirty;        // flushed stores not yet fenced for this wave's loads
};

template <class SM>
__device__ __forceinline__ void out_flush(SM &S, Out &O) {
  __syncthreads();
  // the partial 16-B word at `flushed` is written byte by byte: the bytes before `flushed` may
  // belong to someone else (k_zstd_exec_blocks writes neighbouring blocks concurrently)
  const uint64_t a = (O.flushed + 15) & ~(uint64_t)15, b = (O.pos + 15) & ~(uint64_t)15;
  for (uint64_t q = O.flushed + lane_id(); q < a && q < O.pos; q += 64) O.out[q] = S.ring[q & ZRMASK];
  for (uint64_t p = a + (uint64_t)lane_id() * 16; p < b; p += 64 * 16) {
    if (p + 16 <= O.cap) {
      *(uint4 *)(O.out + p) = *(const uint4 *)&S.ring[p & ZRMASK];
    } else {
      for (uint64_t q = p; q < O.cap && q < p + 16; q++) O.out[q] = S.ring[q & ZRMASK];
    }
  }
  O.flushed = O.pos;
  O.dirty = true;
  __syncthreads();
}
// make room for n more bytes in the ring (n <= ZBATCH)
template <class SM>
__device__ __forceinline__ void out_reserve(SM &S, Out &O, uint64_t n) {
  if (O.pos + n > O.flushed + ZRING - 1024) out_flush(S, O);
}
__device__ __forceinline__ void out_fence(Out &O) {
  if (O.dirty) {
    __threadfence_block();
    O.dirty = false;
  }
}
template <class SM>
__device__ __forceinline__ uint8_t src_byte(SM &S, const Out &O, uint64_t s, uint64_t wend) {
  if (s + ZRING >= wend) return S.ring[s & ZRMASK];
  // flushed output of this wave: an sc1 load (bypasses L1) after out_fence
  const uint32_t *w = (const uint32_t *)((uintptr_t)(O.out + s) & ~(uintptr_t)3);
  return (uint8_t)(__hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) >> (8 * ((uintptr_t)(O.out + s) & 3)));
}
typedef unsigned int zv4u __attribute__((ext_vector_type(4)));
// Copy n <= ZBATCH bytes of global memory into LDS bytes dst[(pos + k) & mask] with 16-byte loads,
// every load issued before the first LDS write (a byte loop would pay the memory latency per step).
// The aligned 16-B blocks never extend past the 16-B block holding the last wanted byte.
__device__ __forceinline__ void lds_copy_in(uint8_t *dst, uint64_t mask, uint64_t pos, const uint8_t *src,
                                            uint32_t n) {
  const uintptr_t base = (uintptr_t)src & ~(uintptr_t)15;
  const uint32_t head = (uint32_t)((uintptr_t)src - base);
  const uint32_t nvec = (head + n + 15) >> 4;  // <= 257 for n <= 4096
  constexpr int R = ZBATCH / 16 / 64 + 1;
  zv4u v[R];
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t idx = lane_id() + 64 * r;
    if (idx < nvec) v[r] = __builtin_nontemporal_load((const zv4u *)(base + 16ull * idx));
  }
#pragma unroll
  for (int r = 0; r < R; r++) {
    const uint32_t idx = lane_id() + 64 * r;
    if (idx < nvec) {
      const uint32_t w[4] = {v[r].x, v[r].y, v[r].z, v[r].w};
#pragma unroll
      for (int j = 0; j < 16; j++) {
        const int32_t k = (int32_t)(16 * idx + j) - (int32_t)head;
        if (k >= 0 && (uint32_t)k < n) dst[(pos + (uint32_t)k) & mask] = (uint8_t)(w[j >> 2] >> (8 * (j & 3)));
      }
    }
  }
}

// copy n bytes from global memory (raw block / literals) to the output
template <class SM>
__device__ void out_copy_global(SM &S, Out &O, const uint8_t *src, uint64_t n) {
  for (uint64_t done = 0; done < n;) {
    const uint64_t c = min<uint64_t>(n - done, ZBATCH);
    out_reserve(S, O, c);
    lds_copy_in(S.ring, ZRMASK, O.pos, src + done, (uint32_t)c);
    O.pos += c;
    done += c;
  }
}
template <class SM>
__device__ void out_rle(SM &S, Out &O, uint8_t v, uint64_t n) {
  for (uint64_t done = 0; done < n;) {
    const uint64_t c = min<uint64_t>(n - done, ZBATCH);
    out_reserve(S, O, c);
    for (uint64_t k = lane_id(); k < c; k += 64) S.ring[(O.pos + k) & ZRMASK] = v;
    O.pos += c;
    done += c;
  }
}
// match of length n at distance d (d <= pos - frame_start, checked by the caller)
template <class SM>
__device__ void out_match(SM &S, Out &O, uint32_t d, uint64_t n) {
  const uint64_t p = O.pos;
  const float inv = 1.0f / (float)d;
  for (uint64_t done = 0; done < n;) {
    const uint64_t c = min<uint64_t>(n - done, ZBATCH);
    out_reserve(S, O, c);
    const uint64_t wend = O.pos + c;
    if (U(__ballot(p - d + ZRING < wend) != 0)) out_fence(O);
    for (uint64_t k = lane_id(); k < c; k += 64) {
      const uint64_t i = done + k;
      uint64_t rm;
      if (d >= n) {
        rm = i;
      } else if (i < 1u << 20) {
        uint32_t q = (uint32_t)((float)i * inv);
        int64_t r = (int64_t)i - (int64_t)q * d;
        while (r < 0) r += d;
        while (r >= d) r -= d;
        rm = (uint64_t)r;
      } else {
        rm = i % d;
      }
      S.ring[(p + i) & ZRMASK] = src_byte(S, O, p - d + rm, wend);
    }
    O.pos += c;
    done += c;
  }
}

}  // namespace

// One wave per item. lit: per-item literal scratch (BLOCK_MAX + 64 bytes each).
__global__ __launch_bounds__(64) void k_zstd(ZgItem *items, uint32_t *status, uint8_t *dst, uint64_t slot_bytes,
                                             uint8_t *lit_scratch, uint64_t lit_stride, const uint32_t *zmode) {
  __shared__ ZSmem S;
  const uint32_t item = blockIdx.x;
  const ZgItem it = items[item];
  if (status[item] || (it.flags & ZG_ITEM_FILL)) return;
  if (zmode && zmode[item] != ZMODE_SERIAL) return;  // decoded by the block-parallel path
  const int lane = lane_id();
  const uint8_t *in = (const uint8_t *)it.src;
  const In I{in, it.len};
  Out O{dst + (uint64_t)item * slot_bytes, slot_bytes, 0, 0, false};
  uint8_t *lit = lit_scratch + (uint64_t)item * lit_stride;
  uint32_t err = 0;
  uint64_t ip = 0;
  bool any_frame = false;
#define ZFAIL(code)   \
  {                   \
    err = (code);     \
    break;            \
  }
  while (!err && ip < it.len) {
    const uint32_t magic = I.le32(ip);
    if (ip + 4 > it.len) ZFAIL(ZG_CORRUPT_STREAM);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (ip + 8 > it.len) ZFAIL(ZG_CORRUPT_STREAM);
      const uint64_t sz = I.le32(ip + 4);
      ip += 8 + sz;
      if (ip > it.len) ZFAIL(ZG_CORRUPT_STREAM);
      continue;
    }
    if (magic != 0xFD2FB528u) ZFAIL(ZG_CORRUPT_STREAM);
    ip += 4;
    any_frame = true;
    const uint32_t fhd = I.b(ip++);
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, has_ck = (fhd >> 2) & 1, did_flag = fhd & 3;
    if (fhd & 8) ZFAIL(ZG_CORRUPT_STREAM);  // reserved bit
    if (!single) ip++;                      // window descriptor
    const uint32_t did_sz = did_flag == 3 ? 4 : did_flag;
    uint32_t did = 0;
    for (uint32_t k = 0; k < did_sz; k++) did |= I.b(ip + k) << (8 * k);
    ip += did_sz;
    if (did != 0) ZFAIL(ZG_CORRUPT_STREAM);  // no dictionary configured
    const uint32_t fcs_sz = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
    uint64_t fcs = 0;
    for (uint32_t k = 0; k < fcs_sz; k++) fcs |= (uint64_t)I.b(ip + k) << (8 * k);
    if (fcs_sz == 2) fcs += 256;
    ip += fcs_sz;
    if (ip > it.len) ZFAIL(ZG_CORRUPT_STREAM);
    if (fcs_sz && O.pos + fcs > O.cap) ZFAIL(ZG_DECODED_SIZE_MISMATCH);
    const uint64_t frame_start = O.pos;
    uint32_t rep0 = 1, rep1 = 4, rep2 = 8;
    bool have_huf = false, have_ll = false, have_ml = false, have_of = false;
    uint32_t huf_log = 0, ll_log = 0, ml_log = 0, of_log = 0;
    bool last = false;
    while (!last && !err) {
      if (ip + 3 > it.len) ZFAIL(ZG_CORRUPT_STREAM);
      const uint32_t bh = I.le24(ip);
      ip += 3;
      last = bh & 1;
      const uint32_t btype = (bh >> 1) & 3, bsize = bh >> 3;
      if (btype == 3) ZFAIL(ZG_CORRUPT_STREAM);
      if (btype == 0) {  // raw
        if (ip + bsize > it.len) ZFAIL(ZG_CORRUPT_STREAM);
        if (O.pos + bsize > O.cap) ZFAIL(ZG_DECODED_SIZE_MISMATCH);
        out_copy_global(S, O, in + ip, bsize);
        ip += bsize;
        continue;
      }
      if (btype == 1) {  // RLE
        if (ip + 1 > it.len) ZFAIL(ZG_CORRUPT_STREAM);
        if (O.pos + bsize > O.cap) ZFAIL(ZG_DECODED_SIZE_MISMATCH);
        out_rle(S, O, (uint8_t)I.b(ip), bsize);
        ip += 1;
        continue;
      }
      // ---- compressed block ----
      if (bsize > BLOCK_MAX || ip + bsize > it.len) ZFAIL(ZG_CORRUPT_STREAM);
      const uint64_t bend = ip + bsize;
      uint64_t p = ip;
      // literals section header
      const uint32_t b0 = I.b(p);
      const uint32_t ltype = b0 & 3, sfmt = (b0 >> 2) & 3;
      uint32_t regen = 0, csize = 0, lhdr = 0, nstreams = 1;
      if (ltype <= 1) {
        if (sfmt == 0 || sfmt == 2) { regen = b0 >> 3; lhdr = 1; }
        else if (sfmt == 1) { regen = (b0 >> 4) | (I.b(p + 1) << 4); lhdr = 2; }
        else { regen = (b0 >> 4) | (I.b(p + 1) << 4) | (I.b(p + 2) << 12); lhdr = 3; }
      } else {
        nstreams = sfmt == 0 ? 1 : 4;
        if (sfmt <= 1) {
          const uint32_t v = I.le24(p);
          regen = (v >> 4) & 0x3FF; csize = (v >> 14) & 0x3FF; lhdr = 3;
        } else if (sfmt == 2) {
          const uint32_t v = I.le32(p);
          regen = (v >> 4) & 0x3FFF; csize = (v >> 18) & 0x3FFF; lhdr = 4;
        } else {
          const uint64_t v = (uint64_t)I.le32(p) | ((uint64_t)I.b(p + 4) << 32);
          regen = (uint32_t)(v >> 4) & 0x3FFFF; csize = (uint32_t)(v >> 22) & 0x3FFFF; lhdr = 5;
        }
      }
      if (regen > BLOCK_MAX) ZFAIL(ZG_CORRUPT_STREAM);
      p += lhdr;
      const uint8_t *lsrc = lit;
      if (ltype == 0) {
        if (p + regen > bend) ZFAIL(ZG_CORRUPT_STREAM);
        lsrc = in + p;
        p += regen;
      } else if (ltype == 1) {
        if (p + 1 > bend) ZFAIL(ZG_CORRUPT_STREAM);
        const uint8_t v = (uint8_t)I.b(p);
        for (uint32_t k = lane; k < regen; k += 64) lit[k] = v;
        p += 1;
        __threadfence_block();
      } else {
        if (p + csize > bend) ZFAIL(ZG_CORRUPT_STREAM);
        uint64_t q = p;
        if (ltype == 2) {
          const uint32_t used = read_huffman(I, q, csize, S, huf_log, in, it.len);
          if (!used) ZFAIL(ZG_CORRUPT_STREAM);
          have_huf = true;
          q += used;
        } else if (!have_huf) {
          ZFAIL(ZG_CORRUPT_STREAM);  // treeless without a previous table
        }
        const uint64_t send = p + csize;
        // stream bounds
        uint64_t s_lo[4], s_hi[4];
        uint32_t s_n[4];
        if (nstreams == 1) {
          s_lo[0] = q; s_hi[0] = send; s_n[0] = regen;
        } else {
          if (q + 6 > send) ZFAIL(ZG_CORRUPT_STREAM);
          const uint32_t l1 = I.le16(q), l2 = I.le16(q + 2), l3 = I.le16(q + 4);
          const uint64_t b = q + 6;
          if (b + l1 + l2 + l3 > send) ZFAIL(ZG_CORRUPT_STREAM);
          s_lo[0] = b; s_hi[0] = b + l1;
          s_lo[1] = s_hi[0]; s_hi[1] = s_lo[1] + l2;
          s_lo[2] = s_hi[1]; s_hi[2] = s_lo[2] + l3;
          s_lo[3] = s_hi[2]; s_hi[3] = send;
          const uint32_t seg = (regen + 3) / 4;
          if (3 * seg > regen) ZFAIL(ZG_CORRUPT_STREAM);
          s_n[0] = s_n[1] = s_n[2] = seg;
          s_n[3] = regen - 3 * seg;
        }
        // lanes 0..nstreams-1 decode their stream
        uint32_t bad = 0;
        if (lane < (int)nstreams) {
          const uint64_t lo = lane == 0 ? s_lo[0] : lane == 1 ? s_lo[1] : lane == 2 ? s_lo[2] : s_lo[3];
          const uint64_t hi = lane == 0 ? s_hi[0] : lane == 1 ? s_hi[1] : lane == 2 ? s_hi[2] : s_hi[3];
          const uint32_t ns = lane == 0 ? s_n[0] : lane == 1 ? s_n[1] : lane == 2 ? s_n[2] : s_n[3];
          uint32_t out0 = 0;
          if (nstreams == 4) out0 = lane * ((regen + 3) / 4);
          const uintptr_t mis = (uintptr_t)in & 3;
          LaneBits L;
          L.words = (const uint32_t *)((uintptr_t)in - mis);
          L.nwords = (uint32_t)((it.len + mis + 3) / 4);
          const uint32_t lastb = hi > lo ? in[hi - 1] : 0u;
          if (lastb == 0) {
            bad = 1;
          } else {
            L.cur = (int64_t)(hi - 1 + mis) * 8 + (31 - __builtin_clz(lastb));
            L.lo_bit = (int64_t)(lo + mis) * 8;
            lane_bits_init(L);
            const uint32_t tl = huf_log;
            for (uint32_t k = 0; k < ns; k++) {
              const uint32_t idx = lane_peek(L, tl);
              const uint32_t e = S.huf[idx];
              L.cur -= e >> 8;
              lit[out0 + k] = (uint8_t)e;
              if (L.cur < L.lo_bit) { bad = 1; break; }
            }
            if (L.cur != L.lo_bit) bad = 1;
          }
        }
        if (U(__ballot(bad != 0) != 0)) ZFAIL(ZG_CORRUPT_STREAM);
        __threadfence_block();
        p = send;
      }
      // ---- sequences section ----
      uint32_t nseq = 0;
      if (p < bend) {
        const uint32_t c0 = I.b(p);
        if (c0 < 128) { nseq = c0; p += 1; }
        else if (c0 < 255) { nseq = ((c0 - 128) << 8) + I.b(p + 1); p += 2; }
        else { nseq = I.le16(p + 1) + 0x7F00; p += 3; }
      } else {
        ZFAIL(ZG_CORRUPT_STREAM);  // the Number_of_Sequences field is mandatory
      }
      uint64_t litpos = 0;
      if (nseq) {
        if (p >= bend) ZFAIL(ZG_CORRUPT_STREAM);
        const uint32_t modes = I.b(p++);
        if (modes & 3) ZFAIL(ZG_CORRUPT_STREAM);
        const uint32_t llm = modes >> 6, ofm = (modes >> 4) & 3, mlm = (modes >> 2) & 3;
        // LL, OF, ML table descriptions in that order
        bool ok = true;
        for (int t = 0; t < 3 && ok; t++) {
          const uint32_t mode = t == 0 ? llm : t == 1 ? ofm : mlm;
          Fse *T = t == 0 ? S.ll : t == 1 ? S.of : S.ml;
          const uint32_t maxs = t == 0 ? 35 : t == 1 ? 31 : 52, maxl = t == 0 ? 9 : t == 1 ? 8 : 9;
          uint32_t lg = 0;
          if (mode == 0) {
            if (t == 0) { build_fse_default(T, c_ll_def, 36, 6, S.norm, S.tmp); lg = 6; }
            else if (t == 1) { build_fse_default(T, c_of_def, 29, 5, S.norm, S.tmp); lg = 5; }
            else { build_fse_default(T, c_ml_def, 53, 6, S.norm, S.tmp); lg = 6; }
          } else if (mode == 1) {
            if (p >= bend) { ok = false; break; }
            const uint32_t sym = I.b(p++);
            if (sym > maxs) { ok = false; break; }
            build_fse_rle(T, sym);
            lg = 0;
          } else if (mode == 2) {
            uint32_t acc, ns;
            const uint32_t used = read_ncount(I, p, bend - p, S.norm, maxs, maxl, acc, ns);
            if (!used) { ok = false; break; }
            __syncthreads();
            build_fse(T, S.norm, ns, acc, S.tmp);
            p += used;
            lg = acc;
          } else {
            const bool have = t == 0 ? have_ll : t == 1 ? have_of : have_ml;
            if (!have) { ok = false; break; }
            lg = t == 0 ? ll_log : t == 1 ? of_log : ml_log;
          }
          if (t == 0) { ll_log = lg; have_ll = true; }
          else if (t == 1) { of_log = lg; have_of = true; }
          else { ml_log = lg; have_ml = true; }
        }
        if (!ok) ZFAIL(ZG_CORRUPT_STREAM);
        BitsBack R;
        if (!bb_init(R, in, it.len, p, bend)) ZFAIL(ZG_CORRUPT_STREAM);
        uint32_t sll = bb_read(R, ll_log), sof = bb_read(R, of_log), sml = bb_read(R, ml_log);
        uint32_t remaining = nseq;
        while (remaining && !err) {
          // ---- decode a batch of sequences (one per lane) ----
          uint32_t r_ll = 0, r_ml = 0, r_of = 0;
          uint32_t cnt = 0;
          uint64_t span = 0, lspan = 0;
          bool big_pending = false;
          uint32_t big_ll = 0, big_ml = 0, big_of = 0;
          while (cnt < 64 && remaining && span < ZBATCH) {
            const Fse eo = S.of[sof], em = S.ml[sml], el = S.ll[sll];
            const uint32_t ofc = U(eo.sym), mlc = U(em.sym), llc = U(el.sym);
            if (ofc > 31 || mlc > 52 || llc > 35) { err = ZG_CORRUPT_STREAM; break; }
            uint32_t ofv;
            if (ofc <= 25) {
              ofv = (1u << ofc) + bb_read(R, ofc);
            } else {  // up to 31 extra bits
              const uint32_t hi = bb_read(R, ofc - 16);
              const uint32_t lo = bb_read(R, 16);
              ofv = (1u << ofc) + ((hi << 16) | lo);
            }
            const uint32_t ml = c_ml_base[mlc] + bb_read(R, c_ml_bits[mlc]);
            const uint32_t ll = c_ll_base[llc] + bb_read(R, c_ll_bits[llc]);
            uint32_t off;
            if (ofv > 3) {
              off = ofv - 3;
              rep2 = rep1; rep1 = rep0; rep0 = off;
            } else {
              const uint32_t idx = ofv - 1 + (ll == 0 ? 1 : 0);
              if (idx == 0) {
                off = rep0;
              } else if (idx == 1) {
                off = rep1; rep1 = rep0; rep0 = off;
              } else if (idx == 2) {
                off = rep2; rep2 = rep1; rep1 = rep0; rep0 = off;
              } else {
                off = rep0 - 1; rep2 = rep1; rep1 = rep0; rep0 = off;
              }
            }
            remaining--;
            if (remaining) {  // state updates: LL, ML, OF
              sll = U(el.base) + bb_read(R, U(el.nb));
              sml = U(em.base) + bb_read(R, U(em.nb));
              sof = U(eo.base) + bb_read(R, U(eo.nb));
            }
            if (ll >= ZBIG || ml >= ZBIG) {  // executed alone after this batch
              big_pending = true;
              big_ll = ll; big_ml = ml; big_of = off;
              break;
            }
            if (lane == (int)cnt) { r_ll = ll; r_ml = ml; r_of = off; }
            cnt++;
            span += ll + ml;
            lspan += ll;
          }
          if (err) break;
          if (bb_overflow(R)) ZFAIL(ZG_CORRUPT_STREAM);
          // ---- execute the batch ----
          if (cnt) {
            const uint64_t out_base = O.pos;
            if (out_base + span > O.cap) ZFAIL(ZG_DECODED_SIZE_MISMATCH);
            if (litpos + lspan > regen) ZFAIL(ZG_CORRUPT_STREAM);
            out_reserve(S, O, span);
            const bool mine = lane < (int)cnt;
            uint32_t a = mine ? r_ll : 0u, b = mine ? r_ll + r_ml : 0u;
            for (int o = 1; o < 64; o <<= 1) {
              const uint32_t ta = __shfl_up(a, o, 64), tb = __shfl_up(b, o, 64);
              if (lane >= o) { a += ta; b += tb; }
            }
            S.pfx_lit[lane] = a;  // inclusive prefix of literal lengths
            S.pfx_out[lane] = b;  // inclusive prefix of sequence spans
            // match validity: offset within the frame's output so far
            const uint64_t mstart = out_base + b - (mine ? r_ml : 0u);
            const bool badoff = mine && r_ml && (r_of == 0 || (uint64_t)r_of > mstart - frame_start);
            if (U(__ballot(badoff) != 0)) ZFAIL(ZG_CORRUPT_STREAM);
            __syncthreads();
            // literal runs of the whole batch
            const uint32_t L = (uint32_t)lspan;
            for (uint32_t k = lane; k < L; k += 64) {
              uint32_t lo2 = 0, hi2 = cnt - 1;  // first sequence with pfx_lit > k
              while (lo2 < hi2) {
                const uint32_t mid = (lo2 + hi2) >> 1;
                if (S.pfx_lit[mid] > k) hi2 = mid; else lo2 = mid + 1;
              }
              const uint32_t prev_lit = lo2 ? S.pfx_lit[lo2 - 1] : 0u, prev_out = lo2 ? S.pfx_out[lo2 - 1] : 0u;
              const uint64_t dstp = out_base + prev_out + (k - prev_lit);
              S.ring[dstp & ZRMASK] = __builtin_nontemporal_load(lsrc + litpos + k);
            }
            // matches in order
            const uint64_t wend = out_base + span;
            uint64_t mm = __ballot(mine && r_ml > 0);
            if (U(__ballot(mine && r_ml > 0 && mstart - r_of + ZRING < wend) != 0)) out_fence(O);
            while (mm) {
              const int j = __builtin_ctzll(mm);
              mm &= mm - 1;
              const uint32_t ml = U(__builtin_amdgcn_readlane(r_ml, j));
              const uint32_t d = U(__builtin_amdgcn_readlane(r_of, j));
              const uint64_t ps = out_base + U(__builtin_amdgcn_readlane(b, j)) - ml;
              const float inv = 1.0f / (float)d;
              for (uint32_t i = lane; i < ml; i += 64) {
                uint32_t rm = i;
                if (d < ml) {
                  uint32_t q = (uint32_t)((float)i * inv);
                  int32_t r = (int32_t)i - (int32_t)(q * d);
                  if (r < 0) r += d;
                  if (r >= (int32_t)d) r -= d;
                  rm = (uint32_t)r;
                }
                S.ring[(ps + i) & ZRMASK] = src_byte(S, O, ps - d + rm, wend);
              }
            }
            __syncthreads();
            O.pos = wend;
            litpos += lspan;
          }
          if (big_pending) {
            if (O.pos + big_ll + big_ml > O.cap) ZFAIL(ZG_DECODED_SIZE_MISMATCH);
            if (litpos + big_ll > regen) ZFAIL(ZG_CORRUPT_STREAM);
            out_copy_global(S, O, lsrc + litpos, big_ll);
            litpos += big_ll;
            if (big_ml) {
              if (big_of == 0 || (uint64_t)big_of > O.pos - frame_start) ZFAIL(ZG_CORRUPT_STREAM);
              out_match(S, O, big_of, big_ml);
            }
          }
        }
        if (err) break;
        if (!bb_exact_end(R)) ZFAIL(ZG_CORRUPT_STREAM);
      } else if (p != bend) {
        ZFAIL(ZG_CORRUPT_STREAM);
      }
      // last literals
      if (litpos > regen) ZFAIL(ZG_CORRUPT_STREAM);
      if (O.pos + (regen - litpos) > O.cap) ZFAIL(ZG_DECODED_SIZE_MISMATCH);
      out_copy_global(S, O, lsrc + litpos, regen - litpos);
      ip = bend;
    }
    if (err) break;
    if (fcs_sz && O.pos - frame_start != fcs) ZFAIL(ZG_CORRUPT_STREAM);
    if (has_ck) {
      if (ip + 4 > it.len) ZFAIL(ZG_CORRUPT_STREAM);
      const uint32_t want = I.le32(ip);
      ip += 4;
      out_flush(S, O);
      out_fence(O);
      const uint64_t h = xxh64(O.out + frame_start, O.pos - frame_start);
      if ((uint32_t)h != want) ZFAIL(ZG_CORRUPT_STREAM);
    }
  }
#undef ZFAIL
  if (!err && !any_frame) err = ZG_CORRUPT_STREAM;
  if (!err) out_flush(S, O);
  if (lane == 0) {
    if (err) {
      status[item] = err;
    } else {
      items[item].src = (uint64_t)O.out;
      items[item].len = O.pos;
    }
  }
}

// =================================================================================================
// Block-parallel path (items whose blocks fit the scratch; k_zstd above is the fallback).
//
// A zstd frame is a chain of blocks whose sizes are in their 3-byte headers, so both the entropy
// decoding and most of the sequence execution parallelise over blocks:
//   k_zstd_scan    one wave per item: walk frames and block headers, parse each compressed block's
//                  literal / sequence section headers, resolve "treeless" literals and "repeat" FSE
//                  modes to the block that defined the table; one ZBlk record per block
//   k_zstd_blocks  one wave per block: Huffman literals into the literal scratch, FSE sequences into
//                  the sequence scratch. Repeat offsets are resolved symbolically ("incoming rep k,
//                  minus j"), so no block waits for its predecessor; the block's outgoing rep state
//                  is kept in the same symbolic form
//   k_zstd_plan    one wave per item: block output offsets (prefix sum), concrete incoming rep state
//                  per block (composing the symbolic transforms), frame content size checks
//   k_zstd_exec_blocks  one wave per block: executes the block into its own output range. A match
//                  whose source lies in an earlier block, or touches bytes deferred before it (an
//                  exact per-byte taint bitmap in LDS), is deferred: recorded in place of the
//                  consumed sequences; everything else is final. Matches of a batch resolve in rounds
//                  (see k_gzip)
//   k_zstd_fixup   one wave per item, blocks in order: a block with deferred matches is loaded whole
//                  into LDS (<= 128 KiB), its deferred matches run there (sources in earlier blocks
//                  are final by then), and it is written back; then the frame checksums.
//                  Deferral chains can span a whole frame (a run continuing across blocks), so this
//                  pass is serial per frame, but it touches only the deferred matches, in LDS
// =================================================================================================
namespace {

constexpr uint32_t ZB_RAW = 0, ZB_RLE = 1, ZB_CMP = 2;
constexpr uint32_t ZBF_FIRST = 1u << 8, ZBF_LAST = 1u << 9, ZBF_FCS = 1u << 10, ZBF_CK = 1u << 11;
constexpr uint32_t ZSYM = 0x80000000u;      // symbolic offset: ZSYM | slot << 24 | minus

struct ZBlk {
  uint32_t flags;             // bits 0-1 block type, 2-3 literal type, 4 four streams, ZBF_*
  uint32_t in_off, in_size;   // block content (raw data / rle byte / compressed content), item-relative
  uint32_t out_size;          // decoded size: raw/rle from the header, compressed from k_zstd_blocks
  uint32_t regen;             // literal count
  uint32_t lit_off, lit_end;  // raw literals: data; rle: the byte; huffman: streams (jump table first)
  uint32_t huf_off;           // Huffman tree description in effect
  uint32_t nseq, seq_off, seq_end;  // sequence bitstream
  uint32_t tab_off[3];        // LL / OF / ML table source (rle: symbol byte; fse: NCount)
  uint32_t tab_mode;          // 2 bits per table: 0 predefined, 1 rle, 2 fse
  uint32_t lit_buf;           // literal scratch offset (huffman / rle literals)
  uint32_t seq_buf;           // first sequence in the item's sequence scratch
  uint32_t ck;                // frame checksum (last block of a frame with one)
  uint64_t fcs;               // frame content size (first block of a frame with one)
  uint32_t rep_out[3];        // outgoing rep offsets (symbolic in the incoming ones)
  uint32_t rep_in[3];         // incoming rep offsets (concrete, from k_zstd_plan)
  uint32_t out_off;           // item-relative output offset (k_zstd_plan)
  uint32_t frame_off;         // output offset of the block's frame
  uint32_t def_n;             // deferred matches recorded by k_zstd_exec_blocks
  uint32_t def_done;          // deferred matches resolved so far
};

struct ZScanSmem {
  int16_t norm[64];
};

// literals (Huffman table) and sequences (FSE tables) are decoded one after the other: the two
// table sets share LDS
struct ZDecSmem {
  union {
    uint16_t huf[1 << MAX_HUF_LOG];
    struct {
      Fse ll[512], ml[512], of[256];
    };
  };
  Fse wt[64];
  int16_t norm[64];
  uint8_t weights[256];
  uint16_t hsorted[256];
  uint32_t tmp[32];
};

struct ZExecSmem {
  uint8_t ring[ZRING];
  uint32_t taint[BLOCK_MAX / 32];  // one bit per output byte of the block: deferred (not yet final)
  uint8_t lit_stage[ZBATCH];       // the batch's literals, staged with 16-B loads
  uint32_t pfx_lit[64], pfx_out[64];
};

// coherent byte read of output this wave (or an earlier kernel) wrote: an agent-scope relaxed
// atomic load is an sc1 load that bypasses the CU's L1 (MI355X_MICROARCH.md, hand-off table)
__device__ __forceinline__ uint8_t load_out_byte(const uint8_t *p) {
  const uint32_t *w = (const uint32_t *)((uintptr_t)p & ~(uintptr_t)3);
  const uint32_t v = __hip_atomic_load(w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return (uint8_t)(v >> (8 * ((uintptr_t)p & 3)));
}

__device__ __forceinline__ uint32_t sym_dec(uint32_t x) { return (x & ZSYM) ? x + 1 : x - 1; }
__device__ __forceinline__ uint32_t sym_eval(uint32_t x, uint32_t r0, uint32_t r1, uint32_t r2) {
  if (!(x & ZSYM)) return x;
  const uint32_t slot = (x >> 24) & 3, minus = x & 0xFFFFFF;
  return (slot == 0 ? r0 : slot == 1 ? r1 : r2) - minus;
}

// exact-range output flush for a block (its neighbours belong to other waves): bytes [from, to)
template <class SM>
__device__ __forceinline__ void blk_flush(SM &S, uint8_t *out, uint64_t from, uint64_t to) {
  __syncthreads();
  const uint64_t a = (from + 15) & ~(uint64_t)15, b = to & ~(uint64_t)15;
  if (a >= b) {
    for (uint64_t p = from + lane_id(); p < to; p += 64) out[p] = S.ring[p & ZRMASK];
  } else {
    for (uint64_t p = from + lane_id(); p < a; p += 64) out[p] = S.ring[p & ZRMASK];
    for (uint64_t p = a + (uint64_t)lane_id() * 16; p < b; p += 64 * 16)
      *(uint4 *)(out + p) = *(const uint4 *)&S.ring[p & ZRMASK];
    for (uint64_t p = b + lane_id(); p < to; p += 64) out[p] = S.ring[p & ZRMASK];
  }
  __syncthreads();
}

// exact-range write-back of a block image img[0, to - from) to out[from, to)
__device__ __forceinline__ void blk_flush_img(const uint8_t *img, uint8_t *out, uint64_t from, uint64_t to) {
  __syncthreads();
  const uint64_t a = (from + 15) & ~(uint64_t)15, b = to & ~(uint64_t)15;
  if (a >= b) {
    for (uint64_t p = from + lane_id(); p < to; p += 64) out[p] = img[p - from];
  } else {
    for (uint64_t p = from + lane_id(); p < a; p += 64) out[p] = img[p - from];
    for (uint64_t p = a + (uint64_t)lane_id() * 16; p < b; p += 64 * 16) {
      const uint8_t *q = img + (p - from);
      uint4 v;
      if (((p - from) & 3) == 0) {
        v = make_uint4(*(const uint32_t *)q, *(const uint32_t *)(q + 4), *(const uint32_t *)(q + 8),
                       *(const uint32_t *)(q + 12));
      } else {
        uint32_t w[4];
        for (int j = 0; j < 4; j++)
          w[j] = q[4 * j] | (q[4 * j + 1] << 8) | (q[4 * j + 2] << 16) | ((uint32_t)q[4 * j + 3] << 24);
        v = make_uint4(w[0], w[1], w[2], w[3]);
      }
      *(uint4 *)(out + p) = v;
    }
    for (uint64_t p = b + lane_id(); p < to; p += 64) out[p] = img[p - from];
  }
  __syncthreads();
}

}  // namespace

__global__ __launch_bounds__(64) void k_zstd_scan(const ZgItem *items, uint32_t *status, ZBlk *blks,
                                                  uint32_t blk_cap, uint32_t *nblk, uint32_t *zmode,
                                                  uint64_t lit_stride, uint64_t seq_cap) {
  __shared__ ZScanSmem S;
  const uint32_t item = blockIdx.x;
  const ZgItem it = items[item];
  const int lane = lane_id();
  if (status[item] || (it.flags & ZG_ITEM_FILL)) {
    if (lane == 0) { nblk[item] = 0; zmode[item] = ZMODE_SKIP; }
    return;
  }
  if (it.len >= 0xFFFFFFF0ull) {  // 32-bit record offsets: decode such items serially
    if (lane == 0) { nblk[item] = 0; zmode[item] = ZMODE_SERIAL; }
    return;
  }
  const uint8_t *in = (const uint8_t *)it.src;
  const In I{in, it.len};
  ZBlk *B = blks + (uint64_t)item * blk_cap;
  uint32_t nb = 0, err = 0;
  bool serial = false, any_frame = false;
  uint64_t ip = 0, lit_used = 0, seq_used = 0;
#define SFAIL(code) { err = (code); break; }
  while (!err && !serial && ip < it.len) {
    const uint32_t magic = I.le32(ip);
    if (ip + 4 > it.len) SFAIL(ZG_CORRUPT_STREAM);
    if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  // skippable frame
      if (ip + 8 > it.len) SFAIL(ZG_CORRUPT_STREAM);
      ip += 8 + (uint64_t)I.le32(ip + 4);
      if (ip > it.len) SFAIL(ZG_CORRUPT_STREAM);
      continue;
    }
    if (magic != 0xFD2FB528u) SFAIL(ZG_CORRUPT_STREAM);
    ip += 4;
    any_frame = true;
    const uint32_t fhd = I.b(ip++);
    const uint32_t fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, has_ck = (fhd >> 2) & 1, did_flag = fhd & 3;
    if (fhd & 8) SFAIL(ZG_CORRUPT_STREAM);
    if (!single) ip++;
    const uint32_t did_sz = did_flag == 3 ? 4 : did_flag;
    uint32_t did = 0;
    for (uint32_t k = 0; k < did_sz; k++) did |= I.b(ip + k) << (8 * k);
    ip += did_sz;
    if (did != 0) SFAIL(ZG_CORRUPT_STREAM);
    const uint32_t fcs_sz = fcs_flag == 0 ? (single ? 1 : 0) : (fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8);
    uint64_t fcs = 0;
    for (uint32_t k = 0; k < fcs_sz; k++) fcs |= (uint64_t)I.b(ip + k) << (8 * k);
    if (fcs_sz == 2) fcs += 256;
    ip += fcs_sz;
    if (ip > it.len) SFAIL(ZG_CORRUPT_STREAM);
    bool first = true, last = false;
    uint32_t huf_src = 0xFFFFFFFFu;                      // tree in effect (treeless literals reuse it)
    uint32_t tmode[3] = {3, 3, 3}, toff[3] = {0, 0, 0};  // 3 = no table yet
    while (!last && !err) {
      if (nb == blk_cap) { serial = true; break; }
      if (ip + 3 > it.len) SFAIL(ZG_CORRUPT_STREAM);
      const uint32_t bh = I.le24(ip);
      ip += 3;
      last = bh & 1;
      const uint32_t btype = (bh >> 1) & 3, bsize = bh >> 3;
      if (btype == 3) SFAIL(ZG_CORRUPT_STREAM);
      ZBlk R{};
      R.flags = btype | (first ? ZBF_FIRST : 0u) | (last ? ZBF_LAST : 0u);
      if (first && fcs_sz) { R.flags |= ZBF_FCS; R.fcs = fcs; }
      first = false;
      R.in_off = (uint32_t)ip;
      if (btype == 0) {
        if (ip + bsize > it.len) SFAIL(ZG_CORRUPT_STREAM);
        R.in_size = bsize;
        R.out_size = bsize;
        ip += bsize;
      } else if (btype == 1) {
        if (ip + 1 > it.len) SFAIL(ZG_CORRUPT_STREAM);
        R.in_size = 1;
        R.out_size = bsize;
        ip += 1;
      } else {
        if (bsize > BLOCK_MAX || ip + bsize > it.len) SFAIL(ZG_CORRUPT_STREAM);
        const uint64_t bend = ip + bsize;
        R.in_size = bsize;
        uint64_t p = ip;
        const uint32_t b0 = I.b(p);
        const uint32_t ltype = b0 & 3, sfmt = (b0 >> 2) & 3;
        uint32_t regen = 0, csize = 0, lhdr = 0, four = 0;
        if (ltype <= 1) {
          if (sfmt == 0 || sfmt == 2) { regen = b0 >> 3; lhdr = 1; }
          else if (sfmt == 1) { regen = (b0 >> 4) | (I.b(p + 1) << 4); lhdr = 2; }
          else { regen = (b0 >> 4) | (I.b(p + 1) << 4) | (I.b(p + 2) << 12); lhdr = 3; }
        } else {
          four = sfmt == 0 ? 0 : 1;
          if (sfmt <= 1) { const uint32_t v = I.le24(p); regen = (v >> 4) & 0x3FF; csize = (v >> 14) & 0x3FF; lhdr = 3; }
          else if (sfmt == 2) { const uint32_t v = I.le32(p); regen = (v >> 4) & 0x3FFF; csize = (v >> 18) & 0x3FFF; lhdr = 4; }
          else {
            const uint64_t v = (uint64_t)I.le32(p) | ((uint64_t)I.b(p + 4) << 32);
            regen = (uint32_t)(v >> 4) & 0x3FFFF; csize = (uint32_t)(v >> 22) & 0x3FFFF; lhdr = 5;
          }
        }
        if (regen > BLOCK_MAX) SFAIL(ZG_CORRUPT_STREAM);
        p += lhdr;
        R.flags |= (ltype << 2) | (four << 4);
        R.regen = regen;
        if (ltype == 0) {
          if (p + regen > bend) SFAIL(ZG_CORRUPT_STREAM);
          R.lit_off = (uint32_t)p;
          R.lit_end = (uint32_t)(p + regen);
          p += regen;
        } else if (ltype == 1) {
          if (p + 1 > bend) SFAIL(ZG_CORRUPT_STREAM);
          R.lit_off = (uint32_t)p;
          p += 1;
        } else {
          if (p + csize > bend) SFAIL(ZG_CORRUPT_STREAM);
          uint64_t q = p;
          if (ltype == 2) {  // tree description: FSE-compressed weights (hb < 128) or 4-bit weights
            const uint32_t hb = I.b(q);
            const uint32_t tsz = hb < 128 ? 1 + hb : 1 + (hb - 127 + 1) / 2;
            if (hb == 0 || tsz > csize) SFAIL(ZG_CORRUPT_STREAM);
            huf_src = (uint32_t)q;
            q += tsz;
          } else if (huf_src == 0xFFFFFFFFu) {
            SFAIL(ZG_CORRUPT_STREAM);  // treeless without a previous table
          }
          R.huf_off = huf_src;
          R.lit_off = (uint32_t)q;
          R.lit_end = (uint32_t)(p + csize);
          p += csize;
        }
        if (ltype != 0) {  // rle / huffman literals are materialised in the literal scratch
          R.lit_buf = (uint32_t)lit_used;
          lit_used += regen;
          if (lit_used > lit_stride) { serial = true; break; }
        }
        // sequences section header
        if (p >= bend) SFAIL(ZG_CORRUPT_STREAM);
        uint32_t nseq = 0;
        const uint32_t c0 = I.b(p);
        if (c0 < 128) { nseq = c0; p += 1; }
        else if (c0 < 255) { nseq = ((c0 - 128) << 8) + I.b(p + 1); p += 2; }
        else { nseq = I.le16(p + 1) + 0x7F00; p += 3; }
        R.nseq = nseq;
        if (nseq) {
          if (p >= bend) SFAIL(ZG_CORRUPT_STREAM);
          const uint32_t modes = I.b(p++);
          if (modes & 3) SFAIL(ZG_CORRUPT_STREAM);
          const uint32_t mm[3] = {modes >> 6, (modes >> 4) & 3, (modes >> 2) & 3};  // LL, OF, ML
          bool ok = true;
          for (int t = 0; t < 3 && ok; t++) {
            const uint32_t maxs = t == 0 ? 35 : t == 1 ? 31 : 52, maxl = t == 0 ? 9 : t == 1 ? 8 : 9;
            if (mm[t] == 0) {
              tmode[t] = 0;
              toff[t] = 0;
            } else if (mm[t] == 1) {
              if (p >= bend || I.b(p) > maxs) { ok = false; break; }
              tmode[t] = 1;
              toff[t] = (uint32_t)p;
              p += 1;
            } else if (mm[t] == 2) {
              uint32_t acc, ns;
              const uint32_t used = read_ncount(I, p, bend - p, S.norm, maxs, maxl, acc, ns);
              if (!used) { ok = false; break; }
              tmode[t] = 2;
              toff[t] = (uint32_t)p;
              p += used;
            } else if (tmode[t] == 3) {
              ok = false;  // repeat mode without a previous table
            }
          }
          if (!ok) SFAIL(ZG_CORRUPT_STREAM);
          R.tab_mode = tmode[0] | (tmode[1] << 2) | (tmode[2] << 4);
          R.tab_off[0] = toff[0];
          R.tab_off[1] = toff[1];
          R.tab_off[2] = toff[2];
          R.seq_off = (uint32_t)p;
          R.seq_end = (uint32_t)bend;
          R.seq_buf = (uint32_t)seq_used;
          seq_used += nseq;
          if (seq_used > seq_cap) { serial = true; break; }
        } else if (p != bend) {
          SFAIL(ZG_CORRUPT_STREAM);
        }
        ip = bend;
      }
      if (last && has_ck) {
        if (ip + 4 > it.len) SFAIL(ZG_CORRUPT_STREAM);
        R.flags |= ZBF_CK;
        R.ck = I.le32(ip);
        ip += 4;
      }
      if (lane == 0) B[nb] = R;
      nb++;
    }
  }
#undef SFAIL
  if (!err && !serial && !any_frame) err = ZG_CORRUPT_STREAM;
  if (lane == 0) {
    nblk[item] = serial ? 0u : nb;
    zmode[item] = serial ? ZMODE_SERIAL : (err ? ZMODE_SKIP : ZMODE_PARALLEL);
    if (err && !serial) status[item] = err;
  }
}

// One wave per (item, block) record, grid-stride. Sequences land as {ll, ml, offset symbol}.
__global__ __launch_bounds__(64) void k_zstd_blocks(const ZgItem *items, uint32_t *status, ZBlk *blks,
                                                    uint32_t blk_cap, const uint32_t *nblk,
                                                    const uint32_t *zmode, uint32_t n_items, uint8_t *lit_scratch,
                                                    uint64_t lit_stride, uint32_t *seq_scratch, uint64_t seq_cap) {
  __shared__ ZDecSmem S;
  const int lane = lane_id();
  const uint64_t total = (uint64_t)n_items * blk_cap;
  for (uint64_t g = blockIdx.x; g < total; g += gridDim.x) {
    const uint32_t item = (uint32_t)(g / blk_cap), bi = (uint32_t)(g % blk_cap);
    if (bi >= nblk[item] || zmode[item] != ZMODE_PARALLEL) continue;
    ZBlk *Bp = blks + g;
    const uint32_t flags = U(Bp->flags);
    if ((flags & 3) != ZB_CMP) continue;
    const ZgItem it = items[item];
    const uint8_t *in = (const uint8_t *)it.src;
    const In I{in, it.len};
    const uint32_t ltype = (flags >> 2) & 3, regen = U(Bp->regen);
    uint8_t *lit = lit_scratch + (uint64_t)item * lit_stride + U(Bp->lit_buf);
    bool bad = false;
    __syncthreads();  // the previous record's table reads are done before they are rebuilt
    // ---- literals ----
    if (ltype == 1) {
      const uint8_t v = (uint8_t)I.b(U(Bp->lit_off));
      for (uint32_t k = lane; k < regen; k += 64) lit[k] = v;
    } else if (ltype >= 2) {
      const uint32_t huf_off = U(Bp->huf_off), lo0 = U(Bp->lit_off), lend = U(Bp->lit_end);
      uint32_t tl = 0;
      if (!read_huffman(I, huf_off, it.len - huf_off, S, tl, in, it.len)) {
        bad = true;
      } else {
        const uint32_t nstreams = (flags >> 4) & 1 ? 4 : 1;
        uint64_t s_lo[4], s_hi[4];
        uint32_t s_n[4];
        if (nstreams == 1) {
          s_lo[0] = lo0; s_hi[0] = lend; s_n[0] = regen;
        } else {
          const uint64_t q = lo0;
          if (q + 6 > lend) bad = true;
          const uint32_t l1 = I.le16(q), l2 = I.le16(q + 2), l3 = I.le16(q + 4);
          const uint64_t b = q + 6;
          if (b + l1 + l2 + l3 > lend) bad = true;
          s_lo[0] = b; s_hi[0] = b + l1;
          s_lo[1] = s_hi[0]; s_hi[1] = s_lo[1] + l2;
          s_lo[2] = s_hi[1]; s_hi[2] = s_lo[2] + l3;
          s_lo[3] = s_hi[2]; s_hi[3] = lend;
          const uint32_t seg = (regen + 3) / 4;
          if (3 * seg > regen) bad = true;
          s_n[0] = s_n[1] = s_n[2] = seg;
          s_n[3] = regen - 3 * seg;
        }
        uint32_t lbad = 0;
        if (!bad && lane < (int)nstreams) {
          const uint64_t lo = lane == 0 ? s_lo[0] : lane == 1 ? s_lo[1] : lane == 2 ? s_lo[2] : s_lo[3];
          const uint64_t hi = lane == 0 ? s_hi[0] : lane == 1 ? s_hi[1] : lane == 2 ? s_hi[2] : s_hi[3];
          const uint32_t ns = lane == 0 ? s_n[0] : lane == 1 ? s_n[1] : lane == 2 ? s_n[2] : s_n[3];
          const uint32_t out0 = nstreams == 4 ? lane * ((regen + 3) / 4) : 0u;
          const uintptr_t mis = (uintptr_t)in & 3;
          LaneBits L;
          L.words = (const uint32_t *)((uintptr_t)in - mis);
          L.nwords = (uint32_t)((it.len + mis + 3) / 4);
          const uint32_t lastb = hi > lo ? in[hi - 1] : 0u;
          if (lastb == 0) {
            lbad = 1;
          } else {
            L.cur = (int64_t)(hi - 1 + mis) * 8 + (31 - __builtin_clz(lastb));
            L.lo_bit = (int64_t)(lo + mis) * 8;
            lane_bits_init(L);
            for (uint32_t k = 0; k < ns; k++) {
              const uint32_t e = S.huf[lane_peek(L, tl)];
              L.cur -= e >> 8;
              lit[out0 + k] = (uint8_t)e;
              if (L.cur < L.lo_bit) { lbad = 1; break; }
            }
            if (L.cur != L.lo_bit) lbad = 1;
          }
        }
        if (__ballot(lbad != 0)) bad = true;
      }
    }
    __syncthreads();  // Huffman table reads done: the FSE tables reuse its LDS
    // ---- sequences ----
    const uint32_t nseq = U(Bp->nseq);
    uint64_t sum_ll = 0, sum_ml = 0;
    uint32_t r0 = ZSYM | (0u << 24), r1 = ZSYM | (1u << 24), r2 = ZSYM | (2u << 24);
    if (!bad && nseq) {
      const uint32_t tm = U(Bp->tab_mode);
      uint32_t lg[3] = {0, 0, 0};
      for (int t = 0; t < 3 && !bad; t++) {
        const uint32_t mode = (tm >> (2 * t)) & 3, off = U(Bp->tab_off[t]);
        Fse *T = t == 0 ? S.ll : t == 1 ? S.of : S.ml;
        const uint32_t maxs = t == 0 ? 35 : t == 1 ? 31 : 52, maxl = t == 0 ? 9 : t == 1 ? 8 : 9;
        if (mode == 0) {
          if (t == 0) { build_fse_default(T, c_ll_def, 36, 6, S.norm, S.tmp); lg[t] = 6; }
          else if (t == 1) { build_fse_default(T, c_of_def, 29, 5, S.norm, S.tmp); lg[t] = 5; }
          else { build_fse_default(T, c_ml_def, 53, 6, S.norm, S.tmp); lg[t] = 6; }
        } else if (mode == 1) {
          build_fse_rle(T, I.b(off));
          lg[t] = 0;
        } else {
          uint32_t acc, ns;
          if (!read_ncount(I, off, it.len - off, S.norm, maxs, maxl, acc, ns)) { bad = true; break; }
          __syncthreads();
          build_fse(T, S.norm, ns, acc, S.tmp);
          lg[t] = acc;
        }
      }
      BitsBack R;
      if (!bad && !bb_init(R, in, it.len, U(Bp->seq_off), U(Bp->seq_end))) bad = true;
      if (!bad) {
        uint32_t sll = bb_read(R, lg[0]), sof = bb_read(R, lg[1]), sml = bb_read(R, lg[2]);
        uint32_t *out = seq_scratch + ((uint64_t)item * seq_cap + U(Bp->seq_buf)) * 3;
        uint32_t remaining = nseq, done = 0;
        while (remaining && !bad) {
          uint32_t r_ll = 0, r_ml = 0, r_of = 0, cnt = 0;
          while (cnt < 64 && remaining) {
            const Fse eo = S.of[sof], em = S.ml[sml], el = S.ll[sll];
            const uint32_t ofc = U(eo.sym), mlc = U(em.sym), llc = U(el.sym);
            if (ofc > 31 || mlc > 52 || llc > 35) { bad = true; break; }
            uint32_t ofv;
            if (ofc <= 25) {
              ofv = (1u << ofc) + bb_read(R, ofc);
            } else {
              const uint32_t hi = bb_read(R, ofc - 16);
              const uint32_t lo = bb_read(R, 16);
              ofv = (1u << ofc) + ((hi << 16) | lo);
            }
            const uint32_t ml = c_ml_base[mlc] + bb_read(R, c_ml_bits[mlc]);
            const uint32_t ll = c_ll_base[llc] + bb_read(R, c_ll_bits[llc]);
            remaining--;
            if (remaining) {
              sll = U(el.base) + bb_read(R, U(el.nb));
              sml = U(em.base) + bb_read(R, U(em.nb));
              sof = U(eo.base) + bb_read(R, U(eo.nb));
            }
            // repeat offsets, symbolically in the block's incoming rep state (RFC 8878 3.1.1.5)
            uint32_t off;
            if (ofv > 3) {
              off = ofv - 3;
              if (off & ZSYM) { bad = true; break; }  // beyond any window we decode
              r2 = r1; r1 = r0; r0 = off;
            } else {
              const uint32_t idx = ofv - 1 + (ll == 0 ? 1 : 0);
              if (idx == 0) {
                off = r0;
              } else if (idx == 1) {
                off = r1; r1 = r0; r0 = off;
              } else if (idx == 2) {
                off = r2; r2 = r1; r1 = r0; r0 = off;
              } else {
                off = sym_dec(r0); r2 = r1; r1 = r0; r0 = off;
              }
            }
            if (lane == (int)cnt) { r_ll = ll; r_ml = ml; r_of = off; }
            sum_ll += ll;
            sum_ml += ml;
            cnt++;
          }
          if (bad) break;
          if (lane < (int)cnt) {
            uint32_t *o = out + (uint64_t)(done + lane) * 3;
            o[0] = r_ll;
            o[1] = r_ml;
            o[2] = r_of;
          }
          done += cnt;
        }
        if (!bad && (bb_overflow(R) || !bb_exact_end(R))) bad = true;
      }
    }
    if (!bad && sum_ll > regen) bad = true;
    if (!bad && regen + sum_ml > BLOCK_MAX) bad = true;  // a block decodes to at most 128 KiB
    if (lane == 0) {
      if (bad) {
        status[item] = ZG_CORRUPT_STREAM;
      } else {
        Bp->out_size = (uint32_t)(regen + sum_ml);
        Bp->rep_out[0] = r0;
        Bp->rep_out[1] = r1;
        Bp->rep_out[2] = r2;
      }
    }
  }
}

// One wave per item: output offsets, incoming rep offsets, frame size checks.
__global__ __launch_bounds__(64) void k_zstd_plan(const ZgItem *items, uint32_t *status, ZBlk *blks,
                                                  uint32_t blk_cap, const uint32_t *nblk, const uint32_t *zmode,
                                                  uint64_t slot_bytes) {
  const uint32_t item = blockIdx.x;
  if (zmode[item] != ZMODE_PARALLEL || status[item]) return;
  const int lane = lane_id();
  ZBlk *B = blks + (uint64_t)item * blk_cap;
  const uint32_t nb = nblk[item];
  uint64_t pos = 0, frame_off = 0;
  uint32_t r0 = 1, r1 = 4, r2 = 8, err = 0;
  for (uint32_t bi = 0; bi < nb; bi++) {
    const uint32_t flags = U(B[bi].flags);
    if (flags & ZBF_FIRST) {
      frame_off = pos;
      r0 = 1; r1 = 4; r2 = 8;
    }
    if (lane == 0) {
      B[bi].out_off = (uint32_t)pos;
      B[bi].frame_off = (uint32_t)frame_off;
      B[bi].rep_in[0] = r0;
      B[bi].rep_in[1] = r1;
      B[bi].rep_in[2] = r2;
    }
    if ((flags & 3) == ZB_CMP && U(B[bi].nseq)) {
      const uint32_t o0 = U(B[bi].rep_out[0]), o1 = U(B[bi].rep_out[1]), o2 = U(B[bi].rep_out[2]);
      const uint32_t n0 = sym_eval(o0, r0, r1, r2), n1 = sym_eval(o1, r0, r1, r2), n2 = sym_eval(o2, r0, r1, r2);
      r0 = n0; r1 = n1; r2 = n2;
    }
    pos += U(B[bi].out_size);
    if (pos > slot_bytes || pos >= 0xFFFFFFF0ull) { err = ZG_DECODED_SIZE_MISMATCH; break; }
  }
  // frame content sizes: every frame whose first block has ZBF_FCS
  if (!err) {
    uint64_t fstart = 0, fcs = 0;
    bool has = false;
    for (uint32_t bi = 0; bi < nb; bi++) {
      const uint32_t flags = U(B[bi].flags);
      if (flags & ZBF_FIRST) {
        fstart = U(B[bi].out_off);
        has = flags & ZBF_FCS;
        fcs = (uint64_t)U((uint32_t)B[bi].fcs) | ((uint64_t)U((uint32_t)(B[bi].fcs >> 32)) << 32);
      }
      if ((flags & ZBF_LAST) && has && (uint64_t)U(B[bi].out_off) + U(B[bi].out_size) - fstart != fcs) {
        err = ZG_CORRUPT_STREAM;
        break;
      }
    }
  }
  if (lane == 0 && err) status[item] = err;
}

// One wave per (item, block) record, grid-stride: execute the block into its output range.
__global__ __launch_bounds__(64) void k_zstd_exec_blocks(const ZgItem *items, uint32_t *status, ZBlk *blks,
                                                         uint32_t blk_cap, const uint32_t *nblk,
                                                         const uint32_t *zmode, uint32_t n_items, uint8_t *dst,
                                                         uint64_t slot_bytes, const uint8_t *lit_scratch,
                                                         uint64_t lit_stride, const uint32_t *seq_scratch,
                                                         uint64_t seq_cap) {
  __shared__ ZExecSmem S;
  const int lane = lane_id();
  const uint64_t total = (uint64_t)n_items * blk_cap;
  for (uint64_t g = blockIdx.x; g < total; g += gridDim.x) {
    const uint32_t item = (uint32_t)(g / blk_cap), bi = (uint32_t)(g % blk_cap);
    if (bi >= nblk[item] || zmode[item] != ZMODE_PARALLEL || status[item]) continue;
    ZBlk *Bp = blks + g;
    const ZgItem it = items[item];
    const uint8_t *in = (const uint8_t *)it.src;
    uint8_t *out = dst + (uint64_t)item * slot_bytes;
    const uint32_t flags = U(Bp->flags), type = flags & 3;
    const uint64_t bstart = U(Bp->out_off);
    const uint32_t out_size = U(Bp->out_size);
    __syncthreads();  // the previous record's LDS use is over
    if (type != ZB_CMP) {  // raw / rle: no dependencies
      Out O{out, bstart + out_size, bstart, bstart, false};
      if (type == ZB_RAW) out_copy_global(S, O, in + U(Bp->in_off), out_size);
      else if (type == ZB_RLE) out_rle(S, O, (uint8_t)U(in[U(Bp->in_off)]), out_size);
      blk_flush(S, out, O.flushed, O.pos);
      continue;
    }
    uint32_t err = 0;
    const uint32_t ltype = (flags >> 2) & 3, regen = U(Bp->regen), nseq = U(Bp->nseq);
    const uint8_t *lsrc = ltype == 0 ? in + U(Bp->lit_off) : lit_scratch + (uint64_t)item * lit_stride + U(Bp->lit_buf);
    const uint32_t *seqs = seq_scratch + ((uint64_t)item * seq_cap + U(Bp->seq_buf)) * 3;
    // deferred matches {pos, distance, length} overwrite the block's already consumed sequences
    uint32_t *defl = const_cast<uint32_t *>(seqs);
    const uint32_t ri0 = U(Bp->rep_in[0]), ri1 = U(Bp->rep_in[1]), ri2 = U(Bp->rep_in[2]);
    const uint64_t frame_off = U(Bp->frame_off);
    for (uint32_t k = lane; k < BLOCK_MAX / 32; k += 64) S.taint[k] = 0;
    __syncthreads();
    Out O{out, bstart + out_size, bstart, bstart, false};
    uint32_t ndef = 0;
    uint64_t litpos = 0;
    uint32_t base = 0;
    // taint test of block-relative byte range [a, b) (a < b): any deferred byte in it?
    auto tainted = [&](uint64_t a, uint64_t b) -> bool {
      for (uint64_t w = a >> 5; w <= (b - 1) >> 5; w++) {
        uint32_t m = S.taint[w];
        const uint32_t lo = w == (a >> 5) ? (uint32_t)(a & 31) : 0u;
        const uint32_t hi = w == ((b - 1) >> 5) ? (uint32_t)((b - 1) & 31) : 31u;
        m &= (hi == 31 ? 0xFFFFFFFFu : ((1u << (hi + 1)) - 1)) & ~((1u << lo) - 1);
        if (m) return true;
      }
      return false;
    };
    auto mark = [&](uint64_t a, uint64_t b) {  // block-relative [a, b), this lane only
      for (uint64_t w = a >> 5; w <= (b - 1) >> 5; w++) {
        const uint32_t lo = w == (a >> 5) ? (uint32_t)(a & 31) : 0u;
        const uint32_t hi = w == ((b - 1) >> 5) ? (uint32_t)((b - 1) & 31) : 31u;
        atomicOr(&S.taint[w], (hi == 31 ? 0xFFFFFFFFu : ((1u << (hi + 1)) - 1)) & ~((1u << lo) - 1));
      }
    };
    while (base < nseq && !err) {
      const uint32_t avail = min<uint32_t>(64, nseq - base);
      uint32_t r_ll = 0, r_ml = 0, r_of = 0;
      if (lane < (int)avail) {
        const uint32_t *q = seqs + (uint64_t)(base + lane) * 3;
        r_ll = q[0];
        r_ml = q[1];
        r_of = sym_eval(q[2], ri0, ri1, ri2);
      }
      // batch: consecutive sequences up to ZBATCH bytes; a big one (>= ZBIG) goes alone
      uint32_t cnt = 0;
      uint64_t span = 0, lspan = 0;
      bool big = false;
      while (cnt < avail) {
        const uint32_t ll = __builtin_amdgcn_readlane(r_ll, cnt), ml = __builtin_amdgcn_readlane(r_ml, cnt);
        if (ll >= ZBIG || ml >= ZBIG) {
          big = cnt == 0;
          if (big) cnt = 1;
          break;
        }
        if (span + ll + ml > ZBATCH) break;
        cnt++;
        span += ll + ml;
        lspan += ll;
      }
      if (big) {
        span = (uint64_t)__builtin_amdgcn_readlane(r_ll, 0) + __builtin_amdgcn_readlane(r_ml, 0);
        lspan = __builtin_amdgcn_readlane(r_ll, 0);
      }
      const uint64_t out_base = O.pos;
      if (out_base + span > O.cap) { err = ZG_CORRUPT_STREAM; break; }
      if (litpos + lspan > regen) { err = ZG_CORRUPT_STREAM; break; }
      const bool mine = lane < (int)cnt;
      const uint32_t sll = mine ? r_ll : 0u, sml = mine ? r_ml : 0u;
      uint32_t a = sll, b = sll + sml;
      for (int o = 1; o < 64; o <<= 1) {
        const uint32_t ta = __shfl_up(a, o, 64), tb = __shfl_up(b, o, 64);
        if (lane >= o) { a += ta; b += tb; }
      }
      const uint64_t mstart = out_base + b - sml;
      if (__ballot(mine && sml && (r_of == 0 || (uint64_t)r_of > mstart - frame_off))) { err = ZG_CORRUPT_STREAM; break; }
      if (big) {
        // literal run then a long match, each through the ring in ZBATCH pieces
        const uint32_t bll = __builtin_amdgcn_readlane(r_ll, 0), bml = __builtin_amdgcn_readlane(r_ml, 0);
        const uint32_t bof = __builtin_amdgcn_readlane(r_of, 0);
        out_copy_global(S, O, lsrc + litpos, bll);
        litpos += bll;
        if (bml) {
          const uint64_t p = O.pos, src = p - bof;
          bool tnt = src < bstart;
          if (!tnt) {
            const uint64_t ra = src - bstart, rb = ra + min<uint64_t>(bml, bof);
            bool t = false;
            for (uint64_t w0 = (ra >> 5) + lane; w0 <= ((rb - 1) >> 5); w0 += 64) t |= tainted(max<uint64_t>(ra, w0 << 5), min<uint64_t>(rb, (w0 + 1) << 5));
            tnt = __ballot(t) != 0;
          }
          if (tnt) {  // defer the whole match
            for (uint64_t w0 = ((p - bstart) >> 5) + lane; w0 <= ((p - bstart + bml - 1) >> 5); w0 += 64)
              mark(max<uint64_t>(p - bstart, w0 << 5), min<uint64_t>(p - bstart + bml, (w0 + 1) << 5));
            if (lane == 0) { defl[3 * ndef] = (uint32_t)p; defl[3 * ndef + 1] = bof; defl[3 * ndef + 2] = bml; }
            ndef++;
            for (uint64_t done = 0; done < bml;) {  // keep the ring positions consistent (garbage)
              const uint64_t c = min<uint64_t>(bml - done, ZBATCH);
              out_reserve(S, O, c);
              O.pos += c;
              done += c;
            }
            __syncthreads();
          } else {
            out_match(S, O, bof, bml);
          }
        }
        base += 1;
        continue;
      }
      // ---- regular batch ----
      out_reserve(S, O, span);
      S.pfx_lit[lane] = a;
      S.pfx_out[lane] = b;
      const uint32_t Lb = (uint32_t)lspan;
      lds_copy_in(S.lit_stage, ~0ull, 0, lsrc + litpos, Lb);
      __syncthreads();
      for (uint32_t k = lane; k < Lb; k += 64) {
        uint32_t lo2 = 0, hi2 = cnt - 1;  // first sequence with pfx_lit > k
        while (lo2 < hi2) {
          const uint32_t mid = (lo2 + hi2) >> 1;
          if (S.pfx_lit[mid] > k) hi2 = mid; else lo2 = mid + 1;
        }
        const uint32_t prev_lit = lo2 ? S.pfx_lit[lo2 - 1] : 0u, prev_out = lo2 ? S.pfx_out[lo2 - 1] : 0u;
        S.ring[(out_base + prev_out + (k - prev_lit)) & ZRMASK] = S.lit_stage[k];
      }
      const uint64_t wend = out_base + span;
      const uint64_t msrc = mstart - r_of;
      if (__ballot(mine && sml > 0 && msrc + ZRING < wend)) out_fence(O);
      bool pending = mine && sml > 0, deferred = false;
      uint64_t pm;
      while ((pm = __ballot(pending)) != 0) {
        const int first = __builtin_ctzll(pm);
        const uint32_t F_lo = __builtin_amdgcn_readlane((uint32_t)mstart, first);
        const uint32_t F_hi = __builtin_amdgcn_readlane((uint32_t)(mstart >> 32), first);
        const uint64_t F = ((uint64_t)F_hi << 32) | F_lo;
        const uint32_t flen = __builtin_amdgcn_readlane(sml, first);
        const bool ready = pending && (lane == first || (sml <= 32 && msrc + sml <= F));
        // taint: source in an earlier block, or touching a deferred byte
        bool tnt = false;
        if (ready) {
          if (msrc < bstart) {
            tnt = true;
          } else if (sml <= 32 || lane != first) {
            tnt = tainted(msrc - bstart, msrc - bstart + min<uint32_t>(sml, r_of));
          }
        }
        if (flen > 32) {  // the first pending match is long: taint-check and copy cooperatively
          const uint32_t fd = __builtin_amdgcn_readlane(r_of, first);
          bool ft = __builtin_amdgcn_readlane((uint32_t)tnt, first) != 0;
          if (!ft) {
            const uint64_t ra = F - fd - bstart, rb = ra + min<uint32_t>(flen, fd);
            bool t = false;
            for (uint64_t w0 = (ra >> 5) + lane; w0 <= ((rb - 1) >> 5); w0 += 64)
              t |= tainted(max<uint64_t>(ra, w0 << 5), min<uint64_t>(rb, (w0 + 1) << 5));
            ft = __ballot(t) != 0;
          }
          if (ft) {
            for (uint64_t w0 = ((F - bstart) >> 5) + lane; w0 <= ((F - bstart + flen - 1) >> 5); w0 += 64)
              mark(max<uint64_t>(F - bstart, w0 << 5), min<uint64_t>(F - bstart + flen, (w0 + 1) << 5));
            if (lane == first) deferred = true;
          } else {
            const float inv = 1.0f / (float)fd;
            for (uint32_t i = lane; i < flen; i += 64) {
              uint32_t rm = i;
              if (fd < flen) {
                uint32_t q = (uint32_t)((float)i * inv);
                int32_t r = (int32_t)i - (int32_t)(q * fd);
                if (r < 0) r += fd;
                if (r >= (int32_t)fd) r -= fd;
                rm = (uint32_t)r;
              }
              S.ring[(F + i) & ZRMASK] = src_byte(S, O, F - fd + rm, wend);
            }
          }
          if (lane == first) pending = false;
          __syncthreads();
          continue;
        }
        if (ready) {
          if (tnt) {
            mark(mstart - bstart, mstart - bstart + sml);
            deferred = true;
          } else {
            for (uint32_t i0 = 0; i0 < sml; i0 += 4) {
              uint8_t v[4];
#pragma unroll
              for (int k = 0; k < 4; k++) {
                const uint32_t i = i0 + k;
                const uint32_t r = i < r_of ? i : i % r_of;
                v[k] = i < sml ? src_byte(S, O, msrc + r, wend) : (uint8_t)0;
              }
#pragma unroll
              for (int k = 0; k < 4; k++)
                if (i0 + k < sml) S.ring[(mstart + i0 + k) & ZRMASK] = v[k];
            }
          }
          pending = false;
        }
        __syncthreads();
      }
      // record this batch's deferred matches in output order
      const uint64_t dm = __ballot(deferred);
      const uint32_t nd = __builtin_popcountll(dm);
      if (nd) {
        if (deferred) {  // ndef + k <= base + lane: a consumed sequence slot
          const uint32_t k = ndef + __builtin_popcountll(dm & ((1ull << lane) - 1));
          defl[3 * k] = (uint32_t)mstart;
          defl[3 * k + 1] = r_of;
          defl[3 * k + 2] = sml;
        }
        ndef += nd;
      }
      __syncthreads();
      O.pos = wend;
      litpos += lspan;
      base += cnt;
    }
    if (!err) {
      if (litpos > regen) {
        err = ZG_CORRUPT_STREAM;
      } else {
        out_copy_global(S, O, lsrc + litpos, regen - litpos);
        if (O.pos != bstart + out_size) err = ZG_CORRUPT_STREAM;
      }
    }
    if (!err) blk_flush(S, out, O.flushed, O.pos);
    if (lane == 0) {
      if (err) status[item] = err;
      Bp->def_n = err ? 0u : ndef;
      Bp->def_done = 0;
    }
    __syncthreads();
  }
}

// One wave per item, 128 KiB of LDS: blocks in order; a block with deferred matches is loaded into
// LDS, its deferred matches (in output order) run there, and it is written back.
__global__ __launch_bounds__(64) void k_zstd_fixup(ZgItem *items, uint32_t *status, const ZBlk *blks,
                                                   uint32_t blk_cap, const uint32_t *nblk, const uint32_t *zmode,
                                                   uint8_t *dst, uint64_t slot_bytes, const uint32_t *seq_scratch,
                                                   uint64_t seq_cap) {
  __shared__ uint8_t img[BLOCK_MAX];
  const uint32_t item = blockIdx.x;
  const int lane = lane_id();
  if (zmode[item] != ZMODE_PARALLEL || status[item]) return;
  uint8_t *out = dst + (uint64_t)item * slot_bytes;
  const ZBlk *B = blks + (uint64_t)item * blk_cap;
  const uint32_t nb = nblk[item];
  uint32_t err = 0;
  uint64_t end = 0, fstart = 0;
  bool wrote = false;  // this wave has written output: its later loads of earlier blocks use sc1
  for (uint32_t bi = 0; bi < nb && !err; bi++) {
    const uint32_t flags = U(B[bi].flags);
    const uint64_t bstart = U(B[bi].out_off);
    const uint32_t bsize = U(B[bi].out_size);
    if (flags & ZBF_FIRST) fstart = bstart;
    end = bstart + bsize;
    const uint32_t ndef = (flags & 3) == ZB_CMP ? U(B[bi].def_n) : 0u;
    if (ndef) {
      const uint32_t *defl = seq_scratch + ((uint64_t)item * seq_cap + U(B[bi].seq_buf)) * 3;
      for (uint32_t o = 0; o < bsize; o += ZBATCH)
        lds_copy_in(img, ~0ull, o, out + bstart + o, min<uint32_t>(ZBATCH, bsize - o));
      __syncthreads();
      for (uint32_t k0 = 0; k0 < ndef; k0 += 64) {
        const uint32_t k = k0 + lane;
        const bool valid = k < ndef;
        uint64_t p = 0;
        uint32_t d = 1, len = 0;
        if (valid) {
          p = defl[3 * k];
          d = defl[3 * k + 1];
          len = defl[3 * k + 2];
        }
        const uint64_t src = p - d;
        bool pending = valid;
        uint64_t pm;
        while ((pm = __ballot(pending)) != 0) {
          const int first = __builtin_ctzll(pm);
          const uint32_t F_lo = __builtin_amdgcn_readlane((uint32_t)p, first);
          const uint32_t F_hi = __builtin_amdgcn_readlane((uint32_t)(p >> 32), first);
          const uint64_t F = ((uint64_t)F_hi << 32) | F_lo;
          const uint32_t flen = __builtin_amdgcn_readlane(len, first);
          if (flen > 32) {  // long: the whole wave copies it
            const uint32_t fd = __builtin_amdgcn_readlane(d, first);
            const float inv = 1.0f / (float)fd;
            for (uint32_t i = lane; i < flen; i += 64) {
              uint32_t rm = i;
              if (fd < flen) {
                uint32_t q = (uint32_t)((float)i * inv);
                int32_t r = (int32_t)i - (int32_t)(q * fd);
                if (r < 0) r += fd;
                if (r >= (int32_t)fd) r -= fd;
                rm = (uint32_t)r;
              }
              const uint64_t sb = F - fd + rm;
              img[F - bstart + i] = sb >= bstart ? img[sb - bstart] : (wrote ? load_out_byte(out + sb) : out[sb]);
            }
            if (lane == first) pending = false;
            __syncthreads();
            continue;
          }
          const bool ready = pending && len <= 32 && (lane == first || src + len <= F);
          if (ready) {
            for (uint32_t i0 = 0; i0 < len; i0 += 4) {
              uint8_t v[4];
#pragma unroll
              for (int j = 0; j < 4; j++) {
                const uint32_t i = i0 + j;
                const uint64_t sb = src + (i < d ? i : i % d);
                v[j] = i < len ? (sb >= bstart ? img[sb - bstart] : (wrote ? load_out_byte(out + sb) : out[sb]))
                               : (uint8_t)0;
              }
#pragma unroll
              for (int j = 0; j < 4; j++)
                if (i0 + j < len) img[p - bstart + i0 + j] = v[j];
            }
            pending = false;
          }
          __syncthreads();
        }
      }
      blk_flush_img(img, out, bstart, bstart + bsize);
      __builtin_amdgcn_s_waitcnt(0);  // written back before any later load of it
      __threadfence_block();
      wrote = true;
    }
    if ((flags & ZBF_LAST) && (flags & ZBF_CK)) {
      __threadfence();
      const uint64_t h = xxh64(out + fstart, end - fstart);
      if ((uint32_t)h != U(B[bi].ck)) err = ZG_CORRUPT_STREAM;
    }
  }
  if (lane == 0) {
    if (err) {
      status[item] = err;
    } else {
      items[item].src = (uint64_t)out;
      items[item].len = end;
    }
  }
}

void zstd_scratch_layout(uint64_t slot_bytes, uint32_t &blk_cap, uint64_t &blk_bytes, uint64_t &lit_stride,
                         uint64_t &seq_cap) {
  blk_cap = (uint32_t)std::min<uint64_t>(slot_bytes / 32768 + 64, 1u << 20);
  blk_bytes = sizeof(ZBlk);
  lit_stride = std::max<uint64_t>(slot_bytes, BLOCK_MAX + 64);
  lit_stride = (lit_stride + 255) & ~(uint64_t)255;
  seq_cap = slot_bytes / 4 + 1024;  // sequences per item (each decodes >= 3 bytes; typical >= 8)
}
hipError_t launch_zstd(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                       const ZstdScratch &Z, hipStream_t s) {
  if (!n_items) return hipSuccess;
  ZBlk *blks = (ZBlk *)Z.blks;
  hipLaunchKernelGGL(k_zstd_scan, dim3(n_items), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                     Z.lit_stride, Z.seq_cap);
  const uint64_t recs = (uint64_t)n_items * Z.blk_cap;
  const uint32_t grid = (uint32_t)std::min<uint64_t>(recs, 256 * 16);
  hipLaunchKernelGGL(k_zstd_blocks, dim3(grid), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                     n_items, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap);
  hipLaunchKernelGGL(k_zstd_plan, dim3(n_items), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                     slot_bytes);
  hipLaunchKernelGGL(k_zstd_exec_blocks, dim3(grid), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                     n_items, dst, slot_bytes, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap);
  hipLaunchKernelGGL(k_zstd_fixup, dim3(n_items), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                     dst, slot_bytes, Z.seq, Z.seq_cap);
  hipLaunchKernelGGL(k_zstd, dim3(n_items), dim3(64), 0, s, items, status, dst, slot_bytes, Z.lit, Z.lit_stride,
                     Z.mode);
  return hipGetLastError();
}

}  // namespace zgpu
