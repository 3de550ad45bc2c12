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
#include <type_traits>

#include "../common.hpp"
#include "launch.hpp"
#include "xxh.hpp"

#include <cstdlib>

namespace zgpu {

#ifdef ZG_PROFILE
// lab builds only (tools/lab/zstd_lab.cpp): k_zstd_exec per-phase shader-clock totals
__device__ unsigned long long g_zprof[13];
#define ZP_DECL uint64_t zp_acc[13] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}
#define ZP_T(v) const uint64_t v = clock64()
#define ZP_ADD(slot, t0) zp_acc[slot] += clock64() - (t0)
#define ZP_FLUSH do { if (__lane_id() == 0) for (int k_ = 0; k_ < 13; k_++) atomicAdd(&g_zprof[k_], (unsigned long long)zp_acc[k_]); } while (0)
#else
#define ZP_DECL
#define ZP_T(v)
#define ZP_ADD(slot, t0)
#define ZP_FLUSH
#endif
#ifdef ZG_SQ_PROFILE
// lab-only sequence-decoder profile: [0] table-build clocks, [1] decode clocks, [2] sequences,
// [3] blocks with sequences, [4] epochs (lane-group decoder), [5] records visited
__device__ unsigned long long g_sqprof[20];  // [8 + 4 t + mode]: table modes (LL, OF, ML) in the scan
#define SQP_T(v) const uint64_t v = clock64()
#define SQP_ADD(slot, x) do { if (__lane_id() == 0) atomicAdd(&g_sqprof[slot], (unsigned long long)(x)); } while (0)
#else
#define SQP_T(v)
#define SQP_ADD(slot, x) do { } while (0)
#endif

namespace {

constexpr int ZRING = 16384, ZRMASK = ZRING - 1;
constexpr int ZBATCH = 4096;         // max output span of one sequence batch
constexpr uint32_t ZBIG = 2048;      // sequences with a longer run are executed alone, chunked
constexpr uint32_t BLOCK_MAX = 131072;
constexpr uint32_t MAX_HUF_LOG = 12;
// a block's Huffman decoding table in the literal scratch, right before its literals: 2^12 u16
// entries + a 16-B header holding the table log (0: invalid description)
constexpr uint32_t HUF_TAB = (1u << MAX_HUF_LOG) * 2 + 16;
#ifndef ZG_HUF_SPLIT
#define ZG_HUF_SPLIT 1  // Huffman tables built by k_zstd_huf (one wave per block) ahead of k_zstd_lits
#endif
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
// LDS hand-off between the lanes of ONE wave (LDS operations of a wave complete in order): a compiler
// fence and a wave barrier. WS=false keeps the workgroup barrier (1-wave workgroups: the same thing).
template <bool WS>
__device__ __forceinline__ void zsync() {
  if (WS) {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
  } else {
    __syncthreads();
  }
}

// ---- uniform forward byte access (headers) ----
struct In {
  const uint8_t *p;
  uint64_t n;
  __device__ __forceinline__ uint32_t b(uint64_t i) const { return i < n ? U(p[i]) : 0u; }
  __device__ __forceinline__ uint32_t le16(uint64_t i) const { return b(i) | (b(i + 1) << 8); }
  __device__ __forceinline__ uint32_t le24(uint64_t i) const { return le16(i) | (b(i + 2) << 16); }
  __device__ __forceinline__ uint32_t le32(uint64_t i) const { return le24(i) | (b(i + 3) << 24); }
  __device__ __forceinline__ uint64_t le40(uint64_t i) const { return (uint64_t)le32(i) | ((uint64_t)b(i + 4) << 32); }
};

// ---- uniform forward byte access through a 256-byte register window (one load per window, not
// one dependent load per header byte): lane l holds word wk + l of the aligned item buffer ----
struct InW {
  const uint32_t *words;
  uint64_t n, nwords;
  uint32_t mis;
  int64_t wk;
  uint32_t w;
  __device__ InW(const uint8_t *p, uint64_t n_) : n(n_), wk(-1000000), w(0) {
    mis = (uint32_t)((uintptr_t)p & 3);
    words = (const uint32_t *)((uintptr_t)p - mis);
    nwords = (n_ + mis + 3) / 4;
  }
  __device__ __forceinline__ uint32_t b(uint64_t i) {
    if (i >= n) return 0u;
    const int64_t k = (int64_t)((i + mis) >> 2);
    if (k < wk || k >= wk + 64) {
      wk = k;
      const uint64_t kl = (uint64_t)k + lane_id();
      w = kl < nwords ? words[kl] : 0u;
    }
    const uint32_t word = U(__builtin_amdgcn_readlane(w, (int)(k - wk)));
    return (word >> (8 * ((i + mis) & 3))) & 0xFFu;
  }
  __device__ __forceinline__ uint32_t le16(uint64_t i) { return b(i) | (b(i + 1) << 8); }
  __device__ __forceinline__ uint32_t le24(uint64_t i) { return le16(i) | (b(i + 2) << 16); }
  __device__ __forceinline__ uint32_t le32(uint64_t i) { return le24(i) | (b(i + 3) << 24); }
  // bytes [i, i + 5) in one go (two readlanes), zero past the item
  __device__ __forceinline__ uint64_t le40(uint64_t i) {
    if (i + 5 > n) return (uint64_t)le32(i) | ((uint64_t)b(i + 4) << 32);
    const int64_t k = (int64_t)((i + mis) >> 2);
    if (k < wk || k + 1 >= wk + 64) {
      wk = k;
      const uint64_t kl = (uint64_t)k + lane_id();
      w = kl < nwords ? words[kl] : 0u;
    }
    const uint64_t v = (uint64_t)U(__builtin_amdgcn_readlane(w, (int)(k - wk))) |
                       ((uint64_t)U(__builtin_amdgcn_readlane(w, (int)(k - wk + 1))) << 32);
    return v >> (8 * ((i + mis) & 3));
  }
};

// ---- per-lane forward byte access (k_zstd_scan's block parse: one lane per block) ----
struct InL {
  const uint32_t *words;
  uint64_t n, nwords;
  uint32_t mis;
  __device__ InL(const uint8_t *p, uint64_t n_) : n(n_) {
    mis = (uint32_t)((uintptr_t)p & 3);
    words = (const uint32_t *)((uintptr_t)p - mis);
    nwords = (n_ + mis + 3) / 4;
  }
  __device__ __forceinline__ uint32_t w(uint64_t k) const { return k < nwords ? words[k] : 0u; }
  __device__ __forceinline__ uint32_t b(uint64_t i) const {
    if (i >= n) return 0u;
    return (w((i + mis) >> 2) >> (8 * ((i + mis) & 3))) & 0xFFu;
  }
  __device__ __forceinline__ uint64_t le40(uint64_t i) const {  // zero past the item
    if (i + 5 > n) {
      uint64_t v = 0;
      for (uint32_t k = 0; k < 5; k++) v |= (uint64_t)b(i + k) << (8 * k);
      return v;
    }
    const uint64_t k = (i + mis) >> 2;
    const uint64_t v = (uint64_t)w(k) | ((uint64_t)w(k + 1) << 32);
    return (v >> (8 * ((i + mis) & 3))) & 0xFFFFFFFFFFull;
  }
  __device__ __forceinline__ uint32_t le16(uint64_t i) const { return (uint32_t)le40(i) & 0xFFFFu; }
  __device__ __forceinline__ uint32_t le24(uint64_t i) const { return (uint32_t)le40(i) & 0xFFFFFFu; }
  __device__ __forceinline__ uint32_t le32(uint64_t i) const { return (uint32_t)le40(i); }
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
// STORE = false: only the description's size (k_zstd_scan's per-lane block parse; norm unused).
template <class IN, bool STORE = true>
__device__ uint32_t read_ncount(IN &I, uint64_t off, uint64_t avail, int16_t *norm, uint32_t max_sym,
                                uint32_t max_log, uint32_t &acc_log, uint32_t &nsym) {
  uint64_t bit = 0;
  auto peek32 = [&](uint64_t b) -> uint32_t {
    const uint64_t byte = off + (b >> 3);
    return (uint32_t)(I.le40(byte) >> (b & 7));
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
  if constexpr (STORE)
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
    if constexpr (STORE) norm[s] = (int16_t)count;
    s++;
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

// Build an FSE decoding table from normalized counts (FSE_buildDTable semantics, RFC 8878 4.1.1),
// all 64 lanes of the wave at once (lane s owns symbol s; nsym <= 64). The spread visits positions
// p_i = i * step & mask, skipping those above the low-probability region; the k-th visited position
// takes the symbol whose cumulative count range holds k, so each lane places its share of i directly
// (a prefix count of valid i, a 6-step binary search of the cumulative counts). A position's state
// counter is its symbol's count plus the symbol's earlier occurrences in table order: per 64
// positions, the lanes holding one symbol find each other with 6 ballots (symbol bits). The old
// scalar form walked the table twice, one LDS round trip per position (~0.1 ms per table).
// `norm` is consumed: it holds the per-symbol running counters afterwards.
template <bool WS = false>
__device__ void build_fse(Fse *T, int16_t *norm, uint32_t nsym, uint32_t acc_log, uint32_t *tmp) {
  (void)tmp;
  const uint32_t size = 1u << acc_log, mask = size - 1;
  const int lane = lane_id();
  const uint64_t lt = (1ull << lane) - 1;
  const int32_t c = lane < (int)nsym ? (int32_t)norm[lane] : 0;
  const uint64_t lowm = __ballot(c == -1);
  const uint32_t nlow = (uint32_t)__popcll(lowm);
  const uint32_t high = size - 1 - nlow;
  if (c == -1) T[size - 1 - (uint32_t)__popcll(lowm & lt)].sym = (uint8_t)lane;  // the top, in symbol order
  // cumulative counts: start_s (exclusive); past nsym a value no k reaches
  const uint32_t cnt = c > 0 ? (uint32_t)c : 0u;
  uint32_t inc = cnt;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(inc, o, 64);
    if (lane >= o) inc += t;
  }
  const uint32_t start = lane < (int)nsym ? inc - cnt : 0xFFFFu;
  const uint32_t step = (size >> 1) + (size >> 3) + 3;
  const uint32_t per = (size + 63) >> 6, i0 = (uint32_t)lane * per;
  uint32_t nv = 0;
  for (uint32_t j = 0; j < per; j++) {
    const uint32_t i = i0 + j;
    nv += (i < size && ((i * step) & mask) <= high) ? 1u : 0u;
  }
  uint32_t kx = nv;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t t = __shfl_up(kx, o, 64);
    if (lane >= o) kx += t;
  }
  uint32_t k = kx - nv;  // rank of this lane's first valid i
  for (uint32_t j = 0; j < per; j++) {
    const uint32_t i = i0 + j, pos = (i * step) & mask;
    const bool v = i < size && pos <= high;
    uint32_t sl = 0;
    for (int st = 32; st; st >>= 1) {
      const uint32_t sv = (uint32_t)__shfl((int)start, (int)(sl + st), 64);
      if (sv <= k) sl += st;
    }
    if (v) {
      T[pos].sym = (uint8_t)sl;
      k++;
    }
  }
  if (lane < (int)nsym) norm[lane] = (int16_t)(c == -1 ? 1 : c);
  zsync<WS>();
  for (uint32_t b = 0; b < size; b += 64) {
    const uint32_t u = b + (uint32_t)lane;
    const bool v = u < size;
    const uint32_t s = v ? (uint32_t)T[u].sym : 0u;
    uint64_t peer = __ballot(v);
#pragma unroll
    for (int bit = 0; bit < 6; bit++) {
      const bool on = (s >> bit) & 1;
      const uint64_t bb = __ballot(v && on);
      peer &= on ? bb : ~bb;
    }
    const uint32_t rank = (uint32_t)__popcll(peer & lt), pc = (uint32_t)__popcll(peer);
    const uint32_t nx = v ? (uint32_t)(uint16_t)norm[s] : 0u, jn = nx + rank;
    zsync<WS>();
    if (v && rank == 0) norm[s] = (int16_t)(nx + pc);
    if (v) {
      const uint32_t nb = acc_log - highbit(jn);
      T[u].nb = (uint8_t)nb;
      T[u].base = (uint16_t)((jn << nb) - size);
    }
    zsync<WS>();
  }
}

template <bool WS = false>
__device__ void build_fse_rle(Fse *T, uint32_t sym) {
  if (lane_id() == 0) {
    T[0].sym = (uint8_t)sym;
    T[0].nb = 0;
    T[0].base = 0;
  }
  zsync<WS>();
}

template <bool WS = false>
__device__ void build_fse_default(Fse *T, const int16_t *def, uint32_t nsym, uint32_t acc_log, int16_t *norm,
                                  uint32_t *tmp) {  // norm: scratch
  for (uint32_t s = lane_id(); s < nsym; s += 64) norm[s] = def[s];
  zsync<WS>();
  build_fse<WS>(T, norm, nsym, acc_log, tmp);
}

// ---- Huffman (literals) ----
// Parse the tree description and build the decoding table. Returns bytes consumed, 0 on error.
template <class SM, bool WS = false>
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
    zsync<WS>();
  } else {
    used = 1 + hb;
    if (used > avail || hb == 0) return 0;
    uint32_t acc, ns;
    In Ic = I;
    const uint32_t h = read_ncount(Ic, off + 1, hb, S.norm, 15, 6, acc, ns);
    if (!h) return 0;
    zsync<WS>();
    build_fse<WS>(S.wt, S.norm, ns, acc, S.tmp);
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
    zsync<WS>();
  }
  // weights -> table log, implied last weight
  if (lane < 16) S.tmp[lane] = 0;
  zsync<WS>();
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
  zsync<WS>();
  const uint32_t nsym = nw + 1;
  // rank counts
  for (uint32_t n = lane; n < nsym; n += 64) {
    const uint32_t w = S.weights[n];
    if (w) atomicAdd(&S.tmp[w], 1u);
  }
  zsync<WS>();
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
  zsync<WS>();
  // fill: entries of weight class W occupy [start[W], start[W] + cnt[W] * 2^(W-1))
  const uint32_t size = 1u << tl;
  for (uint32_t e = lane; e < size; e += 64) {
    uint32_t W = 1;
    while (W < tl && e >= start[W + 1]) W++;
    const uint32_t len = 1u << (W - 1);
    const uint32_t sym = S.hsorted[sbase[W] + (e - start[W]) / len];
    S.huf[e] = (uint16_t)(((tl + 1 - W) << 8) | sym);
  }
  zsync<WS>();
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
typedef __attribute__((address_space(1))) uint32_t gu32;  // global-memory word (no flat access)
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

// The serial decoder: one wave decodes one item. lit: per-item literal scratch (BLOCK_MAX + 64 bytes
// each).
__device__ __attribute__((noinline)) void zstd_serial_item(ZSmem &S, uint32_t item, ZgItem *items, uint32_t *status,
                                                           uint8_t *dst, uint64_t slot_bytes, uint8_t *lit_scratch,
                                                           uint64_t lit_stride) {
  const ZgItem it = items[item];
  if (status[item] || (it.flags & ZG_ITEM_FILL)) return;
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

// Serial fallback. ser_list == NULL: one wave per item, every item the scan marked ZMODE_SERIAL (the
// standalone serial decoder, zmode NULL: all items). Otherwise a small persistent grid over the
// items k_zstd_scan compacted into ser_list[0 .. *ser_count): with none, every wave exits at once.
__global__ __launch_bounds__(64) void k_zstd(ZgItem *items, uint32_t *status, uint8_t *dst, uint64_t slot_bytes,
                                             uint8_t *lit_scratch, uint64_t lit_stride, const uint32_t *zmode,
                                             const uint32_t *ser_list, const unsigned long long *ser_count) {
  __shared__ ZSmem S;
  if (ser_list) {
    const uint64_t n = *ser_count;
    for (uint64_t k = blockIdx.x; k < n; k += gridDim.x) {
      zstd_serial_item(S, ser_list[k], items, status, dst, slot_bytes, lit_scratch, lit_stride);
      __syncthreads();
    }
    return;
  }
  const uint32_t item = blockIdx.x;
  if (zmode && zmode[item] != ZMODE_SERIAL) return;  // decoded by the block-parallel path
  zstd_serial_item(S, item, items, status, dst, slot_bytes, lit_scratch, lit_stride);
}

// =================================================================================================
// Block-parallel path (items whose blocks fit the scratch; k_zstd above is the fallback).
//
// A zstd frame is a chain of blocks whose sizes are in their 3-byte headers, so the entropy decoding
// parallelises over blocks; the sequence execution (LZ77 copies, which in real data reach across
// blocks all the time) runs per item:
//   k_zstd_scan    one wave per item: walk frames and block headers, parse each compressed block's
//                  literal / sequence section headers, resolve "treeless" literals and "repeat" FSE
//                  modes to the block that defined the table; one ZBlk record per block
//   k_zstd_lits    256 threads per block: Huffman literals into the literal scratch (all lanes
//                  decode, see the kernel)
//   k_zstd_blocks  one wave per block: FSE sequences into the sequence scratch. Repeat offsets are
//                  resolved symbolically ("incoming rep k, minus j"), so no block waits for its
//                  predecessor; the block's outgoing rep state is kept in the same symbolic form
//   k_zstd_plan    one wave per item: block output offsets (prefix sum), concrete incoming rep state
//                  per block (composing the symbolic transforms), frame content size checks
//   k_zstd_exec_item  one wave per item: sequence execution through a 64 KiB LDS ring, far match
//                  sources staged per batch; frame checksums
// =================================================================================================
namespace {

constexpr uint32_t ZB_RAW = 0, ZB_RLE = 1, ZB_CMP = 2;
constexpr uint32_t ZBF_FIRST = 1u << 8, ZBF_LAST = 1u << 9, ZBF_FCS = 1u << 10, ZBF_CK = 1u << 11;
constexpr uint32_t ZSYM = 0x80000000u;      // symbolic offset: ZSYM | slot << 24 | minus
// normalized-count scratch: per block record 3 tables x 64 int16 (counts of symbols 0..52; [62] the
// accuracy log, [63] the symbol count)
constexpr uint32_t ZNORM = 3 * 64;

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
  uint32_t norm_src[3];       // fse: 1 + the block whose description k_zstd_scan parsed into the normalized
                              // count scratch (ZNORM per block), 0: none (k_zstd_blocks parses tab_off)
  uint32_t lit_buf;           // literal scratch offset (huffman / rle literals)
  uint32_t seq_buf;           // first sequence in the item's sequence scratch
  uint32_t ck;                // frame checksum (last block of a frame with one)
  uint64_t fcs;               // frame content size (first block of a frame with one)
  uint32_t rep_out[3];        // outgoing rep offsets (symbolic in the incoming ones)
  uint32_t rep_in[3];         // incoming rep offsets (concrete, from k_zstd_plan)
  uint32_t out_off;           // item-relative output offset (k_zstd_plan)
  uint32_t frame_off;         // output offset of the block's frame
  // how far the block's matches reach back from its start (k_zstd_blocks): max(offset - position)
  // over concrete offsets, min(minus + position) per rep slot over symbolic ones
  int32_t reach_c;
  uint32_t reach_m[3];
  uint32_t seg;               // 1: an executor segment starts at this block (k_zstd_plan)
  uint64_t in_src;            // record 0: the item's encoded bytes (k_zstd_plan; the executor's
                              // last segment rewrites the item record while others may still start)
};

struct ZScanSmem {
  int16_t norm[64];
};

// literals (Huffman table) and sequences (FSE tables) are decoded one after the other: the two
// table sets share LDS
// sequence decoding table entry: the code's value base and extra-bit count with the FSE transition
// (one 8-byte LDS read per table per sequence); nbx == 0xFF marks a code outside the format
struct SeqX {
  uint32_t base;
  uint16_t next;
  uint8_t nb, nbx;
};
#ifndef ZG_BLK_WPE
#define ZG_BLK_WPE 6  // waves per SIMD k_zstd_blocks is compiled for
#endif
#ifndef ZG_SEQ_PACK
#define ZG_SEQ_PACK 1  // 4-byte sequence tables (below); 0: 8-byte SeqX
#endif
#ifndef ZG_SEQ_REP_SEL
#define ZG_SEQ_REP_SEL 0  // 1: repeat-offset update as selects (lab A/B r04ae: blocks 3.60 -> 3.94-4.17 ms, off)
#endif
#ifndef ZG_SEQ_SPLIT
#define ZG_SEQ_SPLIT 1  // k_zstd_blocks walks only the FSE state chain; fields and reps per 64-batch by lanes
#endif
#ifndef ZG_SEQ_ONE_FSE
#define ZG_SEQ_ONE_FSE 1  // one FSE scratch table, folded into its SeqX table at once (0: three tables)
#endif
#if ZG_SEQ_PACK
// 4-byte sequence decoding entry: bits 0-8 next state base, 9-12 state bits, 13-17 value extra bits,
// 18-23 code (LL/ML: index of its value base; OF: the offset code itself, value base 1 << code), bit
// 31 a code outside the format. Everything the bit stream's order depends on (state and extra bit
// counts) is in the entry; the LL/ML value base is a scalar constant load off that critical chain.
// Each table is built as FSE entries in place (also 4 bytes) and repacked entry by entry, so the
// three tables take 5 KiB of LDS (the 8-byte SeqX tables and their FSE scratch took 12 KiB): ~2x
// the waves per CU for this latency-bound serial decoder.
constexpr uint32_t SQ_BAD = 0x80000000u;
__device__ __forceinline__ uint32_t sq_pack(uint32_t next, uint32_t nb, uint32_t nbx, uint32_t code) {
  return next | (nb << 9) | (nbx << 13) | (code << 18);
}
struct ZDecSmem {
  uint32_t xl[512], xm[512], xo[256];
  int16_t norm[64];
  uint32_t tmp[32];
};
#else
struct ZDecSmem {
#if ZG_SEQ_ONE_FSE
  Fse fse[512];  // one FSE table at a time: built, then folded into its SeqX table
#else
  Fse ll[512], ml[512], of[256];
#endif
  SeqX xl[512], xm[512], xo[256];
  int16_t norm[64];
  uint32_t tmp[32];
};
#endif



__device__ __forceinline__ uint32_t sym_dec(uint32_t x) { return (x & ZSYM) ? x + 1 : x - 1; }
__device__ __forceinline__ uint32_t sym_eval(uint32_t x, uint32_t r0, uint32_t r1, uint32_t r2) {
  if (!(x & ZSYM)) return x;
  const uint32_t slot = (x >> 24) & 3, minus = x & 0xFFFFFF;
  return (slot == 0 ? r0 : slot == 1 ? r1 : r2) - minus;
}

}  // namespace

// Block records per item the record-strided kernels walk: blk_cap, or the batch's largest block count
// (k_zstd_scan's atomicMax; a blosc table of 256 KiB frames has 2 of its 72 record slots in use)
__device__ __forceinline__ uint64_t rec_blocks(uint32_t blk_cap, const unsigned long long *max_nblk) {
  return max_nblk ? min<uint64_t>(blk_cap, *max_nblk) : blk_cap;
}

// The uniform one-wave frame walk: every block header and section header in order, one register
// window load per position. k_zstd_scan below takes it for frames of more blocks than its LDS holds.
__device__ __attribute__((noinline)) void scan_uniform(ZScanSmem &S, uint32_t item, const ZgItem *items,
                                                        uint32_t *status, ZBlk *blks, uint32_t blk_cap,
                                                        uint32_t *nblk, uint32_t *zmode, uint64_t lit_stride,
                                                        uint64_t seq_cap, uint32_t force_serial,
                                                        unsigned long long *counters, uint32_t *ser_list,
                                                        unsigned long long *ser_count, unsigned long long *max_nblk) {
  const ZgItem it = items[item];
  const int lane = lane_id();
  if (status[item] || (it.flags & ZG_ITEM_FILL)) {
    if (lane == 0) { nblk[item] = 0; zmode[item] = ZMODE_SKIP; }
    return;
  }
  if (it.len >= 0xFFFFFFF0ull || force_serial) {  // 32-bit record offsets: decode such items serially
    if (lane == 0) {
      nblk[item] = 0;
      zmode[item] = ZMODE_SERIAL;
      if (counters) atomicAdd(&counters[0], 1ull);
      if (ser_list) ser_list[atomicAdd(ser_count, 1ull)] = item;
    }
    return;
  }
  const uint8_t *in = (const uint8_t *)it.src;
  InW I(in, it.len);
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
#if ZG_HUF_SPLIT
          if (ltype >= 2) lit_used = ((lit_used + 15) & ~(uint64_t)15) + HUF_TAB;  // the block's table
#endif
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
#ifdef ZG_SQ_PROFILE
          if (lane == 0) for (int t = 0; t < 3; t++) atomicAdd(&g_sqprof[8 + t * 4 + mm[t]], 1ull);
#endif
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
    if (counters && (serial || !err)) atomicAdd(&counters[serial ? 0 : 1], 1ull);  // serial / block-parallel items
    if (serial && ser_list) ser_list[atomicAdd(ser_count, 1ull)] = item;
    if (max_nblk && !serial && !err) atomicMax(max_nblk, (unsigned long long)nb);
  }
}

// k_zstd_scan: one wave per item, in three passes over the frame. (A) a uniform walk of the frame and
// block headers alone -- one dependent load per block (the next header is bsize bytes on), recorded in
// LDS; (B) every compressed block's literal / sequence section headers and FSE table descriptions
// parsed by its own lane (per-lane loads: 64 blocks at once); (C) a uniform pass over the LDS records in
// block order: treeless literals and repeat table modes resolved to the block that defined them, the
// literal / sequence scratch offsets, the first error or scratch overflow. The one-walk form took
// ~22 us per 128 KiB block of a C5 frame (dependent header reads in series: 2.8 ms a frame).
#ifndef ZG_SCAN_LDS_BLOCKS
#define ZG_SCAN_LDS_BLOCKS 144
#endif
constexpr uint32_t SCAN_LB = ZG_SCAN_LDS_BLOCKS;
struct ZScan2Smem {
  ZBlk R[SCAN_LB];
  uint32_t err[SCAN_LB];
};
constexpr uint32_t TREE_NONE = 0xFFFFFFFFu;

__global__ __launch_bounds__(64) void k_zstd_scan(const ZgItem *items, uint32_t *status, ZBlk *blks,
                                                  uint32_t blk_cap, uint32_t *nblk, uint32_t *zmode,
                                                  uint64_t lit_stride, uint64_t seq_cap, uint32_t force_serial,
                                                  unsigned long long *counters, uint32_t *ser_list,
                                                  unsigned long long *ser_count, unsigned long long *max_nblk,
                                                  int16_t *norms) {
  __shared__ ZScanSmem S;
  __shared__ ZScan2Smem Q;
  const uint32_t item = blockIdx.x;
  const ZgItem it = items[item];
  const int lane = lane_id();
  if (status[item] || (it.flags & ZG_ITEM_FILL)) {
    if (lane == 0) { nblk[item] = 0; zmode[item] = ZMODE_SKIP; }
    return;
  }
  if (it.len >= 0xFFFFFFF0ull || force_serial) {  // 32-bit record offsets: decode such items serially
    if (lane == 0) {
      nblk[item] = 0;
      zmode[item] = ZMODE_SERIAL;
      if (counters) atomicAdd(&counters[0], 1ull);
      if (ser_list) ser_list[atomicAdd(ser_count, 1ull)] = item;
    }
    return;
  }
  const uint8_t *in = (const uint8_t *)it.src;
  InW I(in, it.len);
  // ---- (A) frame and block headers ----
  uint32_t nb = 0, err = 0;
  bool serial = false, any_frame = false, full = false;
  uint64_t ip = 0;
#define SFAIL(code) { err = (code); break; }
  while (!err && !serial && !full && ip < it.len) {
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
    while (!last && !err) {
      if (nb == blk_cap) { serial = true; break; }
      if (nb == SCAN_LB) { full = true; break; }
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
        R.in_size = bsize;
        ip += bsize;
      }
      if (last && has_ck) {
        if (ip + 4 > it.len) SFAIL(ZG_CORRUPT_STREAM);
        R.flags |= ZBF_CK;
        R.ck = I.le32(ip);
        ip += 4;
      }
      if (lane == 0) Q.R[nb] = R;
      nb++;
    }
  }
#undef SFAIL
  if (full) {  // more blocks than the LDS records hold: the one-walk form
    scan_uniform(S, item, items, status, blks, blk_cap, nblk, zmode, lit_stride, seq_cap, force_serial, counters,
                 ser_list, ser_count, max_nblk);
    return;
  }
  __syncthreads();
  // ---- (B) compressed blocks' sections, one lane per block ----
  {
    const InL L(in, it.len);
    for (uint32_t bi = lane; bi < nb; bi += 64) {
      ZBlk &R = Q.R[bi];
      uint32_t e = 0;
      if ((R.flags & 3) == ZB_CMP) {
        do {
          const uint64_t bend = (uint64_t)R.in_off + R.in_size;
          uint64_t p = R.in_off;
          const uint32_t b0 = L.b(p);
          const uint32_t ltype = b0 & 3, sfmt = (b0 >> 2) & 3;
          uint32_t regen = 0, csize = 0, lhdr = 0, four = 0;
          if (ltype <= 1) {
            if (sfmt == 0 || sfmt == 2) { regen = b0 >> 3; lhdr = 1; }
            else if (sfmt == 1) { regen = (b0 >> 4) | (L.b(p + 1) << 4); lhdr = 2; }
            else { regen = (b0 >> 4) | (L.b(p + 1) << 4) | (L.b(p + 2) << 12); lhdr = 3; }
          } else {
            four = sfmt == 0 ? 0 : 1;
            if (sfmt <= 1) { const uint32_t v = L.le24(p); regen = (v >> 4) & 0x3FF; csize = (v >> 14) & 0x3FF; lhdr = 3; }
            else if (sfmt == 2) { const uint32_t v = L.le32(p); regen = (v >> 4) & 0x3FFF; csize = (v >> 18) & 0x3FFF; lhdr = 4; }
            else {
              const uint64_t v = L.le40(p);
              regen = (uint32_t)(v >> 4) & 0x3FFFF; csize = (uint32_t)(v >> 22) & 0x3FFFF; lhdr = 5;
            }
          }
          if (regen > BLOCK_MAX) { e = ZG_CORRUPT_STREAM; break; }
          p += lhdr;
          R.flags |= (ltype << 2) | (four << 4);
          R.regen = regen;
          R.huf_off = TREE_NONE;
          if (ltype == 0) {
            if (p + regen > bend) { e = ZG_CORRUPT_STREAM; break; }
            R.lit_off = (uint32_t)p;
            R.lit_end = (uint32_t)(p + regen);
            p += regen;
          } else if (ltype == 1) {
            if (p + 1 > bend) { e = ZG_CORRUPT_STREAM; break; }
            R.lit_off = (uint32_t)p;
            p += 1;
          } else {
            if (p + csize > bend) { e = ZG_CORRUPT_STREAM; break; }
            uint64_t q = p;
            if (ltype == 2) {  // tree description: FSE-compressed weights (hb < 128) or 4-bit weights
              const uint32_t hb = L.b(q);
              const uint32_t tsz = hb < 128 ? 1 + hb : 1 + (hb - 127 + 1) / 2;
              if (hb == 0 || tsz > csize) { e = ZG_CORRUPT_STREAM; break; }
              R.huf_off = (uint32_t)q;  // this block's own tree
              q += tsz;
            }
            R.lit_off = (uint32_t)q;
            R.lit_end = (uint32_t)(p + csize);
            p += csize;
          }
          if (p >= bend) { e = ZG_CORRUPT_STREAM; break; }
          uint32_t nseq = 0;
          const uint32_t c0 = L.b(p);
          if (c0 < 128) { nseq = c0; p += 1; }
          else if (c0 < 255) { nseq = ((c0 - 128) << 8) + L.b(p + 1); p += 2; }
          else { nseq = L.le16(p + 1) + 0x7F00; p += 3; }
          R.nseq = nseq;
          if (nseq) {
            if (p >= bend) { e = ZG_CORRUPT_STREAM; break; }
            const uint32_t modes = L.b(p++);
            if (modes & 3) { e = ZG_CORRUPT_STREAM; break; }
            const uint32_t mm[3] = {modes >> 6, (modes >> 4) & 3, (modes >> 2) & 3};  // LL, OF, ML
            uint32_t raw = 0;
            for (int t = 0; t < 3 && !e; t++) {
              const uint32_t maxs = t == 0 ? 35 : t == 1 ? 31 : 52, maxl = t == 0 ? 9 : t == 1 ? 8 : 9;
              raw |= mm[t] << (2 * t);  // 3: repeat, resolved in (C)
              R.tab_off[t] = 0;
              if (mm[t] == 1) {
                if (p >= bend || L.b(p) > maxs) { e = ZG_CORRUPT_STREAM; break; }
                R.tab_off[t] = (uint32_t)p;
                p += 1;
              } else if (mm[t] == 2) {
                uint32_t acc, ns, used;
                if (norms) {  // the counts kept for k_zstd_blocks (it then skips the serial parse)
                  int16_t *nr = norms + ((uint64_t)item * blk_cap + bi) * ZNORM + t * 64;
                  used = read_ncount<const InL, true>(L, p, bend - p, nr, maxs, maxl, acc, ns);
                  nr[62] = (int16_t)acc;
                  nr[63] = (int16_t)ns;
                } else {
                  used = read_ncount<const InL, false>(L, p, bend - p, nullptr, maxs, maxl, acc, ns);
                }
                if (!used) { e = ZG_CORRUPT_STREAM; break; }
                R.tab_off[t] = (uint32_t)p;
                p += used;
              }
            }
            if (e) break;
            R.tab_mode = raw;
            R.seq_off = (uint32_t)p;
            R.seq_end = (uint32_t)bend;
          } else if (p != bend) {
            e = ZG_CORRUPT_STREAM;
            break;
          }
        } while (false);
      }
      Q.err[bi] = e;
    }
  }
  __syncthreads();
  // ---- (C) in block order: tree / table references, scratch offsets, the first error or overflow ----
  uint32_t nbv = nb;
  if (!serial && !err) {
    uint64_t lit_used = 0, seq_used = 0;
    uint32_t huf_src = TREE_NONE, tmode[3] = {3, 3, 3}, toff[3] = {0, 0, 0};  // 3 = no table yet
    uint32_t tsrc[3] = {0, 0, 0};  // 1 + the block that defined each table (its counts in `norms`)
    for (uint32_t bi = 0; bi < nb; bi++) {
      ZBlk &R = Q.R[bi];
      const uint32_t flags = U(R.flags);
      if (flags & ZBF_FIRST) {  // a new frame: no tree, no tables
        huf_src = TREE_NONE;
        tmode[0] = tmode[1] = tmode[2] = 3;
      }
      if ((flags & 3) != ZB_CMP) continue;
      if (U(Q.err[bi])) { err = ZG_CORRUPT_STREAM; nbv = bi; break; }
      const uint32_t ltype = (flags >> 2) & 3, regen = U(R.regen), nseq = U(R.nseq);
      uint32_t huf = 0;
      if (ltype == 2) huf_src = huf = U(R.huf_off);
      else if (ltype == 3) {
        if (huf_src == TREE_NONE) { err = ZG_CORRUPT_STREAM; nbv = bi; break; }  // treeless without a tree
        huf = huf_src;
      }
      uint32_t lit_buf = 0;
      if (ltype != 0) {  // rle / huffman literals are materialised in the literal scratch
#if ZG_HUF_SPLIT
        if (ltype >= 2) lit_used = ((lit_used + 15) & ~(uint64_t)15) + HUF_TAB;  // the block's table
#endif
        lit_buf = (uint32_t)lit_used;
        lit_used += regen;
        if (lit_used > lit_stride) { serial = true; break; }
      }
      uint32_t tab_mode = 0, seq_buf = 0;
      if (nseq) {
        const uint32_t raw = U(R.tab_mode);
        bool ok = true;
        for (int t = 0; t < 3; t++) {
          const uint32_t m = (raw >> (2 * t)) & 3;
          if (m == 3) {
            if (tmode[t] == 3) ok = false;  // repeat mode without a previous table
          } else {
            tmode[t] = m;
            toff[t] = U(R.tab_off[t]);
            tsrc[t] = (m == 2 && norms) ? bi + 1 : 0u;
          }
        }
        if (!ok) { err = ZG_CORRUPT_STREAM; nbv = bi; break; }
        tab_mode = tmode[0] | (tmode[1] << 2) | (tmode[2] << 4);
        seq_buf = (uint32_t)seq_used;
        seq_used += nseq;
        if (seq_used > seq_cap) { serial = true; break; }
      }
      if (lane == 0) {
        R.huf_off = huf;
        R.lit_buf = lit_buf;
        R.tab_mode = tab_mode;
        if (nseq) {
          R.tab_off[0] = toff[0];
          R.tab_off[1] = toff[1];
          R.tab_off[2] = toff[2];
          R.norm_src[0] = tsrc[0];
          R.norm_src[1] = tsrc[1];
          R.norm_src[2] = tsrc[2];
        }
        R.seq_buf = seq_buf;
      }
    }
  }
  if (!err && !serial && !any_frame) err = ZG_CORRUPT_STREAM;
  __syncthreads();
  // ---- (D) the records, one lane per block ----
  if (!serial && !err) {
    ZBlk *B = blks + (uint64_t)item * blk_cap;
    for (uint32_t bi = lane; bi < nb; bi += 64) B[bi] = Q.R[bi];
  }
  if (lane == 0) {
    nblk[item] = serial ? 0u : nbv;
    zmode[item] = serial ? ZMODE_SERIAL : (err ? ZMODE_SKIP : ZMODE_PARALLEL);
    if (err && !serial) status[item] = err;
    if (counters && (serial || !err)) atomicAdd(&counters[serial ? 0 : 1], 1ull);  // serial / block-parallel items
    if (serial && ser_list) ser_list[atomicAdd(ser_count, 1ull)] = item;
    if (max_nblk && !serial && !err) atomicMax(max_nblk, (unsigned long long)nb);
  }
}

// One wave per (item, block) record, grid-stride. Sequences land as {ll, ml, offset symbol}.
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ZG_BLK_WPE, 8))) void k_zstd_blocks(const ZgItem *items, uint32_t *status, ZBlk *blks,
                                                    uint32_t blk_cap, const uint32_t *nblk,
                                                    const uint32_t *zmode, uint32_t n_items, uint8_t *lit_scratch,
                                                    uint64_t lit_stride, uint32_t *seq_scratch, uint64_t seq_cap,
                                                    const unsigned long long *max_nblk, const int16_t *norms) {
  __shared__ ZDecSmem S;
  const int lane = lane_id();
  const uint64_t total = (uint64_t)n_items * rec_blocks(blk_cap, max_nblk);
  for (uint64_t g = blockIdx.x; g < total; g += gridDim.x) {
    // block-major record order: block bi of every item before block bi+1 of any, so that items
    // with few blocks (many small frames, e.g. blosc streams) spread over all workgroups
    const uint32_t item = (uint32_t)(g % n_items), bi = (uint32_t)(g / n_items);
    if (bi >= nblk[item] || zmode[item] != ZMODE_PARALLEL) continue;
    ZBlk *Bp = blks + (uint64_t)item * blk_cap + bi;
    const uint32_t flags = U(Bp->flags);
    if ((flags & 3) != ZB_CMP) continue;
    const ZgItem it = items[item];
    const uint8_t *in = (const uint8_t *)it.src;
    const In I{in, it.len};
    const uint32_t ltype = (flags >> 2) & 3, regen = U(Bp->regen);
    uint8_t *lit = lit_scratch + (uint64_t)item * lit_stride + U(Bp->lit_buf);
    bool bad = false;
    __syncthreads();  // the previous record's table reads are done before they are rebuilt
    // literals: k_zstd_lits
    (void)ltype;
    (void)regen;
    (void)lit;
    // ---- sequences ----
    const uint32_t nseq = U(Bp->nseq);
    uint64_t sum_ll = 0, sum_ml = 0;
    uint32_t r0 = ZSYM | (0u << 24), r1 = ZSYM | (1u << 24), r2 = ZSYM | (2u << 24);
    int32_t reach_c = INT32_MIN;
    uint32_t reach_m0 = ~0u, reach_m1 = ~0u, reach_m2 = ~0u;
    SQP_ADD(5, 1);
    if (!bad && nseq) {
      SQP_T(sq_t0);
      const uint32_t tm = U(Bp->tab_mode);
      uint32_t lg[3] = {0, 0, 0};
      for (int t = 0; t < 3 && !bad; t++) {
        const uint32_t mode = (tm >> (2 * t)) & 3, off = U(Bp->tab_off[t]);
#if ZG_SEQ_PACK
        Fse *T = (Fse *)(t == 0 ? S.xl : t == 1 ? S.xo : S.xm);  // built in place, repacked below
#elif ZG_SEQ_ONE_FSE
        Fse *T = S.fse;
#else
        Fse *T = t == 0 ? S.ll : t == 1 ? S.of : S.ml;
#endif
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
          SQP_T(nc0);
          const uint32_t nsrc = U(Bp->norm_src[t]);
          if (norms && nsrc) {  // counts the scan parsed (its lanes, one block each, in parallel)
            const int16_t *nr = norms + ((uint64_t)item * blk_cap + (nsrc - 1)) * ZNORM + t * 64;
            const int16_t v = nr[lane];
            acc = (uint32_t)nr[62];
            ns = (uint32_t)nr[63];
            S.norm[lane] = v;
          } else {
            InW Ic(in, it.len);  // the description through a register window, not a load per byte
            if (!read_ncount(Ic, off, it.len - off, S.norm, maxs, maxl, acc, ns)) { bad = true; break; }
          }
          __syncthreads();
          SQP_T(nc1);
          build_fse(T, S.norm, ns, acc, S.tmp);
          SQP_T(nc2);
          SQP_ADD(6, nc1 - nc0);
          SQP_ADD(7, nc2 - nc1);
          lg[t] = acc;
        }
        // value bases / extra bits folded into the decoding table
        __syncthreads();
        for (uint32_t u = lane; u < (1u << lg[t]); u += 64) {
          const Fse e = T[u];
#if ZG_SEQ_PACK
          uint32_t x;
          if (t == 0) x = e.sym <= 35 ? sq_pack(e.base, e.nb, c_ll_bits[e.sym], e.sym) : SQ_BAD;
          else if (t == 1) x = e.sym <= 31 ? sq_pack(e.base, e.nb, e.sym, e.sym) : SQ_BAD;
          else x = e.sym <= 52 ? sq_pack(e.base, e.nb, c_ml_bits[e.sym], e.sym) : SQ_BAD;
          ((uint32_t *)T)[u] = x;  // same entry, same lane: in place
#else
          if (t == 0) {
            const bool ok = e.sym <= 35;
            S.xl[u] = SeqX{ok ? c_ll_base[e.sym] : 0u, e.base, e.nb, (uint8_t)(ok ? c_ll_bits[e.sym] : 0xFF)};
          } else if (t == 1) {
            const bool ok = e.sym <= 31;
            S.xo[u] = SeqX{ok ? (1u << e.sym) : 0u, e.base, e.nb, (uint8_t)(ok ? e.sym : 0xFF)};
          } else {
            const bool ok = e.sym <= 52;
            S.xm[u] = SeqX{ok ? c_ml_base[e.sym] : 0u, e.base, e.nb, (uint8_t)(ok ? c_ml_bits[e.sym] : 0xFF)};
          }
#endif
        }
        if (ZG_SEQ_ONE_FSE && !ZG_SEQ_PACK) __syncthreads();  // the next table reuses S.fse
      }
      if (!ZG_SEQ_ONE_FSE || ZG_SEQ_PACK) __syncthreads();
      SQP_T(sq_t1);
      SQP_ADD(0, sq_t1 - sq_t0);
      // Backward bit container in SGPRs: C holds bits [32 * lw, 32 * lw + have) of the aligned item
      // words, the next unread bit at bit 63; refilled a word at a time from the BitsBack register
      // window (readlane), so a field read is three scalar operations.
      BitsBack R;
      if (!bad && !bb_init(R, in, it.len, U(Bp->seq_off), U(Bp->seq_end))) bad = true;
      if (!bad) {
#if ZG_SEQ_SPLIT && ZG_SEQ_PACK
        // Split decoder. The serial part is only the FSE state chain: three table entries give every
        // bit count of the sequence, so the next three states are read positionally (one 64-bit
        // window read below the sequence's extra bits) while the entries and the bit position are
        // parked in lane cnt. Every 64 sequences the lanes extract their own extra-bit fields (three
        // item words each), and the batch's repeat offsets are resolved by an inclusive scan of
        // rep-state transforms: a sequence maps the incoming (r0, r1, r2) to three values that are
        // literal offsets or ZSYM | slot << 24 | minus references to the incoming ones (the block's
        // symbolic reps, above), and transforms compose slot by slot. The container decoder below
        // (ZG_SEQ_SPLIT=0) spent ~120 scalar instructions a sequence on the one chain.
        // Positions are 32-bit, relative to word kb0 of the item (a little below the stream start). The
        // chain reads its 64-bit windows by readlane from wcur = words [wb, wb + 64); wnext = words
        // [wb - 60, wb + 4) is loaded one slide ahead, so a slide (every 60 words) waits for nothing.
        const int32_t kb0 = (int32_t)(R.lo_bit >> 5) - 8;
        const int32_t lo_r = (int32_t)(R.lo_bit - (int64_t)kb0 * 32);
        int32_t Pr = (int32_t)(R.cur - (int64_t)kb0 * 32);  // bits not read: the next bit read is Pr - 1
        int32_t wb = ((Pr - 1) >> 5) - 61;
        uint32_t wcur = ldw(R, kb0 + wb + lane), wnext = ldw(R, kb0 + wb - 60 + lane);
        auto bits64 = [&](int32_t q) -> uint64_t {  // stream bits from q up (q at most 3 words below the last)
          int32_t d = (q >> 5) - wb;
          if (__builtin_expect(d < 0, 0)) {
            // keeps the copy inside the branch: hoisted above it, the copy read wnext on every sequence
            // and so waited for its load right after each slide
            asm volatile("" : "+v"(wnext));
            wcur = wnext;
            wb -= 60;
            d += 60;
            wnext = ldw(R, kb0 + wb - 60 + lane);
          }
          const uint32_t lo = U(__builtin_amdgcn_readlane(wcur, d)), hi = U(__builtin_amdgcn_readlane(wcur, d + 1));
          return ((((uint64_t)hi) << 32) | lo) >> (q & 31);
        };
        uint32_t sll, sof, sml;
        {
          const int32_t q = Pr - (int32_t)(lg[0] + lg[1] + lg[2]);
          const uint64_t w = bits64(q);
          sml = (uint32_t)w & ((1u << lg[2]) - 1);
          sof = (uint32_t)(w >> lg[2]) & ((1u << lg[1]) - 1);
          sll = (uint32_t)(w >> (lg[2] + lg[1])) & ((1u << lg[0]) - 1);
          Pr = q;
        }
        uint32_t *out = seq_scratch + ((uint64_t)item * seq_cap + U(Bp->seq_buf)) * 3;
        auto compose = [](uint32_t x, uint32_t a0, uint32_t a1, uint32_t a2) -> uint32_t {
          if (!(x & ZSYM)) return x;
          const uint32_t sl = (x >> 24) & 3, m = x & 0xFFFFFF, v = sl == 0 ? a0 : sl == 1 ? a1 : a2;
          return (v & ZSYM) ? v + m : v - m;
        };
        uint32_t done = 0;
        while (done < nseq && !bad) {
          const uint32_t nb = min(64u, nseq - done);
          int32_t r_p = 0, p3 = Pr;
          uint32_t r_o = 0, r_m = 0, r_l = 0;
          // straight-line chain: no branch but the loop's and the rare slide. A code outside the format
          // is caught by the lanes after the batch (its entry's fields are zero, so the chain stays in
          // the tables); each sequence's entries and position go to lane cnt by v_writelane.
          for (uint32_t cnt = 0; cnt < nb; cnt++) {
            const uint32_t ow = U(S.xo[sof]), mw = U(S.xm[sml]), lwd = U(S.xl[sll]);
            // (the lane select goes through m0: gfx9 writelane reads one SGPR besides m0)
            asm volatile(
                "s_mov_b32 m0, %4\n\t"
                "v_writelane_b32 %0, %5, m0\n\t"
                "v_writelane_b32 %1, %6, m0\n\t"
                "v_writelane_b32 %2, %7, m0\n\t"
                "v_writelane_b32 %3, %8, m0"
                : "+v"(r_p), "+v"(r_o), "+v"(r_m), "+v"(r_l)
                : "s"(cnt), "s"(Pr), "s"(ow), "s"(mw), "s"(lwd)
                : "m0");
            p3 = Pr - (int32_t)(((ow >> 13) & 31) + ((mw >> 13) & 31) + ((lwd >> 13) & 31));
            const uint32_t nl = (lwd >> 9) & 15, nm = (mw >> 9) & 15, no = (ow >> 9) & 15;
            const int32_t q = p3 - (int32_t)(nl + nm + no);
            const uint64_t w = bits64(q);
            sof = (ow & 511) + ((uint32_t)w & ((1u << no) - 1));
            sml = (mw & 511) + ((uint32_t)(w >> no) & ((1u << nm) - 1));
            sll = (lwd & 511) + ((uint32_t)(w >> (no + nm)) & ((1u << nl) - 1));
            Pr = q;
          }
          if (done + nb == nseq) Pr = p3;  // the block's last sequence reads no state update
          if (__any(lane < (int)nb && ((r_o | r_m | r_l) & SQ_BAD))) { bad = true; break; }
          // lane l: sequence done + l's fields, from the three item words holding its extra bits
          const bool mine = lane < (int)nb;
          uint32_t ll = 0, ml = 0, ofv = 0;
          if (mine) {
            const uint32_t oc = (r_o >> 13) & 31, mb = (r_m >> 13) & 31, lb = (r_l >> 13) & 31;
            const int32_t p0 = r_p, p3 = p0 - (int32_t)(oc + mb + lb);
            const int32_t k0 = p3 >> 5;
            const uint32_t w0 = ldw(R, kb0 + k0), w1 = ldw(R, kb0 + k0 + 1), w2 = ldw(R, kb0 + k0 + 2);
            const uint32_t mbs = c_ml_base[(r_m >> 18) & 63], lbs = c_ll_base[(r_l >> 18) & 63];
            const int32_t base = k0 * 32;
            auto ext = [&](int32_t q, uint32_t n) -> uint32_t {  // n <= 31; q + n - base <= 94
              const uint32_t r = (uint32_t)(q - base), j = r >> 5;
              const uint64_t v = j == 0 ? (((uint64_t)w1 << 32) | w0) : j == 1 ? (((uint64_t)w2 << 32) | w1) : (uint64_t)w2;
              return (uint32_t)(v >> (r & 31)) & ((1u << n) - 1);
            };
            ofv = (1u << oc) + ext(p0 - (int32_t)oc, oc);
            ml = mbs + ext(p0 - (int32_t)(oc + mb), mb);
            ll = lbs + ext(p3, lb);
          }
          // the sequence's rep-state transform; lanes past cnt hold the identity
          const uint32_t I0 = ZSYM, I1 = ZSYM | (1u << 24), I2 = ZSYM | (2u << 24);
          uint32_t t0, t1, t2;
          bool lbad = false;
          if (ofv > 3) {
            t0 = ofv - 3;
            lbad = (t0 & ZSYM) != 0;  // beyond any window we decode
            t1 = I0;
            t2 = I1;
          } else {
            const uint32_t idx = ofv - 1 + (ll == 0 ? 1u : 0u);  // 0..3 (ofv 1..3), 0 off the batch
            t0 = idx == 0 ? I0 : idx == 1 ? I1 : idx == 2 ? I2 : I0 + 1;
            t1 = idx == 0 ? I1 : I0;
            t2 = idx <= 1 ? I2 : I1;
          }
          if (__any(lbad)) { bad = true; break; }
          uint32_t inc = ll + ml, incl = ll;
          for (int o = 1; o < 64; o <<= 1) {
            const uint32_t a0 = __shfl_up(t0, o, 64), a1 = __shfl_up(t1, o, 64), a2 = __shfl_up(t2, o, 64);
            const uint32_t u = __shfl_up(inc, o, 64), ul = __shfl_up(incl, o, 64);
            if (lane >= o) {
              const uint32_t c0 = compose(t0, a0, a1, a2), c1 = compose(t1, a0, a1, a2), c2 = compose(t2, a0, a1, a2);
              t0 = c0;
              t1 = c1;
              t2 = c2;
              inc += u;
              incl += ul;
            }
          }
          const uint32_t off = compose(t0, r0, r1, r2);
          {
            const uint32_t n1 = compose(t1, r0, r1, r2), n2 = compose(t2, r0, r1, r2);
            r0 = __shfl(off, 63, 64);
            r1 = __shfl(n1, 63, 64);
            r2 = __shfl(n2, 63, 64);
          }
          {  // the batch's reach back from the block start (exact, per match)
            const int32_t p = (int32_t)(sum_ll + sum_ml + inc - ml);  // this lane's match start
            int32_t rc = INT32_MIN;
            uint32_t m0 = ~0u, m1 = ~0u, m2 = ~0u;
            if (mine && ml) {
              if (!(off & ZSYM)) {
                rc = (int32_t)off - p;
              } else {
                const uint32_t slot = (off >> 24) & 3, mv = (off & 0xFFFFFF) + (uint32_t)p;
                if (slot == 0) m0 = mv;
                else if (slot == 1) m1 = mv;
                else m2 = mv;
              }
            }
            for (int o = 32; o; o >>= 1) {
              rc = max(rc, __shfl_xor(rc, o, 64));
              m0 = min(m0, __shfl_xor(m0, o, 64));
              m1 = min(m1, __shfl_xor(m1, o, 64));
              m2 = min(m2, __shfl_xor(m2, o, 64));
            }
            reach_c = max(reach_c, rc);
            reach_m0 = min(reach_m0, m0);
            reach_m1 = min(reach_m1, m1);
            reach_m2 = min(reach_m2, m2);
          }
          {
            const uint32_t tot = __shfl(inc, 63, 64), totl = __shfl(incl, 63, 64);
            sum_ll += totl;
            sum_ml += tot - totl;
          }
          if (mine) {
            uint32_t *o = out + (uint64_t)(done + lane) * 3;
            o[0] = ll;
            o[1] = ml;
            o[2] = off;
          }
          done += nb;
        }
        // the stream must end exactly on its first bit
        if (!bad && Pr != lo_r) bad = true;
#else
        auto word = [&](int32_t k) -> uint32_t {
          if (k < R.wb - 16) {  // slide the window pair down, prefetching the next lower window
            R.wb -= 64;
            R.wcur = R.wprev;
            R.wprev = ldw(R, R.wb - 64 + lane_id());
          }
          return wget(R, k);
        };
        const int64_t p0 = R.cur;
        int32_t lw = (int32_t)((p0 - 1) >> 5) - 1;
        int32_t have = (int32_t)(p0 - 32 * (int64_t)lw);  // (32, 64]
        uint64_t C = (((uint64_t)word(lw + 1) << 32) | word(lw)) << (64 - have);
        auto refill = [&]() {
          if (have <= 32) {
            lw--;
            C |= (uint64_t)word(lw) << (32 - have);
            have += 32;
          }
        };
        auto rd = [&](uint32_t n) -> uint32_t {  // n <= 31 bits
          const uint32_t v = (uint32_t)((C >> 1) >> (63 - n));
          C <<= n;
          have -= (int32_t)n;
          return v;
        };
        uint32_t sll = rd(lg[0]), sof = rd(lg[1]);
        refill();
        uint32_t sml = rd(lg[2]);
        uint32_t *out = seq_scratch + ((uint64_t)item * seq_cap + U(Bp->seq_buf)) * 3;
        uint32_t remaining = nseq, done = 0;
#if !ZG_SEQ_PACK
        const uint2 *XO = (const uint2 *)S.xo, *XM = (const uint2 *)S.xm, *XL = (const uint2 *)S.xl;
#endif
        while (remaining && !bad) {
          uint32_t r_ll = 0, r_ml = 0, r_of = 0, cnt = 0;
          while (cnt < 64 && remaining) {
#if ZG_SEQ_PACK
            const uint32_t ow = U(S.xo[sof]), mw = U(S.xm[sml]), lwd = U(S.xl[sll]);
            if ((ow | mw | lwd) & SQ_BAD) { bad = true; break; }
            const uint32_t oc = (ow >> 18) & 63, mc = (mw >> 18) & 63, lc = (lwd >> 18) & 63;
            refill();
            const uint32_t ofv = (1u << oc) + rd(oc);
            refill();
            const uint32_t ml = c_ml_base[mc] + rd((mw >> 13) & 31);
            const uint32_t ll = c_ll_base[lc] + rd((lwd >> 13) & 31);
            remaining--;
            if (remaining) {
              refill();
              sll = (lwd & 511) + rd((lwd >> 9) & 15);
              sml = (mw & 511) + rd((mw >> 9) & 15);
              sof = (ow & 511) + rd((ow >> 9) & 15);
            }
#else
            const uint2 eo = XO[sof], em = XM[sml], el = XL[sll];
            const uint32_t ob = U(eo.x), ow = U(eo.y), mb = U(em.x), mw = U(em.y), lb = U(el.x), lwd = U(el.y);
            if ((ow | mw | lwd) & 0x80000000u) { bad = true; break; }
            refill();
            const uint32_t ofv = ob + rd(ow >> 24);
            refill();
            const uint32_t ml = mb + rd(mw >> 24);
            const uint32_t ll = lb + rd(lwd >> 24);
            remaining--;
            if (remaining) {
              refill();
              sll = (lwd & 0xFFFF) + rd((lwd >> 16) & 0xFF);
              sml = (mw & 0xFFFF) + rd((mw >> 16) & 0xFF);
              sof = (ow & 0xFFFF) + rd((ow >> 16) & 0xFF);
            }
#endif
            // repeat offsets, symbolically in the block's incoming rep state (RFC 8878 3.1.1.5)
#if ZG_SEQ_REP_SEL
            // as selects (the branchy form cost ~25 scalar instructions and four branches a sequence
            // on a decoder bound by the CU's scalar unit): k = 0 new offset, else 1 + repeat index
            const bool lit0 = ll == 0;
            const uint32_t k = ofv > 3 ? 0u : ofv + (lit0 ? 1u : 0u);  // 1..4: repeat index 0..3
            if (k == 0 && ((ofv - 3) & ZSYM)) { bad = true; break; }   // beyond any window we decode
            const uint32_t off = k == 0 ? ofv - 3 : k == 1 ? r0 : k == 2 ? r1 : k == 3 ? r2 : sym_dec(r0);
            const uint32_t n2 = (k == 0 || k >= 3) ? r1 : r2;  // rotations: every case but index 0/1 keeps r2
            const uint32_t n1 = k == 1 ? r1 : r0;
            r2 = n2;
            r1 = n1;
            r0 = off;
#else
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
#endif
            if (lane == (int)cnt) { r_ll = ll; r_ml = ml; r_of = off; }
            sum_ll += ll;
            sum_ml += ml;
            cnt++;
          }
          if (bad) break;
          {  // the batch's reach back from the block start (exact, per match)
            const uint64_t bpos = sum_ll + sum_ml;  // block position after the batch
            uint32_t inc = lane < (int)cnt ? r_ll + r_ml : 0u;
            for (int o = 1; o < 64; o <<= 1) {
              const uint32_t t = __shfl_up(inc, o, 64);
              if (lane >= o) inc += t;
            }
            const uint32_t tot = __shfl(inc, 63, 64);
            const int32_t p = (int32_t)(bpos - tot + inc - r_ml);  // this lane's match start
            int32_t rc = INT32_MIN;
            uint32_t m0 = ~0u, m1 = ~0u, m2 = ~0u;
            if (lane < (int)cnt && r_ml) {
              if (!(r_of & ZSYM)) {
                rc = (int32_t)r_of - p;
              } else {
                const uint32_t slot = (r_of >> 24) & 3, mv = (r_of & 0xFFFFFF) + (uint32_t)p;
                if (slot == 0) m0 = mv;
                else if (slot == 1) m1 = mv;
                else m2 = mv;
              }
            }
            for (int o = 32; o; o >>= 1) {
              rc = max(rc, __shfl_xor(rc, o, 64));
              m0 = min(m0, __shfl_xor(m0, o, 64));
              m1 = min(m1, __shfl_xor(m1, o, 64));
              m2 = min(m2, __shfl_xor(m2, o, 64));
            }
            reach_c = max(reach_c, rc);
            reach_m0 = min(reach_m0, m0);
            reach_m1 = min(reach_m1, m1);
            reach_m2 = min(reach_m2, m2);
          }
          if (lane < (int)cnt) {
            uint32_t *o = out + (uint64_t)(done + lane) * 3;
            o[0] = r_ll;
            o[1] = r_ml;
            o[2] = r_of;
          }
          done += cnt;
        }
        // the stream must end exactly on its first bit
        if (!bad && (int64_t)lw * 32 + have != R.lo_bit) bad = true;
#endif
      }
      SQP_T(sq_t2);
      SQP_ADD(1, sq_t2 - sq_t1);
      SQP_ADD(2, nseq);
      SQP_ADD(3, 1);
    }
    if (!bad && sum_ll > regen) bad = true;
    if (!bad && regen + sum_ml > BLOCK_MAX) bad = true;  // a block decodes to at most 128 KiB
    if (lane == 0) {
      if (bad) {
        status[item] = ZG_CORRUPT_STREAM;
      } else {
        Bp->out_size = (uint32_t)(regen + sum_ml);
        Bp->reach_c = reach_c;
        Bp->reach_m[0] = reach_m0;
        Bp->reach_m[1] = reach_m1;
        Bp->reach_m[2] = reach_m2;
        Bp->rep_out[0] = r0;
        Bp->rep_out[1] = r1;
        Bp->rep_out[2] = r2;
      }
    }
  }
}

// -------------------------------------------------------------------------------------------------
// Lane-group sequence decoder (ZGPU_ZSTD_SEQ=1, default): ZG_SEQ_G blocks per wave, one lane each.
// k_zstd_blocks above runs one block per wave as wave-uniform scalar code (~120 scalar instructions a
// sequence), and the CU's one scalar unit, shared by the ~20 waves resident on it, bounded the
// whole decoder. Here the serial FSE chain of a block runs in one lane's vector registers, so one
// vector instruction advances ZG_SEQ_G blocks and four SIMDs share the work: each lane has its own
// backward bit container (refilled from a 4-word prefetch queue of its block's stream), its three
// states, its repeat offsets (symbolic, as above) and its block's three tables, built into its own
// slot of LDS by the whole wave before the decode (5 KiB per block). Output and record fields are
// those of k_zstd_blocks.
#ifndef ZG_SEQ_G
#define ZG_SEQ_G 4
#endif
#ifndef ZG_SEQ_WN
#define ZG_SEQ_WN 128  // staged stream words per block and epoch
#endif
#ifndef ZG_SEQ_POS
#define ZG_SEQ_POS 0  // 1: positional field reader (lab r06p: blocks 5.01 -> 5.74 ms at 64 L0 chunks, off)
#endif
template <int G>
struct ZDecLgSmem {
  uint32_t xl[G][512], xm[G][512], xo[G][256];
  uint32_t win[G][ZG_SEQ_WN];
  uint32_t llb[36], mlb[53];
  int16_t norm[64];
  uint32_t tmp[32];
};

#ifndef ZG_SEQ_WPE
#define ZG_SEQ_WPE 1  // lane-group decoder: minimum waves per SIMD the register allocation must allow
#endif
template <int G>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(ZG_SEQ_WPE, 8))) void k_zstd_blocks_lg(const ZgItem *items, uint32_t *status, ZBlk *blks,
                                                       uint32_t blk_cap, const uint32_t *nblk, const uint32_t *zmode,
                                                       uint32_t n_items, uint32_t *seq_scratch, uint64_t seq_cap,
                                                       const unsigned long long *max_nblk) {
  __shared__ ZDecLgSmem<G> S;
  const int lane = lane_id();
  for (int k = lane; k < 53; k += 64) {
    if (k < 36) S.llb[k] = c_ll_base[k];
    S.mlb[k] = c_ml_base[k];
  }
  const uint64_t total = (uint64_t)n_items * rec_blocks(blk_cap, max_nblk);
  for (uint64_t g0 = (uint64_t)blockIdx.x * G; g0 < total; g0 += (uint64_t)gridDim.x * G) {
    SQP_T(sq_t0);
    SQP_ADD(5, G);
    // ---- the wave builds the tables of its G records, one record at a time; lane k keeps record
    // k's fields (block-major record order, as k_zstd_blocks)
    bool mine = false, bad = false;
    ZBlk *Bp = nullptr;
    uint32_t item = 0, nseq = 0, regen = 0, lg0 = 0, lg1 = 0, lg2 = 0, seq_off = 0, seq_end = 0, seq_buf = 0;
    for (int k = 0; k < G; k++) {
      const uint64_t g = g0 + k;
      if (g >= total) break;
      const uint32_t it_k = (uint32_t)(g % n_items), bi = (uint32_t)(g / n_items);
      if (bi >= nblk[it_k] || zmode[it_k] != ZMODE_PARALLEL) continue;
      ZBlk *B = blks + (uint64_t)it_k * blk_cap + bi;
      const uint32_t flags = U(B->flags);
      if ((flags & 3) != ZB_CMP) continue;
      const ZgItem it = items[it_k];
      const In I{(const uint8_t *)it.src, it.len};
      const uint32_t ns_k = U(B->nseq);
      bool bad_k = false;
      uint32_t lg[3] = {0, 0, 0};
      if (ns_k) {
        const uint32_t tm = U(B->tab_mode);
        __syncthreads();  // the previous use of norm / tmp is done
        for (int t = 0; t < 3 && !bad_k; t++) {
          const uint32_t mode = (tm >> (2 * t)) & 3, off = U(B->tab_off[t]);
          Fse *T = (Fse *)(t == 0 ? S.xl[k] : t == 1 ? S.xo[k] : S.xm[k]);  // built in place, repacked below
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
            InW Ic((const uint8_t *)it.src, it.len);
            if (!read_ncount(Ic, off, it.len - off, S.norm, maxs, maxl, acc, ns)) { bad_k = true; break; }
            __syncthreads();
            build_fse(T, S.norm, ns, acc, S.tmp);
            lg[t] = acc;
          }
          __syncthreads();
          for (uint32_t u = lane; u < (1u << lg[t]); u += 64) {
            const Fse e = T[u];
            uint32_t x;
            if (t == 0) x = e.sym <= 35 ? sq_pack(e.base, e.nb, c_ll_bits[e.sym], e.sym) : SQ_BAD;
            else if (t == 1) x = e.sym <= 31 ? sq_pack(e.base, e.nb, e.sym, e.sym) : SQ_BAD;
            else x = e.sym <= 52 ? sq_pack(e.base, e.nb, c_ml_bits[e.sym], e.sym) : SQ_BAD;
            ((uint32_t *)T)[u] = x;
          }
        }
      }
      if (lane == k) {
        mine = true;
        bad = bad_k;
        Bp = B;
        item = it_k;
        nseq = ns_k;
        regen = U(B->regen);
        lg0 = lg[0];
        lg1 = lg[1];
        lg2 = lg[2];
        seq_off = U(B->seq_off);
        seq_end = U(B->seq_end);
        seq_buf = U(B->seq_buf);
      }
    }
    __syncthreads();
    // ---- every lane decodes its own block's sequences, in epochs: the wave stages the next ZG_SEQ_WN
    // words of each lane's stream into LDS (one coalesced load per lane and block, one wait), then
    // each lane decodes until fewer than three staged words remain below its position (a sequence
    // takes at most three refills). No global load inside the decode loop, so the sequence stores
    // are never waited on, and a sequence's three table reads and three word reads issue together.
    uint64_t sum_ll = 0, sum_ml = 0;
    uint32_t r0 = ZSYM | (0u << 24), r1 = ZSYM | (1u << 24), r2 = ZSYM | (2u << 24);
    int32_t reach_c = INT32_MIN;
    uint32_t reach_m0 = ~0u, reach_m1 = ~0u, reach_m2 = ~0u;
    const uint32_t *words = nullptr;
    int32_t nwords = 0, lw = 0, have = 0, lo_w = 0;
    int64_t lo_bit = 0, P = 0;  // P (ZG_SEQ_POS): stream bits not read yet; the next bit read is P - 1
    uint64_t C = 0;
    bool act = false;
    uint32_t sll = 0, sof = 0, sml = 0, n = 0;
    uint32_t *out = nullptr;
    if (mine && !bad && nseq) {
      const ZgItem it = items[item];
      const uint8_t *in = (const uint8_t *)it.src;
      const uintptr_t mis = (uintptr_t)in & 3;
      words = (const uint32_t *)((uintptr_t)in - mis);
      nwords = (int32_t)((it.len + mis + 3) / 4);
      const uint32_t last = seq_end > seq_off ? in[seq_end - 1] : 0u;
      if (last == 0) {
        bad = true;
      } else {
        const int64_t p0 = (int64_t)(seq_end - 1 + mis) * 8 + highbit(last);
        lo_bit = (int64_t)(seq_off + mis) * 8;
        P = p0;
        lw = (int32_t)((p0 - 1) >> 5) - 1;
        have = (int32_t)(p0 - 32 * (int64_t)lw);  // (32, 64]
        auto ld = [&](int32_t k) -> uint32_t { return (k >= 0 && k < nwords) ? words[k] : 0u; };
        C = (((uint64_t)ld(lw + 1) << 32) | ld(lw)) << (64 - have);
        act = true;
        out = seq_scratch + ((uint64_t)item * seq_cap + seq_buf) * 3;
      }
    }
    bool first = true;
    SQP_T(sq_t1);
    SQP_ADD(0, sq_t1 - sq_t0);
#ifdef ZG_SQ_PROFILE
    if (mine && nseq) {
      atomicAdd(&g_sqprof[2], (unsigned long long)nseq);
      atomicAdd(&g_sqprof[3], 1ull);
    }
#endif
    while (__any(act)) {
      SQP_ADD(4, 1);
      // stage words [lw - WN, lw) of every active lane's stream: lane k's window is S.win[k]
      // (positional reader: [kt + 1 - WN, kt + 1), kt the word holding bit P - 1)
      lo_w = ZG_SEQ_POS ? (int32_t)((P - 1) >> 5) + 1 - ZG_SEQ_WN : lw - ZG_SEQ_WN;
#pragma unroll
      for (int k = 0; k < G; k++) {
        const bool ak = __builtin_amdgcn_readlane((int)act, k) != 0;
        if (!ak) continue;
        const uint64_t wp = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(uintptr_t)words, k)) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uintptr_t)words >> 32), k) << 32);
        const int32_t nw = __builtin_amdgcn_readlane(nwords, k), b = __builtin_amdgcn_readlane(lo_w, k);
        const uint32_t *W = (const uint32_t *)(uintptr_t)wp;
        for (int i = lane; i < ZG_SEQ_WN; i += 64) {
          const int32_t w = b + i;
          S.win[k][i] = (w >= 0 && w < nw) ? W[w] : 0u;
        }
      }
      __syncthreads();
#if ZG_SEQ_POS
      // Positional reader: a field of nb bits is stream bits [P - nb, P). A sequence reads at most
      // 31 + 16 + 16 + 9 + 9 + 8 = 89 bits, i.e. words kt = (P - 1) >> 5 down to kt - 3: they are read
      // from the staged window with the three table entries, in one LDS round; the six field
      // positions follow from the entries' bit counts, and the fields are funnel-shifted out of those
      // four words independently (the 64-bit container's refill / shift chain serialised them).
      const uint32_t k = (uint32_t)lane;
      auto win4 = [&](int32_t kt, uint32_t &q0, uint32_t &q1, uint32_t &q2, uint32_t &q3) {
        const uint32_t *wk = &S.win[k][kt - 3 - lo_w];
        q0 = wk[0];
        q1 = wk[1];
        q2 = wk[2];
        q3 = wk[3];
      };
      // bits [q, q + nb) of the stream, nb <= 31, from words base/32 .. base/32 + 3
      auto ext = [](int64_t q, uint32_t nb, int64_t base, uint32_t q0, uint32_t q1, uint32_t q2, uint32_t q3) -> uint32_t {
        const uint32_t r = (uint32_t)(q - base), j = r >> 5, sh = r & 31;
        const uint32_t lo = j == 0 ? q0 : j == 1 ? q1 : j == 2 ? q2 : q3;
        const uint32_t hi = j == 0 ? q1 : j == 1 ? q2 : j == 2 ? q3 : 0u;
        return (uint32_t)((((uint64_t)hi << 32) | lo) >> sh) & ((1u << nb) - 1);
      };
      if (act && first) {  // the three initial states (at most 9 + 8 + 9 bits)
        first = false;
        const int32_t kt = (int32_t)((P - 1) >> 5);
        uint32_t q0, q1, q2, q3;
        win4(kt, q0, q1, q2, q3);
        const int64_t base = (int64_t)(kt - 3) * 32;
        sll = ext(P - lg0, lg0, base, q0, q1, q2, q3);
        P -= lg0;
        sof = ext(P - lg1, lg1, base, q0, q1, q2, q3);
        P -= lg1;
        sml = ext(P - lg2, lg2, base, q0, q1, q2, q3);
        P -= lg2;
      }
      while (act) {
        const int32_t kt = (int32_t)((P - 1) >> 5);
        if (kt - 3 < lo_w) break;  // the next epoch stages the words below
        const uint32_t ow = S.xo[k][sof], mw = S.xm[k][sml], lwd = S.xl[k][sll];
        uint32_t q0, q1, q2, q3;
        win4(kt, q0, q1, q2, q3);
        if ((ow | mw | lwd) & SQ_BAD) { bad = true; act = false; break; }
        const int64_t base = (int64_t)(kt - 3) * 32;
        const uint32_t oc = (ow >> 18) & 63, mc = (mw >> 18) & 63, lc = (lwd >> 18) & 63;
        const uint32_t mbits = (mw >> 13) & 31, lbits = (lwd >> 13) & 31;
        const int64_t P1 = P - oc, P2 = P1 - mbits, P3 = P2 - lbits;
        const uint32_t ofv = (1u << oc) + ext(P1, oc, base, q0, q1, q2, q3);
        const uint32_t ml = S.mlb[mc] + ext(P2, mbits, base, q0, q1, q2, q3);
        const uint32_t ll = S.llb[lc] + ext(P3, lbits, base, q0, q1, q2, q3);
        n++;
        P = P3;
        if (n < nseq) {
          const uint32_t nl = (lwd >> 9) & 15, nm = (mw >> 9) & 15, no = (ow >> 9) & 15;
          const int64_t P4 = P3 - nl, P5 = P4 - nm, P6 = P5 - no;
          sll = (lwd & 511) + ext(P4, nl, base, q0, q1, q2, q3);
          sml = (mw & 511) + ext(P5, nm, base, q0, q1, q2, q3);
          sof = (ow & 511) + ext(P6, no, base, q0, q1, q2, q3);
          P = P6;
        }
        // repeat offsets, symbolically in the block's incoming rep state (RFC 8878 3.1.1.5), as
        // selects: kk = 0 a new offset, else 1 + repeat index
        const uint32_t kk = ofv > 3 ? 0u : ofv + (ll == 0 ? 1u : 0u);
        if (kk == 0 && ((ofv - 3) & ZSYM)) { bad = true; act = false; break; }  // beyond any window we decode
        const uint32_t s3 = (r0 & ZSYM) ? r0 + 1 : r0 - 1;
        uint32_t off = ofv - 3;
        off = kk == 1 ? r0 : off;
        off = kk == 2 ? r1 : off;
        off = kk == 3 ? r2 : off;
        off = kk == 4 ? s3 : off;
        const uint32_t n2 = (kk == 0 || kk >= 3) ? r1 : r2;
        const uint32_t n1 = kk == 1 ? r1 : r0;
        r2 = n2;
        r1 = n1;
        r0 = off;
        // how far the match reaches back from the block start (exact, per match)
        const int32_t p = (int32_t)(sum_ll + sum_ml + ll);
        const bool isc = !(off & ZSYM);
        const uint32_t slot = (off >> 24) & 3, mv = (off & 0xFFFFFF) + (uint32_t)p;
        reach_c = isc ? max(reach_c, (int32_t)off - p) : reach_c;
        reach_m0 = (!isc && slot == 0) ? min(reach_m0, mv) : reach_m0;
        reach_m1 = (!isc && slot == 1) ? min(reach_m1, mv) : reach_m1;
        reach_m2 = (!isc && slot >= 2) ? min(reach_m2, mv) : reach_m2;
        sum_ll += ll;
        sum_ml += ml;
        uint32_t *o = out + (uint64_t)(n - 1) * 3;
        o[0] = ll;
        o[1] = ml;
        o[2] = off;
        if (n == nseq) {
          act = false;
          if (P != lo_bit) bad = true;  // the stream must end exactly on its first bit
        }
      }
#else
      if (act && first) {  // the three initial states
        first = false;
        // the container holds > 32 bits, at most 9 + 8 read before the refill
        sll = (uint32_t)((C >> 1) >> (63 - lg0));
        C <<= lg0;
        have -= (int32_t)lg0;
        sof = (uint32_t)((C >> 1) >> (63 - lg1));
        C <<= lg1;
        have -= (int32_t)lg1;
        if (have <= 32) {
          lw--;
          C |= (uint64_t)S.win[lane][lw - lo_w] << (32 - have);
          have += 32;
        }
        sml = (uint32_t)((C >> 1) >> (63 - lg2));
        C <<= lg2;
        have -= (int32_t)lg2;
      }
      const uint32_t k = (uint32_t)lane;
      while (act && lw - 3 >= lo_w) {
        // everything this sequence can read: its three table entries and the next three words
        const uint32_t ow = S.xo[k][sof], mw = S.xm[k][sml], lwd = S.xl[k][sll];
        uint32_t w1 = S.win[k][lw - 1 - lo_w], w2 = S.win[k][lw - 2 - lo_w], w3 = S.win[k][lw - 3 - lo_w];
        if ((ow | mw | lwd) & SQ_BAD) { bad = true; act = false; break; }
        auto refill = [&]() {
          const bool nd = have <= 32;
          C |= nd ? (uint64_t)w1 << (32 - have) : 0ull;
          have += nd ? 32 : 0;
          lw -= nd ? 1 : 0;
          w1 = nd ? w2 : w1;
          w2 = nd ? w3 : w2;
        };
        auto rd = [&](uint32_t nb) -> uint32_t {  // nb <= 31 bits
          const uint32_t v = (uint32_t)((C >> 1) >> (63 - nb));
          C <<= nb;
          have -= (int32_t)nb;
          return v;
        };
        const uint32_t oc = (ow >> 18) & 63, mc = (mw >> 18) & 63, lc = (lwd >> 18) & 63;
        refill();
        const uint32_t ofv = (1u << oc) + rd(oc);
        refill();
        const uint32_t ml = S.mlb[mc] + rd((mw >> 13) & 31);
        const uint32_t ll = S.llb[lc] + rd((lwd >> 13) & 31);
        n++;
        if (n < nseq) {
          refill();
          sll = (lwd & 511) + rd((lwd >> 9) & 15);
          sml = (mw & 511) + rd((mw >> 9) & 15);
          sof = (ow & 511) + rd((ow >> 9) & 15);
        }
        // repeat offsets, symbolically in the block's incoming rep state (RFC 8878 3.1.1.5), as
        // selects: kk = 0 a new offset, else 1 + repeat index
        const uint32_t kk = ofv > 3 ? 0u : ofv + (ll == 0 ? 1u : 0u);
        if (kk == 0 && ((ofv - 3) & ZSYM)) { bad = true; act = false; break; }  // beyond any window we decode
        const uint32_t s3 = (r0 & ZSYM) ? r0 + 1 : r0 - 1;
        uint32_t off = ofv - 3;
        off = kk == 1 ? r0 : off;
        off = kk == 2 ? r1 : off;
        off = kk == 3 ? r2 : off;
        off = kk == 4 ? s3 : off;
        const uint32_t n2 = (kk == 0 || kk >= 3) ? r1 : r2;
        const uint32_t n1 = kk == 1 ? r1 : r0;
        r2 = n2;
        r1 = n1;
        r0 = off;
        // how far the match reaches back from the block start (exact, per match)
        const int32_t p = (int32_t)(sum_ll + sum_ml + ll);
        const bool isc = !(off & ZSYM);
        const uint32_t slot = (off >> 24) & 3, mv = (off & 0xFFFFFF) + (uint32_t)p;
        reach_c = isc ? max(reach_c, (int32_t)off - p) : reach_c;
        reach_m0 = (!isc && slot == 0) ? min(reach_m0, mv) : reach_m0;
        reach_m1 = (!isc && slot == 1) ? min(reach_m1, mv) : reach_m1;
        reach_m2 = (!isc && slot >= 2) ? min(reach_m2, mv) : reach_m2;
        sum_ll += ll;
        sum_ml += ml;
        uint32_t *o = out + (uint64_t)(n - 1) * 3;
        o[0] = ll;
        o[1] = ml;
        o[2] = off;
        if (n == nseq) {
          act = false;
          // the stream must end exactly on its first bit
          if ((int64_t)lw * 32 + have != lo_bit) bad = true;
        }
      }
#endif
      __syncthreads();  // this epoch's window reads are done before the next staging
    }
    SQP_T(sq_t2);
    SQP_ADD(1, sq_t2 - sq_t1);
    if (mine) {
      if (!bad && sum_ll > regen) bad = true;
      if (!bad && regen + sum_ml > BLOCK_MAX) bad = true;  // a block decodes to at most 128 KiB
      if (bad) {
        status[item] = ZG_CORRUPT_STREAM;
      } else {
        Bp->out_size = (uint32_t)(regen + sum_ml);
        Bp->reach_c = reach_c;
        Bp->reach_m[0] = reach_m0;
        Bp->reach_m[1] = reach_m1;
        Bp->reach_m[2] = reach_m2;
        Bp->rep_out[0] = r0;
        Bp->rep_out[1] = r1;
        Bp->rep_out[2] = r2;
      }
    }
    __syncthreads();  // the tables are rebuilt for the next records
  }
}

// -------------------------------------------------------------------------------------------------
// Huffman literals, 256 threads per block record. One symbol costs a wave ~15 instructions whoever
// decodes it, so the four streams are decoded by all 256 lanes: every stream is cut into equal bit
// segments (64 per stream with 4 streams, 256 with 1), each lane decodes one. A lane that does not
// start at a known symbol boundary starts LIT_WARM bits early: Huffman decoding self-synchronises,
// and the lane is known to be right once the first boundary it reaches inside its segment equals the
// exit boundary of the lane before it (decoding from a boundary is deterministic). Lanes that do not
// meet are re-decoded from their predecessor's exit (repair rounds). Pass 1 finds every segment's
// entry, exit and symbol count; pass 2 decodes again and writes the symbols at the prefix-summed
// offsets. The compressed literal section is staged in LDS first (sections over LIT_LDS read global).
// -------------------------------------------------------------------------------------------------
#ifndef ZG_LIT_LDS
#define ZG_LIT_LDS (8 * 1024)
#endif
constexpr uint32_t LIT_LDS = ZG_LIT_LDS;
#ifndef ZG_LIT_WARM
#define ZG_LIT_WARM 128
#endif
constexpr int32_t LIT_WARM = ZG_LIT_WARM;
constexpr uint32_t LIT_THREADS = 256;
#ifndef ZG_LIT_WPE
#define ZG_LIT_WPE 4  // min waves per SIMD k_zstd_lits is compiled for (4: 100 VGPRs, no spills, with staging)
#endif
constexpr int LIT_STAGE_R = ZG_LIT_WPE >= 4 ? 4 : 8;  // 16-B staging loads in flight per thread
#ifndef ZG_LIT_GRID_PER_CU
#define ZG_LIT_GRID_PER_CU 4
#endif
#ifndef ZG_LIT_PACK
#define ZG_LIT_PACK 1  // decoded literals stored ZG_LIT_PACK_B at a time
#endif
#ifndef ZG_LIT_PACK_B
#define ZG_LIT_PACK_B 8
#endif
#ifndef ZG_LIT_GWIN
#define ZG_LIT_GWIN 4  // literal sections beyond LIT_LDS: 1 per-lane 16-B window, 2 32-B + prefetch,
                       // 3 64-B + prefetch, 4 GBlk (32-B blocks moved in lockstep rounds)
#endif
#ifndef ZG_LIT_STAGE
#define ZG_LIT_STAGE 1  // 1: a lane's decoded literals leave through an LDS window, stored as whole
                        // aligned ZG_LIT_STAGE_W-B pieces (16-B stores) instead of 8-B stores
#endif
#ifndef ZG_LIT_STAGE_W
#define ZG_LIT_STAGE_W 32  // staging window bytes per lane: one 32-B sector (lab PMC: literal writes
                           // 2,994 -> 643 MB per launch on 64 C5 chunks, 1.2x the literal bytes)
#endif
#ifndef ZG_LIT_STG_PITCH
#define ZG_LIT_STG_PITCH (2 * ZG_LIT_STAGE_W)  // bytes per lane: two windows (pass 1's record stores are
                                               // deferred a round, below; with the 8 KiB section stage
                                               // the workgroup keeps 37 KB of LDS: 4 per CU)
#endif
#ifndef ZG_LIT_ILP
#define ZG_LIT_ILP 1  // Huffman chains per lane (2: a lane decodes two segments, interleaved)
#endif
static_assert(ZG_LIT_ILP == 1 || (ZG_LIT_ILP == 2 && ZG_LIT_STAGE && ZG_LIT_PACK && ZG_LIT_PACK_B == 8),
              "two chains per lane need the staged 8-B literal writer");
constexpr uint32_t LIT_SEGS = LIT_THREADS * ZG_LIT_ILP;  // segments per block record
#if ZG_LIT_STAGE
constexpr uint32_t LIT_STG_W = ZG_LIT_STAGE_W;
constexpr uint32_t LIT_STG_PITCH = ZG_LIT_STG_PITCH;
static_assert(LIT_STG_PITCH % 16 == 0 && LIT_STG_PITCH >= LIT_STG_W, "staging window pitch");
#endif

struct ZLitSmem {
  uint16_t huf[1 << MAX_HUF_LOG];
  Fse wt[64];
  int16_t norm[64];
  uint8_t weights[256];
  uint16_t hsorted[256];
  uint32_t tmp[32];
  int32_t entry[LIT_SEGS], exit_[LIT_SEGS];
  uint32_t cnt[LIT_SEGS], wsum[4 * ZG_LIT_ILP];
  uint32_t ctl[4];  // table log, flags
  uint32_t lin[LIT_LDS / 4 + 8];
#if ZG_LIT_STAGE
  uint4 stg[LIT_SEGS * LIT_STG_PITCH / 16];  // per-segment output windows
#endif
};

// backward bit container: C holds bits [lp, p) of the word array, bit p-1 at C bit 63
struct HufLane {
  uint64_t C;
  int32_t v, lp;
};
template <class Wd>
__device__ __forceinline__ void hl_init(HufLane &H, int32_t p, const Wd &word) {
  const int32_t k = (p - 1) >> 5;
  const uint64_t V = ((uint64_t)word(k) << 32) | word(k - 1);
  H.lp = (k - 1) * 32;
  H.v = p - H.lp;  // (32, 64]
  H.C = V << (64 - H.v);
}
// word-reader hooks of hl_run: a plain reader always has the word; GBlk (below) has it only inside
// its current block
template <class Wd>
__device__ __forceinline__ void wd_start(const Wd &, const HufLane &) {}

// Literal-section words through a window of one 32-B block plus the block below it, moved in
// lockstep (ZG_LIT_GWIN 4). The per-lane prefetching readers (GWordPF) let each lane switch blocks on
// its own; but a wave's load counter is shared, so a lane switching blocks waited for every load the
// other lanes had just issued (s_waitcnt vmcnt(0)), one memory round trip nearly every symbol step
// (C5: ~2,000 cycles per step). Here a lane whose next word lies below its block stops; once every
// lane of the wave has stopped or finished, the stopped lanes take the prefetched block (loaded one
// round - ~40 symbols - earlier) and prefetch the next one. No load is waited for inside a round.
struct GBlk {
  const gu32 *Wp;
  int64_t lim;
  mutable uintptr_t cb;   // address of the current block
  mutable zv4u a0, a1;    // block A
  mutable zv4u b0, b1;    // block B
  mutable uint32_t cur;   // 0: A is the current block and B the one below it; 1: the reverse
  __device__ __forceinline__ static void ld(uintptr_t b, zv4u &x0, zv4u &x1) {
    const __attribute__((address_space(1))) zv4u *q = (const __attribute__((address_space(1))) zv4u *)b;
    x0 = q[0];
    x1 = q[1];
  }
  __device__ __forceinline__ uintptr_t below(uintptr_t b) const {  // never before Wp's block
    return b > ((uintptr_t)Wp & ~(uintptr_t)31) ? b - 32 : b;
  }
  __device__ __forceinline__ uint32_t operator()(int32_t k) const { return (k >= 0 && k < lim) ? Wp[k] : 0u; }
  // window at the block of word k (the next word the lane reads), k clamped into the section
  __device__ __forceinline__ void start(int32_t k) const {
    const int32_t kc = k < 0 ? 0 : (k >= lim ? (int32_t)(lim - 1) : k);
    cb = (uintptr_t)(Wp + kc) & ~(uintptr_t)31;
    ld(cb, a0, a1);
    cur = 0;
  }
  // A current again (hl_run's rounds alternate A and B in unrolled code, so no block is ever copied
  // between registers in a round - a copy of a prefetched block is a wait for it)
  __device__ __forceinline__ void norm() const {
    if (cur) {
      const zv4u t0 = a0, t1 = a1;
      a0 = b0;
      a1 = b1;
      b0 = t0;
      b1 = t1;
      cur = 0;
    }
  }
  // Straight-line (selects, no branches): written with ?: chains and short-circuit tests the
  // compiler branched on every condition, and the symbol loop became ~50 scalar exec-mask
  // instructions a step.
  template <int P>
  __device__ __forceinline__ bool get(int32_t k, uint32_t &w) const {
    const bool inr = (k >= 0) & ((int64_t)k < lim);
    const uintptr_t a = (uintptr_t)(Wp + k);
    const bool inb = (uint32_t)((a ^ cb) >> 5) == 0u;  // same 32-B block (the low 32 bits decide:
                                                        // k moves by words from inside cb's block)
    const uint32_t i = (uint32_t)(a >> 2);
    const zv4u lo = P ? b0 : a0, hi = P ? b1 : a1;
    const bool h4 = (i & 4u) != 0u, h1 = (i & 1u) != 0u, h2 = (i & 2u) != 0u;
    const uint32_t x0 = h4 ? hi.x : lo.x, x1 = h4 ? hi.y : lo.y, x2 = h4 ? hi.z : lo.z, x3 = h4 ? hi.w : lo.w;
    const uint32_t y0 = h1 ? x1 : x0, y1 = h1 ? x3 : x2;
    const uint32_t v = h2 ? y1 : y0;
    w = (inr & inb) ? v : 0u;
    return !inr | inb;
  }
  // start of a round reading block P: wait for everything issued before (the block itself was
  // prefetched a round ago), then prefetch the block below into the other registers. The explicit
  // wait comes first on purpose: left to the compiler, pass 2's stores (same counter, unordered
  // against loads) and the merged paths of the lanes' exits got a vmcnt(0) placed after the
  // prefetch, a wait for it. (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15.)
  template <int P>
  __device__ __forceinline__ void pre() const {
    __builtin_amdgcn_s_waitcnt(0x0F70);
    if (P == 0) ld(below(cb), b0, b1);
    else ld(below(cb), a0, a1);
  }
  // block P is used up: the block below (prefetched into the other registers) becomes current
  __device__ __forceinline__ void adv() const { cb -= 32; }
};
__device__ __forceinline__ void wd_start(const GBlk &w, const HufLane &H) { w.start((H.lp >> 5) - 1); }
template <class Wd>
struct WdBlocks {
  static constexpr bool value = false;
};
template <>
struct WdBlocks<GBlk> {
  static constexpr bool value = true;
};
template <int P, class Wd>
__device__ __forceinline__ bool wd_get_p(const Wd &w, int32_t k, uint32_t &out) {
  if constexpr (WdBlocks<Wd>::value) return w.template get<P>(k, out);
  else {
    out = w(k);
    return true;
  }
}

#ifndef ZG_LIT_BF
#define ZG_LIT_BF 1  // 1: both passes' symbol loops in straight-line form (hl_count_bf / hl_write_bf)
#endif
// Pass 1's loop without branches inside a step: the refill is computed every step and applied under a
// mask, and the loop has one exit (done, or blocked on a GBlk window). The scalar unit is shared by
// the CU's four SIMDs, and the branchy form spent ~50 scalar (exec-mask) instructions per step for
// ~45 vector ones.
template <int P, class Wd>
__device__ __forceinline__ uint32_t wd_getm(const Wd &w, int32_t k, bool &ok) {
  if constexpr (WdBlocks<Wd>::value) {
    uint32_t v;
    ok = w.template get<P>(k, v);
    return v;
  } else {
    ok = true;
    return w(k);
  }
}
template <class Wd>
__device__ __forceinline__ uint32_t hl_count_bf(HufLane &H, int32_t &p, int32_t stop, uint32_t tl,
                                                const uint16_t *huf, const Wd &word, uint32_t maxn) {
  uint32_t n = 0;
  const uint32_t sh = 64 - tl;
  auto round = [&](auto par) -> bool {
    constexpr int P = decltype(par)::value;
    if constexpr (WdBlocks<Wd>::value) word.template pre<P>();
    bool ok;
    uint32_t wn = wd_getm<P>(word, (H.lp >> 5) - 1, ok);
    bool go = (p > stop) & (n < maxn) & (ok | (H.v > 32));
    while (go) {
      const bool need = H.v <= 32;
      const uint32_t wv = need ? wn : 0u;
      H.C |= (uint64_t)wv << ((uint32_t)(32 - H.v) & 63u);
      const int32_t add = need ? 32 : 0;
      H.v += add;
      H.lp -= add;
      const uint32_t nb = huf[(uint32_t)(H.C >> sh)] >> 8;
      H.C <<= nb;
      H.v -= (int32_t)nb;
      p -= (int32_t)nb;
      n++;
      wn = wd_getm<P>(word, (H.lp >> 5) - 1, ok);
      go = (p > stop) & (n < maxn) & (ok | (H.v > 32));
    }
    return (p > stop) & (n < maxn);  // still running: stopped at the window's end
  };
  if constexpr (WdBlocks<Wd>::value) {
    word.norm();
    for (;;) {
      if (!round(std::integral_constant<int, 0>{})) break;
      word.adv();
      if (!round(std::integral_constant<int, 1>{})) {
        word.cur = 1;
        break;
      }
      word.adv();
    }
  } else {
    round(std::integral_constant<int, 0>{});
  }
  return n;
}

#if ZG_LIT_STAGE
// Pass 2 in the same form: the symbols of a lane go into 8-B words of the output aligned to 8 B; a
// completed word is the one branch of a step (every 8th symbol): the partial head word byte by byte,
// words before the first LIT_STG_W-aligned byte as 8-B stores, the rest through the lane's LDS
// window, stored as whole aligned LIT_STG_W-B pieces.
struct LitWords {
  uint8_t *wp;    // the current output word (8-B aligned)
  uint8_t *win0;  // first LIT_STG_W-aligned address at or after the lane's first byte
  uint64_t *stg8;
  uint64_t acc;
  uint32_t k, k0, staged;
  bool first;     // the current word is the head word (bytes before k0 are not the lane's)
  __device__ __forceinline__ void init(uint8_t *out, uint64_t *stg) {
    k0 = (uint32_t)((uintptr_t)out & 7);
    wp = out - k0;
    win0 = (uint8_t *)(((uintptr_t)out + LIT_STG_W - 1) & ~(uintptr_t)(LIT_STG_W - 1));
    stg8 = stg;
    acc = 0;
    k = k0;
    staged = 0;
    first = k0 != 0;
  }
  __device__ __forceinline__ void word_done() {
    if (first) {
      for (uint32_t i = k0; i < 8; i++) wp[i] = (uint8_t)(acc >> (8 * i));
      first = false;
    } else if (wp < win0) {
      *(uint64_t *)wp = acc;
    } else {
      stg8[staged] = acc;
      if (++staged == LIT_STG_W / 8) {
#ifndef ZG_LIT_NOSTORE  // lab only: the cost of the window stores (output wrong)
        uint4 *g = (uint4 *)(wp - (LIT_STG_W - 8));
        const uint4 *w = (const uint4 *)stg8;
#pragma unroll
        for (uint32_t q = 0; q < LIT_STG_W / 16; q++) g[q] = w[q];
#endif
        staged = 0;
      }
    }
    wp += 8;
    acc = 0;
    k = 0;
  }
  __device__ __forceinline__ void finish() {
    for (uint32_t q = 0; q < staged; q++) *(uint64_t *)(wp - 8 * (staged - q)) = stg8[q];
    for (uint32_t i = first ? k0 : 0u; i < k; i++) wp[i] = (uint8_t)(acc >> (8 * i));
  }
  __device__ __forceinline__ void push_byte(uint32_t b) {
    acc |= (uint64_t)(b & 255u) << (8 * k);
    if (++k == 8) word_done();
  }
  // 8 bytes at once (the next 8 of the stream, byte 0 in the low bits)
  __device__ __forceinline__ void push_word(uint64_t w) {
    const uint32_t kk = k;
    acc |= kk ? (w << (8 * kk)) : w;
    const uint64_t hi = kk ? (w >> (64 - 8 * kk)) : 0ull;
    word_done();
    acc = hi;
    k = kk;
  }
};

template <class Wd>
__device__ __forceinline__ void hl_write_bf(HufLane &H, int32_t &p, int32_t stop, uint32_t tl, const uint16_t *huf,
                                            const Wd &word, uint8_t *out, uint32_t cnt, uint4 *stg) {
  uint32_t n = 0;
  const uint32_t sh = 64 - tl;
  LitWords L;
  L.init(out, (uint64_t *)stg);
  auto round = [&](auto par) -> bool {
    constexpr int P = decltype(par)::value;
    if constexpr (WdBlocks<Wd>::value) word.template pre<P>();
    bool ok;
    uint32_t wn = wd_getm<P>(word, (H.lp >> 5) - 1, ok);
    bool go = (p > stop) & (n < cnt) & (ok | (H.v > 32));
    while (go) {
      const bool need = H.v <= 32;
      const uint32_t wv = need ? wn : 0u;
      H.C |= (uint64_t)wv << ((uint32_t)(32 - H.v) & 63u);
      const int32_t add = need ? 32 : 0;
      H.v += add;
      H.lp -= add;
      const uint32_t e = huf[(uint32_t)(H.C >> sh)];
      const uint32_t nb = e >> 8;
      H.C <<= nb;
      H.v -= (int32_t)nb;
      p -= (int32_t)nb;
      n++;
      L.acc |= (uint64_t)(e & 255u) << (8 * L.k);
      if (++L.k == 8) L.word_done();
      wn = wd_getm<P>(word, (H.lp >> 5) - 1, ok);
      go = (p > stop) & (n < cnt) & (ok | (H.v > 32));
    }
    return (p > stop) & (n < cnt);
  };
  if constexpr (WdBlocks<Wd>::value) {
    word.norm();
    for (;;) {
      if (!round(std::integral_constant<int, 0>{})) break;
      word.adv();
      if (!round(std::integral_constant<int, 1>{})) {
        word.cur = 1;
        break;
      }
      word.adv();
    }
  } else {
    round(std::integral_constant<int, 0>{});
  }
  L.finish();
}
#endif

#ifndef ZG_LIT_REC
#define ZG_LIT_REC 1  // pass 1 keeps its symbols in a per-lane record slot; pass 2 only copies (below)
#endif
// Record slot per lane: REC_OWN bytes of the lane's own chain (from its entry), then REC_RB bytes of
// a repair's true-chain prefix. A lane whose symbols do not fit decodes again (pass 2) instead.
constexpr uint32_t REC_OWN = 1024, REC_RB = 64, REC_SLOT = REC_OWN + REC_RB;
static_assert(REC_OWN % 8 == 0 && REC_RB % 8 == 0, "record slot words");

#if ZG_LIT_STAGE && ZG_LIT_BF
// Pass 1 with records: hl_count_bf's loop, each symbol also packed into 8-B words of the lane's slot
// (symbol i at slot[i]; only the first REC_OWN are kept).
template <class Wd>
__device__ __forceinline__ uint32_t hl_count_rec(HufLane &H, int32_t &p, int32_t stop, uint32_t tl,
                                                 const uint16_t *huf, const Wd &word, uint32_t maxn, uint8_t *slot,
                                                 uint64_t *stg8) {
  // 8-B words through two LIT_STG_W-byte LDS windows of the lane (stg8), a completed window stored
  // as whole 16-B pieces at the start of the next round: right after the round's wait for its
  // prefetched block, so that no wait covers a store issued less than a round before it (one store
  // per 8 symbols was 4x the store instructions, and each round start waited for the last ones).
  constexpr uint32_t WW = LIT_STG_W / 8;  // words per window
  uint32_t n = 0, pend = 0;               // completed windows not stored yet (0..2)
  uint64_t acc = 0;
  const uint32_t sh = 64 - tl;
  auto store_win = [&](uint32_t wi) {     // window wi (slot bytes [W*wi, W*wi + W)) from its LDS half
    uint4 *g = (uint4 *)(slot + (uint64_t)LIT_STG_W * wi);
    const uint4 *w = (const uint4 *)(stg8 + (wi & 1u) * WW);
#pragma unroll
    for (uint32_t q = 0; q < LIT_STG_W / 16; q++) g[q] = w[q];
  };
  auto round = [&](auto par) -> bool {
    constexpr int P = decltype(par)::value;
    if constexpr (WdBlocks<Wd>::value) word.template pre<P>();
    if (pend) {  // the windows completed in the last round
      const uint32_t wn_ = n / LIT_STG_W;  // windows completed so far
      if ((wn_ - pend + 1) * LIT_STG_W <= REC_OWN) store_win(wn_ - pend);
      if (pend == 2 && wn_ * LIT_STG_W <= REC_OWN) store_win(wn_ - 1);
      pend = 0;
    }
    bool ok;
    uint32_t wn = wd_getm<P>(word, (H.lp >> 5) - 1, ok);
    bool go = (p > stop) & (n < maxn) & (ok | (H.v > 32));
    while (go) {
      const bool need = H.v <= 32;
      const uint32_t wv = need ? wn : 0u;
      H.C |= (uint64_t)wv << ((uint32_t)(32 - H.v) & 63u);
      const int32_t add = need ? 32 : 0;
      H.v += add;
      H.lp -= add;
      const uint32_t e = huf[(uint32_t)(H.C >> sh)];
      const uint32_t nb = e >> 8;
      H.C <<= nb;
      H.v -= (int32_t)nb;
      p -= (int32_t)nb;
      const uint32_t k = n & 7u;
      acc |= (uint64_t)(e & 255u) << (8 * k);
      if (k == 7u) {
        const uint32_t wq = n >> 3;  // word index
        stg8[wq & (2 * WW - 1)] = acc;
        if ((wq & (WW - 1)) == WW - 1) {  // window wq / WW complete
          if (pend == 1) {                // the other half still holds one: store it now (rare)
            const uint32_t wi = wq / WW - 1;
            if ((wi + 1) * LIT_STG_W <= REC_OWN) store_win(wi);
          } else {
            pend = 1;
          }
        }
        acc = 0;
      }
      n++;
      wn = wd_getm<P>(word, (H.lp >> 5) - 1, ok);
      go = (p > stop) & (n < maxn) & (ok | (H.v > 32));
    }
    return (p > stop) & (n < maxn);
  };
  if constexpr (WdBlocks<Wd>::value) {
    word.norm();
    for (;;) {
      if (!round(std::integral_constant<int, 0>{})) break;
      word.adv();
      if (!round(std::integral_constant<int, 1>{})) {
        word.cur = 1;
        break;
      }
      word.adv();
    }
  } else {
    round(std::integral_constant<int, 0>{});
  }
  // the completed windows not stored yet, the last incomplete window's whole words, the partial word
  const uint32_t wn_ = n / LIT_STG_W;
  if (pend && wn_ * LIT_STG_W <= REC_OWN) store_win(wn_ - 1);
  const uint32_t wdone = n >> 3, w0 = wdone & ~(uint32_t)(WW - 1);
  if (n <= REC_OWN) {
    for (uint32_t q = w0; q < wdone; q++) *(uint64_t *)(slot + 8 * q) = stg8[q & (2 * WW - 1)];
    if (n & 7u) *(uint64_t *)(slot + (n & ~7u)) = acc;
  }
  return n;
}
#endif

// decode symbols while p > stop (at most maxn); WRITE: out[k] = symbol k
template <bool WRITE, class Wd>
__device__ __forceinline__ uint32_t hl_run(HufLane &H, int32_t &p, int32_t stop, uint32_t tl, const uint16_t *huf,
                                           const Wd &word, uint8_t *out, uint32_t maxn, uint4 *stg = nullptr) {
  uint32_t n = 0;
  const uint32_t sh = 64 - tl;
#if ZG_LIT_PACK
  // symbols are stored ZG_LIT_PACK_B at a time (aligned 8- or 16-B stores; bytes up to the first
  // boundary and the tail singly): 256 lanes writing their own segments byte by byte made every byte
  // a partial-line write-back (PMC: ~17x the literal bytes written)
  constexpr uint32_t PB = ZG_LIT_PACK_B;
  uint64_t acc = 0, acc1 = 0;
  uint32_t k = 0;
  const uint32_t head = WRITE ? (uint32_t)((PB - ((uintptr_t)out & (PB - 1))) & (PB - 1)) : 0u;
#if ZG_LIT_STAGE
  // 8-B words from the first 64-B boundary on go to the lane's LDS window; a completed window leaves
  // as four aligned 16-B stores (a whole half-line at once, no partial-line write-backs)
  static_assert(!ZG_LIT_STAGE || ZG_LIT_PACK_B == 8, "literal staging packs 8-B words");
  const uint32_t head64 = WRITE ? (uint32_t)((LIT_STG_W - ((uintptr_t)out & (LIT_STG_W - 1))) & (LIT_STG_W - 1)) : 0u;
  uint64_t *stg8 = (uint64_t *)stg;
#endif
#endif
  // Rounds: with a block-window reader (GBlk) a lane whose next word lies below its window stops
  // until every lane of the wave has stopped or finished; the window then moves down one block.
  // Other readers never stop: one round.
  auto round = [&](auto par) -> bool {
  constexpr int P = decltype(par)::value;
  if constexpr (WdBlocks<Wd>::value) word.template pre<P>();
  bool blk = false;
  while (p > stop && n < maxn) {
    if (H.v <= 32) {
      uint32_t w;
      if (!wd_get_p<P>(word, (H.lp >> 5) - 1, w)) {
        blk = true;
        break;
      }
      H.C |= (uint64_t)w << (32 - H.v);
      H.v += 32;
      H.lp -= 32;
    }
    const uint32_t e = huf[(uint32_t)(H.C >> sh)];
    const uint32_t nb = e >> 8;
    H.C <<= nb;
    H.v -= (int32_t)nb;
    p -= (int32_t)nb;
#if ZG_LIT_PACK
    if (WRITE) {
      if (n < head) {
        out[n] = (uint8_t)e;
      } else {
        if (PB == 16 && k >= 8) acc1 |= (uint64_t)(e & 255u) << (8 * (k - 8));
        else acc |= (uint64_t)(e & 255u) << (8 * k);
        if (++k == PB) {
          if (PB == 16) {
            *(uint4 *)(out + n - 15) = make_uint4((uint32_t)acc, (uint32_t)(acc >> 32), (uint32_t)acc1, (uint32_t)(acc1 >> 32));
          } else {
#if ZG_LIT_STAGE
            const uint32_t pos = n - 7;
            if (pos < head64) {
              *(uint64_t *)(out + pos) = acc;
            } else {
              const uint32_t r = (pos - head64) & (LIT_STG_W - 1);
              stg8[r >> 3] = acc;
              if (r == LIT_STG_W - 8) {  // window complete: out + pos - r is W-aligned
                uint4 *g = (uint4 *)(out + pos - r);
#pragma unroll
                for (uint32_t q = 0; q < LIT_STG_W / 16; q++) g[q] = stg[q];
              }
            }
#else
            *(uint64_t *)(out + n - 7) = acc;
#endif
          }
          acc = acc1 = 0;
          k = 0;
        }
      }
    }
#else
    if (WRITE) out[n] = (uint8_t)e;
#endif
    n++;
  }
  return blk;
  };
  if constexpr (WdBlocks<Wd>::value) {
    word.norm();
    for (;;) {
      if (!round(std::integral_constant<int, 0>{})) break;
      word.adv();
      if (!round(std::integral_constant<int, 1>{})) {
        word.cur = 1;
        break;
      }
      word.adv();
    }
  } else {
    round(std::integral_constant<int, 0>{});
  }
#if ZG_LIT_PACK
#if ZG_LIT_STAGE
  if (WRITE && n - k > head64) {  // the staged words of the last, incomplete window
    const uint32_t done = n - k;  // bytes stored or staged as whole words
    const uint32_t w0 = done - ((done - head64) & (LIT_STG_W - 1));
    for (uint32_t q = w0; q < done; q += 8) *(uint64_t *)(out + q) = stg8[((q - head64) & (LIT_STG_W - 1)) >> 3];
  }
#endif
  if (WRITE)
    for (uint32_t i = 0; i < k; i++) out[n - k + i] = (uint8_t)((i < 8 ? acc : acc1) >> (8 * (i & 7)));
#endif
  return n;
}

// Literal-section words read from global memory through a per-lane window: a lane walks its segment
// backwards one word at a time, so one aligned 32-B load serves eight words (scattered 4-B loads of
// 256 lanes fetched ~10x the section bytes from HBM), and the next lower 32 B are already in flight
// while the current ones are decoded (the decode otherwise waits a full HBM round trip every
// 128 bits).
struct GWordPF {
  const gu32 *Wp;
  int64_t lim;
  mutable uintptr_t cb;       // address of the cached 32-B block (1: none)
  mutable zv4u c0, c1;        // its words 0-3, 4-7
  mutable zv4u n0, n1;        // the block below it (prefetched)
  mutable uintptr_t nb;       // address of the block in n0/n1 (1: none)
  mutable bool pf;            // the block below cb is still to be prefetched
  __device__ __forceinline__ static void ld(uintptr_t b, zv4u &x0, zv4u &x1) {
    const __attribute__((address_space(1))) zv4u *q = (const __attribute__((address_space(1))) zv4u *)b;
    x0 = q[0];
    x1 = q[1];
  }
  // The prefetch is issued on the first call after a block switch, not at the switch: issued at the
  // switch, next to the copy of the prefetched block into c0/c1, it made the compiler wait for the
  // new loads at once (s_waitcnt vmcnt(0) before the block's first use, the prefetch's result moved
  // between registers), so every switch paid a full memory round trip. Here the only load pending at
  // a switch is the one issued seven words earlier.
  // (The word is picked in each branch: picked after the merge, the compiler's wait for a switch's
  // loads also covered the other branch's prefetch.)
  __device__ __forceinline__ static uint32_t pick(const zv4u &x0, const zv4u &x1, uintptr_t a) {
    const uint32_t i = (uint32_t)(a >> 2) & 7u;
    const zv4u h = i < 4 ? x0 : x1;
    const uint32_t j = i & 3u;
    return j == 0 ? h.x : j == 1 ? h.y : j == 2 ? h.z : h.w;
  }
  __device__ __forceinline__ uint32_t operator()(int32_t k) const {
    if (k < 0 || k >= lim) return 0u;
    const uintptr_t a = (uintptr_t)(Wp + k), b = a & ~(uintptr_t)31;
    if (b != cb) {
      if (b == nb) {  // the next lower block: take the prefetched copy
        c0 = n0;
        c1 = n1;
      } else {
        ld(b, c0, c1);
      }
      cb = b;
      nb = 1;
      pf = b > ((uintptr_t)Wp & ~(uintptr_t)31);  // the block below still holds words of the section
      return pick(c0, c1, a);
    }
    const uint32_t w = pick(c0, c1, a);
    if (pf) {
      ld(b - 32, n0, n1);
      nb = b - 32;
      pf = false;
    }
    return w;
  }
};

// A 64-B window with the 64-B block below it prefetched (ZG_LIT_GWIN 3): a lane reads each 128-B line
// of its segment in two pieces instead of four. 256 lanes per workgroup read 256 lines spread over a
// section, and between a lane's pieces of one line L2 has usually evicted it, so every piece was a
// fabric fetch of its own (C5 PMC: ~4x the compressed literal bytes fetched).
struct GWordPF64 {
  const gu32 *Wp;
  int64_t lim;
  mutable uintptr_t cb;  // address of the cached 64-B block (1: none)
  mutable zv4u c[4];     // its words
  mutable zv4u n[4];     // the block below it (prefetched)
  __device__ __forceinline__ static void ld(uintptr_t b, zv4u *x) {
    const __attribute__((address_space(1))) zv4u *q = (const __attribute__((address_space(1))) zv4u *)b;
#pragma unroll
    for (int i = 0; i < 4; i++) x[i] = q[i];
  }
  __device__ __forceinline__ uint32_t operator()(int32_t k) const {
    if (k < 0 || k >= lim) return 0u;
    const uintptr_t a = (uintptr_t)(Wp + k), b = a & ~(uintptr_t)63;
    if (b != cb) {
      if (b + 64 == cb) {
#pragma unroll
        for (int i = 0; i < 4; i++) c[i] = n[i];
      } else {
        ld(b, c);
      }
      cb = b;
      if (b > ((uintptr_t)Wp & ~(uintptr_t)63)) ld(b - 64, n);
    }
    const uint32_t i = (uint32_t)(a >> 2) & 15u;
    const zv4u h = (i >> 2) == 0 ? c[0] : (i >> 2) == 1 ? c[1] : (i >> 2) == 2 ? c[2] : c[3];
    const uint32_t j = i & 3u;
    return j == 0 ? h.x : j == 1 ? h.y : j == 2 ? h.z : h.w;
  }
};

struct GWord {
  const gu32 *Wp;
  int64_t lim;
  mutable uintptr_t cb;  // address of the cached 16-B block (1: none)
  mutable zv4u c;
  __device__ __forceinline__ uint32_t operator()(int32_t k) const {
    if (k < 0 || k >= lim) return 0u;
    const uintptr_t a = (uintptr_t)(Wp + k), b = a & ~(uintptr_t)15;
    if (b != cb) {
      cb = b;
      c = *(const __attribute__((address_space(1))) zv4u *)b;
    }
    const uint32_t i = (uint32_t)(a >> 2) & 3u;
    return i == 0 ? c.x : i == 1 ? c.y : i == 2 ? c.z : c.w;
  }
};

#ifdef ZG_LIT_STATS
// lab counters (tools/lab/zstd_lab.cpp): blocks, blocks with repairs, repair rounds, lanes re-decoded,
// symbols, warm-up symbols, lanes
__device__ unsigned long long g_litstats[8];
#define LS_ADD(k, v) atomicAdd(&g_litstats[k], (unsigned long long)(v))
#else
#define LS_ADD(k, v) ((void)0)
#endif
#ifdef ZG_LIT_PROF
// lab phase clocks of k_zstd_lits (thread 0 of each workgroup, s_memtime ticks): pass 1, repairs,
// prefix + checks, pass 2, staging of the section (LDS path), records
__device__ unsigned long long g_litprof[8];
#define LP_T(v) const uint64_t v = (threadIdx.x == 0) ? __builtin_amdgcn_s_memtime() : 0
#define LP_ADD(k, a, b) do { if (threadIdx.x == 0) atomicAdd(&g_litprof[k], (unsigned long long)((b) - (a))); } while (0)
#else
#define LP_T(v) ((void)0)
#define LP_ADD(k, a, b) ((void)0)
#endif

// uncached word reads for the rare repair walks (the cached readers' state stays out of them)
template <class Wd>
__device__ __forceinline__ uint32_t word_raw(const Wd &w, int32_t k) { return w(k); }
__device__ __forceinline__ uint32_t word_raw(const GWordPF &w, int32_t k) { return (k >= 0 && k < w.lim) ? w.Wp[k] : 0u; }
__device__ __forceinline__ uint32_t word_raw(const GWordPF64 &w, int32_t k) { return (k >= 0 && k < w.lim) ? w.Wp[k] : 0u; }
__device__ __forceinline__ uint32_t word_raw(const GWord &w, int32_t k) { return (k >= 0 && k < w.lim) ? w.Wp[k] : 0u; }
__device__ __forceinline__ uint32_t word_raw(const GBlk &w, int32_t k) { return w(k); }
template <class Wd>
struct RawWord {
  const Wd &w;
  __device__ __forceinline__ uint32_t operator()(int32_t k) const { return word_raw(w, k); }
};

// one symbol of a lane's chain (position p moves down by the code length)
template <class Wd>
__device__ __forceinline__ uint32_t hl_step(HufLane &H, int32_t &p, uint32_t tl, const uint16_t *huf, const Wd &word) {
  if (H.v <= 32) {
    H.C |= (uint64_t)word((H.lp >> 5) - 1) << (32 - H.v);
    H.v += 32;
    H.lp -= 32;
  }
  const uint32_t e = huf[(uint32_t)(H.C >> (64 - tl))];
  const uint32_t nb = e >> 8;
  H.C <<= nb;
  H.v -= (int32_t)nb;
  p -= (int32_t)nb;
  return e & 255u;
}

#ifndef ZG_LIT_SYNC
#define ZG_LIT_SYNC 1  // repair by sync-point search (0: re-decode the whole segment)
#endif

template <class Wd>
__device__ bool lits_decode(ZLitSmem &S, const Wd &word, uint32_t nstreams, const int32_t *top, const int32_t *lob,
                            const uint32_t *nsym, uint32_t tl, uint8_t *lit, uint32_t seg, uint8_t *slot = nullptr) {
  const uint32_t t = threadIdx.x;
  const uint32_t G = LIT_THREADS / nstreams;
  const uint32_t s = t / G, j = t % G;
  const int32_t T0 = s == 0 ? top[0] : s == 1 ? top[1] : s == 2 ? top[2] : top[3];
  const int32_t L0 = s == 0 ? lob[0] : s == 1 ? lob[1] : s == 2 ? lob[2] : lob[3];
  const uint32_t NS = s == 0 ? nsym[0] : s == 1 ? nsym[1] : s == 2 ? nsym[2] : nsym[3];
  const int64_t len = (int64_t)T0 - L0;
  const int32_t tj = T0 - (int32_t)(len * j / G), tj1 = T0 - (int32_t)(len * (j + 1) / G);
  const uint32_t maxn = NS + 1;  // a segment never holds more symbols than its stream
  LP_T(tp0);
  // pass 1: entry / exit / count (its own copy of a cached reader, dead after the pass)
  {
    const Wd w1 = word;
    HufLane H;
    int32_t p = j == 0 ? T0 : min(T0, tj + LIT_WARM);
    hl_init(H, p, w1);
    wd_start(w1, H);
#if ZG_LIT_BF
    if (j) {
      const uint32_t wn = hl_count_bf(H, p, tj, tl, S.huf, w1, 0xFFFFFFFFu);
      LS_ADD(5, wn);
      (void)wn;
    }
    S.entry[t] = p;
#if ZG_LIT_REC && ZG_LIT_STAGE
    S.cnt[t] = slot ? hl_count_rec(H, p, tj1, tl, S.huf, w1, maxn, slot, (uint64_t *)&S.stg[t * (LIT_STG_PITCH / 16)])
                    : hl_count_bf(H, p, tj1, tl, S.huf, w1, maxn);
#else
    S.cnt[t] = hl_count_bf(H, p, tj1, tl, S.huf, w1, maxn);
#endif
#else
    if (j) {
      const uint32_t wn = hl_run<false>(H, p, tj, tl, S.huf, w1, nullptr, 0xFFFFFFFFu);
      LS_ADD(5, wn);
      (void)wn;
    }
    S.entry[t] = p;
    S.cnt[t] = hl_run<false>(H, p, tj1, tl, S.huf, w1, nullptr, maxn);
#endif
    S.exit_[t] = p;
  }
  __syncthreads();
  LP_T(tp1);
  LP_ADD(0, tp0, tp1);
  // records: the lane's final symbols are rec_nt repair-prefix symbols (slot tail) followed by its own
  // symbols [rec_nw, cnt_own) (none when the true chain left the segment without meeting the lane's)
  const uint32_t cnt_own = S.cnt[t];
  uint32_t rec_nw = 0, rec_nt = 0;
  bool rec_full = false, rec_again = false, fixed_once = false;  // rec_again: fixed twice (a chain further up changed after
                                             // the first fix): the records no longer describe it
  // repair rounds: a lane whose entry is not its predecessor's exit re-decodes from that exit once
  // the predecessor is right (a lane is right when its entry is right)
  for (uint32_t round = 0; round < G; round++) {
    const bool wrong = j != 0 && S.entry[t] != S.exit_[t - 1];
    const bool pred_ok = j <= 1 || S.entry[t - 1] == S.exit_[t - 2];
    __syncthreads();
    int32_t ne = 0, nx = 0;
    uint32_t nc = 0;
    const bool fix = wrong && pred_ok;
#ifdef ZG_LIT_STATS
    if (fix) LS_ADD(3, 1);
    if (t == 0 && round == 0) LS_ADD(0, 1);
#endif
    if (fix) {
#if ZG_LIT_SYNC
      // The lane's own chain (from its warm-up entry) is wrong only until it meets the true chain
      // (from the predecessor's exit): walk both, always stepping the one further up the stream,
      // until they meet (the count differs by the symbols each took to get there; the exit is the
      // lane's own) or the true chain leaves the segment without meeting it (its count and exit).
      // Huffman chains meet within a few symbols, so a repair costs a few symbols, not a segment.
      const RawWord<Wd> rw{word};
      HufLane Ht, Hw;
      int32_t pt = S.exit_[t - 1], pw = S.entry[t];
      ne = pt;
      hl_init(Ht, pt, rw);
      hl_init(Hw, pw, rw);
      uint32_t nt = 0, nw = 0;
      bool full_now = false;
      for (;;) {
        if (pt == pw) {
          nc = S.cnt[t] - nw + nt;
          nx = S.exit_[t];
          break;
        }
        if (pt <= tj1 || nt > maxn || nw > maxn) {
          nc = nt;
          nx = pt;
          full_now = true;
          break;
        }
        if (pt > pw) {
          const uint32_t e = hl_step(Ht, pt, tl, S.huf, rw);
          if (slot && nt < REC_RB) slot[REC_OWN + nt] = (uint8_t)e;
          nt++;
        } else {
          hl_step(Hw, pw, tl, S.huf, rw);
          nw++;
        }
      }
      rec_again = rec_again || fixed_once;
      fixed_once = true;
      rec_full = full_now;
      rec_nw = nw;
      rec_nt = nt;
#else
      HufLane H;
      int32_t p = S.exit_[t - 1];
      ne = p;
      hl_init(H, p, word);
      wd_start(word, H);
      nc = hl_run<false>(H, p, tj1, tl, S.huf, word, nullptr, maxn);
      rec_again = true;  // nothing recorded on this path: decode again
      nx = p;
#endif
    }
    if (__syncthreads_or(wrong) == 0) break;
#ifdef ZG_LIT_STATS
    if (t == 0) {
      LS_ADD(2, 1);
      if (round == 0) LS_ADD(1, 1);
    }
#endif
    if (fix) {
      S.entry[t] = ne;
      S.exit_[t] = nx;
      S.cnt[t] = nc;
    }
    __syncthreads();
  }
  LP_T(tp2);
  LP_ADD(1, tp1, tp2);
  // every lane right now; per-stream symbol count and exact end
  uint32_t c = S.cnt[t];
  LS_ADD(4, c);
  LS_ADD(6, 1);
  const uint32_t lane = lane_id();
  uint32_t incl = c;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u = __shfl_up(incl, o, 64);
    if ((int)lane >= o) incl += u;
  }
  if (lane == 63) S.wsum[t >> 6] = incl;
  __syncthreads();
  uint32_t base = 0;
  if (nstreams == 1)
    for (uint32_t w = 0; w < (t >> 6); w++) base += S.wsum[w];
  const uint32_t off = base + incl - c;
  uint32_t total = 0;
  if (nstreams == 1) total = S.wsum[0] + S.wsum[1] + S.wsum[2] + S.wsum[3];
  else total = S.wsum[s];
  bool bad = total != NS || S.entry[t] != (j == 0 ? T0 : S.exit_[t - 1]);
  if (j == G - 1 && S.exit_[t] != L0) bad = true;
  if (__syncthreads_or(bad)) return false;
  LP_T(tp3);
  LP_ADD(2, tp2, tp3);
  bool redo = c != 0;  // pass 2 (decode again, writing) for this lane
#if ZG_LIT_REC && ZG_LIT_STAGE && ZG_LIT_BF
  // The lane's slot stores (pass 1, repairs) before its reads, and the CU's vector L1 invalidated:
  // stores do not update lines the L1 already holds, and the slot's lines were read (and cached) by
  // this lane's copy of the previous record - without the invalidate it read that record's bytes.
  if (slot) {
    __builtin_amdgcn_s_waitcnt(0);                      // the stores acknowledged (in L2)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");  // buffer_inv: the L1 refetches
  }
  if (slot && c) {
    // the recorded symbols, copied: fall back to pass 2 when a part did not fit its slot region
    // c = the first npre true-chain symbols of a repair, then own symbols from rec_nw on. (Chains can
    // meet below the segment's end, after the own chain's last symbol: then the segment is the true
    // chain's first c symbols and nothing of the own chain.)
    const uint32_t npre = min(rec_nt, c), n_own = c - npre;
    const bool fits = !rec_again && npre <= REC_RB &&
                      (n_own == 0 || (!rec_full && rec_nw + n_own == cnt_own && cnt_own <= REC_OWN));
    if (fits) {
      redo = false;
      LitWords L;
      L.init(lit + (uint64_t)s * seg + off, (uint64_t *)&S.stg[t * (LIT_STG_PITCH / 16)]);
      for (uint32_t i = 0; i < npre; i++) L.push_byte(slot[REC_OWN + i]);
      if (n_own) {
        // own symbols [rec_nw, cnt_own): aligned 8-B slot words, funnel-shifted
        const uint32_t a = rec_nw & 7u;
        const uint64_t *sw = (const uint64_t *)(slot + (rec_nw & ~7u));
        uint64_t cur = sw[0];
        uint32_t i = 0;
        // 64 bytes per group: the group's eight loads in flight together (one round trip, not eight)
        for (; i + 64 <= n_own; i += 64) {
          uint64_t w[8];
#pragma unroll
          for (int q = 0; q < 8; q++) w[q] = sw[(i >> 3) + 1 + q];
#pragma unroll
          for (int q = 0; q < 8; q++) {
            L.push_word(a ? (cur >> (8 * a)) | (w[q] << (64 - 8 * a)) : cur);
            cur = w[q];
          }
        }
        for (; i + 8 <= n_own; i += 8) {
          const uint64_t nxt = sw[(i >> 3) + 1];
          L.push_word(a ? (cur >> (8 * a)) | (nxt << (64 - 8 * a)) : cur);
          cur = nxt;
        }
        if (i < n_own) {
          const uint64_t nxt = (a + (n_own - i) > 8) ? sw[(i >> 3) + 1] : 0ull;
          const uint64_t w = a ? (cur >> (8 * a)) | (nxt << (64 - 8 * a)) : cur;
          for (uint32_t q = 0; q < n_own - i; q++) L.push_byte((uint32_t)(w >> (8 * q)));
        }
      }
      L.finish();
    }
  }
  LS_ADD(7, redo ? 1 : 0);
#ifdef ZG_LIT_REC_DEBUG  // lab: decode each copied lane again and report the first differing byte
  if (slot && c && !redo) {
    __builtin_amdgcn_s_waitcnt(0);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    const RawWord<Wd> rw{word};
    HufLane Hd;
    int32_t pd = S.entry[t];
    hl_init(Hd, pd, rw);
    const uint8_t *o = lit + (uint64_t)s * seg + off;
    for (uint32_t i = 0; i < c; i++) {
      const uint32_t e = hl_step(Hd, pd, tl, S.huf, rw);
      if ((uint8_t)e != o[i]) {
        printf("litrec: t %u s %u j %u c %u i %u exp %u got %u | cnt_own %u nw %u nt %u full %d entry %d exit %d tj %d tj1 %d\n",
               t, s, j, c, i, e, (uint32_t)o[i], cnt_own, rec_nw, rec_nt, (int)rec_full, S.entry[t], S.exit_[t], tj, tj1);
        break;
      }
    }
  }
#endif
#endif
  // pass 2: decode again, writing
  if (redo) {
    const Wd w2 = word;
    HufLane H;
    int32_t p = S.entry[t];
    hl_init(H, p, w2);
    wd_start(w2, H);
#if ZG_LIT_STAGE && ZG_LIT_BF
    hl_write_bf(H, p, tj1, tl, S.huf, w2, lit + (uint64_t)s * seg + off, c, &S.stg[t * (LIT_STG_PITCH / 16)]);
#elif ZG_LIT_STAGE
    hl_run<true>(H, p, tj1, tl, S.huf, w2, lit + (uint64_t)s * seg + off, c, &S.stg[t * (LIT_STG_PITCH / 16)]);
#else
    hl_run<true>(H, p, tj1, tl, S.huf, w2, lit + (uint64_t)s * seg + off, c);
#endif
  }
#ifdef ZG_LIT_PROF
  __syncthreads();
  LP_T(tp4);
  LP_ADD(3, tp3, tp4);
  LP_ADD(5, 0, 1);
#endif
  return true;
}

#if ZG_LIT_ILP == 2
// Two chains per lane. A symbol step is one dependent LDS table read plus ~15 instructions; with
// one chain per lane the wave waits out that read every symbol and the SIMD issues a third of its
// cycles (4 waves each). A lane here owns segments t and t + LIT_THREADS of the record's 512 and
// advances both every step, so two table reads are in flight per wave.

// Writer of one chain's decoded literals (hl_run<true>'s packing): bytes up to the first 8-B
// boundary singly, then 8-B words, from the first LIT_STG_W-aligned byte on through the segment's
// LDS window as whole aligned LIT_STG_W-B pieces.
struct LitPack {
  uint8_t *out;
  uint64_t *stg8;
  uint64_t acc;
  uint32_t k, n, head, head64;
  __device__ __forceinline__ void init(uint8_t *o, uint4 *stg) {
    out = o;
    stg8 = (uint64_t *)stg;
    acc = 0;
    k = n = 0;
    head = (uint32_t)((8 - ((uintptr_t)o & 7)) & 7);
    head64 = (uint32_t)((LIT_STG_W - ((uintptr_t)o & (LIT_STG_W - 1))) & (LIT_STG_W - 1));
  }
  __device__ __forceinline__ void push(uint32_t e) {
    if (n < head) {
      out[n] = (uint8_t)e;
    } else {
      acc |= (uint64_t)(e & 255u) << (8 * k);
      if (++k == 8) {
        const uint32_t pos = n - 7;
        if (pos < head64) {
          *(uint64_t *)(out + pos) = acc;
        } else {
          const uint32_t r = (pos - head64) & (LIT_STG_W - 1);
          stg8[r >> 3] = acc;
          if (r == LIT_STG_W - 8) {  // window complete: out + pos - r is W-aligned
            uint4 *g = (uint4 *)(out + pos - r);
            const uint4 *w = (const uint4 *)stg8;
#pragma unroll
            for (uint32_t q = 0; q < LIT_STG_W / 16; q++) g[q] = w[q];
          }
        }
        acc = 0;
        k = 0;
      }
    }
    n++;
  }
  __device__ __forceinline__ void finish() {
    if (n - k > head64) {  // the staged words of the last, incomplete window
      const uint32_t done = n - k;
      const uint32_t w0 = done - ((done - head64) & (LIT_STG_W - 1));
      for (uint32_t q = w0; q < done; q += 8) *(uint64_t *)(out + q) = stg8[((q - head64) & (LIT_STG_W - 1)) >> 3];
    }
    for (uint32_t i = 0; i < k; i++) out[n - k + i] = (uint8_t)(acc >> (8 * i));
  }
};

// Advance two chains while p > stop and n < maxn, each on its own word reader; both table reads of
// a step are issued before either is used.
template <bool WRITE, class Wd>
__device__ __forceinline__ void hl_run2(HufLane &H0, int32_t &p0, int32_t stop0, uint32_t &n0, uint32_t max0,
                                        const Wd &w0, HufLane &H1, int32_t &p1, int32_t stop1, uint32_t &n1,
                                        uint32_t max1, const Wd &w1, uint32_t tl, const uint16_t *huf, LitPack *P0,
                                        LitPack *P1) {
  const uint32_t sh = 64 - tl;
  bool a0 = p0 > stop0 && n0 < max0, a1 = p1 > stop1 && n1 < max1;
  while (a0 || a1) {
    if (a0 && H0.v <= 32) {
      H0.C |= (uint64_t)w0((H0.lp >> 5) - 1) << (32 - H0.v);
      H0.v += 32;
      H0.lp -= 32;
    }
    if (a1 && H1.v <= 32) {
      H1.C |= (uint64_t)w1((H1.lp >> 5) - 1) << (32 - H1.v);
      H1.v += 32;
      H1.lp -= 32;
    }
    const uint32_t e0 = huf[(uint32_t)(H0.C >> sh)], e1 = huf[(uint32_t)(H1.C >> sh)];
    if (a0) {
      const uint32_t nb = e0 >> 8;
      H0.C <<= nb;
      H0.v -= (int32_t)nb;
      p0 -= (int32_t)nb;
      if (WRITE) P0->push(e0);
      n0++;
      a0 = p0 > stop0 && n0 < max0;
    }
    if (a1) {
      const uint32_t nb = e1 >> 8;
      H1.C <<= nb;
      H1.v -= (int32_t)nb;
      p1 -= (int32_t)nb;
      if (WRITE) P1->push(e1);
      n1++;
      a1 = p1 > stop1 && n1 < max1;
    }
  }
}

__device__ __forceinline__ int32_t pick4(const int32_t *a, uint32_t s) {
  return s == 0 ? a[0] : s == 1 ? a[1] : s == 2 ? a[2] : a[3];
}
__device__ __forceinline__ uint32_t pick4(const uint32_t *a, uint32_t s) {
  return s == 0 ? a[0] : s == 1 ? a[1] : s == 2 ? a[2] : a[3];
}

// lits_decode with LIT_SEGS = 512 segments (same passes, repair rule and output layout).
template <class Wd>
__device__ bool lits_decode2(ZLitSmem &S, const Wd &word, uint32_t nstreams, const int32_t *top, const int32_t *lob,
                             const uint32_t *nsym, uint32_t tl, uint8_t *lit, uint32_t seg) {
  const uint32_t t = threadIdx.x;
  const uint32_t G = LIT_SEGS / nstreams;  // segments per stream (a multiple of 64)
  uint32_t gi[2], si[2], ji[2], NS[2];
  int32_t T0[2], L0[2], tj[2], tj1[2];
#pragma unroll
  for (int c = 0; c < 2; c++) {
    gi[c] = t + c * LIT_THREADS;
    si[c] = gi[c] / G;
    ji[c] = gi[c] % G;
    T0[c] = pick4(top, si[c]);
    L0[c] = pick4(lob, si[c]);
    NS[c] = pick4(nsym, si[c]);
    const int64_t len = (int64_t)T0[c] - L0[c];
    tj[c] = T0[c] - (int32_t)(len * ji[c] / G);
    tj1[c] = T0[c] - (int32_t)(len * (ji[c] + 1) / G);
  }
  // pass 1: entry / exit / count of both segments
  {
    const Wd wa = word, wb = word;
    HufLane H0, H1;
    int32_t p0 = ji[0] == 0 ? T0[0] : min(T0[0], tj[0] + LIT_WARM);
    int32_t p1 = ji[1] == 0 ? T0[1] : min(T0[1], tj[1] + LIT_WARM);
    hl_init(H0, p0, wa);
    hl_init(H1, p1, wb);
    uint32_t n0 = 0, n1 = 0;
    hl_run2<false>(H0, p0, ji[0] ? tj[0] : p0, n0, 0xFFFFFFFFu, wa, H1, p1, ji[1] ? tj[1] : p1, n1, 0xFFFFFFFFu, wb,
                   tl, S.huf, nullptr, nullptr);
    LS_ADD(5, n0 + n1);
    S.entry[gi[0]] = p0;
    S.entry[gi[1]] = p1;
    n0 = n1 = 0;
    hl_run2<false>(H0, p0, tj1[0], n0, NS[0] + 1, wa, H1, p1, tj1[1], n1, NS[1] + 1, wb, tl, S.huf, nullptr, nullptr);
    S.cnt[gi[0]] = n0;
    S.cnt[gi[1]] = n1;
    S.exit_[gi[0]] = p0;
    S.exit_[gi[1]] = p1;
  }
  __syncthreads();
  // repair rounds (lits_decode's rule, per segment)
  for (uint32_t round = 0; round < G; round++) {
    bool wrong[2], fix[2];
    int32_t ne[2] = {0, 0}, nx[2] = {0, 0};
    uint32_t nc[2] = {0, 0};
#pragma unroll
    for (int c = 0; c < 2; c++) {
      const uint32_t g = gi[c], j = ji[c];
      wrong[c] = j != 0 && S.entry[g] != S.exit_[g - 1];
      fix[c] = wrong[c] && (j <= 1 || S.entry[g - 1] == S.exit_[g - 2]);
    }
    __syncthreads();
    for (int c = 0; c < 2; c++) {
      if (!fix[c]) continue;
      const uint32_t g = gi[c];
      const uint32_t maxn = NS[c] + 1;
      const RawWord<Wd> rw{word};
      HufLane Ht, Hw;
      int32_t pt = S.exit_[g - 1], pw = S.entry[g];
      ne[c] = pt;
      hl_init(Ht, pt, rw);
      hl_init(Hw, pw, rw);
      uint32_t nt = 0, nw = 0;
      for (;;) {
        if (pt == pw) {
          nc[c] = S.cnt[g] - nw + nt;
          nx[c] = S.exit_[g];
          break;
        }
        if (pt <= tj1[c] || nt > maxn || nw > maxn) {
          nc[c] = nt;
          nx[c] = pt;
          break;
        }
        if (pt > pw) {
          hl_step(Ht, pt, tl, S.huf, rw);
          nt++;
        } else {
          hl_step(Hw, pw, tl, S.huf, rw);
          nw++;
        }
      }
    }
    if (__syncthreads_or(wrong[0] || wrong[1]) == 0) break;
#pragma unroll
    for (int c = 0; c < 2; c++)
      if (fix[c]) {
        S.entry[gi[c]] = ne[c];
        S.exit_[gi[c]] = nx[c];
        S.cnt[gi[c]] = nc[c];
      }
    __syncthreads();
  }
  // prefix sums in segment order: wave-chain k = c * 4 + wave holds segments [64k, 64k + 64)
  const uint32_t c0 = S.cnt[gi[0]], c1 = S.cnt[gi[1]];
  LS_ADD(4, c0 + c1);
  LS_ADD(6, 2);
  const uint32_t lane = lane_id(), wave = t >> 6;
  uint32_t i0 = c0, i1 = c1;
  for (int o = 1; o < 64; o <<= 1) {
    const uint32_t u0 = __shfl_up(i0, o, 64), u1 = __shfl_up(i1, o, 64);
    if ((int)lane >= o) {
      i0 += u0;
      i1 += u1;
    }
  }
  if (lane == 63) {
    S.wsum[wave] = i0;
    S.wsum[4 + wave] = i1;
  }
  __syncthreads();
  auto pre = [&S](uint32_t k) {  // symbols in wave-chains before k
    uint32_t b = 0;
    for (uint32_t q = 0; q < k; q++) b += S.wsum[q];
    return b;
  };
  uint32_t off[2];
  bool bad = false;
#pragma unroll
  for (int c = 0; c < 2; c++) {
    const uint32_t g = gi[c], j = ji[c], k = c * 4 + wave;
    const uint32_t k0 = si[c] * G / 64, k1 = (si[c] + 1) * G / 64;  // the stream's wave-chains
    const uint32_t sb = pre(k0);
    off[c] = pre(k) + (c ? i1 - c1 : i0 - c0) - sb;
    if (pre(k1) - sb != NS[c]) bad = true;
    if (S.entry[g] != (j == 0 ? T0[c] : S.exit_[g - 1])) bad = true;
    if (j == G - 1 && S.exit_[g] != L0[c]) bad = true;
  }
  if (__syncthreads_or(bad)) return false;
  // pass 2: decode again, writing
  if (c0 || c1) {
    const Wd wa = word, wb = word;
    HufLane H0, H1;
    int32_t p0 = S.entry[gi[0]], p1 = S.entry[gi[1]];
    hl_init(H0, p0, wa);
    hl_init(H1, p1, wb);
    LitPack P0, P1;
    P0.init(lit + (uint64_t)si[0] * seg + off[0], &S.stg[gi[0] * (LIT_STG_PITCH / 16)]);
    P1.init(lit + (uint64_t)si[1] * seg + off[1], &S.stg[gi[1] * (LIT_STG_PITCH / 16)]);
    uint32_t n0 = 0, n1 = 0;
    hl_run2<true>(H0, p0, tj1[0], n0, c0, wa, H1, p1, tj1[1], n1, c1, wb, tl, S.huf, &P0, &P1);
    P0.finish();
    P1.finish();
  }
  return true;
}
#endif

#if ZG_HUF_SPLIT
struct ZHufSmem {
  uint16_t huf[1 << MAX_HUF_LOG];
  Fse wt[64];
  int16_t norm[64];
  uint8_t weights[256];
  uint16_t hsorted[256];
  uint32_t tmp[32];
};

// One wave per Huffman-literal block record (block-major, like k_zstd_lits): parse the tree
// description in effect and build the decoding table into the literal scratch ahead of the block's
// literals. Kept out of k_zstd_lits: the table build needs ~110 more VGPRs than the decode, which
// held the 256-lane literal decoder to 2 workgroups per CU while 3 of its 4 waves waited.
__global__ __launch_bounds__(64) void k_zstd_huf(const ZgItem *items, const uint32_t *status, const ZBlk *blks,
                                                 uint32_t blk_cap, const uint32_t *nblk, const uint32_t *zmode,
                                                 uint32_t n_items, uint8_t *lit_scratch, uint64_t lit_stride,
                                                 const unsigned long long *max_nblk) {
  __shared__ __attribute__((aligned(16))) ZHufSmem S;
  const uint32_t lane = threadIdx.x;
  const uint64_t total = (uint64_t)n_items * rec_blocks(blk_cap, max_nblk);
  for (uint64_t g = blockIdx.x; g < total; g += gridDim.x) {
    const uint32_t item = (uint32_t)(g % n_items), bi = (uint32_t)(g / n_items);  // block-major order
    if (bi >= nblk[item] || zmode[item] != ZMODE_PARALLEL) continue;
    const ZBlk *Bp = blks + (uint64_t)item * blk_cap + bi;
    const uint32_t flags = Bp->flags;
    if ((flags & 3) != ZB_CMP || ((flags >> 2) & 3) < 2) continue;
    const ZgItem it = items[item];
    const uint8_t *in = (const uint8_t *)it.src;
    const uint32_t huf_off = Bp->huf_off;
    uint8_t *tab = lit_scratch + (uint64_t)item * lit_stride + Bp->lit_buf - HUF_TAB;
    __syncthreads();  // the previous record's LDS use is over
    const In I{in, it.len};
    uint32_t tl = 0;
    const uint32_t ok = read_huffman<ZHufSmem, false>(I, huf_off, it.len - huf_off, S, tl, in, it.len);
    __syncthreads();
    if (ok) {
      const uint32_t n16 = ((2u << tl) + 15) / 16;  // tables of 2^tl u16 entries (tl >= 1)
      for (uint32_t v = lane; v < n16; v += 64) ((uint4 *)tab)[v] = ((const uint4 *)S.huf)[v];
    }
    if (lane == 0) *(uint32_t *)(tab + (HUF_TAB - 16)) = ok ? tl : 0u;
  }
}
#endif
// Blocks whose output is their literals alone (raw, rle, or compressed without sequences) depend on
// nothing before them: k_zstd_direct writes them into the slot with the whole GPU ahead of the
// per-item execution, which only flushes up to them and steps over (at least XDIRECT bytes: a
// shorter block costs the executor less than the restart of its ring).
constexpr uint32_t XDIRECT = 4096;
__device__ __forceinline__ bool x_direct_block(uint32_t flags, uint32_t nseq, uint32_t out_size) {
  const uint32_t type = flags & 3;
  return out_size >= XDIRECT && (type == ZB_RAW || type == ZB_RLE || (type == ZB_CMP && nseq == 0));
}

// A compressed block without sequences is its literals: when k_zstd_plan has run before the literal
// decoder (one stream, no aliases: launch_zstd_pass), k_zstd_lits writes them straight into the slot
// at the block's output offset and k_zstd_direct leaves the block alone - the literal scratch round
// trip (written by the literal decoder, read and written again by the direct copy) was 17.7 GB of
// C5's 149 GB per step. The predicate both kernels apply:
__device__ __forceinline__ bool lits_in_slot(uint32_t flags, uint32_t nseq, uint32_t regen, uint32_t out_size,
                                             uint32_t out_off, uint64_t slot_bytes) {
  return (flags & 3) == ZB_CMP && ((flags >> 2) & 3) != 0 && nseq == 0 && regen == out_size && out_size >= XDIRECT &&
         (uint64_t)out_off + out_size <= slot_bytes;
}


#if ZG_LIT_ILP == 2
#define ZG_LITS_DECODE(...) lits_decode2(__VA_ARGS__)
#else
#define ZG_LITS_DECODE(...) lits_decode(__VA_ARGS__, slot)
#endif
__global__ __launch_bounds__(LIT_THREADS) __attribute__((amdgpu_waves_per_eu(ZG_LIT_WPE, 8))) void k_zstd_lits(const ZgItem *items, uint32_t *status, const ZBlk *blks,
                                                           uint32_t blk_cap, const uint32_t *nblk,
                                                           const uint32_t *zmode, uint32_t n_items,
                                                           uint8_t *lit_scratch, uint64_t lit_stride,
                                                           uint8_t *lit_rec, const unsigned long long *max_nblk,
                                                           uint8_t *dst = nullptr, uint64_t slot_bytes = 0) {
  __shared__ ZLitSmem S;
  const uint32_t t = threadIdx.x;
  // this lane's record slot (ZG_LIT_REC; nullptr: every lane decodes twice)
  uint8_t *const slot = lit_rec ? lit_rec + ((uint64_t)blockIdx.x * LIT_THREADS + t) * REC_SLOT : nullptr;
  (void)slot;
  const uint64_t total = (uint64_t)n_items * rec_blocks(blk_cap, max_nblk);
  for (uint64_t g = blockIdx.x; g < total; g += gridDim.x) {
    const uint32_t item = (uint32_t)(g % n_items), bi = (uint32_t)(g / n_items);  // block-major order
    if (bi >= nblk[item] || zmode[item] != ZMODE_PARALLEL) continue;
    const ZBlk *Bp = blks + (uint64_t)item * blk_cap + bi;
    const uint32_t flags = Bp->flags;
    const uint32_t ltype = (flags >> 2) & 3;
    if ((flags & 3) != ZB_CMP || ltype == 0) continue;
    const ZgItem it = items[item];
    const uint8_t *in = (const uint8_t *)it.src;
    const uint32_t regen = Bp->regen;
    uint8_t *const lit_s = lit_scratch + (uint64_t)item * lit_stride + Bp->lit_buf;
    uint8_t *lit = lit_s;
    if (dst && status[item] == 0 && lits_in_slot(flags, Bp->nseq, regen, Bp->out_size, Bp->out_off, slot_bytes))
      lit = dst + (uint64_t)item * slot_bytes + Bp->out_off;
    __syncthreads();  // the previous record's LDS use is over
    if (ltype == 1) {  // RLE literals
      const uint8_t v = in[Bp->lit_off];
      for (uint32_t k = t; k < regen; k += LIT_THREADS) lit[k] = v;
      continue;
    }
    const uint32_t lo0 = Bp->lit_off, lend = Bp->lit_end;
#if ZG_HUF_SPLIT
    // the table k_zstd_huf built: 16-B loads, one per thread
    const uint8_t *tab = lit_s - HUF_TAB;
    const uint32_t tl = *(const uint32_t *)(tab + (HUF_TAB - 16));
    if (tl) {
      const uint32_t n16 = ((2u << tl) + 15) / 16;  // tables of 2^tl u16 entries (tl >= 1)
      for (uint32_t v = t; v < n16; v += LIT_THREADS) ((uint4 *)S.huf)[v] = ((const uint4 *)tab)[v];
    }
    __syncthreads();
#else
    const uint32_t huf_off = Bp->huf_off;
    if (t < 64) {  // wave 0 builds the table
      const In I{in, it.len};
      uint32_t tl = 0;
      const uint32_t ok = read_huffman<ZLitSmem, true>(I, huf_off, it.len - huf_off, S, tl, in, it.len);
      if (t == 0) {
        S.ctl[0] = ok ? tl : 0u;
      }
    }
    __syncthreads();
    const uint32_t tl = S.ctl[0];
#endif
    bool bad = tl == 0;
    const uint32_t nstreams = (flags >> 4) & 1 ? 4 : 1;
    uint64_t s_lo[4] = {lo0, 0, 0, 0}, s_hi[4] = {lend, 0, 0, 0};
    uint32_t s_n[4] = {regen, 0, 0, 0};
    const uint32_t seg = (regen + 3) / 4;
    if (!bad && nstreams == 4) {
      const uint64_t q = lo0;
      if (q + 6 > lend) bad = true;
      const uint32_t l1 = in[q] | (in[q + 1] << 8), l2 = in[q + 2] | (in[q + 3] << 8), l3 = in[q + 4] | (in[q + 5] << 8);
      const uint64_t b = q + 6;
      if (b + l1 + l2 + l3 > lend) bad = true;
      s_lo[0] = b; s_hi[0] = b + l1;
      s_lo[1] = s_hi[0]; s_hi[1] = s_lo[1] + l2;
      s_lo[2] = s_hi[1]; s_hi[2] = s_lo[2] + l3;
      s_lo[3] = s_hi[2]; s_hi[3] = lend;
      if (3 * seg > regen) bad = true;
      s_n[0] = s_n[1] = s_n[2] = seg;
      s_n[3] = regen - 3 * seg;
    }
    // bit positions relative to the staged (or global) word base
    const uintptr_t mis = (uintptr_t)in & 3;
    const uint32_t *words = (const uint32_t *)((uintptr_t)in - mis);
    const int64_t nwords_item = (int64_t)((it.len + mis + 3) / 4);
    const int64_t wbase = (int64_t)((s_lo[0] + mis) >> 2);          // first word of the section
    const int64_t wend = (int64_t)(((nstreams == 4 ? s_hi[3] : s_hi[0]) + mis + 3) >> 2);  // one past its last word
    int32_t top[4] = {0, 0, 0, 0}, lob[4] = {0, 0, 0, 0};
#pragma unroll
    for (uint32_t k = 0; k < 4; k++) {
      if (k < nstreams && !bad) {
        const uint32_t lastb = s_hi[k] > s_lo[k] ? in[s_hi[k] - 1] : 0u;
        if (lastb == 0) bad = true;
        top[k] = (int32_t)((int64_t)(s_hi[k] - 1 + mis) * 8 + (lastb ? highbit(lastb) : 0u) - wbase * 32);
        lob[k] = (int32_t)((int64_t)(s_lo[k] + mis) * 8 - wbase * 32);
      }
    }
    bool ok = false;
    if (!bad) {
      const int64_t nw = wend - wbase;
      if (nw * 4 <= (int64_t)LIT_LDS) {
        // 16-B loads, LIT_STAGE_R per thread in flight before the first LDS write
        const int64_t a16 = wbase & ~(int64_t)3, n16 = (wend - a16 + 3) >> 2;
        const uint32_t sh = (uint32_t)(wbase - a16);  // words of the first vector before the section
        for (int64_t v0 = 0; v0 < n16; v0 += LIT_STAGE_R * LIT_THREADS) {
          zv4u r[LIT_STAGE_R];
#pragma unroll
          for (int q = 0; q < LIT_STAGE_R; q++) {
            const int64_t v = v0 + q * LIT_THREADS + t;
            if (v < n16) {
              const gu32 *src = (const gu32 *)(words + a16 + 4 * v);
              if (a16 + 4 * v + 4 <= nwords_item) {
                r[q] = *(const __attribute__((address_space(1))) zv4u *)src;
              } else {  // the item's last words: never read past its end
                const int64_t lim = nwords_item - (a16 + 4 * v);
                r[q] = zv4u{src[0], lim > 1 ? src[1] : 0u, lim > 2 ? src[2] : 0u, 0u};
              }
            }
          }
#pragma unroll
          for (int q = 0; q < LIT_STAGE_R; q++) {
            const int64_t v = v0 + q * LIT_THREADS + t;
            if (v < n16) {
              const uint32_t w4[4] = {r[q].x, r[q].y, r[q].z, r[q].w};
#pragma unroll
              for (int e = 0; e < 4; e++) {
                const int64_t k = 4 * v + e - sh;
                if (k >= 0 && k < nw) S.lin[k] = w4[e];
              }
            }
          }
        }
        __syncthreads();
        const int32_t n32 = (int32_t)nw;
        auto word = [n32](int32_t k) -> uint32_t {
          const bool in = (uint32_t)k < (uint32_t)n32;
          const uint32_t v = S.lin[in ? k : 0];
          return in ? v : 0u;
        };
        ok = ZG_LITS_DECODE(S, word, nstreams, top, lob, s_n, tl, lit, seg);
      } else {
        const gu32 *Wp = (const gu32 *)(words + wbase);
        const int64_t lim = nwords_item - wbase;
#if ZG_LIT_GWIN == 4
        const GBlk word{Wp, lim, 1, {}, {}, {}, {}, 0};
#elif ZG_LIT_GWIN == 3
        GWordPF64 word{Wp, lim, 1, {}, {}};
#elif ZG_LIT_GWIN == 2
        const GWordPF word{Wp, lim, 1, zv4u{0, 0, 0, 0}, zv4u{0, 0, 0, 0}, zv4u{0, 0, 0, 0}, zv4u{0, 0, 0, 0}, 1, false};
#elif ZG_LIT_GWIN
        const GWord word{Wp, lim, 1, zv4u{0, 0, 0, 0}};
#else
        auto word = [Wp, lim](int32_t k) -> uint32_t { return (k >= 0 && k < lim) ? Wp[k] : 0u; };
#endif
        ok = ZG_LITS_DECODE(S, word, nstreams, top, lob, s_n, tl, lit, seg);
      }
    }
    if (!ok && t == 0) status[item] = ZG_CORRUPT_STREAM;
  }
}

// One wave per item: output offsets, incoming rep offsets, frame size checks.
// Executor segments: an item's blocks are cut where no later match reaches back before the cut (and
// not inside a checksummed frame); each segment gets its own k_zstd_exec_item wave. Byte-shuffled
// images cut at their byte planes (tools/lab/zstd_taint.cpp: no match crosses the plane boundary).
#ifndef ZG_XSEG
#define ZG_XSEG 12
#endif
// executor segments per item of the wave executor (at most; ZGPU_ZSTD_XSEG overrides it for both
// executors, ZGPU_ZSTD_XSEG_WIDE for this one). Round 5 measured 2, 3, 4 and 8 within 1 % with 3 best
// (profiles/r05/r05xs_zstd_exec_segment_major_xcd_ab.txt); with round 6's faster sequence decoder
// and the plan group the L0 executors end the C5 step, and more segments shorten them: C5 73.2 (3),
// 72.5 (8), 70.8 (12), 71.3 (16), 103 (32) ms (profiles/r06/r06zfg_*); blosc-zstd's 2-block frames
// cut into 2 at most either way
constexpr uint32_t XSEG = ZG_XSEG;

__global__ __launch_bounds__(64) void k_zstd_plan(const ZgItem *items, uint32_t *status, ZBlk *blks,
                                                  uint32_t blk_cap, const uint32_t *nblk, const uint32_t *zmode,
                                                  uint64_t slot_bytes, uint32_t xseg, uint64_t *alias,
                                                  const uint8_t *lit_scratch, uint64_t lit_stride) {
  const uint32_t item = blockIdx.x;
  const int lane = lane_id();
  if (alias && lane == 0)
    for (uint32_t r = 0; r < ZALIAS; r++) alias[3 * (ZALIAS * item + r) + 2] = 0;  // none
  if (zmode[item] != ZMODE_PARALLEL || status[item]) return;
  ZBlk *B = blks + (uint64_t)item * blk_cap;
  const uint32_t nb = nblk[item];
  if (lane == 0 && nb) B[0].in_src = items[item].src;
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
  if (!err) {
    // valid cuts (backward: the least source position of the matches from the block on), then up to
    // xseg - 1 of them chosen forward at equal shares of the estimated execution cost
    uint64_t smin = ~0ull, total_w = 0, vmask = 0;  // vmask: lane l holds the cuts at blocks 64 l ..
    bool ck = false;
    const bool cuts = nb <= 64 * 64;
    uint32_t al[ZALIAS] = {~0u, ~0u};  // aliased blocks (ZstdScratch::alias): the earliest candidates
    for (uint32_t bi = nb; cuts && bi-- > 0;) {
      const uint32_t flags = U(B[bi].flags), type = flags & 3, nsq = U(B[bi].nseq), osz = U(B[bi].out_size);
      if (flags & ZBF_LAST) ck = flags & ZBF_CK;
      const uint64_t off = U(B[bi].out_off);
      if (type == ZB_CMP && nsq) {
        int64_t reach = (int32_t)U((uint32_t)B[bi].reach_c);
        for (int k = 0; k < 3; k++) {
          const uint32_t m = U(B[bi].reach_m[k]);
          if (m != ~0u) reach = max<int64_t>(reach, (int64_t)U(B[bi].rep_in[k]) - (int64_t)m);
        }
        const int64_t ms = (int64_t)off - reach;
        smin = min<uint64_t>(smin, ms < 0 ? 0ull : (uint64_t)ms);
      }
      // a block no later match reads (it has no matches itself) and no checksum covers
      if (alias && !ck && x_direct_block(flags, nsq, osz) && smin >= off + osz &&
          (type != ZB_CMP || U(B[bi].regen) == osz)) {
        al[1] = al[0];
        al[0] = bi;
      }
      const bool valid = bi > 0 && smin >= off && (!ck || (flags & ZBF_FIRST));
      total_w += (type == ZB_CMP ? 8ull * nsq : 0ull) + (x_direct_block(flags, nsq, osz) ? 0u : osz / 16);
      if (valid && lane == (int)(bi >> 6)) vmask |= 1ull << (bi & 63);
    }
    uint64_t acc = 0;
    uint32_t k = 1;
    for (uint32_t bi = 0; bi < nb; bi++) {
      uint32_t seg = bi == 0;
      if (cuts) {
        const uint32_t flags = U(B[bi].flags), type = flags & 3, nsq = U(B[bi].nseq), osz = U(B[bi].out_size);
        const uint64_t vm = (uint64_t)U(__builtin_amdgcn_readlane((uint32_t)vmask, (int)(bi >> 6))) |
                            ((uint64_t)U(__builtin_amdgcn_readlane((uint32_t)(vmask >> 32), (int)(bi >> 6))) << 32);
        if (((vm >> (bi & 63)) & 1) && k < xseg && acc * xseg >= total_w * k) {
          seg = 1;
          k++;
        }
        acc += (type == ZB_CMP ? 8ull * nsq : 0ull) + (x_direct_block(flags, nsq, osz) ? 0u : osz / 16);
      }
      if (lane == 0) B[bi].seg = seg;
    }
    if (alias && lane == 0) {
      const uint8_t *in = (const uint8_t *)items[item].src;
      for (uint32_t r = 0; r < ZALIAS && al[r] != ~0u; r++) {
        const ZBlk &L = B[al[r]];
        const uint32_t fl = L.flags, ty = fl & 3;
        const uint64_t src = ty == ZB_RLE ? ZALIAS_RLE | in[L.in_off]
                             : ty == ZB_RAW ? (uint64_t)(in + L.in_off)
                             : ((fl >> 2) & 3) == 0 ? (uint64_t)(in + L.lit_off)
                                                    : (uint64_t)(lit_scratch + (uint64_t)item * lit_stride + L.lit_buf);
        alias[3 * (ZALIAS * item + r)] = src;
        alias[3 * (ZALIAS * item + r) + 1] = L.out_off;
        alias[3 * (ZALIAS * item + r) + 2] = L.out_size;
      }
    }
  }
  if (lane == 0 && err) status[item] = err;
}



__global__ __launch_bounds__(256) void k_zstd_direct(const ZgItem *items, const uint32_t *status, const ZBlk *blks,
                                                    uint32_t blk_cap, const uint32_t *nblk, const uint32_t *zmode,
                                                    uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                                                    const uint8_t *lit_scratch, uint64_t lit_stride,
                                                    const uint64_t *alias, const unsigned long long *max_nblk,
                                                    int lits_direct) {
  const uint64_t recs = (uint64_t)n_items * rec_blocks(blk_cap, max_nblk);
  const uint32_t tid = threadIdx.x;
  for (uint64_t rec = blockIdx.x; rec < recs; rec += gridDim.x) {
    const uint32_t item = (uint32_t)(rec % n_items), bi = (uint32_t)(rec / n_items);  // block-major order
    if (zmode[item] != ZMODE_PARALLEL || status[item] || bi >= nblk[item]) continue;
    const ZBlk &b = blks[(uint64_t)item * blk_cap + bi];
    const uint32_t flags = b.flags, type = flags & 3, n = b.out_size;
    if (!x_direct_block(flags, b.nseq, n)) continue;
    if (type == ZB_CMP && b.regen != n) continue;  // corrupt: k_zstd_exec_item reports it
    if (lits_direct && lits_in_slot(flags, b.nseq, b.regen, n, b.out_off, slot_bytes)) continue;  // k_zstd_lits wrote it
    if (alias) {  // the consumer reads an aliased block where it is
      const uint64_t *a = alias + 3 * ZALIAS * (uint64_t)item;
      bool al = false;
      for (uint32_t r = 0; r < ZALIAS; r++) al |= a[3 * r + 2] && a[3 * r + 1] == b.out_off;
      if (al) continue;
    }
    const uint8_t *in = (const uint8_t *)items[item].src;
    uint8_t *o = dst + (uint64_t)item * slot_bytes + b.out_off;
    if (type == ZB_RLE) {
      const uint8_t v = in[b.in_off];
      const uint32_t w = v * 0x01010101u;
      const uint32_t head = min<uint32_t>(n, (16 - ((uintptr_t)o & 15)) & 15);
      if (tid < head) o[tid] = v;
      const uint32_t nv = (n - head) / 16;
      for (uint32_t k = tid; k < nv; k += 256) *(zv4u *)(o + head + 16 * k) = zv4u{w, w, w, w};
      for (uint32_t k = head + 16 * nv + tid; k < n; k += 256) o[k] = v;
      continue;
    }
    const uint8_t *src = type == ZB_RAW ? in + b.in_off
                         : ((flags >> 2) & 3) == 0 ? in + b.lit_off
                                                   : lit_scratch + (uint64_t)item * lit_stride + b.lit_buf;
    // destination-aligned 16-B vectors, each from two aligned source vectors and byte-aligns
    const uint32_t head = min<uint32_t>(n, (16 - ((uintptr_t)o & 15)) & 15);
    if (tid < head) o[tid] = src[tid];
    const uint32_t nv = (n - head) / 16;
    const uintptr_t s0 = (uintptr_t)(src + head);
    const uint32_t m = (uint32_t)(s0 & 15);
    const zv4u *sv = (const zv4u *)(s0 & ~(uintptr_t)15);
    for (uint32_t k = tid; k < nv; k += 256) {
      const zv4u lo = __builtin_nontemporal_load(sv + k);
      zv4u r = lo;
      if (m) {
        const zv4u hi = __builtin_nontemporal_load(sv + k + 1);
        const uint32_t sh = m & 3;  // bytes
        const uint32_t q = m >> 2;
        const uint32_t w0 = lo[0], w1 = lo[1], w2 = lo[2], w3 = lo[3], w4 = hi[0], w5 = hi[1], w6 = hi[2];
        const uint32_t c0 = q == 0 ? w0 : q == 1 ? w1 : q == 2 ? w2 : w3;
        const uint32_t c1 = q == 0 ? w1 : q == 1 ? w2 : q == 2 ? w3 : w4;
        const uint32_t c2 = q == 0 ? w2 : q == 1 ? w3 : q == 2 ? w4 : w5;
        const uint32_t c3 = q == 0 ? w3 : q == 1 ? w4 : q == 2 ? w5 : w6;
        const uint32_t c4 = q == 0 ? w4 : q == 1 ? w5 : q == 2 ? w6 : hi[3];
        r = zv4u{__builtin_amdgcn_alignbyte(c1, c0, sh), __builtin_amdgcn_alignbyte(c2, c1, sh),
                 __builtin_amdgcn_alignbyte(c3, c2, sh), __builtin_amdgcn_alignbyte(c4, c3, sh)};
      }
      __builtin_nontemporal_store(r, (zv4u *)(o + head) + k);
    }
    for (uint32_t k = head + 16 * nv + tid; k < n; k += 256) o[k] = src[k];
  }
}

// -------------------------------------------------------------------------------------------------
// k_zstd_exec_item (kernels/zstd_exec.inc) in two configurations, chosen per launch by launch_zstd:
//   xwide  - 8 KiB ring, 4 KiB batches, 256 staged far vectors, 2 waves/SIMD (18.2 KiB LDS, 256
//            VGPRs): fastest per wave; a grid of few waves per CU (C5-like batches of 16 MiB frames)
//   xdense - 4 KiB ring, 2 KiB batches, 128 staged vectors, 4 waves/SIMD (9.9 KiB LDS, 128 VGPRs):
//            twice the resident waves, for grids of many small frames (blosc's 256 KiB blocks)
// -------------------------------------------------------------------------------------------------
#ifndef ZG_XBATCH
#define ZG_XBATCH 4096
#endif
constexpr uint32_t XBATCH = ZG_XBATCH;  // max output span of one executor batch (ZBATCH: the serial decoder's)
#ifndef ZG_XRING
#define ZG_XRING 8192
#endif
constexpr uint32_t XRING = ZG_XRING, XRMASK = XRING - 1;
static_assert((XRING & XRMASK) == 0 && XRING >= 2 * XBATCH, "exec ring: a power of two holding two batches");
#ifndef ZG_XSTAGE_V
#define ZG_XSTAGE_V 256
#endif
constexpr uint32_t XSTAGE_V = ZG_XSTAGE_V;  // staged far-source vectors (16 B) per batch
#ifndef ZG_XWPE
#define ZG_XWPE 2  // the executor is compiled for >= 2 waves/SIMD (VGPR + AGPR <= 256)
#endif
#ifndef ZG_XPL
#define ZG_XPL 64
#endif
constexpr uint32_t XPL = ZG_XPL;  // bytes of a short match its own lane copies (the rest: the wave)
static_assert(XPL % 16 == 0 && XPL >= 16 && XPL <= 512, "XPL: 16-B pieces, at most a short match");
#ifndef ZG_XLI
#define ZG_XLI 1
#endif
constexpr uint32_t XLI = ZG_XLI;  // long matches the wave copies per step (their loads together)
namespace xwide {
#define ZX_BATCH ZG_XBATCH
#define ZX_RING ZG_XRING
#define ZX_STAGE_V ZG_XSTAGE_V
#define ZX_WPE ZG_XWPE
#include "zstd_exec.inc"
#undef ZX_BATCH
#undef ZX_RING
#undef ZX_STAGE_V
#undef ZX_WPE
}  // namespace xwide
#ifndef ZG_XD_BATCH
#define ZG_XD_BATCH 2048
#endif
#ifndef ZG_XD_RING
#define ZG_XD_RING 4096
#endif
#ifndef ZG_XD_STAGE_V
#define ZG_XD_STAGE_V 128
#endif
#ifndef ZG_XD_WPE
#define ZG_XD_WPE 4
#endif
namespace xdense {
#define ZX_BATCH ZG_XD_BATCH
#define ZX_RING ZG_XD_RING
#define ZX_STAGE_V ZG_XD_STAGE_V
#define ZX_WPE ZG_XD_WPE
#include "zstd_exec.inc"
#undef ZX_BATCH
#undef ZX_RING
#undef ZX_STAGE_V
#undef ZX_WPE
}  // namespace xdense
// k_zstd_exec_win (kernels/zstd_xwin.inc): one 512-thread workgroup per segment, 32 KiB windows
// resolved in parallel by pointer jumping in LDS; the default executor (ZGPU_ZSTD_XWIN=0: the wave
// executors above)
#include "zstd_xwin.inc"
#ifndef ZG_XSEG_WIN
#define ZG_XSEG_WIN 8
#endif
constexpr uint32_t XSEG_WIN = ZG_XSEG_WIN;  // executor segments per item (at most) for k_zstd_exec_win
#ifndef ZG_XWIN_MAX_WPC
#define ZG_XWIN_MAX_WPC 4
#endif
// executor grids of at least this many waves (items x segments) per CU take xdense
#ifndef ZG_XDENSE_WPC
#define ZG_XDENSE_WPC 64
#endif
constexpr uint32_t XDENSE_WAVES_PER_CU = ZG_XDENSE_WPC;
// launch_zstd splits a batch into two pipelined halves (ZstdScratch::s2) from 2 x this many items
constexpr uint32_t ZSPLIT_MIN = 1024;

uint64_t zstd_lit_rec_bytes(uint32_t &wgs) {
  static const uint64_t cap = [] {
    const char *e = std::getenv("ZGPU_ZSTD_LGRID");
    return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : (uint64_t)device_cu_count() * ZG_LIT_GRID_PER_CU;
  }();
  static const bool on = [] {
    const char *e = std::getenv("ZGPU_ZSTD_LIT_REC");
    return ZG_LIT_REC && (!e || std::atoi(e) != 0);
  }();
  wgs = on ? (uint32_t)cap : 0u;
  return on ? cap * LIT_THREADS * REC_SLOT : 0ull;
}
uint64_t zstd_norm_bytes() { return ZNORM * sizeof(int16_t); }
void zstd_scratch_layout(uint64_t slot_bytes, uint32_t &blk_cap, uint64_t &blk_bytes, uint64_t &lit_stride,
                         uint64_t &seq_cap) {
  blk_cap = (uint32_t)std::min<uint64_t>(slot_bytes / 32768 + 64, 1u << 20);
  blk_bytes = sizeof(ZBlk);
  // literals (<= the decoded size) + one Huffman table per block (HUF_TAB per >= 64 KiB of output on
  // typical frames; frames of many tiny Huffman blocks overflow it and take the serial decoder)
  lit_stride = std::max<uint64_t>(slot_bytes + slot_bytes / 8, BLOCK_MAX + 64 + 2 * HUF_TAB);
  lit_stride = (lit_stride + 255) & ~(uint64_t)255;
  seq_cap = slot_bytes / 4 + 1024;  // sequences per item (each decodes >= 3 bytes; typical >= 8)
}
// One pass of the block-parallel pipeline over n_items items on stream s; ev_entropy (nullable) is
// recorded on s once the entropy kernels (and the side stream's sequence decode) are done.
static hipError_t launch_zstd_pass(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst,
                                   uint64_t slot_bytes, const ZstdScratch &Z, hipStream_t s, hipEvent_t ev_entropy) {
  if (!n_items) return hipSuccess;
  ZBlk *blks = (ZBlk *)Z.blks;
  const bool listed = Z.ser_list && Z.ser_count;
  hipLaunchKernelGGL(k_zstd_scan, dim3(n_items), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                     Z.lit_stride, Z.seq_cap, Z.force_serial, Z.counters, listed ? Z.ser_list : nullptr,
                     listed ? Z.ser_count : nullptr, Z.max_nblk, Z.norm);
  const uint64_t recs = (uint64_t)n_items * Z.blk_cap;
  // grids of the record-strided entropy kernels (overridable for tuning: ZGPU_ZSTD_GRID, ZGPU_ZSTD_LGRID)
  static const uint64_t g_cap = [] {
    const char *e = std::getenv("ZGPU_ZSTD_GRID");
    return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : (uint64_t)device_cu_count() * 16;
  }();
  static const uint64_t l_cap = [] {
    const char *e = std::getenv("ZGPU_ZSTD_LGRID");
    // one resident wave of workgroups: the device's CUs x ZG_LIT_GRID_PER_CU workgroups of 256 lanes each
    return e ? std::max<uint64_t>(1, std::strtoull(e, nullptr, 10)) : (uint64_t)device_cu_count() * ZG_LIT_GRID_PER_CU;
  }();
  const uint32_t grid = (uint32_t)std::min<uint64_t>(recs, g_cap);
  const uint32_t lgrid = (uint32_t)std::min<uint64_t>(recs, l_cap);
  // the sequence decoder reads only the scan's block records and writes its own fields of them (and
  // the sequence scratch): with a side stream it runs beside the literal kernels
  const bool fork = Z.side && Z.ev_fork && Z.ev_join;
  hipStream_t sq = fork ? Z.side : s;
  // literal-only blocks decoded straight into the slot (lits_in_slot): needs k_zstd_plan's output
  // offsets before the literal decoder, i.e. the sequence decoder on the same stream, and no aliases
  static const bool lit_direct_env = [] {
    const char *e = std::getenv("ZGPU_ZSTD_LITDIRECT");
    return !e || std::atoi(e) != 0;
  }();
  const bool lits_first = Z.lits_first && !fork;
  const bool lit_direct = lit_direct_env && !fork && !Z.alias && !lits_first;
  // executor segments per item: ZG_XSEG (ZGPU_ZSTD_XSEG: tuning)
  static const uint32_t xseg_env = [] {
    const char *e = std::getenv("ZGPU_ZSTD_XSEG");
    return e ? (uint32_t)std::min<unsigned long>(64, std::max<unsigned long>(1, std::strtoul(e, nullptr, 10))) : 0u;
  }();
  // executor: the windowed workgroup executor for batches the wave executor would leave mostly idle
  // (fewer than ZG_XWIN_MAX_WPC of its waves per CU: lone frames, per-chunk calls, C5's L1 and small
  // levels); the wave executor for batches that fill the GPU with waves (C5's L0 halves, blosc-zstd),
  // where the window executor's whole-CU workgroups measured slower beside the other lanes' entropy
  // kernels (C5 100 vs 91-94 ms with it everywhere, profiles/r06/r06h_*). ZGPU_ZSTD_XWIN=0/1 forces
  // one (read per call: tests run both).
  const char *xw_s = std::getenv("ZGPU_ZSTD_XWIN");
  const int xw_env = xw_s ? std::atoi(xw_s) : -1;
  const char *xwpc_s = std::getenv("ZGPU_ZSTD_XWIN_WPC");  // the threshold's waves per CU (A/B)
  const uint64_t xwpc = xwpc_s ? (uint64_t)std::atoi(xwpc_s) : ZG_XWIN_MAX_WPC;
  // (the threshold counts 3 waves per item, round 5's segment count: C5's L1 and small levels take the
  // window executor, its L0 halves the wave executor)
  const bool xwin_on = xw_env >= 0 ? xw_env != 0 : (uint64_t)n_items * 3 < (uint64_t)device_cu_count() * xwpc;
  static const uint32_t xseg_wide_env = [] {  // A/B: the wave executor's segments only
    const char *e = std::getenv("ZGPU_ZSTD_XSEG_WIDE");
    return e ? (uint32_t)std::min<unsigned long>(64, std::max<unsigned long>(1, std::strtoul(e, nullptr, 10))) : 0u;
  }();
  static const uint32_t xseg_win_env = [] {  // A/B: the window executor's segments only
    const char *e = std::getenv("ZGPU_ZSTD_XSEG_WIN");
    return e ? (uint32_t)std::min<unsigned long>(64, std::max<unsigned long>(1, std::strtoul(e, nullptr, 10))) : 0u;
  }();
  const uint32_t xseg = xseg_env               ? xseg_env
                        : xwin_on              ? (xseg_win_env ? xseg_win_env : XSEG_WIN)
                                               : (xseg_wide_env ? xseg_wide_env : XSEG);

  if (fork) {
    hipError_t e = hipEventRecord(Z.ev_fork, s);
    if (e == hipSuccess) e = hipStreamWaitEvent(Z.side, Z.ev_fork, 0);
    if (e != hipSuccess) return e;
  }
  // one resident wave of the sequence decoder: CUs x 4 SIMDs x ZG_BLK_WPE waves (ZGPU_ZSTD_BLK_WPE: fewer,
  // leaving CU slots to concurrent plans' kernels; A/B)
  static const uint64_t blk_wpe = [] {
    const char *e = std::getenv("ZGPU_ZSTD_BLK_WPE");
    const int v = e ? std::atoi(e) : 0;
    return (uint64_t)(v > 0 && v <= ZG_BLK_WPE ? v : 0);
  }();
  const uint32_t bgrid = (uint32_t)std::min<uint64_t>(
      recs, blk_wpe ? (uint64_t)device_cu_count() * 4 * blk_wpe
                    : std::max<uint64_t>(g_cap, (uint64_t)device_cu_count() * 4 * ZG_BLK_WPE));
  // sequence decoder: 0 one wave per block (k_zstd_blocks, the split chain decoder: lab 64 L0 chunks
  // 1.63 ms against the lane groups' 5.0, C5 82.0 -> 74.7 ms, profiles/r06/r06pqr_*), 1 lane groups
  // (k_zstd_blocks_lg, the round-5 default); ZGPU_ZSTD_SEQ forces one
  const char *xp_s = std::getenv("ZGPU_ZSTD_XPAR");
  const bool par = xwin_on && Z.ext && Z.ext_cnt && n_items <= Z.ext_items && (!xp_s || std::atoi(xp_s) != 0);
  static const int seq_env = [] {
    const char *e = std::getenv("ZGPU_ZSTD_SEQ");
    return e ? std::atoi(e) : -1;
  }();
  const int seq_mode = seq_env >= 0 ? seq_env : 0;
  auto launch_seq = [&] {
    if (seq_mode == 1) {
      // one resident wave of the lane-group decoder: its LDS (5 KiB per block) sets the waves per CU
      const uint64_t per_cu = std::max<uint64_t>(1, (160u << 10) / ((sizeof(ZDecLgSmem<ZG_SEQ_G>) + 1023) & ~size_t(1023)));
      const uint64_t lrecs = (recs + ZG_SEQ_G - 1) / ZG_SEQ_G;
      const uint32_t lg_grid = (uint32_t)std::min<uint64_t>(lrecs, (uint64_t)device_cu_count() * per_cu);
      hipLaunchKernelGGL(k_zstd_blocks_lg<ZG_SEQ_G>, dim3(lg_grid), dim3(64), 0, sq, items, status, blks, Z.blk_cap,
                         Z.nblk, Z.mode, n_items, Z.seq, Z.seq_cap, Z.max_nblk);
    } else {
      hipLaunchKernelGGL(k_zstd_blocks, dim3(bgrid), dim3(64), 0, sq, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                         n_items, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap, Z.max_nblk, Z.norm);
    }
  };
  if (!lits_first) launch_seq();
  if (fork) {
    hipError_t e = hipEventRecord(Z.ev_join, Z.side);
    if (e != hipSuccess) return e;
  }
  if (lit_direct)  // output offsets first: the literal decoder writes literal-only blocks into the slot
    hipLaunchKernelGGL(k_zstd_plan, dim3(n_items), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                       slot_bytes, xseg, Z.alias, Z.lit, Z.lit_stride);
#if ZG_HUF_SPLIT
  hipLaunchKernelGGL(k_zstd_huf, dim3(grid), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode, n_items,
                     Z.lit, Z.lit_stride, Z.max_nblk);
#endif
  // record slots: one per lane of the persistent grid (allocated for l_cap workgroups)
  uint8_t *lit_rec = (ZG_LIT_REC && Z.lit_rec && lgrid <= Z.lit_rec_wgs) ? Z.lit_rec : nullptr;
  hipLaunchKernelGGL(k_zstd_lits, dim3(lgrid), dim3(LIT_THREADS), 0, s, items, status, blks, Z.blk_cap, Z.nblk,
                     Z.mode, n_items, Z.lit, Z.lit_stride, lit_rec, Z.max_nblk, lit_direct ? dst : nullptr, slot_bytes);
  if (lits_first) launch_seq();  // same stream: after the literal decoder
  if (fork) {
    hipError_t e = hipStreamWaitEvent(s, Z.ev_join, 0);
    if (e != hipSuccess) return e;
  }
  if (ev_entropy) {
    hipError_t e = hipEventRecord(ev_entropy, s);
    if (e != hipSuccess) return e;
  }
  if (!lit_direct)
    hipLaunchKernelGGL(k_zstd_plan, dim3(n_items), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                       slot_bytes, xseg, Z.alias, Z.lit, Z.lit_stride);
  hipLaunchKernelGGL(k_zstd_direct, dim3(grid), dim3(256), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                     n_items, dst, slot_bytes, Z.lit, Z.lit_stride, Z.alias, Z.max_nblk, lit_direct ? 1 : 0);
  // executor configuration: xdense when the grid has many waves per CU (ZGPU_ZSTD_XDENSE=0/1 forces one)
  const char *xd_s = std::getenv("ZGPU_ZSTD_XDENSE");  // read per call (tests force both)
  const int xd_env = xd_s ? std::atoi(xd_s) : -1;
  const bool dense = xd_env >= 0 ? xd_env != 0
                                 : (uint64_t)n_items * xseg >= (uint64_t)device_cu_count() * XDENSE_WAVES_PER_CU;
  // latency mode (ZGPU_ZSTD_XPAR=0 off; read per call): batches the plan gave ext arrays
  if (par) {
    const uint64_t tot = (uint64_t)n_items * slot_bytes;
    hipError_t e = hipMemsetAsync(Z.ext, 0xFF, tot * 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(Z.ext_cnt, 0, ZEXT_ROUNDS * 8, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_zstd_exec_win<true>, dim3(device_cu_count()), dim3(xwin::THREADS), 0, s, items, status,
                       blks, Z.blk_cap, Z.nblk, Z.mode, dst, slot_bytes, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap,
                       n_items, Z.ext, Z.max_nblk);
    // rounds: a reference hops back at least one window range (or one table's sub-window, >= 1 KiB on
    // real data) per step, so log2 of the slot's KiB + 2 rounds; a round after the last reference
    // returns at once
    uint32_t rounds = 2;
    while (rounds < ZEXT_ROUNDS && (1ull << (rounds - 2)) < slot_bytes / 1024 + 1) rounds++;
    const uint32_t g2 = (uint32_t)std::min<uint64_t>((tot / 4 + 255) / 256, (uint64_t)device_cu_count() * 16);
    uint32_t *ea = Z.ext, *eb = Z.ext + tot;
    for (uint32_t r = 0; r < rounds; r++) {
      hipLaunchKernelGGL(k_zstd_ext_round, dim3(g2), dim3(256), 0, s, ea, eb, dst, slot_bytes, tot,
                         r ? Z.ext_cnt + r - 1 : (const unsigned long long *)nullptr, Z.ext_cnt + r);
      std::swap(ea, eb);
    }
    hipLaunchKernelGGL(k_zstd_par_finish, dim3(n_items), dim3(64), 0, s, items, status, blks, Z.blk_cap, Z.nblk, Z.mode,
                       dst, slot_bytes);
  } else if (xwin_on)
    hipLaunchKernelGGL(k_zstd_exec_win<false>, dim3(n_items * xseg), dim3(xwin::THREADS), 0, s, items, status, blks,
                       Z.blk_cap, Z.nblk, Z.mode, dst, slot_bytes, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap, xseg,
                       (uint32_t *)nullptr, (const unsigned long long *)nullptr);
  else if (dense)
    hipLaunchKernelGGL(xdense::k_zstd_exec_item, dim3(n_items * xseg), dim3(64), 0, s, items, status, blks, Z.blk_cap,
                       Z.nblk, Z.mode, dst, slot_bytes, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap, xseg);
  else
    hipLaunchKernelGGL(xwide::k_zstd_exec_item, dim3(n_items * xseg), dim3(64), 0, s, items, status, blks, Z.blk_cap,
                       Z.nblk, Z.mode, dst, slot_bytes, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap, xseg);
  if (!listed) {
    hipLaunchKernelGGL(k_zstd, dim3(n_items), dim3(64), 0, s, items, status, dst, slot_bytes, Z.lit, Z.lit_stride,
                       Z.mode, nullptr, nullptr);
  } else if (Z.launch_serial) {
    // the compacted serial items: a persistent grid of at most 4 waves per CU
    const uint32_t sgrid = (uint32_t)std::min<uint64_t>(n_items, (uint64_t)device_cu_count() * 4);
    hipLaunchKernelGGL(k_zstd, dim3(sgrid), dim3(64), 0, s, items, status, dst, slot_bytes, Z.lit, Z.lit_stride,
                       Z.mode, Z.ser_list, Z.ser_count);
  }
  return hipGetLastError();
}

hipError_t launch_zstd(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                       const ZstdScratch &Z, hipStream_t s) {
  // read per call (tests switch these knobs between calls): ZGPU_ZSTD_SPLIT_MIN splits small batches
  const char *sm = std::getenv("ZGPU_ZSTD_SPLIT_MIN");
  const uint32_t split_min = sm ? (uint32_t)std::max<unsigned long>(1, std::strtoul(sm, nullptr, 10)) : ZSPLIT_MIN;
  if (!Z.s2 || !Z.ev_half || !Z.ev_done || n_items < 2 * split_min)
    return launch_zstd_pass(items, status, n_items, dst, slot_bytes, Z, s, nullptr);
  // Two halves (ZstdScratch::s2): the second half's entropy kernels start once the first half's are
  // done, so they run beside the first half's executor; the caller's stream joins the second half.
  const uint32_t h = n_items / 2;
  ZstdScratch A = Z;
  A.s2 = nullptr;
  hipError_t e = launch_zstd_pass(items, status, h, dst, slot_bytes, A, s, Z.ev_half);
  if (e != hipSuccess) return e;
  ZstdScratch B = Z;
  B.s2 = nullptr;
  B.blks = (uint8_t *)Z.blks + (uint64_t)h * Z.blk_cap * sizeof(ZBlk);
  B.nblk = Z.nblk + h;
  B.mode = Z.mode + h;
  B.lit = Z.lit + (uint64_t)h * Z.lit_stride;
  B.seq = Z.seq + (uint64_t)h * Z.seq_cap * 3;
  B.alias = Z.alias ? Z.alias + (uint64_t)h * 3 * ZALIAS : nullptr;
  B.ser_list = nullptr;  // the second half's serial fallback runs unlisted (one wave per item)
  B.ser_count = nullptr;
  if ((e = hipStreamWaitEvent(Z.s2, Z.ev_half, 0)) != hipSuccess) return e;
  e = launch_zstd_pass(items + h, status + h, n_items - h, dst + (uint64_t)h * slot_bytes, slot_bytes, B, Z.s2,
                       nullptr);
  if (e != hipSuccess) return e;
  if ((e = hipEventRecord(Z.ev_done, Z.s2)) != hipSuccess) return e;
  return hipStreamWaitEvent(s, Z.ev_done, 0);
}

}  // namespace zgpu
