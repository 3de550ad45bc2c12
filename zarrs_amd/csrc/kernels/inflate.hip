// gzip member decode (RFC 1952 header/trailer + RFC 1951 DEFLATE) for gfx950.
//
// Reference behaviour restated: zarrs/src/array/codec/bytes_to_bytes/gzip/gzip_codec.rs:110-120 —
// flate2 1.1 `bufread::GzDecoder::read_to_end` (miniz_oxide backend): parse the first member's
// header, inflate its DEFLATE stream, check the trailer CRC-32 and ISIZE (at the end of k_gzip, with
// crc.hpp's parallel CRC); any malformed input -> io::Error -> CodecError::IOError
// (ZG_CORRUPT_STREAM here). Bytes after the first member are ignored, as GzDecoder does.
//
// Design (one 64-lane wavefront = one workgroup = one gzip stream):
//  * Symbol decode is inherently serial, so every lane runs the same decode loop on wave-uniform
//    values (readfirstlane keeps them in SGPRs); there is no divergence and no broadcast step.
//  * Bit reader: the compressed stream is read as aligned 32-bit words through two 256-byte register
//    windows (one word per lane, one coalesced load each); a refill is a v_readlane, and the next
//    window is loaded a full window ahead, so the decode loop never waits on HBM.
//  * Huffman tables live in LDS: a 9-bit root table for literal/length and an 8-bit one for
//    distances, each entry already holding the decoded meaning (literal byte, or length/distance base
//    + extra-bit count); a root prefix of longer codes points to a second-level table indexed by the
//    next bits (zlib's two-level scheme), so every code of real data decodes by table lookups (a code
//    set whose subtables outgrow their LDS space takes a canonical count/first slow path for those
//    prefixes). Tables are built cooperatively by the 64 lanes (ballot ranks, parallel root fill,
//    subtables allocated by an LDS counter).
//  * Symbol decode: every lane decodes, branch-free, the whole symbol (code, extra bits, distance)
//    that would start at its bit offset of a 63-bit lookahead window; the window's symbols are
//    chained by pointer jumping (ds_bpermute doublings, up to 16 symbols per window: C3 data has at
//    most 11 per 64 bits) and compacted into an LDS record array.
//  * Decoded symbols (up to 64 per batch, one per lane) are then executed in parallel:
//    a wave prefix sum places them, literals are written at once, matches resolve in rounds by exact
//    dependencies (a long match copied by all lanes: out[p+i] = out[p-d+(i mod d)], so overlapping
//    copies need no serialisation), through a 1 KiB LDS ring that holds the recent output; sources
//    older than the ring come from the flushed output in HBM. The ring is flushed to the item's slot
//    with 16-byte stores.
//  * LDS per stream is 7.0 KiB (ring 1 KiB, tables 4.6 KiB; the header scratch shares its space with
//    the batch records) and the kernel is held at 96 VGPRs: 5 streams per SIMD.
#include <hip/hip_runtime.h>

#include <cstdlib>
#include <type_traits>

#include "../common.hpp"
#include "crc.hpp"
#include "launch.hpp"

namespace zgpu {

#ifdef ZG_PROFILE
// lab builds only (tools/lab): per-phase shader-clock totals, summed over waves
__device__ unsigned long long g_prof[16];
// per-wave accumulators (prof_acc[], declared by PROF_DECL), flushed once per wave by PROF_FLUSH
#define PROF_DECL uint64_t prof_acc[16] = {0}
#define PROF_T(v) const uint64_t v = clock64()
#define PROF_ADD(slot, t0) prof_acc[slot] += clock64() - (t0)
#define PROF_CNT(slot, n) prof_acc[slot] += (n)  // event counts: 5 match rounds, 6 batches, 7 symbols
#define PROF_FLUSH do { if (__lane_id() == 0) for (int k_ = 0; k_ < 16; k_++) atomicAdd(&g_prof[k_], (unsigned long long)prof_acc[k_]); } while (0)
#else
#define PROF_DECL
#define PROF_FLUSH
#define PROF_T(v)
#define PROF_ADD(slot, t0)
#define PROF_CNT(slot, n)
#endif

namespace {

#ifndef ZG_INFLATE_RING
#define ZG_INFLATE_RING 1024
#endif
// LDS ring of recent output (power of two). Small on purpose: sources older than the ring are read
// back from the flushed output (L2-resident), and a 1 KiB ring (512-B batches, 256-B flushes)
// measured faster than 2 KiB (42.5 -> 39.5 ms) and 512 B (40.5 ms) on C3 chunks at the same 5 waves
// per SIMD (profiles/r02_gzip_lab_ring_ab.txt).
constexpr int RING = ZG_INFLATE_RING;
constexpr int RMASK = RING - 1;
#ifndef ZG_INFLATE_BATCH_CAP
#define ZG_INFLATE_BATCH_CAP (RING / 2)
#endif
#ifndef ZG_INFLATE_FLUSH_MIN
#define ZG_INFLATE_FLUSH_MIN (RING / 4)
#endif
constexpr int BATCH_CAP = ZG_INFLATE_BATCH_CAP;  // a batch takes symbols while it holds fewer bytes
constexpr int FLUSH_MIN = ZG_INFLATE_FLUSH_MIN;  // flush the ring to the slot once this many are pending
// Unflushed bytes never exceed the ring: fewer than FLUSH_MIN before a batch, and a batch takes
// symbols while it holds fewer than BATCH_CAP bytes, the last one a match of at most 258. So every
// source older than the ring has been flushed, and no unflushed byte is overwritten.
static_assert((FLUSH_MIN - 1) + (BATCH_CAP - 1) + 258 <= RING, "gzip ring: unflushed bytes must fit it");
#ifndef ZG_INFLATE_LROOT
#define ZG_INFLATE_LROOT 9
#endif
#ifndef ZG_INFLATE_LSUB
#define ZG_INFLATE_LSUB 352
#endif
#ifndef ZG_INFLATE_DSUB
#define ZG_INFLATE_DSUB 32
#endif
constexpr int LROOT = ZG_INFLATE_LROOT, DROOT = 8;
// Second-level tables for codes longer than the root. zlib's bound for 286 symbols with a 9-bit
// root is 852 entries in all (340 in subtables); distance subtables are sized for real data (C3
// chunks need at most 16 entries with an 8-bit root): prefixes past the space take the slow path.
constexpr int LSUB = ZG_INFLATE_LSUB, DSUB = ZG_INFLATE_DSUB;
#ifndef ZG_INFLATE_SELECT
#define ZG_INFLATE_SELECT 1  // lane symbol decode by selects instead of divergent branches
#endif
#ifndef ZG_INFLATE_XDEP
#define ZG_INFLATE_XDEP 1  // matches resolve by exact dependencies (0: first-pending frontier)
#endif
#ifndef ZG_INFLATE_RANGE
#define ZG_INFLATE_RANGE 1  // a match's readiness: pending mask vs the index range of its source
#endif
#ifndef ZG_INFLATE_XW
#define ZG_INFLATE_XW 8  // > 0: in-ring matches up to this many bytes copy through aligned ring words
#endif
#ifndef ZG_INFLATE_BW
#define ZG_INFLATE_BW 1  // window words by plain readlanes when they lie in one register window
#endif
#ifndef ZG_INFLATE_PJ
#define ZG_INFLATE_PJ 1  // chain a window's symbols by pointer jumping (0: scalar walk)
#endif
#ifndef ZG_INFLATE_PJL
#define ZG_INFLATE_PJL 2  // pointer-jumping doublings: a window chains up to 2^(PJL+1) symbols
#endif

// table entry: bits 0-3 code length (0 = longer than the root: slow path), 4-5 kind,
// 6-9 extra bits, 16-31 value (literal byte / length base / distance base)
constexpr uint32_t K_LIT = 0, K_LEN = 1, K_EOB = 2, K_BAD = 3;
// lookahead stop flags (above the advance / output-length fields of a lane's symbol info)
constexpr uint32_t F_EOB = 1u << 17, F_BAD = 1u << 18, F_SLOW = 1u << 19;
// table entry with code length 0 and this bit: a subtable at index bits 16-31, indexed by the next
// bits 6-9 bits of the stream; entries are then complete (code length = the whole code)
constexpr uint32_t F_SUBT = 1u << 10;

__constant__ uint16_t c_len_base[29] = {3,  4,  5,  6,  7,  8,  9,  10, 11,  13,  15,  17,  19,  23, 27,
                                        31, 35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
__constant__ uint8_t c_len_extra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2,
                                        2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
__constant__ uint16_t c_dist_base[30] = {1,   2,   3,   4,   5,   7,    9,    13,   17,   25,
                                         33,  49,  65,  97,  129, 193,  257,  385,  513,  769,
                                         1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
__constant__ uint8_t c_dist_extra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6,
                                         6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};
__constant__ uint8_t c_clen_order[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};

struct HuffMeta {  // canonical code description for the slow path
  uint16_t count[16];
  uint16_t first[16];
  uint16_t offs[16];
  uint16_t maxlen;
};

struct Smem {
  union {  // the output ring, also read as aligned words (no generic-pointer cast of LDS)
    uint8_t ring[RING];
    uint32_t ring32[RING / 4];
  };
  union {
    struct {  // Huffman decoding tables
      uint32_t ltab[(1 << LROOT) + LSUB];
      uint32_t dtab[(1 << DROOT) + DSUB];
    };
    CrcTables crc;  // after the last block: the gzip trailer's CRC-32 of the decoded stream
  };
  uint8_t sink[4];  // the executor's discarded byte stores (branch-free short copies)
  uint16_t lsorted[288];
  uint16_t dsorted[32];
  HuffMeta lm, dm, cm;
  uint32_t tmp[16];
  union {
    struct {  // a dynamic block header (decoded before the block's symbol batches)
      uint8_t lens[320];  // code lengths: 0..HLIT-1 literal/length, then distances
      uint8_t clens[20];
      uint16_t csorted[20];
    };
    struct {  // a symbol batch
      uint32_t rec[64];   // the batch's symbols: literal byte, or (1<<31)|(dist<<9)|len
      union {             // output interval of each symbol in the batch (match dependencies)
        uint16_t rbeg[64];
        uint4 rbeg4[8];   // eight 16-B segments of 8 entries (the pivot search)
      };
      uint16_t rend[64];
    };
  };
};

// The pipelined latency mode (k_gzip<false, true>): wave 0 decodes the symbol regions of round r+1
// while wave 1 executes round r's records. Its own batch intervals (Smem's share their space with the
// block header wave 0 parses meanwhile) and the hand-off: per message slot the message, the round's
// symbol count and each decoder lane's region (first symbol, record offset, count), and the output
// state the waves pass back and forth when wave 0 writes output itself (stored blocks, the canonical
// slow path, the stream's end).
constexpr uint32_t P_END = 0, P_ROUND = 1, P_SYNC = 2;
struct SmemP : Smem {
  union {
    uint16_t rbeg[64];
    uint4 rbeg4[8];
  };
  uint16_t rend[64];
  uint32_t p_msg[2], p_total[2], p_err;
  uint64_t p_pos, p_flushed;
  uint32_t p_rb[2][64], p_ro[2][64], p_cnt[2][64];
  uint32_t p_crc_bad;  // wave 1's CRC-32C check of the stream (crc_tail 1) failed
  CrcTables c32c;      // its tables (the Huffman tables' space is wave 0's meanwhile)
};

__device__ __forceinline__ uint32_t U(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ int lane_id() { return __lane_id(); }
// Syncs inside k_gzip are wave syncs: its workgroup is one wave (throughput mode) or two waves with
// roles of their own (k_gzip<.., true>, the pipelined latency mode), whose only workgroup barriers
// are the hand-offs between them. In a one-wave workgroup this is what __syncthreads() was.
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
  __builtin_amdgcn_wave_barrier();
}
// inclusive wave64 prefix sum: row shifts within 16 lanes, then row broadcasts (DPP, no LDS)
__device__ __forceinline__ uint32_t wave_incl_sum(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);  // row_bcast:15
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);  // row_bcast:31
  return x;
}

// ---------------------------------------------------------------------------------------------
// Bit reader over aligned 32-bit words held in two per-lane register windows.
// ---------------------------------------------------------------------------------------------
struct Bits {
  const uint32_t *base;  // aligned word stream
  uint32_t nwords;       // words that may be loaded (covering the item)
  uint32_t wcur;         // index of the first word of the current window
  uint32_t win0, win1;   // current / next window (lane l holds word wcur + l / wcur + 64 + l)
  uint32_t wnext;        // next word to append to the bit buffer
  uint64_t bb;           // bit buffer (LSB first)
  uint32_t nb;           // valid bits in bb
  uint64_t consumed;     // bits consumed from the start of the aligned stream
};

__device__ __forceinline__ uint32_t load_word(const Bits &B, uint32_t w) {
  return w < B.nwords ? B.base[w] : 0u;
}

__device__ __forceinline__ void bits_seek(Bits &B, uint64_t bitpos) {
  // position the reader at an absolute bit offset of the aligned stream
  const uint32_t w = (uint32_t)(bitpos >> 5);
  B.wcur = w & ~63u;
  B.win0 = load_word(B, B.wcur + lane_id());
  B.win1 = load_word(B, B.wcur + 64 + lane_id());
  B.wnext = w;
  B.bb = 0;
  B.nb = 0;
  B.consumed = (uint64_t)w * 32;
  // fill and drop the leading bits
  const uint32_t skip = (uint32_t)(bitpos & 31);
  // append one word
  {
    const uint32_t word = U(__builtin_amdgcn_readlane(B.win0, (int)(B.wnext - B.wcur)));
    B.bb = word;
    B.nb = 32;
    B.wnext++;
  }
  B.bb >>= skip;
  B.nb -= skip;
  B.consumed += skip;
}

// Move the window pair forward until word w is in the first window.
__device__ __forceinline__ void bits_advance_to(Bits &B, uint32_t w) {
  while ((int32_t)(w - B.wcur) >= 64) {  // forward only
    B.wcur += 64;
    B.win0 = B.win1;
    B.win1 = load_word(B, B.wcur + 64 + lane_id());
  }
}

// word wcur + k (k < 128) of the window pair, as a uniform value
__device__ __forceinline__ uint32_t win_word(const Bits &B, uint32_t k) {
  return k < 64 ? U(__builtin_amdgcn_readlane(B.win0, (int)k)) : U(__builtin_amdgcn_readlane(B.win1, (int)(k - 64)));
}

// The five aligned words w..w+4 (160 bits) as uniform values.
__device__ __forceinline__ void bits_words(Bits &B, uint32_t w, uint32_t &W0, uint32_t &W1, uint32_t &W2,
                                           uint32_t &W3, uint32_t &W4) {
  bits_advance_to(B, w);
  const uint32_t k = w - B.wcur;
#if ZG_INFLATE_BW
  if (k <= 59) {  // all five in the first window (the common case): five plain readlanes
    W0 = U(__builtin_amdgcn_readlane(B.win0, (int)k));
    W1 = U(__builtin_amdgcn_readlane(B.win0, (int)k + 1));
    W2 = U(__builtin_amdgcn_readlane(B.win0, (int)k + 2));
    W3 = U(__builtin_amdgcn_readlane(B.win0, (int)k + 3));
    W4 = U(__builtin_amdgcn_readlane(B.win0, (int)k + 4));
    return;
  }
#endif
  W0 = win_word(B, k);
  W1 = win_word(B, k + 1);
  W2 = win_word(B, k + 2);
  W3 = win_word(B, k + 3);
  W4 = win_word(B, k + 4);
}

// Re-position the reader at an absolute (forward) bit offset without reloading the windows.
__device__ __forceinline__ void bits_seek_in(Bits &B, uint64_t bitpos) {
  const uint32_t w = (uint32_t)(bitpos >> 5);
  bits_advance_to(B, w);
  const uint32_t k = w - B.wcur;
  const uint32_t a = win_word(B, k), b = win_word(B, k + 1);
  const uint32_t sk = (uint32_t)(bitpos & 31);
  B.bb = (((uint64_t)b << 32) | a) >> sk;
  B.nb = 64 - sk;
  B.wnext = w + 2;
  B.consumed = bitpos;
}

__device__ __forceinline__ void bits_refill(Bits &B) {
  if (B.nb <= 32) {
    // windows only ever advance past words already consumed (the walk re-reads from `consumed`)
    bits_advance_to(B, (uint32_t)(B.consumed >> 5));
    const uint32_t word = win_word(B, B.wnext - B.wcur);  // wnext <= consumed word + 3: < 128
    B.bb |= (uint64_t)word << B.nb;
    B.nb += 32;
    B.wnext++;
  }
}

__device__ __forceinline__ uint32_t bits_peek(const Bits &B, uint32_t n) { return (uint32_t)B.bb & ((1u << n) - 1); }
__device__ __forceinline__ void bits_drop(Bits &B, uint32_t n) {
  B.bb >>= n;
  B.nb -= n;
  B.consumed += n;
}
__device__ __forceinline__ uint32_t bits_get(Bits &B, uint32_t n) {
  bits_refill(B);
  const uint32_t v = bits_peek(B, n);
  bits_drop(B, n);
  return v;
}

__device__ __forceinline__ uint32_t rev_bits(uint32_t v, uint32_t n) { return __builtin_bitreverse32(v) >> (32 - n); }

// ---------------------------------------------------------------------------------------------
// Cooperative canonical-Huffman table build. lens[n] code lengths (LDS). kind: 0 litlen, 1 dist,
// 2 code-length codes (root 7 = max length: no slow path). Returns false on an invalid code set
// (over-subscribed, or incomplete with more than one code: zlib inflate_table rules).
// ---------------------------------------------------------------------------------------------
// table entry for symbol `sym` of an alphabet (kind as in build_table) with code length L
__device__ __forceinline__ uint32_t table_entry(int kind, uint32_t sym, uint32_t L) {
  if (kind == 0) {
    if (sym < 256) return (sym << 16) | (K_LIT << 4) | L;
    if (sym == 256) return (K_EOB << 4) | L;
    if (sym < 286) return ((uint32_t)c_len_base[sym - 257] << 16) | ((uint32_t)c_len_extra[sym - 257] << 6) | (K_LEN << 4) | L;
    return (K_BAD << 4) | L;
  }
  if (kind == 1) {
    if (sym < 30) return ((uint32_t)c_dist_base[sym] << 16) | ((uint32_t)c_dist_extra[sym] << 6) | (K_LEN << 4) | L;
    return (K_BAD << 4) | L;
  }
  return (sym << 16) | L;
}

__device__ bool build_table(const uint8_t *lens, uint32_t n, uint32_t root, uint32_t *tab, uint16_t *sorted,
                            HuffMeta &M, int kind, uint32_t *tmp, uint32_t sub_cap) {
  const int lane = lane_id();
  if (lane < 16) tmp[lane] = 0;
  wsync();
  for (uint32_t s = lane; s < n; s += 64) {
    const uint32_t l = lens[s];
    if (l) atomicAdd(&tmp[l], 1u);
  }
  wsync();
  // uniform: counts, validity, first codes, offsets
  uint32_t cnt[16];
  for (int l = 0; l < 16; l++) cnt[l] = U(tmp[l]);
  int left = 1;
  uint32_t maxlen = 0;
  for (int l = 1; l < 16; l++) {
    left <<= 1;
    left -= (int)cnt[l];
    if (cnt[l]) maxlen = l;
    if (left < 0) return false;  // over-subscribed
  }
  if (left > 0 && maxlen != 1 && maxlen != 0) return false;  // incomplete set (zlib inflate_table)
  if (kind == 2 && (left > 0 || maxlen == 0)) return false;    // code-length codes must be complete
  // canonical first codes (RFC 1951 3.2.2): next_code[l] = (next_code[l-1] + count[l-1]) << 1
  uint32_t first[16];
  {
    uint32_t code = 0;
    first[0] = 0;
    for (int l = 1; l < 16; l++) {
      code = (code + (l > 1 ? cnt[l - 1] : 0)) << 1;
      first[l] = code;
    }
  }
  if (lane == 0) {
    uint32_t off = 0;
    for (int l = 1; l < 16; l++) {
      M.count[l] = (uint16_t)cnt[l];
      M.first[l] = (uint16_t)first[l];
      M.offs[l] = (uint16_t)off;
      off += cnt[l];
    }
    M.maxlen = (uint16_t)maxlen;
    tmp[0] = 0;  // subtable allocation counter (the counts were read above)
  }
  wsync();
  // sorted symbols (by length, then symbol) via ballot ranks. The per-length offsets and codes are
  // read from M in LDS (uniform addresses): private arrays indexed by a loop variable would live in
  // scratch memory (one scratch round trip per access; 17 % of k_gzip's time went to table builds)
  uint32_t lv[5];  // n <= 320 lengths: five per lane
#pragma unroll
  for (int j = 0; j < 5; j++) {
    const uint32_t s = 64u * j + (uint32_t)lane;
    lv[j] = s < n ? lens[s] : 0u;
  }
  for (uint32_t L = 1; L <= maxlen; L++) {
    uint32_t b = U(M.offs[L]);
#pragma unroll
    for (int j = 0; j < 5; j++) {
      if (64u * j >= n) break;
      const uint64_t m = __ballot(lv[j] == L);
      if (lv[j] == L) sorted[b + __builtin_popcountll(m & ((1ull << lane) - 1))] = (uint16_t)(64u * j + lane);
      b += __builtin_popcountll(m);
    }
  }
  wsync();
  // root table fill: entry e <-> R-bit MSB-first prefix v = reverse(e). A prefix of codes longer
  // than the root gets a subtable of 2^sb entries (sb = its longest code - root), indexed by the next
  // sb stream bits; subtables are allocated from tab[size..size+sub_cap) by an LDS counter (tmp[0]).
  const uint32_t size = 1u << root;
  for (uint32_t e = lane; e < size; e += 64) {
    const uint32_t v = rev_bits(e, root);
    uint32_t entry = (K_BAD << 4) | 0xF;  // invalid code marker (len 15 so it is consumed; flagged bad)
    bool found = false;
    for (uint32_t L = 1; L <= root && L <= maxlen && !found; L++) {
      const uint32_t c = v >> (root - L), f = M.first[L];
      if (c - f < M.count[L]) {
        entry = table_entry(kind, sorted[M.offs[L] + c - f], L);
        found = true;
      }
    }
    if (!found && maxlen > root) {
      uint32_t sb = 0;
      for (uint32_t L = root + 1; L <= maxlen; L++) {
        const uint32_t lo = v << (L - root), hi = (v + 1) << (L - root), f = M.first[L], k = M.count[L];
        if (k && f < hi && f + k > lo) sb = L - root;
      }
      if (sb) {
        const uint32_t base = atomicAdd(&tmp[0], 1u << sb);
        entry = 0;  // subtable space exhausted: the canonical slow path
        if (base + (1u << sb) <= sub_cap) entry = ((size + base) << 16) | (sb << 6) | F_SUBT;
      }
    }
    tab[e] = entry;
  }
  wsync();
  if (maxlen > root) {
    // Subtables, filled by symbol (zlib's replication) with all lanes: first every allocated entry
    // invalid (an incomplete code's holes), then each code longer than the root writes its entries:
    // with d = L - root bits past the prefix, the entries x = rev(last d code bits) + j * 2^d of its
    // prefix's subtable. (Filling by entry took one lane 2^sb canonical searches in a row.)
    const uint32_t used = min(U(tmp[0]), sub_cap);
    for (uint32_t x = lane; x < used; x += 64) tab[size + x] = (K_BAD << 4) | 0xF;
    wsync();
    const uint32_t i0 = U(M.offs[root + 1]), i1 = U(M.offs[maxlen]) + U(M.count[maxlen]);
    for (uint32_t i = i0 + lane; i < i1; i += 64) {
      const uint32_t sym = sorted[i], L = lens[sym];
      const uint32_t code = M.first[L] + (i - M.offs[L]);  // MSB-first, L bits
      const uint32_t d = L - root;
      const uint32_t pe = tab[rev_bits(code >> d, root)];
      if (!(pe & F_SUBT)) continue;  // its prefix took the slow path (no subtable space)
      const uint32_t sb = (pe >> 6) & 15, sbase = pe >> 16;
      const uint32_t ent = table_entry(kind, sym, L);
      for (uint32_t x = rev_bits(code & ((1u << d) - 1), d); x < (1u << sb); x += 1u << d) tab[sbase + x] = ent;
    }
    wsync();
  }
  return true;
}

// Decode one symbol with a root table; returns the table-style entry (slow path resolves long codes).
__device__ __forceinline__ uint32_t decode_sym(Bits &B, const uint32_t *tab, uint32_t root, const uint16_t *sorted,
                                               const HuffMeta &M, int kind) {
  bits_refill(B);
  uint32_t e = U(tab[bits_peek(B, root)]);
  if (e & 15) {
    bits_drop(B, e & 15);
    return e;
  }
  // slow path: codes longer than the root, canonical walk from length root+1
  uint32_t v = rev_bits(bits_peek(B, root), root);
  uint32_t L = root;
  const uint32_t maxlen = U(M.maxlen);
  uint32_t sym = 0xFFFF;
  uint64_t bb = B.bb >> root;
  while (L < maxlen) {
    L++;
    v = (v << 1) | (uint32_t)(bb & 1);
    bb >>= 1;
    const uint32_t first = U(M.first[L]), cnt = U(M.count[L]);
    if (v - first < cnt) {
      sym = U(sorted[U(M.offs[L]) + v - first]);
      break;
    }
  }
  if (sym == 0xFFFF) return (K_BAD << 4) | 15;
  bits_drop(B, L);
  if (kind == 0) {
    if (sym < 256) return (sym << 16) | (K_LIT << 4) | 15;
    if (sym == 256) return (K_EOB << 4) | 15;
    if (sym < 286) return ((uint32_t)c_len_base[sym - 257] << 16) | ((uint32_t)c_len_extra[sym - 257] << 6) | (K_LEN << 4) | 15;
    return (K_BAD << 4) | 15;
  }
  if (sym < 30) return ((uint32_t)c_dist_base[sym] << 16) | ((uint32_t)c_dist_extra[sym] << 6) | (K_LEN << 4) | 15;
  return (K_BAD << 4) | 15;
}

__device__ __forceinline__ void build_fixed_lens(uint8_t *lens) {
  for (uint32_t s = lane_id(); s < 320; s += 64) {
    uint8_t l;
    if (s < 144) l = 8;
    else if (s < 256) l = 9;
    else if (s < 280) l = 7;
    else if (s < 288) l = 8;
    else l = 5;  // 30 distance codes (+2 invalid) of length 5, stored at 288..319
    lens[s] = l;
  }
  wsync();
}

// One lane's symbol at a 64-bit lookahead value V = Vhi:Vlo (the stream from the symbol's first
// bit): literal/length code (+ subtable), length extra bits, distance code (+ subtable), distance
// extra bits — at most 48 bits. info: bits 0-7 advance in bits, 8-16 output bytes, 17+ stop flags;
// rec: the literal byte, or (1<<31)|(dist<<9)|len.
__device__ __forceinline__ void lane_symbol(const Smem &S, uint32_t Vlo, uint32_t Vhi, uint32_t &info, uint32_t &rec) {
  const uint64_t V = ((uint64_t)Vhi << 32) | Vlo;
  uint32_t E = S.ltab[Vlo & ((1u << LROOT) - 1)];
  if (E & F_SUBT) E = S.ltab[(E >> 16) + ((Vlo >> LROOT) & ((1u << ((E >> 6) & 15)) - 1))];
  const uint32_t L = E & 15, kind = (E >> 4) & 3, lx = (E >> 6) & 15;
  const uint32_t s1 = L + lx;  // <= 20
  uint32_t D = S.dtab[(Vlo >> s1) & ((1u << DROOT) - 1)];
  if (D & F_SUBT) D = S.dtab[(D >> 16) + ((uint32_t)(V >> (s1 + DROOT)) & ((1u << ((D >> 6) & 15)) - 1))];
  const uint32_t DL = D & 15, dx = (D >> 6) & 15, s2 = s1 + DL;
#if ZG_INFLATE_SELECT
  // every kind computed, then selected (no divergent branches)
  const uint32_t len = (E >> 16) + ((Vlo >> L) & ((1u << lx) - 1));
  const uint32_t dist = (D >> 16) + ((uint32_t)(V >> s2) & ((1u << dx) - 1));
  const uint32_t i_len = DL == 0 ? F_SLOW : (((D >> 4) & 3) != K_LEN ? F_BAD : ((s2 + dx) | (len << 8)));
  const uint32_t i_oth = kind == K_EOB ? (L | F_EOB) : F_BAD;
  info = kind == K_LIT ? (L | (1u << 8)) : (kind == K_LEN ? i_len : i_oth);
  rec = kind == K_LIT ? (E >> 16) : (0x80000000u | (dist << 9) | len);
#else
  if (kind == K_LIT) {
    info = L | (1u << 8);
    rec = E >> 16;
  } else if (kind == K_LEN) {
    const uint32_t len = (E >> 16) + ((Vlo >> L) & ((1u << lx) - 1));
    const uint32_t dist = (D >> 16) + ((uint32_t)(V >> s2) & ((1u << dx) - 1));
    info = (s2 + dx) | (len << 8);
    rec = 0x80000000u | (dist << 9) | len;
    if (DL == 0) info = F_SLOW;  // distance code past the subtable space
    else if (((D >> 4) & 3) != K_LEN) info = F_BAD;
  } else {
    info = kind == K_EOB ? (L | F_EOB) : F_BAD;
    rec = 0;
  }
#endif
  if (L == 0) info = F_SLOW;  // literal/length code past the subtable space
}

// A code longer than its table's root whose prefix got no subtable space (a stream whose code set
// outgrows LSUB / DSUB): this lane walks the canonical code from root + 1 (the HuffMeta counts and
// the sorted symbols build_table keeps), so the segmented decode goes on instead of handing the rest
// of the block to the one-symbol-at-a-time path (one such block made a shard's slowest stream ~60 %
// slower). Returns a table entry (code length in bits 0-3) or a K_BAD one.
__device__ __forceinline__ uint32_t lane_canon(uint64_t bits, const uint32_t *tab, uint32_t root, const uint16_t *sorted,
                                            const HuffMeta &M, int kind) {
  uint32_t E = tab[(uint32_t)bits & ((1u << root) - 1)];
  if (E & F_SUBT) E = tab[(E >> 16) + ((uint32_t)(bits >> root) & ((1u << ((E >> 6) & 15)) - 1))];
  if (E & 15) return E;
  uint32_t v = rev_bits((uint32_t)bits & ((1u << root) - 1), root), L = root, sym = 0xFFFF;
  uint64_t b = bits >> root;
  const uint32_t maxlen = M.maxlen;
  while (L < maxlen) {
    L++;
    v = (v << 1) | (uint32_t)(b & 1);
    b >>= 1;
    const uint32_t first = M.first[L], cnt = M.count[L];
    if (v - first < cnt) {
      sym = sorted[M.offs[L] + v - first];
      break;
    }
  }
  return sym == 0xFFFF ? ((K_BAD << 4) | 15) : table_entry(kind, sym, L);
}
__device__ __forceinline__ void lane_symbol_slow(const Smem &S, uint64_t V, uint32_t &info, uint32_t &rec) {
  const uint32_t E = lane_canon(V, S.ltab, LROOT, S.lsorted, S.lm, 0);
  const uint32_t L = E & 15, kind = (E >> 4) & 3, lx = (E >> 6) & 15;
  rec = 0;
  if (kind == K_LIT) {
    info = L | (1u << 8);
    rec = E >> 16;
  } else if (kind == K_EOB) {
    info = L | F_EOB;
  } else if (kind == K_LEN) {
    const uint32_t len = (E >> 16) + ((uint32_t)(V >> L) & ((1u << lx) - 1));
    const uint32_t s1 = L + lx;
    const uint32_t D = lane_canon(V >> s1, S.dtab, DROOT, S.dsorted, S.dm, 1);
    const uint32_t DL = D & 15, dx = (D >> 6) & 15;
    if (((D >> 4) & 3) != K_LEN) {
      info = F_BAD;
    } else {
      const uint32_t dist = (D >> 16) + ((uint32_t)(V >> (s1 + DL)) & ((1u << dx) - 1));
      info = (s1 + DL + dx) | (len << 8);
      rec = 0x80000000u | (dist << 9) | len;
    }
  } else {
    info = F_BAD;
  }
}

// Flush output bytes [from, to) (absolute positions) from the ring to the slot with 16-B stores.
// Words straddling `to` are rewritten by the next flush.
// The gzip trailer's CRC-32 by one wave (crc.hpp's helpers index by threadIdx / blockDim, and in the
// pipelined kernel the second wave has left by then): slice-by-4 tables in LDS, 64 lane segments
// merged by the GF(2) shift tree.
__device__ inline void wave_crc_tables(CrcTables &T, uint32_t poly) {
  const uint32_t l = (uint32_t)lane_id();
  for (uint32_t i = l; i < 256; i += 64) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ poly : c >> 1;
    T.t[0][i] = c;
  }
  wsync();
  for (uint32_t i = l; i < 256; i += 64) {
    uint32_t c = T.t[0][i];
    for (int k = 1; k < 4; k++) {
      c = (c >> 8) ^ T.t[0][c & 0xff];
      T.t[k][i] = c;
    }
  }
  if (l < 32) T.x2n[l] = poly == POLY_CRC32C ? c_x2n_crc32c[l] : c_x2n_crc32[l];
  wsync();
}
__device__ inline uint32_t wave_crc(const uint8_t *p, uint64_t n, const CrcTables &T, uint32_t poly) {
  const uint32_t l = (uint32_t)lane_id();
  uint64_t seg = (n + 63) / 64;
  seg = (seg + 15) & ~(uint64_t)15;  // 16-B aligned segments: the inner loop runs on 16-B loads
  const uint64_t b0 = min<uint64_t>((uint64_t)l * seg, n), b1 = min<uint64_t>(b0 + seg, n);
  uint32_t c = crc_segment(p + b0, b1 - b0, T);
  uint64_t len = b1 - b0;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t c2 = __shfl_down(c, off, 64);
    const uint64_t l2 = __shfl_down(len, off, 64);
    if (l % (2 * off) == 0 && l + off < 64) {
      c = crc_combine(c, c2, l2, T.x2n, poly);
      len += l2;
    }
  }
  return U(__shfl(c, 0, 64));
}

// Where decoded byte p of a stream lives: its slot (base + p), or, for a direct item (GzDirect), the
// output array: row p >> lbs of the chunk, whose index splits over the row axes innermost first
// (extent 2^sh[k] each, the outermost unbounded), at column p & (2^lbs - 1). 16-B pieces never
// straddle a row (rows are multiples of 16 bytes on 16-B aligned addresses).
#ifndef ZG_GZ_DIRECT_READS
#define ZG_GZ_DIRECT_READS 0  // 1: a direct item lives only in the array (sources older than the ring read
                              // back from its rows, no slot copy); 0: the slot is written too (A/B)
#endif
struct OutMap {
  uint8_t *slot;  // the item's slot: always written (sources older than the ring are read back from it)
  uint8_t *base;
  uint32_t o0, o1;  // output byte stride of the inner and the outer row axis (nd 3; nd 2: o0 only)
  uint32_t cfg;     // bit 31: direct; bits 0-7: lbs; bits 8-15: log2 of the inner row axis' extent
  uint32_t want;    // the chunk's bytes: a stream decoding longer writes only its slot past them
  __device__ __forceinline__ uint8_t *at(uint64_t p) const {
    const uint32_t lbs = cfg & 255, sh = (cfg >> 8) & 255;
    const uint32_t r = (uint32_t)(p >> lbs);
    return base + (p & ((1ull << lbs) - 1)) + (uint64_t)(r & ((1u << sh) - 1u)) * o0 + (uint64_t)(r >> sh) * o1;
  }
  __device__ __forceinline__ const uint8_t *rd(uint64_t p) const {  // a source byte older than the ring
    return (ZG_GZ_DIRECT_READS && (cfg >> 31) && p < want) ? at(p) : slot + p;
  }
};

#if ZG_GZ_DIRECT_READS
// The CRC of decoded bytes [0, n) of a direct item: wave_crc's lane segments, each run over its row pieces.
__device__ inline uint32_t wave_crc_map(const OutMap &O, uint64_t n, const CrcTables &T, uint32_t poly) {
  if (!(O.cfg >> 31) || n > O.want) return wave_crc(O.slot, n, T, poly);
  const uint32_t l = (uint32_t)lane_id(), lbs = O.cfg & 255;
  uint64_t seg = (n + 63) / 64;
  seg = (seg + 15) & ~(uint64_t)15;
  const uint64_t b0 = min<uint64_t>((uint64_t)l * seg, n), b1 = min<uint64_t>(b0 + seg, n);
  uint32_t c = 0xFFFFFFFFu;
  for (uint64_t q = b0; q < b1;) {
    const uint64_t e = min<uint64_t>(b1, ((q >> lbs) + 1) << lbs);
    c = crc_run(c, O.at(q), e - q, T);
    q = e;
  }
  c = ~c;
  uint64_t len = b1 - b0;
  for (int off = 1; off < 64; off <<= 1) {
    const uint32_t c2 = __shfl_down(c, off, 64);
    const uint64_t l2 = __shfl_down(len, off, 64);
    if (l % (2 * off) == 0 && l + off < 64) {
      c = crc_combine(c, c2, l2, T.x2n, poly);
      len += l2;
    }
  }
  return U(__shfl(c, 0, 64));
}
#endif

__device__ __forceinline__ void flush(const Smem &S, const OutMap &O, uint64_t cap, uint64_t from, uint64_t to) {
  const uint64_t a = from & ~(uint64_t)15, b = (to + 15) & ~(uint64_t)15;
  for (uint64_t p = a + (uint64_t)lane_id() * 16; p < b; p += 64 * 16) {
    if (p + 16 <= cap) {
      const uint4 v = *(const uint4 *)&S.ring[p & RMASK];
      const bool d = (O.cfg >> 31) && p < O.want;  // want is a multiple of 16
      if (!ZG_GZ_DIRECT_READS || !d) *(uint4 *)(O.slot + p) = v;
      if (d) *(uint4 *)O.at(p) = v;
    } else {
      for (uint64_t q = p; q < cap && q < p + 16; q++) {
        const bool d = (O.cfg >> 31) && q < O.want;
        if (!ZG_GZ_DIRECT_READS || !d) O.slot[q] = S.ring[q & RMASK];
        if (d) *O.at(q) = S.ring[q & RMASK];
      }
    }
  }
}

#ifndef ZG_INFLATE_SEG
#define ZG_INFLATE_SEG 1  // Huffman blocks: every lane decodes a region of the stream serially (k_gzip's seg path)
#endif
#ifndef ZG_INFLATE_SEGB
#define ZG_INFLATE_SEGB 512  // bits of the stream per lane region
#endif
#ifndef ZG_INFLATE_OVL
#define ZG_INFLATE_OVL 384  // a lane starts decoding this many bits before its region (chains converge)
#endif
#ifndef ZG_INFLATE_SEGCAP
#define ZG_INFLATE_SEGCAP 96  // symbol records per lane region (a fuller region ends the round there)
#endif
#ifndef ZG_INFLATE_PCL
#define ZG_INFLATE_PCL 1  // dynamic-header code lengths decoded lane-parallel (pointer-jumped windows)
#endif
#ifndef ZG_INFLATE_PIV
#define ZG_INFLATE_PIV 1  // exec_batch: match source ranges by a two-level pivot search (no LDS search chain)
#endif
#ifndef ZG_INFLATE_XFETCH
#define ZG_INFLATE_XFETCH 1  // executor batches: region lookup by ballots + records loaded a batch ahead
#endif
#ifndef ZG_INFLATE_MAXREP
#define ZG_INFLATE_MAXREP 8  // out-of-sync lanes re-decoded per round from their predecessor's exit
#endif
constexpr uint32_t SEGB = ZG_INFLATE_SEGB, OVL = ZG_INFLATE_OVL, SEGCAP = ZG_INFLATE_SEGCAP;
static_assert(OVL <= SEGB && SEGB >= 64, "a lane starts inside its predecessor's region");
constexpr uint32_t SG_END = 0, SG_EOB = 1, SG_BAD = 2, SG_SLOW = 3, SG_CAP = 4, SG_PAST = 5;

// One lane's view of the aligned word stream: words wi..wi+2 (96 bits) in registers, the next one
// loaded ahead; positions are absolute bits of the aligned stream (the Bits domain).
#ifndef ZG_INFLATE_LPF
#define ZG_INFLATE_LPF 4  // words a lane's reader loads ahead of the three it decodes from (1..4)
#endif
struct LaneRd {
  const uint32_t *base;
  uint32_t nwords, wi, w0, w1, w2, pf, pf1, pf2, pf3;
  __device__ __forceinline__ uint32_t ld(uint32_t k) const { return k < nwords ? base[k] : 0u; }
  __device__ __forceinline__ void seek(uint64_t p) {
    wi = (uint32_t)(p >> 5);
    w0 = ld(wi);
    w1 = ld(wi + 1);
    w2 = ld(wi + 2);
    pf = ld(wi + 3);
    if (ZG_INFLATE_LPF > 1) pf1 = ld(wi + 4);
    if (ZG_INFLATE_LPF > 2) pf2 = ld(wi + 5);
    if (ZG_INFLATE_LPF > 3) pf3 = ld(wi + 6);
  }
  // forward to the word holding bit p; the word ZG_INFLATE_LPF past the decode window is loaded
  // then, so a load has ~LPF * 32 bits of decoding (a few symbols each) to arrive: the lanes' regions
  // lie 64 B apart, every load of the wave touches 64 lines, and 3 words ahead stalled on HBM
  __device__ __forceinline__ void adv(uint64_t p) {
    while ((uint32_t)(p >> 5) > wi) {
      w0 = w1;
      w1 = w2;
      w2 = pf;
      if (ZG_INFLATE_LPF > 1) pf = pf1;
      if (ZG_INFLATE_LPF > 2) pf1 = pf2;
      if (ZG_INFLATE_LPF > 3) pf2 = pf3;
      wi++;
      const uint32_t nx = ld(wi + 2 + ZG_INFLATE_LPF);
      if (ZG_INFLATE_LPF == 1) pf = nx;
      else if (ZG_INFLATE_LPF == 2) pf1 = nx;
      else if (ZG_INFLATE_LPF == 3) pf2 = nx;
      else pf3 = nx;
    }
  }
  __device__ __forceinline__ void peek(uint64_t p, uint32_t &lo, uint32_t &hi) const {
    const uint32_t o = (uint32_t)p & 31;
    lo = __builtin_amdgcn_alignbit(w1, w0, o);
    hi = __builtin_amdgcn_alignbit(w2, w1, o);
  }
};

// One lane decodes serially from bit p (a symbol start of its chain) while p < s_end. Symbols starting
// at or after s_own are its region's: their records go to rec[0..n) (at most SEGCAP), and mask marks
// the region's first 64 bit positions that start a symbol. Returns why it stopped; p is then the
// exit (SG_END: the first symbol start >= s_end), the bit after the end-of-block code (SG_EOB), or
// the symbol it stopped at. A stop before its region (SG_PAST) leaves the lane out of sync.
__device__ __forceinline__ uint32_t seg_decode(const Smem &S, LaneRd &R, uint64_t &p, uint64_t s_own,
                                               uint64_t s_end, uint64_t end_bits, uint32_t *rec, uint32_t &n,
                                               uint64_t &mask) {
  n = 0;
  mask = 0;
  R.seek(p);
  while (p < s_end) {
    if (p >= end_bits) return SG_PAST;
    R.adv(p);
    uint32_t lo, hi, info, r;
    R.peek(p, lo, hi);
    lane_symbol(S, lo, hi, info, r);
    if (info == F_SLOW) lane_symbol_slow(S, ((uint64_t)hi << 32) | lo, info, r);
    const bool own = p >= s_own;
    if (own && p - s_own < 64) mask |= 1ull << (uint32_t)(p - s_own);
    if (info >= F_EOB) {
      if (!own) return SG_PAST;
      if (info == (F_EOB | (info & 255))) {
        p += info & 255;
        return SG_EOB;
      }
      return (info & F_BAD) ? SG_BAD : SG_SLOW;
    }
    if (own) {
      if (n == SEGCAP) return SG_CAP;
      rec[n++] = r;
    }
    p += info & 255;
  }
  return SG_END;
}

__device__ __forceinline__ uint64_t shfl_up64(uint64_t v) {
  const uint32_t lo = (uint32_t)__shfl_up((int)(uint32_t)v, 1, 64), hi = (uint32_t)__shfl_up((int)(uint32_t)(v >> 32), 1, 64);
  return ((uint64_t)hi << 32) | lo;
}

// Execute one batch of symbols: lane t < cnt holds symbol record rec_in (a literal byte, or
// (1<<31)|(dist<<9)|len); `bytes` = the batch's output bytes (pos + bytes <= cap checked by the
// caller). Literals are written at once, matches resolve in rounds by exact dependencies; the ring is
// flushed to the slot once FLUSH_MIN bytes are pending. Returns false for a distance past the output
// start (corrupt stream).
#ifdef ZG_PROFILE
#define XPROF(k, n) pa[k] += (n)
#else
#define XPROF(k, n)
#endif
template <class SM>
__device__ __forceinline__ bool exec_batch(SM &S, const OutMap &O, uint64_t cap, uint64_t &pos, uint64_t &flushed,
                                           uint32_t cnt, uint32_t bytes, uint32_t rec_in, uint64_t *pa) {
  (void)pa;
  const int lane = lane_id();
  wsync();
  const bool mine = lane < (int)cnt;
  const uint32_t rec = mine ? rec_in : 0u;
  const bool is_match = mine && (rec >> 31);
  const uint32_t ln = mine ? (is_match ? (rec & 511) : 1u) : 0u;
  const uint64_t mypos = pos + wave_incl_sum(ln) - ln;  // output offsets: a wave prefix sum
  if (mine && !is_match) S.ring[mypos & RMASK] = (uint8_t)rec;
  const uint64_t batch_end = pos + bytes;
  const uint32_t mlen = rec & 511, md = (rec >> 9) & 0xFFFF;
  const uint64_t msrc = mypos - md;
  if (__ballot(is_match && md > mypos)) return false;  // distance too far back
  // sources older than the ring are read back from the flushed output
  if (__ballot(is_match && msrc + RING < batch_end)) __threadfence_block();
#if ZG_INFLATE_XDEP
  // Matches resolve in rounds by exact dependencies: a match waits only while the last symbol
  // starting before the end of its source (found once per batch by a binary search over the
  // symbols' output offsets) is a pending match whose output reaches into that source. A match
  // reads at most min(len, dist) source bytes (dest byte i takes source byte i mod dist), all
  // before its own output, so ready matches never depend on each other. Long ready matches are
  // copied by the whole wave one after another, short ones by their own lane.
  const int32_t s_rel = (int32_t)(msrc - pos);                   // source start, batch-relative
  const int32_t e_rel = s_rel + (int32_t)min(mlen, md);          // source end
#if ZG_INFLATE_RANGE
  // The symbols whose output overlaps the source are an index range [lo, hi] (output offsets
  // are monotonic): hi = the last symbol starting before e_rel, lo = the last starting at or
  // before s_rel; both found by one interleaved binary search per batch. A round then tests
  // the pending mask against the range, with no LDS read.
#if ZG_INFLATE_PIV
  // Two-level search without a chain of dependent LDS reads: the entries 0, 8, .., 56 (uniform,
  // by readlane) pick the 8-entry segment, one 16-B LDS read of that segment finishes it. Lanes
  // past the batch hold 0xFFFF (above any query).
  const uint32_t rv = mine ? (uint32_t)(mypos - pos) : 0xFFFFu;
  S.rbeg[lane] = (uint16_t)rv;
  int32_t piv[8];
#pragma unroll
  for (int k = 0; k < 8; k++) piv[k] = (int32_t)U(__builtin_amdgcn_readlane((int)rv, 8 * k));
  wsync();
  int32_t hi = -1, lo = 0;
  if (is_match && e_rel > 0) {
    int32_t a = 0, b = 0;  // pivots < e_rel (>= 1: entry 0 is 0), pivots <= s_rel
#pragma unroll
    for (int k = 0; k < 8; k++) {
      a += piv[k] < e_rel;
      b += piv[k] <= s_rel;
    }
    const uint4 wa = S.rbeg4[a - 1];
    const uint4 wb = S.rbeg4[b > 0 ? b - 1 : 0];
    const uint32_t va[4] = {wa.x, wa.y, wa.z, wa.w}, vb[4] = {wb.x, wb.y, wb.z, wb.w};
    int32_t ca = 0, cb = 0;
#pragma unroll
    for (int k = 0; k < 4; k++) {
      ca += ((int32_t)(va[k] & 0xFFFF) < e_rel) + ((int32_t)(va[k] >> 16) < e_rel);
      cb += ((int32_t)(vb[k] & 0xFFFF) <= s_rel) + ((int32_t)(vb[k] >> 16) <= s_rel);
    }
    hi = 8 * (a - 1) + ca - 1;
    lo = b > 0 ? 8 * (b - 1) + cb - 1 : 0;
  }
#else
  if (mine) S.rbeg[lane] = (uint16_t)(mypos - pos);
  wsync();
  int32_t hi = -1, lo = 0;
  if (is_match && e_rel > 0) {
    hi = 0;
#pragma unroll
    for (int32_t step = 32; step; step >>= 1) {
      if (hi + step < (int32_t)cnt && (int32_t)S.rbeg[hi + step] < e_rel) hi += step;
      if (lo + step < (int32_t)cnt && (int32_t)S.rbeg[lo + step] <= s_rel) lo += step;
    }
  }
#endif
  const uint64_t rmask = hi < 0 ? 0ull : (hi >= 63 ? ~0ull : ((2ull << hi) - 1)) & ~((1ull << lo) - 1);
#else
  if (mine) S.rend[lane] = (uint16_t)(mypos - pos + (is_match ? mlen : 1u));
  if (mine) S.rbeg[lane] = (uint16_t)(mypos - pos);
  wsync();
  int32_t hi = -1;  // the last symbol that starts before e_rel
  if (is_match && e_rel > 0) {
    hi = 0;
#pragma unroll
    for (int32_t step = 32; step; step >>= 1)
      if (hi + step < (int32_t)cnt && (int32_t)S.rbeg[hi + step] < e_rel) hi += step;
  }
#endif
  bool pending = is_match;
  uint64_t pm;
  XPROF(6, 1);
  XPROF(7, cnt);
  while ((pm = __ballot(pending)) != 0) {
    XPROF(5, 1);
    bool ready = false;
    if (pending) {
#if ZG_EXP_ONEROUND  // lab experiment only (wrong output): every match ready in the first round
      ready = true;
#elif ZG_INFLATE_RANGE
      ready = (pm & rmask) == 0;
#else
      const uint64_t m = hi < 0 ? 0ull : pm & (hi >= 63 ? ~0ull : ((2ull << hi) - 1));
      ready = m == 0 || (int32_t)S.rend[63 - __builtin_clzll(m)] <= s_rel;
#endif
    }
    const uint64_t lm = __ballot(ready && mlen > 32);
    if (lm) {  // the first long ready match, by the whole wave (the others wait a round)
      const int f = __builtin_ctzll(lm);
      const uint32_t F_lo = __builtin_amdgcn_readlane((uint32_t)mypos, f);
      const uint32_t F_hi = __builtin_amdgcn_readlane((uint32_t)(mypos >> 32), f);
      const uint64_t F = ((uint64_t)F_hi << 32) | F_lo;
      const uint32_t flen = __builtin_amdgcn_readlane(mlen, f), fd = __builtin_amdgcn_readlane(md, f);
      const float inv = 1.0f / (float)fd;
      // every source byte lies before F (final): all loads (<= 5 per lane, len <= 258) are issued
      // before the first store, one wait for all of them
      uint8_t v[5];
#pragma unroll
      for (int j = 0; j < 5; j++) {
        const uint32_t i = (uint32_t)lane + 64u * j;
        uint32_t q = (uint32_t)((float)i * inv);
        int32_t rm = (int32_t)i - (int32_t)(q * fd);
        if (rm < 0) rm += fd;
        if (rm >= (int32_t)fd) rm -= fd;
        const uint64_t src = F - fd + (uint32_t)rm;
        v[j] = i < flen ? ((src + RING >= batch_end) ? S.ring[src & RMASK] : __builtin_nontemporal_load(O.rd(src))) : 0;
      }
#pragma unroll
      for (int j = 0; j < 5; j++) {
        const uint32_t i = (uint32_t)lane + 64u * j;
        if (i < flen) S.ring[(F + i) & RMASK] = v[j];
      }
    }
    if (lm && lane == __builtin_ctzll(lm)) pending = false;
    ready = ready && mlen <= 32;
    const bool in_ring = msrc + RING >= batch_end;
#if ZG_INFLATE_XW == 8
    if (ready && in_ring && mlen <= 8) {
      // a short match whose source is in the ring (99 % of C3's): the 8 bytes from the source start
      // as two byte-aligned words of three aligned ring reads, byte k of the copy = source byte
      // k mod d (an overlapping copy repeats its period); 8 unconditional byte stores, the ones past
      // the match's length into a sink byte (no exec-mask branches)
      const uint32_t a0 = (uint32_t)(msrc >> 2), sh = (uint32_t)(msrc & 3);
      const uint32_t w0 = S.ring32[a0 & (RING / 4 - 1)], w1 = S.ring32[(a0 + 1) & (RING / 4 - 1)],
                     w2 = S.ring32[(a0 + 2) & (RING / 4 - 1)];
      const uint64_t V = ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
      uint32_t r = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        uint8_t *dst = k < mlen ? &S.ring[(mypos + k) & RMASK] : &S.sink[0];
        *dst = (uint8_t)(V >> (8 * r));
        r = r + 1 == md ? 0u : r + 1;
      }
      pending = false;
    } else
#elif ZG_INFLATE_XW
    if (ready && in_ring && md >= mlen && mlen <= ZG_INFLATE_XW) {
      // a short source wholly in the ring, not overlapping the copy: aligned ring words (all
      // loads in flight together), byte-aligned in registers
      const uint32_t a0 = (uint32_t)(msrc >> 2), sh = (uint32_t)(msrc & 3), nw = (sh + mlen + 3) >> 2;
      uint32_t w[ZG_INFLATE_XW / 4 + 1];
#pragma unroll
      for (uint32_t j = 0; j <= ZG_INFLATE_XW / 4; j++) w[j] = j < nw ? S.ring32[(a0 + j) & (RING / 4 - 1)] : 0u;
#pragma unroll
      for (uint32_t j = 0; j < ZG_INFLATE_XW / 4; j++) {
        const uint32_t v = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          if (4 * j + k < mlen) S.ring[(mypos + 4 * j + k) & RMASK] = (uint8_t)(v >> (8 * k));
      }
      pending = false;
    } else
#endif
    if (ready) {
      // byte i of the copy takes source byte i mod d: the remainder advanced per byte (no division)
      uint32_t r = 0;
      for (uint32_t i0 = 0; i0 < mlen; i0 += 4) {
        uint8_t v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t i = i0 + k;
          const uint64_t src = msrc + r;
          v[k] = (i < mlen) ? (in_ring ? S.ring[src & RMASK] : __builtin_nontemporal_load(O.rd(src))) : 0;
          r = r + 1 == md ? 0u : r + 1;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (i0 + k < mlen) S.ring[(mypos + i0 + k) & RMASK] = v[k];
      }
      pending = false;
    }
  }
#else
  // Matches resolve in rounds: every pending match whose source lies entirely before the first
  // pending match (or that IS the first one) copies its bytes itself; dest byte i takes source
  // byte msrc + (i mod d), which is always final, so a lane's copy has no inner dependency.
  bool pending = is_match;
  uint64_t pm;
  XPROF(6, 1);
  XPROF(7, cnt);
  while ((pm = __ballot(pending)) != 0) {
    XPROF(5, 1);
    const int first = __builtin_ctzll(pm);
    const uint32_t F_lo = __builtin_amdgcn_readlane((uint32_t)mypos, first);
    const uint32_t F_hi = __builtin_amdgcn_readlane((uint32_t)(mypos >> 32), first);
    const uint64_t F = ((uint64_t)F_hi << 32) | F_lo;
    const uint32_t flen = __builtin_amdgcn_readlane(mlen, first);
    if (flen > 32) {  // a long match: copied by the whole wave once it is the first pending
      const uint32_t fd = __builtin_amdgcn_readlane(md, first);
      const float inv = 1.0f / (float)fd;
      for (uint32_t i = lane; i < flen; i += 64) {
        uint32_t q = (uint32_t)((float)i * inv);
        int32_t rm = (int32_t)i - (int32_t)(q * fd);
        if (rm < 0) rm += fd;
        if (rm >= (int32_t)fd) rm -= fd;
        const uint64_t src = F - fd + (uint32_t)rm;
        const uint8_t v = (src + RING >= batch_end) ? S.ring[src & RMASK] : __builtin_nontemporal_load(O.rd(src));
        S.ring[(F + i) & RMASK] = v;
      }
      if (lane == first) pending = false;
      continue;
    }
    const bool ready = pending && mlen <= 32 && (lane == first || msrc + mlen <= F);
    const bool in_ring = msrc + RING >= batch_end;
#if ZG_INFLATE_XW == 8
    if (ready && in_ring && mlen <= 8) {
      // a short match whose source is in the ring (99 % of C3's): the 8 bytes from the source start
      // as two byte-aligned words of three aligned ring reads, byte k of the copy = source byte
      // k mod d (an overlapping copy repeats its period); 8 unconditional byte stores, the ones past
      // the match's length into a sink byte (no exec-mask branches)
      const uint32_t a0 = (uint32_t)(msrc >> 2), sh = (uint32_t)(msrc & 3);
      const uint32_t w0 = S.ring32[a0 & (RING / 4 - 1)], w1 = S.ring32[(a0 + 1) & (RING / 4 - 1)],
                     w2 = S.ring32[(a0 + 2) & (RING / 4 - 1)];
      const uint64_t V = ((uint64_t)__builtin_amdgcn_alignbyte(w2, w1, sh) << 32) | __builtin_amdgcn_alignbyte(w1, w0, sh);
      uint32_t r = 0;
#pragma unroll
      for (uint32_t k = 0; k < 8; k++) {
        uint8_t *dst = k < mlen ? &S.ring[(mypos + k) & RMASK] : &S.sink[0];
        *dst = (uint8_t)(V >> (8 * r));
        r = r + 1 == md ? 0u : r + 1;
      }
      pending = false;
    } else
#elif ZG_INFLATE_XW
    if (ready && in_ring && md >= mlen && mlen <= ZG_INFLATE_XW) {
      // a short source wholly in the ring, not overlapping the copy: aligned ring words (all
      // loads in flight together), byte-aligned in registers
      const uint32_t a0 = (uint32_t)(msrc >> 2), sh = (uint32_t)(msrc & 3), nw = (sh + mlen + 3) >> 2;
      uint32_t w[ZG_INFLATE_XW / 4 + 1];
#pragma unroll
      for (uint32_t j = 0; j <= ZG_INFLATE_XW / 4; j++) w[j] = j < nw ? S.ring32[(a0 + j) & (RING / 4 - 1)] : 0u;
#pragma unroll
      for (uint32_t j = 0; j < ZG_INFLATE_XW / 4; j++) {
        const uint32_t v = __builtin_amdgcn_alignbyte(w[j + 1], w[j], sh);
#pragma unroll
        for (uint32_t k = 0; k < 4; k++)
          if (4 * j + k < mlen) S.ring[(mypos + 4 * j + k) & RMASK] = (uint8_t)(v >> (8 * k));
      }
      pending = false;
    } else
#endif
    if (ready) {
      // byte i of the copy takes source byte i mod d: the remainder advanced per byte (no division)
      uint32_t r = 0;
      for (uint32_t i0 = 0; i0 < mlen; i0 += 4) {
        uint8_t v[4];
#pragma unroll
        for (int k = 0; k < 4; k++) {
          const uint32_t i = i0 + k;
          const uint64_t src = msrc + r;
          v[k] = (i < mlen) ? (in_ring ? S.ring[src & RMASK] : __builtin_nontemporal_load(O.rd(src))) : 0;
          r = r + 1 == md ? 0u : r + 1;
        }
#pragma unroll
        for (int k = 0; k < 4; k++)
          if (i0 + k < mlen) S.ring[(mypos + i0 + k) & RMASK] = v[k];
      }
      pending = false;
    }
  }
#endif
  pos = batch_end;
  if (pos - flushed >= FLUSH_MIN) {
    wsync();
    flush(S, O, cap, flushed, pos);
    flushed = pos;
    wsync();
  }
  return true;
}
#undef XPROF

}  // namespace

#ifndef ZG_INFLATE_WPE
#define ZG_INFLATE_WPE 5
#endif
// One wave per item. gzip (ZLIB = false, RFC 1952): the trailer's CRC-32 and ISIZE are checked here
// (gzip_codec.rs:110-120: flate2's GzDecoder fails on a mismatch); aux is unused.
// zlib (ZLIB = true, RFC 1950; blosc's zlib streams, c-blosc zlib_wrap_decompress = zlib uncompress):
// only items whose kind is BL_KIND_ZLIB and status BL_SKIP; aux[i] = {Adler-32, 0}, status 0 on
// success (the Adler-32 check follows in k_adler32_check).
template <bool ZLIB, bool PIPE = false>
__global__ __launch_bounds__(PIPE ? 128 : 64) __attribute__((amdgpu_waves_per_eu(PIPE ? 4 : ZG_INFLATE_WPE, 8))) void k_gzip(
    ZgItem *items, uint32_t *status, const uint32_t *kind, uint8_t *dst, uint64_t slot_bytes, uint2 *aux,
    const uint32_t *order, uint32_t *seg_scr, int crc_tail, GzDirect gd) {
  static_assert(!(ZLIB && PIPE), "the pipelined mode is for gzip streams");
  __shared__ std::conditional_t<PIPE, SmemP, Smem> S;
#if !ZG_INFLATE_XFETCH
  __shared__ uint16_t seg_base[65], seg_skip[64];
#endif
  PROF_DECL;
  PROF_T(t_all);
  const uint32_t item = order ? order[blockIdx.x] : blockIdx.x;
  if (ZLIB ? (kind[item] != BL_KIND_ZLIB || status[item] != BL_SKIP) : status[item] != 0) return;
  const ZgItem it = items[item];
  if (it.flags & ZG_ITEM_FILL) return;
  const int lane = lane_id();
  uint8_t *out = dst + (uint64_t)item * slot_bytes;
  const uint64_t cap = slot_bytes;
  OutMap O;
  O.slot = O.base = out;
  O.cfg = O.want = 0;
  O.o0 = O.o1 = 0;
  if (!ZLIB && gd.dout && !(it.flags & ZG_ITEM_PARTIAL)) {
    // a whole chunk on 16-B aligned output rows: decoded straight into the array (GzDirect)
    const uint32_t nd = gd.nd;
    const uint64_t *g = gd.geom + (uint64_t)item * 3 * nd;
    bool whole = true;
    uint64_t off = 0;
    for (uint32_t d = 0; d < nd; d++) {
      whole = whole && g[d] == 0 && g[nd + d] == gd.cshape[d];
      off += g[2 * nd + d] * gd.ostr[d];
    }
    uint8_t *b = gd.dout + off;
    if (whole && ((uintptr_t)b & 15) == 0) {
      // rows: nd 1 one row; nd 2 row index r -> r * ostr[0]; nd 3 (r mod n1) * ostr[1] + (r / n1) * ostr[0]
      O.base = b;
      const uint32_t sh = nd == 3 ? (uint32_t)__builtin_ctzll(gd.cshape[1]) : 31u;
      O.o0 = nd == 3 ? (uint32_t)gd.ostr[1] : nd == 2 ? (uint32_t)gd.ostr[0] : 0u;
      O.o1 = nd == 3 ? (uint32_t)gd.ostr[0] : 0u;
      O.cfg = 0x80000000u | gd.lbs | (sh << 8);
      O.want = (uint32_t)gd.want;
    }
  }
  const uint8_t *in = (const uint8_t *)it.src;
  uint64_t in_len = it.len;
  // The crc32c codec after gzip (C3's inner chain [bytes, gzip, crc32c]; crc32c_codec.rs:108-141)
  // folded into the pipelined kernel: the stream's last 4 bytes are its CRC-32C, which wave 1 checks
  // while wave 0 parses the first block header (crc_tail 1; 2: stripped, not verified).
  if ((PIPE || crc_tail == 3) && crc_tail) {  // crc_tail 3 (one-wave kernel): stripped, verified beside it
    if (in_len < 4) {
      if (lane == 0) status[item] = ZG_CRC_INPUT_TOO_SHORT;
      return;
    }
    in_len -= 4;
  }
  uint32_t err = 0;
  uint64_t hp;
  if (ZLIB) {
    // ---- RFC 1950 header: CM 8, CINFO <= 7, FCHECK, no preset dictionary (zlib: Z_NEED_DICT) ----
    hp = 2;
    if (in_len < 7) {
      err = ZG_CORRUPT_STREAM;
    } else {
      const uint32_t cmf = U(in[0]), flg = U(in[1]);
      if ((cmf & 15) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20)) err = ZG_CORRUPT_STREAM;
    }
  } else {
    // ---- RFC 1952 header (uniform byte reads) ----
    hp = 10;
    if (in_len < 18) err = ZG_CORRUPT_STREAM;
    uint32_t flg = 0;
    if (!err) {
      if (U(in[0]) != 0x1f || U(in[1]) != 0x8b || U(in[2]) != 8) err = ZG_CORRUPT_STREAM;
      flg = U(in[3]);
      if (flg & 0xE0) err = ZG_CORRUPT_STREAM;  // reserved flag bits
    }
    if (!err && (flg & 4)) {  // FEXTRA
      const uint32_t xlen = U(in[hp]) | (U(in[hp + 1]) << 8);  // hp + 2 <= 18 <= in_len
      hp += 2 + xlen;
      if (hp > in_len) err = ZG_CORRUPT_STREAM;
    }
    if (!err && (flg & 8)) {  // FNAME
      while (hp < in_len && U(in[hp]) != 0) hp++;
      hp++;
    }
    if (!err && (flg & 16)) {  // FCOMMENT
      while (hp < in_len && U(in[hp]) != 0) hp++;
      hp++;
    }
    if (!err && (flg & 2)) hp += 2;  // FHCRC
    if (!err && hp + 8 > in_len) err = ZG_CORRUPT_STREAM;
  }
  if (err) {
    if constexpr (PIPE) {
      // the chain decodes crc32c before gzip (crc32c_codec.rs:108-141): a stream whose CRC-32C fails
      // is INVALID_CHECKSUM even when its gzip header is corrupt too, as with k_crc32c_strip. Wave 0
      // checks it here (wave 1 has not split off yet and returns).
      if (crc_tail == 1 && !(it.flags & ZG_ITEM_PARTIAL)) {
        if (threadIdx.x >= 64) return;
        wave_crc_tables(S.c32c, POLY_CRC32C);
        const uint32_t c = wave_crc(in, in_len, S.c32c, POLY_CRC32C);
        const uint32_t st = U(in[in_len]) | (U(in[in_len + 1]) << 8) | (U(in[in_len + 2]) << 16) |
                            (U(in[in_len + 3]) << 24);
        if (c != st) err = ZG_INVALID_CHECKSUM;
      }
    }
    if (lane == 0 && threadIdx.x < 64) status[item] = err;
    return;
  }

  // ---- bit reader over the aligned stream ----
  Bits B;
  const uintptr_t mis = (uintptr_t)in & 3;
  B.base = (const uint32_t *)((uintptr_t)in - mis);
  B.nwords = (uint32_t)((in_len + mis + 3) / 4);
  const uint64_t end_bits = (in_len + mis) * 8;
  bits_seek(B, (hp + mis) * 8);

  uint64_t pos = 0;        // output bytes produced (absolute)
  uint64_t flushed = 0;    // output bytes flushed to the slot
  bool last = false;
  // pipelined mode: the message protocol (every message one workgroup barrier; a sync takes two more)
  uint32_t pm = 0;    // messages wave 0 has posted
  bool held = false;  // wave 0 holds the output state (between dsync and drelease)
  auto post = [&](uint32_t msg) {
    if constexpr (PIPE) {
      if (lane == 0) S.p_msg[pm & 1] = msg;
      __threadfence_block();
      __syncthreads();
      pm++;
    }
  };
  auto dsync = [&]() {  // take the output state from wave 1 (it finishes its round first)
    if constexpr (PIPE) {
      post(P_SYNC);
      __syncthreads();  // wave 1 has written it
      pos = S.p_pos;
      flushed = S.p_flushed;
      if (!err) err = S.p_err;
      held = true;
    }
  };
  auto drelease = [&]() {  // hand it back
    if constexpr (PIPE) {
      if (lane == 0) {
        S.p_pos = pos;
        S.p_flushed = flushed;
        S.p_err = err;
      }
      __threadfence_block();
      __syncthreads();
      held = false;
    }
  };
  if constexpr (PIPE) {
    if (threadIdx.x == 0) {
      S.p_msg[0] = S.p_msg[1] = P_END;
      S.p_crc_bad = 0;
    }
    __syncthreads();
    if (threadIdx.x >= 64) {
      // ---- wave 1: the stream's CRC-32C, then the executor of wave 0's rounds ----
      if (crc_tail == 1 && !(it.flags & ZG_ITEM_PARTIAL)) {
        wave_crc_tables(S.c32c, POLY_CRC32C);
        const uint32_t c = wave_crc(in, in_len, S.c32c, POLY_CRC32C);
        const uint32_t st = U(in[in_len]) | (U(in[in_len + 1]) << 8) | (U(in[in_len + 2]) << 16) |
                            (U(in[in_len + 3]) << 24);
        if (lane == 0 && c != st) S.p_crc_bad = 1;
      }
      uint64_t xpos = 0, xfl = 0;
      uint32_t xerr = 0;
      const uint32_t *rbase = seg_scr + (uint64_t)blockIdx.x * 2 * 64 * SEGCAP;
      for (uint32_t m = 0;; m++) {
        __syncthreads();  // wave 0's next message
        const uint32_t slot = m & 1, msg = S.p_msg[slot];
        if (msg == P_END) break;
        if (msg == P_SYNC) {
          if (lane == 0) {
            S.p_pos = xpos;
            S.p_flushed = xfl;
            S.p_err = xerr;
          }
          __threadfence_block();
          __syncthreads();  // wave 0 takes the output state
          __syncthreads();  // and hands it back
          xpos = S.p_pos;
          xfl = S.p_flushed;
          xerr = S.p_err;
          continue;
        }
        if (xerr) continue;
        const uint32_t total = S.p_total[slot];
        const uint32_t rb_l = S.p_rb[slot][lane], ro_l = S.p_ro[slot][lane], cnt_l = S.p_cnt[slot][lane];
        const uint32_t *wrec = rbase + (uint64_t)slot * 64 * SEGCAP;
        auto fetch = [&](uint32_t g) -> uint32_t {
          const uint64_t has = __ballot(cnt_l != 0 && rb_l <= g);
          const int k0 = has ? 63 - __builtin_clzll(has) : 0;
          uint32_t rb = U(__builtin_amdgcn_readlane((int)rb_l, k0));
          uint32_t ro = U(__builtin_amdgcn_readlane((int)ro_l, k0));
          uint64_t st = __ballot(cnt_l != 0 && rb_l > g && rb_l < g + 64);
          while (st) {
            const int k = __builtin_ctzll(st);
            st &= st - 1;
            const uint32_t b = U(__builtin_amdgcn_readlane((int)rb_l, k));
            const uint32_t o = U(__builtin_amdgcn_readlane((int)ro_l, k));
            if (g + (uint32_t)lane >= b) {
              rb = b;
              ro = o;
            }
          }
          const uint32_t idx = g + (uint32_t)lane;
          return idx < total ? wrec[ro + (idx - rb)] : 0u;
        };
        uint32_t rec_next = total ? fetch(0) : 0u;
        for (uint32_t g = 0; g < total && !xerr;) {
          const uint32_t idx = g + (uint32_t)lane;
          const uint32_t rec = rec_next;
          const uint32_t ln = idx < total ? ((rec >> 31) ? (rec & 511) : 1u) : 0u;
          const uint32_t inc = wave_incl_sum(ln);
          const bool take = idx < total && inc - ln < (uint32_t)BATCH_CAP;
          const uint32_t bc = (uint32_t)__builtin_popcountll(__ballot(take));
          const uint32_t bytes = U(__builtin_amdgcn_readlane((int)inc, (int)bc - 1));
          if (xpos + bytes > cap) {
            xerr = ZG_DECODED_SIZE_MISMATCH;
            break;
          }
          if (g + bc < total) rec_next = fetch(g + bc);  // in flight while this batch executes
          if (!exec_batch(S, O, cap, xpos, xfl, bc, bytes, rec, nullptr)) xerr = ZG_CORRUPT_STREAM;
          g += bc;
        }
      }
      return;
    }
  }
  while (!last && !err) {
    PROF_T(t_hdr);
    bits_refill(B);
    last = bits_get(B, 1);
    const uint32_t type = bits_get(B, 2);
    if (type == 0) {  // ---- stored block ----
      if (PIPE && !held) dsync();  // wave 0 writes the block's bytes itself
      const uint32_t r = (uint32_t)(B.consumed & 7);
      bits_drop(B, r ? 8 - r : 0);  // to a byte boundary (nb is a multiple of 8 here)
      bits_refill(B);
      const uint32_t ln = bits_get(B, 16), nln = bits_get(B, 16);
      if ((ln ^ 0xFFFF) != nln) { err = ZG_CORRUPT_STREAM; break; }
      const uint64_t byte0 = B.consumed / 8 - mis;  // byte offset in `in`
      if (byte0 + ln > in_len) { err = ZG_CORRUPT_STREAM; break; }
      if (pos + ln > cap) { err = ZG_DECODED_SIZE_MISMATCH; break; }
      for (uint32_t done = 0; done < ln;) {
        const uint32_t n = min<uint32_t>(ln - done, BATCH_CAP);
        for (uint32_t k = lane; k < n; k += 64) S.ring[(pos + k) & RMASK] = in[byte0 + done + k];
        wsync();
        flush(S, O, cap, flushed, pos + n);
        pos += n;
        flushed = pos;
        done += n;
        wsync();
      }
      bits_seek(B, (byte0 + ln + mis) * 8);
      if (PIPE) drelease();
      continue;
    }
    if (type == 3) { err = ZG_CORRUPT_STREAM; break; }
    uint32_t hlit = 288, hdist = 32;
    if (type == 1) {
      build_fixed_lens(S.lens);
    } else {  // ---- dynamic header ----
      PROF_T(t_cl);
      hlit = bits_get(B, 5) + 257;
      hdist = bits_get(B, 5) + 1;
      const uint32_t hclen = bits_get(B, 4) + 4;
      if (hlit > 286 || hdist > 30) { err = ZG_CORRUPT_STREAM; break; }
      if (lane < 20) S.clens[lane] = 0;
      wsync();
      for (uint32_t k = 0; k < hclen; k++) {  // (a private array indexed by k would live in scratch)
        const uint32_t v = bits_get(B, 3);
        if (lane == 0) S.clens[c_clen_order[k]] = (uint8_t)v;
      }
      wsync();
      if (!build_table(S.clens, 19, 7, S.ltab, S.csorted, S.cm, 2, S.tmp, 0)) { err = ZG_CORRUPT_STREAM; break; }
      // code lengths for literal/length + distance alphabets (ltab used as a 128-entry 7-bit table)
      uint32_t n = 0, prev = 0;
      const uint32_t total = hlit + hdist;
#if ZG_INFLATE_PCL
      // Lane-parallel, as the lookahead symbol decode: lane l decodes the code-length symbol (code +
      // repeat bits, <= 14 bits) that would start at bit bp + l of a 63-bit window, the window's
      // symbols are chained by pointer jumping, their runs placed by a prefix sum and written at
      // once; a repeat-previous code (16) takes the value of the last explicit length before it
      // (a ballot mask, not a scan). ~10 windows per header instead of ~150 dependent steps.
      {
        uint64_t bp = B.consumed;
        bool have = false;  // a length was decoded before (16 needs one: zlib "invalid bit length repeat")
        while (n < total && !err) {
          uint32_t W0, W1, W2, W3, W4;
          bits_words(B, (uint32_t)(bp >> 5), W0, W1, W2, W3, W4);
          const uint32_t bit = (uint32_t)(bp & 31) + (uint32_t)lane;
          const uint32_t wi = bit >> 5;
          const uint32_t a0 = wi == 0 ? W0 : (wi == 1 ? W1 : W2);
          const uint32_t a1 = wi == 0 ? W1 : (wi == 1 ? W2 : W3);
          const uint32_t a2 = wi == 0 ? W2 : (wi == 1 ? W3 : W4);
          const uint32_t lo = __builtin_amdgcn_alignbit(a1, a0, bit & 31), hi = __builtin_amdgcn_alignbit(a2, a1, bit & 31);
          const uint32_t e = S.ltab[lo & 127];
          const uint32_t L = e & 15, sym = e >> 16;
          const uint32_t xb = sym == 16 ? 2u : (sym == 17 ? 3u : (sym == 18 ? 7u : 0u));
          const uint32_t xv = (uint32_t)((((uint64_t)hi << 32) | lo) >> L) & ((1u << xb) - 1u);
          const uint32_t adv = L + xb;
          const uint32_t rep = sym < 16 ? 1u : (sym == 18 ? 11u : 3u) + xv;
          // pointer jumping: p = the offset of this lane's (t-th) symbol in the window
          uint32_t J = lane == 63 ? 63u : min<uint32_t>((uint32_t)lane + adv, 63u);
          uint32_t p = (lane & 1) ? U(__builtin_amdgcn_readlane(J, 0)) : 0u;
#pragma unroll
          for (int k = 1; k <= 4; k++) {
            J = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(J << 2), (int)J);
            const uint32_t q = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(p << 2), (int)J);
            if ((lane >> k) & 1) p = q;
          }
          const uint32_t sym_t = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(p << 2), (int)sym);
          const uint32_t rep_t = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(p << 2), (int)rep);
          const uint32_t adv_t = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(p << 2), (int)adv);
          const bool valid = p < 63 && lane < 32;
          const uint32_t r = valid ? rep_t : 0u;
          const uint32_t incl = wave_incl_sum(r), excl = incl - r;
          const bool take = valid && excl < total - n;
          const uint64_t tm = __ballot(take);
          const uint32_t m = (uint32_t)__builtin_popcountll(tm);
          if (!m) {  // no symbol fits the window: a corrupt stream
            err = ZG_CORRUPT_STREAM;
            break;
          }
          // the value a symbol writes: its length (< 16), 0 (17, 18), or the last explicit one (16)
          const uint64_t expl = __ballot(take && sym_t != 16);
          const uint64_t upto = expl & (lane == 63 ? ~0ull : ((2ull << lane) - 1));
          const int src = upto ? 63 - __builtin_clzll(upto) : -1;
          const uint32_t own = sym_t < 16 ? sym_t : 0u;
          const uint32_t from = (uint32_t)__builtin_amdgcn_ds_bpermute((int)((src < 0 ? 0 : src) << 2), (int)own);
          if (__ballot(take && sym_t == 16 && src < 0 && !have)) {
            err = ZG_CORRUPT_STREAM;
            break;
          }
          const uint32_t val = src < 0 ? prev : from;
          const uint32_t last = m - 1;
          const uint32_t n_new = n + U(__builtin_amdgcn_readlane(incl, (int)last));
          if (n_new > total) {  // a run past the last length
            err = ZG_CORRUPT_STREAM;
            break;
          }
          if (take)
            for (uint32_t k = 0; k < r; k++) {
              const uint32_t si = n + excl + k;
              S.lens[si < hlit ? si : 288 + (si - hlit)] = (uint8_t)val;
            }
          if (expl) {
            const int hs = 63 - __builtin_clzll(expl);
            prev = U(__builtin_amdgcn_readlane(own, hs));
          }
          have = true;
          n = n_new;
          bp += U(__builtin_amdgcn_readlane(p, (int)last)) + U(__builtin_amdgcn_readlane(adv_t, (int)last));
          if (bp > end_bits) err = ZG_CORRUPT_STREAM;
        }
        if (!err) bits_seek_in(B, bp);
        wsync();
      }
#else
      while (n < total) {
        bits_refill(B);
        const uint32_t e = U(S.ltab[bits_peek(B, 7)]);
        bits_drop(B, e & 15);
        const uint32_t sym = e >> 16;
        uint32_t rep = 0, val = 0;
        if (sym < 16) {
          val = sym;
          rep = 1;
          prev = sym;
        } else if (sym == 16) {
          if (n == 0) { err = ZG_CORRUPT_STREAM; break; }
          val = prev;
          rep = 3 + bits_get(B, 2);
        } else if (sym == 17) {
          rep = 3 + bits_get(B, 3);
          val = 0;
          prev = 0;
        } else {
          rep = 11 + bits_get(B, 7);
          val = 0;
          prev = 0;
        }
        if (n + rep > total) { err = ZG_CORRUPT_STREAM; break; }
        for (uint32_t k = lane; k < rep; k += 64) {
          const uint32_t s = n + k;
          S.lens[s < hlit ? s : 288 + (s - hlit)] = (uint8_t)val;
        }
        n += rep;
      }
#endif
      if (err) break;
      // zero the unused tails so the table builders see exactly hlit / hdist symbols
      for (uint32_t s = lane; s < 320; s += 64) {
        if ((s >= hlit && s < 288) || s >= 288 + hdist) S.lens[s] = 0;
      }
      wsync();
      if (U(S.lens[256]) == 0) { err = ZG_CORRUPT_STREAM; break; }  // missing end-of-block code
      PROF_ADD(8, t_cl);
    }
    PROF_T(t_lt);
    if (!build_table(S.lens, 288, LROOT, S.ltab, S.lsorted, S.lm, 0, S.tmp, LSUB)) { err = ZG_CORRUPT_STREAM; break; }
    PROF_ADD(9, t_lt);
    PROF_T(t_dt);
    if (!build_table(S.lens + 288, 32, DROOT, S.dtab, S.dsorted, S.dm, 1, S.tmp, DSUB)) { err = ZG_CORRUPT_STREAM; break; }
    PROF_ADD(10, t_dt);
    PROF_CNT(12, 1);  // blocks
    PROF_ADD(0, t_hdr);
    (void)hlit;
    (void)hdist;

    bool eob = false;
#if ZG_INFLATE_SEG
    // ---- segmented rounds: lane l decodes the stream region [r0 + l*SEGB, r0 + (l+1)*SEGB) serially,
    // starting OVL bits early so that its chain has met the true one by then (Huffman codes
    // self-synchronise); lane l is right once the true chain's exit from lane l-1's region is a
    // symbol start on its own chain (else it re-decodes from that exit). The region records then
    // run through the batch executor in order. A code past the subtable space ends the path (the
    // lookahead loop below takes the rest of the block).
    if (seg_scr) {
      if (PIPE && held) drelease();  // wave 1 executes this block's rounds
      LaneRd R{B.base, B.nwords, 0, 0, 0, 0, 0, 0, 0, 0};
      uint64_t r0 = B.consumed;
      bool fallback = false;
      while (!eob && !err && !fallback) {
        // this round's record slots (pipelined: the message slot's half of the stream's two)
        uint32_t *myrec = seg_scr + ((uint64_t)blockIdx.x * (PIPE ? 128 : 64) + (PIPE ? (pm & 1) * 64 : 0) +
                                     (uint32_t)lane) * SEGCAP;
        PROF_T(t_sd);
        const uint64_t s_own = r0 + (uint64_t)lane * SEGB, s_end = s_own + SEGB;
        uint64_t p = lane ? s_own - OVL : r0;
        uint32_t n;
        uint64_t mask;
        uint32_t st = seg_decode(S, R, p, s_own, s_end, end_bits, myrec, n, mask);
        PROF_CNT(13, 1);  // rounds
        PROF_T(t_rep);
        uint32_t skip = 0;
        bool ok = lane == 0;
        bool repaired = false;
        // the valid prefix: lane l is right when lane l-1 is and ended at the end of its region at
        // a symbol start of lane l's chain; out-of-sync lanes are re-decoded from that exit
        for (int rep = 0;; rep++) {
          const uint64_t e = shfl_up64(p);
          const uint32_t stp = (uint32_t)__shfl_up((int)st, 1, 64);
          if (lane && !repaired) {
            const uint64_t d = e - s_own;
            ok = stp == SG_END && e >= s_own && d < 64 && ((mask >> (uint32_t)d) & 1);
            skip = ok ? (uint32_t)__builtin_popcountll(mask & ((1ull << (uint32_t)d) - 1)) : 0u;
          }  // a repaired lane started at its predecessor's true exit: right (ok stays set)
          const uint64_t bad = __ballot(!ok);
          // every lane before the first bad one is right (the chain of checks)
          const int j = bad ? __builtin_ctzll(bad) : 64;
          if (j == 64) break;
          const uint32_t stj = (uint32_t)__builtin_amdgcn_readlane((int)st, j - 1);
          if (stj != SG_END || rep >= ZG_INFLATE_MAXREP) {
            if (lane >= j) ok = false;
            break;
          }
          if (lane == j) {  // re-decode from the true exit of lane j-1's region
            p = e;
            st = seg_decode(S, R, p, e, s_end, end_bits, myrec, n, mask);
            skip = 0;
            repaired = true;
            ok = true;
          }
          // the lanes after j re-check against the updated exits; the earlier ones stay right
          PROF_CNT(3, 1);
        }
        PROF_ADD(14, t_rep);
        // the round ends at the last valid lane
        const uint64_t vm = __ballot(ok);
        const int J = (vm == ~0ull) ? 64 : __builtin_ctzll(~vm);
        const uint32_t stl = (uint32_t)__builtin_amdgcn_readlane((int)st, J - 1);
        const uint64_t pl = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)(p >> 32), J - 1) << 32) |
                            (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)p, J - 1);
        // records of the valid lanes, in stream order: lane l's region holds the round's symbols
        // [rb_l, rb_l + cnt_l), its records start at word ro_l of the scratch
        const uint32_t cnt_l = (lane < J) ? n - skip : 0u;
        const uint32_t incl = wave_incl_sum(cnt_l);
        const uint32_t total = U(__builtin_amdgcn_readlane((int)incl, 63));
#if ZG_INFLATE_XFETCH
        const uint32_t rb_l = incl - cnt_l;
        const uint32_t ro_l = (uint32_t)lane * SEGCAP + skip;  // in this stream's 64 record slots
        if constexpr (PIPE) {
          // hand the round to wave 1 and decode the next one meanwhile
          const uint32_t slot = pm & 1;
          S.p_rb[slot][lane] = rb_l;
          S.p_ro[slot][lane] = ro_l;
          S.p_cnt[slot][lane] = cnt_l;
          if (lane == 0) S.p_total[slot] = total;
          post(P_ROUND);
        }
        const uint32_t *wrec = seg_scr + (uint64_t)blockIdx.x * 64 * SEGCAP;
        __threadfence_block();  // the records (global) before other lanes read them
        wsync();
        PROF_ADD(1, t_sd);
        PROF_T(t_sx);
        // The batch starting at symbol g: lane t takes symbol g + t. Its region comes from ballots over
        // the lane regions (the one holding g, then the few that start inside the batch: no LDS
        // search), and a batch's records are loaded while the previous batch executes.
        auto fetch = [&](uint32_t g) -> uint32_t {
          const uint64_t has = __ballot(cnt_l != 0 && rb_l <= g);
          const int k0 = has ? 63 - __builtin_clzll(has) : 0;
          uint32_t rb = U(__builtin_amdgcn_readlane((int)rb_l, k0));
          uint32_t ro = U(__builtin_amdgcn_readlane((int)ro_l, k0));
          uint64_t st = __ballot(cnt_l != 0 && rb_l > g && rb_l < g + 64);
          while (st) {  // the regions starting inside the batch, in stream order
            const int k = __builtin_ctzll(st);
            st &= st - 1;
            const uint32_t b = U(__builtin_amdgcn_readlane((int)rb_l, k));
            const uint32_t o = U(__builtin_amdgcn_readlane((int)ro_l, k));
            if (g + (uint32_t)lane >= b) {
              rb = b;
              ro = o;
            }
          }
          const uint32_t idx = g + (uint32_t)lane;
          return idx < total ? wrec[ro + (idx - rb)] : 0u;
        };
        uint32_t rec_next = (!PIPE && total) ? fetch(0) : 0u;
        for (uint32_t g = 0; !PIPE && g < total && !err;) {
          const uint32_t idx = g + (uint32_t)lane;
          const uint32_t rec = rec_next;
          const uint32_t ln = idx < total ? ((rec >> 31) ? (rec & 511) : 1u) : 0u;
#else
        seg_base[lane] = (uint16_t)(incl - cnt_l);
        seg_skip[lane] = (uint16_t)skip;
        if (lane == 63) seg_base[64] = (uint16_t)incl;
        __threadfence_block();  // the records (global) and bases (LDS) before other lanes read them
        wsync();
        PROF_ADD(1, t_sd);
        PROF_T(t_sx);
        for (uint32_t g = 0; g < total && !err;) {
          const uint32_t idx = g + (uint32_t)lane;
          uint32_t rec = 0, ln = 0;
          if (idx < total) {
            int k = 0;  // the lane region holding symbol idx: the last k with seg_base[k] <= idx
#pragma unroll
            for (int step = 32; step; step >>= 1)
              if (k + step < 64 && seg_base[k + step] <= idx) k += step;
            rec = seg_scr[((uint64_t)blockIdx.x * 64 + (uint32_t)k) * SEGCAP + seg_skip[k] + (idx - seg_base[k])];
            ln = (rec >> 31) ? (rec & 511) : 1u;
          }
#endif
          const uint32_t inc = wave_incl_sum(ln);
          const bool take = idx < total && inc - ln < (uint32_t)BATCH_CAP;
          const uint64_t tm = __ballot(take);
          const uint32_t bc = (uint32_t)__builtin_popcountll(tm);
          const uint32_t bytes = U(__builtin_amdgcn_readlane((int)inc, (int)bc - 1));
          if (pos + bytes > cap) {
            err = ZG_DECODED_SIZE_MISMATCH;
            break;
          }
          PROF_CNT(7, bc);
          PROF_CNT(6, 1);
#if ZG_INFLATE_XFETCH
          if (g + bc < total) rec_next = fetch(g + bc);  // in flight while this batch executes
#endif
#if ZG_EXP_NOEXEC  // lab experiment only (wrong output): records fetched and batched, not executed
          pos += bytes;
          if (__ballot(rec == 0xFFFFFFFFu)) err = ZG_CORRUPT_STREAM;
#elif defined(ZG_PROFILE)
          if (!exec_batch(S, O, cap, pos, flushed, bc, bytes, rec, prof_acc)) err = ZG_CORRUPT_STREAM;
#else
          if (!exec_batch(S, O, cap, pos, flushed, bc, bytes, rec, nullptr)) err = ZG_CORRUPT_STREAM;
#endif
          g += bc;
        }
        PROF_ADD(2, t_sx);
        if (err) break;
        if (stl == SG_EOB) {
          eob = true;
          bits_seek(B, pl);
        } else if (stl == SG_END || stl == SG_CAP) {
          r0 = pl;
        } else if (stl == SG_SLOW) {
          fallback = true;
          PROF_CNT(15, 1);  // blocks finished by the canonical slow path
          bits_seek(B, pl);
        } else {
          err = ZG_CORRUPT_STREAM;
        }
        wsync();
      }
      if (err) break;
      if (!fallback) continue;  // the block is done (its end-of-block code consumed)
    }
#endif
    // ---- symbol batches ----
    if (PIPE && !eob && !err && !held) dsync();  // wave 0 executes these batches itself
    while (!eob && !err) {
      PROF_T(t_dec);
      uint32_t cnt = 0, bytes = 0;
      uint64_t bp = B.consumed;  // absolute bit position of the next symbol
      while (cnt < 64 && bytes < BATCH_CAP && !eob && !err) {
        // Lane-parallel lookahead: lane l decodes a whole symbol (literal/length code, length extra
        // bits, distance code, distance extra bits: at most 36 bits with root-table codes) as if one
        // started at bit bp + l. The scalar walk then only chains the advances (one readlane per
        // symbol), and the symbols on the chain are compacted into the batch's record array.
        uint32_t W0, W1, W2, W3, W4;
        bits_words(B, (uint32_t)(bp >> 5), W0, W1, W2, W3, W4);
        const uint32_t bit = (uint32_t)(bp & 31) + (uint32_t)lane;
        const uint32_t wi = bit >> 5;
        const uint32_t a0 = wi == 0 ? W0 : (wi == 1 ? W1 : W2);
        const uint32_t a1 = wi == 0 ? W1 : (wi == 1 ? W2 : W3);
        const uint32_t a2 = wi == 0 ? W2 : (wi == 1 ? W3 : W4);
        uint32_t info, rec;
        lane_symbol(S, __builtin_amdgcn_alignbit(a1, a0, bit & 31), __builtin_amdgcn_alignbit(a2, a1, bit & 31), info, rec);
#if ZG_INFLATE_PJ
        // Chain the window's symbols by pointer jumping, with no per-symbol scalar work: J_k(x) is
        // the bit offset 2^k symbols after offset x (64: past the window, or after a stop symbol);
        // lane t composes the J_k of the bits of t into p = the offset of the window's t-th symbol,
        // then gathers that symbol. Output offsets are a wave prefix sum; the batch caps (64
        // symbols, BATCH_CAP bytes) cut a prefix, as the scalar walk did.
        bool slow = false;
        uint32_t o = 0;
        {
          // symbol starts 0..62 of the window; lane 63 is the sink (J = 63 maps to itself), standing
          // for "past the window" and "after a stop symbol", so the gathers need no range checks
          uint32_t J = (lane == 63 || info >= F_EOB) ? 63u : min<uint32_t>((uint32_t)lane + (info & 255), 63u);
          uint32_t p = (lane & 1) ? U(__builtin_amdgcn_readlane(J, 0)) : 0u;
#pragma unroll
          for (int k = 1; k <= ZG_INFLATE_PJL; k++) {
            J = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(J << 2), (int)J);
            const uint32_t q = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(p << 2), (int)J);
            if ((lane >> k) & 1) p = q;
          }
          const uint32_t info_t = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(p << 2), (int)info);
          const uint32_t rec_t = (uint32_t)__builtin_amdgcn_ds_bpermute((int)(p << 2), (int)rec);
          constexpr uint32_t NS = 2u << ZG_INFLATE_PJL;  // symbols a window can chain
          const bool valid = p < 63 && info_t < F_EOB && (uint32_t)lane < NS;
          const uint32_t olen = valid ? info_t >> 8 : 0u;
          const uint32_t incl = wave_incl_sum(olen), excl = incl - olen;
          const bool take = valid && cnt + (uint32_t)lane < 64 && bytes + excl < BATCH_CAP;
          const uint32_t m = (uint32_t)__builtin_popcountll(__ballot(take));
          if (take) S.rec[cnt + lane] = rec_t;
          if (m) {
            o = U(__builtin_amdgcn_readlane(p + (info_t & 255), (int)(m - 1)));
            bytes += U(__builtin_amdgcn_readlane(incl, (int)(m - 1)));
            cnt += m;
          }
          if (m < NS && cnt < 64 && bytes < BATCH_CAP) {
            const uint32_t pm = U(__builtin_amdgcn_readlane(p, (int)m));
            if (pm < 63) {  // symbol m starts in the window and is not valid: a stop symbol
              const uint32_t a = U(__builtin_amdgcn_readlane(info_t, (int)m));
              o = pm;
              if (a == (F_EOB | (a & 255))) {
                o += a & 255;
                eob = true;
              } else if (a & F_BAD) {
                err = ZG_CORRUPT_STREAM;
              } else {
                slow = true;
              }
            }
          }
        }
        bp += o;
#else
        uint64_t chain = 0;
        uint32_t o = 0, n = 0;
        bool slow = false;
        while (o < 64 && cnt + n < 64 && bytes < BATCH_CAP) {
          const uint32_t a = U(__builtin_amdgcn_readlane(info, o));
          if (a >= F_EOB) {
            if (a == (F_EOB | (a & 255))) {
              o += a & 255;
              eob = true;
            } else if (a & F_BAD) {
              err = ZG_CORRUPT_STREAM;
            } else {
              slow = true;
            }
            break;
          }
          chain |= 1ull << o;
          n++;
          bytes += a >> 8;
          o += a & 255;
        }
        if ((chain >> lane) & 1) S.rec[cnt + __builtin_amdgcn_mbcnt_hi((uint32_t)(chain >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)chain, 0u))] = rec;
        cnt += n;
        bp += o;
#endif
        if (slow && !err && cnt < 64 && bytes < BATCH_CAP) {
          // one symbol through the canonical slow path (codes longer than the root)
          bits_seek_in(B, bp);
          const uint32_t e = decode_sym(B, S.ltab, LROOT, S.lsorted, S.lm, 0);
          const uint32_t kind = (e >> 4) & 3;
          uint32_t r = 0;
          bool has = false;
          if (kind == K_LIT) {
            r = e >> 16;
            has = true;
            bytes++;
          } else if (kind == K_EOB) {
            eob = true;
          } else if (kind == K_BAD) {
            err = ZG_CORRUPT_STREAM;
          } else {
            bits_refill(B);
            const uint32_t lx = (e >> 6) & 15;
            const uint32_t len = (e >> 16) + bits_peek(B, lx);
            bits_drop(B, lx);
            const uint32_t de = decode_sym(B, S.dtab, DROOT, S.dsorted, S.dm, 1);
            if (((de >> 4) & 3) != K_LEN) {
              err = ZG_CORRUPT_STREAM;
            } else {
              bits_refill(B);
              const uint32_t dx = (de >> 6) & 15;
              const uint32_t dist = (de >> 16) + bits_peek(B, dx);
              bits_drop(B, dx);
              r = 0x80000000u | (dist << 9) | len;
              has = true;
              bytes += len;
            }
          }
          if (has) {
            if (lane == 0) S.rec[cnt] = r;
            cnt++;
          }
          bp = B.consumed;
        }
        if (bp > end_bits) err = ZG_CORRUPT_STREAM;  // ran past the input
      }
      bits_seek_in(B, bp);
      if (err) break;
      if (pos + bytes > cap) { err = ZG_DECODED_SIZE_MISMATCH; break; }
      // ---- execute the batch ----
      PROF_ADD(1, t_dec);
      PROF_T(t_exe);
      wsync();
#ifdef ZG_PROFILE
      if (!exec_batch(S, O, cap, pos, flushed, cnt, bytes, S.rec[lane], prof_acc)) { err = ZG_CORRUPT_STREAM; break; }
#else
      if (!exec_batch(S, O, cap, pos, flushed, cnt, bytes, S.rec[lane], nullptr)) { err = ZG_CORRUPT_STREAM; break; }
#endif
      PROF_ADD(2, t_exe);
    }
  }
  if constexpr (PIPE) {  // the output state back from wave 1, which then leaves
    if (!held) dsync();
    drelease();
    post(P_END);
    if (S.p_crc_bad) err = ZG_INVALID_CHECKSUM;  // the crc32c stage fails first, as in the chain order
  }
  if (!err && flushed < pos) {
    wsync();
    flush(S, O, cap, flushed, pos);
    flushed = pos;
  }
  if (!err) {
    const uint32_t r = (uint32_t)(B.consumed & 7);
    bits_drop(B, r ? 8 - r : 0);
    bits_refill(B);
    if (ZLIB) {  // trailer: Adler-32, big endian
      const uint32_t b0 = bits_get(B, 8), b1 = bits_get(B, 8), b2 = bits_get(B, 8), b3 = bits_get(B, 8);
      if (B.consumed > end_bits) err = ZG_CORRUPT_STREAM;
      if (lane == 0 && !err) aux[item] = make_uint2((b0 << 24) | (b1 << 16) | (b2 << 8) | b3, 0u);
    } else {  // trailer: CRC-32 then ISIZE (little endian), checked against the decoded stream
      const uint32_t crc_lo = bits_get(B, 16);
      const uint32_t crc_hi = bits_get(B, 16);
      const uint32_t isz_lo = bits_get(B, 16);
      const uint32_t isz_hi = bits_get(B, 16);
      const uint32_t crc = crc_lo | (crc_hi << 16), isz = isz_lo | (isz_hi << 16);
      if (B.consumed > end_bits) err = ZG_CORRUPT_STREAM;
      if (!err) {
        // The whole stream is in the slot (flushed by this wave: a workgroup-scope fence makes its
        // stores visible to its own loads); the Huffman tables' LDS holds the CRC tables now. 64
        // lanes, 2 KiB segments of a C3 chunk each: ~0.3 % of the stream's decode time, and no
        // second kernel re-reading every decoded byte.
        __threadfence_block();
        wsync();
        PROF_T(t_crc);
        wave_crc_tables(S.crc, POLY_CRC32);
#if ZG_GZ_DIRECT_READS
        const uint32_t c = wave_crc_map(O, pos, S.crc, POLY_CRC32);
#else
        const uint32_t c = wave_crc(out, pos, S.crc, POLY_CRC32);
#endif
        PROF_ADD(11, t_crc);
        if (c != crc || isz != (uint32_t)pos) err = ZG_CORRUPT_STREAM;
      }
    }
  }
  if (lane == 0) {
    if (err) {
      status[item] = err;
    } else {
      items[item].src = (uint64_t)out;
      items[item].len = pos;
      if (ZLIB) status[item] = 0;
      if (O.cfg >> 31) {  // in the array already: the scatter skips it (its size check is made here)
        if (pos != O.want) status[item] = ZG_DECODED_SIZE_MISMATCH;
        else items[item].flags = it.flags | ZG_ITEM_DIRECT;
      }
    }
  }
  PROF_ADD(4, t_all);
  PROF_FLUSH;
}

// LPT order of a one-wave-per-stream launch: the items by descending encoded length, so the longest
// streams are dispatched first and the launch's last round is made of the shortest ones (C3: 15,625
// streams on 5,120 resident waves). One workgroup, a counting sort on 1024 length buckets; failed
// and fill items go last.
__global__ __launch_bounds__(1024) void k_order_by_len(const ZgItem *items, const uint32_t *status, uint32_t n,
                                                       uint32_t *order) {
  __shared__ uint32_t cnt[1024];
  __shared__ uint32_t s_max;
  const uint32_t t = threadIdx.x;
  cnt[t] = 0;
  if (t == 0) s_max = 0;
  __syncthreads();
  auto len_of = [&](uint32_t i) -> uint32_t {
    const ZgItem it = items[i];
    if (status[i] || (it.flags & ZG_ITEM_FILL)) return 0;
    return it.len > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)it.len;
  };
  uint32_t m = 0;
  for (uint32_t i = t; i < n; i += 1024) m = max(m, len_of(i));
  atomicMax(&s_max, m);
  __syncthreads();
  uint32_t shift = 0;
  while ((s_max >> shift) >= 1024) shift++;
  for (uint32_t i = t; i < n; i += 1024) atomicAdd(&cnt[1023 - (len_of(i) >> shift)], 1u);
  __syncthreads();
  const uint32_t v = cnt[t];
  for (uint32_t off = 1; off < 1024; off <<= 1) {  // inclusive scan (Hillis-Steele)
    const uint32_t x = t >= off ? cnt[t - off] : 0;
    __syncthreads();
    cnt[t] += x;
    __syncthreads();
  }
  cnt[t] -= v;  // exclusive: the bucket's first slot
  __syncthreads();
  for (uint32_t i = t; i < n; i += 1024) order[atomicAdd(&cnt[1023 - (len_of(i) >> shift)], 1u)] = i;
}

// Batches of at most this many streams take the pipelined kernel (ZGPU_GZIP_PIPE_MAX; 0: never): a
// stream then costs two waves, one decoding the next round while the other executes this one, so its
// latency is the longer of the two instead of their sum - the time of a lone shard call.
// The record scratch is always sized for GZIP_PIPE_CAP; the environment (read per launch: tests run
// both kernels in one process) can only lower the threshold.
constexpr uint32_t GZIP_PIPE_CAP = 2048;
uint32_t gzip_pipe_max() {
  const char *e = std::getenv("ZGPU_GZIP_PIPE_MAX");
  return e ? (uint32_t)std::min<unsigned long>(std::strtoul(e, nullptr, 10), GZIP_PIPE_CAP) : GZIP_PIPE_CAP;
}

uint64_t gzip_seg_scratch_bytes(uint32_t n_items) {
  static const bool on = [] {
    const char *e = std::getenv("ZGPU_GZIP_SEG");
    return ZG_INFLATE_SEG && (!e || std::atoi(e) != 0);
  }();
  // the pipelined kernel double-buffers a stream's record slots
  const uint64_t slots = (uint64_t)n_items + std::min<uint64_t>(n_items, GZIP_PIPE_CAP);
  return on ? slots * 64 * SEGCAP * 4 : 0;
}

hipError_t launch_gzip(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                       uint32_t *order, uint32_t *seg_scr, hipStream_t s, int crc_tail, const GzDirect *direct,
                       const GzCrcFork *crc_fork) {
  const GzDirect gd = direct ? *direct : GzDirect{};
  if (!n_items) return hipSuccess;
  static const bool lpt = [] {
    const char *e = std::getenv("ZGPU_GZIP_LPT");
    return !e || std::atoi(e) != 0;
  }();
  if (!lpt || n_items < 2) order = nullptr;
  if (!gzip_seg_scratch_bytes(1)) seg_scr = nullptr;
  const bool pipe = seg_scr && n_items <= gzip_pipe_max();  // few streams: the pipelined latency mode
  // a trailing crc32c: checked inside the pipelined kernel (its second wave is idle at the start), by
  // k_crc32c_strip ahead of the one-wave kernel (inside it the check cost more HBM traffic: r05cal)
  int tail_mode = 0;  // what the one-wave kernel does with the trailing crc32c (3: strips it itself)
  bool merge = false;
  if (crc_tail && !pipe) {
    if (crc_fork) {
      // verified on the side stream while k_gzip decodes (the check is HBM-bound, the decode latency-
      // bound); a stripped-unverified tail (crc_tail 2) needs no check at all
      tail_mode = 3;
      if (crc_tail == 1) {
        hipError_t e = hipMemcpyAsync(crc_fork->snap_items, items, (size_t)n_items * sizeof(ZgItem),
                                      hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess)
          e = hipMemcpyAsync(crc_fork->snap_status, status, (size_t)n_items * 4, hipMemcpyDeviceToDevice, s);
        if (e == hipSuccess) e = hipEventRecord(crc_fork->ev_fork, s);
        if (e == hipSuccess) e = hipStreamWaitEvent(crc_fork->side, crc_fork->ev_fork, 0);
        if (e == hipSuccess)
          e = launch_crc32c_check(crc_fork->snap_items, crc_fork->snap_status, crc_fork->bad, n_items, crc_fork->side);
        if (e == hipSuccess) e = hipEventRecord(crc_fork->ev_join, crc_fork->side);
        if (e != hipSuccess) return e;
        merge = true;
      }
    } else {
      const hipError_t e = launch_crc32c_strip(items, status, n_items, 0, crc_tail == 1 ? 1 : 0, s);
      if (e != hipSuccess) return e;
    }
  }
  if (order) hipLaunchKernelGGL(k_order_by_len, dim3(1), dim3(1024), 0, s, items, status, n_items, order);
  if (pipe)
    hipLaunchKernelGGL((k_gzip<false, true>), dim3(n_items), dim3(128), 0, s, items, status, nullptr, dst, slot_bytes,
                       nullptr, order, seg_scr, crc_tail, gd);
  else
    hipLaunchKernelGGL(k_gzip<false>, dim3(n_items), dim3(64), 0, s, items, status, nullptr, dst, slot_bytes, nullptr,
                       order, seg_scr, tail_mode, gd);
  if (merge) {
    hipError_t e = hipGetLastError();
    if (e == hipSuccess) e = hipStreamWaitEvent(s, crc_fork->ev_join, 0);
    if (e == hipSuccess) e = launch_crc32c_merge(status, crc_fork->bad, n_items, s);
    if (e != hipSuccess) return e;
  }
  return hipGetLastError();
}

hipError_t launch_zlib_streams(ZgItem *subs, uint32_t *sub_status, const uint32_t *sub_kind, uint32_t n_sub,
                               uint8_t *dst, uint64_t slot, uint2 *aux, uint32_t *seg_scr, hipStream_t s) {
  if (!n_sub) return hipSuccess;
  if (!gzip_seg_scratch_bytes(1)) seg_scr = nullptr;
  hipLaunchKernelGGL(k_gzip<true>, dim3(n_sub), dim3(64), 0, s, subs, sub_status, sub_kind, dst, slot, aux,
                     nullptr, seg_scr, 0, GzDirect{});
  return hipGetLastError();
}

}  // namespace zgpu
