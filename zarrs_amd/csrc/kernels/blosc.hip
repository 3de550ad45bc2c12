// blosc (c-blosc 1.x frame, format version 1/2) decode on gfx950: SURVEY.md §8(f) rank 2.
//
// Reference: zarrs' blosc codec (zarrs/src/array/codec/bytes_to_bytes/blosc/blosc_codec_via_blosc_src.rs
// :132-142 do_decode -> blosc_validate + blosc_decompress_bytes, blosc_via_blosc_src.rs:115-191), i.e.
// c-blosc 1.21 (blosc-src 0.3.6) blosc_decompress_ctx. The frame:
//   16-B header {version, versionlz, flags, typesize, nbytes u32, blocksize u32, cbytes u32}
//   flags: 0x1 byte shuffle, 0x2 memcpyed (raw payload after the header), 0x4 bitshuffle,
//          0x10 blocks not split, bits 5-7 compressor format (0 blosclz, 1 lz4/lz4hc, 2 snappy,
//          3 zlib, 4 zstd); every one of them decodes here (formats 5-7 -> UNSUPPORTED)
//   bstarts[nblocks] i32, then per block nsplit = (split && not the leftover block) ? typesize : 1
//   streams of {csize i32, payload}; csize == neblock means stored.
// A block's streams concatenate to the shuffled block, then unshuffle / bitunshuffle (format 2:
// only when the block's element count is a multiple of 8, else the block is stored unshuffled).
//
// GPU decomposition (one plan stage, items = the chain's leaf chunks):
//   k_blosc_info     one thread per item: header checks, #blocks, #streams, compressor (read back
//                    to the host to size the stream table on a plan's first execution)
//   k_blosc_layout   later executions: the table's layout as device prefix sums, checked against the
//                    capacities the first execution recorded (no host round trip)
//   k_blosc_streams  one wave per item: walks bstarts + split sizes in parallel over blocks, writes
//                    one ZgItem per compressed stream (+ its kind) and one record per block
//   zstd streams     the block-parallel zstd pipeline (launch_zstd) over the stream table
//   k_lz4, k_blosclz, k_snappy  one wave per lz4 / blosclz / snappy stream (input staged through
//                    an LDS window, recent output in an LDS ring)
//   zlib streams     k_gzip's DEFLATE decoder with the RFC 1950 wrapper (inflate.hip), then the
//                    Adler-32 trailer check (k_adler32_check, crc.hip)
//   k_blosc_finish   one workgroup per block: gathers the block's streams and unshuffles /
//                    bitunshuffles them into the item's output slot (fused: no extra pass)
#include "launch.hpp"

namespace zgpu {


__device__ __forceinline__ uint32_t ld_u32(const uint8_t *p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}
__device__ __forceinline__ void set_status(uint32_t *st, uint32_t v) { atomicCAS(st, 0u, v); }

__global__ __launch_bounds__(64) void k_blosc_info(const ZgItem *items, uint32_t *status, uint32_t n_items,
                                                   uint64_t slot_bytes, BlInfo *info) {
  const uint32_t i = blockIdx.x * 64 + threadIdx.x;
  if (i >= n_items) return;
  BlInfo r{0, 0, BL_COMP_SKIP, 0, 0, 0};
  const ZgItem it = items[i];
  if (status[i] || (it.flags & ZG_ITEM_FILL)) {
    info[i] = r;
    return;
  }
  const uint8_t *h = (const uint8_t *)it.src;
  uint32_t err = 0;
  if (it.len < 16) err = ZG_CORRUPT_STREAM;
  uint32_t ver = 0, flags = 0, ts = 0, nbytes = 0, bs = 0, cbytes = 0;
  if (!err) {
    ver = h[0];
    flags = h[2];
    ts = h[3];
    nbytes = ld_u32(h + 4);
    bs = ld_u32(h + 8);
    cbytes = ld_u32(h + 12);
    // blosc_cbuffer_validate: version, header cbytes within the buffer
    if (ver > 2 || cbytes < 16 || cbytes > it.len) err = ZG_CORRUPT_STREAM;
    else if (nbytes > slot_bytes) err = ZG_DECODED_SIZE_MISMATCH;
  }
  if (!err && (flags & 0x2)) {  // memcpyed: the payload is the data
    if (16ull + nbytes > cbytes) err = ZG_CORRUPT_STREAM;
    r = BlInfo{nbytes ? 1u : 0u, nbytes ? 1u : 0u, BL_COMP_MEMCPY, 0, nbytes, ver};
  } else if (!err && nbytes) {
    const uint32_t comp = flags >> 5;
    if (ts == 0 || bs == 0) err = ZG_CORRUPT_STREAM;
    else if (comp > BL_COMP_ZSTD) err = ZG_UNSUPPORTED;  // formats 5-7 are not defined by c-blosc 1.x
    if (!err) {
      const uint32_t lo = nbytes % bs, nfull = nbytes / bs, nblk = nfull + (lo ? 1 : 0);
      const uint32_t nsplit = (flags & 0x10) ? 1 : ts;
      if (16ull + 4ull * nblk > cbytes) err = ZG_CORRUPT_STREAM;
      const uint32_t ne = bs / nsplit;
      r = BlInfo{nfull * nsplit + (lo ? 1 : 0), nblk, comp, ne > lo ? ne : lo, nbytes, ver};
    }
  } else if (!err) {
    r = BlInfo{0, 0, BL_COMP_MEMCPY, 0, 0, ver};
  }
  if (err) {
    status[i] = err;
    r = BlInfo{0, 0, BL_COMP_SKIP, 0, 0, 0};
  }
  info[i] = r;
}

// The stream table's layout on the device (one workgroup): per-item {first stream, first block} as
// exclusive prefix sums of BlInfo, checked against the capacities of a cached layout. Entries past
// this execution's totals are made inert (skipped streams, empty blocks); on overflow every entry is,
// *ovf is set and the host re-runs the plan with a read-back layout (plan_statuses).
__global__ __launch_bounds__(1024) void k_blosc_layout(const BlInfo *info, uint32_t n_items, uint64_t *bases,
                                                       BlCaps caps, uint32_t *sub_status, uint32_t *sub_kind,
                                                       BlBlock *blocks, unsigned long long *ovf) {
  __shared__ uint64_t ssub[1024], sblk[1024];
  __shared__ uint32_t s_ne, s_kinds;
  const uint32_t t = threadIdx.x;
  if (t == 0) s_ne = 0, s_kinds = 0;
  const uint32_t per = (n_items + 1023) / 1024, i0 = min(t * per, n_items), i1 = min(i0 + per, n_items);
  uint64_t nsub = 0, nblk = 0;
  uint32_t ne = 0, kinds = 0;
  for (uint32_t i = i0; i < i1; i++) {
    const BlInfo I = info[i];
    if (I.comp == BL_COMP_SKIP) continue;
    nsub += I.nsub;
    nblk += I.nblk;
    ne = max(ne, I.max_ne);
    if (I.nsub) kinds |= I.comp == BL_COMP_ZSTD ? BL_HAS_ZSTD : I.comp == BL_COMP_LZ4 ? BL_HAS_LZ4
                        : I.comp == BL_COMP_BLOSCLZ ? BL_HAS_BLOSCLZ : I.comp == BL_COMP_ZLIB ? BL_HAS_ZLIB
                        : I.comp == BL_COMP_SNAPPY ? BL_HAS_SNAPPY : 0u;
  }
  ssub[t] = nsub;
  sblk[t] = nblk;
  __syncthreads();
  if (ne) atomicMax(&s_ne, ne);
  if (kinds) atomicOr(&s_kinds, kinds);
  for (uint32_t off = 1; off < 1024; off <<= 1) {  // inclusive scans
    const uint64_t a = t >= off ? ssub[t - off] : 0, b = t >= off ? sblk[t - off] : 0;
    __syncthreads();
    ssub[t] += a;
    sblk[t] += b;
    __syncthreads();
  }
  uint64_t bs = ssub[t] - nsub, bb = sblk[t] - nblk;
  for (uint32_t i = i0; i < i1; i++) {
    const BlInfo I = info[i];
    bases[2 * i] = bs;
    bases[2 * i + 1] = bb;
    if (I.comp == BL_COMP_SKIP) continue;
    bs += I.nsub;
    bb += I.nblk;
  }
  const uint64_t tot_sub = ssub[1023], tot_blk = sblk[1023];
  const bool over = tot_sub > caps.n_sub || tot_blk > caps.n_blk || s_ne > caps.max_ne || (s_kinds & ~caps.kinds);
  if (over && t == 0) *ovf = 1ull;
  for (uint64_t k = over ? t : tot_sub + t; k < caps.n_sub; k += 1024) {
    sub_status[k] = BL_SKIP;
    sub_kind[k] = BL_KIND_RAW;
  }
  for (uint64_t k = over ? t : tot_blk + t; k < caps.n_blk; k += 1024)
    blocks[k] = BlBlock{0, 0, 0, 0, 0, 0, 0, 1, 1};
}

__global__ __launch_bounds__(64) void k_blosc_streams(ZgItem *items, uint32_t *status, const BlInfo *info,
                                                      const uint64_t *bases, ZgItem *subs, uint32_t *sub_status,
                                                      uint32_t *sub_kind, BlBlock *blocks, uint8_t *dst,
                                                      uint64_t slot_bytes, const unsigned long long *ovf,
                                                      uint32_t direct, uint64_t want, uint64_t row_bytes,
                                                      const uint64_t *need, unsigned long long *n_decoded) {
  const uint32_t item = blockIdx.x, lane = threadIdx.x;
  const BlInfo I = info[item];
  if (I.comp == BL_COMP_SKIP || status[item] || *ovf) return;
  // the decoded bytes this item's selection reads (a partial read: only the blocks covering them)
  const uint64_t nlo = need ? need[2 * item] : 0, nhi = need ? need[2 * item + 1] : UINT64_MAX;
  uint32_t n_dec = 0;
  const ZgItem it = items[item];
  const uint8_t *h = (const uint8_t *)it.src;
  const uint64_t sub0 = bases[2 * item], blk0 = bases[2 * item + 1];
  bool bad = false;
  uint64_t blk_bytes = I.nbytes;  // the largest block
  if (I.comp == BL_COMP_MEMCPY) {
    if (lane == 0 && I.nblk) {
      subs[sub0] = ZgItem{it.src + 16, I.nbytes, item, 0, 0, 0};
      sub_status[sub0] = BL_SKIP;
      sub_kind[sub0] = BL_KIND_RAW;
      blocks[blk0] = BlBlock{item, I.nbytes, 0, (uint32_t)sub0, 1, I.nbytes, 0, 1, I.ver};
      n_dec = 1;
    }
  } else {
    const uint32_t flags = h[2], ts = h[3], bs = ld_u32(h + 8), cbytes = ld_u32(h + 12);
    const uint32_t lo = I.nbytes % bs, nsplit_full = (flags & 0x10) ? 1 : ts;
    const uint32_t mode = ((flags & 0x1) && ts > 1) ? 1u : (flags & 0x4) ? 2u : 0u;
    blk_bytes = bs;
    for (uint32_t b = lane; b < I.nblk; b += 64) {
      const bool left = lo && b == I.nblk - 1;
      const uint32_t bsize = left ? lo : bs, nsplit = left ? 1 : nsplit_full, ne = bsize / nsplit;
      const uint64_t s0 = sub0 + (uint64_t)b * nsplit_full;
      for (uint32_t j = 0; j < nsplit; j++) {  // every record valid (and skipped) unless parsed below
        subs[s0 + j] = ZgItem{0, 0, item, ZG_ITEM_FILL, 0, 0};
        sub_status[s0 + j] = BL_SKIP;
        sub_kind[s0 + j] = BL_KIND_RAW;
      }
      if ((uint64_t)b * bs >= nhi || (uint64_t)b * bs + bsize <= nlo) {  // not read by the selection
        blocks[blk0 + b] = BlBlock{item, 0u, (uint64_t)b * bs, (uint32_t)s0, 0u, ne, mode, ts, I.ver};
        continue;
      }
      n_dec++;
      bool ok = true;
      int64_t p = (int32_t)ld_u32(h + 16 + 4ull * b);
      if (p < 16 + 4ll * I.nblk || p > (int64_t)cbytes || bsize % nsplit) ok = false;
      for (uint32_t j = 0; j < nsplit && ok; j++) {
        if (p + 4 > (int64_t)cbytes) {
          ok = false;
          break;
        }
        const int64_t cs = (int32_t)ld_u32(h + p);
        p += 4;
        if (cs < 0 || p + cs > (int64_t)cbytes) {
          ok = false;
          break;
        }
        const bool raw = (uint64_t)cs == ne;
        // bitshuffled blocks hold long literal runs and matches: decoded one stream per wave (BL_SUB_WIDE)
        subs[s0 + j] = ZgItem{it.src + (uint64_t)p, (uint64_t)cs, item,
                              (mode == 2 && I.comp != BL_COMP_ZSTD && I.comp != BL_COMP_ZLIB) ? BL_SUB_WIDE : 0u, 0, 0};
        sub_kind[s0 + j] = raw ? BL_KIND_RAW
                           : I.comp == BL_COMP_ZSTD ? BL_KIND_ZSTD
                           : I.comp == BL_COMP_LZ4  ? BL_KIND_LZ4
                           : I.comp == BL_COMP_ZLIB ? BL_KIND_ZLIB
                           : I.comp == BL_COMP_SNAPPY ? BL_KIND_SNAPPY
                                                    : BL_KIND_BLOSCLZ;
        sub_status[s0 + j] = (!raw && I.comp == BL_COMP_ZSTD) ? 0u : BL_SKIP;
        p += cs;
      }
      if (!ok) bad = true;
      blocks[blk0 + b] = BlBlock{item, ok ? bsize : 0u, (uint64_t)b * bs, (uint32_t)s0, ok ? nsplit : 0u, ne, mode,
                                 ts, I.ver};
    }
  }
  bad = __any(bad);
  for (int o = 32; o; o >>= 1) n_dec += __shfl_xor(n_dec, o, 64);
  if (lane == 0 && n_decoded && n_dec) atomicAdd(n_decoded, (unsigned long long)n_dec);
  if (lane == 0) {
    if (bad) {
      set_status(&status[item], ZG_CORRUPT_STREAM);
    } else {  // the item's decoded bytes will be in its slot (written by k_blosc_finish)
      items[item].src = (uint64_t)(dst + (uint64_t)item * slot_bytes);
      items[item].len = I.nbytes;
      // or straight in the output rows (a size mismatch takes the slot path: the scatter reports it
      // after the decode, as the chain's size check follows the codec's)
      if (direct && I.nbytes == want && blk_bytes <= (uint64_t)(BL_DIRECT_ROWS - 2) * row_bytes)
        items[item].flags = it.flags | ZG_ITEM_DIRECT;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Serial LZ77 stream decoders (lz4, blosclz, snappy), one wave per stream. The token parse is
// inherently serial. Every token / length / offset byte comes from an LDS window of the compressed
// stream (LZW bytes, refilled with coalesced 16-B loads when the parse leaves it), literal runs are
// copied from the window by all lanes, and a match is copied from an LDS ring of the last LZR output
// bytes (or, further back, from the wave's own earlier output in HBM).
// At 8 waves per SIMD the decoders are issue-bound, not latency-bound (PMC on the 4 GiB blosc lz4
// workload: ~80 SALU + 42 VALU instructions per sequence, 27 % of wave time issuing, 8 waves sharing
// a SIMD): positions are 32-bit (a blosc stream and its output are < 2 GiB), the window is addressed
// by its stream offset, and a copy of at most 64 bytes (nearly all of them) is one predicated pass
// (lz4 131.7 -> 151.2 GiB/s against 64-bit positions and loop copies).
// ---------------------------------------------------------------------------------------------
#ifndef ZG_LZ_RING
#define ZG_LZ_RING 4096  // bytes of recent output kept in LDS
#endif
#ifndef ZG_LZW  // input window: 1 KiB + the 4 KiB ring = 5 KiB per one-wave workgroup -> 8 waves per SIMD
#define ZG_LZW 1024     // (a 4 KiB window: 5 waves, lz4 43.1 -> 35.4 ms: r03s_blosc_lz_window_ab)
#endif
constexpr uint32_t LZW = ZG_LZW;
constexpr uint32_t LZR = ZG_LZ_RING, LZRM = LZR - 1;
static_assert((LZR & LZRM) == 0 && LZR >= 64 && LZW % 1024 == 0, "lz ring / window sizes");

struct Lz32 {
  uintptr_t base;  // the stream
  uint32_t cs;     // its length (< 2^31)
  int32_t wo;      // stream offset of win[0] (a 16-B aligned address: -15 .. 0 for the first window)
  uint32_t safe;   // output below this is known written (the wave's stores waited for)
  uint8_t *win, *ring, *out;

  // load the window holding stream offset p (uniform across the wave)
  __device__ void fill(uint32_t p) {
    __syncthreads();
    const uintptr_t a = (base + p) & ~(uintptr_t)15, hi = base + cs;
    wo = (int32_t)(int64_t)(a - base);
    for (uint32_t v = threadIdx.x; v < LZW / 16; v += 64) {
      const uintptr_t q = a + 16ull * v;
      if (q >= hi) break;
      if (q >= base && q + 16 <= hi) {
        *(uint4 *)(win + 16 * v) = *(const uint4 *)q;
      } else {  // the stream's first / last partial vector: bytes inside it only
        for (uint32_t k = 0; k < 16; k++)
          if (q + k >= base && q + k < hi) win[16 * v + k] = *(const uint8_t *)(q + k);
      }
    }
    __syncthreads();
  }
  __device__ __forceinline__ uint32_t rd(uint32_t p) {
    uint32_t k = p - (uint32_t)wo;
    if (k >= LZW) {
      fill(p);
      k = p - (uint32_t)wo;
    }
    return win[k];
  }
  // out[op .. op+n) = stream[ip .. ip+n) (window bytes from LDS, the rest from HBM), and to the ring
  __device__ __forceinline__ void lits(uint32_t op, uint32_t ip, uint32_t n) {
    for (uint32_t i = threadIdx.x; i < n; i += 64) {
      const uint32_t q = ip + i, k = q - (uint32_t)wo;
      const uint8_t v = k < LZW ? win[k] : ((const uint8_t *)base)[q];
      out[op + i] = v;
      ring[(op + i) & LZRM] = v;
    }
  }
  // A match of length ml at distance off (1 <= off <= op): byte i is out[op - off + (i mod off)],
  // which precedes the match, so lanes never read what another lane of this copy writes. From the
  // ring when source and copy fit in it; else from HBM after waiting for the wave's own stores
  // (workgroup scope = this CU's L1, which its write-through stores keep coherent).
  __device__ __forceinline__ void match(uint32_t op, uint32_t off, uint32_t ml) {
    const uint32_t lane = threadIdx.x;
    if (off + ml <= LZR) {
      if (ml <= 64) {
        if (lane < ml) {
          const uint8_t v = ring[(op - off + (off >= ml ? lane : lane % off)) & LZRM];
          ring[(op + lane) & LZRM] = v;
          out[op + lane] = v;
        }
      } else {
        for (uint32_t i = lane; i < ml; i += 64) {
          const uint8_t v = ring[(op - off + (off >= ml ? i : i % off)) & LZRM];
          ring[(op + i) & LZRM] = v;
          out[op + i] = v;
        }
      }
      return;
    }
    if (op - off + min(off, ml) > safe) {
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      safe = op;
    }
    const uint8_t *src = out + (op - off);
    for (uint32_t i = lane; i < ml; i += 64) {
      const uint8_t v = src[off >= ml ? i : i % off];
      out[op + i] = v;
      ring[(op + i) & LZRM] = v;
    }
  }
};

// the decoder's setup: err when the stream is empty or too long for 32-bit positions
#define LZ32_SETUP(KIND)                                                                       \
  __shared__ __attribute__((aligned(16))) uint8_t win[LZW];                                  \
  __shared__ uint8_t ring[LZR];                                                               \
  const uint32_t s = blockIdx.x, lane = threadIdx.x;                                          \
  if (sub_kind[s] != (KIND) || sub_status[s] != BL_SKIP) return;                              \
  const ZgItem it = subs[s];                                                                  \
  uint32_t err = it.len == 0 || it.len >= 0x7FFFFFFFull;                                      \
  const uint32_t cs = err ? 0u : (uint32_t)it.len;                                            \
  const uint32_t cap = (uint32_t)min<uint64_t>(slot, 0x7FFFFFFFull);                         \
  Lz32 L{(uintptr_t)it.src, cs, 0, 0, win, ring, dst + (uint64_t)s * slot};                   \
  if (!err) L.fill(0);                                                                        \
  uint32_t ip = 0, op = 0

#define LZ32_FINISH()                                  \
  if (lane == 0) {                                     \
    sub_status[s] = err ? ZG_CORRUPT_STREAM : 0u;      \
    subs[s].src = (uint64_t)L.out;                     \
    subs[s].len = op;                                  \
  }

// LZ4 block format (lz4_Block_format.md): sequences {token, literal length, literals, offset u16,
// match length}; the last sequence has literals only.
__global__ __launch_bounds__(64) void k_lz4(ZgItem *subs, uint32_t *sub_status, const uint32_t *sub_kind,
                                            uint32_t n_sub, uint8_t *dst, uint64_t slot) {
  LZ32_SETUP(BL_KIND_LZ4);
  while (!err) {
    if (ip >= cs) { err = 1; break; }
    const uint32_t token = L.rd(ip++);
    uint32_t ll = token >> 4;
    if (ll == 15) {
      uint32_t b;
      do {
        if (ip >= cs) { err = 1; break; }
        b = L.rd(ip++);
        ll += b;
      } while (b == 255 && ll < 0x7FFFFFFFu);
      if (err) break;
    }
    if (ll > cs - ip || ll > cap - op) { err = 1; break; }
    L.lits(op, ip, ll);
    ip += ll;
    op += ll;
    if (ip == cs) break;  // last sequence: literals only
    if (cs - ip < 2) { err = 1; break; }
    const uint32_t off = L.rd(ip) | (L.rd(ip + 1) << 8);
    ip += 2;
    if (off == 0 || off > op) { err = 1; break; }
    uint32_t ml = token & 15;
    if (ml == 15) {
      uint32_t b;
      do {
        if (ip >= cs) { err = 1; break; }
        b = L.rd(ip++);
        ml += b;
      } while (b == 255 && ml < 0x7FFFFFFFu);
      if (err) break;
    }
    ml += 4;
    if (ml > cap - op) { err = 1; break; }
    L.match(op, off, ml);
    op += ml;
  }
  LZ32_FINISH();
}

// ---- several lz4 streams per wave ----
// The one-stream-per-wave decoder spends ~155 instructions per sequence, most of them scalar parse
// work, and a copy uses ~24 of 64 lanes. Here a wave decodes 64 / G streams at once, G lanes each:
// the parse runs in vector registers (every group of G lanes holds its stream's uniform state), so
// one instruction advances all the wave's streams; copies use the group's G lanes. Streams come
// from a compacted list (k_lz_list) so no group idles on stored or other-kind streams.
#ifndef ZG_LZM_G
#define ZG_LZM_G 32
#endif
__global__ __launch_bounds__(1024) void k_lz_list(const ZgItem *subs, const uint32_t *sub_kind,
                                                  const uint32_t *sub_status, uint32_t n_sub, uint32_t kind,
                                                  uint32_t wide, uint32_t *list) {
  __shared__ uint32_t wsum[16], s_base;
  const uint32_t t = threadIdx.x, w = t >> 6, l = t & 63;
  if (t == 0) s_base = 0;
  __syncthreads();
  for (uint32_t c = 0; c < n_sub; c += 1024) {
    const uint32_t i = c + t;
    const bool f = i < n_sub && sub_kind[i] == kind && sub_status[i] == BL_SKIP &&
                   ((subs[i].flags & BL_SUB_WIDE) != 0) == (wide != 0);
    const uint64_t m = __ballot(f);
    if (l == 0) wsum[w] = (uint32_t)__builtin_popcountll(m);
    __syncthreads();
    uint32_t off = s_base + (uint32_t)__builtin_popcountll(m & ((1ull << l) - 1));
    for (uint32_t k = 0; k < w; k++) off += wsum[k];
    if (f) list[1 + off] = i;
    __syncthreads();
    if (t == 0) {
      uint32_t tot = 0;
      for (uint32_t k = 0; k < 16; k++) tot += wsum[k];
      s_base += tot;
    }
    __syncthreads();
  }
  if (t == 0) list[0] = s_base;
}

// one stream's state in a group of G lanes (uniform within the group); methods are called by whole groups
template <int G>
struct LzG {
  uintptr_t base;
  uint32_t cs, gl, safe;
  int32_t wo;
  uint8_t *win, *ring, *out;

  __device__ void fill(uint32_t p) {
    const uintptr_t a = (base + p) & ~(uintptr_t)15, hi = base + cs;
    wo = (int32_t)(int64_t)(a - base);
    for (uint32_t v = gl; v < LZW / 16; v += G) {
      const uintptr_t q = a + 16ull * v;
      if (q >= hi) break;
      if (q >= base && q + 16 <= hi) {
        *(uint4 *)(win + 16 * v) = *(const uint4 *)q;
      } else {
        for (uint32_t b = 0; b < 16; b++)
          if (q + b >= base && q + b < hi) win[16 * v + b] = *(const uint8_t *)(q + b);
      }
    }
    // The group's other lanes read these window bytes next (rd). A group lives inside one wave (G <=
    // 64) and one wave's LDS operations complete in issue order, so no workgroup barrier is needed;
    // the wavefront-scope fence keeps the compiler from moving those reads above the stores.
    static_assert(G <= 64, "a stream's lane group must lie within one wave");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
  }
  __device__ __forceinline__ uint32_t rd(uint32_t p) {
    uint32_t kk = p - (uint32_t)wo;
    if (kk >= LZW) {
      fill(p);
      kk = p - (uint32_t)wo;
    }
    return win[kk];
  }
  __device__ __forceinline__ void lits(uint32_t op, uint32_t ip, uint32_t n) {
    for (uint32_t i = gl; i < n; i += G) {
      const uint32_t q = ip + i, kk = q - (uint32_t)wo;
      const uint8_t v = kk < LZW ? win[kk] : ((const uint8_t *)base)[q];
      out[op + i] = v;
      ring[(op + i) & LZRM] = v;
    }
  }
  __device__ __forceinline__ void match(uint32_t op, uint32_t off, uint32_t ml) {
    if (off + ml <= LZR) {
      for (uint32_t i = gl; i < ml; i += G) {
        const uint8_t v = ring[(op - off + (off >= ml ? i : i % off)) & LZRM];
        ring[(op + i) & LZRM] = v;
        out[op + i] = v;
      }
      return;
    }
    if (op - off + min(off, ml) > safe) {  // the wave's own stores of the source: wait for them
      __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
      safe = op;
    }
    const uint8_t *src = out + (op - off);
    for (uint32_t i = gl; i < ml; i += G) {
      const uint8_t v = src[off >= ml ? i : i % off];
      out[op + i] = v;
      ring[(op + i) & LZRM] = v;
    }
  }
};

// group setup: stream k of the list for group g; act = the group has a stream to decode
#define LZG_SETUP()                                                                            \
  constexpr uint32_t NG = 64 / G;                                                              \
  __shared__ __attribute__((aligned(16))) uint8_t win_all[NG][LZW];                           \
  __shared__ uint8_t ring_all[NG][LZR];                                                        \
  const uint32_t lane = threadIdx.x, g = lane / G;                                             \
  const uint32_t k = blockIdx.x * NG + g, cnt = list[0];                                       \
  if (blockIdx.x * NG >= cnt) return;                                                          \
  const bool have = k < cnt;                                                                   \
  const uint32_t s = have ? list[1 + k] : 0u;                                                  \
  const ZgItem it = have ? subs[s] : ZgItem{0, 0, 0, 0, 0, 0};                                 \
  uint32_t err = have && (it.len == 0 || it.len >= 0x7FFFFFFFull);                             \
  const uint32_t cs = (have && !err) ? (uint32_t)it.len : 0u;                                  \
  const uint32_t cap = (uint32_t)min<uint64_t>(slot, 0x7FFFFFFFull);                          \
  LzG<G> L{(uintptr_t)it.src, cs, lane % G, 0, 0, win_all[g], ring_all[g], dst + (uint64_t)s * slot}; \
  uint32_t ip = 0, op = 0;                                                                     \
  bool act = have && !err;                                                                     \
  if (act) L.fill(0)

#define LZG_FINISH()                                   \
  if (have && lane % G == 0) {                         \
    sub_status[s] = err ? ZG_CORRUPT_STREAM : 0u;      \
    subs[s].src = (uint64_t)L.out;                     \
    subs[s].len = op;                                  \
  }

template <int G>
__global__ __launch_bounds__(64) void k_lz4m(ZgItem *subs, uint32_t *sub_status, const uint32_t *list,
                                             uint8_t *dst, uint64_t slot) {
  LZG_SETUP();
  while (__ballot(act)) {
    if (!act) continue;
    const uint32_t token = L.rd(ip++);
    uint32_t ll = token >> 4;
    if (ll == 15) {
      uint32_t b;
      do {
        if (ip >= cs) { err = 1; break; }
        b = L.rd(ip++);
        ll += b;
      } while (b == 255 && ll < 0x7FFFFFFFu);
    }
    if (!err && (ll > cs - ip || ll > cap - op)) err = 1;
    if (!err) {
      L.lits(op, ip, ll);
      ip += ll;
      op += ll;
      if (ip == cs) {
        act = false;  // last sequence: literals only
      } else if (cs - ip < 2) {
        err = 1;
      } else {
        const uint32_t off = L.rd(ip) | (L.rd(ip + 1) << 8);
        ip += 2;
        uint32_t ml = token & 15;
        if (off == 0 || off > op) err = 1;
        if (!err && ml == 15) {
          uint32_t b;
          do {
            if (ip >= cs) { err = 1; break; }
            b = L.rd(ip++);
            ml += b;
          } while (b == 255 && ml < 0x7FFFFFFFu);
        }
        ml += 4;
        if (!err && (ml > cap - op || ip >= cs)) err = 1;  // a stream ends with a literals-only sequence
        if (!err) {
          L.match(op, off, ml);
          op += ml;
        }
      }
    }
    if (err) act = false;
  }
  LZG_FINISH();
}

// blosclz (the format below, k_blosclz), several streams per wave
template <int G>
__global__ __launch_bounds__(64) void k_blosclzm(ZgItem *subs, uint32_t *sub_status, const uint32_t *list,
                                                 uint8_t *dst, uint64_t slot) {
  LZG_SETUP();
  uint32_t ctrl = act ? L.rd(ip++) & 31u : 0u;
  while (__ballot(act)) {
    if (!act) continue;
    if (ctrl >= 32) {
      uint32_t len = (ctrl >> 5) - 1;
      const uint32_t ofs = (ctrl & 31u) << 8;
      uint32_t code = 0;
      if (len == 6) {
        do {
          if (cs - ip <= 1) { err = 1; break; }
          code = L.rd(ip++);
          len += code;
        } while (code == 255 && len < 0x7FFFFFFFu);
      } else if (cs - ip <= 1) {
        err = 1;
      }
      if (!err) {
        code = L.rd(ip++);
        len += 3;
        uint32_t dist = ofs + code + 1;
        if (code == 255 && ofs == (31u << 8)) {
          if (cs - ip <= 1) {
            err = 1;
          } else {
            dist = (L.rd(ip) << 8) + L.rd(ip + 1) + 8192;
            ip += 2;
          }
        }
        if (!err && (len > cap - op || dist > op)) err = 1;
        if (!err) {
          L.match(op, dist, len);
          op += len;
        }
      }
    } else {
      const uint32_t run = ctrl + 1;
      if (run > cap - op || run > cs - ip) {
        err = 1;
      } else {
        L.lits(op, ip, run);
        op += run;
        ip += run;
      }
    }
    if (err || ip >= cs) {
      act = false;
    } else {
      ctrl = L.rd(ip++);
    }
  }
  LZG_FINISH();
}

// snappy (the format below, k_snappy), several streams per wave
template <int G>
__global__ __launch_bounds__(64) void k_snappym(ZgItem *subs, uint32_t *sub_status, const uint32_t *list,
                                                uint8_t *dst, uint64_t slot) {
  LZG_SETUP();
  uint64_t want = 0;
  // preamble: little-endian base-128 varint (<= 5 bytes, < 2^32)
  for (uint32_t kk = 0; act; kk++) {
    if (ip >= cs || kk == 5) { err = 1; break; }
    const uint32_t b = L.rd(ip++);
    want |= (uint64_t)(b & 127) << (7 * kk);
    if (!(b & 128)) break;
  }
  if (act && !err && want > cap) err = 1;
  if (err) act = false;
  const uint32_t w32 = (uint32_t)want;
  if (act && ip >= cs) act = false;  // no elements
  while (__ballot(act)) {
    if (!act) continue;
    const uint32_t tag = L.rd(ip++);
    if ((tag & 3) == 0) {  // literal
      uint64_t len = (tag >> 2) + 1;
      if (len > 60) {
        const uint32_t nb = (uint32_t)len - 60;  // 1..4 length bytes
        if (nb > cs - ip) {
          err = 1;
        } else {
          uint64_t v = 0;
          for (uint32_t q = 0; q < nb; q++) v |= (uint64_t)L.rd(ip + q) << (8 * q);
          ip += nb;
          len = v + 1;
        }
      }
      if (!err && (len > cs - ip || len > w32 - op)) err = 1;
      if (!err) {
        L.lits(op, ip, (uint32_t)len);
        ip += (uint32_t)len;
        op += (uint32_t)len;
      }
    } else {
      uint32_t len = 0;
      uint64_t off = 0;
      if ((tag & 3) == 1) {
        if (cs - ip < 1) {
          err = 1;
        } else {
          len = 4 + ((tag >> 2) & 7);
          off = ((tag >> 5) << 8) | L.rd(ip);
          ip += 1;
        }
      } else if ((tag & 3) == 2) {
        if (cs - ip < 2) {
          err = 1;
        } else {
          len = 1 + (tag >> 2);
          off = L.rd(ip) | (L.rd(ip + 1) << 8);
          ip += 2;
        }
      } else {
        if (cs - ip < 4) {
          err = 1;
        } else {
          len = 1 + (tag >> 2);
          off = (uint64_t)L.rd(ip) | ((uint64_t)L.rd(ip + 1) << 8) | ((uint64_t)L.rd(ip + 2) << 16) |
                ((uint64_t)L.rd(ip + 3) << 24);
          ip += 4;
        }
      }
      if (!err && (off == 0 || off > op || len > w32 - op)) err = 1;
      if (!err) {
        L.match(op, (uint32_t)off, len);
        op += len;
      }
    }
    if (err || ip >= cs) act = false;
  }
  if (have && !err && op != w32) err = 1;
  LZG_FINISH();
}

// blosclz (c-blosc 1.21 blosclz.c, blosclz_decompress; restated, checked against c-blosc in
// tests/test_gpu_blosc.py): a FastLZ-style stream. The first control byte (low 5 bits) opens a
// literal run; a control byte c < 32 is a run of c + 1 literals; c >= 32 is a match of length
// (c >> 5) + 2 (7 -> extended by following bytes until one is not 255) whose distance is
// ((c & 31) << 8) + next byte + 1, or, when that byte is 255 and c & 31 == 31, a 16-bit big-endian
// value + 8192 (MAX_DISTANCE 8191 + 1). The stream ends when its bytes are consumed.
__global__ __launch_bounds__(64) void k_blosclz(ZgItem *subs, uint32_t *sub_status, const uint32_t *sub_kind,
                                                uint32_t n_sub, uint8_t *dst, uint64_t slot) {
  LZ32_SETUP(BL_KIND_BLOSCLZ);
  uint32_t ctrl = err ? 0u : L.rd(ip++) & 31u;
  while (!err) {
    if (ctrl >= 32) {
      uint32_t len = (ctrl >> 5) - 1;
      const uint32_t ofs = (ctrl & 31u) << 8;
      uint32_t code;
      if (len == 6) {
        do {
          if (cs - ip <= 1) { err = 1; break; }
          code = L.rd(ip++);
          len += code;
        } while (code == 255 && len < 0x7FFFFFFFu);
        if (err) break;
      } else if (cs - ip <= 1) {
        err = 1;
        break;
      }
      code = L.rd(ip++);
      len += 3;
      uint32_t dist = ofs + code + 1;
      if (code == 255 && ofs == (31u << 8)) {
        if (cs - ip <= 1) { err = 1; break; }
        dist = (L.rd(ip) << 8) + L.rd(ip + 1) + 8192;
        ip += 2;
      }
      if (len > cap - op || dist > op) { err = 1; break; }
      L.match(op, dist, len);
      op += len;
    } else {
      const uint32_t run = ctrl + 1;
      if (run > cap - op || run > cs - ip) { err = 1; break; }
      L.lits(op, ip, run);
      op += run;
      ip += run;
    }
    if (ip >= cs) break;
    ctrl = L.rd(ip++);
  }
  LZ32_FINISH();
}

// snappy (raw format, format_description.txt of google/snappy; c-blosc 1.21 snappy_wrap_decompress =
// snappy_uncompress): a varint of the uncompressed length, then elements by the tag's low 2 bits —
// 00 literal (length - 1 in the tag's upper 6 bits, or 60..63: in the next 1..4 bytes), 01 copy of
// 4 + ((tag >> 2) & 7) bytes at an 11-bit offset ((tag >> 5) << 8 | next byte), 10 / 11 copy of
// 1 + (tag >> 2) bytes at a 2 / 4-byte little-endian offset. Offset 0 or past the output is an error;
// the output must be exactly the preamble's length and the input consumed exactly.
__global__ __launch_bounds__(64) void k_snappy(ZgItem *subs, uint32_t *sub_status, const uint32_t *sub_kind,
                                               uint32_t n_sub, uint8_t *dst, uint64_t slot) {
  LZ32_SETUP(BL_KIND_SNAPPY);
  uint64_t want = 0;
  // preamble: little-endian base-128 varint (<= 5 bytes, < 2^32)
  for (uint32_t k = 0; !err; k++) {
    if (ip >= cs || k == 5) { err = 1; break; }
    const uint32_t b = L.rd(ip++);
    want |= (uint64_t)(b & 127) << (7 * k);
    if (!(b & 128)) break;
  }
  if (!err && want > cap) err = 1;
  const uint32_t w32 = (uint32_t)want;
  while (!err && ip < cs) {
    const uint32_t tag = L.rd(ip++);
    if ((tag & 3) == 0) {  // literal
      uint64_t len = (tag >> 2) + 1;
      if (len > 60) {
        const uint32_t nb = (uint32_t)len - 60;  // 1..4 length bytes
        if (nb > cs - ip) { err = 1; break; }
        uint64_t v = 0;
        for (uint32_t k = 0; k < nb; k++) v |= (uint64_t)L.rd(ip + k) << (8 * k);
        ip += nb;
        len = v + 1;
      }
      if (len > cs - ip || len > w32 - op) { err = 1; break; }
      L.lits(op, ip, (uint32_t)len);
      ip += (uint32_t)len;
      op += (uint32_t)len;
    } else {
      uint32_t len;
      uint64_t off;
      if ((tag & 3) == 1) {
        if (cs - ip < 1) { err = 1; break; }
        len = 4 + ((tag >> 2) & 7);
        off = ((tag >> 5) << 8) | L.rd(ip);
        ip += 1;
      } else if ((tag & 3) == 2) {
        if (cs - ip < 2) { err = 1; break; }
        len = 1 + (tag >> 2);
        off = L.rd(ip) | (L.rd(ip + 1) << 8);
        ip += 2;
      } else {
        if (cs - ip < 4) { err = 1; break; }
        len = 1 + (tag >> 2);
        off = (uint64_t)L.rd(ip) | ((uint64_t)L.rd(ip + 1) << 8) | ((uint64_t)L.rd(ip + 2) << 16) |
              ((uint64_t)L.rd(ip + 3) << 24);
        ip += 4;
      }
      if (off == 0 || off > op || len > w32 - op) { err = 1; break; }
      L.match(op, (uint32_t)off, len);
      op += len;
    }
  }
  if (!err && op != w32) err = 1;
  LZ32_FINISH();
}

// One workgroup per block: the block's streams (decoded, or stored in the frame) are the shuffled
// block; unshuffle / bitunshuffle into the item's output slot.
__global__ __launch_bounds__(256) void k_blosc_finish(const BlBlock *blocks, const ZgItem *subs,
                                                      const uint32_t *sub_status, const uint32_t *sub_kind,
                                                      uint32_t *status, uint8_t *dst, uint64_t slot_bytes,
                                                      const ZgItem *items, uint8_t *dout, const uint64_t *geom,
                                                      ZgScatter sc, const uint64_t *alias) {
  const BlBlock B = blocks[blockIdx.x];
  __shared__ uint64_t src[256];
  // zstd blocks left where they are (ZstdScratch::alias): stream j's bytes [a_off, a_off + a_len) of
  // entry r are at a_src[j][r] (or all one byte: ZALIAS_RLE)
  __shared__ uint64_t a_src[256][ZALIAS];
  __shared__ uint32_t a_off[256][ZALIAS], a_len[256][ZALIAS];
  __shared__ uint64_t s_row[BL_DIRECT_ROWS];  // direct output: the output address of each row the block covers
  __shared__ uint32_t bad;
  if (threadIdx.x == 0) bad = status[B.item] ? 2u : 0u;  // one read: other blocks may set it meanwhile
  __syncthreads();
  if (bad) return;
  for (uint32_t j = threadIdx.x; j < B.nsplit; j += 256) {
    const uint32_t s = B.first_sub + j;
    const ZgItem it = subs[s];
    if (sub_kind[s] != BL_KIND_RAW && (sub_status[s] != 0 || it.len != B.ne)) bad = 1;
    if (j < 256) {
      src[j] = it.src;
      const bool al = alias && sub_kind[s] == BL_KIND_ZSTD;
      for (uint32_t r = 0; r < ZALIAS; r++) {
        const uint64_t *a = alias + 3 * (ZALIAS * (uint64_t)s + r);
        const uint64_t off = al ? a[1] : 0, len = al ? a[2] : 0;
        const bool ok = len && off + len <= it.len;
        a_src[j][r] = ok ? a[0] : 0ull;
        a_off[j][r] = ok ? (uint32_t)off : 0u;
        a_len[j][r] = ok ? (uint32_t)len : 0u;
      }
    }
  }
  __syncthreads();
  if (bad) {
    if (threadIdx.x == 0) set_status(&status[B.item], ZG_CORRUPT_STREAM);
    return;
  }
  if (B.nsplit > 256) {  // typesize is a u8 header field: cannot happen; keep the guard
    if (threadIdx.x == 0) set_status(&status[B.item], ZG_CORRUPT_STREAM);
    return;
  }
  uint8_t *out = dst + (uint64_t)B.item * slot_bytes + B.out_off;
  const uint32_t ne = B.ne, ts = B.ts, bsize = B.bsize;
  auto in = [&](uint32_t q) -> uint8_t {
    const uint32_t j = ne ? q / ne : 0, l = q - j * ne;
#pragma unroll
    for (uint32_t r = 0; r < ZALIAS; r++) {
      const uint32_t d = l - a_off[j][r];
      if (d < a_len[j][r]) {
        const uint64_t a = a_src[j][r];
        return (a & ZALIAS_RLE) ? (uint8_t)a : ((const uint8_t *)a)[d];
      }
    }
    return ((const uint8_t *)src[j])[l];
  };
  bool aliased = false;
  for (uint32_t j = 0; j < B.nsplit; j++)
    for (uint32_t r = 0; r < ZALIAS; r++) aliased |= a_len[j][r] != 0;
  // direct output: chunk byte c lives in row c / Lb (C order over the chunk's leading axes) at
  // column c mod Lb; the block's rows are resolved once into s_row
  const bool direct = dout && (items[B.item].flags & ZG_ITEM_DIRECT);
  const uint32_t nd = sc.nd;
  const uint32_t Lb = direct ? (uint32_t)(sc.chunk_shape[nd - 1] * sc.es) : 1u;
  const uint32_t c0 = (uint32_t)B.out_off, r0 = c0 / Lb;
  if (direct && bsize) {
    const uint64_t *g = geom + (uint64_t)B.item * 3 * nd;  // sel_start (0) | sel_shape | out_start
    const uint32_t nr = (c0 + bsize - 1) / Lb - r0 + 1;
    for (uint32_t k = threadIdx.x; k < nr; k += 256) {
      uint64_t r = r0 + k, e = g[2 * nd + nd - 1];
      for (int d = (int)nd - 2; d >= 0; d--) {
        const uint64_t ext = sc.chunk_shape[d], c = r % ext;
        r /= ext;
        e += (g[2 * nd + d] + c) * sc.out_stride[d];
      }
      s_row[k] = (uint64_t)dout + e * sc.es;
    }
    __syncthreads();
  }
  auto dptr = [&](uint32_t q) -> uint8_t * {  // destination of block byte q
    if (!direct) return out + q;
    const uint32_t c = c0 + q, r = c / Lb;
    return (uint8_t *)s_row[r - r0] + (c - r * Lb);
  };
  // byte plane i of a shuffled block: one pointer (or one byte value: bit i of rle) when the plane
  // lies inside one aliased range of its stream or outside all of them
  const uint8_t *pl[4];
  uint32_t rle = 0, rle_v[4] = {0, 0, 0, 0};
  bool planes = B.mode == 1 && (ts == 2 || ts == 4) && ne;
  for (uint32_t i = 0; planes && i < ts; i++) {
    const uint32_t neb = bsize / ts, q = i * neb, j = q / ne, l = q - j * ne;
    pl[i] = (const uint8_t *)src[j] + l;
    for (uint32_t r = 0; r < ZALIAS; r++) {
      const uint32_t ao = a_off[j][r], al = a_len[j][r];
      if (!al || l + neb <= ao || l >= ao + al) continue;  // disjoint
      if (l < ao || l + neb > ao + al) {  // straddles the range: the byte loop
        planes = false;
        break;
      }
      const uint64_t a = a_src[j][r];
      if (a & ZALIAS_RLE) {
        rle |= 1u << i;
        rle_v[i] = (uint32_t)(a & 255) * 0x01010101u;
      } else {
        pl[i] = (const uint8_t *)a + (l - ao);
      }
    }
  }
  if (planes && bsize % (16 * ts) == 0 && ((uintptr_t)out & 15) == 0 && (c0 & 15) == 0) {
    // u16 / u32 fast path: 16 elements per thread, a 16-B load from each byte plane and ts 16-B
    // stores of the interleaved bytes (the generic loop below moves a byte per lane with two
    // integer divisions). Planes stored inside the frame (incompressible byte planes, e.g. noise
    // low bytes, or an aliased zstd block) sit at any address: unaligned 16-B global loads (gfx950
    // runs in unaligned mode)
    const uint32_t neb = bsize / ts;
    auto ldv = [&](uint32_t i, uint32_t v) -> uint4 {
      if ((rle >> i) & 1) return make_uint4(rle_v[i], rle_v[i], rle_v[i], rle_v[i]);
      uint4 r;
      __builtin_memcpy(&r, pl[i] + 16ull * v, 16);
      return r;
    };
    {
      // output vector k of the block (16 B, never across a row: rows are 16-B multiples)
      auto o = [&](uint32_t k) -> uint4 & { return *(uint4 *)dptr(16 * k); };
      for (uint32_t v = threadIdx.x; v < neb / 16; v += 256) {
        if (ts == 2) {
          const uint4 a = ldv(0, v), b = ldv(1, v);
          const uint32_t aw[4] = {a.x, a.y, a.z, a.w}, bw[4] = {b.x, b.y, b.z, b.w};
          uint32_t r[8];
#pragma unroll
          for (int k = 0; k < 4; k++) {
            r[2 * k] = (aw[k] & 0xffu) | ((bw[k] & 0xffu) << 8) | ((aw[k] & 0xff00u) << 8) | ((bw[k] & 0xff00u) << 16);
            r[2 * k + 1] = ((aw[k] >> 16) & 0xffu) | (((bw[k] >> 16) & 0xffu) << 8) | ((aw[k] >> 24) << 16) |
                           ((bw[k] >> 24) << 24);
          }
          o(2 * v) = make_uint4(r[0], r[1], r[2], r[3]);
          o(2 * v + 1) = make_uint4(r[4], r[5], r[6], r[7]);
        } else {
          const uint4 p0 = ldv(0, v), p1 = ldv(1, v), p2 = ldv(2, v), p3 = ldv(3, v);
          const uint32_t w0[4] = {p0.x, p0.y, p0.z, p0.w}, w1[4] = {p1.x, p1.y, p1.z, p1.w},
                         w2[4] = {p2.x, p2.y, p2.z, p2.w}, w3[4] = {p3.x, p3.y, p3.z, p3.w};
#pragma unroll
          for (int k = 0; k < 4; k++) {  // output word e of element group k: byte e of each plane
            uint32_t r[4];
#pragma unroll
            for (int e = 0; e < 4; e++)
              r[e] = ((w0[k] >> (8 * e)) & 0xffu) | (((w1[k] >> (8 * e)) & 0xffu) << 8) |
                     (((w2[k] >> (8 * e)) & 0xffu) << 16) | (((w3[k] >> (8 * e)) & 0xffu) << 24);
            o(4 * v + k) = make_uint4(r[0], r[1], r[2], r[3]);
          }
        }
      }
      return;
    }
  }
  if (B.mode == 1) {  // byte unshuffle (shuffle.c unshuffle_generic): dest[j*ts+i] = src[i*neb+j]
    const uint32_t neb = bsize / ts, body = neb * ts;
    for (uint32_t q = threadIdx.x; q < bsize; q += 256) {
      uint8_t v;
      if (q < body) {
        const uint32_t j = q / ts, i = q - j * ts;
        v = in(i * neb + j);
      } else {
        v = in(q);
      }
      *dptr(q) = v;
    }
  } else if (B.mode == 2 && bsize >= ts) {  // bitunshuffle (bshuf_untrans_bit_elem)
    const uint32_t size = bsize / ts;
    const uint32_t n8 = (B.ver == 2) ? ((size % 8) ? 0u : size) : size - size % 8;
    const uint32_t body = n8 * ts, rb = n8 / 8;  // rb: bytes per bit-row
    // Element j, byte b, bit k is bit j of bit-row 8b + k. A thread takes 8 elements (column byte g
    // of every row: coalesced across the threads) and per output byte b transposes the 8x8 bit
    // matrix of rows 8b..8b+7 (three masked swaps of a u64).
    const uint8_t *s0 = (const uint8_t *)src[0];
    const bool one = B.nsplit == 1 && !aliased;
    const bool vec = (ts == 2 || ts == 4) && !direct && ((uintptr_t)out & 15) == 0;
    for (uint32_t g = threadIdx.x; g < rb; g += 256) {
      auto row = [&](uint32_t r) -> uint64_t { return one ? s0[r * rb + g] : in(r * rb + g); };
      uint32_t wd[8];
      for (uint32_t b = 0; b < ts; b++) {
        uint64_t x = 0;
#pragma unroll
        for (uint32_t k = 0; k < 8; k++) x |= row(8 * b + k) << (8 * k);
        uint64_t t = (x ^ (x >> 7)) & 0x00AA00AA00AA00AAull;
        x ^= t ^ (t << 7);
        t = (x ^ (x >> 14)) & 0x0000CCCC0000CCCCull;
        x ^= t ^ (t << 14);
        t = (x ^ (x >> 28)) & 0x00000000F0F0F0F0ull;
        x ^= t ^ (t << 28);  // byte m: bits of element 8g + m's byte b
        if (vec) {
          if (ts == 2) {
#pragma unroll
            for (uint32_t w = 0; w < 4; w++) {
              const uint32_t lo = (uint32_t)(x >> (16 * w)) & 0xffu, hi = (uint32_t)(x >> (16 * w + 8)) & 0xffu;
              wd[w] = b ? wd[w] | (lo << 8) | (hi << 24) : lo | (hi << 16);
            }
          } else {
#pragma unroll
            for (uint32_t m = 0; m < 8; m++) {
              const uint32_t v = ((uint32_t)(x >> (8 * m)) & 0xffu) << (8 * b);
              wd[m] = b ? wd[m] | v : v;
            }
          }
        } else {
          for (uint32_t m = 0; m < 8; m++) *dptr((8 * g + m) * ts + b) = (uint8_t)(x >> (8 * m));
        }
      }
      if (vec) {
        uint4 *o4 = (uint4 *)(out + 8ull * g * ts);
        o4[0] = make_uint4(wd[0], wd[1], wd[2], wd[3]);
        if (ts == 4) o4[1] = make_uint4(wd[4], wd[5], wd[6], wd[7]);
      }
    }
    for (uint32_t q = body + threadIdx.x; q < bsize; q += 256) *dptr(q) = in(q);
  } else {
    for (uint32_t q = threadIdx.x; q < bsize; q += 256) *dptr(q) = in(q);
  }
}

hipError_t launch_blosc_info(const ZgItem *items, uint32_t *status, uint32_t n_items, uint64_t slot_bytes,
                             BlInfo *info, hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_blosc_info, dim3((n_items + 63) / 64), dim3(64), 0, s, items, status, n_items, slot_bytes,
                     info);
  return hipGetLastError();
}

hipError_t launch_blosc_layout(const BlInfo *info, uint32_t n_items, uint64_t *bases, const BlCaps &caps,
                               const BlDecode &D, hipStream_t s) {
  if (!n_items) return hipSuccess;
  hipLaunchKernelGGL(k_blosc_layout, dim3(1), dim3(1024), 0, s, info, n_items, bases, caps, D.sub_status, D.sub_kind,
                     D.blocks, D.ovf);
  return hipGetLastError();
}

hipError_t launch_blosc_decode(ZgItem *items, uint32_t *status, uint32_t n_items, const BlInfo *info,
                               const BlDecode &D, uint8_t *dst, uint64_t slot_bytes, hipStream_t s) {
  if (!n_items) return hipSuccess;
  const uint32_t direct = D.dout ? 1u : 0u;
  const uint64_t want = D.sc.nelem * D.sc.es, row_bytes = direct ? D.sc.chunk_shape[D.sc.nd - 1] * D.sc.es : 1;
  hipLaunchKernelGGL(k_blosc_streams, dim3(n_items), dim3(64), 0, s, items, status, info, D.bases, D.subs,
                     D.sub_status, D.sub_kind, D.blocks, dst, slot_bytes, D.ovf, direct, want, row_bytes, D.need,
                     D.blocks_decoded);
  if (D.n_zstd) {
    hipError_t e = launch_zstd(D.subs, D.sub_status, (uint32_t)D.n_sub, D.tmp, D.sub_slot, D.zs, s);
    if (e != hipSuccess) return e;
  }
  if (D.n_lz4 && D.lz_list && ZG_LZM_G < 64) {
    uint32_t *wl = D.lz_list + D.n_sub + 1;  // the wide list
    hipLaunchKernelGGL(k_lz_list, dim3(1), dim3(1024), 0, s, D.subs, D.sub_kind, D.sub_status, (uint32_t)D.n_sub,
                       (uint32_t)BL_KIND_LZ4, 0u, D.lz_list);
    hipLaunchKernelGGL(k_lz_list, dim3(1), dim3(1024), 0, s, D.subs, D.sub_kind, D.sub_status, (uint32_t)D.n_sub,
                       (uint32_t)BL_KIND_LZ4, 1u, wl);
    constexpr uint32_t NG = 64 / ZG_LZM_G;
    hipLaunchKernelGGL(k_lz4m<ZG_LZM_G>, dim3((uint32_t)((D.n_sub + NG - 1) / NG)), dim3(64), 0, s, D.subs,
                       D.sub_status, D.lz_list, D.tmp, D.sub_slot);
    hipLaunchKernelGGL(k_lz4m<64>, dim3((uint32_t)D.n_sub), dim3(64), 0, s, D.subs, D.sub_status, wl, D.tmp,
                       D.sub_slot);
  } else if (D.n_lz4) {
    hipLaunchKernelGGL(k_lz4, dim3((uint32_t)D.n_sub), dim3(64), 0, s, D.subs, D.sub_status, D.sub_kind,
                       (uint32_t)D.n_sub, D.tmp, D.sub_slot);
  }
  if (D.n_zlib) {
    hipError_t e = launch_zlib_streams(D.subs, D.sub_status, D.sub_kind, (uint32_t)D.n_sub, D.tmp, D.sub_slot, D.zaux, D.zseg, s);
    if (e == hipSuccess) e = launch_adler32_check(D.subs, D.sub_status, D.sub_kind, (uint32_t)D.n_sub, D.zaux, s);
    if (e != hipSuccess) return e;
  }
  if (D.n_snappy && D.lz_list && ZG_LZM_G < 64) {
    uint32_t *wl = D.lz_list + D.n_sub + 1;  // the wide list
    hipLaunchKernelGGL(k_lz_list, dim3(1), dim3(1024), 0, s, D.subs, D.sub_kind, D.sub_status, (uint32_t)D.n_sub,
                       (uint32_t)BL_KIND_SNAPPY, 0u, D.lz_list);
    hipLaunchKernelGGL(k_lz_list, dim3(1), dim3(1024), 0, s, D.subs, D.sub_kind, D.sub_status, (uint32_t)D.n_sub,
                       (uint32_t)BL_KIND_SNAPPY, 1u, wl);
    constexpr uint32_t NG = 64 / ZG_LZM_G;
    hipLaunchKernelGGL(k_snappym<ZG_LZM_G>, dim3((uint32_t)((D.n_sub + NG - 1) / NG)), dim3(64), 0, s, D.subs,
                       D.sub_status, D.lz_list, D.tmp, D.sub_slot);
    hipLaunchKernelGGL(k_snappym<64>, dim3((uint32_t)D.n_sub), dim3(64), 0, s, D.subs, D.sub_status, wl, D.tmp,
                       D.sub_slot);
  } else if (D.n_snappy) {
    hipLaunchKernelGGL(k_snappy, dim3((uint32_t)D.n_sub), dim3(64), 0, s, D.subs, D.sub_status, D.sub_kind,
                       (uint32_t)D.n_sub, D.tmp, D.sub_slot);
  }
  if (D.n_blosclz && D.lz_list && ZG_LZM_G < 64) {
    uint32_t *wl = D.lz_list + D.n_sub + 1;  // the wide list
    hipLaunchKernelGGL(k_lz_list, dim3(1), dim3(1024), 0, s, D.subs, D.sub_kind, D.sub_status, (uint32_t)D.n_sub,
                       (uint32_t)BL_KIND_BLOSCLZ, 0u, D.lz_list);
    hipLaunchKernelGGL(k_lz_list, dim3(1), dim3(1024), 0, s, D.subs, D.sub_kind, D.sub_status, (uint32_t)D.n_sub,
                       (uint32_t)BL_KIND_BLOSCLZ, 1u, wl);
    constexpr uint32_t NG = 64 / ZG_LZM_G;
    hipLaunchKernelGGL(k_blosclzm<ZG_LZM_G>, dim3((uint32_t)((D.n_sub + NG - 1) / NG)), dim3(64), 0, s, D.subs,
                       D.sub_status, D.lz_list, D.tmp, D.sub_slot);
    hipLaunchKernelGGL(k_blosclzm<64>, dim3((uint32_t)D.n_sub), dim3(64), 0, s, D.subs, D.sub_status, wl, D.tmp,
                       D.sub_slot);
  } else if (D.n_blosclz) {
    hipLaunchKernelGGL(k_blosclz, dim3((uint32_t)D.n_sub), dim3(64), 0, s, D.subs, D.sub_status, D.sub_kind,
                       (uint32_t)D.n_sub, D.tmp, D.sub_slot);
  }
  if (D.n_blk)
    hipLaunchKernelGGL(k_blosc_finish, dim3((uint32_t)D.n_blk), dim3(256), 0, s, D.blocks, D.subs, D.sub_status,
                       D.sub_kind, status, dst, slot_bytes, items, D.dout, D.geom, D.sc,
                       D.n_zstd ? D.zs.alias : nullptr);
  return hipGetLastError();
}

}  // namespace zgpu
