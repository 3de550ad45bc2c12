// Host-callable launchers of the gfx950 kernels (defined in the .hip translation units).
#pragma once
#include <hip/hip_runtime.h>

#include "../common.hpp"

#include <cstdlib>

namespace zgpu {

// Largest grid (in blocks of `threads`) one launch may use: gridDim.x * blockDim.x must stay below
// 2^32 on HIP, so bigger block ranges are launched in slices. ZGPU_MAX_GRID lowers it (tests force
// the sliced launches with it).
inline uint64_t max_grid_blocks(uint32_t threads) {
  uint64_t m = (0xFFFFFFFFull / threads) & ~(uint64_t)0xFFF;
  if (const char *e = std::getenv("ZGPU_MAX_GRID")) {
    const uint64_t v = std::strtoull(e, nullptr, 10);
    if (v && v < m) m = v;
  }
  return m;
}

// Compute units of the current device (queried once per device; grids sized to the chip, not a
// hard-coded 256).
inline uint32_t device_cu_count() {
  static uint32_t cache[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (!cache[dev]) {
    int n = 0;
    if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
    cache[dev] = (uint32_t)n;
  }
  return cache[dev];
}

enum ScatterMode : uint32_t { SCATTER_ROWS = 0, SCATTER_TILED = 1, SCATTER_GENERIC = 2 };
// slabs (TILE x TILE tiles at consecutive values of ZgScatter::tile_b) per tiled-scatter block
constexpr __host__ __device__ int tiled_slabs(uint32_t es) { return es == 8 ? 2 : 4; }

hipError_t launch_scatter(const ZgItem *items, const uint64_t *geom, uint32_t *status, const ZgScatter &P,
                          uint8_t *out, uint32_t n_items, uint32_t mode, uint64_t units_per_item,
                          hipStream_t s, uint32_t *live_scratch = nullptr);  // (n_items + 1) u32: rows mode
                                                                            // over the items not yet written
uint64_t scatter_units_per_item(uint32_t mode, const ZgScatter &P, const uint64_t *max_sel_shape);

// Box copy between device arrays: run r (C order over the `outer` axes of `shape`) is run_bytes
// contiguous bytes at src_base + sum(c_d * src_stride[d]) -> dst_base + sum(c_d * dst_stride[d]).
struct ZgBoxCopy {
  uint32_t outer, pad0;
  uint64_t shape[ZG_MAXD], src_stride[ZG_MAXD], dst_stride[ZG_MAXD];
  uint64_t src_base, dst_base, run_bytes, n_runs;
};
hipError_t launch_box_copy(const uint8_t *src, uint8_t *dst, const ZgBoxCopy &P, hipStream_t s);

// crc32c (Castagnoli) verify + strip of a 4-byte LE checksum at the start or end of each item.
// verify: 0 never, 1 unless the item is on the partial path.
hipError_t launch_crc32c_strip(ZgItem *items, uint32_t *status, uint32_t n_items, int at_start, int verify,
                               hipStream_t s);

// Shard index: decode every shard's index (bytes{endian} + optional crc32c chain), then resolve
// each sharded item's {src,len} or fill flag.  index_crc: 0 none, 1 end, 2 start.
struct ZgIndexSpec {
  uint64_t n_inner;      // inner chunks per shard
  uint64_t index_bytes;  // encoded index size (incl. checksums)
  uint32_t at_start;     // sharding index_location
  uint32_t big_endian;   // index bytes codec endianness
  uint32_t n_crc;        // number of crc32c codecs in the index chain (<= 4)
  uint32_t crc_at_start[4];
  uint32_t verify;       // validate_checksums
};
// keep_err: shards whose status is already non-zero keep it and are skipped (nested sharding's
// middle level, whose statuses come from resolving them through the outer index)
hipError_t launch_shard_index(const ZgShard *shards, uint32_t n_shards, const ZgIndexSpec &spec,
                              uint64_t *index, uint32_t *shard_status, int keep_err, hipStream_t s);
// nested sharding: resolved middle-shard records -> a shard table ({0,0} when empty) + statuses
hipError_t launch_mid_shards(const ZgItem *mids, const uint32_t *mid_status, uint32_t n, ZgShard *shards,
                             uint32_t *shard_status, hipStream_t s);
hipError_t launch_item_resolve(ZgItem *items, uint32_t *status, uint32_t n_items, const ZgShard *shards,
                               const uint64_t *index, const uint32_t *shard_status, uint64_t n_inner,
                               unsigned long long *enc_bytes, hipStream_t s);

// gzip (RFC 1952) member decode: header parse, DEFLATE inflate into dst slots, trailer CRC-32 (IEEE)
// + ISIZE check of the inflated bytes. On return items[i] points at its slot.
// order: n_items u32 of scratch for the LPT dispatch order (descending encoded length), or NULL
// seg_scr: gzip_seg_scratch_bytes(n_items) of record scratch for the segmented symbol decode (NULL:
// the lookahead decode); 0 bytes when that path is off (ZGPU_GZIP_SEG=0)
uint64_t gzip_seg_scratch_bytes(uint32_t n_items);
// A trailing crc32c verified on a side stream beside the one-wave gzip kernel (GzCrcFork; nullptr: by
// k_crc32c_strip ahead of it): snapshots of n_items items and statuses, n_items flags.
struct GzCrcFork {
  hipStream_t side;
  hipEvent_t ev_fork, ev_join;
  ZgItem *snap_items;
  uint32_t *snap_status, *bad;
};
hipError_t launch_crc32c_check(const ZgItem *items, const uint32_t *status, uint32_t *bad, uint32_t n_items,
                               hipStream_t s);
hipError_t launch_crc32c_merge(uint32_t *status, const uint32_t *bad, uint32_t n_items, hipStream_t s);
hipError_t launch_gzip(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                       uint32_t *order, uint32_t *seg_scr, hipStream_t s, int crc_tail = 0,
                       const GzDirect *direct = nullptr,  // direct: whole chunks into the output rows
                       const GzCrcFork *crc_fork = nullptr);
// zstd (RFC 8878) frame decode into dst slots: block-parallel (scan, per-block entropy decode,
// per-item execution) with the serial one-wave-per-item decoder as the fallback.
struct ZstdScratch {
  void *blks;            // n_items * blk_cap block records
  uint32_t *nblk, *mode;  // per item
  uint8_t *lit;          // n_items * lit_stride literal scratch
  uint64_t lit_stride;
  uint32_t *seq;         // n_items * seq_cap sequences of 3 u32
  uint64_t seq_cap;
  uint32_t blk_cap;
  int16_t *norm = nullptr;  // n_items * blk_cap * zstd_norm_bytes(): FSE counts the scan parsed (nullable)
  uint32_t force_serial = 0;               // every item on the serial one-wave decoder (tests, ZGPU_ZSTD_FORCE_SERIAL)
  unsigned long long *counters = nullptr;  // [serial-fallback items, block-parallel items] (nullable)
  // compacted serial-fallback items (nullable: the fallback then runs one wave per item): k_zstd_scan
  // appends them, the fallback is a small persistent grid over the list, launched only when
  // launch_serial (a plan whose last execution had no serial item skips it and re-runs on the flag)
  uint32_t *ser_list = nullptr;
  unsigned long long *ser_count = nullptr;
  uint32_t launch_serial = 1;
  // Fork for the sequence decoder (nullable: one stream): k_zstd_blocks needs only the scan, so it
  // runs on `side` beside the Huffman literal kernels and joins before k_zstd_plan
  hipStream_t side = nullptr;
  hipEvent_t ev_fork = nullptr, ev_join = nullptr;
  // one stream only: Huffman literals before the sequences (ZGPU_ZSTD_LITS_FIRST; the literal decoder
  // then writes literal-only blocks to the scratch, as k_zstd_plan has not placed them yet)
  uint32_t lits_first = 0;
  // literal record slots (k_zstd_lits pass 1 keeps its symbols; nullable: every lane decodes twice):
  // zstd_lit_rec_bytes() bytes for lit_rec_wgs workgroups
  uint8_t *lit_rec = nullptr;
  uint32_t lit_rec_wgs = 0;
  // Block aliases (nullable; the blosc stage sets it: its consumer k_blosc_finish reads the decoded
  // streams itself). Per item ZALIAS entries {src, off, len}: a block that needs no execution (raw,
  // rle, or literals only), that no later match reads and no checksum covers, is left where its
  // bytes already are (in the frame or the literal scratch; rle: src = ZALIAS_RLE | byte) and
  // k_zstd_direct does not copy it into the slot: item bytes [off, off + len) are src[0 .. len).
  // len = 0: none. Byte-shuffled blosc blocks of noisy data: the low-byte plane is a raw block.
  uint64_t *alias = nullptr;
  // Two halves (nullable s2: one pass): the second half of the items runs on stream s2, its entropy
  // kernels after the first half's (ev_half), beside the first half's executor; the caller's stream
  // waits for ev_done. Both halves share the side stream and the literal record slots (their literal
  // kernels never overlap).
  hipStream_t s2 = nullptr;
  hipEvent_t ev_half = nullptr, ev_done = nullptr;
  // the batch's largest block count per item (nullable; zeroed before the call, k_zstd_scan's
  // atomicMax): the record-strided kernels walk n_items x that many records, not x blk_cap
  unsigned long long *max_nblk = nullptr;
  // Latency mode of the window executor (nullable: off): two ext arrays of ext_items * slot u32 each
  // (the external references of k_zstd_exec_win<true>) and ZEXT_ROUNDS round counters
  uint32_t *ext = nullptr;
  unsigned long long *ext_cnt = nullptr;
  uint64_t ext_items = 0;
};
constexpr uint32_t ZALIAS = 2;
// latency mode: batches of at most this many decoded bytes (n_items x slot) get the ext arrays
constexpr uint64_t ZPAR_MAX_BYTES = 128ull << 20;
constexpr uint32_t ZEXT_ROUNDS = 24;
constexpr uint64_t ZALIAS_RLE = 1ull << 63;
uint64_t zstd_lit_rec_bytes(uint32_t &wgs);
// bytes of FSE-count scratch per block record (ZstdScratch::norm)
uint64_t zstd_norm_bytes();
void zstd_scratch_layout(uint64_t slot_bytes, uint32_t &blk_cap, uint64_t &blk_bytes, uint64_t &lit_stride,
                         uint64_t &seq_cap);
hipError_t launch_zstd(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                       const ZstdScratch &Z, hipStream_t s);
// standalone unshuffle (when shuffle is not directly above the bytes codec)
hipError_t launch_unshuffle(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *dst, uint64_t slot_bytes,
                            uint32_t elementsize, hipStream_t s);
// decoded-size hint per item of a whole-shard compressor stage (kernels/probe.hip); 0 = unknown
enum : uint32_t { SIZE_HINT_GZIP = 0, SIZE_HINT_ZSTD = 1, SIZE_HINT_BLOSC = 2 };
hipError_t launch_size_hint(const ZgItem *items, const uint32_t *status, uint32_t n, uint32_t kind, uint64_t *hint,
                            hipStream_t s);

// encode (write path): array -> encoded chunk layouts (transposes, endianness, innermost shuffle)
struct ZgEncode {
  uint32_t nd, es, comp, swap, shuffle, aligned;
  uint32_t tile_b, pad0;             // tiled encode: decoded axis batched TJ slabs per block (ZG_MAXD: none)
  uint64_t nelem;                    // elements per chunk
  uint64_t data_off;                 // bytes before the data in each chunk (crc32c at start)
  uint64_t enc_shape[ZG_MAXD];       // encoded (transposed) chunk shape
  uint32_t dec_axis[ZG_MAXD];        // encoded axis a is decoded axis dec_axis[a]
  uint64_t array_shape[ZG_MAXD];
  uint64_t array_stride[ZG_MAXD];    // elements
  uint64_t dec_shape[ZG_MAXD];       // chunk shape (decoded axes)
  uint64_t enc_stride_of_dec[ZG_MAXD];  // encoded linear stride (elements) of each decoded axis
  uint8_t fill[16];
};
hipError_t launch_encode_gather(const uint64_t *dsts, const uint64_t *starts, const uint8_t *array,
                                const ZgEncode &P, uint32_t n_chunks, hipStream_t s);
hipError_t launch_crc32c_encode(const uint64_t *dsts, uint32_t n, uint64_t lo, uint64_t len, int at_start,
                                hipStream_t s);
// sharding_indexed encode of fixed-size inner chains: fill check of every inner chunk (geometry of
// `inner`, origins `starts`), C-order layout + raw index per shard, copy of the encoded inner chunks
// (temporary slots of E_pitch bytes) into the shards. The index crc32c codecs run afterwards
// (launch_crc32c_encode over index_ptr).
struct ZgShardLayoutArgs {
  uint64_t n_inner, E, E_pitch, index_bytes, pre;
  uint32_t at_start, big_endian;
};
hipError_t launch_shard_encode(const uint64_t *starts, const uint8_t *array, const ZgEncode &inner, uint32_t n_chunks,
                               uint32_t *nonfill, const uint8_t *tmp, const ZgShardLayoutArgs &A,
                               const uint64_t *shard_dst, uint64_t *inner_off, uint64_t *index_ptr,
                               uint64_t *shard_len, uint32_t n_shards, hipStream_t s);

// ---- variable-length write path (compressing chains) ----
// gzip member encode (deflate_enc.hip): item i's bytes -> a member written at slot i + GZE_HDR (the
// headroom takes crc32c codecs located at the start), items rewritten to it. sym_scratch holds
// gzip_encode_grid(n) * GZE_BLK_SYMS u32 symbol records. zlib: a zlib stream (RFC 1950, Adler-32
// trailer) at slot i + GZE_HDR + 8 instead of a gzip member (blosc's zlib streams).
constexpr uint32_t GZE_BLK_SYMS = 16384;  // symbols per DEFLATE block
constexpr uint64_t GZE_HDR = 62;          // member offset in a slot (its bit stream then starts word-aligned)
uint32_t gzip_encode_grid(uint32_t n_items);
hipError_t launch_gzip_encode(ZgItem *items, uint32_t *status, uint32_t n_items, uint8_t *slots, uint64_t slot_bytes,
                              uint32_t *sym_scratch, int level, hipStream_t s, bool zlib = false);
// zstd frame encode (zstd_enc.hip): item i's bytes (at most max_len) -> one single-segment frame at
// slot i + ZE_HDR, items rewritten to it; the work is cut into 1 MiB segments, one wave each.
// scratch: zstd_encode_scratch(n_items, max_len) bytes
constexpr uint64_t ZE_HDR = 64;
uint64_t zstd_encode_scratch(uint32_t n_items, uint64_t max_len);
hipError_t launch_zstd_encode(ZgItem *items, uint32_t *status, uint32_t n_items, uint64_t max_len, uint8_t *slots,
                              uint64_t slot_bytes, uint8_t *scratch, int checksum, hipStream_t s);
// crc32c of each item's bytes written after them (or before them with at_start: src moves back 4)
hipError_t launch_crc32c_items(ZgItem *items, const uint32_t *status, uint32_t n, int at_start, hipStream_t s);
// each item's bytes into dst[i] (capacity cap[i], else DECODED_SIZE_MISMATCH); lens[i] = length
hipError_t launch_encode_place(const ZgItem *items, uint32_t *status, const uint64_t *dst, const uint64_t *cap,
                               uint64_t *lens, uint32_t n, hipStream_t s);
// fill check of every inner chunk (launch_shard_encode's first kernel)
hipError_t launch_fill_check(const uint64_t *starts, const uint8_t *array, const ZgEncode &inner, uint32_t n_chunks,
                             uint32_t *nonfill, hipStream_t s);
// sharding_indexed layout over inner chunks of variable length (items, n_shards * n_inner of them);
// A.E_pitch = a shard destination's capacity. shard_status: 0, 1 (an inner chunk failed), or
// DECODED_SIZE_MISMATCH (capacity); a failed shard gets index_ptr 0 (the index crc launch skips it)
hipError_t launch_shard_encode_var(const uint64_t *starts, const uint8_t *array, const ZgEncode &inner,
                                   uint32_t n_chunks, uint32_t *nonfill, const ZgItem *items,
                                   const uint32_t *item_status, const ZgShardLayoutArgs &A, const uint64_t *shard_dst,
                                   uint64_t *inner_off, uint64_t *index_ptr, uint64_t *shard_len,
                                   uint32_t *shard_status, uint32_t n_shards, hipStream_t s);

// blosc (c-blosc 1.x frames): stream table built on the device, sized on the host from BlInfo (first
// execution of a plan) or from the capacities that execution recorded (later executions)
enum : uint32_t { BL_COMP_BLOSCLZ = 0, BL_COMP_LZ4 = 1, BL_COMP_SNAPPY = 2, BL_COMP_ZLIB = 3, BL_COMP_ZSTD = 4, BL_COMP_MEMCPY = 0x100,
                  BL_COMP_SKIP = 0xFFFFFFFFu };
#define BL_SKIP 0x100u  // stream status: not (yet) decoded by the zstd pipeline / a stream decoder
enum : uint32_t { BL_KIND_RAW = 0, BL_KIND_LZ4 = 1, BL_KIND_SNAPPY = 2, BL_KIND_ZLIB = 3, BL_KIND_ZSTD = 4,
                  BL_KIND_BLOSCLZ = 5 };
struct BlInfo {     // per item (read back)
  uint32_t nsub;    // compressed streams
  uint32_t nblk;    // blocks
  uint32_t comp;    // BL_COMP_*
  uint32_t max_ne;  // largest stream decoded size
  uint32_t nbytes;  // decoded size
  uint32_t ver;     // frame format version
};
struct BlBlock {
  uint32_t item, bsize;
  uint64_t out_off;  // in the item's decoded bytes
  uint32_t first_sub, nsplit, ne, mode, ts, ver;  // mode 0 none, 1 byte unshuffle, 2 bitunshuffle
};
constexpr uint32_t BL_SUB_WIDE = 0x80000000u;  // stream ZgItem flag: decode it with a whole wave
struct BlDecode {
  const uint64_t *bases;  // per item {first stream, first block}
  ZgItem *subs;
  uint32_t *sub_status, *sub_kind;
  BlBlock *blocks;
  uint8_t *tmp;           // n_sub * sub_slot decoded streams
  uint64_t sub_slot;
  ZstdScratch zs;
  uint64_t n_sub, n_blk, n_zstd, n_lz4, n_blosclz, n_zlib, n_snappy;  // with a cached layout: capacities (n_* > 0 = launched)
  uint2 *zaux;            // zlib streams: {Adler-32 trailer, -} per stream
  uint32_t *zseg;         // zlib streams: the segmented symbol decode's record scratch (nullable)
  uint32_t *lz_list;      // lz4 / blosclz / snappy streams: {count, stream indices} (k_lz_list), two lists of
                          // n_sub + 1 entries: streams decoded two per wave, then bitshuffled ones (BL_SUB_WIDE)
  unsigned long long *ovf;  // set by k_blosc_layout when a cached layout is too small (ctl counter)
  // Direct output (dout non-null): blosc is the last stage and the scatter would copy whole chunks'
  // rows unchanged (rows kernel, no swap / shuffle / transpose, 16-B aligned rows; checked on the
  // host). An item whose decoded size is right and whose blocks span at most BL_DIRECT_ROWS rows is
  // marked ZG_ITEM_DIRECT by k_blosc_streams; k_blosc_finish then writes its unshuffled blocks
  // straight into the output rows (geom: the plan's per-item geometry, sc: its scatter parameters).
  uint8_t *dout;
  const uint64_t *geom;
  ZgScatter sc;
  // per item the decoded byte range [need[2i], need[2i+1]) its selection needs (nullable: all); blocks
  // outside it are neither parsed nor decoded. blocks_decoded counts the decoded blocks (ctl counter)
  const uint64_t *need;
  unsigned long long *blocks_decoded;
};
constexpr uint32_t BL_DIRECT_ROWS = 2048;  // rows per block (LDS row table of k_blosc_finish)
// Capacities of a blosc stream table sized by an earlier execution of the same plan: the layout of
// this execution is computed on the device (k_blosc_layout) and checked against them, so the stage
// needs no host read-back. BL_KINDS_*: compressors the earlier execution launched decoders for.
enum : uint32_t { BL_HAS_ZSTD = 1, BL_HAS_LZ4 = 2, BL_HAS_BLOSCLZ = 4, BL_HAS_ZLIB = 8, BL_HAS_SNAPPY = 16 };
struct BlCaps {
  uint64_t n_sub, n_blk, max_ne;
  uint32_t kinds;
};
// zlib (RFC 1950) streams of a blosc stream table: DEFLATE by the k_gzip machinery (streams whose
// kind is BL_KIND_ZLIB and status BL_SKIP; status 0 on success), then the Adler-32 trailer check
hipError_t launch_zlib_streams(ZgItem *subs, uint32_t *sub_status, const uint32_t *sub_kind, uint32_t n_sub,
                               uint8_t *dst, uint64_t slot, uint2 *aux, uint32_t *seg_scr, hipStream_t s);
hipError_t launch_adler32_check(const ZgItem *subs, uint32_t *sub_status, const uint32_t *sub_kind, uint32_t n_sub,
                                const uint2 *aux, hipStream_t s);
hipError_t launch_blosc_layout(const BlInfo *info, uint32_t n_items, uint64_t *bases, const BlCaps &caps,
                               const BlDecode &D, hipStream_t s);
hipError_t launch_blosc_info(const ZgItem *items, uint32_t *status, uint32_t n_items, uint64_t slot_bytes,
                             BlInfo *info, hipStream_t s);
hipError_t launch_blosc_decode(ZgItem *items, uint32_t *status, uint32_t n_items, const BlInfo *info,
                               const BlDecode &D, uint8_t *dst, uint64_t slot_bytes, hipStream_t s);

// blosc encode (blosc_enc.hip): item i's nbytes -> one c-blosc 1.x frame at slot i + BLE_HDR, items
// rewritten to it. comp: BL_COMP_BLOSCLZ, BL_COMP_LZ4 (lz4 / lz4hc streams), BL_COMP_ZLIB or BL_COMP_ZSTD;
// shuffle 0 / 1 byte / 2 bit
constexpr uint64_t BLE_HDR = 64;
struct BloscEnc {
  uint32_t comp, shuffle, ts, nsplit, nblk, spi;  // spi: streams per item
  uint64_t nbytes, bs, ne_max;
};
BloscEnc blosc_enc_params(uint32_t comp, uint32_t shuffle, uint32_t ts, uint64_t nbytes, uint64_t blocksize);
uint64_t blosc_encode_scratch(const BloscEnc &E, uint32_t n_items);
hipError_t launch_blosc_encode(ZgItem *items, uint32_t *status, uint32_t n_items, const BloscEnc &E, uint8_t *slots,
                               uint64_t slot_bytes, uint8_t *scratch, int zlevel, hipStream_t s);

}  // namespace zgpu
