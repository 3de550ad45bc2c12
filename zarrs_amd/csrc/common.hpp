// Shared host/device definitions for the zgpu decode pipeline (gfx950).
//
// Device data layout (one "plan" = one batch of chunk descriptors):
//   Item[n_items]      leaf chunk work items (a plain chunk, or one inner chunk of a shard):
//                      current encoded byte range {src,len} that each b2b stage rewrites in place
//   geom[n_items][3*nd] u64: sel_start (leaf-chunk relative), sel_shape, out_start (output array)
//   status[n_items]    u32 per-item status (0 = ok; first error sticks, later stages skip)
//   Shard[n_shards]    sharded descriptors: encoded shard {ptr,len}; index decoded into
//   index[n_shards][n_inner*2] u64 (offset, nbytes) per inner chunk, C order of inner coords
#pragma once
#include <stdint.h>

#define ZG_MAXD 8

// item flags
#define ZG_ITEM_FILL 0x1u     // write the fill value (missing chunk / empty inner chunk)
#define ZG_ITEM_PARTIAL 0x2u  // partial-decoder path: crc32c strips without verifying
#define ZG_ITEM_SHARDED 0x4u  // src/len resolved on device from the shard index
#define ZG_ITEM_DIRECT 0x8u   // already written into the output by its last stage: the scatter skips it

struct ZgItem {
  uint64_t src;    // device address of the current encoded bytes
  uint64_t len;    // current byte length
  uint32_t desc;   // owning descriptor
  uint32_t flags;  // ZG_ITEM_*
  uint32_t shard;  // shard slot (sharded items)
  uint32_t inner;  // inner chunk linear index inside the shard
};

struct ZgShard {
  uint64_t ptr;  // device address of the encoded shard
  uint64_t len;
};

// Parameters of the final fused stage: bytes codec (endianness) + transpose(s) + scatter
// into the output subset (+ an innermost numcodecs.shuffle when it sits directly above bytes).
struct ZgScatter {
  uint32_t nd;
  uint32_t es;        // element size (bytes)
  uint32_t comp;      // component size for endianness swap
  uint32_t swap;      // 1: stored big-endian -> reverse each component
  uint32_t shuffle;   // 1: fused unshuffle with elementsize == es
  uint32_t tile_a;    // decoded axis that is innermost in the encoded layout (tiled kernel)
  uint32_t tile_b;    // tiled kernel: axis batched TJ slabs per block (smallest encoded stride
                      // among the other axes: adjacent slabs are adjacent encoded rows); ZG_MAXD = none
  uint32_t pad0;      // u16 unshuffle A/B (ZGPU_UNSHUFFLE_WIDE): 0 8-B plane loads, 1 / 2 16-B (nt / plain)
  uint64_t chunk_shape[ZG_MAXD];  // leaf decoded shape
  uint64_t enc_stride[ZG_MAXD];   // encoded linear stride (elements) of each decoded axis
  uint64_t out_stride[ZG_MAXD];   // output array C strides (elements)
  uint64_t nelem;                 // elements per leaf chunk
  uint8_t fill[16];
};

// k_gzip writing whole chunks straight into the output rows (the gzip stage last before a rows scatter
// with no swap / shuffle / transpose): an item whose selection is its whole chunk and whose output
// rows are 16-B aligned is decoded into the array, flagged ZG_ITEM_DIRECT, and the scatter skips it.
// Chunk byte p lives in row p >> lbs (C order over the leading axes) at column p & (2^lbs - 1).
struct GzDirect {
  uint8_t *dout;         // output array; nullptr: every item decodes into its slot
  const uint64_t *geom;  // per item: sel_start | sel_shape | out_start (ZG_MAXD-free: 3 * nd)
  uint64_t want;         // decoded bytes of a whole chunk
  uint64_t cshape[4];    // chunk shape
  uint64_t ostr[4];      // output byte stride of each axis
  uint32_t nd;           // <= 3 (axis 1 of a 3-d chunk has a power-of-two extent); byte strides < 4 GiB
  uint32_t lbs;          // log2 of the row bytes (chunk_shape[nd-1] * es, >= 16)
};

// device status codes (== zgpu.h)
#define ZG_OK 0u
#define ZG_INVALID_CHECKSUM 1u
#define ZG_DECODED_SIZE_MISMATCH 2u
#define ZG_SHARD_INDEX_OOB 3u
#define ZG_CORRUPT_STREAM 4u
#define ZG_INVALID_BYTE_RANGE 5u
#define ZG_UNSUPPORTED 6u
#define ZG_CRC_INPUT_TOO_SHORT 7u
#define ZG_SHARD_TOO_SMALL 8u
#define ZG_SHUFFLE_LENGTH 9u
