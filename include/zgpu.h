/*
 * zgpu.h — C ABI of the MI355X-native Zarr chunk-decode codec pipeline (libzgpu.so).
 *
 * This is the drop-in boundary that a zarrs runtime codec plugin binds (see INTEGRATION.md for
 * the Rust FFI stub). Plain pointers and sizes only; no torch or HIP types in any signature.
 * Reference interfaces replaced (paths relative to the zarrs workspace root):
 *
 *   zgpu_chain_create   <- CodecChain::from_metadata + CodecChain::with_context
 *                          (zarrs/src/array/codec/array_to_bytes/codec_chain.rs:105-169,192-229),
 *                          Codec::from_metadata via the runtime registry
 *                          (zarrs_codec/src/lib.rs:279-318,372-449)
 *   zgpu_decode_batch   <- CodecChainBound::decode_into (codec_chain.rs:592-646) for full chunks and
 *                          ArrayPartialDecoderTraits::partial_decode_into
 *                          (zarrs_codec/src/codec_traits/array_partial_sync.rs:66-129) for partial
 *                          selections; for a sharding_indexed chain, ShardingCodecBound::decode_into
 *                          (sharding/sharding_codec.rs:617-707) and ShardingPartialDecoder
 *                          (sharding/sharding_partial_decoder_sync.rs:311-400). Batched: one call
 *                          decodes many chunks (per-chunk calls are a degenerate batch).
 *   zgpu_retrieve_array_subset
 *                       <- Array::retrieve_array_subset_into (zarrs/src/array/array_ops/
 *                          array_read_ops_common.rs:20-179, array_read_ops_array.rs:231-375):
 *                          the array-level batched driver that feeds zgpu_decode_batch.
 *   zgpu_decode_files / zgpu_retrieve_array_subset_files
 *                       <- the same, with the encoded chunks read from a filesystem store:
 *                          FilesystemStore::get / get_partial_many (zarrs_filesystem/src/lib.rs:
 *                          323-470) feeding array_read_ops_array.rs:290-300, with the reads of
 *                          one sub-batch overlapped with the H2D copy and decode of the previous.
 *   zgpu_encode_batch   <- CodecChain::encode (codec_chain.rs:528-555), fixed-size chains
 *   zgpu_encode_chunks  <- the same for variable-length chains: GzipCodec::encode (gzip_codec.rs:
 *                          96-107), ZstdCodec::encode (zstd_codec.rs:100-111), crc32c around them, and
 *                          ShardingCodecBound::encode_bounded (sharding_codec.rs:924-1085)
 *   status codes        <- CodecError variants (zarrs_codec/src/lib.rs:617-686), 1:1 (see below).
 *
 * Threading: every entry point is thread-safe. Calls on one context run concurrently: each takes one
 * of the context's lanes (stream + copy streams; ZGPU_CTX_LANES, default 8) for its duration and
 * waits when all are busy; the context's pooled memory is shared under an allocator lock. A plan
 * serialises its own executes.
 * Stream ordering: a call runs on the caller's hip_stream (device inputs/outputs must be ready in
 * that stream's order), or with hip_stream NULL on the context's own stream, which first waits for
 * all work queued so far on the legacy default stream.
 * Memory: the caller owns every encoded input and the output; the library owns its scratch.
 */
#ifndef ZGPU_H
#define ZGPU_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZGPU_MAX_DIMS 8

/* Status codes (per chunk and per call). Mapping onto zarrs_codec::CodecError:
 *  ZGPU_INVALID_CHECKSUM       -> CodecError::InvalidChecksum            (crc32c_codec.rs:130-133)
 *  ZGPU_DECODED_SIZE_MISMATCH  -> CodecError::UnexpectedChunkDecodedSize / InvalidBytesLength
 *                                 (ArrayBytes::validate, zarrs_codec/src/array_bytes.rs:376-386)
 *  ZGPU_SHARD_INDEX_OOB        -> CodecError::Other("The shard index references out-of-bounds
 *                                 bytes. The chunk may be corrupted.") (sharding_codec.rs:682-686)
 *  ZGPU_CORRUPT_STREAM         -> CodecError::IOError (gzip_codec.rs:116-118, zstd_codec.rs:119-128)
 *  ZGPU_INVALID_BYTE_RANGE     -> CodecError::InvalidByteRangeError
 *  ZGPU_UNSUPPORTED            -> CodecError::UnsupportedDataType / unsupported codec
 *  ZGPU_CRC_INPUT_TOO_SHORT    -> CodecError::Other("crc32c decoder expects a 32 bit input")
 *  ZGPU_SHARD_TOO_SMALL        -> CodecError::Other("The encoded shard is smaller than the
 *                                 expected size of its index.") (sharding_codec.rs:1277-1281)
 *  ZGPU_SHUFFLE_LENGTH         -> CodecError::Other("the shuffle codec expects the input byte
 *                                 length to be an integer multiple of the elementsize")
 *  ZGPU_INVALID_ARGUMENT       -> bad metadata / geometry (CodecCreateError, InvalidArraySubset)
 *  ZGPU_HIP_ERROR              -> device runtime failure (no zarrs equivalent)
 *  ZGPU_STORAGE_ERROR          -> StorageError::IOError from the filesystem store (open/read
 *                                 failures other than a missing key; zarrs_storage/src/lib.rs)
 */
enum {
  ZGPU_OK = 0,
  ZGPU_INVALID_CHECKSUM = 1,
  ZGPU_DECODED_SIZE_MISMATCH = 2,
  ZGPU_SHARD_INDEX_OOB = 3,
  ZGPU_CORRUPT_STREAM = 4,
  ZGPU_INVALID_BYTE_RANGE = 5,
  ZGPU_UNSUPPORTED = 6,
  ZGPU_CRC_INPUT_TOO_SHORT = 7,
  ZGPU_SHARD_TOO_SMALL = 8,
  ZGPU_SHUFFLE_LENGTH = 9,
  ZGPU_INVALID_ARGUMENT = 10,
  ZGPU_HIP_ERROR = 11,
  ZGPU_STORAGE_ERROR = 12,
};

/* decode flags */
#define ZGPU_ENC_DEVICE 0x1u  /* desc.enc / chunk_ptrs are device pointers (else host memory)  */
#define ZGPU_OUT_DEVICE 0x2u  /* out is a device pointer (else host memory)                    */
#define ZGPU_NO_VALIDATE 0x4u /* override: CodecOptions::validate_checksums = false for the call */
#define ZGPU_DIRECT_IO 0x8u   /* filesystem reads: FilesystemStoreOptions::direct_io (O_DIRECT)   */
#define ZGPU_ONE_STREAM 0x10u /* every kernel of the call on hip_stream (no internal side stream,
                                 e.g. zstd's sequence decoder beside its literal decoder): for callers
                                 that run independent plans concurrently on streams of their own   */
#define ZGPU_ZSTD_LITS_FIRST 0x40u /* zstd, with ZGPU_ONE_STREAM: the plan decodes its Huffman literals
                                 before its sequences. For callers overlapping plans on streams of
                                 their own: a plan whose executor ends the overlap gets its literals
                                 (throughput-bound) done while the other plans decode sequences
                                 (latency-bound). Output identical either way.                     */

typedef struct zgpu_ctx zgpu_ctx;
typedef struct zgpu_chain zgpu_chain;
typedef struct zgpu_plan zgpu_plan;

/* One context per GPU: owns a HIP stream, device scratch and pinned staging. zgpu_ctx_destroy drops
 * the caller's reference: chains, plans and caches created on the context hold references of their
 * own, so the context is freed when the last of them is destroyed (any destruction order is safe). */
int zgpu_ctx_create(int hip_device, zgpu_ctx **out);
void zgpu_ctx_destroy(zgpu_ctx *ctx);
/* Live references of a context (1 + its chains, plans and caches; diagnostics and tests). */
int64_t zgpu_ctx_refcount(const zgpu_ctx *ctx);
/* Return the context's cached free device and pinned buffers to HIP (buffers in use stay). The
 * device pool also trims itself past ZGPU_POOL_CAP_MB (default 16 GiB) of free blocks. */
int zgpu_ctx_release_cached(zgpu_ctx *ctx);
/* The context's pooled memory in bytes (diagnostics and tests; any pointer may be NULL): device
 * blocks in use and cached free, pinned host blocks in use and cached free. */
int zgpu_ctx_pool_stats(const zgpu_ctx *ctx, uint64_t *dev_live, uint64_t *dev_free, uint64_t *host_live,
                        uint64_t *host_free);
/* Last error message of the calling thread on this context ("" if none). */
const char *zgpu_last_error(const zgpu_ctx *ctx);
const char *zgpu_status_name(int status);
/* Library version string, and the device kernels' ISA ("gfx950"). */
const char *zgpu_version(void);

/*
 * Parse and bind a codec chain.
 *  codecs_json : the Zarr V3 "codecs" JSON array (nested sharding_indexed configs included).
 *                Supported: transpose, bytes, sharding_indexed (nested to any depth, with codecs
 *                around the inner shardings and bytes->bytes codecs after any of them),
 *                crc32c (+numcodecs.crc32c), gzip, zstd, numcodecs.shuffle, blosc (blosclz, lz4,
 *                lz4hc, zlib, snappy, zstd; shuffle / bitshuffle). Others -> ZGPU_UNSUPPORTED.
 *  data_type   : Zarr V3 data type name ("float32", "uint16", ...); fixed-size types only.
 *  fill        : native-endian fill value bytes (FillValue::as_ne_bytes), fill_len == dtype size.
 *  validate_checksums : CodecOptions::validate_checksums (zarrs default true, options.rs:24-33).
 */
int zgpu_chain_create(zgpu_ctx *ctx, const char *codecs_json, const char *data_type,
                      const void *fill, uint32_t fill_len, int validate_checksums,
                      zgpu_chain **out);
void zgpu_chain_destroy(zgpu_chain *chain);
/* Bytes per element of the bound data type. */
uint32_t zgpu_chain_element_size(const zgpu_chain *chain);

/* One chunk (or shard) to decode into the output array. */
typedef struct {
  const void *enc;                      /* encoded bytes; NULL = missing chunk -> fill value     */
  uint64_t enc_len;
  uint64_t chunk_shape[ZGPU_MAX_DIMS];  /* decoded chunk (shard) shape                          */
  uint64_t sel_start[ZGPU_MAX_DIMS];    /* wanted region of the chunk (chunk-relative)          */
  uint64_t sel_shape[ZGPU_MAX_DIMS];    /*   == chunk_shape & start 0 -> full decode path       */
  uint64_t out_start[ZGPU_MAX_DIMS];    /* where the region lands in the output array           */
} zgpu_chunk_desc;

/*
 * Decode n chunks into one C-order output array of shape out_shape[ndim].
 * A selection covering the whole chunk takes the full decode path (checksums verified);
 * a partial selection takes the partial-decoder path (crc32c stripped, not verified; for
 * sharding only the intersecting inner chunks are decoded), exactly as zarrs'
 * retrieve_chunk_subset_into does (array_read_ops_array.rs:346-375).
 * Output regions of different descriptors must be disjoint (ArrayBytesFixedDisjointView).
 * status[n] (optional) receives each chunk's status. Returns the first non-zero chunk status
 * (zarrs' try_for_each semantics) or a call-level error. hip_stream NULL = context stream.
 * A descriptor whose status is non-zero leaves its output region undefined (untouched, or partly
 * written: e.g. a blosc chunk decoded straight into the output, some of whose blocks failed), as
 * zarrs leaves a view whose decode_into failed; every other descriptor's region is complete.
 * The call is synchronous with respect to the host (statuses are final on return).
 * Any chain zgpu_chain_create accepts, and descriptors of different chunk shapes in one batch (e.g.
 * a rectilinear grid), decode here: one fused launch sequence per chunk shape when the chain is
 * "fused" (unsharded; or sharding_indexed, optionally behind transposes, with no bytes->bytes codec
 * after it and at most one plain nested sharding_indexed inside), else composed from fused ones:
 * whole-shard bytes->bytes codecs are decoded into device buffers first, and deeper or wrapped
 * nested shards are resolved through their outer index (read back) into descriptors of the inner
 * chain; transposes before a sharding_indexed of the second kind decode each selection in the
 * encoded (transposed) frame first, then transpose and scatter it.
 */
int zgpu_decode_batch(zgpu_chain *chain, uint32_t ndim, const zgpu_chunk_desc *descs,
                      uint64_t n, void *out, const uint64_t *out_shape, uint32_t flags,
                      int32_t *status, void *hip_stream);

/*
 * The output of a decode as a window of a larger C-order array: ArrayBytesDecodeIntoTarget /
 * ArrayBytesFixedDisjointView (zarrs_codec/src/array_bytes_fixed_disjoint_view.rs:12-207, the
 * target of CodecChainBound::decode_into, codec_chain.rs:592-646, and of
 * ShardingCodecBound::decode_into, sharding_codec.rs:617-707): base points at element [0,...,0] of
 * an array of array_shape; the view is the box [start, start + shape). Descriptors' out_start are
 * relative to the view (as with zgpu_decode_batch's out_shape = shape). Bytes of the array outside
 * the parts of the view the descriptors cover are never written.
 */
typedef struct {
  void *base;
  uint64_t array_shape[ZGPU_MAX_DIMS];
  uint64_t start[ZGPU_MAX_DIMS];
  uint64_t shape[ZGPU_MAX_DIMS];
} zgpu_out_view;

/* Concurrent-call coalescing (host inputs and host output only; ignored otherwise): calls carrying
 * this flag on the same chain, with the same flags and ndim, that arrive within the context's
 * collect window are decoded as ONE batch -- one packed H2D copy of their encoded bytes, one launch
 * sequence over all their chunks, one D2H copy -- and each caller gets its own statuses, its own
 * first-error return value and its own output window. This turns zarrs' per-shard decode_into calls
 * from rayon workers (array_read_ops_common.rs:173-176, sharding_codec.rs:617-707) into GPU-sized
 * batches without changing the read path. */
#define ZGPU_COALESCE 0x20u

/*
 * zgpu_decode_batch into a window of a larger array (host or device, ZGPU_OUT_DEVICE). A device
 * window is decoded in place (the scatter writes through the whole array's strides). A host window is
 * decoded into HBM and copied back box-wise (only the window's bytes cross PCIe; rows are placed by
 * host threads from pinned staging). Same statuses and return value as zgpu_decode_batch.
 */
int zgpu_decode_into(zgpu_chain *chain, uint32_t ndim, const zgpu_chunk_desc *descs, uint64_t n,
                     const zgpu_out_view *view, uint32_t flags, int32_t *status, void *hip_stream);

/*
 * zgpu_decode_batch with host inputs whose decoded output stays in library-owned pinned memory:
 * *data points at the C-order window of shape out_shape (prod(out_shape) * element size bytes),
 * valid until zgpu_result_release(*result). For callers that can only COPY into their target, as a
 * zarrs codec plugin must (ArrayBytesFixedDisjointView exposes copy_from_slice and no pointer,
 * zarrs_codec/src/array_bytes_fixed_disjoint_view.rs:177-206): decoding into a caller buffer and
 * then copying that into the view would cross host memory twice. ZGPU_COALESCE applies as for
 * zgpu_decode_batch (the pointer then lies inside the batch's pack, shared with its other callers).
 * On a failure *data is NULL and *result NULL. Host inputs only (ZGPU_ENC_DEVICE / ZGPU_OUT_DEVICE
 * -> ZGPU_INVALID_ARGUMENT).
 */
typedef struct zgpu_result zgpu_result;
int zgpu_decode_pinned(zgpu_chain *chain, uint32_t ndim, const zgpu_chunk_desc *descs, uint64_t n,
                       const uint64_t *out_shape, uint32_t flags, int32_t *status, const void **data,
                       zgpu_result **result);
void zgpu_result_release(zgpu_result *result);

/*
 * Coalescing policy of a context (ZGPU_COALESCE): a call waits at most window_us for other calls
 * to join its batch; a batch closes early at max_calls calls or max_bytes encoded bytes. Defaults:
 * 200 us, 8 calls, 1 GiB (env ZGPU_COALESCE_US / ZGPU_COALESCE_CALLS / ZGPU_COALESCE_BYTES).
 * Batches of one context run concurrently on its lanes.
 */
int zgpu_ctx_set_coalescing(zgpu_ctx *ctx, uint32_t window_us, uint32_t max_calls, uint64_t max_bytes);
/* Coalescing statistics of a context since its creation: batches executed and calls they carried. */
int zgpu_ctx_coalescing_stats(const zgpu_ctx *ctx, uint64_t *batches, uint64_t *calls);

/*
 * Prepared form of zgpu_decode_batch for device-resident inputs that are decoded repeatedly
 * (benchmarks, hipGraph capture): the descriptor table is planned and uploaded once. Plans take
 * fused chains and one chunk shape only (see zgpu_decode_batch); others -> ZGPU_UNSUPPORTED.
 * zgpu_plan_execute enqueues the decode on the stream and, if status != NULL, waits and returns
 * per-chunk statuses; with status == NULL it returns immediately after enqueue.
 * An asynchronous execute's output is valid only once zgpu_plan_status has returned for it: a blosc
 * input that outgrows the stream-table layout the plan recorded on its first execution is detected
 * on the device, nothing of it is decoded, and zgpu_plan_status re-runs the execution with a
 * read-back layout (ZGPU_CTR_BLOSC_RERUN) before it returns the statuses. Likewise a plan whose last
 * execution had no item for the serial zstd decoder skips that kernel; an input that needs it is
 * re-run by zgpu_plan_status with the kernel launched. A hipGraph capture of zgpu_plan_execute
 * therefore needs inputs whose blosc layout and zstd frame structure do not change between replays.
 */
int zgpu_plan_create(zgpu_chain *chain, uint32_t ndim, const zgpu_chunk_desc *descs, uint64_t n,
                     const uint64_t *out_shape, uint32_t flags, zgpu_plan **out);
int zgpu_plan_execute(zgpu_plan *plan, void *out, int32_t *status, void *hip_stream);
/* Wait for the plan's last execute on hip_stream and return its per-chunk statuses (first non-zero
 * status as the return value): lets independent plans (e.g. the levels of a multiscale pyramid)
 * run concurrently on separate streams. */
int zgpu_plan_status(zgpu_plan *plan, int32_t *status, void *hip_stream);
void zgpu_plan_destroy(zgpu_plan *plan);
/* Algorithmic HBM bytes of one execute (encoded bytes read + index bytes + decoded bytes
 * written), the figure bench.py prices the roofline with. */
uint64_t zgpu_plan_algorithmic_bytes(const zgpu_plan *plan);

/*
 * Plan group: one decode over the independent parts of a batch, each part one chunk shape and one
 * output (the levels of a multiscale pyramid; zarrs runs one rayon loop per array,
 * array_read_ops_common.rs:111-179). The group creates the parts' plans and places them on streams of
 * its own (at most ZGPU_GROUP_LANES, default 4 = HIP's default hardware queues): a part with at least
 * 1/(4 x lanes) of the group's encoded bytes gets a lane, the smaller parts share one lane (largest
 * first), the lanes left over go to the largest part, split into pieces of balanced encoded bytes; zstd
 * literals-first on the largest part's first piece and on the small-part lane (group.cpp). Part p has
 * n_descs[p] descriptors descs[p] decoded with chains[p] into an output of out_shapes[p] (ndim dims);
 * flags as zgpu_plan_create (ZGPU_ENC_DEVICE required). zgpu_group_execute enqueues every part behind
 * the work already on hip_stream (NULL: the legacy default stream) and makes hip_stream wait for all
 * of them; outs[p] is part p's output. status (NULL: asynchronous, read with zgpu_group_status)
 * receives the per-descriptor statuses, concatenated in part order; the return value is the first
 * non-zero one.
 */
typedef struct zgpu_group zgpu_group;
int zgpu_group_create(zgpu_chain *const *chains, uint32_t ndim, uint32_t n_parts, const zgpu_chunk_desc *const *descs,
                      const uint64_t *n_descs, const uint64_t *const *out_shapes, uint32_t flags, zgpu_group **out);
int zgpu_group_execute(zgpu_group *group, void *const *outs, int32_t *status, void *hip_stream);
int zgpu_group_status(zgpu_group *group, int32_t *status, void *hip_stream);
/* The group's plans: returns how many; for the first n, their lane, part and literals-first flag. */
uint32_t zgpu_group_layout(const zgpu_group *group, uint32_t *lane_of, uint32_t *part_of, uint32_t *lits_first,
                           uint32_t n);
uint64_t zgpu_group_algorithmic_bytes(const zgpu_group *group);
/* zgpu_plan_counters summed over the group's plans (after zgpu_group_status). */
uint32_t zgpu_group_counters(const zgpu_group *group, uint64_t *out, uint32_t n);
void zgpu_group_destroy(zgpu_group *group);

/* Device counters of a plan's last execute (after its statuses were read) or of the calling
 * thread's last decode call (zgpu_decode_batch / zgpu_decode_files / zgpu_retrieve_*), summed over
 * its sub-batches. Writes min(n, ZGPU_N_COUNTERS) values, returns how many were written. */
#define ZGPU_CTR_ENC_BYTES 0     /* encoded bytes read (resolved inner-chunk ranges of sharded items) */
#define ZGPU_CTR_ZSTD_SERIAL 1   /* zstd items decoded by the serial one-wave fallback decoder     */
#define ZGPU_CTR_ZSTD_PARALLEL 2 /* zstd items decoded by the block-parallel pipeline              */
#define ZGPU_CTR_BLOSC_RERUN 3   /* 1 when a blosc input outgrew the stream-table layout recorded by
                                    the plan's first execution and the execution was re-run with a
                                    read-back layout (later executions are asynchronous otherwise) */
#define ZGPU_CTR_BLOSC_BLOCKS 4  /* blosc blocks decoded: a partial selection decodes only the blocks
                                    covering the bytes it reads (blosc_partial_decoder.rs:33-60)     */
#define ZGPU_CTR_ITEMS 5         /* leaf items the call planned: chunks, or inner chunks of shards that meet
                                    the selection (each decoded, or filled when empty)                 */
#define ZGPU_N_COUNTERS 6
uint32_t zgpu_plan_counters(const zgpu_plan *plan, uint64_t *out, uint32_t n);
uint32_t zgpu_last_counters(uint64_t *out, uint32_t n);

/* Detail of the calling thread's last call that returned ZGPU_DECODED_SIZE_MISMATCH, for
 * CodecError::UnexpectedChunkDecodedSize(InvalidBytesLengthError::new(len, expected_len))
 * (zarrs_codec/src/lib.rs:491-501,632): the failing descriptor, the decoded length the final stage
 * saw and the expected length of the (inner) chunk. len == UINT64_MAX: a decompressor produced more
 * than expected_len bytes and stopped (its total is not known). Returns 1 if a detail is available. */
int zgpu_last_size_mismatch(uint64_t *desc, uint64_t *len, uint64_t *expected_len);

/*
 * Array::retrieve_array_subset_into over a regular chunk grid. chunk_ptrs/chunk_lens are
 * indexed by the C-order linear chunk-grid index (grid = ceil(array_shape/chunk_shape));
 * chunk_ptrs[i] == NULL means the key is missing (fill value). out holds prod(sel_shape)
 * elements in C order. Returns the first failing chunk's status.
 */
int zgpu_retrieve_array_subset(zgpu_chain *chain, uint32_t ndim, const uint64_t *array_shape,
                               const uint64_t *chunk_shape, const void *const *chunk_ptrs,
                               const uint64_t *chunk_lens, const uint64_t *sel_start,
                               const uint64_t *sel_shape, void *out, uint32_t flags,
                               void *hip_stream);

/*
 * zgpu_retrieve_array_subset over several GPUs of one node from one process (one chain per device,
 * each created on that device's context; same codecs and data type). The subset's chunk rows along
 * axis 0 are cut into n_dev contiguous groups and decoded concurrently, device d taking group d
 * (array_read_ops_common.rs:173-176: chunks are independent). Encoded chunks are host-resident
 * (ZGPU_ENC_DEVICE is rejected): each device uploads its own over its own link. Host `out`: every
 * device writes its rows straight into place. ZGPU_OUT_DEVICE: `out` is on chains[0]'s device; the
 * other devices decode into their own HBM and copy their rows into `out` peer-to-peer (xGMI).
 * Synchronous. Returns the first failing status in chunk (= device) order.
 */
int zgpu_retrieve_array_subset_multi(zgpu_chain *const *chains, uint32_t n_dev, uint32_t ndim,
                                     const uint64_t *array_shape, const uint64_t *chunk_shape,
                                     const void *const *chunk_ptrs, const uint64_t *chunk_lens,
                                     const uint64_t *sel_start, const uint64_t *sel_shape, void *out,
                                     uint32_t flags);

/*
 * Encoded chunks in a filesystem store. One byte range of one file per descriptor:
 * path = FilesystemStore::key_to_fspath(key) (zarrs_filesystem/src/lib.rs:173-179); path NULL or a
 * file that does not exist = missing key -> fill value (lib.rs:339-343,428-430); len == UINT64_MAX
 * reads from offset to the end of the file (ByteRange::FromStart(offset, None)); a range past the
 * end of the file gives that descriptor ZGPU_INVALID_BYTE_RANGE (lib.rs:437-447).
 */
typedef struct {
  const char *path;
  uint64_t offset;
  uint64_t len;
} zgpu_file_range;

/*
 * zgpu_decode_batch with descs[i].enc/enc_len taken from files[i] (the caller's enc fields are
 * ignored). The batch is cut into sub-batches (in descriptor order); a pool of host threads reads
 * sub-batch k+1 with positional reads (O_DIRECT page reads with ZGPU_DIRECT_IO, falling back to
 * buffered reads where the filesystem has no O_DIRECT) into pinned staging while sub-batch k is
 * copied to HBM and decoded. out is device memory (ZGPU_OUT_DEVICE) or host memory.
 * Hard I/O errors (not ENOENT) fail the call with ZGPU_STORAGE_ERROR.
 */
int zgpu_decode_files(zgpu_chain *chain, uint32_t ndim, const zgpu_chunk_desc *descs,
                      const zgpu_file_range *files, uint64_t n, void *out, const uint64_t *out_shape,
                      uint32_t flags, int32_t *status, void *hip_stream);

/*
 * zgpu_retrieve_array_subset over a filesystem store: chunk_paths[i] is the path of the chunk with
 * C-order linear grid index i (NULL or nonexistent = missing key); each chunk file is read whole.
 */
int zgpu_retrieve_array_subset_files(zgpu_chain *chain, uint32_t ndim, const uint64_t *array_shape,
                                     const uint64_t *chunk_shape, const char *const *chunk_paths,
                                     const uint64_t *sel_start, const uint64_t *sel_shape, void *out,
                                     uint32_t flags, void *hip_stream);

/*
 * Write path: CodecChain::encode (zarrs/src/array/codec/array_to_bytes/
 * codec_chain.rs:528-555) for fixed-size chains -- transpose, bytes (endianness), numcodecs.shuffle
 * (innermost, elementsize = data type size), crc32c (end or start, any number). Compressing codecs
 * and sharding_indexed return ZGPU_UNSUPPORTED here: they go through zgpu_encode_chunks.
 * zgpu_chain_encoded_size: encoded bytes of one chunk of chunk_shape (BytesRepresentation::FixedSize),
 * -1 if the chain's encoded size is not fixed.
 * zgpu_encode_batch: encode the chunks whose origins are descs[i].chunk_start (in elements) of the
 * device-resident C-order array (array_shape) into descs[i].dst (device memory, >= encoded size).
 * Chunk regions past the array edge encode the fill value. flags must be
 * ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE.
 */
typedef struct {
  void *dst;
  uint64_t dst_cap;
  uint64_t chunk_start[ZGPU_MAX_DIMS];
} zgpu_encode_desc;
int64_t zgpu_chain_encoded_size(const zgpu_chain *chain, uint32_t ndim, const uint64_t *chunk_shape);
int zgpu_encode_batch(zgpu_chain *chain, uint32_t ndim, const uint64_t *chunk_shape, const void *array,
                      const uint64_t *array_shape, const zgpu_encode_desc *descs, uint64_t n, uint32_t flags,
                      void *hip_stream);
/*
 * zgpu_encode_batch plus the variable-length chains: gzip (one DEFLATE stream of dynamic-Huffman or
 * stored blocks in a gzip member, k_gzip_encode), zstd (one single-segment frame of 64 KiB blocks:
 * Huffman / RLE / raw literals, predefined-FSE sequences, optional XXH64 content checksum; encoded in
 * 1 MiB segments, one wave each, k_zstd_encode_seg + k_zstd_frame), crc32c around them,
 * the fixed-size stages in front, and sharding_indexed over a fixed-size or compressing inner chain
 * (ShardingCodecBound::encode_bounded, sharding_codec.rs:924-1085, with SubchunkWriteOrder::C: inner
 * chunks in C order of the inner grid, an inner chunk equal to the fill value everywhere omitted,
 * index bytes{endian} + crc32c at the start or end). The compressed bytes are valid streams that
 * every gzip / zstd decoder reads back to the input; they are not byte-identical to zlib's or
 * libzstd's output (the Zarr specification fixes the decoded bytes, not the encoder). blosc
 * (BloscCodec::encode, blosc_codec_via_blosc_src.rs:113-128) writes c-blosc 1.x frames with
 * blosclz, lz4 / lz4hc, snappy, zlib or zstd streams after a byte shuffle / bitshuffle (frames any
 * c-blosc 1.x decoder reads, not byte-identical to c-blosc's).
 * enc_lens[n] receives each chunk's encoded length; descs[i].dst_cap must be >=
 * zgpu_chain_encoded_bound. zgpu_chain_encoded_bound: the fixed size, or the worst case
 * (gzip_codec.rs:122-136, zstd_codec.rs:132-147; a shard: every inner chunk at its bound + index),
 * -1 if unbounded.
 */
int64_t zgpu_chain_encoded_bound(const zgpu_chain *chain, uint32_t ndim, const uint64_t *chunk_shape);
/* One chunk (or shard) of chunk_shape from host bytes (C order), encoded on the GPU as
 * zgpu_encode_chunks does; *enc / *enc_len: the encoded bytes in library-owned pinned memory, valid
 * until zgpu_result_release(*result) -- the codec plugin's CodecChain::encode /
 * ShardingCodecBound::encode (sharding_codec.rs:351-376), which must return owned host bytes. */
int zgpu_encode_pinned(zgpu_chain *chain, uint32_t ndim, const uint64_t *chunk_shape, const void *decoded,
                       const void **enc, uint64_t *enc_len, zgpu_result **result);
int zgpu_encode_chunks(zgpu_chain *chain, uint32_t ndim, const uint64_t *chunk_shape, const void *array,
                       const uint64_t *array_shape, const zgpu_encode_desc *descs, uint64_t n, uint32_t flags,
                       uint64_t *enc_lens, void *hip_stream);

/*
 * HBM-resident decoded-chunk cache: ChunkCacheDecodedLruSizeLimit (zarrs/src/array/chunk_cache/
 * chunk_cache_lru.rs:270) used through ArrayCached::retrieve_array_subset (zarrs/src/array/array_ops/
 * array_read_ops_array_cached.rs:315-412). One cache per array (as an ArrayCached owns its cache):
 * whole decoded chunks (full decode path, checksums verified) in a pool of floor(capacity / chunk
 * bytes) HBM slots, keyed by the C-order chunk-grid index; a missing key is cached as "no chunk" (fill
 * value); least recently used chunks are evicted. A read decodes all of its misses into their slots in
 * one batch, then gathers the subset from HBM. A read touching more chunks than the cache holds is
 * decoded directly (nothing new cached). Arguments as zgpu_retrieve_array_subset.
 */
typedef struct zgpu_cache zgpu_cache;
int zgpu_cache_create(zgpu_ctx *ctx, uint64_t capacity_bytes, zgpu_cache **out);
void zgpu_cache_destroy(zgpu_cache *cache);
int zgpu_cache_clear(zgpu_cache *cache);
int zgpu_cache_stats(zgpu_cache *cache, uint64_t *hits, uint64_t *misses, uint64_t *entries, uint64_t *bytes_used);
int zgpu_cache_retrieve_array_subset(zgpu_cache *cache, zgpu_chain *chain, uint32_t ndim, const uint64_t *array_shape,
                                     const uint64_t *chunk_shape, const void *const *chunk_ptrs,
                                     const uint64_t *chunk_lens, const uint64_t *sel_start, const uint64_t *sel_shape,
                                     void *out, uint32_t flags, void *hip_stream);

/*
 * DLPack export of a decoded subset left in HBM (the reference exports CPU tensors only:
 * zarrs/src/array/array_dlpack_ext.rs:44-70, Device::CPU). The zgpu_dl_* types are layout-identical to
 * DLPack's DLDevice / DLDataType / DLTensor / DLManagedTensor (dlpack.h, unversioned ABI, consumed
 * through a PyCapsule named "dltensor"); device_type is kDLROCM (10). The library allocates the buffer
 * on the chain's device; the consumer calls deleter(tensor) when done. cache may be NULL.
 */
#define ZGPU_DL_ROCM 10
typedef struct { int32_t device_type; int32_t device_id; } zgpu_dl_device;
typedef struct { uint8_t code; uint8_t bits; uint16_t lanes; } zgpu_dl_data_type;
typedef struct {
  void *data;
  zgpu_dl_device device;
  int32_t ndim;
  zgpu_dl_data_type dtype;
  int64_t *shape;
  int64_t *strides; /* NULL: compact row-major */
  uint64_t byte_offset;
} zgpu_dl_tensor;
typedef struct zgpu_dl_managed_tensor {
  zgpu_dl_tensor dl_tensor;
  void *manager_ctx;
  void (*deleter)(struct zgpu_dl_managed_tensor *self);
} zgpu_dl_managed_tensor;
int zgpu_retrieve_array_subset_dlpack(zgpu_cache *cache, zgpu_chain *chain, uint32_t ndim, const uint64_t *array_shape,
                                      const uint64_t *chunk_shape, const void *const *chunk_ptrs,
                                      const uint64_t *chunk_lens, const uint64_t *sel_start, const uint64_t *sel_shape,
                                      uint32_t flags, void *hip_stream, zgpu_dl_managed_tensor **out);

#ifdef __cplusplus
}
#endif
#endif /* ZGPU_H */
