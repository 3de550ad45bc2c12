/*
 * zarrs_oracle.h — CPU restatement of the zarrs chunk-decode codec pipeline.
 *
 * TEST INFRASTRUCTURE ONLY. This is the parity oracle and the timed CPU baseline
 * ("cpu_baseline.kind = port"). Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load it. The product (zarrs_amd/, libzgpu.so) never links it.
 *
 * Every function cites the zarrs file:line it restates (paths relative to the zarrs
 * workspace root). Third-party arithmetic the reference pulls from crates that are not
 * vendored is restated on the host libraries that implement the same published algorithm:
 *   - crc32c 0.6.5 (zarrs/Cargo.toml:56): table-driven reflected Castagnoli, poly 0x82F63B78
 *   - flate2 1.1 / miniz_oxide (Cargo.toml:58): RFC 1951/1952 inflate via system zlib 1.2.11
 *   - zstd 0.13 / zstd-sys (Cargo.toml:102): RFC 8878 via system libzstd.so.1 (1.4.8)
 *   - ndarray 0.17 permuted_axes (Cargo.toml:67): restated as explicit index arithmetic
 * Parity pinning: tests/test_oracle_golden.py checks this oracle against the reference's
 * own fixtures (zarrs/tests/data/...) and known-answer tests, committed under tests/golden/.
 */
#ifndef ZARRS_ORACLE_H
#define ZARRS_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* status codes: identical numbering to include/zgpu.h */
enum {
  ORC_OK = 0,
  ORC_INVALID_CHECKSUM = 1,
  ORC_DECODED_SIZE_MISMATCH = 2,
  ORC_SHARD_INDEX_OOB = 3,
  ORC_CORRUPT_STREAM = 4,
  ORC_INVALID_BYTE_RANGE = 5,
  ORC_UNSUPPORTED = 6,
  ORC_CRC_INPUT_TOO_SHORT = 7,
  ORC_SHARD_TOO_SMALL = 8,
  ORC_SHUFFLE_LENGTH = 9,
  ORC_INVALID_ARGUMENT = 10,
};

typedef struct orc_chain orc_chain;

/* Chain construction (mirror of CodecChain::from_metadata + with_context,
 * zarrs/src/array/codec/array_to_bytes/codec_chain.rs:105-229). Codecs are appended in
 * metadata order: array->array first, then exactly one array->bytes, then bytes->bytes. */
orc_chain *orc_chain_new(uint32_t elem_size, uint32_t component_size, const void *fill);
void orc_chain_free(orc_chain *c);
int orc_chain_add_transpose(orc_chain *c, uint32_t ndim, const uint32_t *order);
int orc_chain_add_bytes(orc_chain *c, int big_endian);
/* takes ownership of inner and index chains */
int orc_chain_add_sharding(orc_chain *c, uint32_t ndim, const uint64_t *inner_shape,
                           orc_chain *inner, orc_chain *index, int index_at_start);
int orc_chain_add_crc32c(orc_chain *c, int at_start);
int orc_chain_add_gzip(orc_chain *c, int level);
int orc_chain_add_zstd(orc_chain *c, int level, int checksum);
int orc_chain_add_blosc(orc_chain *c, const char *cname, int clevel, int shuffle, uint32_t typesize,
                        uint64_t blocksize);
int orc_chain_add_shuffle(orc_chain *c, uint32_t elementsize);

/* Full chunk decode (CodecChainBound::decode, codec_chain.rs:557-590). out must hold
 * prod(shape)*elem_size bytes. validate = CodecOptions::validate_checksums. */
int orc_decode_chunk(const orc_chain *c, const uint8_t *enc, uint64_t enc_len, uint32_t ndim,
                     const uint64_t *shape, int validate, uint8_t *out);

/* Chunk encode (CodecChainBound::encode, codec_chain.rs:528-555). *enc is malloc'd. */
int orc_encode_chunk(const orc_chain *c, const uint8_t *dec, uint32_t ndim, const uint64_t *shape,
                     uint8_t **enc, uint64_t *enc_len);
void orc_free(void *p);

/* Array read op (Array::retrieve_array_subset_into, array_read_ops_common.rs:20-179):
 * chunks indexed by C-order chunk-grid linear index; chunk_ptrs[i]==NULL => missing (fill).
 * Full-coverage chunks take decode_into (checksums verified); partially covered chunks take
 * the partial decoder (array_read_ops_array.rs:346-375), whose crc32c stage only strips. */
int orc_retrieve_array_subset(const orc_chain *c, uint32_t ndim, const uint64_t *array_shape,
                              const uint64_t *chunk_shape, const uint8_t *const *chunk_ptrs,
                              const uint64_t *chunk_lens, const uint64_t *sel_start,
                              const uint64_t *sel_shape, uint8_t *out, int nthreads, int validate);

/* primitives */
uint32_t orc_crc32c(uint32_t crc, const uint8_t *p, uint64_t n); /* standard (init/xorout ~0) */
uint32_t orc_crc32_ieee(const uint8_t *p, uint64_t n);
const char *orc_status_name(int s);

#ifdef __cplusplus
}
#endif
#endif
