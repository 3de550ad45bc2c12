// Codec chain model: parse + bind of the Zarr V3 "codecs" metadata list.
// Mirrors CodecChain::from_metadata / with_context
// (zarrs/src/array/codec/array_to_bytes/codec_chain.rs:105-169,192-229): array->array codecs,
// exactly one array->bytes codec, then bytes->bytes codecs; decode runs them in reverse.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

#include "json.hpp"

namespace zgpu {

enum class CodecKind { Transpose, Bytes, Sharding, Crc32c, Gzip, Zstd, Shuffle, Blosc };

struct Chain;

struct Codec {
  CodecKind kind;
  std::string name;
  std::vector<uint32_t> order;        // transpose
  bool big_endian = false;            // bytes
  bool at_start = false;              // crc32c location / sharding index_location
  int level = 0;                      // gzip / zstd
  bool checksum = false;              // zstd
  uint32_t elementsize = 4;           // shuffle; blosc typesize
  std::string cname;                  // blosc compressor (decode reads the compressor from the header)
  int shuffle = -1;                   // blosc: 0 noshuffle, 1 byte shuffle, 2 bitshuffle, -1 absent
  uint64_t blocksize = 0;             // blosc: 0 = automatic
  std::vector<uint64_t> inner_shape;  // sharding
  std::shared_ptr<Chain> inner, index;
};

struct Chain {
  std::vector<Codec> a2a;
  Codec a2b;
  std::vector<Codec> b2b;
  uint32_t es = 0, comp = 0;
  uint8_t fill[16] = {0};
  std::string data_type;
};

struct ChainError {
  int status;
  std::string msg;
};

// Data type name -> (element size, endianness component size); false if unsupported.
bool data_type_info(const std::string &name, uint32_t &es, uint32_t &comp);

// Throws ChainError.
std::shared_ptr<Chain> parse_chain(const Json &codecs, const std::string &data_type, const uint8_t *fill);

// Encoded byte size of a chain for a fixed decoded element count, or -1 if not fixed-size
// (BytesRepresentation::FixedSize, sharding.rs:163-176).
int64_t chain_fixed_encoded_size(const Chain &c, uint64_t nelem);

// Upper bound of one chunk's encoded size for an array->bytes `bytes` chain (BytesRepresentation::
// BoundedSize): crc32c +4, gzip as GzipCodec::encoded_representation (gzip_codec.rs:122-136, zlib's
// deflateBound), zstd as ZstdCodec's (zstd_codec.rs:132-147); -1 if unbounded (e.g. blosc here).
int64_t chain_encoded_bound(const Chain &c, uint64_t nelem);
uint64_t gzip_bound(uint64_t n);
uint64_t zstd_bound(uint64_t n);

}  // namespace zgpu
