// Codec chain parsing (see chain.hpp). Reference: codec_chain.rs:192-229 (from_metadata: exactly one
// array->bytes codec, error otherwise), zarrs_codec/src/lib.rs:372-449 (name -> codec lookup), and the
// per-codec configurations in zarrs_metadata_ext/src/codec/registered/{transpose,bytes,sharding,
// crc32c,gzip,zstd,shuffle}.rs.
#include "chain.hpp"

#include <cstring>

#include "../../include/zgpu.h"

namespace zgpu {

bool data_type_info(const std::string &n, uint32_t &es, uint32_t &comp) {
  struct E { const char *name; uint32_t es, comp; };
  static const E tab[] = {
      {"bool", 1, 1},    {"int8", 1, 1},    {"uint8", 1, 1},    {"int16", 2, 2},     {"uint16", 2, 2},
      {"float16", 2, 2}, {"bfloat16", 2, 2}, {"int32", 4, 4},   {"uint32", 4, 4},    {"float32", 4, 4},
      {"int64", 8, 8},   {"uint64", 8, 8},  {"float64", 8, 8},  {"complex64", 8, 4}, {"complex128", 16, 8},
  };
  for (const E &e : tab)
    if (n == e.name) {
      es = e.es;
      comp = e.comp;
      return true;
    }
  return false;
}

static std::shared_ptr<Chain> parse(const Json &codecs, const std::string &dt, uint32_t es, uint32_t comp,
                                    const uint8_t *fill);

enum class Role { A2A, A2B, B2B };

// Codec names zarrs itself creates (zarrs/src/array/codec/**: impl_extension_aliases! v3 names and
// aliases) that this pipeline does not implement. zarrs would create and use such a codec even with
// "must_understand": false, so it is an error here rather than a skip (skipping would decode wrongly).
static bool zarrs_knows(const std::string &n) {
  static const char *names[] = {
      "bitround", "numcodecs.bitround", "cast_value", "numcodecs.fixedscaleoffset", "reshape", "zarrs.squeeze",
      "packbits", "numcodecs.pcodec", "zfp", "zarrs.zfp", "numcodecs.zfpy", "zarrs.vlen", "zarrs.vlen_v2",
      "vlen-bytes", "vlen-utf8", "vlen-array", "zarrs.optional", "numcodecs.adler32", "numcodecs.bz2",
      "numcodecs.fletcher32", "zarrs.gdeflate", "numcodecs.zlib"};
  for (const char *k : names)
    if (n == k) return true;
  return n.rfind("https://codec.zarrs.dev/", 0) == 0;
}

// Codec::from_metadata for one entry (zarrs_codec/src/lib.rs:372-449 with the per-codec
// configurations of zarrs_metadata_ext/src/codec/registered/*.rs). Throws ChainError when the codec
// cannot be created (unknown name or invalid configuration).
static Role create_codec(Codec &k, const Json *cfg, const std::string &dt, uint32_t es, uint32_t comp,
                         const uint8_t *fill) {
  auto cfg_get = [&](const char *key) -> const Json * { return cfg ? cfg->get(key) : nullptr; };
  if (k.name == "transpose") {
    k.kind = CodecKind::Transpose;
    const Json *o = cfg_get("order");
    if (!o || o->kind != Json::Arr) throw ChainError{ZGPU_INVALID_ARGUMENT, "transpose: missing order"};
    uint32_t seen = 0;
    for (const Json &v : o->arr) {
      int64_t a = v.as_int();
      if (a < 0 || a >= (int64_t)o->arr.size() || a >= ZGPU_MAX_DIMS || ((seen >> a) & 1))
        throw ChainError{ZGPU_INVALID_ARGUMENT, "transpose: order is not a permutation"};
      seen |= 1u << a;
      k.order.push_back((uint32_t)a);
    }
    return Role::A2A;
  }
  if (k.name == "bytes" || k.name == "endian") {  // "endian": legacy alias (array_to_bytes/bytes.rs:53-55)
    k.kind = CodecKind::Bytes;
    const Json *e = cfg_get("endian");
    if (e && e->kind == Json::Str) {
      if (e->s == "big") k.big_endian = true;
      else if (e->s != "little") throw ChainError{ZGPU_INVALID_ARGUMENT, "bytes: bad endian"};
    } else if (comp > 1) {
      // BytesCodecEndiannessMissingError (zarrs_data_type/src/codec_traits/bytes.rs:109-110)
      throw ChainError{ZGPU_INVALID_ARGUMENT, "bytes: endian required for multi-byte data types"};
    }
    return Role::A2B;
  }
  if (k.name == "sharding_indexed") {
    k.kind = CodecKind::Sharding;
    const Json *cs = cfg_get("chunk_shape");
    if (!cs || cs->kind != Json::Arr) throw ChainError{ZGPU_INVALID_ARGUMENT, "sharding: missing chunk_shape"};
    for (const Json &v : cs->arr) {
      int64_t s = v.as_int();
      if (s <= 0) throw ChainError{ZGPU_INVALID_ARGUMENT, "sharding: chunk_shape must be positive"};
      k.inner_shape.push_back((uint64_t)s);
    }
    const Json *ic = cfg_get("codecs");
    if (!ic) throw ChainError{ZGPU_INVALID_ARGUMENT, "sharding: missing codecs"};
    k.inner = parse(*ic, dt, es, comp, fill);
    Json defidx = Json::parse(R"([{"name":"bytes","configuration":{"endian":"little"}},{"name":"crc32c"}])");
    const Json *xc = cfg_get("index_codecs");
    const uint8_t ffill[8] = {0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff, 0xff};
    k.index = parse(xc ? *xc : defidx, "uint64", 8, 8, ffill);
    const Json *loc = cfg_get("index_location");
    if (loc && loc->kind == Json::Str) {
      if (loc->s == "start") k.at_start = true;
      else if (loc->s != "end") throw ChainError{ZGPU_INVALID_ARGUMENT, "sharding: bad index_location"};
    }
    return Role::A2B;
  }
  if (k.name == "crc32c" || k.name == "numcodecs.crc32c") {
    k.kind = CodecKind::Crc32c;
    const Json *loc = cfg_get("location");
    if (loc && loc->kind == Json::Str && loc->s == "start") k.at_start = true;
  } else if (k.name == "gzip") {
    k.kind = CodecKind::Gzip;
    const Json *l = cfg_get("level");
    k.level = l ? (int)l->as_int() : 5;
  } else if (k.name == "zstd" || k.name == "numcodecs.zstd") {
    k.kind = CodecKind::Zstd;
    const Json *l = cfg_get("level");
    k.level = l ? (int)l->as_int() : 0;
    const Json *cs = cfg_get("checksum");
    k.checksum = cs && cs->kind == Json::Bool && cs->b;
  } else if (k.name == "blosc" || k.name == "numcodecs.blosc") {
    // blosc_codec_via_blosc_src.rs: cname / clevel / shuffle / typesize / blocksize; the decoder
    // reads everything it needs (compressor, shuffle, typesize, block size) from the frame header
    k.kind = CodecKind::Blosc;
    const Json *cn = cfg_get("cname");
    k.cname = cn && cn->kind == Json::Str ? cn->s : "lz4";
    static const char *known[] = {"blosclz", "lz4", "lz4hc", "snappy", "zlib", "zstd"};
    bool ok = false;
    for (const char *n : known) ok = ok || k.cname == n;
    if (!ok) throw ChainError{ZGPU_INVALID_ARGUMENT, "blosc: unknown cname '" + k.cname + "'"};
    const Json *l = cfg_get("clevel");
    k.level = l ? (int)l->as_int() : 5;
    const Json *t = cfg_get("typesize");
    k.elementsize = t && t->kind != Json::Null ? (uint32_t)t->as_int() : 0;
    // shuffle: "noshuffle" / "shuffle" / "bitshuffle" (V3), 0 / 1 / 2 / -1 = auto (numcodecs: bit
    // shuffle for 1-byte items, else byte shuffle)
    if (const Json *sh = cfg_get("shuffle")) {
      if (sh->kind == Json::Str) {
        k.shuffle = sh->s == "noshuffle" ? 0 : sh->s == "shuffle" ? 1 : sh->s == "bitshuffle" ? 2 : -2;
        if (k.shuffle == -2) throw ChainError{ZGPU_INVALID_ARGUMENT, "blosc: unknown shuffle '" + sh->s + "'"};
      } else if (sh->kind != Json::Null) {
        const int v = (int)sh->as_int();
        k.shuffle = v == -1 ? (k.elementsize == 1 ? 2 : 1) : v;
        if (k.shuffle < 0 || k.shuffle > 2) throw ChainError{ZGPU_INVALID_ARGUMENT, "blosc: shuffle out of range"};
      }
    }
    const Json *bsz = cfg_get("blocksize");
    k.blocksize = bsz && bsz->kind != Json::Null ? (uint64_t)bsz->as_int() : 0;
  } else if (k.name == "numcodecs.shuffle" || k.name == "shuffle") {
    k.kind = CodecKind::Shuffle;
    const Json *e = cfg_get("elementsize");
    k.elementsize = e ? (uint32_t)e->as_int() : 4;
    if (k.elementsize == 0) throw ChainError{ZGPU_INVALID_ARGUMENT, "shuffle: elementsize must be > 0"};
  } else {
    throw ChainError{ZGPU_UNSUPPORTED, "codec '" + k.name + "' is not supported by the GPU pipeline"};
  }
  return Role::B2B;
}

// CodecChain::from_metadata (codec_chain.rs:192-229): every entry is created and sorted by its kind
// (array->array, array->bytes, bytes->bytes; metadata order kept within each kind); an entry that
// cannot be created is skipped when it says "must_understand": false (:197-206); exactly one
// array->bytes codec. MetadataV3 accepts "name" or {name, configuration?, must_understand?} and
// nothing else (zarrs_metadata/src/v3/metadata.rs:114-149).
static std::shared_ptr<Chain> parse(const Json &codecs, const std::string &dt, uint32_t es, uint32_t comp,
                                    const uint8_t *fill) {
  if (codecs.kind != Json::Arr) throw ChainError{ZGPU_INVALID_ARGUMENT, "codecs must be a JSON array"};
  auto c = std::make_shared<Chain>();
  c->es = es;
  c->comp = comp;
  c->data_type = dt;
  if (fill) std::memcpy(c->fill, fill, es);
  bool have_a2b = false;
  for (const Json &m : codecs.arr) {
    Codec k;
    const Json *cfg = nullptr;
    bool must_understand = true;
    if (m.kind == Json::Str) {
      k.name = m.s;
    } else if (m.kind == Json::Obj && m.get("name") && m.get("name")->kind == Json::Str) {
      for (const auto &kv : m.obj)
        if (kv.first != "name" && kv.first != "configuration" && kv.first != "must_understand")
          throw ChainError{ZGPU_INVALID_ARGUMENT, "codec metadata: unknown field '" + kv.first + "'"};
      k.name = m.get("name")->as_str();
      cfg = m.get("configuration");
      if (const Json *mu = m.get("must_understand")) {
        if (mu->kind != Json::Bool) throw ChainError{ZGPU_INVALID_ARGUMENT, "must_understand must be a bool"};
        must_understand = mu->b;
      }
    } else {
      throw ChainError{ZGPU_INVALID_ARGUMENT, "codec metadata must be \"name\" or {name, configuration}"};
    }
    Role role;
    try {
      role = create_codec(k, cfg, dt, es, comp, c->fill);
    } catch (const ChainError &e) {
      // zarrs skips an optional codec it cannot create (unknown name or invalid configuration); a
      // codec zarrs would create but the GPU pipeline lacks stays an error
      if (must_understand || (e.status == ZGPU_UNSUPPORTED && zarrs_knows(k.name))) throw;
      continue;
    }
    if (role == Role::A2A) {
      c->a2a.push_back(k);
    } else if (role == Role::A2B) {
      if (have_a2b) throw ChainError{ZGPU_INVALID_ARGUMENT, "multiple array to bytes codecs"};
      c->a2b = k;
      have_a2b = true;
    } else {
      c->b2b.push_back(k);
    }
  }
  if (!have_a2b) throw ChainError{ZGPU_INVALID_ARGUMENT, "missing array to bytes codec"};
  return c;
}

std::shared_ptr<Chain> parse_chain(const Json &codecs, const std::string &dt, const uint8_t *fill) {
  uint32_t es, comp;
  if (!data_type_info(dt, es, comp)) throw ChainError{ZGPU_UNSUPPORTED, "data type '" + dt + "'"};
  return parse(codecs, dt, es, comp, fill);
}

int64_t chain_fixed_encoded_size(const Chain &c, uint64_t nelem) {
  if (c.a2b.kind != CodecKind::Bytes) return -1;
  int64_t n = (int64_t)(nelem * c.es);
  for (const Codec &k : c.b2b) {
    if (k.kind == CodecKind::Crc32c) n += 4;
    else if (k.kind != CodecKind::Shuffle) return -1;
  }
  return n;
}

uint64_t gzip_bound(uint64_t n) { return n + 10 + 8 + (n + 7) / 8 + (n + 63) / 64 + 5; }

// ZstdCodec::encoded_representation (zstd_codec.rs:132-147): header/trailer 4 + 14 + 4 bytes and a
// 3-byte block header per 1000 bytes
uint64_t zstd_bound(uint64_t n) { return n + 4 + 14 + 4 + 3 * ((n + 999) / 1000); }

int64_t chain_encoded_bound(const Chain &c, uint64_t nelem) {
  if (c.a2b.kind != CodecKind::Bytes) return -1;
  uint64_t n = nelem * c.es;
  for (const Codec &k : c.b2b) {
    if (k.kind == CodecKind::Crc32c) n += 4;
    else if (k.kind == CodecKind::Gzip) n = gzip_bound(n);
    else if (k.kind == CodecKind::Zstd) n = zstd_bound(n);
    else if (k.kind == CodecKind::Blosc) n += 16;  // BLOSC_MAX_OVERHEAD (blosc_via_blosc_src.rs:80)
    else if (k.kind != CodecKind::Shuffle) return -1;
  }
  return (int64_t)n;
}

}  // namespace zgpu
