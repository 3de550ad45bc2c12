/*
 * zarrs_oracle.c — CPU restatement of the zarrs chunk-decode pipeline.
 * TEST INFRASTRUCTURE ONLY (parity oracle + timed CPU baseline). See zarrs_oracle.h.
 *
 * Reference citations are relative to the zarrs workspace root (zarrs 0.24.0-dev):
 *   CC = zarrs/src/array/codec/array_to_bytes/codec_chain.rs
 *   SH = zarrs/src/array/codec/array_to_bytes/sharding.rs
 *   SC = zarrs/src/array/codec/array_to_bytes/sharding/sharding_codec.rs
 *   SP = zarrs/src/array/codec/array_to_bytes/sharding/sharding_partial_decoder_sync.rs
 *   TR = zarrs/src/array/codec/array_to_array/transpose.rs
 *   BY = zarrs_data_type/src/codec_traits/bytes.rs
 *   CR = zarrs/src/array/codec/bytes_to_bytes/crc32c/crc32c_codec.rs
 *   GZ = zarrs/src/array/codec/bytes_to_bytes/gzip/gzip_codec.rs
 *   ZS = zarrs/src/array/codec/bytes_to_bytes/zstd/zstd_codec.rs
 *   SF = zarrs/src/array/codec/bytes_to_bytes/shuffle/shuffle_codec.rs
 *   RO = zarrs/src/array/array_ops/array_read_ops_common.rs, RA = .../array_read_ops_array.rs
 */
#include "zarrs_oracle.h"

#include <pthread.h>
#include <stdatomic.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* ---- libzstd.so.1 public ABI (the image ships the library without its header) ---- */
typedef struct ZSTD_CCtx_s ZSTD_CCtx;
typedef struct ZSTD_DCtx_s ZSTD_DStream;
typedef struct { const void *src; size_t size; size_t pos; } ZSTD_inBuffer;
typedef struct { void *dst; size_t size; size_t pos; } ZSTD_outBuffer;
extern unsigned ZSTD_isError(size_t code);
extern unsigned long long ZSTD_decompressBound(const void *src, size_t srcSize);
extern size_t ZSTD_decompress(void *dst, size_t dstCapacity, const void *src, size_t srcSize);
extern ZSTD_CCtx *ZSTD_createCCtx(void);
extern size_t ZSTD_freeCCtx(ZSTD_CCtx *);
extern size_t ZSTD_CCtx_setParameter(ZSTD_CCtx *, int param, int value);
extern size_t ZSTD_compress2(ZSTD_CCtx *, void *dst, size_t cap, const void *src, size_t n);
extern size_t ZSTD_compressBound(size_t srcSize);
extern ZSTD_DStream *ZSTD_createDStream(void);
extern size_t ZSTD_freeDStream(ZSTD_DStream *);
extern size_t ZSTD_initDStream(ZSTD_DStream *);
extern size_t ZSTD_decompressStream(ZSTD_DStream *, ZSTD_outBuffer *, ZSTD_inBuffer *);
/* ---- c-blosc 1.21 public ABI (blosc-src 0.3.6 vendors c-blosc 1.21.x; zarrs/Cargo.toml:103) ---- */
extern int blosc_cbuffer_validate(const void *cbuffer, size_t cbytes, size_t *nbytes);
extern int blosc_decompress_ctx(const void *src, void *dest, size_t destsize, int numinternalthreads);
extern int blosc_compress_ctx(int clevel, int doshuffle, size_t typesize, size_t nbytes, const void *src,
                              void *dest, size_t destsize, const char *compressor, size_t blocksize,
                              int numinternalthreads);
#define ZSTD_c_compressionLevel 100
#define ZSTD_c_checksumFlag 201
#define ZSTD_CONTENTSIZE_ERROR (0ULL - 2)

#define MAXD 8
enum { K_TRANSPOSE = 1, K_BYTES, K_SHARDING, K_CRC32C, K_GZIP, K_ZSTD, K_SHUFFLE, K_BLOSC };

typedef struct {
  int kind;
  uint32_t ndim;
  uint32_t order[MAXD];      /* transpose */
  int big_endian;            /* bytes */
  int at_start;              /* crc32c location / sharding index_location */
  int level, checksum;       /* gzip / zstd */
  int bl_shuffle;            /* blosc: 0 noshuffle, 1 shuffle, 2 bitshuffle */
  uint32_t bl_typesize;      /* blosc */
  uint64_t bl_blocksize;     /* blosc (0 = automatic) */
  char bl_cname[16];         /* blosc compressor name */
  uint32_t elementsize;      /* shuffle */
  uint64_t inner[MAXD];      /* sharding subchunk shape */
  orc_chain *inner_chain, *index_chain;
} codec_t;

struct orc_chain {
  uint32_t es, comp;
  uint8_t fill[16];
  int n_a2a, has_a2b, n_b2b;
  codec_t a2a[8], a2b, b2b[8];
};

typedef struct { uint8_t *p; uint64_t n; int owned; } buf_t;

static void buf_drop(buf_t *b) {
  if (b->owned) free(b->p);
  b->p = NULL; b->n = 0; b->owned = 0;
}

static uint64_t prod(uint32_t nd, const uint64_t *s) {
  uint64_t p = 1;
  for (uint32_t i = 0; i < nd; i++) p *= s[i];
  return p;
}

const char *orc_status_name(int s) {
  static const char *names[] = {"OK", "INVALID_CHECKSUM", "DECODED_SIZE_MISMATCH",
                                "SHARD_INDEX_OOB", "CORRUPT_STREAM", "INVALID_BYTE_RANGE",
                                "UNSUPPORTED", "CRC_INPUT_TOO_SHORT", "SHARD_TOO_SMALL",
                                "SHUFFLE_LENGTH", "INVALID_ARGUMENT"};
  return (s >= 0 && s <= 10) ? names[s] : "UNKNOWN";
}

/* ===================== checksums ===================== */
static uint32_t crc32c_tab[8][256];
static pthread_once_t crc_once = PTHREAD_ONCE_INIT;
static void crc_init(void) {
  for (uint32_t i = 0; i < 256; i++) {
    uint32_t c = i;
    for (int k = 0; k < 8; k++) c = (c & 1) ? (c >> 1) ^ 0x82F63B78u : c >> 1;
    crc32c_tab[0][i] = c;
  }
  for (uint32_t i = 0; i < 256; i++)
    for (int t = 1; t < 8; t++)
      crc32c_tab[t][i] = (crc32c_tab[t - 1][i] >> 8) ^ crc32c_tab[0][crc32c_tab[t - 1][i] & 0xff];
}

/* crc32c crate semantics: crc32c(data) = reflected Castagnoli, init/xorout 0xFFFFFFFF.
 * `crc` is a previous result for chaining (0 for a fresh checksum). */
uint32_t orc_crc32c(uint32_t crc, const uint8_t *p, uint64_t n) {
  pthread_once(&crc_once, crc_init);
  uint32_t c = ~crc;
  while (n >= 8) { /* slice-by-8 */
    uint32_t lo = c ^ ((uint32_t)p[0] | (uint32_t)p[1] << 8 | (uint32_t)p[2] << 16 | (uint32_t)p[3] << 24);
    uint32_t hi = (uint32_t)p[4] | (uint32_t)p[5] << 8 | (uint32_t)p[6] << 16 | (uint32_t)p[7] << 24;
    c = crc32c_tab[7][lo & 0xff] ^ crc32c_tab[6][(lo >> 8) & 0xff] ^ crc32c_tab[5][(lo >> 16) & 0xff] ^
        crc32c_tab[4][lo >> 24] ^ crc32c_tab[3][hi & 0xff] ^ crc32c_tab[2][(hi >> 8) & 0xff] ^
        crc32c_tab[1][(hi >> 16) & 0xff] ^ crc32c_tab[0][hi >> 24];
    p += 8; n -= 8;
  }
  while (n--) c = (c >> 8) ^ crc32c_tab[0][(c ^ *p++) & 0xff];
  return ~c;
}

uint32_t orc_crc32_ieee(const uint8_t *p, uint64_t n) {
  uLong c = crc32(0L, Z_NULL, 0);
  while (n) {
    uInt k = n > (1u << 30) ? (1u << 30) : (uInt)n;
    c = crc32(c, p, k);
    p += k; n -= k;
  }
  return (uint32_t)c;
}

/* ===================== chain construction ===================== */
orc_chain *orc_chain_new(uint32_t es, uint32_t comp, const void *fill) {
  if (es == 0 || es > 16 || comp == 0 || es % comp) return NULL;
  orc_chain *c = calloc(1, sizeof(*c));
  c->es = es; c->comp = comp;
  if (fill) memcpy(c->fill, fill, es);
  return c;
}

void orc_chain_free(orc_chain *c) {
  if (!c) return;
  if (c->has_a2b && c->a2b.kind == K_SHARDING) {
    orc_chain_free(c->a2b.inner_chain);
    orc_chain_free(c->a2b.index_chain);
  }
  free(c);
}

int orc_chain_add_transpose(orc_chain *c, uint32_t nd, const uint32_t *order) {
  if (c->has_a2b || c->n_a2a >= 8 || nd > MAXD) return ORC_INVALID_ARGUMENT;
  uint32_t seen = 0;
  for (uint32_t i = 0; i < nd; i++) {
    if (order[i] >= nd || (seen >> order[i]) & 1) return ORC_INVALID_ARGUMENT;
    seen |= 1u << order[i];
  }
  codec_t *k = &c->a2a[c->n_a2a++];
  memset(k, 0, sizeof(*k));
  k->kind = K_TRANSPOSE; k->ndim = nd;
  memcpy(k->order, order, nd * sizeof(uint32_t));
  return ORC_OK;
}

int orc_chain_add_bytes(orc_chain *c, int big) {
  if (c->has_a2b) return ORC_INVALID_ARGUMENT;
  memset(&c->a2b, 0, sizeof(codec_t));
  c->a2b.kind = K_BYTES; c->a2b.big_endian = big; c->has_a2b = 1;
  return ORC_OK;
}

int orc_chain_add_sharding(orc_chain *c, uint32_t nd, const uint64_t *inner, orc_chain *ic,
                           orc_chain *xc, int at_start) {
  if (c->has_a2b || nd > MAXD || !ic || !xc) return ORC_INVALID_ARGUMENT;
  memset(&c->a2b, 0, sizeof(codec_t));
  c->a2b.kind = K_SHARDING; c->a2b.ndim = nd;
  memcpy(c->a2b.inner, inner, nd * 8);
  c->a2b.inner_chain = ic; c->a2b.index_chain = xc; c->a2b.at_start = at_start;
  c->has_a2b = 1;
  return ORC_OK;
}

static codec_t *add_b2b(orc_chain *c, int kind) {
  if (!c->has_a2b || c->n_b2b >= 8) return NULL;
  codec_t *k = &c->b2b[c->n_b2b++];
  memset(k, 0, sizeof(*k));
  k->kind = kind;
  return k;
}
int orc_chain_add_crc32c(orc_chain *c, int at_start) {
  codec_t *k = add_b2b(c, K_CRC32C);
  if (!k) return ORC_INVALID_ARGUMENT;
  k->at_start = at_start;
  return ORC_OK;
}
int orc_chain_add_gzip(orc_chain *c, int level) {
  codec_t *k = add_b2b(c, K_GZIP);
  if (!k) return ORC_INVALID_ARGUMENT;
  k->level = level;
  return ORC_OK;
}
int orc_chain_add_zstd(orc_chain *c, int level, int checksum) {
  codec_t *k = add_b2b(c, K_ZSTD);
  if (!k) return ORC_INVALID_ARGUMENT;
  k->level = level; k->checksum = checksum;
  return ORC_OK;
}
/* BL = zarrs/src/array/codec/bytes_to_bytes/blosc/{blosc_codec_via_blosc_src.rs,blosc_via_blosc_src.rs} */
int orc_chain_add_blosc(orc_chain *c, const char *cname, int clevel, int shuffle, uint32_t typesize,
                        uint64_t blocksize) {
  if (!cname || strlen(cname) >= 16 || shuffle < 0 || shuffle > 2) return ORC_INVALID_ARGUMENT;
  codec_t *k = add_b2b(c, K_BLOSC);
  if (!k) return ORC_INVALID_ARGUMENT;
  k->level = clevel; k->bl_shuffle = shuffle; k->bl_typesize = typesize; k->bl_blocksize = blocksize;
  strcpy(k->bl_cname, cname);
  return ORC_OK;
}
int orc_chain_add_shuffle(orc_chain *c, uint32_t es) {
  if (es == 0) return ORC_INVALID_ARGUMENT;
  codec_t *k = add_b2b(c, K_SHUFFLE);
  if (!k) return ORC_INVALID_ARGUMENT;
  k->elementsize = es;
  return ORC_OK;
}

/* encoded byte size for a fixed decoded size (encoded_representation), -1 if not fixed.
 * bytes/transpose/sharding(no)/crc32c(+4)/shuffle(same)/gzip,zstd(unbounded). */
static int64_t chain_fixed_encoded_size(const orc_chain *c, uint64_t nelem) {
  if (!c->has_a2b || c->a2b.kind != K_BYTES) return -1;
  int64_t n = (int64_t)(nelem * c->es);
  for (int i = 0; i < c->n_b2b; i++) {
    switch (c->b2b[i].kind) {
      case K_CRC32C: n += 4; break;
      case K_SHUFFLE: break;
      default: return -1;
    }
  }
  return n;
}

void orc_free(void *p) { free(p); }

/* ===================== bytes->bytes decode (reverse order) ===================== */
/* CR:108-141 (full) / CR:143-158 + strip_suffix_partial_decoder.rs:39-62 (partial: strip only) */
static int crc32c_decode(const codec_t *k, buf_t *b, int verify) {
  if (b->n < 4) return ORC_CRC_INPUT_TOO_SHORT;
  const uint8_t *data = k->at_start ? b->p + 4 : b->p;
  const uint8_t *stored = k->at_start ? b->p : b->p + b->n - 4;
  uint64_t n = b->n - 4;
  if (verify) {
    uint32_t c = orc_crc32c(0, data, n);
    uint8_t le[4] = {c & 0xff, (c >> 8) & 0xff, (c >> 16) & 0xff, c >> 24};
    if (memcmp(le, stored, 4) != 0) return ORC_INVALID_CHECKSUM;
  }
  /* decode returns data.to_vec(): a copy (kept for cost parity with the reference) */
  uint8_t *o = malloc(n ? n : 1);
  memcpy(o, data, n);
  buf_drop(b);
  b->p = o; b->n = n; b->owned = 1;
  return ORC_OK;
}

/* GZ:110-120 — flate2 GzDecoder::read_to_end: first gzip member, trailer CRC-32 + ISIZE checked */
static int gzip_decode(buf_t *b, uint64_t hint) {
  z_stream s;
  memset(&s, 0, sizeof(s));
  if (inflateInit2(&s, 15 + 16) != Z_OK) return ORC_CORRUPT_STREAM;
  uint64_t cap = hint ? hint : (b->n * 4 + 64), len = 0;
  uint8_t *o = malloc(cap);
  s.next_in = b->p;
  uint64_t in_left = b->n;
  int r;
  for (;;) {
    if (len == cap) { cap *= 2; o = realloc(o, cap); }
    uInt ain = in_left > (1u << 30) ? (1u << 30) : (uInt)in_left;
    s.avail_in = ain;
    uInt aout = (cap - len) > (1u << 30) ? (1u << 30) : (uInt)(cap - len);
    s.next_out = o + len; s.avail_out = aout;
    r = inflate(&s, Z_NO_FLUSH);
    len += aout - s.avail_out;
    in_left -= ain - s.avail_in;
    if (r == Z_STREAM_END) break;
    if (r == Z_BUF_ERROR && s.avail_out != 0) { r = Z_DATA_ERROR; break; } /* truncated input */
    if (r != Z_OK && r != Z_BUF_ERROR) break;
  }
  inflateEnd(&s);
  if (r != Z_STREAM_END) { free(o); return ORC_CORRUPT_STREAM; }
  buf_drop(b);
  b->p = o; b->n = len; b->owned = 1;
  return ORC_OK;
}

/* BL blosc_codec_via_blosc_src.rs:132-142 (do_decode): blosc_validate -> destsize, then
 * blosc_decompress_ctx (blosc_via_blosc_src.rs:115-121,162-191); invalid -> CodecError::Other */
static int blosc_decode(buf_t *b) {
  size_t dest = 0;
  if (blosc_cbuffer_validate(b->p, b->n, &dest) != 0) return ORC_CORRUPT_STREAM;
  uint8_t *o = malloc(dest ? dest : 1);
  int r = blosc_decompress_ctx(b->p, o, dest, 1);
  if (r < 0 || (size_t)r != dest || (r == 0 && dest != 0)) { free(o); return ORC_CORRUPT_STREAM; }
  buf_drop(b); b->p = o; b->n = dest; b->owned = 1;
  return ORC_OK;
}

/* ZS:113-130 — bulk decompress with ZSTD_decompressBound, else streaming decode_all */
static int zstd_decode(buf_t *b) {
  unsigned long long bound = ZSTD_decompressBound(b->p, b->n);
  if (bound != ZSTD_CONTENTSIZE_ERROR) {
    uint8_t *o = malloc(bound ? bound : 1);
    size_t r = ZSTD_decompress(o, bound, b->p, b->n);
    if (ZSTD_isError(r)) { free(o); return ORC_CORRUPT_STREAM; }
    buf_drop(b);
    b->p = o; b->n = r; b->owned = 1;
    return ORC_OK;
  }
  ZSTD_DStream *ds = ZSTD_createDStream();
  ZSTD_initDStream(ds);
  uint64_t cap = b->n * 4 + 1024, len = 0;
  uint8_t *o = malloc(cap);
  ZSTD_inBuffer in = {b->p, b->n, 0};
  for (;;) {
    if (cap - len < 65536) { cap *= 2; o = realloc(o, cap); }
    ZSTD_outBuffer out = {o + len, cap - len, 0};
    size_t r = ZSTD_decompressStream(ds, &out, &in);
    len += out.pos;
    if (ZSTD_isError(r)) { free(o); ZSTD_freeDStream(ds); return ORC_CORRUPT_STREAM; }
    if (in.pos == in.size && out.pos < out.size) {
      if (r != 0) { free(o); ZSTD_freeDStream(ds); return ORC_CORRUPT_STREAM; }
      break;
    }
  }
  ZSTD_freeDStream(ds);
  buf_drop(b);
  b->p = o; b->n = len; b->owned = 1;
  return ORC_OK;
}

/* SF:109-129 */
static int shuffle_decode(const codec_t *k, buf_t *b) {
  uint64_t es = k->elementsize;
  if (b->n % es) return ORC_SHUFFLE_LENGTH;
  uint64_t count = b->n / es, n = b->n;
  uint8_t *o = malloc(n ? n : 1);
  for (uint64_t i = 0; i < es; i++) {
    const uint8_t *src = b->p + i * count;
    for (uint64_t j = 0; j < count; j++) o[j * es + i] = src[j];
  }
  buf_drop(b);
  b->p = o; b->n = n; b->owned = 1;
  return ORC_OK;
}

/* ===================== index helpers (zarrs_chunk_grid ravel/unravel) ===================== */
static void cstrides(uint32_t nd, const uint64_t *shape, uint64_t *st) {
  uint64_t s = 1;
  for (int d = (int)nd - 1; d >= 0; d--) { st[d] = s; s *= shape[d]; }
}

/* Copy region [src_start, src_start+shape) of a C-order array `src` (src_shape) into
 * region at dst_start of C-order `dst` (dst_shape); element size es.
 * ArrayBytesFixedDisjointView::copy_from_slice (array_bytes_fixed_disjoint_view.rs:177-206). */
static void copy_region(uint32_t nd, uint64_t es, const uint8_t *src, const uint64_t *src_shape,
                        const uint64_t *src_start, uint8_t *dst, const uint64_t *dst_shape,
                        const uint64_t *dst_start, const uint64_t *shape) {
  if (nd == 0) { memcpy(dst, src, es); return; }
  if (prod(nd, shape) == 0) return;
  uint64_t ss[MAXD], ds[MAXD], idx[MAXD] = {0};
  cstrides(nd, src_shape, ss);
  cstrides(nd, dst_shape, ds);
  uint64_t run = shape[nd - 1] * es;
  for (;;) {
    uint64_t so = 0, doff = 0;
    for (uint32_t d = 0; d < nd; d++) {
      so += (src_start[d] + idx[d]) * ss[d];
      doff += (dst_start[d] + idx[d]) * ds[d];
    }
    memcpy(dst + doff * es, src + so * es, run);
    int d = (int)nd - 2;
    for (; d >= 0; d--) {
      if (++idx[d] < shape[d]) break;
      idx[d] = 0;
    }
    if (d < 0) break;
  }
}

/* ArrayBytesFixedDisjointView::fill (array_bytes_fixed_disjoint_view.rs:144-166) */
static void fill_region(uint32_t nd, uint64_t es, const uint8_t *fill, uint8_t *dst,
                        const uint64_t *dst_shape, const uint64_t *dst_start,
                        const uint64_t *shape) {
  if (prod(nd, shape) == 0) return;
  uint64_t ds[MAXD], idx[MAXD] = {0};
  cstrides(nd, dst_shape, ds);
  for (;;) {
    uint64_t doff = 0;
    for (uint32_t d = 0; d < nd; d++) doff += (dst_start[d] + idx[d]) * ds[d];
    for (uint64_t i = 0; i < shape[nd - 1]; i++) memcpy(dst + (doff + i) * es, fill, es);
    int d = (int)nd - 2;
    for (; d >= 0; d--) {
      if (++idx[d] < shape[d]) break;
      idx[d] = 0;
    }
    if (d < 0) break;
  }
}

/* TR:223-266 + transpose_codec.rs:264-281. Decode: input has the encoded shape
 * E = permute(D, order); output dec[c] = enc[e], e_a = c[order[a]]. `encode` reverses. */
static void transpose_apply(uint32_t nd, const uint32_t *order, const uint64_t *dshape, uint64_t es,
                            const uint8_t *in, uint8_t *out, int encode) {
  uint64_t eshape[MAXD], est[MAXD], sd[MAXD], idx[MAXD] = {0};
  for (uint32_t a = 0; a < nd; a++) eshape[a] = dshape[order[a]];
  cstrides(nd, eshape, est);
  for (uint32_t a = 0; a < nd; a++) sd[order[a]] = est[a]; /* encoded stride of decoded axis */
  uint64_t n = prod(nd, dshape);
  if (n == 0) return;
  for (uint64_t lin = 0; lin < n; lin++) {
    uint64_t e = 0;
    for (uint32_t d = 0; d < nd; d++) e += idx[d] * sd[d];
    if (encode) memcpy(out + e * es, in + lin * es, es);
    else memcpy(out + lin * es, in + e * es, es);
    for (int d = (int)nd - 1; d >= 0; d--) {
      if (++idx[d] < dshape[d]) break;
      idx[d] = 0;
    }
  }
}

/* BY:97-131 — reverse every component when the stored endianness is not native (LE host) */
static void byteswap(uint8_t *p, uint64_t n, uint32_t comp) {
  if (comp <= 1) return;
  for (uint64_t i = 0; i + comp <= n; i += comp)
    for (uint32_t a = 0, b = comp - 1; a < b; a++, b--) {
      uint8_t t = p[i + a]; p[i + a] = p[i + b]; p[i + b] = t;
    }
}

/* ===================== chain decode (region form) ===================== */
static int decode_region(const orc_chain *c, const uint8_t *enc, uint64_t len, uint32_t nd,
                         const uint64_t *shape, const uint64_t *sel_start,
                         const uint64_t *sel_shape, int partial, int validate, uint8_t *out,
                         const uint64_t *out_shape, const uint64_t *out_start);

/* Inner (codec) concurrency of the calling chunk task: zarrs splits its thread budget into outer
 * (chunks) x inner (subchunks of a shard), concurrency.rs:23-69 / sharding_codec.rs:648-655. */
static __thread int g_inner_threads = 1;

typedef struct {
  const orc_chain *ic;
  const uint8_t *enc;
  uint64_t len;
  uint32_t nd;
  const uint64_t *inner, *out_shape;
  uint8_t *out;
  int partial, validate;
  uint64_t n;
  const uint64_t *work;  /* per item: off, size, cst[nd], osh[nd], opos[nd] */
  atomic_ullong next;
  atomic_int err;
} inner_job_t;

static void *inner_worker(void *arg) {
  inner_job_t *J = arg;
  const uint32_t nd = J->nd, stride = 2 + 3 * nd;
  for (;;) {
    uint64_t t = atomic_fetch_add(&J->next, 1);
    if (t >= J->n) break;
    const uint64_t *w = J->work + t * stride;
    int st = decode_region(J->ic, J->enc + w[0], w[1], nd, J->inner, w + 2, w + 2 + nd, J->partial, J->validate,
                           J->out, J->out_shape, w + 2 + 2 * nd);
    if (st) {
      int z = 0;
      atomic_compare_exchange_strong(&J->err, &z, st);
    }
  }
  return NULL;
}

/* Shard decode into an output region. Full path: SC:617-707 (all subchunks, crc verified);
 * partial path: SP:311-400 (intersecting subchunks, inner partial decoders, crc stripped only).
 * Index: SH:178-194, SC:1262-1298 (index chain fully decoded, crc verified in both paths). */
static int shard_region(const orc_chain *c, const uint8_t *enc, uint64_t len, uint32_t nd,
                        const uint64_t *shape, const uint64_t *sel_start, const uint64_t *sel_shape,
                        int partial, int validate, uint8_t *out, const uint64_t *out_shape,
                        const uint64_t *out_start) {
  const codec_t *k = &c->a2b;
  if (k->ndim != nd) return ORC_INVALID_ARGUMENT;
  uint64_t cps[MAXD + 1], n_inner = 1;
  for (uint32_t d = 0; d < nd; d++) { /* SH:136-154 */
    if (k->inner[d] == 0 || shape[d] % k->inner[d]) return ORC_INVALID_ARGUMENT;
    cps[d] = shape[d] / k->inner[d];
    n_inner *= cps[d];
  }
  cps[nd] = 2; /* SH:156-161 */
  int64_t isz = chain_fixed_encoded_size(k->index_chain, n_inner * 2);
  if (isz < 0) return ORC_UNSUPPORTED; /* index chain must be FixedSize, SH:163-176 */
  if (len < (uint64_t)isz) return ORC_SHARD_TOO_SMALL;
  const uint8_t *ienc = k->at_start ? enc : enc + len - isz;
  uint64_t *index = malloc(n_inner * 16);
  int st = decode_region(k->index_chain, ienc, (uint64_t)isz, nd + 1, cps, (uint64_t[MAXD + 1]){0},
                         cps, 0, validate, (uint8_t *)index, cps, (uint64_t[MAXD + 1]){0});
  if (st) { free(index); return st; }
  uint64_t lo[MAXD], hi[MAXD], idx[MAXD];
  for (uint32_t d = 0; d < nd; d++) {
    lo[d] = sel_start[d] / k->inner[d];
    hi[d] = sel_shape[d] ? (sel_start[d] + sel_shape[d] - 1) / k->inner[d] + 1 : lo[d];
    if (hi[d] == lo[d]) { free(index); return ORC_OK; }
    idx[d] = lo[d];
  }
  if (g_inner_threads > 1) {
    /* collect the intersecting subchunks, fill/validate serially, decode on inner threads */
    const uint32_t stride = 2 + 3 * nd;
    uint64_t cap = 1;
    for (uint32_t d = 0; d < nd; d++) cap *= hi[d] - lo[d];
    uint64_t *work = malloc(cap * stride * 8), nw = 0;
    for (;;) {
      uint64_t lin = 0, *w = work + nw * stride;
      for (uint32_t d = 0; d < nd; d++) {
        lin = lin * cps[d] + idx[d];
        uint64_t cs = idx[d] * k->inner[d], ce = cs + k->inner[d];
        uint64_t s0 = sel_start[d] > cs ? sel_start[d] : cs;
        uint64_t s1 = sel_start[d] + sel_shape[d] < ce ? sel_start[d] + sel_shape[d] : ce;
        w[2 + d] = s0 - cs;
        w[2 + nd + d] = s1 - s0;
        w[2 + 2 * nd + d] = out_start[d] + (s0 - sel_start[d]);
      }
      uint64_t off = index[2 * lin], size = index[2 * lin + 1];
      if (off == UINT64_MAX && size == UINT64_MAX) {
        fill_region(nd, c->es, c->fill, out, out_shape, w + 2 + 2 * nd, w + 2 + nd);
      } else if (off > len || size > len - off) {
        free(work);
        free(index);
        return ORC_SHARD_INDEX_OOB;
      } else {
        w[0] = off;
        w[1] = size;
        nw++;
      }
      int d = (int)nd - 1;
      for (; d >= 0; d--) {
        if (++idx[d] < hi[d]) break;
        idx[d] = lo[d];
      }
      if (d < 0) break;
    }
    inner_job_t J;
    memset(&J, 0, sizeof(J));
    J.ic = k->inner_chain; J.enc = enc; J.len = len; J.nd = nd; J.inner = k->inner;
    J.out_shape = out_shape; J.out = out; J.partial = partial; J.validate = validate; J.n = nw; J.work = work;
    atomic_init(&J.next, 0);
    atomic_init(&J.err, 0);
    int nt = g_inner_threads < 64 ? g_inner_threads : 64;
    if ((uint64_t)nt > nw) nt = nw ? (int)nw : 1;
    pthread_t th[64];
    for (int i = 1; i < nt; i++) pthread_create(&th[i], NULL, inner_worker, &J);
    inner_worker(&J);
    for (int i = 1; i < nt; i++) pthread_join(th[i], NULL);
    free(work);
    free(index);
    return atomic_load(&J.err);
  }
  for (;;) {
    uint64_t lin = 0, cst[MAXD], ost[MAXD], osh[MAXD], opos[MAXD];
    for (uint32_t d = 0; d < nd; d++) {
      lin = lin * cps[d] + idx[d];
      uint64_t cs = idx[d] * k->inner[d], ce = cs + k->inner[d];
      uint64_t s0 = sel_start[d] > cs ? sel_start[d] : cs;
      uint64_t s1 = sel_start[d] + sel_shape[d] < ce ? sel_start[d] + sel_shape[d] : ce;
      cst[d] = s0 - cs; osh[d] = s1 - s0;
      opos[d] = out_start[d] + (s0 - sel_start[d]);
      ost[d] = cs;
    }
    (void)ost;
    uint64_t off = index[2 * lin], size = index[2 * lin + 1];
    if (off == UINT64_MAX && size == UINT64_MAX) {
      fill_region(nd, c->es, c->fill, out, out_shape, opos, osh);
    } else if (off > len || size > len - off) {
      free(index);
      return ORC_SHARD_INDEX_OOB;
    } else {
      st = decode_region(k->inner_chain, enc + off, size, nd, k->inner, cst, osh, partial, validate,
                         out, out_shape, opos);
      if (st) { free(index); return st; }
    }
    int d = (int)nd - 1;
    for (; d >= 0; d--) {
      if (++idx[d] < hi[d]) break;
      idx[d] = lo[d];
    }
    if (d < 0) break;
  }
  free(index);
  return ORC_OK;
}

/* CC:557-646 — b2b decode in reverse, a2b decode, a2a decode in reverse, then copy into the
 * output view. `partial`=1 restates the partial-decoder chain (CC:684-745): crc32c strips only. */
static int decode_region(const orc_chain *c, const uint8_t *enc, uint64_t len, uint32_t nd,
                         const uint64_t *shape, const uint64_t *sel_start,
                         const uint64_t *sel_shape, int partial, int validate, uint8_t *out,
                         const uint64_t *out_shape, const uint64_t *out_start) {
  if (!c->has_a2b) return ORC_INVALID_ARGUMENT;
  uint64_t shapes[9][MAXD];
  memcpy(shapes[0], shape, nd * 8);
  for (int i = 0; i < c->n_a2a; i++) {
    if (c->a2a[i].ndim != nd) return ORC_INVALID_ARGUMENT;
    for (uint32_t a = 0; a < nd; a++) shapes[i + 1][a] = shapes[i][c->a2a[i].order[a]];
  }
  const uint64_t *ashape = shapes[c->n_a2a];
  uint64_t nelem = prod(nd, shape), nbytes = nelem * c->es;
  buf_t b = {(uint8_t *)enc, len, 0};
  for (int i = c->n_b2b - 1; i >= 0; i--) {
    const codec_t *k = &c->b2b[i];
    int st = ORC_OK;
    switch (k->kind) {
      case K_CRC32C: st = crc32c_decode(k, &b, validate && !partial); break;
      case K_GZIP: st = gzip_decode(&b, i == 0 ? nbytes : 0); break;
      case K_ZSTD: st = zstd_decode(&b); break;
      case K_SHUFFLE: st = shuffle_decode(k, &b); break;
      case K_BLOSC: st = blosc_decode(&b); break;
      default: st = ORC_UNSUPPORTED;
    }
    if (st) { buf_drop(&b); return st; }
  }
  uint64_t zero[MAXD] = {0};
  int full_sel = 1;
  for (uint32_t d = 0; d < nd; d++)
    if (sel_start[d] != 0 || sel_shape[d] != shape[d]) full_sel = 0;
  if (c->a2b.kind == K_SHARDING) {
    int st;
    if (c->n_a2a == 0) {
      st = shard_region(c, b.p, b.n, nd, shape, sel_start, sel_shape, partial, validate, out,
                        out_shape, out_start);
    } else { /* a2a before sharding: decode the whole shard, then permute (rare) */
      uint8_t *tmp = malloc(nbytes ? nbytes : 1);
      st = shard_region(c, b.p, b.n, nd, ashape, zero, ashape, partial, validate, tmp, ashape, zero);
      for (int i = c->n_a2a - 1; i >= 0 && !st; i--) {
        uint8_t *t2 = malloc(nbytes ? nbytes : 1);
        transpose_apply(nd, c->a2a[i].order, shapes[i], c->es, tmp, t2, 0);
        free(tmp); tmp = t2;
      }
      if (!st) copy_region(nd, c->es, tmp, shape, sel_start, out, out_shape, out_start, sel_shape);
      free(tmp);
    }
    buf_drop(&b);
    return st;
  }
  /* bytes codec: bytes_codec.rs:203-219; size check = ArrayBytes::validate (array_bytes.rs:376-386) */
  if (b.n != nbytes) { buf_drop(&b); return ORC_DECODED_SIZE_MISMATCH; }
  if (c->a2b.big_endian && c->comp > 1) {
    if (!b.owned) { /* Cow::into_owned */
      uint8_t *o = malloc(nbytes ? nbytes : 1);
      memcpy(o, b.p, nbytes);
      b.p = o; b.owned = 1;
    }
    byteswap(b.p, nbytes, c->comp);
  }
  for (int i = c->n_a2a - 1; i >= 0; i--) {
    uint8_t *o = malloc(nbytes ? nbytes : 1);
    transpose_apply(nd, c->a2a[i].order, shapes[i], c->es, b.p, o, 0);
    buf_drop(&b);
    b.p = o; b.n = nbytes; b.owned = 1;
  }
  if (full_sel && out_shape == shape) {
    memcpy(out, b.p, nbytes);
  } else {
    copy_region(nd, c->es, b.p, shape, sel_start, out, out_shape, out_start, sel_shape);
  }
  buf_drop(&b);
  return ORC_OK;
}

int orc_decode_chunk(const orc_chain *c, const uint8_t *enc, uint64_t len, uint32_t nd,
                     const uint64_t *shape, int validate, uint8_t *out) {
  uint64_t zero[MAXD] = {0};
  if (nd > MAXD) return ORC_INVALID_ARGUMENT;
  return decode_region(c, enc, len, nd, shape, zero, shape, 0, validate, out, shape, zero);
}

/* ===================== encode (test-data generation) ===================== */
static int b2b_encode(const codec_t *k, buf_t *b) {
  switch (k->kind) {
    case K_CRC32C: { /* CR:88-106 */
      uint32_t cs = orc_crc32c(0, b->p, b->n);
      uint8_t *o = malloc(b->n + 4), le[4] = {cs & 0xff, (cs >> 8) & 0xff, (cs >> 16) & 0xff, cs >> 24};
      if (k->at_start) { memcpy(o, le, 4); memcpy(o + 4, b->p, b->n); }
      else { memcpy(o, b->p, b->n); memcpy(o + b->n, le, 4); }
      uint64_t n = b->n + 4;
      buf_drop(b); b->p = o; b->n = n; b->owned = 1;
      return ORC_OK;
    }
    case K_GZIP: {
      z_stream s;
      memset(&s, 0, sizeof(s));
      if (deflateInit2(&s, k->level, Z_DEFLATED, 15 + 16, 8, Z_DEFAULT_STRATEGY) != Z_OK)
        return ORC_INVALID_ARGUMENT;
      uint64_t cap = deflateBound(&s, b->n) + 64;
      uint8_t *o = malloc(cap);
      s.next_in = b->p; s.avail_in = (uInt)b->n;
      s.next_out = o; s.avail_out = (uInt)cap;
      int r = deflate(&s, Z_FINISH);
      uint64_t n = s.total_out;
      deflateEnd(&s);
      if (r != Z_STREAM_END) { free(o); return ORC_CORRUPT_STREAM; }
      buf_drop(b); b->p = o; b->n = n; b->owned = 1;
      return ORC_OK;
    }
    case K_ZSTD: { /* ZS:100-111 */
      ZSTD_CCtx *cc = ZSTD_createCCtx();
      ZSTD_CCtx_setParameter(cc, ZSTD_c_compressionLevel, k->level);
      ZSTD_CCtx_setParameter(cc, ZSTD_c_checksumFlag, k->checksum);
      size_t cap = ZSTD_compressBound(b->n);
      uint8_t *o = malloc(cap);
      size_t r = ZSTD_compress2(cc, o, cap, b->p, b->n);
      ZSTD_freeCCtx(cc);
      if (ZSTD_isError(r)) { free(o); return ORC_CORRUPT_STREAM; }
      buf_drop(b); b->p = o; b->n = r; b->owned = 1;
      return ORC_OK;
    }
    case K_BLOSC: { /* BL blosc_via_blosc_src.rs:64-110 (blosc_compress_bytes) */
      size_t cap = b->n + 16;
      uint8_t *o = malloc(cap);
      int r = blosc_compress_ctx(k->level, k->bl_shuffle, k->bl_typesize ? k->bl_typesize : 1, b->n, b->p, o, cap,
                                 k->bl_cname, k->bl_blocksize, 1);
      if (r <= 0) { free(o); return ORC_CORRUPT_STREAM; }
      buf_drop(b); b->p = o; b->n = (uint64_t)r; b->owned = 1;
      return ORC_OK;
    }
    case K_SHUFFLE: { /* SF:86-107 */
      uint64_t es = k->elementsize;
      if (b->n % es) return ORC_SHUFFLE_LENGTH;
      uint64_t count = b->n / es, n = b->n;
      uint8_t *o = malloc(n ? n : 1);
      for (uint64_t i = 0; i < count; i++)
        for (uint64_t j = 0; j < es; j++) o[j * count + i] = b->p[i * es + j];
      buf_drop(b); b->p = o; b->n = n; b->owned = 1;
      return ORC_OK;
    }
  }
  return ORC_UNSUPPORTED;
}

static int chain_encode(const orc_chain *c, const uint8_t *dec, uint32_t nd, const uint64_t *shape,
                        buf_t *res);

/* Shard encode (SC:873-1261 restated minimally): subchunks in lexicographic order; a subchunk
 * equal to the fill value everywhere is stored as empty (u64::MAX, u64::MAX). */
static int shard_encode(const orc_chain *c, const uint8_t *dec, uint32_t nd, const uint64_t *shape,
                        buf_t *res) {
  const codec_t *k = &c->a2b;
  uint64_t cps[MAXD + 1], n_inner = 1;
  for (uint32_t d = 0; d < nd; d++) {
    if (shape[d] % k->inner[d]) return ORC_INVALID_ARGUMENT;
    cps[d] = shape[d] / k->inner[d];
    n_inner *= cps[d];
  }
  cps[nd] = 2;
  uint64_t *index = malloc(n_inner * 16);
  uint64_t inner_n = prod(nd, k->inner), inner_b = inner_n * c->es;
  uint8_t *tmp = malloc(inner_b ? inner_b : 1);
  uint64_t cap = 1024, len = 0;
  uint8_t *body = malloc(cap);
  int64_t isz = chain_fixed_encoded_size(k->index_chain, n_inner * 2);
  if (isz < 0) { free(index); free(tmp); free(body); return ORC_UNSUPPORTED; }
  uint64_t base = k->at_start ? (uint64_t)isz : 0;
  uint64_t zero[MAXD] = {0};
  for (uint64_t lin = 0; lin < n_inner; lin++) {
    uint64_t rem = lin, st[MAXD];
    for (int d = (int)nd - 1; d >= 0; d--) { st[d] = (rem % cps[d]) * k->inner[d]; rem /= cps[d]; }
    copy_region(nd, c->es, dec, shape, st, tmp, k->inner, zero, k->inner);
    int all_fill = 1;
    for (uint64_t e = 0; e < inner_n && all_fill; e++)
      if (memcmp(tmp + e * c->es, c->fill, c->es)) all_fill = 0;
    if (all_fill) { index[2 * lin] = index[2 * lin + 1] = UINT64_MAX; continue; }
    buf_t eb;
    int r = chain_encode(k->inner_chain, tmp, nd, k->inner, &eb);
    if (r) { free(index); free(tmp); free(body); return r; }
    while (len + eb.n > cap) { cap *= 2; body = realloc(body, cap); }
    memcpy(body + len, eb.p, eb.n);
    index[2 * lin] = base + len; index[2 * lin + 1] = eb.n;
    len += eb.n;
    buf_drop(&eb);
  }
  buf_t ib;
  int r = chain_encode(k->index_chain, (uint8_t *)index, nd + 1, cps, &ib);
  free(index); free(tmp);
  if (r) { free(body); return r; }
  uint8_t *o = malloc(len + ib.n);
  if (k->at_start) { memcpy(o, ib.p, ib.n); memcpy(o + ib.n, body, len); }
  else { memcpy(o, body, len); memcpy(o + len, ib.p, ib.n); }
  res->p = o; res->n = len + ib.n; res->owned = 1;
  buf_drop(&ib); free(body);
  return ORC_OK;
}

static int chain_encode(const orc_chain *c, const uint8_t *dec, uint32_t nd, const uint64_t *shape,
                        buf_t *res) {
  if (!c->has_a2b) return ORC_INVALID_ARGUMENT;
  uint64_t nbytes = prod(nd, shape) * c->es;
  uint64_t shapes[9][MAXD];
  memcpy(shapes[0], shape, nd * 8);
  for (int i = 0; i < c->n_a2a; i++)
    for (uint32_t a = 0; a < nd; a++) shapes[i + 1][a] = shapes[i][c->a2a[i].order[a]];
  buf_t b;
  b.p = malloc(nbytes ? nbytes : 1); b.n = nbytes; b.owned = 1;
  memcpy(b.p, dec, nbytes);
  for (int i = 0; i < c->n_a2a; i++) {
    uint8_t *o = malloc(nbytes ? nbytes : 1);
    transpose_apply(nd, c->a2a[i].order, shapes[i], c->es, b.p, o, 1);
    buf_drop(&b); b.p = o; b.n = nbytes; b.owned = 1;
  }
  if (c->a2b.kind == K_SHARDING) {
    buf_t s;
    int r = shard_encode(c, b.p, nd, shapes[c->n_a2a], &s);
    buf_drop(&b);
    if (r) return r;
    b = s;
  } else if (c->a2b.big_endian) {
    byteswap(b.p, nbytes, c->comp);
  }
  for (int i = 0; i < c->n_b2b; i++) {
    int r = b2b_encode(&c->b2b[i], &b);
    if (r) { buf_drop(&b); return r; }
  }
  *res = b;
  return ORC_OK;
}

int orc_encode_chunk(const orc_chain *c, const uint8_t *dec, uint32_t nd, const uint64_t *shape,
                     uint8_t **enc, uint64_t *enc_len) {
  buf_t b;
  int r = chain_encode(c, dec, nd, shape, &b);
  if (r) return r;
  *enc = b.p; *enc_len = b.n;
  return ORC_OK;
}

/* ===================== array read op ===================== */
typedef struct {
  const orc_chain *c;
  uint32_t nd;
  const uint64_t *ashape, *cshape, *sel_start, *sel_shape;
  const uint8_t *const *ptrs;
  const uint64_t *lens;
  uint8_t *out;
  int validate;
  uint64_t lo[MAXD], hi[MAXD], ngrid[MAXD], n;
  atomic_ullong next;
  int *status;
  int inner_threads;
} job_t;

/* RO:111-179 retrieve_chunk closure + RA:346-375 full-vs-partial branch */
static int do_chunk(job_t *j, uint64_t t) {
  uint32_t nd = j->nd;
  uint64_t ci[MAXD], rem = t, lin = 0, gst[MAXD];
  for (int d = (int)nd - 1; d >= 0; d--) {
    uint64_t w = j->hi[d] - j->lo[d];
    ci[d] = j->lo[d] + rem % w; rem /= w;
  }
  for (uint32_t d = 0; d < nd; d++) {
    (void)gst;
    lin = lin * j->ngrid[d] + ci[d];
  }
  uint64_t cst[MAXD], osh[MAXD], opos[MAXD];
  int full = 1;
  for (uint32_t d = 0; d < nd; d++) {
    uint64_t cs = ci[d] * j->cshape[d], ce = cs + j->cshape[d];
    uint64_t s0 = j->sel_start[d] > cs ? j->sel_start[d] : cs;
    uint64_t s1 = j->sel_start[d] + j->sel_shape[d] < ce ? j->sel_start[d] + j->sel_shape[d] : ce;
    cst[d] = s0 - cs; osh[d] = s1 - s0; opos[d] = s0 - j->sel_start[d];
    if (cst[d] != 0 || osh[d] != j->cshape[d]) full = 0;
  }
  const uint8_t *p = j->ptrs[lin];
  if (!p) { /* missing chunk: copy_fill_value_into */
    fill_region(nd, j->c->es, j->c->fill, j->out, j->sel_shape, opos, osh);
    return ORC_OK;
  }
  return decode_region(j->c, p, j->lens[lin], nd, j->cshape, cst, osh, !full, j->validate, j->out,
                       j->sel_shape, opos);
}

static void *worker(void *arg) {
  job_t *j = arg;
  g_inner_threads = j->inner_threads;
  for (;;) {
    uint64_t t = atomic_fetch_add(&j->next, 1);
    if (t >= j->n) break;
    j->status[t] = do_chunk(j, t);
  }
  return NULL;
}

int orc_retrieve_array_subset(const orc_chain *c, uint32_t nd, const uint64_t *ashape,
                              const uint64_t *cshape, const uint8_t *const *ptrs,
                              const uint64_t *lens, const uint64_t *sel_start,
                              const uint64_t *sel_shape, uint8_t *out, int nthreads, int validate) {
  if (nd == 0 || nd > MAXD) return ORC_INVALID_ARGUMENT;
  job_t *j = calloc(1, sizeof(job_t));
  j->c = c; j->nd = nd; j->ashape = ashape; j->cshape = cshape; j->sel_start = sel_start;
  j->sel_shape = sel_shape; j->ptrs = ptrs; j->lens = lens; j->out = out; j->validate = validate;
  j->n = 1;
  for (uint32_t d = 0; d < nd; d++) {
    if (cshape[d] == 0) { free(j); return ORC_INVALID_ARGUMENT; }
    j->ngrid[d] = (ashape[d] + cshape[d] - 1) / cshape[d];
    j->lo[d] = sel_start[d] / cshape[d];
    j->hi[d] = sel_shape[d] ? (sel_start[d] + sel_shape[d] - 1) / cshape[d] + 1 : j->lo[d];
    if (j->hi[d] > j->ngrid[d] || sel_start[d] + sel_shape[d] > ashape[d]) {
      free(j);
      return ORC_INVALID_ARGUMENT;
    }
    j->n *= j->hi[d] - j->lo[d];
  }
  atomic_init(&j->next, 0);
  j->status = calloc(j->n ? j->n : 1, sizeof(int));
  if (nthreads < 1) nthreads = 1;
  /* outer x inner split of the thread budget (concurrency.rs:23-48) */
  j->inner_threads = j->n ? nthreads / (int)((uint64_t)nthreads < j->n ? (uint64_t)nthreads : j->n) : 1;
  if (j->inner_threads < 1) j->inner_threads = 1;
  if ((uint64_t)nthreads > j->n) nthreads = (int)(j->n ? j->n : 1);
  pthread_t th[256];
  if (nthreads > 256) nthreads = 256;
  for (int i = 1; i < nthreads; i++) pthread_create(&th[i], NULL, worker, j);
  worker(j);
  for (int i = 1; i < nthreads; i++) pthread_join(th[i], NULL);
  g_inner_threads = 1;
  /* deterministic "first error" (try_for_each): the lowest chunk index wins */
  int st = ORC_OK;
  for (uint64_t t = 0; t < j->n && !st; t++) st = j->status[t];
  free(j->status);
  free(j);
  return st;
}
