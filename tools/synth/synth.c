/*
 * synth.c — synthetic workload WRITER for bench.py's C3/C5 configurations.
 *
 * Not product code and not the oracle: it produces encoded Zarr chunks/shards the way zarrs'
 * encode path lays them out, so the GPU decoder has realistic inputs, and it regenerates the
 * decoded values so bench.py can check decode(encode(x)) == x on the device without any CPU
 * decoder. Layouts written (zarrs workspace paths):
 *   sharding_indexed  inner chunks back to back in C order of the inner grid, then the index
 *                     [cps..., 2] u64 LE (offset, nbytes) + its crc32c (index_location end)
 *                     (zarrs/src/array/codec/array_to_bytes/sharding/sharding_codec.rs:924-1261,
 *                     sharding.rs:156-235)
 *   crc32c            4-byte LE Castagnoli checksum appended (crc32c_codec.rs:90-100)
 *   gzip              RFC 1952 member (zlib deflate, wbits 31) (gzip_codec.rs:90-108)
 *   zstd              one frame from ZSTD_compress2, checksum flag as configured (zstd_codec.rs:95-111)
 *   numcodecs.shuffle enc[i*count + j] = dec[j*es + i] (shuffle_codec.rs:86-107)
 * Threads: pthreads over independent chunks.
 */
#define _GNU_SOURCE
#include <math.h>
#include <nmmintrin.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <zlib.h>

/* libzstd.so.1 public ABI (the image ships the library without its header) */
typedef struct ZSTD_CCtx_s ZSTD_CCtx;
extern unsigned ZSTD_isError(size_t code);
extern ZSTD_CCtx *ZSTD_createCCtx(void);
extern size_t ZSTD_freeCCtx(ZSTD_CCtx *);
extern size_t ZSTD_CCtx_setParameter(ZSTD_CCtx *, int param, int value);
extern size_t ZSTD_compress2(ZSTD_CCtx *, void *dst, size_t cap, const void *src, size_t n);
extern size_t ZSTD_compressBound(size_t srcSize);
#define ZSTD_c_compressionLevel 100
#define ZSTD_c_checksumFlag 201

uint32_t synth_crc32c(const uint8_t *p, uint64_t n) {
  uint64_t c = 0xFFFFFFFFu;
  while (n >= 8) {
    uint64_t w;
    memcpy(&w, p, 8);
    c = _mm_crc32_u64(c, w);
    p += 8;
    n -= 8;
  }
  uint32_t c32 = (uint32_t)c;
  while (n--) c32 = _mm_crc32_u8(c32, *p++);
  return c32 ^ 0xFFFFFFFFu;
}

static uint64_t gzip_member(const uint8_t *src, uint64_t n, int level, uint8_t *dst, uint64_t cap) {
  z_stream s;
  memset(&s, 0, sizeof(s));
  if (deflateInit2(&s, level, Z_DEFLATED, 31, 8, Z_DEFAULT_STRATEGY) != Z_OK) return 0;
  s.next_in = (Bytef *)src;
  s.avail_in = (uInt)n;
  s.next_out = dst;
  s.avail_out = (uInt)cap;
  int r = deflate(&s, Z_FINISH);
  uint64_t out = s.total_out;
  deflateEnd(&s);
  return r == Z_STREAM_END ? out : 0;
}

/* ---------------------------------------------------------------------------------------------
 * Values
 * ------------------------------------------------------------------------------------------- */
static inline uint64_t mix64(uint64_t x) {
  x ^= x >> 30;
  x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27;
  x *= 0x94d049bb133111ebull;
  x ^= x >> 31;
  return x;
}
/* approximately N(0,1) from a hash (sum of 4 uniforms, rescaled): deterministic per voxel */
static inline float hnorm(uint64_t key) {
  uint64_t h = mix64(key);
  float s = (float)(h & 0xFFFF) + (float)((h >> 16) & 0xFFFF) + (float)((h >> 32) & 0xFFFF) +
            (float)(h >> 48);
  return (s / 65535.0f - 2.0f) * 1.7320508f;
}

/* C3: round(256*(sin(0.05x)+cos(0.03y)+0.5 sin(0.07z)) + N(0,1)) / 256 at array coords (x,y,z) */
static inline float c3_value(uint64_t x, uint64_t y, uint64_t z) {
  const float s = sinf(0.05f * (float)x) + cosf(0.03f * (float)y) + 0.5f * sinf(0.07f * (float)z);
  const uint64_t key = (x * 2048ull + y) * 2048ull + z + 7ull * 0x9E3779B97F4A7C15ull;
  return rintf(256.0f * s + hnorm(key)) / 256.0f;
}

typedef struct {
  const uint64_t *origin, *shape, *full;  /* region origin, region shape, region strides base */
  float *out;
  int t, nt;
} c3_job;

static void *c3_fill_worker(void *arg) {
  c3_job *J = (c3_job *)arg;
  for (uint64_t i = J->t; i < J->shape[0]; i += J->nt)
    for (uint64_t j = 0; j < J->shape[1]; j++) {
      float *row = J->out + (i * J->shape[1] + j) * J->shape[2];
      for (uint64_t k = 0; k < J->shape[2]; k++)
        row[k] = c3_value(J->origin[0] + i, J->origin[1] + j, J->origin[2] + k);
    }
  return NULL;
}

/* Fill out[shape] (C order, f32) with the C3 values of the region at `origin`. */
void synth_c3_values(const uint64_t *origin, const uint64_t *shape, float *out, int nthreads) {
  pthread_t th[256];
  c3_job jobs[256];
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (c3_job){origin, shape, shape, out, t, nthreads};
    pthread_create(&th[t], NULL, c3_fill_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

/* ---------------------------------------------------------------------------------------------
 * Sharded shard writer: [bytes little, gzip level, crc32c] inner chunks, [bytes little, crc32c]
 * index at the end. The decoded shard is `dec` (C order, shard_shape, f32 / element size es).
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  const uint8_t *dec;
  const uint64_t *ss, *is;
  uint64_t cps[3], n_inner, inner_bytes, es;
  int level;
  uint8_t **bufs;
  uint64_t *lens;
  int t, nt;
  int err;
} shard_job;

static void *shard_worker(void *arg) {
  shard_job *J = (shard_job *)arg;
  uint8_t *tmp = (uint8_t *)malloc(J->inner_bytes);
  const uint64_t cap = J->inner_bytes + J->inner_bytes / 8 + 1024;
  for (uint64_t c = J->t; c < J->n_inner; c += J->nt) {
    const uint64_t ci = c / (J->cps[1] * J->cps[2]), cj = (c / J->cps[2]) % J->cps[1], ck = c % J->cps[2];
    /* gather the inner chunk (C order) */
    uint8_t *w = tmp;
    for (uint64_t i = 0; i < J->is[0]; i++)
      for (uint64_t j = 0; j < J->is[1]; j++) {
        const uint64_t off = (((ci * J->is[0] + i) * J->ss[1] + cj * J->is[1] + j) * J->ss[2] + ck * J->is[2]) * J->es;
        memcpy(w, J->dec + off, J->is[2] * J->es);
        w += J->is[2] * J->es;
      }
    uint8_t *b = (uint8_t *)malloc(cap + 4);
    const uint64_t n = gzip_member(tmp, J->inner_bytes, J->level, b, cap);
    if (!n) J->err = 1;
    const uint32_t crc = synth_crc32c(b, n);
    memcpy(b + n, &crc, 4);
    J->bufs[c] = b;
    J->lens[c] = n + 4;
  }
  free(tmp);
  return NULL;
}

/* Returns a malloc'd shard (free with synth_free) and its length; 0 on success. */
int synth_gzip_crc_shard(const void *dec, uint64_t es, const uint64_t *shard_shape, const uint64_t *inner_shape,
                         int level, int nthreads, uint8_t **out, uint64_t *out_len) {
  shard_job base;
  memset(&base, 0, sizeof(base));
  base.dec = (const uint8_t *)dec;
  base.ss = shard_shape;
  base.is = inner_shape;
  base.es = es;
  base.level = level;
  base.n_inner = 1;
  for (int d = 0; d < 3; d++) {
    base.cps[d] = shard_shape[d] / inner_shape[d];
    base.n_inner *= base.cps[d];
  }
  base.inner_bytes = inner_shape[0] * inner_shape[1] * inner_shape[2] * es;
  base.bufs = (uint8_t **)calloc(base.n_inner, sizeof(uint8_t *));
  base.lens = (uint64_t *)calloc(base.n_inner, sizeof(uint64_t));
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  shard_job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = base;
    jobs[t].t = t;
    jobs[t].nt = nthreads;
    pthread_create(&th[t], NULL, shard_worker, &jobs[t]);
  }
  int err = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    err |= jobs[t].err;
  }
  uint64_t total = 0;
  for (uint64_t c = 0; c < base.n_inner; c++) total += base.lens[c];
  const uint64_t index_bytes = base.n_inner * 16;
  uint8_t *s = (uint8_t *)malloc(total + index_bytes + 4);
  uint64_t *index = (uint64_t *)(s + total);
  uint64_t off = 0;
  for (uint64_t c = 0; c < base.n_inner; c++) {
    memcpy(s + off, base.bufs[c], base.lens[c]);
    index[2 * c] = off; /* little-endian host */
    index[2 * c + 1] = base.lens[c];
    off += base.lens[c];
    free(base.bufs[c]);
  }
  const uint32_t icrc = synth_crc32c((const uint8_t *)index, index_bytes);
  memcpy(s + total + index_bytes, &icrc, 4);
  free(base.bufs);
  free(base.lens);
  *out = s;
  *out_len = total + index_bytes + 4;
  return err;
}

/* ---------------------------------------------------------------------------------------------
 * C5: [bytes little, numcodecs.shuffle{es}, zstd{level, checksum}] chunks, many in parallel.
 * chunk c's decoded bytes are dec + offs[c], length lens[c]; outputs malloc'd per chunk.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  const uint8_t *dec;
  const uint64_t *offs, *lens;
  uint64_t n, es;
  int level, checksum;
  uint8_t **outs;
  uint64_t *out_lens;
  int t, nt, err;
} zjob;

static void *zworker(void *arg) {
  zjob *J = (zjob *)arg;
  ZSTD_CCtx *cc = ZSTD_createCCtx();
  ZSTD_CCtx_setParameter(cc, ZSTD_c_compressionLevel, J->level);
  ZSTD_CCtx_setParameter(cc, ZSTD_c_checksumFlag, J->checksum);
  for (uint64_t c = J->t; c < J->n; c += J->nt) {
    const uint8_t *src = J->dec + J->offs[c];
    const uint64_t n = J->lens[c], count = n / J->es;
    uint8_t *sh = (uint8_t *)malloc(n ? n : 1);
    for (uint64_t i = 0; i < J->es; i++)
      for (uint64_t j = 0; j < count; j++) sh[i * count + j] = src[j * J->es + i];
    const size_t cap = ZSTD_compressBound(n);
    uint8_t *b = (uint8_t *)malloc(cap);
    size_t r = ZSTD_compress2(cc, b, cap, sh, n);
    if (ZSTD_isError(r)) {
      J->err = 1;
      r = 0;
    }
    free(sh);
    J->outs[c] = b;
    J->out_lens[c] = r;
  }
  ZSTD_freeCCtx(cc);
  return NULL;
}

int synth_shuffle_zstd_chunks(const void *dec, uint64_t es, const uint64_t *offs, const uint64_t *lens, uint64_t n,
                              int level, int checksum, int nthreads, uint8_t **outs, uint64_t *out_lens) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  zjob jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (zjob){(const uint8_t *)dec, offs, lens, n, es, level, checksum, outs, out_lens, t, nthreads, 0};
    pthread_create(&th[t], NULL, zworker, &jobs[t]);
  }
  int err = 0;
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    err |= jobs[t].err;
  }
  return err;
}

void synth_free(void *p) { free(p); }

/* ---------------------------------------------------------------------------------------------
 * C5: OME-Zarr-style uint16 level 0: background 100 + K Gaussian blobs (amplitude <= 4000) +
 * noise ~ sqrt(mean) * N(0,1) (Poisson approximation), clipped to u16. Blobs are separable
 * (gx[x] * gy[y] * gz[z]) and evaluated only inside their 4-sigma boxes.
 * ------------------------------------------------------------------------------------------- */
typedef struct {
  uint64_t nz, ny, nx;
  int nblobs;
  const float *cz, *cy, *cx, *sg, *amp;
  uint16_t *out;
  int t, nt;
  uint64_t seed;
} c5_job;

static void *c5_worker(void *arg) {
  c5_job *J = (c5_job *)arg;
  float *acc = (float *)malloc(J->nx * sizeof(float));
  float *gy = (float *)malloc(J->nblobs * sizeof(float));
  for (uint64_t z = J->t; z < J->nz; z += J->nt) {
    for (uint64_t y = 0; y < J->ny; y++) {
      for (uint64_t x = 0; x < J->nx; x++) acc[x] = 100.0f;
      for (int b = 0; b < J->nblobs; b++) {
        const float s = J->sg[b], dz = (float)z - J->cz[b], dy = (float)y - J->cy[b];
        if (fabsf(dz) > 4 * s || fabsf(dy) > 4 * s) continue;
        const float gzy = J->amp[b] * expf(-(dz * dz + dy * dy) / (2 * s * s));
        long x0 = (long)(J->cx[b] - 4 * s), x1 = (long)(J->cx[b] + 4 * s) + 1;
        if (x0 < 0) x0 = 0;
        if (x1 > (long)J->nx) x1 = (long)J->nx;
        for (long x = x0; x < x1; x++) {
          const float dx = (float)x - J->cx[b];
          acc[x] += gzy * expf(-dx * dx / (2 * s * s));
        }
      }
      uint16_t *row = J->out + (z * J->ny + y) * J->nx;
      for (uint64_t x = 0; x < J->nx; x++) {
        const float m = acc[x];
        float v = m + sqrtf(m) * hnorm(((z * J->ny + y) * J->nx + x) ^ J->seed);
        v = rintf(v);
        if (v < 0) v = 0;
        if (v > 65535.0f) v = 65535.0f;
        row[x] = (uint16_t)v;
      }
    }
  }
  free(acc);
  free(gy);
  return NULL;
}

/* blobs: nblobs entries of (cz, cy, cx, sigma, amplitude) each */
void synth_c5_level0(uint64_t nz, uint64_t ny, uint64_t nx, int nblobs, const float *cz, const float *cy,
                     const float *cx, const float *sg, const float *amp, uint64_t seed, uint16_t *out,
                     int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  pthread_t th[256];
  c5_job jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (c5_job){nz, ny, nx, nblobs, cz, cy, cx, sg, amp, out, t, nthreads, seed};
    pthread_create(&th[t], NULL, c5_worker, &jobs[t]);
  }
  for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
}

// The drop-in emulation's stand-in for zarrs' CPU shuffle codec (bench.py C5 dropin_leg): the loop of
// zarrs/src/array/codec/bytes_to_bytes/shuffle/shuffle_codec.rs:109-129 compiled natively, as zarrs'
// Rust loop is (numpy's strided column copies are several times slower than either).
void synth_unshuffle(const uint8_t *enc, uint8_t *dec, uint64_t n, uint64_t es) {
  const uint64_t count = n / es;
  if (es == 2) {
    const uint8_t *lo = enc, *hi = enc + count;
    for (uint64_t j = 0; j < count; j++) {
      dec[2 * j] = lo[j];
      dec[2 * j + 1] = hi[j];
    }
    return;
  }
  for (uint64_t i = 0; i < es; i++)
    for (uint64_t j = 0; j < count; j++) dec[j * es + i] = enc[i * count + j];
}
