// C++ harness of the drop-in boundary: links libzgpu.so through include/zgpu.h only (no Python, no
// torch), the way a cgo/JNI/Rust FFI binding would. Part 1 runs anywhere (argument checks, status
// names, version, context creation failing cleanly without a GPU). Part 2 needs a HIP device: it
// decodes host-resident chunks of two chains (bytes+crc32c, and a hand-built sharding_indexed shard
// with an empty inner chunk) bit-exactly against values computed here, and checks the statuses the
// reference raises (InvalidChecksum, UnexpectedChunkDecodedSize with its lengths).
// Exit code 0 = pass; "gpu: skipped" is printed when no device exists (part 2 not run).
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../../include/zgpu.h"

static int failures = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      std::fprintf(stderr, "FAIL %s:%d: %s\n", __FILE__, __LINE__, #c); \
      failures++;                                                      \
    }                                                                  \
  } while (0)

// reflected CRC-32C (Castagnoli), the crc32c codec's checksum (crc32c_codec.rs:88-106)
static uint32_t crc32c(const uint8_t *p, size_t n) {
  uint32_t c = 0xFFFFFFFFu;
  for (size_t i = 0; i < n; i++) {
    c ^= p[i];
    for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0x82F63B78u & (0u - (c & 1u)));
  }
  return c ^ 0xFFFFFFFFu;
}

static void put_u32(std::vector<uint8_t> &v, uint32_t x) {
  for (int k = 0; k < 4; k++) v.push_back((uint8_t)(x >> (8 * k)));
}
static void put_u64(std::vector<uint8_t> &v, uint64_t x) {
  for (int k = 0; k < 8; k++) v.push_back((uint8_t)(x >> (8 * k)));
}

static zgpu_chunk_desc desc(const void *enc, uint64_t len, std::initializer_list<uint64_t> shape) {
  zgpu_chunk_desc d;
  std::memset(&d, 0, sizeof(d));
  d.enc = enc;
  d.enc_len = len;
  int i = 0;
  for (uint64_t s : shape) {
    d.chunk_shape[i] = s;
    d.sel_shape[i] = s;
    i++;
  }
  return d;
}

static void part1() {
  CHECK(std::strcmp(zgpu_status_name(ZGPU_OK), "OK") == 0);
  CHECK(std::strcmp(zgpu_status_name(ZGPU_INVALID_CHECKSUM), "INVALID_CHECKSUM") == 0);
  CHECK(std::strcmp(zgpu_status_name(ZGPU_STORAGE_ERROR), "STORAGE_ERROR") == 0);
  CHECK(std::strcmp(zgpu_status_name(999), "UNKNOWN") == 0);
  CHECK(std::strstr(zgpu_version(), "gfx950") != nullptr);
  CHECK(zgpu_ctx_create(0, nullptr) == ZGPU_INVALID_ARGUMENT);
  zgpu_ctx *c = nullptr;
  CHECK(zgpu_ctx_create(-1, &c) != ZGPU_OK && c == nullptr);
  CHECK(zgpu_chain_create(nullptr, "[]", "uint8", nullptr, 0, 1, nullptr) == ZGPU_INVALID_ARGUMENT);
  CHECK(zgpu_decode_batch(nullptr, 1, nullptr, 0, nullptr, nullptr, 0, nullptr, nullptr) == ZGPU_INVALID_ARGUMENT);
  uint64_t ctr[ZGPU_N_COUNTERS];
  CHECK(zgpu_last_counters(ctr, ZGPU_N_COUNTERS) == ZGPU_N_COUNTERS);
  CHECK(zgpu_chain_encoded_size(nullptr, 1, nullptr) == -1);
  CHECK(zgpu_decode_into(nullptr, 1, nullptr, 0, nullptr, 0, nullptr, nullptr) == ZGPU_INVALID_ARGUMENT);
  CHECK(zgpu_ctx_set_coalescing(nullptr, 1, 1, 1) == ZGPU_INVALID_ARGUMENT);
}

static void part2(zgpu_ctx *ctx) {
  // [bytes little, crc32c] uint16, three chunks of 100 elements; chunk 1 corrupted
  const char *codecs = R"([{"name":"bytes","configuration":{"endian":"little"}},{"name":"crc32c"}])";
  zgpu_chain *ch = nullptr;
  const uint16_t fill = 0;
  CHECK(zgpu_chain_create(ctx, codecs, "uint16", &fill, 2, 1, &ch) == ZGPU_OK);
  CHECK(zgpu_chain_element_size(ch) == 2);
  CHECK(zgpu_chain_encoded_size(ch, 1, std::vector<uint64_t>{100}.data()) == 204);
  std::vector<std::vector<uint8_t>> enc(3);
  for (int c = 0; c < 3; c++) {
    for (int i = 0; i < 100; i++) {
      const uint16_t v = (uint16_t)(c * 1000 + i * 7);
      enc[c].push_back((uint8_t)v);
      enc[c].push_back((uint8_t)(v >> 8));
    }
    put_u32(enc[c], crc32c(enc[c].data(), 200));
  }
  std::vector<zgpu_chunk_desc> d;
  for (int c = 0; c < 3; c++) {
    d.push_back(desc(enc[c].data(), enc[c].size(), {100}));
    d.back().out_start[0] = 100 * c;
  }
  std::vector<uint16_t> out(300, 0xFFFF);
  const uint64_t oshape[1] = {300};
  int32_t st[3] = {-1, -1, -1};
  CHECK(zgpu_decode_batch(ch, 1, d.data(), 3, out.data(), oshape, 0, st, nullptr) == ZGPU_OK);
  for (int i = 0; i < 300; i++) CHECK(out[i] == (uint16_t)((i / 100) * 1000 + (i % 100) * 7));
  enc[1][10] ^= 1;
  CHECK(zgpu_decode_batch(ch, 1, d.data(), 3, out.data(), oshape, 0, st, nullptr) == ZGPU_INVALID_CHECKSUM);
  CHECK(st[0] == 0 && st[1] == ZGPU_INVALID_CHECKSUM && st[2] == 0);
  CHECK(zgpu_decode_batch(ch, 1, d.data(), 3, out.data(), oshape, ZGPU_NO_VALIDATE, st, nullptr) == ZGPU_OK);
  // UnexpectedChunkDecodedSize(len 200, expected 202) for a chunk declared one element longer
  zgpu_chunk_desc big = desc(enc[0].data(), enc[0].size(), {101});
  const uint64_t bshape[1] = {101};
  std::vector<uint16_t> out2(101);
  CHECK(zgpu_decode_batch(ch, 1, &big, 1, out2.data(), bshape, 0, st, nullptr) == ZGPU_DECODED_SIZE_MISMATCH);
  uint64_t di = 9, len = 0, exp = 0;
  CHECK(zgpu_last_size_mismatch(&di, &len, &exp) == 1);
  CHECK(di == 0 && len == 200 && exp == 202);
  zgpu_chain_destroy(ch);

  // sharding_indexed u16 [4,4] shard of [2,2] inner chunks [bytes, crc32c], index [bytes, crc32c] at
  // the end; inner chunk 2 empty (u64::MAX pair -> fill 9), chunks stored out of order
  const char *scodecs =
      R"([{"name":"sharding_indexed","configuration":{"chunk_shape":[2,2],)"
      R"("codecs":[{"name":"bytes","configuration":{"endian":"little"}},{"name":"crc32c"}],)"
      R"("index_codecs":[{"name":"bytes","configuration":{"endian":"little"}},{"name":"crc32c"}],)"
      R"("index_location":"end"}}])";
  const uint16_t sfill = 9;
  CHECK(zgpu_chain_create(ctx, scodecs, "uint16", &sfill, 2, 1, &ch) == ZGPU_OK);
  std::vector<uint8_t> shard;
  uint64_t off[4], nb[4];
  const int order[3] = {3, 0, 1};
  for (int k : order) {
    std::vector<uint8_t> c;
    for (int e = 0; e < 4; e++) {
      const uint16_t v = (uint16_t)(100 * k + e);
      c.push_back((uint8_t)v);
      c.push_back((uint8_t)(v >> 8));
    }
    put_u32(c, crc32c(c.data(), 8));
    off[k] = shard.size();
    nb[k] = c.size();
    shard.insert(shard.end(), c.begin(), c.end());
  }
  off[2] = nb[2] = ~0ull;
  std::vector<uint8_t> idx;
  for (int k = 0; k < 4; k++) {
    put_u64(idx, off[k]);
    put_u64(idx, nb[k]);
  }
  put_u32(idx, crc32c(idx.data(), idx.size()));
  shard.insert(shard.end(), idx.begin(), idx.end());
  zgpu_chunk_desc sd = desc(shard.data(), shard.size(), {4, 4});
  const uint64_t sshape[2] = {4, 4};
  std::vector<uint16_t> so(16, 0);
  CHECK(zgpu_decode_batch(ch, 2, &sd, 1, so.data(), sshape, 0, st, nullptr) == ZGPU_OK);
  for (int y = 0; y < 4; y++)
    for (int x = 0; x < 4; x++) {
      const int k = (y / 2) * 2 + x / 2, e = (y % 2) * 2 + x % 2;
      CHECK(so[y * 4 + x] == (k == 2 ? 9 : 100 * k + e));
    }
  // a partial selection: rows 1..2, cols 1..3 (partial decoder path)
  sd.sel_start[0] = 1;
  sd.sel_start[1] = 1;
  sd.sel_shape[0] = 2;
  sd.sel_shape[1] = 3;
  const uint64_t pshape[2] = {2, 3};
  std::vector<uint16_t> po(6, 0);
  CHECK(zgpu_decode_batch(ch, 2, &sd, 1, po.data(), pshape, 0, st, nullptr) == ZGPU_OK);
  for (int y = 0; y < 2; y++)
    for (int x = 0; x < 3; x++) CHECK(po[y * 3 + x] == so[(y + 1) * 4 + x + 1]);

  // decode_into a window of a larger host array ([6,9], window at [1,2] of shape [4,4]: the
  // ArrayBytesFixedDisjointView a ShardingCodecBound::decode_into receives); bytes outside stay
  sd.sel_start[0] = sd.sel_start[1] = 0;
  sd.sel_shape[0] = sd.sel_shape[1] = 4;
  std::vector<uint16_t> big_arr(6 * 9, 7777);
  zgpu_out_view v;
  std::memset(&v, 0, sizeof v);
  v.base = big_arr.data();
  v.array_shape[0] = 6;
  v.array_shape[1] = 9;
  v.start[0] = 1;
  v.start[1] = 2;
  v.shape[0] = v.shape[1] = 4;
  CHECK(zgpu_decode_into(ch, 2, &sd, 1, &v, 0, st, nullptr) == ZGPU_OK);
  for (int y = 0; y < 6; y++)
    for (int x = 0; x < 9; x++) {
      const bool in = y >= 1 && y < 5 && x >= 2 && x < 6;
      CHECK(big_arr[y * 9 + x] == (in ? so[(y - 1) * 4 + (x - 2)] : 7777));
    }
  v.start[1] = 6;  // the window must lie inside its array
  CHECK(zgpu_decode_into(ch, 2, &sd, 1, &v, 0, st, nullptr) == ZGPU_INVALID_ARGUMENT);

  // ZGPU_COALESCE from 8 host threads, each its own window of one [8,16] array (two shards side by side
  // per row of shards): every caller gets its own status; one caller's shard has a corrupt index crc
  CHECK(zgpu_ctx_set_coalescing(ctx, 20000, 8, 0) == ZGPU_OK);
  std::vector<uint8_t> bad = shard;
  bad[bad.size() - 1] ^= 0x40;
  std::vector<uint16_t> arr(16 * 8, 0);
  int rc[8];
  std::vector<std::thread> th;
  for (int t = 0; t < 8; t++)
    th.emplace_back([&, t] {
      zgpu_chunk_desc d = desc(t == 5 ? bad.data() : shard.data(), shard.size(), {4, 4});
      zgpu_out_view w;
      std::memset(&w, 0, sizeof w);
      w.base = arr.data();
      w.array_shape[0] = 16;
      w.array_shape[1] = 8;
      w.start[0] = 4 * (t / 2);
      w.start[1] = 4 * (t % 2);
      w.shape[0] = w.shape[1] = 4;
      int32_t s1 = -1;
      rc[t] = zgpu_decode_into(ch, 2, &d, 1, &w, ZGPU_COALESCE, &s1, nullptr);
    });
  for (auto &x : th) x.join();
  uint64_t batches = 0, calls = 0;
  CHECK(zgpu_ctx_coalescing_stats(ctx, &batches, &calls) == ZGPU_OK);
  CHECK(calls >= 8 && batches < calls);
  for (int t = 0; t < 8; t++) {
    CHECK(rc[t] == (t == 5 ? ZGPU_INVALID_CHECKSUM : ZGPU_OK));
    if (t == 5) continue;
    for (int y = 0; y < 4; y++)
      for (int x = 0; x < 4; x++) CHECK(arr[(4 * (t / 2) + y) * 8 + 4 * (t % 2) + x] == so[y * 4 + x]);
  }
  zgpu_chain_destroy(ch);
}

int main() {
  part1();
  zgpu_ctx *ctx = nullptr;
  if (zgpu_ctx_create(0, &ctx) == ZGPU_OK) {
    part2(ctx);
    zgpu_ctx_destroy(ctx);
    std::printf("gpu: ran\n");
  } else {
    std::printf("gpu: skipped (%s)\n", zgpu_last_error(nullptr));
  }
  std::printf("%s (%d failures)\n", failures ? "FAIL" : "PASS", failures);
  return failures ? 1 : 0;
}
