// libzgpu: host orchestration of the MI355X chunk-decode pipeline behind the C ABI of include/zgpu.h.
//
// A batch of chunk descriptors is planned on the host into leaf work items (a plain chunk, or one
// inner chunk of a shard that intersects the selection), uploaded once, and decoded by a short
// sequence of batched kernels, each over ALL items of the batch:
//   [sharded]  k_shard_index (index chain decode + crc32c verify per shard)
//              k_item_resolve (index lookup per item: byte range, empty -> fill, out-of-bounds)
//   b2b stages in reverse metadata order (codec_chain.rs:612-617):
//              crc32c verify+strip (pointer arithmetic, no copy) | gzip | zstd | unshuffle
//   final      fused bytes(endian) + transpose + (innermost shuffle) + scatter/fill into the output
// Per-item statuses come back in one D2H copy; the first failing item of a descriptor gives that
// descriptor's status (try_for_each semantics, sharding_codec.rs:702-704).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <condition_variable>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/zgpu.h"
#include "chain.hpp"
#include "common.hpp"
#include "kernels/launch.hpp"
#include "fsstore.hpp"
#include "internal.hpp"
#include "xfer.hpp"

using namespace zgpu;

namespace {

thread_local std::string g_last_error;
// device counters in the plan's control block (u64 each, cleared per execute)
enum { CTR_ENC_BYTES = 0, CTR_ZSTD_SERIAL = 1, CTR_ZSTD_PARALLEL = 2, CTR_BLOSC_RERUN = 3, CTR_BLOSC_BLOCKS = 4,
       CTR_ITEMS = 5, CTR_N = 6 };  // CTR_ITEMS is host-side (the plan's leaf items)
// internal ctl slots (not reported): a cached blosc layout was outgrown (the execution is re-run)
enum { CTR_BLOSC_OVF = 31, CTR_SCRATCH = 30, CTR_ZSTD_NSER = 29, CTR_ZSTD_MAXBLK = 28 };  // not reported (device-side flags / sinks)
thread_local uint64_t g_last_counters[CTR_N];
// UnexpectedChunkDecodedSize detail of the last call's first DECODED_SIZE_MISMATCH descriptor
struct SizeDetail {
  int valid = 0;
  uint64_t desc = 0, len = 0, expected = 0;
};
thread_local SizeDetail g_size_detail;

struct HipFail {
  hipError_t e;
  const char *what;
};
#define HIPCHK(x)                                   \
  do {                                              \
    hipError_t _e = (x);                            \
    if (_e != hipSuccess) throw HipFail{_e, #x};    \
  } while (0)

}  // namespace

// ------------------------------------------------------------------------------------------------
// Context: one per GPU. Owns a caching device allocator (grow-only pools reused across calls so a
// steady-state decode performs no hipMalloc) and a small pool of "lanes" (a stream, two copy streams
// and an ordering event): concurrent calls on one context each take a lane and run side by side on
// the GPU (zarrs calls a codec from many rayon workers at once); a call that finds every lane busy
// waits for one. ZGPU_CTX_LANES sets the pool size (default 8: coalesced drop-in calls measured
// 10.7 -> 11.6 GiB/s going from 4 to 8, profiles/r04o_dropin_lanes_ab.txt).
// ------------------------------------------------------------------------------------------------
struct Coalescer;
static void delete_coalescer(Coalescer *co);

struct Lane {
  hipStream_t stream = nullptr;              // the call's stream when the caller passes none
  hipStream_t copy[2] = {nullptr, nullptr};  // H2D / D2H streams of the pipelined host paths (lazy)
  hipStream_t out_hi = nullptr;               // high-priority stream of a coalesced batch's pack + D2H (lazy)
  hipEvent_t order_ev = nullptr;              // legacy-stream -> lane-stream ordering (pick_stream)
};

// A lane's stream. HIP maps streams onto GPU_MAX_HW_QUEUES hardware queues (4 by default), and
// kernels of different streams sharing a queue run one after the other: 8 lanes (plus their pack
// streams) on 4 queues serialised the drop-in's concurrent calls. A stream with a CU mask gets a
// hardware queue of its own; with every CU in the mask (ZGPU_LANE_QUEUES=1) it is an ordinary stream
// otherwise. HIP creates CU-masked streams as blocking streams (ordered against the legacy null stream,
// unlike the non-blocking lanes they replace), and has no flags argument for them: with
// ZGPU_LANE_QUEUES=1, work a caller queues on the null stream serialises with the lanes.
static hipError_t lane_stream_create(hipStream_t *s, int device) {
  static const bool own = [] {
    const char *e = std::getenv("ZGPU_LANE_QUEUES");
    return e && std::atoi(e) != 0;
  }();
  if (own) {
    int ncu = 0;
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && ncu > 0) {
      std::vector<uint32_t> mask((ncu + 31) / 32, ~0u);
      if (ncu % 32) mask.back() = (1u << (ncu % 32)) - 1;
      const hipError_t e = hipExtStreamCreateWithCUMask(s, (uint32_t)mask.size(), mask.data());
      if (e == hipSuccess) return e;
      (void)hipGetLastError();
    }
  }
  return hipStreamCreateWithFlags(s, hipStreamNonBlocking);
}

struct zgpu_ctx {
  int device = 0;
  // Lifetime: zgpu_ctx_destroy drops the caller's reference; every chain, plan and cache created on
  // the context holds one more, so a context outlives the objects that use it in whatever order a
  // garbage-collected binding destroys them. The last reference frees the context (no HIP call runs
  // from a static destructor: the library has none).
  std::atomic<int64_t> refs{1};
  std::mutex mu;  // the allocator pools
  std::multimap<size_t, void *> free_dev;  // size -> ptr
  std::map<void *, size_t> live_dev;
  std::multimap<size_t, void *> free_host;
  std::map<void *, size_t> live_host;
  // lanes
  std::mutex lane_mu;
  std::condition_variable lane_cv;
  std::vector<Lane *> lanes_all, lanes_free;
  uint32_t max_lanes = 8;
  hipStream_t peer = nullptr;  // peer copies of the multi-device read (lazy)
  struct Coalescer *co = nullptr;  // ZGPU_COALESCE batching (lazy, under mu)

  Lane *acquire_lane() {
    std::unique_lock<std::mutex> lk(lane_mu);
    while (lanes_free.empty()) {
      if (lanes_all.size() < max_lanes) {
        auto L = std::make_unique<Lane>();
        HIPCHK(hipSetDevice(device));
        HIPCHK(lane_stream_create(&L->stream, device));
        lanes_all.push_back(L.get());
        lanes_free.push_back(L.release());
        break;
      }
      lane_cv.wait(lk);
    }
    Lane *L = lanes_free.back();
    lanes_free.pop_back();
    return L;
  }
  void release_lane(Lane *L) {
    {
      std::lock_guard<std::mutex> lk(lane_mu);
      lanes_free.push_back(L);
    }
    lane_cv.notify_one();
  }

  // Device pool: sizes rounded up to classes (1/8 of a power of two above 1 MiB: <= 12.5 % slack) so
  // that buffers of batches of varying size are reused instead of accumulating; the free blocks are
  // capped (ZGPU_POOL_CAP_MB, default 16 GiB: the largest are returned to HIP beyond it). Without the
  // cap, thousands of concurrent per-chunk calls (the codec plugin's pattern) of varying batch sizes
  // grew the pool until the device had no memory left for a kernel's scratch.
  size_t free_dev_bytes = 0;
  size_t pool_cap = (size_t)16 << 30;
  static size_t size_class(size_t b) {
    b = std::max<size_t>(256, (b + 255) & ~(size_t)255);
    if (b <= (1u << 20)) return b;
    size_t p = (size_t)1 << (63 - __builtin_clzll(b - 1));  // largest power of two < b
    const size_t step = p / 8;
    return (b + step - 1) / step * step;
  }
  void trim_free_locked(size_t keep) {
    while (free_dev_bytes > keep && !free_dev.empty()) {
      auto it = std::prev(free_dev.end());  // the largest free block
      (void)hipFree(it->second);
      free_dev_bytes -= it->first;
      free_dev.erase(it);
    }
  }
  void *dev_alloc(size_t bytes) {
    std::lock_guard<std::mutex> lk(mu);
    bytes = size_class(bytes);
    auto it = free_dev.lower_bound(bytes);
    if (it != free_dev.end() && it->first <= bytes + bytes / 4 + (1u << 20)) {
      void *p = it->second;
      live_dev[p] = it->first;
      free_dev_bytes -= it->first;
      free_dev.erase(it);
      return p;
    }
    void *p = nullptr;
    hipError_t e = hipMalloc(&p, bytes);
    if (e != hipSuccess) {  // release the cache and retry once
      (void)hipGetLastError();
      trim_free_locked(0);
      HIPCHK(hipMalloc(&p, bytes));
    }
    live_dev[p] = bytes;
    return p;
  }
  void dev_free(void *p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu);
    auto it = live_dev.find(p);
    if (it == live_dev.end()) return;
    free_dev.emplace(it->second, p);
    free_dev_bytes += it->second;
    live_dev.erase(it);
    if (free_dev_bytes > pool_cap) trim_free_locked(pool_cap / 2);
  }
  // Pinned host pool: the same size classes, free blocks capped at ZGPU_PINNED_CAP_MB (default 4 GiB;
  // the largest go back to HIP beyond it) -- per-chunk pinned results of varying size otherwise
  // accumulate a free block per distinct size
  size_t free_host_bytes = 0;
  size_t host_cap = (size_t)4 << 30;
  void trim_host_locked(size_t keep) {
    while (free_host_bytes > keep && !free_host.empty()) {
      auto it = std::prev(free_host.end());
      (void)hipHostFree(it->second);
      free_host_bytes -= it->first;
      free_host.erase(it);
    }
  }
  void *host_alloc(size_t bytes) {
    std::lock_guard<std::mutex> lk(mu);
    bytes = std::max<size_t>(4096, size_class((bytes + 4095) & ~(size_t)4095));
    auto it = free_host.lower_bound(bytes);
    if (it != free_host.end() && it->first <= bytes + bytes / 4 + (1u << 20)) {
      void *p = it->second;
      live_host[p] = it->first;
      free_host_bytes -= it->first;
      free_host.erase(it);
      return p;
    }
    void *p = nullptr;
    if (hipHostMalloc(&p, bytes, hipHostMallocDefault) != hipSuccess) {  // release the cache and retry once
      (void)hipGetLastError();
      trim_host_locked(0);
      HIPCHK(hipHostMalloc(&p, bytes, hipHostMallocDefault));
    }
    live_host[p] = bytes;
    return p;
  }
  void host_free(void *p) {
    if (!p) return;
    std::lock_guard<std::mutex> lk(mu);
    auto it = live_host.find(p);
    if (it == live_host.end()) return;
    free_host.emplace(it->second, p);
    free_host_bytes += it->second;
    live_host.erase(it);
    if (free_host_bytes > host_cap) trim_host_locked(host_cap / 2);
  }
  ~zgpu_ctx() {
    (void)hipSetDevice(device);
    for (Lane *L : lanes_all) {
      if (L->stream) (void)hipStreamSynchronize(L->stream);
      if (L->out_hi) (void)hipStreamSynchronize(L->out_hi);
    }
    for (auto &kv : free_dev) (void)hipFree(kv.second);
    for (auto &kv : live_dev) (void)hipFree(kv.first);
    for (auto &kv : free_host) (void)hipHostFree(kv.second);
    for (auto &kv : live_host) (void)hipHostFree(kv.first);
    for (Lane *L : lanes_all) {
      if (L->stream) (void)hipStreamDestroy(L->stream);
      if (L->order_ev) (void)hipEventDestroy(L->order_ev);
      if (L->out_hi) (void)hipStreamDestroy(L->out_hi);
      for (hipStream_t cs : L->copy)
        if (cs) (void)hipStreamDestroy(cs);
      delete L;
    }
    if (peer) (void)hipStreamDestroy(peer);
    delete_coalescer(co);
    (void)hipGetLastError();  // teardown failures must not surface in the caller's next HIP error check
  }
};

void zgpu::ctx_ref(zgpu_ctx *c) {
  if (c) c->refs.fetch_add(1, std::memory_order_relaxed);
}
void zgpu::ctx_unref(zgpu_ctx *c) {
  if (c && c->refs.fetch_sub(1, std::memory_order_acq_rel) == 1) delete c;
}

// A call's lane for its whole duration (RAII).
struct LaneScope {
  zgpu_ctx *C;
  Lane *L;
  explicit LaneScope(zgpu_ctx *c) : C(c), L(c->acquire_lane()) {}
  ~LaneScope() { C->release_lane(L); }
  LaneScope(const LaneScope &) = delete;
  LaneScope &operator=(const LaneScope &) = delete;
};

struct zgpu_chain {
  zgpu_ctx *ctx;
  std::shared_ptr<Chain> chain;
  bool validate;
};

// ------------------------------------------------------------------------------------------------
// Plan
// ------------------------------------------------------------------------------------------------
enum StageKind { ST_CRC32C, ST_GZIP, ST_ZSTD, ST_UNSHUFFLE, ST_BLOSC };
struct Stage {
  StageKind kind;
  int at_start = 0;
  uint32_t elementsize = 0;
  int pool = 0;  // destination slot pool for materialising stages
};

struct zgpu_plan {
  zgpu_ctx *ctx = nullptr;
  std::mutex mu;  // one execute / status at a time per plan
  Lane own{};     // the plan's stream for executes without a caller stream (lazy)
  std::shared_ptr<Chain> chain;
  const Chain *leaf = nullptr;
  bool validate = true;
  uint32_t nd = 0;
  uint64_t n_desc = 0;
  uint32_t flags = 0;
  std::vector<uint64_t> out_shape;
  // host tables
  std::vector<ZgItem> items;
  std::vector<uint64_t> geom;
  std::vector<uint32_t> item_desc_status;  // plan-time per-desc status
  std::vector<ZgShard> shards;
  std::vector<Stage> stages;
  ZgScatter scatter{};
  uint32_t scatter_mode = SCATTER_GENERIC;
  uint64_t scatter_units = 0;
  bool sharded = false, nested = false;
  ZgIndexSpec ispec{}, ispec2{};  // ispec2: the middle shards' index (nested sharding)
  std::vector<ZgItem> mids;       // nested: one record per intersecting middle shard
  uint64_t slot_bytes = 0;
  int n_pools = 0;
  uint64_t alg_bytes_static = 0;  // decoded bytes written + (unsharded) encoded bytes + index bytes
  // device buffers
  ZgItem *d_items = nullptr, *d_items_init = nullptr;
  uint64_t *d_geom = nullptr;
  uint32_t *d_status = nullptr;
  ZgShard *d_shards = nullptr;
  uint64_t *d_index = nullptr;
  uint32_t *d_shard_status = nullptr;
  // nested sharding: middle shard records (resolved through the outer index each execution), their
  // status, the middle shards as a shard table, and their decoded indexes
  ZgItem *d_mids = nullptr, *d_mids_init = nullptr;
  uint32_t *d_mid_status = nullptr, *d_shard_status2 = nullptr;
  ZgShard *d_mid_shards = nullptr;
  uint64_t *d_index2 = nullptr;
  uint8_t *d_pool[2] = {nullptr, nullptr};
  ZstdScratch zs{};  // block-parallel zstd scratch (allocated when the chain has zstd)
  // side stream of the zstd sequence decoder (created on first use with the priority of the stream
  // the plan first runs on; ZGPU_ZSTD_FORK=0 keeps one stream)
  hipStream_t zside = nullptr;
  hipEvent_t zev[2] = {nullptr, nullptr};
  void zstd_fork(ZstdScratch &Z, hipStream_t s) {
    static const bool on = [] {
      const char *e = std::getenv("ZGPU_ZSTD_FORK");
      return !e || std::atoi(e) != 0;
    }();
    if (!on || (flags & ZGPU_ONE_STREAM)) return;
    if (!zside) {
      int prio = 0;
      if (s) (void)hipStreamGetPriority(s, &prio);
      HIPCHK(hipStreamCreateWithPriority(&zside, hipStreamNonBlocking, prio));
      for (hipEvent_t &e : zev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    Z.side = zside;
    Z.ev_fork = zev[0];
    Z.ev_join = zev[1];
  }
  // zstd in two pipelined halves (ZstdScratch::s2; blosc stream tables of many frames): opt-in with
  // ZGPU_ZSTD_SPLIT=1 (blosc-zstd bench 32.6 -> 35.6 ms with it: the halves' kernels contend more than
  // they overlap, profiles/r04an_zstd_split_ab.txt)
  hipStream_t zs2 = nullptr;
  hipEvent_t zev2[2] = {nullptr, nullptr};
  void zstd_split(ZstdScratch &Z, hipStream_t s) {
    const char *e = std::getenv("ZGPU_ZSTD_SPLIT");  // read per call (tests switch it)
    if (!e || std::atoi(e) == 0 || !Z.side) return;
    if (!zs2) {
      int prio = 0;
      if (s) (void)hipStreamGetPriority(s, &prio);
      HIPCHK(hipStreamCreateWithPriority(&zs2, hipStreamNonBlocking, prio));
      for (hipEvent_t &e : zev2) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    }
    Z.s2 = zs2;
    Z.ev_half = zev2[0];
    Z.ev_done = zev2[1];
  }
  // blosc stage scratch (grown on demand; the stream table is sized from the frame headers)
  struct Grow {
    void *p = nullptr;
    size_t n = 0;
  };
  Grow bl_info, bl_bases, bl_subs, bl_sub_status, bl_sub_kind, bl_blocks, bl_tmp, bl_zblks, bl_znblk, bl_zmode,
      bl_zlit, bl_zseq, bl_zaux, bl_zser, bl_lzl, bl_zseg, bl_zrec, bl_zalias, bl_znorm, gz_crc, live_list;
  uint8_t *bl_h = nullptr;  // pinned: BlInfo read-back (first execution)
  size_t bl_h_n = 0;
  void *grow(Grow &g, size_t bytes) {
    if (g.n < bytes) {
      ctx->dev_free(g.p);
      g.p = ctx->dev_alloc(bytes);
      g.n = bytes;
    }
    return g.p;
  }
  unsigned long long *d_counter = nullptr;
  // control block: [counter (256 B) | per-item status (4 B each)], cleared by ONE memset and read
  // back by ONE D2H copy into pinned memory (h_ctl) per execute
  uint8_t *d_ctl = nullptr, *h_ctl = nullptr;
  size_t ctl_bytes = 0;
  // host-input staging
  uint8_t *d_enc_stage = nullptr;
  uint64_t last_enc_bytes = 0;
  uint64_t last_counters[CTR_N] = {};
  uint8_t *last_out = nullptr;  // output of the last enqueue (a blosc layout overflow re-runs into it)
  BlCaps bl_caps{};             // blosc stream-table capacities recorded by the first execution
  bool bl_caps_valid = false, bl_caps_seen = false;
  bool bl_direct = false;  // the blosc stage may write whole chunks straight into the output (BlDecode::dout)
  bool gz_direct = false;  // the gzip stage may write whole chunks straight into the output (GzDirect)
  GzDirect gz{};
  // blosc as the last stage: per item the decoded byte range its selection needs ([0, max) for whole
  // chunks); blocks outside it are not decoded (blosc_decompress_bytes_partial)
  std::vector<uint64_t> bl_need;
  uint64_t *d_bl_need = nullptr;
  // zstd serial fallback: skipped once an execution of this plan had no serial item (a later one that
  // has some is re-run by plan_statuses with the fallback launched)
  bool zstd_serial_off = false, zstd_serial_skipped = false;
  uint32_t *d_zser = nullptr;
  uint32_t *d_order = nullptr;  // gzip stage: LPT dispatch order of the items
  uint32_t *d_gz_seg = nullptr;  // gzip stage: symbol-record scratch of the segmented decode
  bool no_scatter = false;  // a whole-shard predecode plan: its bytes->bytes stages only (decode_general)

  ~zgpu_plan() {
    if (!ctx) return;
    struct Unref {
      zgpu_ctx *c;
      ~Unref() { ctx_unref(c); }
    } unref{ctx};  // after every buffer below went back to the context's pools
    if (own.stream) {
      (void)hipStreamSynchronize(own.stream);
      (void)hipStreamDestroy(own.stream);
    }
    if (own.order_ev) (void)hipEventDestroy(own.order_ev);
    void *bufs[] = {d_items, d_items_init, d_geom, d_shards, d_index, d_shard_status, d_mids, d_mids_init,
                    d_mid_status, d_shard_status2, d_mid_shards, d_index2, d_bl_need,
                    d_pool[0], d_pool[1], zs.blks, zs.nblk, zs.mode, zs.lit, zs.seq, d_ctl,
                    d_enc_stage, d_zser, d_order, d_gz_seg, zs.lit_rec, zs.ext, zs.ext_cnt, zs.norm};
    for (void *b : bufs) ctx->dev_free(b);
    if (zside) {
      (void)hipStreamSynchronize(zside);
      (void)hipStreamDestroy(zside);
    }
    if (zs2) {
      (void)hipStreamSynchronize(zs2);
      (void)hipStreamDestroy(zs2);
    }
    for (hipEvent_t e : zev2)
      if (e) (void)hipEventDestroy(e);
    for (hipEvent_t e : zev)
      if (e) (void)hipEventDestroy(e);
    for (Grow *g : {&bl_info, &bl_bases, &bl_subs, &bl_sub_status, &bl_sub_kind, &bl_blocks, &bl_tmp, &bl_zblks,
                    &bl_znblk, &bl_zmode, &bl_zlit, &bl_zseq, &bl_zaux, &bl_zser, &bl_lzl, &bl_zseg, &bl_zrec, &bl_zalias,
                    &bl_znorm, &gz_crc, &live_list})
      ctx->dev_free(g->p);
    ctx->host_free(bl_h);
    ctx->host_free(h_ctl);
  }
};

static void reset_call_state() {
  for (uint64_t &c : g_last_counters) c = 0;
  g_size_detail = SizeDetail{};
}

static int set_err(int st, const std::string &m) {
  g_last_error = m;
  return st;
}

int zgpu::set_last_error(int status, const std::string &msg) { return set_err(status, msg); }
zgpu_ctx *zgpu::chain_ctx(const zgpu_chain *c) { return c->ctx; }
const Chain &zgpu::chain_model(const zgpu_chain *c) { return *c->chain; }
bool zgpu::chain_validates(const zgpu_chain *c) { return c->validate; }
int zgpu::ctx_device(const zgpu_ctx *c) { return c->device; }
void *zgpu::ctx_dev_alloc(zgpu_ctx *c, size_t bytes) {  // nullptr on failure
  try {
    HIPCHK(hipSetDevice(c->device));
    return c->dev_alloc(bytes);
  } catch (const HipFail &) {
    return nullptr;
  }
}
void zgpu::ctx_dev_free(zgpu_ctx *c, void *p) { c->dev_free(p); }
hipStream_t zgpu::ctx_copy_stream(zgpu_ctx *c) {  // nullptr on failure
  std::lock_guard<std::mutex> lk(c->lane_mu);
  if (!c->peer && (hipSetDevice(c->device) != hipSuccess ||
                   hipStreamCreateWithFlags(&c->peer, hipStreamNonBlocking) != hipSuccess)) {
    c->peer = nullptr;
    return nullptr;
  }
  return c->peer;
}

// composed permutation of all array->array codecs: encoded axis a <-> decoded axis m[a]
static void composed_axes(const Chain &c, uint32_t nd, uint32_t *m) {
  for (uint32_t a = 0; a < nd; a++) m[a] = a;
  for (const Codec &k : c.a2a) {  // E_{k} axis a <-> E_{k-1} axis order[a]
    uint32_t t[ZG_MAXD];
    for (uint32_t a = 0; a < nd; a++) t[a] = m[k.order[a]];
    std::memcpy(m, t, nd * sizeof(uint32_t));
  }
}

static void build_leaf_stages(zgpu_plan &P, const Chain &leaf, uint64_t nelem) {
  // decode order: last b2b first
  const int nb = (int)leaf.b2b.size();
  int pool = 0;
  uint64_t max_slot = 0;
  bool fused_shuffle = false;
  for (int i = nb - 1; i >= 0; i--) {
    const Codec &k = leaf.b2b[i];
    Stage s;
    if (k.kind == CodecKind::Crc32c) {
      s.kind = ST_CRC32C;
      s.at_start = k.at_start;
      P.stages.push_back(s);
      continue;
    }
    if (k.kind == CodecKind::Shuffle && i == 0 && k.elementsize == leaf.es) {
      fused_shuffle = true;  // fused into the scatter stage
      continue;
    }
    // materialising stage: its output is the encoded representation of codecs [bytes, b2b_0..i-1]
    int64_t out_size = (int64_t)(nelem * leaf.es);
    for (int j = 0; j < i; j++) {
      if (leaf.b2b[j].kind == CodecKind::Crc32c) out_size += 4;
      else if (leaf.b2b[j].kind != CodecKind::Shuffle) out_size = -1;
      if (out_size < 0) break;
    }
    if (out_size < 0) throw ChainError{ZGPU_UNSUPPORTED, "a compressor nested inside another variable-size codec"};
    s.kind = k.kind == CodecKind::Gzip    ? ST_GZIP
             : k.kind == CodecKind::Zstd  ? ST_ZSTD
             : k.kind == CodecKind::Blosc ? ST_BLOSC
                                          : ST_UNSHUFFLE;
    s.elementsize = k.elementsize;
    s.pool = pool;
    pool ^= 1;
    max_slot = std::max<uint64_t>(max_slot, (uint64_t)out_size);
    P.stages.push_back(s);
    P.n_pools = std::min(2, P.n_pools + 1);
  }
  P.slot_bytes = (max_slot + 255) & ~(uint64_t)255;
  P.scatter.shuffle = fused_shuffle;
  {
    const char *e = std::getenv("ZGPU_UNSHUFFLE_WIDE");  // A/B knob: 1 / 2 the 16-B unshuffle (scatter.hip)
    P.scatter.pad0 = e ? (uint32_t)std::max(0, std::min(2, std::atoi(e))) : 0u;
  }
}

// ShardingIndex decode spec (sharding.rs:136-235, sharding_codec.rs:1262-1298): the index chain
// must be bytes (+ crc32c), the only index_codecs zarrs' sharding writes and the GPU decodes.
static ZgIndexSpec index_spec(const Codec &sharding, uint64_t n_inner, bool validate) {
  const Chain &xc = *sharding.index;
  if (xc.a2b.kind != CodecKind::Bytes || !xc.a2a.empty())
    throw ChainError{ZGPU_UNSUPPORTED, "index_codecs must be bytes (+crc32c)"};
  for (const Codec &k : xc.b2b)
    if (k.kind != CodecKind::Crc32c) throw ChainError{ZGPU_UNSUPPORTED, "index_codecs must be bytes (+crc32c)"};
  if (xc.b2b.size() > 4) throw ChainError{ZGPU_UNSUPPORTED, "too many index crc32c codecs"};
  ZgIndexSpec S{};
  S.n_inner = n_inner;
  S.index_bytes = (uint64_t)chain_fixed_encoded_size(xc, n_inner * 2);
  S.at_start = sharding.at_start;
  S.big_endian = xc.a2b.big_endian;
  S.n_crc = (uint32_t)xc.b2b.size();
  for (size_t k = 0; k < xc.b2b.size(); k++) S.crc_at_start[k] = xc.b2b[k].at_start;
  S.verify = validate;
  return S;
}

static void plan_build(zgpu_plan &P, const zgpu_chunk_desc *descs) {
  const Chain &top = *P.chain;
  const uint32_t nd = P.nd;
  P.item_desc_status.assign(P.n_desc, 0);
  const bool shard_chain = top.a2b.kind == CodecKind::Sharding;
  // transpose codecs before sharding_indexed (codec_chain.rs:557-646: the sharding codec decodes the
  // transposed array): the shard and its inner chunk grid live in the encoded frame, encoded axis a
  // <-> decoded axis mo[a]; descriptors are mapped into that frame and the scatter writes through
  // output strides permuted back
  uint32_t mo[ZG_MAXD];
  for (uint32_t a = 0; a < nd; a++) mo[a] = a;
  bool outer_perm = false;
  if (shard_chain) {
    for (const Codec &k : top.a2a)
      if (k.order.size() != nd) throw ChainError{ZGPU_INVALID_ARGUMENT, "transpose order rank != array rank"};
    composed_axes(top, nd, mo);
    for (uint32_t a = 0; a < nd; a++) outer_perm = outer_perm || mo[a] != a;
    if (!top.b2b.empty()) throw ChainError{ZGPU_UNSUPPORTED, "bytes->bytes codecs after sharding_indexed"};
    if (top.a2b.inner_shape.size() != nd) throw ChainError{ZGPU_INVALID_ARGUMENT, "sharding chunk_shape rank"};
  }
  // nested sharding (sharding.rs:107-126 nested_local_subchunk_grids): the outer shard's subchunks
  // are shards themselves ("middle" shards); their indexes are decoded on the device after the outer
  // index resolves them, and the leaf chunks resolve through the middle indexes
  const Chain *mid = nullptr;
  if (shard_chain && top.a2b.inner->a2b.kind == CodecKind::Sharding) {
    mid = top.a2b.inner.get();
    if (!mid->a2a.empty() || !mid->b2b.empty())
      throw ChainError{ZGPU_UNSUPPORTED, "codecs around a nested sharding_indexed"};
    if (mid->a2b.inner->a2b.kind == CodecKind::Sharding)
      throw ChainError{ZGPU_UNSUPPORTED, "sharding_indexed nested more than two deep"};
    if (mid->a2b.inner_shape.size() != nd) throw ChainError{ZGPU_INVALID_ARGUMENT, "sharding chunk_shape rank"};
  }
  const Chain &leaf = shard_chain ? (mid ? *mid->a2b.inner : *top.a2b.inner) : top;
  P.leaf = &leaf;
  P.sharded = shard_chain;
  P.nested = mid != nullptr;
  for (const Codec &k : leaf.a2a)
    if (k.order.size() != nd) throw ChainError{ZGPU_INVALID_ARGUMENT, "transpose order rank != array rank"};

  // leaf chunk shape
  uint64_t leaf_shape[ZG_MAXD];
  uint64_t mid_shape[ZG_MAXD], cps2[ZG_MAXD], n_inner2 = 1;  // nested: middle shard shape, its subchunks
  if (shard_chain) {
    for (uint32_t d = 0; d < nd; d++) leaf_shape[d] = (mid ? mid->a2b.inner_shape : top.a2b.inner_shape)[d];
    for (uint32_t d = 0; d < nd; d++) mid_shape[d] = top.a2b.inner_shape[d];
    if (mid) {
      for (uint32_t d = 0; d < nd; d++) {
        if (!leaf_shape[d] || mid_shape[d] % leaf_shape[d])
          throw ChainError{ZGPU_INVALID_ARGUMENT, "nested sharding: subchunk shape does not divide the shard"};
        cps2[d] = mid_shape[d] / leaf_shape[d];
        n_inner2 *= cps2[d];
      }
    }
  } else if (P.n_desc) {
    for (uint32_t d = 0; d < nd; d++) leaf_shape[d] = descs[0].chunk_shape[d];
  } else {
    for (uint32_t d = 0; d < nd; d++) leaf_shape[d] = 1;
  }
  uint64_t nelem = 1;
  for (uint32_t d = 0; d < nd; d++) nelem *= leaf_shape[d];

  uint64_t out_strides[ZG_MAXD], s = 1;
  for (int d = (int)nd - 1; d >= 0; d--) {
    out_strides[d] = s;
    s *= P.out_shape[d];
  }
  const uint64_t es = top.es;
  uint64_t max_sel[ZG_MAXD] = {0};
  uint64_t n_inner = 1, cps[ZG_MAXD];
  if (shard_chain) {
    int64_t isz = -1;
    for (uint32_t d = 0; d < nd; d++) cps[d] = 0;
    (void)isz;
  }

  for (uint64_t i = 0; i < P.n_desc; i++) {
    const zgpu_chunk_desc &D = descs[i];
    bool ok = true, full = true;
    for (uint32_t d = 0; d < nd; d++) {
      if (D.sel_start[d] + D.sel_shape[d] > D.chunk_shape[d] ||
          D.out_start[d] + D.sel_shape[d] > P.out_shape[d])
        ok = false;
      if (D.sel_start[d] != 0 || D.sel_shape[d] != D.chunk_shape[d]) full = false;
      if (!shard_chain && D.chunk_shape[d] != leaf_shape[d]) ok = false;
    }
    if (!ok) {
      P.item_desc_status[i] = ZGPU_INVALID_ARGUMENT;
      continue;
    }
    uint64_t vol = 1;
    for (uint32_t d = 0; d < nd; d++) vol *= D.sel_shape[d];
    if (vol == 0 && (!full || shard_chain)) continue;  // a zero-extent full chunk still runs its checks
    P.alg_bytes_static += vol * es;
    if (!shard_chain) {
      ZgItem it{};
      it.src = (uint64_t)D.enc;
      it.len = D.enc_len;
      it.desc = (uint32_t)i;
      it.flags = (D.enc ? 0u : ZG_ITEM_FILL) | (full ? 0u : ZG_ITEM_PARTIAL);
      if (D.enc) P.alg_bytes_static += D.enc_len;
      P.items.push_back(it);
      for (uint32_t d = 0; d < nd; d++) P.geom.push_back(D.sel_start[d]);
      for (uint32_t d = 0; d < nd; d++) P.geom.push_back(D.sel_shape[d]);
      for (uint32_t d = 0; d < nd; d++) P.geom.push_back(D.out_start[d]);
      for (uint32_t d = 0; d < nd; d++) max_sel[d] = std::max(max_sel[d], D.sel_shape[d]);
      continue;
    }
    // sharded descriptor: one item per intersecting inner chunk, in the sharding codec's (encoded)
    // frame: axis a is decoded axis mo[a]
    uint64_t c_sh[ZG_MAXD], c_ss[ZG_MAXD], c_sz[ZG_MAXD], c_os[ZG_MAXD];
    for (uint32_t a = 0; a < nd; a++) {
      c_sh[a] = D.chunk_shape[mo[a]];
      c_ss[a] = D.sel_start[mo[a]];
      c_sz[a] = D.sel_shape[mo[a]];
      c_os[a] = D.out_start[mo[a]];
    }
    // subchunks of the (outer) shard: the leaf chunks, or the middle shards when nested
    const uint64_t *sub_shape = mid ? mid_shape : leaf_shape;
    n_inner = 1;
    for (uint32_t d = 0; d < nd; d++) {
      if (c_sh[d] % sub_shape[d]) ok = false;
      cps[d] = c_sh[d] / sub_shape[d];
      n_inner *= cps[d];
    }
    if (!ok) {  // calculate_chunks_per_shard error (sharding.rs:136-154)
      P.item_desc_status[i] = ZGPU_INVALID_ARGUMENT;
      continue;
    }
    if (P.ispec.n_inner && P.ispec.n_inner != n_inner) {
      P.item_desc_status[i] = ZGPU_UNSUPPORTED;  // mixed shard shapes in one batch
      continue;
    }
    P.ispec.n_inner = n_inner;
    const uint32_t shard_slot = (uint32_t)P.shards.size();
    P.shards.push_back(ZgShard{(uint64_t)D.enc, D.enc ? D.enc_len : 0});
    uint64_t lo[ZG_MAXD], hi[ZG_MAXD], idx[ZG_MAXD];
    // one leaf item per intersecting leaf chunk; `sub` (nested: the middle shard, its index slot,
    // its selection [m0, m1) and output origin mo0) or the outer shard itself
    auto add_leaves = [&](uint32_t slot, const uint64_t *m0, const uint64_t *m1, const uint64_t *mo0,
                          const uint64_t *grid) {
      uint64_t llo[ZG_MAXD], lhi[ZG_MAXD], li[ZG_MAXD];
      for (uint32_t d = 0; d < nd; d++) {
        llo[d] = m0[d] / leaf_shape[d];
        lhi[d] = (m1[d] - 1) / leaf_shape[d] + 1;
        li[d] = llo[d];
      }
      for (;;) {
        uint64_t lin = 0;
        ZgItem it{};
        it.desc = (uint32_t)i;
        it.shard = slot;
        it.flags = D.enc ? (ZG_ITEM_SHARDED | (full ? 0u : ZG_ITEM_PARTIAL)) : ZG_ITEM_FILL;
        uint64_t g[3 * ZG_MAXD];
        for (uint32_t d = 0; d < nd; d++) {
          lin = lin * grid[d] + li[d];
          const uint64_t cs = li[d] * leaf_shape[d], ce = cs + leaf_shape[d];
          const uint64_t s0 = std::max(m0[d], cs), s1 = std::min(m1[d], ce);
          g[d] = s0 - cs;
          g[nd + d] = s1 - s0;
          g[2 * nd + d] = mo0[d] + (s0 - m0[d]);
          max_sel[d] = std::max(max_sel[d], s1 - s0);
        }
        it.inner = (uint32_t)lin;
        P.items.push_back(it);
        P.geom.insert(P.geom.end(), g, g + 3 * nd);
        int d = (int)nd - 1;
        for (; d >= 0; d--) {
          if (++li[d] < lhi[d]) break;
          li[d] = llo[d];
        }
        if (d < 0) break;
      }
    };
    if (!mid) {
      uint64_t m1[ZG_MAXD];
      for (uint32_t d = 0; d < nd; d++) m1[d] = c_ss[d] + c_sz[d];
      add_leaves(shard_slot, c_ss, m1, c_os, cps);
      continue;
    }
    if (P.ispec2.n_inner && P.ispec2.n_inner != n_inner2) {
      P.item_desc_status[i] = ZGPU_UNSUPPORTED;
      continue;
    }
    P.ispec2.n_inner = n_inner2;
    for (uint32_t d = 0; d < nd; d++) {
      lo[d] = c_ss[d] / mid_shape[d];
      hi[d] = (c_ss[d] + c_sz[d] - 1) / mid_shape[d] + 1;
      idx[d] = lo[d];
    }
    for (;;) {  // every intersecting middle shard: an index slot, then its leaf chunks
      uint64_t lin = 0, m0[ZG_MAXD], m1[ZG_MAXD], mo0[ZG_MAXD];
      for (uint32_t d = 0; d < nd; d++) {
        lin = lin * cps[d] + idx[d];
        const uint64_t cs = idx[d] * mid_shape[d], ce = cs + mid_shape[d];
        const uint64_t s0 = std::max(c_ss[d], cs), s1 = std::min(c_ss[d] + c_sz[d], ce);
        m0[d] = s0 - cs;
        m1[d] = s1 - cs;
        mo0[d] = c_os[d] + (s0 - c_ss[d]);
      }
      const uint32_t mslot = (uint32_t)P.mids.size();
      ZgItem mi{};
      mi.desc = (uint32_t)i;
      mi.shard = shard_slot;
      mi.inner = (uint32_t)lin;
      mi.flags = D.enc ? ZG_ITEM_SHARDED : ZG_ITEM_FILL;
      P.mids.push_back(mi);
      add_leaves(mslot, m0, m1, mo0, cps2);
      int d = (int)nd - 1;
      for (; d >= 0; d--) {
        if (++idx[d] < hi[d]) break;
        idx[d] = lo[d];
      }
      if (d < 0) break;
    }
  }

  if (shard_chain) {
    P.ispec = index_spec(top.a2b, P.ispec.n_inner, P.validate);
    for (const ZgShard &sh : P.shards)
      if (sh.ptr) P.alg_bytes_static += P.ispec.index_bytes;
    if (mid) {
      P.ispec2 = index_spec(mid->a2b, n_inner2, P.validate);
      for (const ZgItem &m : P.mids)
        if (!(m.flags & ZG_ITEM_FILL)) P.alg_bytes_static += P.ispec2.index_bytes;
    }
  }

  build_leaf_stages(P, leaf, nelem);

  // scatter parameters
  ZgScatter &S = P.scatter;
  S.nd = nd;
  S.es = leaf.es;
  S.comp = leaf.comp;
  S.swap = leaf.a2b.big_endian && leaf.comp > 1;
  S.nelem = nelem;
  std::memcpy(S.fill, leaf.fill, 16);
  uint32_t m[ZG_MAXD];
  composed_axes(leaf, nd, m);
  uint64_t eshape[ZG_MAXD], est[ZG_MAXD];
  for (uint32_t a = 0; a < nd; a++) eshape[a] = leaf_shape[m[a]];
  s = 1;
  for (int a = (int)nd - 1; a >= 0; a--) {
    est[a] = s;
    s *= eshape[a];
  }
  for (uint32_t a = 0; a < nd; a++) S.enc_stride[m[a]] = est[a];
  for (uint32_t d = 0; d < nd; d++) {
    S.chunk_shape[d] = leaf_shape[d];
    S.out_stride[d] = out_strides[mo[d]];
  }
  S.tile_a = m[nd - 1];
  S.tile_b = ZG_MAXD;
  for (uint32_t d = 0; d + 1 < nd; d++) {
    if (d == S.tile_a) continue;
    if (S.tile_b == ZG_MAXD || S.enc_stride[d] <= S.enc_stride[S.tile_b]) S.tile_b = d;
  }
  if (outer_perm && S.out_stride[nd - 1] != 1) {
    P.scatter_mode = SCATTER_GENERIC;  // the row / tile kernels write unit-stride output rows
  } else if (S.tile_a == nd - 1) {
    P.scatter_mode = SCATTER_ROWS;
  } else if (!S.shuffle && (S.es == 1 || S.es == 2 || S.es == 4 || S.es == 8)) {
    P.scatter_mode = SCATTER_TILED;
  } else {
    P.scatter_mode = SCATTER_GENERIC;
  }
  P.scatter_units = P.items.empty() ? 0 : scatter_units_per_item(P.scatter_mode, S, max_sel);

  // blosc as the last stage feeding the rows scatter unchanged (no swap / shuffle / transpose), every
  // decoded item a whole chunk on 16-B aligned output rows: k_blosc_finish writes the rows itself
  if (!P.stages.empty() && P.stages.back().kind == ST_BLOSC && P.scatter_mode == SCATTER_ROWS && !S.swap &&
      !S.shuffle && S.nelem > 0 && S.out_stride[nd - 1] == 1 && (S.chunk_shape[nd - 1] * S.es) % 16 == 0) {
    bool ok = true;
    uint64_t st = 1;
    for (int a = (int)nd - 1; a >= 0 && ok; a--) {
      ok = S.enc_stride[a] == st && (a == (int)nd - 1 || (S.out_stride[a] * S.es) % 16 == 0);
      st *= S.chunk_shape[a];
    }
    for (size_t i = 0; i < P.items.size() && ok; i++) {
      if (P.items[i].flags & ZG_ITEM_FILL) continue;
      const uint64_t *g = P.geom.data() + i * 3 * nd;
      for (uint32_t d = 0; d < nd && ok; d++) ok = g[d] == 0 && g[nd + d] == S.chunk_shape[d];
      ok = ok && (g[2 * nd + nd - 1] * S.es) % 16 == 0;
    }
    P.bl_direct = ok && !std::getenv("ZGPU_BLOSC_NO_DIRECT");
  }
  // gzip as the last stage feeding the rows scatter unchanged (no swap / shuffle / transpose), rows of a
  // power-of-two multiple of 16 bytes, the row axes but the outermost of power-of-two extent: k_gzip
  // writes the items whose selection is their whole chunk into the output rows itself and the scatter
  // takes only the others (C3: the subset's 12,167 interior inner chunks of 15,625). ZGPU_GZIP_DIRECT=0: off.
  {
    const char *gz_env = std::getenv("ZGPU_GZIP_DIRECT");  // read per plan (an A/B knob)
    const bool gz_on = !gz_env || std::atoi(gz_env) != 0;
    const uint64_t Lb = S.chunk_shape[nd - 1] * S.es;
    bool ok = gz_on && !P.stages.empty() && P.stages.back().kind == ST_GZIP && P.scatter_mode == SCATTER_ROWS &&
              !S.swap && !S.shuffle && S.nelem > 0 && nd >= 1 && nd <= 3 && S.out_stride[nd - 1] == 1 && Lb >= 16 &&
              (nd < 2 || S.out_stride[0] * S.es < (1ull << 32)) && S.nelem * S.es < (1ull << 32) &&
              (Lb & (Lb - 1)) == 0;
    uint64_t st = 1;
    for (int a = (int)nd - 1; a >= 0 && ok; a--) {
      ok = S.enc_stride[a] == st && (a == (int)nd - 1 || (S.out_stride[a] * S.es) % 16 == 0) &&
           (a == 0 || a == (int)nd - 1 || (S.chunk_shape[a] & (S.chunk_shape[a] - 1)) == 0);
      st *= S.chunk_shape[a];
    }
    P.gz_direct = ok;
    if (ok) {
      P.gz.want = S.nelem * S.es;
      P.gz.nd = nd;
      P.gz.lbs = (uint32_t)__builtin_ctzll(Lb);
      for (uint32_t d = 0; d < nd; d++) {
        P.gz.cshape[d] = S.chunk_shape[d];
        P.gz.ostr[d] = S.out_stride[d] * S.es;
      }
    }
  }
  // blosc feeding the scatter directly (its decoded bytes are the chunk's encoded-layout elements; a
  // fused unshuffle would interleave planes): a partial selection needs only the byte range between
  // its first and last element in the encoded layout, so only the blocks that cover it are decoded,
  // as the reference's blosc partial decoder does (blosc_partial_decoder.rs:33-60 ->
  // blosc_decompress_bytes_partial, c-blosc's blosc_getitem)
  if (!P.stages.empty() && P.stages.back().kind == ST_BLOSC && !S.shuffle && !std::getenv("ZGPU_BLOSC_NO_PARTIAL")) {
    bool any = false;
    P.bl_need.assign(2 * P.items.size(), 0);
    for (size_t i = 0; i < P.items.size(); i++) {
      P.bl_need[2 * i + 1] = UINT64_MAX;
      if (!(P.items[i].flags & ZG_ITEM_PARTIAL)) continue;
      const uint64_t *g = P.geom.data() + i * 3 * nd;
      uint64_t lo = 0, hi = 0;
      bool empty = false;
      for (uint32_t d = 0; d < nd; d++) {
        if (!g[nd + d]) empty = true;
        lo += g[d] * S.enc_stride[d];
        hi += (g[d] + g[nd + d] - 1) * S.enc_stride[d];
      }
      if (empty) continue;
      P.bl_need[2 * i] = lo * S.es;
      P.bl_need[2 * i + 1] = (hi + 1) * S.es;
      any = true;
    }
    if (!any) P.bl_need.clear();
  }
}

static void plan_upload(zgpu_plan &P, hipStream_t us) {
  zgpu_ctx &C = *P.ctx;
  const size_t ni = P.items.size();
  if (ni) {
    P.d_items = (ZgItem *)C.dev_alloc(ni * sizeof(ZgItem));
    P.d_items_init = (ZgItem *)C.dev_alloc(ni * sizeof(ZgItem));
    P.d_geom = (uint64_t *)C.dev_alloc(P.geom.size() * 8);
    HIPCHK(hipMemcpyAsync(P.d_items_init, P.items.data(), ni * sizeof(ZgItem), hipMemcpyHostToDevice, us));
    HIPCHK(hipMemcpyAsync(P.d_geom, P.geom.data(), P.geom.size() * 8, hipMemcpyHostToDevice, us));
    for (int k = 0; k < P.n_pools; k++) P.d_pool[k] = (uint8_t *)C.dev_alloc(ni * P.slot_bytes);
    if (!P.bl_need.empty()) {
      P.d_bl_need = (uint64_t *)C.dev_alloc(P.bl_need.size() * 8);
      HIPCHK(hipMemcpyAsync(P.d_bl_need, P.bl_need.data(), P.bl_need.size() * 8, hipMemcpyHostToDevice, us));
    }
    for (const Stage &s : P.stages) {
      if (s.kind == ST_GZIP && !P.d_order) {
        P.d_order = (uint32_t *)C.dev_alloc(ni * 4);
        if (const uint64_t b = gzip_seg_scratch_bytes((uint32_t)ni)) P.d_gz_seg = (uint32_t *)C.dev_alloc(b);
      }
      if (s.kind == ST_ZSTD && !P.zs.blks) {
        uint64_t blk_bytes;
        zstd_scratch_layout(P.slot_bytes, P.zs.blk_cap, blk_bytes, P.zs.lit_stride, P.zs.seq_cap);
        P.zs.blks = C.dev_alloc(ni * (uint64_t)P.zs.blk_cap * blk_bytes);
        P.zs.norm = (int16_t *)C.dev_alloc(ni * (uint64_t)P.zs.blk_cap * zstd_norm_bytes());
        P.zs.nblk = (uint32_t *)C.dev_alloc(ni * 4);
        P.zs.mode = (uint32_t *)C.dev_alloc(ni * 4);
        P.zs.lit = (uint8_t *)C.dev_alloc(ni * P.zs.lit_stride);
        P.zs.seq = (uint32_t *)C.dev_alloc(ni * P.zs.seq_cap * 12);
        P.d_zser = (uint32_t *)C.dev_alloc(ni * 4);
        P.zs.ser_list = P.d_zser;
        if (const uint64_t rb = zstd_lit_rec_bytes(P.zs.lit_rec_wgs)) P.zs.lit_rec = (uint8_t *)C.dev_alloc(rb);
        static const uint64_t par_max = [] {  // ZGPU_ZSTD_XPAR_MB: the latency mode's batch limit (tuning)
          const char *e = std::getenv("ZGPU_ZSTD_XPAR_MB");
          return e ? (uint64_t)std::strtoull(e, nullptr, 10) << 20 : ZPAR_MAX_BYTES;
        }();
        if (ni * P.slot_bytes <= par_max) {  // the window executor's latency mode (few frames)
          P.zs.ext = (uint32_t *)C.dev_alloc(2 * ni * P.slot_bytes * 4);
          P.zs.ext_cnt = (unsigned long long *)C.dev_alloc(ZEXT_ROUNDS * 8);
          P.zs.ext_items = ni;
        }
      }
    }
  }
  P.ctl_bytes = 256 + ni * 4;
  P.d_ctl = (uint8_t *)C.dev_alloc(P.ctl_bytes);
  P.h_ctl = (uint8_t *)C.host_alloc(P.ctl_bytes);
  P.d_counter = (unsigned long long *)P.d_ctl;
  P.d_status = (uint32_t *)(P.d_ctl + 256);
  P.zs.counters = P.d_counter + CTR_ZSTD_SERIAL;
  P.zs.ser_count = P.d_counter + CTR_ZSTD_NSER;
  P.zs.max_nblk = P.d_counter + CTR_ZSTD_MAXBLK;
  if (const char *e = std::getenv("ZGPU_ZSTD_FORCE_SERIAL")) P.zs.force_serial = std::atoi(e) != 0;
  if (!P.shards.empty()) {
    P.d_shards = (ZgShard *)C.dev_alloc(P.shards.size() * sizeof(ZgShard));
    P.d_index = (uint64_t *)C.dev_alloc(P.shards.size() * P.ispec.n_inner * 16);
    P.d_shard_status = (uint32_t *)C.dev_alloc(P.shards.size() * 4);
    HIPCHK(hipMemcpyAsync(P.d_shards, P.shards.data(), P.shards.size() * sizeof(ZgShard), hipMemcpyHostToDevice,
                          us));
  }
  if (!P.mids.empty()) {
    const size_t nm = P.mids.size();
    P.d_mids = (ZgItem *)C.dev_alloc(nm * sizeof(ZgItem));
    P.d_mids_init = (ZgItem *)C.dev_alloc(nm * sizeof(ZgItem));
    P.d_mid_status = (uint32_t *)C.dev_alloc(nm * 4);
    P.d_shard_status2 = (uint32_t *)C.dev_alloc(nm * 4);
    P.d_mid_shards = (ZgShard *)C.dev_alloc(nm * sizeof(ZgShard));
    P.d_index2 = (uint64_t *)C.dev_alloc(nm * P.ispec2.n_inner * 16);
    HIPCHK(hipMemcpyAsync(P.d_mids_init, P.mids.data(), nm * sizeof(ZgItem), hipMemcpyHostToDevice, us));
  }
}

// blosc stage: frame headers -> stream table layout -> streams + blocks on the device -> zstd / lz4 /
// blosclz stream decode -> per-block gather + unshuffle into the item slots. The first execution of a
// plan reads the headers back to size the table (the one host round trip of any stage) and records
// the sizes as capacities; later executions lay the table out on the device against them
// (k_blosc_layout) and stay asynchronous. A later input that outgrows them is re-run by plan_statuses.
static void blosc_stage(zgpu_plan &P, const Stage &st, uint8_t *out, hipStream_t s) {
  zgpu_ctx &C = *P.ctx;
  const uint32_t ni = (uint32_t)P.items.size();
  uint8_t *dst = P.d_pool[st.pool];
  BlInfo *info = (BlInfo *)P.grow(P.bl_info, ni * sizeof(BlInfo));
  HIPCHK(launch_blosc_info(P.d_items, P.d_status, ni, P.slot_bytes, info, s));
  uint64_t *d_bases = (uint64_t *)P.grow(P.bl_bases, ni * 16);
  BlDecode D{};
  D.bases = d_bases;
  if (P.bl_direct && ((uintptr_t)out & 15) == 0) {
    D.dout = out;
    D.geom = P.d_geom;
    D.sc = P.scatter;
  }
  D.ovf = P.d_counter + CTR_BLOSC_OVF;
  D.need = P.d_bl_need;
  D.blocks_decoded = P.d_counter + CTR_BLOSC_BLOCKS;
  BlCaps &caps = P.bl_caps;
  const bool cached = P.bl_caps_valid;
  if (!cached) {
    const size_t hbytes = ni * sizeof(BlInfo);
    if (P.bl_h_n < hbytes) {
      C.host_free(P.bl_h);
      P.bl_h = (uint8_t *)C.host_alloc(hbytes);
      P.bl_h_n = hbytes;
    }
    HIPCHK(hipMemcpyAsync(P.bl_h, info, ni * sizeof(BlInfo), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    std::vector<BlInfo> hi(ni);
    std::memcpy(hi.data(), P.bl_h, ni * sizeof(BlInfo));
    BlCaps exact{0, 0, 0, 0};
    for (uint32_t i = 0; i < ni; i++) {
      if (hi[i].comp == BL_COMP_SKIP) continue;
      exact.n_sub += hi[i].nsub;
      exact.n_blk += hi[i].nblk;
      if (hi[i].nsub)
        exact.kinds |= hi[i].comp == BL_COMP_ZSTD ? BL_HAS_ZSTD : hi[i].comp == BL_COMP_LZ4 ? BL_HAS_LZ4
                       : hi[i].comp == BL_COMP_BLOSCLZ ? BL_HAS_BLOSCLZ : hi[i].comp == BL_COMP_ZLIB ? BL_HAS_ZLIB
                       : hi[i].comp == BL_COMP_SNAPPY ? BL_HAS_SNAPPY : 0u;
      exact.max_ne = std::max<uint64_t>(exact.max_ne, hi[i].max_ne);
    }
    // capacities only grow (a plan whose inputs alternate between layouts settles on their maximum)
    if (P.bl_caps_seen) {
      caps.n_sub = std::max(caps.n_sub, exact.n_sub);
      caps.n_blk = std::max(caps.n_blk, exact.n_blk);
      caps.max_ne = std::max(caps.max_ne, exact.max_ne);
      caps.kinds |= exact.kinds;
    } else {
      caps = exact;
    }
    P.bl_caps_seen = P.bl_caps_valid = true;
  }
  D.n_sub = caps.n_sub;
  D.n_blk = caps.n_blk;
  D.n_zstd = caps.kinds & BL_HAS_ZSTD;
  D.n_lz4 = caps.kinds & BL_HAS_LZ4;
  D.n_blosclz = caps.kinds & BL_HAS_BLOSCLZ;
  D.n_zlib = caps.kinds & BL_HAS_ZLIB;
  D.n_snappy = caps.kinds & BL_HAS_SNAPPY;
  const uint64_t ns = std::max<uint64_t>(D.n_sub, 1);
  D.subs = (ZgItem *)P.grow(P.bl_subs, ns * sizeof(ZgItem));
  D.sub_status = (uint32_t *)P.grow(P.bl_sub_status, ns * 4);
  D.sub_kind = (uint32_t *)P.grow(P.bl_sub_kind, ns * 4);
  D.blocks = (BlBlock *)P.grow(P.bl_blocks, std::max<uint64_t>(D.n_blk, 1) * sizeof(BlBlock));
  if (D.n_zstd + D.n_lz4 + D.n_blosclz + D.n_zlib + D.n_snappy) {
    D.sub_slot = (caps.max_ne + 255) & ~(uint64_t)255;
    D.tmp = (uint8_t *)P.grow(P.bl_tmp, D.n_sub * D.sub_slot);
  }
  if (D.n_zlib) {
    D.zaux = (uint2 *)P.grow(P.bl_zaux, D.n_sub * sizeof(uint2));
    if (const uint64_t b = gzip_seg_scratch_bytes((uint32_t)D.n_sub)) D.zseg = (uint32_t *)P.grow(P.bl_zseg, b);
  }
  D.lz_list = (D.n_lz4 || D.n_blosclz || D.n_snappy) ? (uint32_t *)P.grow(P.bl_lzl, 2 * (D.n_sub + 1) * 4) : nullptr;
  if (D.n_zstd) {
    uint64_t blk_bytes;
    zstd_scratch_layout(D.sub_slot, D.zs.blk_cap, blk_bytes, D.zs.lit_stride, D.zs.seq_cap);
    D.zs.blks = P.grow(P.bl_zblks, D.n_sub * (uint64_t)D.zs.blk_cap * blk_bytes);
    D.zs.norm = (int16_t *)P.grow(P.bl_znorm, D.n_sub * (uint64_t)D.zs.blk_cap * zstd_norm_bytes());
    D.zs.nblk = (uint32_t *)P.grow(P.bl_znblk, D.n_sub * 4);
    D.zs.mode = (uint32_t *)P.grow(P.bl_zmode, D.n_sub * 4);
    D.zs.lit = (uint8_t *)P.grow(P.bl_zlit, D.n_sub * D.zs.lit_stride);
    D.zs.seq = (uint32_t *)P.grow(P.bl_zseq, D.n_sub * D.zs.seq_cap * 12);
    D.zs.counters = P.zs.counters;
    D.zs.max_nblk = P.zs.max_nblk;
    D.zs.force_serial = P.zs.force_serial;
    D.zs.ser_list = (uint32_t *)P.grow(P.bl_zser, D.n_sub * 4);
    if (const uint64_t rb = zstd_lit_rec_bytes(D.zs.lit_rec_wgs)) D.zs.lit_rec = (uint8_t *)P.grow(P.bl_zrec, rb);
    // k_blosc_finish reads raw / rle / literal-only zstd blocks where they lie (ZGPU_BLOSC_ALIAS=0: off)
    const char *ae = std::getenv("ZGPU_BLOSC_ALIAS");  // read per call (tests switch it)
    const bool alias_on = !ae || std::atoi(ae) != 0;
    D.zs.alias = alias_on ? (uint64_t *)P.grow(P.bl_zalias, D.n_sub * 3 * ZALIAS * 8) : nullptr;
    D.zs.ser_count = P.zs.ser_count;
    D.zs.launch_serial = P.zs.launch_serial;
    P.zstd_fork(D.zs, s);
    P.zstd_split(D.zs, s);
  }
  // the layout (bases, inert tails past this execution's totals) is always computed on the device
  HIPCHK(launch_blosc_layout(info, ni, d_bases, caps, D, s));
  HIPCHK(launch_blosc_decode(P.d_items, P.d_status, ni, info, D, dst, P.slot_bytes, s));
}

// Enqueue the decode of an uploaded plan on stream s.
static void plan_enqueue(zgpu_plan &P, uint8_t *out, hipStream_t s) {
  const uint32_t ni = (uint32_t)P.items.size();
  P.last_out = out;
  HIPCHK(hipMemsetAsync(P.d_ctl, 0, P.ctl_bytes, s));
  if (!ni) return;
  P.zs.launch_serial = P.zstd_serial_off ? 0u : 1u;
  P.zstd_serial_skipped = P.zstd_serial_off;
  // stages rewrite each item's {src,len} in place; a chain with none reads the uploaded table as is
  const bool mutates = P.sharded || !P.stages.empty();
  ZgItem *items = mutates ? P.d_items : P.d_items_init;
  if (mutates)
    HIPCHK(hipMemcpyAsync(P.d_items, P.d_items_init, ni * sizeof(ZgItem), hipMemcpyDeviceToDevice, s));
  if (P.sharded) {
    HIPCHK(launch_shard_index(P.d_shards, (uint32_t)P.shards.size(), P.ispec, P.d_index, P.d_shard_status, 0, s));
    if (P.nested && !P.mids.empty()) {
      // middle shards: resolved through the outer index, their indexes decoded, then the leaves
      // resolve through them (a middle-shard error reaches every leaf of it via its status)
      const uint32_t nm = (uint32_t)P.mids.size();
      HIPCHK(hipMemcpyAsync(P.d_mids, P.d_mids_init, nm * sizeof(ZgItem), hipMemcpyDeviceToDevice, s));
      HIPCHK(hipMemsetAsync(P.d_mid_status, 0, nm * 4, s));
      HIPCHK(launch_item_resolve(P.d_mids, P.d_mid_status, nm, P.d_shards, P.d_index, P.d_shard_status,
                                 P.ispec.n_inner, P.d_counter + CTR_SCRATCH, s));
      HIPCHK(launch_mid_shards(P.d_mids, P.d_mid_status, nm, P.d_mid_shards, P.d_shard_status2, s));
      HIPCHK(launch_shard_index(P.d_mid_shards, nm, P.ispec2, P.d_index2, P.d_shard_status2, 1, s));
      HIPCHK(launch_item_resolve(P.d_items, P.d_status, ni, P.d_mid_shards, P.d_index2, P.d_shard_status2,
                                 P.ispec2.n_inner, P.d_counter + CTR_ENC_BYTES, s));
    } else if (!P.nested) {
      HIPCHK(launch_item_resolve(P.d_items, P.d_status, ni, P.d_shards, P.d_index, P.d_shard_status, P.ispec.n_inner,
                                 P.d_counter, s));
    }
  }
  int crc_tail = 0;  // a trailing crc32c stage handed to the next gzip stage (launch_gzip places it)
  bool wrote_direct = false;  // a stage wrote whole items into the output (the scatter lists the rest)
  for (size_t si = 0; si < P.stages.size(); si++) {
    const Stage &st = P.stages[si];
    switch (st.kind) {
      case ST_CRC32C:
        if (!st.at_start && si + 1 < P.stages.size() && P.stages[si + 1].kind == ST_GZIP && P.d_gz_seg) {
          crc_tail = P.validate ? 1 : 2;
          break;
        }
        HIPCHK(launch_crc32c_strip(P.d_items, P.d_status, ni, st.at_start, P.validate ? 1 : 0, s));
        break;
      case ST_GZIP: {
        GzDirect gd = P.gz;
        const bool direct = P.gz_direct && si + 1 == P.stages.size() && !P.no_scatter && out &&
                            ((uintptr_t)out & 15) == 0;
        gd.dout = direct ? out : nullptr;
        gd.geom = P.d_geom;
        // A/B (ZGPU_GZIP_CRC_FORK=1): the trailing crc32c checked on the plan's side stream beside the
        // one-wave kernel instead of by k_crc32c_strip ahead of it. It loses on C3 (18.11-18.18 ms against
        // 17.75-17.83 on one box, profiles/r06/r06cf_c3_gzip_crc_fork_ab.txt): the check's workgroups take
        // CU slots from the latency-bound decode
        GzCrcFork cf{};
        const char *fe = std::getenv("ZGPU_GZIP_CRC_FORK");
        const bool fork = crc_tail == 1 && fe && std::atoi(fe) != 0 && !(P.flags & ZGPU_ONE_STREAM);
        if (fork) {
          P.zstd_fork(P.zs, s);  // creates the plan's side stream and events (one compressor per chain)
        }
        if (fork && P.zside) {
          const size_t nb = (size_t)ni * (sizeof(ZgItem) + 8);
          uint8_t *scr = (uint8_t *)P.grow(P.gz_crc, nb);
          cf.side = P.zside;
          cf.ev_fork = P.zev[0];
          cf.ev_join = P.zev[1];
          cf.snap_items = (ZgItem *)scr;
          cf.snap_status = (uint32_t *)(scr + (size_t)ni * sizeof(ZgItem));
          cf.bad = cf.snap_status + ni;
        }
        HIPCHK(launch_gzip(P.d_items, P.d_status, ni, P.d_pool[st.pool], P.slot_bytes, P.d_order, P.d_gz_seg, s,
                           crc_tail, direct ? &gd : nullptr, cf.side ? &cf : nullptr));
        wrote_direct = wrote_direct || direct;
      }
        crc_tail = 0;
        break;
      case ST_ZSTD:
        P.zstd_fork(P.zs, s);
        P.zs.lits_first = (P.flags & ZGPU_ZSTD_LITS_FIRST) && !P.zs.side ? 1u : 0u;
        HIPCHK(launch_zstd(P.d_items, P.d_status, ni, P.d_pool[st.pool], P.slot_bytes, P.zs, s));
        break;
      case ST_BLOSC:
        blosc_stage(P, st, out, s);
        break;
      case ST_UNSHUFFLE:
        HIPCHK(launch_unshuffle(P.d_items, P.d_status, ni, P.d_pool[st.pool], P.slot_bytes, st.elementsize, s));
        break;
    }
  }
  if (!P.no_scatter) {
    // A/B (ZGPU_SCATTER_LIST=1): after the gzip direct rows, the rows scatter over a device-built list
    // of the items still to write instead of the full grid whose written items' blocks exit at once;
    // it lost on C3 (18.22-18.33 vs 17.87-17.94 ms, profiles/r06/r06sl_c3_scatter_list_ab.txt)
    const char *le = std::getenv("ZGPU_SCATTER_LIST");
    uint32_t *live = nullptr;
    if (wrote_direct && le && std::atoi(le) != 0)
      live = (uint32_t *)P.grow(P.live_list, ((size_t)ni + 1) * 4);
    HIPCHK(launch_scatter(items, P.d_geom, P.d_status, P.scatter, out, ni, P.scatter_mode, P.scatter_units, s, live));
  }
}

// InvalidBytesLengthError{len, expected_len} of descriptor d's first mismatching leaf item: the item's
// current {src,len} is the decoded representation the final stage rejected. A materialising stage
// that overflowed its slot leaves src on its input: the decoded length is then only known to exceed
// the expected one (len = UINT64_MAX).
static void size_detail(zgpu_plan &P, uint64_t d, const uint32_t *st, hipStream_t s) {
  const size_t ni = P.items.size();
  for (size_t i = 0; i < ni; i++) {
    if (P.items[i].desc != d || st[i] != ZGPU_DECODED_SIZE_MISMATCH) continue;
    const bool mutates = P.sharded || !P.stages.empty();
    ZgItem it{};
    HIPCHK(hipMemcpyAsync(&it, (mutates ? P.d_items : P.d_items_init) + i, sizeof(ZgItem), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    bool materialised = false, exact = true;
    for (const Stage &stg : P.stages)
      if (stg.kind != ST_CRC32C) materialised = true;
    if (materialised) {
      exact = false;
      for (int k = 0; k < P.n_pools; k++) {
        const uint64_t lo = (uint64_t)P.d_pool[k], hi = lo + ni * P.slot_bytes;
        if (it.src >= lo && it.src < hi) exact = true;
      }
    }
    g_size_detail.valid = 1;
    g_size_detail.desc = d;
    g_size_detail.len = exact ? it.len : UINT64_MAX;
    g_size_detail.expected = P.scatter.nelem * P.scatter.es;
    return;
  }
}

// Read back per-item statuses and reduce them to per-descriptor statuses. Returns the first
// non-zero descriptor status.
static int plan_statuses(zgpu_plan &P, int32_t *status, hipStream_t s) {
  const size_t ni = P.items.size();
  HIPCHK(hipMemcpyAsync(P.h_ctl, P.d_ctl, P.ctl_bytes, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (((const uint64_t *)P.h_ctl)[CTR_BLOSC_OVF]) {
    // the input outgrew the cached blosc layout: nothing was decoded; re-run with a read-back layout
    P.bl_caps_valid = false;
    plan_enqueue(P, P.last_out, s);
    HIPCHK(hipMemcpyAsync(P.h_ctl, P.d_ctl, P.ctl_bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    ((uint64_t *)P.h_ctl)[CTR_BLOSC_RERUN] = 1;
  }
  if (((const uint64_t *)P.h_ctl)[CTR_ZSTD_SERIAL]) {
    if (P.zstd_serial_skipped) {
      // this input has items for the serial zstd decoder, whose launch the plan skipped: re-run with it
      P.zstd_serial_off = false;
      plan_enqueue(P, P.last_out, s);
      HIPCHK(hipMemcpyAsync(P.h_ctl, P.d_ctl, P.ctl_bytes, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
    }
  } else if (((const uint64_t *)P.h_ctl)[CTR_ZSTD_PARALLEL]) {
    P.zstd_serial_off = true;  // no serial item: later executions do not launch the fallback
  }
  std::memcpy(P.last_counters, P.h_ctl, sizeof(P.last_counters));
  P.last_counters[CTR_ITEMS] = ni;
  for (int k = 0; k < CTR_N; k++) g_last_counters[k] += P.last_counters[k];
  const uint32_t *st = (const uint32_t *)(P.h_ctl + 256);
  P.last_enc_bytes = P.last_counters[CTR_ENC_BYTES];
  std::vector<int32_t> ds(P.item_desc_status.begin(), P.item_desc_status.end());
  for (size_t i = 0; i < ni; i++) {
    const uint32_t d = P.items[i].desc;
    if (st[i] && ds[d] == 0) ds[d] = (int32_t)st[i];
  }
  int first = 0;
  uint64_t first_d = 0;
  for (uint64_t d = 0; d < P.n_desc; d++) {
    if (status) status[d] = ds[d];
    if (!first && ds[d]) {
      first = ds[d];
      first_d = d;
    }
  }
  if (first == ZGPU_DECODED_SIZE_MISMATCH && !g_size_detail.valid) size_detail(P, first_d, st, s);
  return first;
}

static zgpu_plan *plan_new(zgpu_ctx *ctx, const std::shared_ptr<Chain> &chain, bool validate, uint32_t nd,
                           const zgpu_chunk_desc *descs, uint64_t n, const uint64_t *out_shape, uint32_t flags) {
  auto P = std::make_unique<zgpu_plan>();
  ctx_ref(ctx);
  P->ctx = ctx;
  P->chain = chain;
  P->validate = validate && !(flags & ZGPU_NO_VALIDATE);
  P->nd = nd;
  P->n_desc = n;
  P->flags = flags;
  P->out_shape.assign(out_shape, out_shape + nd);
  plan_build(*P, descs);
  return P.release();
}

static zgpu_plan *plan_new(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n,
                           const uint64_t *out_shape, uint32_t flags) {
  return plan_new(ch->ctx, ch->chain, ch->validate, nd, descs, n, out_shape, flags);
}

// hip_stream NULL: the context's stream, ordered after all work already queued on the legacy
// default stream (where torch's default stream and plain hipMemcpy/kernels land), so device buffers a
// caller produced there are complete before the decode reads or writes them.
static hipStream_t pick_stream(Lane *L, void *s) {
  if (s) return (hipStream_t)s;
  if (!L->order_ev) HIPCHK(hipEventCreateWithFlags(&L->order_ev, hipEventDisableTiming));
  HIPCHK(hipEventRecord(L->order_ev, nullptr));
  HIPCHK(hipStreamWaitEvent(L->stream, L->order_ev, 0));
  return L->stream;
}

// a plan's own stream (executes without a caller stream: an asynchronous execute and its later
// zgpu_plan_status must meet on one stream)
static Lane *plan_lane(zgpu_plan &P) {
  if (!P.own.stream) HIPCHK(hipStreamCreateWithFlags(&P.own.stream, hipStreamNonBlocking));
  return &P.own;
}

// ------------------------------------------------------------------------------------------------
// General decode: the chains and batches one fused plan does not take, composed from fused plans
// (CodecChain composes any chain, codec_chain.rs:192-229, and zarrs decodes every chunk through its
// own chain and shape):
//  * descriptors of more than one chunk (shard) shape: one plan per shape, on one stream;
//  * bytes->bytes codecs after sharding_indexed (a checksum or compressor over the whole shard): the
//    shards go through those codecs first, stage by stage (the leaf-chunk kernels; slots sized from
//    the streams' own size fields), then decode as plain shards;
//  * sharding nested more than two deep, or codecs around a nested sharding_indexed: the outer shard
//    indexes are decoded on the device and read back, and the intersecting middle shards become the
//    descriptors of the inner chain (recursively, sharding.rs:107-126).
// Synchronous (per-stage read-backs); per-descriptor statuses, first failing item of a descriptor.
// ------------------------------------------------------------------------------------------------
static bool fused_plannable(const Chain &top) {
  if (top.a2b.kind != CodecKind::Sharding) return true;
  if (!top.b2b.empty()) return false;
  const Chain &mid = *top.a2b.inner;
  if (mid.a2b.kind != CodecKind::Sharding) return true;
  return mid.a2a.empty() && mid.b2b.empty() && mid.a2b.inner->a2b.kind != CodecKind::Sharding;
}

static bool same_shape(const zgpu_chunk_desc &a, const zgpu_chunk_desc &b, uint32_t nd) {
  for (uint32_t d = 0; d < nd; d++)
    if (a.chunk_shape[d] != b.chunk_shape[d]) return false;
  return true;
}

static bool uniform_shapes(const zgpu_chunk_desc *descs, uint64_t n, uint32_t nd) {
  for (uint64_t i = 1; i < n; i++)
    if (!same_shape(descs[0], descs[i], nd)) return false;
  return true;
}

static bool desc_geometry_ok(const zgpu_chunk_desc &D, uint32_t nd, const uint64_t *out_shape) {
  for (uint32_t d = 0; d < nd; d++)
    if (D.sel_start[d] + D.sel_shape[d] > D.chunk_shape[d] || D.out_start[d] + D.sel_shape[d] > out_shape[d])
      return false;
  return true;
}

static uint64_t sel_volume(const zgpu_chunk_desc &D, uint32_t nd) {
  uint64_t v = 1;
  for (uint32_t d = 0; d < nd; d++) v *= D.sel_shape[d];
  return v;
}

static bool sel_full(const zgpu_chunk_desc &D, uint32_t nd) {
  for (uint32_t d = 0; d < nd; d++)
    if (D.sel_start[d] != 0 || D.sel_shape[d] != D.chunk_shape[d]) return false;
  return true;
}

// The box [org, org + shape) of a device array (C order, array_shape) into dst + dst_off, compact
// (k_box_copy: one wave per contiguous run).
static void pack_box(const uint8_t *src, uint32_t nd, const uint64_t *array_shape, const uint64_t *org,
                     const uint64_t *shape, uint32_t es, uint8_t *dst, uint64_t dst_off, hipStream_t s) {
  const BoxRuns R = box_runs(nd, array_shape, org, shape, es);
  ZgBoxCopy P{};
  P.outer = R.outer;
  uint64_t cs = R.run_bytes;  // compact strides of the outer axes
  for (int d = (int)R.outer - 1; d >= 0; d--) {
    P.shape[d] = R.shape[d];
    P.src_stride[d] = R.stride[d];
    P.dst_stride[d] = cs;
    cs *= R.shape[d];
  }
  P.src_base = R.base;
  P.dst_base = dst_off;
  P.run_bytes = R.run_bytes;
  P.n_runs = R.n_runs;
  HIPCHK(launch_box_copy(src, dst, P, s));
}

struct GeneralCall {
  zgpu_ctx *C;
  bool validate;
  uint32_t nd;
  uint8_t *out;  // device output array
  const uint64_t *out_shape;
  uint32_t flags;
  hipStream_t s;
  std::vector<std::unique_ptr<zgpu_plan>> keep;  // whole-shard decode slots, alive until the call ends
};

static void decode_general(GeneralCall &G, const std::shared_ptr<Chain> &chain, const zgpu_chunk_desc *descs,
                           uint64_t n, int32_t *status);

// Decode `sub` (sub-descriptor k belongs to caller descriptor owner[k]) and merge: a caller
// descriptor keeps its first error.
static void run_sub(GeneralCall &G, const std::shared_ptr<Chain> &chain, const std::vector<zgpu_chunk_desc> &sub,
                    const std::vector<uint64_t> &owner, int32_t *status) {
  if (sub.empty()) return;
  std::vector<int32_t> st(sub.size(), 0);
  const bool had_detail = g_size_detail.valid;
  decode_general(G, chain, sub.data(), sub.size(), st.data());
  if (!had_detail && g_size_detail.valid) g_size_detail.desc = owner[g_size_detail.desc];
  for (size_t k = 0; k < sub.size(); k++)
    if (st[k] && !status[owner[k]]) status[owner[k]] = st[k];
}

// One bytes->bytes codec applied to whole shards (items[i] = shard i's current bytes; ist[i] its
// status): decoded by a stages-only plan whose slots hold the decoded shards. Compressors size the
// slots from the streams (kernels/probe.hip); a gzip member longer than its ISIZE hint is re-run
// with larger slots up to DEFLATE's 1032:1 bound.
static void shard_stage(GeneralCall &G, const Codec &k, std::vector<ZgItem> &items, std::vector<int32_t> &ist) {
  std::vector<uint32_t> todo;
  for (uint32_t i = 0; i < items.size(); i++)
    if (!ist[i]) todo.push_back(i);
  if (todo.empty()) return;
  Stage st{};
  uint32_t hint_kind = UINT32_MAX;
  switch (k.kind) {
    case CodecKind::Crc32c: st.kind = ST_CRC32C; st.at_start = k.at_start; break;
    case CodecKind::Gzip: st.kind = ST_GZIP; hint_kind = SIZE_HINT_GZIP; break;
    case CodecKind::Zstd: st.kind = ST_ZSTD; hint_kind = SIZE_HINT_ZSTD; break;
    case CodecKind::Blosc: st.kind = ST_BLOSC; hint_kind = SIZE_HINT_BLOSC; break;
    case CodecKind::Shuffle: st.kind = ST_UNSHUFFLE; st.elementsize = k.elementsize; break;
    default: throw ChainError{ZGPU_UNSUPPORTED, "codec '" + k.name + "' after sharding_indexed"};
  }
  uint64_t cap = 0;
  if (st.kind == ST_UNSHUFFLE) {
    for (uint32_t t : todo) cap = std::max(cap, items[t].len);
  } else if (hint_kind != UINT32_MAX) {
    const uint32_t nt = (uint32_t)todo.size();
    std::vector<ZgItem> hi(nt);
    for (uint32_t j = 0; j < nt; j++) hi[j] = items[todo[j]];
    ZgItem *d_it = (ZgItem *)G.C->dev_alloc(nt * sizeof(ZgItem));
    uint8_t *d_buf = (uint8_t *)G.C->dev_alloc(nt * 12);
    std::vector<uint64_t> h(nt, 0);
    hipError_t e = hipMemcpyAsync(d_it, hi.data(), nt * sizeof(ZgItem), hipMemcpyHostToDevice, G.s);
    if (e == hipSuccess) e = hipMemsetAsync(d_buf + nt * 8, 0, nt * 4, G.s);
    if (e == hipSuccess)
      e = launch_size_hint(d_it, (const uint32_t *)(d_buf + nt * 8), nt, hint_kind, (uint64_t *)d_buf, G.s);
    if (e == hipSuccess) e = hipMemcpyAsync(h.data(), d_buf, nt * 8, hipMemcpyDeviceToHost, G.s);
    if (e == hipSuccess) e = hipStreamSynchronize(G.s);
    G.C->dev_free(d_it);
    G.C->dev_free(d_buf);
    if (e != hipSuccess) throw HipFail{e, "whole-shard size hints"};
    for (uint64_t v : h) cap = std::max(cap, v);
  }
  cap = std::max<uint64_t>(cap, 256);
  // one stages-only plan over `set` with slots of `c` bytes; statuses in s, decoded items in res
  auto run = [&](const std::vector<uint32_t> &set, uint64_t c, std::vector<int32_t> &s, std::vector<ZgItem> &res) {
    auto P = std::make_unique<zgpu_plan>();
    ctx_ref(G.C);  // ~zgpu_plan drops it
    P->ctx = G.C;
    P->validate = G.validate;
    P->nd = 1;
    P->n_desc = set.size();
    P->flags = G.flags;
    P->out_shape = {1};
    P->item_desc_status.assign(set.size(), 0);
    for (size_t j = 0; j < set.size(); j++) {
      ZgItem it = items[set[j]];
      it.desc = (uint32_t)j;
      P->items.push_back(it);
    }
    st.pool = 0;
    P->stages = {st};
    P->n_pools = st.kind == ST_CRC32C ? 0 : 1;
    P->slot_bytes = (c + 255) & ~(uint64_t)255;
    P->no_scatter = true;
    plan_upload(*P, G.s);
    plan_enqueue(*P, nullptr, G.s);
    s.assign(set.size(), 0);
    const SizeDetail keep_detail = g_size_detail;
    plan_statuses(*P, s.data(), G.s);
    g_size_detail = keep_detail;  // a shard has no expected decoded size
    res.resize(set.size());
    HIPCHK(hipMemcpyAsync(res.data(), P->d_items, set.size() * sizeof(ZgItem), hipMemcpyDeviceToHost, G.s));
    HIPCHK(hipStreamSynchronize(G.s));
    if (std::find(s.begin(), s.end(), 0) != s.end()) G.keep.push_back(std::move(P));  // slots in use
  };
  // gzip's ISIZE is the decoded size modulo 2^32 (RFC 1952), only a hint: a member that outgrows its
  // slot is re-run ALONE with 8x larger slots, up to DEFLATE's 1032:1 bound and the slot limit
  // (ZGPU_SHARD_SLOT_LIMIT, default 64 GiB); past the limit it fails by itself with
  // DECODED_SIZE_MISMATCH instead of sizing every retried shard's slot for the largest
  static const uint64_t slot_limit = [] {
    const char *e = std::getenv("ZGPU_SHARD_SLOT_LIMIT");
    const uint64_t v = e ? std::strtoull(e, nullptr, 10) : 0;
    return v ? v : (64ull << 30);
  }();
  std::vector<int32_t> s;
  std::vector<ZgItem> res;
  run(todo, std::min(cap, slot_limit), s, res);
  auto settle = [&](uint32_t t, int32_t sj, const ZgItem &r) {
    ist[t] = sj;
    if (!sj) {
      items[t].src = r.src;
      items[t].len = r.len;
    }
  };
  std::vector<uint32_t> again;
  for (size_t j = 0; j < todo.size(); j++) {
    const uint32_t t = todo[j];
    const uint64_t bound = std::min(items[t].len * 1032 + 1024, slot_limit);
    if (s[j] == ZGPU_DECODED_SIZE_MISMATCH && st.kind == ST_GZIP && cap < bound)
      again.push_back(t);
    else
      settle(t, s[j], res[j]);
  }
  for (uint32_t t : again) {
    const uint64_t bound = std::min(items[t].len * 1032 + 1024, slot_limit);
    for (uint64_t c = std::min(cap * 8, bound);; c = std::min(c * 8, bound)) {
      run({t}, c, s, res);
      if (!(s[0] == ZGPU_DECODED_SIZE_MISMATCH && c < bound)) {
        settle(t, s[0], res[0]);
        break;
      }
    }
  }
}

// bytes->bytes codecs after sharding_indexed: decode every selected shard through them (reverse
// order, codec_chain.rs:612-617), then read the decoded shards through the chain without them.
static void predecode_shards(GeneralCall &G, const std::shared_ptr<Chain> &chain, const zgpu_chunk_desc *descs,
                             uint64_t n, int32_t *status) {
  const Chain &top = *chain;
  const uint32_t nd = G.nd;
  std::vector<ZgItem> items;
  std::vector<uint64_t> owner;
  for (uint64_t i = 0; i < n; i++) {
    const zgpu_chunk_desc &D = descs[i];
    if (!desc_geometry_ok(D, nd, G.out_shape)) {
      status[i] = ZGPU_INVALID_ARGUMENT;
      continue;
    }
    if (!D.enc || sel_volume(D, nd) == 0) continue;
    ZgItem it{};
    it.src = (uint64_t)D.enc;
    it.len = D.enc_len;
    it.desc = (uint32_t)items.size();
    it.flags = sel_full(D, nd) ? 0u : ZG_ITEM_PARTIAL;  // a partial read strips crc32c unverified
    items.push_back(it);
    owner.push_back(i);
  }
  std::vector<int32_t> ist(items.size(), 0);
  for (int k = (int)top.b2b.size() - 1; k >= 0; k--) shard_stage(G, top.b2b[k], items, ist);
  auto bare = std::make_shared<Chain>(top);
  bare->b2b.clear();
  std::vector<zgpu_chunk_desc> sub;
  std::vector<uint64_t> sub_owner;
  size_t j = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (status[i]) continue;
    zgpu_chunk_desc D = descs[i];
    if (j < owner.size() && owner[j] == i) {
      const size_t t = j++;
      if (ist[t]) {
        status[i] = ist[t];
        continue;
      }
      D.enc = (const void *)items[t].src;
      D.enc_len = items[t].len;
    }
    sub.push_back(D);
    sub_owner.push_back(i);
  }
  run_sub(G, bare, sub, sub_owner, status);
}

// A sharded chain whose subchunks are shards the fused plan cannot take (codecs around them, or
// sharding below them again): the outer indexes decode on the device (k_shard_index, checksums
// verified) and come back to the host, and every intersecting middle shard becomes a descriptor of
// the inner chain (sharding_codec.rs:617-707 per subchunk; an empty one decodes to the fill value).
static void nested_host(GeneralCall &G, const std::shared_ptr<Chain> &chain, const zgpu_chunk_desc *descs,
                        uint64_t n, int32_t *status) {
  const Chain &top = *chain;
  const uint32_t nd = G.nd;
  const std::vector<uint64_t> &ms = top.a2b.inner_shape;
  if (ms.size() != nd) throw ChainError{ZGPU_INVALID_ARGUMENT, "sharding chunk_shape rank"};
  uint64_t cps[ZG_MAXD], n_inner = 0;
  std::vector<ZgShard> shards;
  std::vector<uint64_t> shard_of(n, UINT64_MAX);
  for (uint64_t i = 0; i < n; i++) {
    const zgpu_chunk_desc &D = descs[i];
    bool ok = desc_geometry_ok(D, nd, G.out_shape);
    uint64_t ni = 1;
    for (uint32_t d = 0; d < nd && ok; d++) {
      if (!ms[d] || D.chunk_shape[d] % ms[d]) ok = false;  // calculate_chunks_per_shard (sharding.rs:136-154)
      else {
        cps[d] = D.chunk_shape[d] / ms[d];
        ni *= cps[d];
      }
    }
    if (!ok) {
      status[i] = ZGPU_INVALID_ARGUMENT;
      continue;
    }
    n_inner = ni;  // one shard shape per call (decode_general groups by shape)
    if (D.enc && sel_volume(D, nd)) {
      shard_of[i] = shards.size();
      shards.push_back(ZgShard{(uint64_t)D.enc, D.enc_len});
    }
  }
  std::vector<uint64_t> index;
  std::vector<uint32_t> sst;
  if (!shards.empty()) {
    const ZgIndexSpec spec = index_spec(top.a2b, n_inner, G.validate);
    const size_t ns = shards.size();
    index.resize(ns * n_inner * 2);
    sst.resize(ns);
    ZgShard *d_sh = (ZgShard *)G.C->dev_alloc(ns * sizeof(ZgShard));
    uint64_t *d_idx = (uint64_t *)G.C->dev_alloc(index.size() * 8);
    uint32_t *d_st = (uint32_t *)G.C->dev_alloc(ns * 4);
    hipError_t e = hipMemcpyAsync(d_sh, shards.data(), ns * sizeof(ZgShard), hipMemcpyHostToDevice, G.s);
    if (e == hipSuccess) e = launch_shard_index(d_sh, (uint32_t)ns, spec, d_idx, d_st, 0, G.s);
    if (e == hipSuccess) e = hipMemcpyAsync(index.data(), d_idx, index.size() * 8, hipMemcpyDeviceToHost, G.s);
    if (e == hipSuccess) e = hipMemcpyAsync(sst.data(), d_st, ns * 4, hipMemcpyDeviceToHost, G.s);
    if (e == hipSuccess) e = hipStreamSynchronize(G.s);
    G.C->dev_free(d_sh);
    G.C->dev_free(d_idx);
    G.C->dev_free(d_st);
    if (e != hipSuccess) throw HipFail{e, "nested shard indexes"};
  }
  std::vector<zgpu_chunk_desc> sub;
  std::vector<uint64_t> owner;
  for (uint64_t i = 0; i < n; i++) {
    const zgpu_chunk_desc &D = descs[i];
    if (status[i] || sel_volume(D, nd) == 0) continue;
    const uint64_t sh = shard_of[i];
    if (sh != UINT64_MAX && sst[sh]) {
      status[i] = (int32_t)sst[sh];
      continue;
    }
    uint64_t lo[ZG_MAXD], hi[ZG_MAXD], idx[ZG_MAXD];
    for (uint32_t d = 0; d < nd; d++) {
      cps[d] = D.chunk_shape[d] / ms[d];
      lo[d] = D.sel_start[d] / ms[d];
      hi[d] = (D.sel_start[d] + D.sel_shape[d] - 1) / ms[d] + 1;
      idx[d] = lo[d];
    }
    for (;;) {  // every intersecting middle shard, C order
      zgpu_chunk_desc M{};
      uint64_t lin = 0;
      for (uint32_t d = 0; d < nd; d++) {
        lin = lin * cps[d] + idx[d];
        const uint64_t cs = idx[d] * ms[d], ce = cs + ms[d];
        const uint64_t s0 = std::max(D.sel_start[d], cs), s1 = std::min(D.sel_start[d] + D.sel_shape[d], ce);
        M.chunk_shape[d] = ms[d];
        M.sel_start[d] = s0 - cs;
        M.sel_shape[d] = s1 - s0;
        M.out_start[d] = D.out_start[d] + (s0 - D.sel_start[d]);
      }
      bool oob = false;
      if (sh != UINT64_MAX) {
        const uint64_t off = index[(sh * n_inner + lin) * 2], size = index[(sh * n_inner + lin) * 2 + 1];
        if (!(off == ~0ull && size == ~0ull)) {
          if (off > D.enc_len || size > D.enc_len - off) oob = true;
          M.enc = (const uint8_t *)D.enc + off;
          M.enc_len = size;
        }
      }
      if (oob) {  // sharding_codec.rs: an inner chunk outside the shard
        status[i] = ZGPU_SHARD_INDEX_OOB;
      } else {
        sub.push_back(M);
        owner.push_back(i);
      }
      int d = (int)nd - 1;
      for (; d >= 0; d--) {
        if (++idx[d] < hi[d]) break;
        idx[d] = lo[d];
      }
      if (d < 0 || oob) break;
    }
  }
  run_sub(G, top.a2b.inner, sub, owner, status);
}

// Transpose codecs before a sharding_indexed the fused plan does not take (bytes->bytes codecs after
// it, or shards with codecs around them / nested deeper below it). zarrs decodes the sharding codec
// on the encoded (transposed) shape, then the transposes (codec_chain.rs:592-646, transpose_codec.rs:
// 264-281), and a partial read asks the sharding partial decoder for the selection's box in the
// encoded frame (transpose_codec_partial.rs). Here every descriptor's selection is decoded by the
// chain without its transposes, in the encoded frame, into its own box of a device buffer (boxes
// stacked along axis 0); the boxes are packed compact (k_box_copy) and then decoded as the leaf chunks
// of [transposes, bytes(native)], which transposes and scatters them into the output in one fused pass.
static void transposed_general(GeneralCall &G, const std::shared_ptr<Chain> &chain, const zgpu_chunk_desc *descs,
                               uint64_t n, int32_t *status) {
  const Chain &top = *chain;
  const uint32_t nd = G.nd, es = top.es;
  uint32_t m[ZG_MAXD];
  composed_axes(top, nd, m);  // encoded axis a <-> decoded axis m[a]
  auto bare = std::make_shared<Chain>(top);
  bare->a2a.clear();
  auto tr = std::make_shared<Chain>(top);
  tr->b2b.clear();
  tr->a2b = Codec{};
  tr->a2b.kind = CodecKind::Bytes;
  tr->a2b.name = "bytes";
  tr->a2b.big_endian = false;  // the decoded elements are native (little-endian) already
  std::vector<zgpu_chunk_desc> enc_descs;
  std::vector<uint64_t> owner, row0;
  uint64_t stacked[ZG_MAXD] = {0};
  for (uint64_t i = 0; i < n; i++) {
    const zgpu_chunk_desc &D = descs[i];
    if (!desc_geometry_ok(D, nd, G.out_shape)) {
      status[i] = ZGPU_INVALID_ARGUMENT;
      continue;
    }
    if (sel_volume(D, nd) == 0) continue;
    zgpu_chunk_desc E = D;
    for (uint32_t a = 0; a < nd; a++) {
      E.chunk_shape[a] = D.chunk_shape[m[a]];
      E.sel_start[a] = D.sel_start[m[a]];
      E.sel_shape[a] = D.sel_shape[m[a]];
      E.out_start[a] = 0;
    }
    E.out_start[0] = stacked[0];
    row0.push_back(stacked[0]);
    stacked[0] += E.sel_shape[0];
    for (uint32_t a = 1; a < nd; a++) stacked[a] = std::max(stacked[a], E.sel_shape[a]);
    enc_descs.push_back(E);
    owner.push_back(i);
  }
  if (enc_descs.empty()) return;
  uint64_t stacked_bytes = es;
  for (uint32_t a = 0; a < nd; a++) stacked_bytes *= stacked[a];
  uint64_t pack_bytes = 0;
  std::vector<uint64_t> pack_off(enc_descs.size());
  for (size_t k = 0; k < enc_descs.size(); k++) {
    pack_off[k] = pack_bytes;
    pack_bytes += sel_volume(enc_descs[k], nd) * es;
  }
  uint8_t *T = (uint8_t *)G.C->dev_alloc(stacked_bytes);
  uint8_t *Pk = nullptr;
  try {
    // the encoded-frame boxes
    GeneralCall G1{G.C, G.validate, nd, T, stacked, G.flags, G.s, {}};
    std::vector<int32_t> st(enc_descs.size(), 0);
    const bool had_detail = g_size_detail.valid;
    decode_general(G1, bare, enc_descs.data(), enc_descs.size(), st.data());
    if (!had_detail && g_size_detail.valid) g_size_detail.desc = owner[g_size_detail.desc];
    Pk = (uint8_t *)G.C->dev_alloc(std::max<uint64_t>(pack_bytes, 1));
    std::vector<zgpu_chunk_desc> leaf;
    std::vector<uint64_t> leaf_owner;
    for (size_t k = 0; k < enc_descs.size(); k++) {
      const uint64_t i = owner[k];
      if (st[k]) {
        status[i] = st[k];
        continue;
      }
      uint64_t org[ZG_MAXD] = {0};
      org[0] = row0[k];
      pack_box(T, nd, stacked, org, enc_descs[k].sel_shape, es, Pk, pack_off[k], G.s);
      zgpu_chunk_desc L{};
      L.enc = Pk + pack_off[k];
      L.enc_len = sel_volume(enc_descs[k], nd) * es;
      for (uint32_t a = 0; a < nd; a++) {
        L.chunk_shape[a] = L.sel_shape[a] = descs[i].sel_shape[a];
        L.sel_start[a] = 0;
        L.out_start[a] = descs[i].out_start[a];
      }
      leaf.push_back(L);
      leaf_owner.push_back(i);
    }
    run_sub(G, tr, leaf, leaf_owner, status);
  } catch (...) {
    G.C->dev_free(T);
    G.C->dev_free(Pk);
    throw;
  }
  G.C->dev_free(T);
  G.C->dev_free(Pk);
}

static void decode_general(GeneralCall &G, const std::shared_ptr<Chain> &chain, const zgpu_chunk_desc *descs,
                           uint64_t n, int32_t *status) {
  for (uint64_t i = 0; i < n; i++) status[i] = 0;
  if (!uniform_shapes(descs, n, G.nd)) {  // one plan per chunk shape
    std::vector<char> done(n, 0);
    for (uint64_t i = 0; i < n; i++) {
      if (done[i]) continue;
      std::vector<zgpu_chunk_desc> sub;
      std::vector<uint64_t> owner;
      for (uint64_t j = i; j < n; j++)
        if (!done[j] && same_shape(descs[i], descs[j], G.nd)) {
          sub.push_back(descs[j]);
          owner.push_back(j);
          done[j] = 1;
        }
      run_sub(G, chain, sub, owner, status);
    }
    return;
  }
  const Chain &top = *chain;
  if (fused_plannable(top)) {
    std::unique_ptr<zgpu_plan> P(plan_new(G.C, chain, G.validate, G.nd, descs, n, G.out_shape, G.flags));
    plan_upload(*P, G.s);
    plan_enqueue(*P, G.out, G.s);
    plan_statuses(*P, status, G.s);
    return;
  }
  if (!top.a2a.empty()) transposed_general(G, chain, descs, n, status);
  else if (!top.b2b.empty()) predecode_shards(G, chain, descs, n, status);
  else nested_host(G, chain, descs, n, status);
}

// ------------------------------------------------------------------------------------------------
// C ABI
// ------------------------------------------------------------------------------------------------
#define ABI_GUARD_BEGIN try {
#define ABI_GUARD_END                                                                          \
  }                                                                                            \
  catch (const ChainError &e) {                                                                \
    return set_err(e.status, e.msg);                                                           \
  }                                                                                            \
  catch (const HipFail &e) {                                                                   \
    return set_err(ZGPU_HIP_ERROR, std::string(e.what) + ": " + hipGetErrorString(e.e));       \
  }                                                                                            \
  catch (const std::exception &e) {                                                            \
    return set_err(ZGPU_INVALID_ARGUMENT, e.what());                                           \
  }

// array_read_ops_common.rs:20-109: subset -> intersecting chunks -> one descriptor per chunk, in
// C order of the chunk grid; lins[k] = descriptor k's C-order linear chunk-grid index.
// Returns ZGPU_OK, -1 for an empty subset (nothing to do), or an error status.
int zgpu::subset_descs(uint32_t nd, const uint64_t *array_shape, const uint64_t *chunk_shape,
                       const uint64_t *sel_start, const uint64_t *sel_shape, std::vector<zgpu_chunk_desc> &descs,
                       std::vector<uint64_t> &lins) {
  uint64_t grid[ZG_MAXD], lo[ZG_MAXD], hi[ZG_MAXD], idx[ZG_MAXD];
  uint64_t nchunks = 1;
  bool empty = false;
  for (uint32_t d = 0; d < nd; d++) {
    if (chunk_shape[d] == 0) return set_err(ZGPU_INVALID_ARGUMENT, "zero chunk extent");
    if (sel_start[d] + sel_shape[d] > array_shape[d])
      return set_err(ZGPU_INVALID_ARGUMENT, "array subset out of bounds");
    grid[d] = (array_shape[d] + chunk_shape[d] - 1) / chunk_shape[d];
    if (sel_shape[d] == 0) {
      empty = true;
      continue;
    }
    lo[d] = sel_start[d] / chunk_shape[d];
    hi[d] = (sel_start[d] + sel_shape[d] - 1) / chunk_shape[d] + 1;
    nchunks *= hi[d] - lo[d];
    idx[d] = lo[d];
  }
  if (empty) return -1;
  descs.reserve(nchunks);
  lins.reserve(nchunks);
  for (;;) {
    zgpu_chunk_desc D{};
    uint64_t lin = 0;
    for (uint32_t d = 0; d < nd; d++) {
      lin = lin * grid[d] + idx[d];
      const uint64_t cs = idx[d] * chunk_shape[d], ce = cs + chunk_shape[d];
      const uint64_t s0 = std::max(sel_start[d], cs), s1 = std::min(sel_start[d] + sel_shape[d], ce);
      D.chunk_shape[d] = chunk_shape[d];
      D.sel_start[d] = s0 - cs;
      D.sel_shape[d] = s1 - s0;
      D.out_start[d] = s0 - sel_start[d];
    }
    descs.push_back(D);
    lins.push_back(lin);
    int d = (int)nd - 1;
    for (; d >= 0; d--) {
      if (++idx[d] < hi[d]) break;
      idx[d] = lo[d];
    }
    if (d < 0) break;
  }
  return ZGPU_OK;
}

extern "C" {

const char *zgpu_version(void) { return "zgpu 0.1.0 (gfx950)"; }

const char *zgpu_status_name(int s) {
  static const char *names[] = {"OK", "INVALID_CHECKSUM", "DECODED_SIZE_MISMATCH", "SHARD_INDEX_OOB",
                                "CORRUPT_STREAM", "INVALID_BYTE_RANGE", "UNSUPPORTED", "CRC_INPUT_TOO_SHORT",
                                "SHARD_TOO_SMALL", "SHUFFLE_LENGTH", "INVALID_ARGUMENT", "HIP_ERROR",
                                "STORAGE_ERROR"};
  return (s >= 0 && s <= 12) ? names[s] : "UNKNOWN";
}

const char *zgpu_last_error(const zgpu_ctx *) { return g_last_error.c_str(); }

int zgpu_ctx_create(int dev, zgpu_ctx **out) {
  ABI_GUARD_BEGIN
  if (!out) return set_err(ZGPU_INVALID_ARGUMENT, "out is NULL");
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (dev < 0 || dev >= n) return set_err(ZGPU_INVALID_ARGUMENT, "no such HIP device");
  HIPCHK(hipSetDevice(dev));
  auto c = std::make_unique<zgpu_ctx>();
  c->device = dev;
  if (const char *e = std::getenv("ZGPU_CTX_LANES")) c->max_lanes = (uint32_t)std::max(1, std::min(64, std::atoi(e)));
  if (const char *e = std::getenv("ZGPU_POOL_CAP_MB")) c->pool_cap = (size_t)std::max(64, std::atoi(e)) << 20;
  if (const char *e = std::getenv("ZGPU_PINNED_CAP_MB")) c->host_cap = (size_t)std::max(64, std::atoi(e)) << 20;
  c->release_lane(c->acquire_lane());  // the first lane up front (stream creation errors surface here)
  *out = c.release();
  return ZGPU_OK;
  ABI_GUARD_END
}

void zgpu_ctx_destroy(zgpu_ctx *c) { ctx_unref(c); }

int64_t zgpu_ctx_refcount(const zgpu_ctx *c) { return c ? c->refs.load() : 0; }

int zgpu_ctx_pool_stats(const zgpu_ctx *c, uint64_t *dev_live, uint64_t *dev_free, uint64_t *host_live,
                        uint64_t *host_free) {
  if (!c) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  zgpu_ctx *m = const_cast<zgpu_ctx *>(c);  // the allocator lock only
  std::lock_guard<std::mutex> lk(m->mu);
  uint64_t dl = 0, hl = 0, hf = 0;
  for (const auto &kv : c->live_dev) dl += kv.second;
  for (const auto &kv : c->live_host) hl += kv.second;
  hf = c->free_host_bytes;
  if (dev_live) *dev_live = dl;
  if (dev_free) *dev_free = c->free_dev_bytes;
  if (host_live) *host_live = hl;
  if (host_free) *host_free = hf;
  return ZGPU_OK;
}

int zgpu_ctx_release_cached(zgpu_ctx *c) {
  if (!c) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> lk(c->mu);
  if (hipSetDevice(c->device) != hipSuccess) (void)hipGetLastError();
  c->trim_free_locked(0);
  c->trim_host_locked(0);
  (void)hipGetLastError();
  return ZGPU_OK;
}

int zgpu_chain_create(zgpu_ctx *ctx, const char *codecs_json, const char *data_type, const void *fill,
                      uint32_t fill_len, int validate, zgpu_chain **out) {
  ABI_GUARD_BEGIN
  if (!ctx || !codecs_json || !data_type || !out) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  uint32_t es, comp;
  if (!data_type_info(data_type, es, comp)) return set_err(ZGPU_UNSUPPORTED, std::string("data type ") + data_type);
  if (fill && fill_len != es) return set_err(ZGPU_INVALID_ARGUMENT, "fill_len != element size");
  uint8_t f[16] = {0};
  if (fill) std::memcpy(f, fill, es);
  Json j = Json::parse(codecs_json);
  auto ch = std::make_unique<zgpu_chain>();
  ch->chain = parse_chain(j, data_type, f);
  ch->validate = validate != 0;
  ctx_ref(ctx);
  ch->ctx = ctx;
  *out = ch.release();
  return ZGPU_OK;
  ABI_GUARD_END
}

void zgpu_chain_destroy(zgpu_chain *c) {
  if (!c) return;
  zgpu_ctx *ctx = c->ctx;
  delete c;
  ctx_unref(ctx);
}

uint32_t zgpu_chain_element_size(const zgpu_chain *c) { return c ? c->chain->es : 0; }

int zgpu_plan_create(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n, const uint64_t *out_shape,
                     uint32_t flags, zgpu_plan **out) {
  ABI_GUARD_BEGIN
  if (!ch || !out || !out_shape || (n && !descs)) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  if (!(flags & ZGPU_ENC_DEVICE)) return set_err(ZGPU_INVALID_ARGUMENT, "plans need device-resident inputs");
  HIPCHK(hipSetDevice(ch->ctx->device));
  LaneScope ls(ch->ctx);
  std::unique_ptr<zgpu_plan> P(plan_new(ch, nd, descs, n, out_shape, flags));
  plan_upload(*P, ls.L->stream);
  HIPCHK(hipStreamSynchronize(ls.L->stream));
  *out = P.release();
  return ZGPU_OK;
  ABI_GUARD_END
}

int zgpu_plan_execute(zgpu_plan *P, void *out, int32_t *status, void *stream) {
  ABI_GUARD_BEGIN
  if (!P || !out) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> lk(P->mu);
  HIPCHK(hipSetDevice(P->ctx->device));
  hipStream_t s = pick_stream(plan_lane(*P), stream);
  reset_call_state();
  plan_enqueue(*P, (uint8_t *)out, s);
  if (!status) return ZGPU_OK;
  return plan_statuses(*P, status, s);
  ABI_GUARD_END
}

int zgpu_plan_status(zgpu_plan *P, int32_t *status, void *stream) {
  ABI_GUARD_BEGIN
  if (!P) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> lk(P->mu);
  HIPCHK(hipSetDevice(P->ctx->device));
  const int rc = plan_statuses(*P, status, stream ? (hipStream_t)stream : plan_lane(*P)->stream);
  if (rc) set_err(rc, zgpu_status_name(rc));
  return rc;
  ABI_GUARD_END
}

void zgpu_plan_destroy(zgpu_plan *P) {
  if (!P) return;
  { std::lock_guard<std::mutex> lk(P->mu); }  // no execute of it still running on another thread
  delete P;
}

uint64_t zgpu_plan_algorithmic_bytes(const zgpu_plan *P) { return P ? P->alg_bytes_static + P->last_enc_bytes : 0; }

uint32_t zgpu_plan_counters(const zgpu_plan *P, uint64_t *out, uint32_t n) {
  if (!P || !out) return 0;
  const uint32_t k = std::min<uint32_t>(n, CTR_N);
  std::memcpy(out, P->last_counters, k * sizeof(uint64_t));
  return k;
}

int zgpu_last_size_mismatch(uint64_t *desc, uint64_t *len, uint64_t *expected_len) {
  if (!g_size_detail.valid) return 0;
  if (desc) *desc = g_size_detail.desc;
  if (len) *len = g_size_detail.len;
  if (expected_len) *expected_len = g_size_detail.expected;
  return 1;
}

uint32_t zgpu_last_counters(uint64_t *out, uint32_t n) {
  if (!out) return 0;
  const uint32_t k = std::min<uint32_t>(n, CTR_N);
  std::memcpy(out, g_last_counters, k * sizeof(uint64_t));
  return k;
}

// Host input and host output, both pinned, descriptors covering the whole output: the batch is cut
// into sub-batches of whole axis-0 row ranges (no descriptor straddles a cut), and sub-batch k's H2D
// (copy stream 0), decode (s) and D2H of its rows (copy stream 1) overlap with its neighbours' --
// PCIe is full duplex, so the host-to-host rate approaches the one-direction bound instead of half
// of it. Returns false (nothing done) when the batch does not cut into at least two sub-batches.
static bool decode_pipelined(zgpu_chain *ch, Lane *LN, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n,
                             uint8_t *out, const uint64_t *out_shape, uint32_t flags, int32_t *status, hipStream_t s,
                             int &rc) {
  constexpr uint64_t K = 16;  // target sub-batches
  zgpu_ctx *C = ch->ctx;
  uint64_t row_bytes = ch->chain->es;
  for (uint32_t d = 1; d < nd; d++) row_bytes *= out_shape[d];
  std::vector<uint64_t> ord(n);
  for (uint64_t i = 0; i < n; i++) ord[i] = i;
  std::sort(ord.begin(), ord.end(), [&](uint64_t a, uint64_t b) {
    return descs[a].out_start[0] != descs[b].out_start[0] ? descs[a].out_start[0] < descs[b].out_start[0] : a < b;
  });
  struct Group { uint64_t b, e, r0, r1; };
  std::vector<Group> groups;
  const uint64_t rows_per = std::max<uint64_t>(1, (out_shape[0] + K - 1) / K);
  uint64_t reach = 0, gb = 0, gr = 0;
  for (uint64_t k = 0; k < n; k++) {
    const zgpu_chunk_desc &d = descs[ord[k]];
    if (k > gb && d.out_start[0] >= reach && d.out_start[0] - gr >= rows_per) {
      groups.push_back(Group{gb, k, gr, d.out_start[0]});
      gb = k;
      gr = d.out_start[0];
    }
    reach = std::max<uint64_t>(reach, d.out_start[0] + d.sel_shape[0]);
  }
  if (groups.empty() || gr != groups.back().r1 || reach != out_shape[0]) return false;
  groups.push_back(Group{gb, n, gr, reach});
  if (groups.front().r0 != 0) return false;
  for (hipStream_t &cs : LN->copy)
    if (!cs) HIPCHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  // encoded bytes: per sub-batch, address-sorted and merged ranges in one device staging buffer
  std::vector<size_t> range_of(n, SIZE_MAX);  // descriptor -> its merged range in its sub-batch
  std::vector<std::vector<HostRange>> granges(groups.size());
  uint64_t total = 0;
  for (size_t g = 0; g < groups.size(); g++) {
    std::vector<uint64_t> idx(ord.begin() + groups[g].b, ord.begin() + groups[g].e);
    std::sort(idx.begin(), idx.end(),
              [&](uint64_t a, uint64_t b) { return (uintptr_t)descs[a].enc < (uintptr_t)descs[b].enc; });
    std::vector<HostRange> &R = granges[g];
    for (uint64_t i : idx) {
      if (!descs[i].enc || !descs[i].enc_len) continue;
      const uint8_t *p = (const uint8_t *)descs[i].enc;
      if (!R.empty() && p <= R.back().src + R.back().len) {
        HostRange &r = R.back();
        const uint64_t end = std::max<uint64_t>((uint64_t)(p - r.src) + descs[i].enc_len, r.len);
        total += end - r.len;
        r.len = end;
      } else {
        total = (total + 255) & ~(uint64_t)255;
        R.push_back(HostRange{p, descs[i].enc_len, total});
        total += descs[i].enc_len;
      }
      range_of[i] = R.size() - 1;
    }
  }
  uint8_t *enc_dev = (uint8_t *)C->dev_alloc(total ? total : 1);
  uint8_t *dout = (uint8_t *)C->dev_alloc(out_shape[0] * row_bytes);
  std::vector<hipEvent_t> ev(2 * groups.size(), nullptr);
  std::vector<std::unique_ptr<zgpu_plan>> plans(groups.size());
  auto cleanup = [&]() {
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    C->dev_free(enc_dev);
    C->dev_free(dout);
  };
  try {
    for (hipEvent_t &e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (size_t g = 0; g < groups.size(); g++) {
      const Group &G = groups[g];
      for (const HostRange &r : granges[g])
        HIPCHK(hipMemcpyAsync(enc_dev + r.dev_off, r.src, r.len, hipMemcpyHostToDevice, LN->copy[0]));
      HIPCHK(hipEventRecord(ev[2 * g], LN->copy[0]));
      std::vector<zgpu_chunk_desc> gd;
      gd.reserve(G.e - G.b);
      for (uint64_t k = G.b; k < G.e; k++) {
        const uint64_t i = ord[k];
        zgpu_chunk_desc d = descs[i];
        const size_t r = range_of[i];
        if (r != SIZE_MAX) {
          const HostRange &hr = granges[g][r];
          d.enc = enc_dev + hr.dev_off + ((const uint8_t *)descs[i].enc - hr.src);
        } else {
          d.enc = nullptr;
        }
        gd.push_back(d);
      }
      plans[g].reset(plan_new(ch, nd, gd.data(), gd.size(), out_shape, flags | ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE));
      plan_upload(*plans[g], s);
      HIPCHK(hipStreamWaitEvent(s, ev[2 * g], 0));
      plan_enqueue(*plans[g], dout, s);
      HIPCHK(hipEventRecord(ev[2 * g + 1], s));
      HIPCHK(hipStreamWaitEvent(LN->copy[1], ev[2 * g + 1], 0));
      HIPCHK(hipMemcpyAsync(out + G.r0 * row_bytes, dout + G.r0 * row_bytes, (G.r1 - G.r0) * row_bytes,
                            hipMemcpyDeviceToHost, LN->copy[1]));
    }
    std::vector<int32_t> all(n, 0);
    for (size_t g = 0; g < groups.size(); g++) {
      const Group &G = groups[g];
      std::vector<int32_t> st(G.e - G.b, 0);
      plan_statuses(*plans[g], st.data(), s);
      for (uint64_t k = G.b; k < G.e; k++) all[ord[k]] = st[k - G.b];
    }
    rc = 0;  // the first failing descriptor in the caller's order
    for (uint64_t i = 0; i < n; i++) {
      if (status) status[i] = all[i];
      if (!rc) rc = all[i];
    }
    HIPCHK(hipStreamSynchronize(LN->copy[1]));
  } catch (...) {
    (void)hipDeviceSynchronize();
    plans.clear();
    cleanup();
    throw;
  }
  plans.clear();
  cleanup();
  return true;
}

}  // extern "C"

// Host inputs -> one device staging buffer: chunks sorted by address and touching / overlapping ones
// merged into ranges; pinned ranges are DMA'd directly (one copy per range), pageable ones through
// the pinned staging slabs. local[i].enc is rewritten to descriptor i's device copy.
struct HostStage {
  zgpu_ctx *C;
  uint8_t *enc = nullptr, *pin = nullptr;
  static constexpr uint64_t slab = 64ull << 20;
  explicit HostStage(zgpu_ctx *c) : C(c) {}
  ~HostStage() {
    C->dev_free(enc);
    C->host_free(pin);
  }
  uint8_t *stage() {  // 2 slabs of pinned staging, only for pageable host buffers
    if (!pin) pin = (uint8_t *)C->host_alloc(2 * slab);
    return pin;
  }
  HostStage(const HostStage &) = delete;
  HostStage &operator=(const HostStage &) = delete;
};

static void stage_host_inputs(HostStage &H, const zgpu_chunk_desc *descs, uint64_t n,
                              std::vector<zgpu_chunk_desc> &local, hipStream_t s) {
  local.assign(descs, descs + n);
  std::vector<uint64_t> order;
  for (uint64_t i = 0; i < n; i++)
    if (descs[i].enc && descs[i].enc_len) order.push_back(i);
  std::sort(order.begin(), order.end(),
            [&](uint64_t a, uint64_t b) { return (uintptr_t)descs[a].enc < (uintptr_t)descs[b].enc; });
  std::vector<HostRange> ranges;
  std::vector<uint64_t> range_of(n, 0);
  uint64_t total = 0;
  for (uint64_t i : order) {
    const uint8_t *p = (const uint8_t *)descs[i].enc;
    if (!ranges.empty() && p <= ranges.back().src + ranges.back().len) {
      HostRange &r = ranges.back();
      const uint64_t end = std::max<uint64_t>((uint64_t)(p - r.src) + descs[i].enc_len, r.len);
      total += end - r.len;
      r.len = end;
    } else {
      total = (total + 255) & ~(uint64_t)255;
      ranges.push_back(HostRange{p, descs[i].enc_len, total});
      total += descs[i].enc_len;
    }
    range_of[i] = ranges.size() - 1;
  }
  if (!total) return;
  H.enc = (uint8_t *)H.C->dev_alloc(total);
  bool pinned = true;
  for (const HostRange &r : ranges)
    if (!host_is_pinned(r.src) || !host_is_pinned(r.src + r.len - 1)) {
      pinned = false;
      break;
    }
  HIPCHK(h2d_ranges(H.enc, ranges, pinned, pinned ? nullptr : H.stage(), HostStage::slab, host_copy_threads(), s));
  for (uint64_t i : order) {
    const HostRange &r = ranges[range_of[i]];
    local[i].enc = H.enc + r.dev_off + ((const uint8_t *)descs[i].enc - r.src);
  }
}

static uint64_t covered_volume(const zgpu_chunk_desc *descs, uint64_t n, uint32_t nd) {
  uint64_t covered = 0;
  for (uint64_t i = 0; i < n; i++) covered += sel_volume(descs[i], nd);
  return covered;
}

static uint64_t volume(const uint64_t *shape, uint32_t nd) {
  uint64_t v = 1;
  for (uint32_t d = 0; d < nd; d++) v *= shape[d];
  return v;
}

// Device-side decode of descriptors whose encoded bytes are on the device into dout (out_shape):
// the general decode, per-descriptor statuses, first failing descriptor as the return value.
static int decode_device(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *dd, uint64_t n, uint8_t *dout,
                         const uint64_t *out_shape, uint32_t flags, int32_t *status, hipStream_t s) {
  GeneralCall G{ch->ctx, ch->validate && !(flags & ZGPU_NO_VALIDATE), nd, dout, out_shape,
                flags | ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE, s, {}};
  std::vector<int32_t> st(n, 0);
  decode_general(G, ch->chain, dd, n, st.data());
  int rc = 0;
  for (uint64_t i = 0; i < n; i++) {
    if (status) status[i] = st[i];
    if (!rc) rc = st[i];
  }
  return rc;
}

// zgpu_decode_batch / zgpu_decode_into on one lane (LN, stream s): every output form.
static int decode_call(zgpu_chain *ch, Lane *LN, hipStream_t s, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n,
                       const zgpu_out_view &V, uint32_t flags, int32_t *status) {
  zgpu_ctx *C = ch->ctx;
  const uint32_t es = ch->chain->es;
  const bool whole = box_is_whole(nd, V.array_shape, V.start, V.shape);
  const uint64_t out_elems = volume(V.shape, nd);
  const bool fused = fused_plannable(*ch->chain) && uniform_shapes(descs, n, nd);
  if (!(flags & ZGPU_ENC_DEVICE) && !(flags & ZGPU_OUT_DEVICE) && n >= 2 && fused && whole) {
    // pinned host in and out, full coverage: the overlapped sub-batch pipeline
    const uint64_t out_b = out_elems * es;
    bool pinned = out_b && host_is_pinned(V.base) && host_is_pinned((const uint8_t *)V.base + out_b - 1);
    for (uint64_t i = 0; i < n && pinned; i++) {
      const uint8_t *e = (const uint8_t *)descs[i].enc;
      if (e && descs[i].enc_len && (!host_is_pinned(e) || !host_is_pinned(e + descs[i].enc_len - 1))) pinned = false;
    }
    int rc = 0;
    if (pinned && covered_volume(descs, n, nd) == out_elems &&
        decode_pipelined(ch, LN, nd, descs, n, (uint8_t *)V.base, V.shape, flags, status, s, rc))
      return rc;
  }
  HostStage H(C);
  std::vector<zgpu_chunk_desc> local;
  const zgpu_chunk_desc *dd = descs;
  if (!(flags & ZGPU_ENC_DEVICE)) {
    stage_host_inputs(H, descs, n, local, s);
    dd = local.data();
  }
  if (flags & ZGPU_OUT_DEVICE) {
    if (whole) return decode_device(ch, nd, dd, n, (uint8_t *)V.base, V.shape, flags, status, s);
    // a window of a device array: decoded in place through the whole array's strides (descriptors
    // shifted by the window origin; one outside its window fails alone, as it would against out_shape)
    std::vector<zgpu_chunk_desc> sub;
    std::vector<uint64_t> owner;
    std::vector<int32_t> st(n, 0);
    for (uint64_t i = 0; i < n; i++) {
      if (!desc_geometry_ok(dd[i], nd, V.shape)) {
        st[i] = ZGPU_INVALID_ARGUMENT;
        continue;
      }
      zgpu_chunk_desc d = dd[i];
      for (uint32_t k = 0; k < nd; k++) d.out_start[k] += V.start[k];
      sub.push_back(d);
      owner.push_back(i);
    }
    std::vector<int32_t> sst(sub.size(), 0);
    decode_device(ch, nd, sub.data(), sub.size(), (uint8_t *)V.base, V.array_shape, flags, sst.data(), s);
    if (g_size_detail.valid) g_size_detail.desc = owner[g_size_detail.desc];
    for (size_t k = 0; k < sub.size(); k++) st[owner[k]] = sst[k];
    int rc = 0;
    for (uint64_t i = 0; i < n; i++) {
      if (status) status[i] = st[i];
      if (!rc) rc = st[i];
    }
    return rc;
  }
  // host output: decoded into a compact device copy of the window, copied back box-wise; parts of the
  // window no descriptor covers keep the caller's bytes (the regions are disjoint,
  // ArrayBytesFixedDisjointView, so equal volumes mean full coverage and no upload)
  const uint64_t out_bytes = out_elems * es;
  uint8_t *dout = (uint8_t *)C->dev_alloc(out_bytes ? out_bytes : 1);
  const BoxRuns R = box_runs(nd, V.array_shape, V.start, V.shape, es);
  int rc = 0;
  try {
    if (covered_volume(descs, n, nd) != out_elems)
      HIPCHK(h2d_box(R, dout, (const uint8_t *)V.base, H.stage(), HostStage::slab, host_copy_threads(), s));
    rc = decode_device(ch, nd, dd, n, dout, V.shape, flags, status, s);
    HIPCHK(d2h_box(R, (uint8_t *)V.base, dout, H.stage(), HostStage::slab, host_copy_threads(), s));
  } catch (...) {
    C->dev_free(dout);
    throw;
  }
  C->dev_free(dout);
  return rc;
}

// ------------------------------------------------------------------------------------------------
// Coalescing of concurrent host-in / host-out calls (ZGPU_COALESCE). zarrs' read path calls the codec
// once per shard (or chunk) from each rayon worker (array_read_ops_common.rs:173-176,
// sharding_codec.rs:617-707), and one shard's inner chunks fill a few percent of the GPU's decode
// waves. Calls on one chain that arrive within the collect window become ONE batch: the first caller
// (the batch's leader) waits for the window to close (or the batch to fill), stacks every caller's
// window along axis 0 of one device output (trailing axes padded to the largest), uploads all
// encoded bytes in one packed H2D, decodes everything in one launch sequence, packs the windows
// compactly on the device (k_box_copy) and copies them back in one D2H into pinned memory. Every
// caller then places its own window's rows into its host array (in parallel) and returns its own
// statuses. Batches of one context run concurrently, each on a lane of its own.
// ------------------------------------------------------------------------------------------------
struct CoCall {
  zgpu_chain *ch;
  uint32_t nd;
  const zgpu_chunk_desc *descs;
  uint64_t n;
  zgpu_out_view V;
  uint32_t flags;
  int32_t *status;
  uint64_t enc_bytes = 0;
  // results, set by the leader
  bool done = false, call_error = false;  // call_error: the batch failed as a whole (rc, err)
  int rc = 0;
  std::string err;
  SizeDetail sd;
  uint64_t pack_off = 0;  // byte offset of this caller's compact window in the batch's host pack
};

struct CoBatch {
  zgpu_ctx *C = nullptr;
  std::vector<CoCall *> calls;
  uint64_t bytes = 0;
  bool closed = false;
  std::condition_variable cv;
  uint8_t *pack = nullptr;  // pinned: every caller's window, compact, back to back
  uint64_t id = 0;          // trace id
  ~CoBatch() {
    if (pack) C->host_free(pack);
  }
};

struct CoKey {
  zgpu_chain *ch;
  uint32_t flags, nd;
  bool operator<(const CoKey &o) const {
    return ch != o.ch ? ch < o.ch : flags != o.flags ? flags < o.flags : nd < o.nd;
  }
};

struct Coalescer {
  std::mutex mu;
  std::map<CoKey, std::shared_ptr<CoBatch>> open;
  uint32_t window_us = 200, max_calls = 8;
  uint64_t max_bytes = 1ull << 30;
  uint64_t batches = 0, calls = 0, seq = 0;
  uint64_t active = 0;  // coalescable calls inside coalesced_call (under mu)
  // Batches decoding at once (under mu): a leader waits for a slot while its batch keeps taking
  // joiners. Each batch is a synchronous H2D -> decode -> D2H chain on its lane; with more of them than
  // the process's HIP hardware queues (4 by default) their kernels queue behind each other, and a few
  // larger batches fill the GPU better (drop-in sweep, profiles/r05/r05d8_dropin_rect_pack_inflight_cap.txt).
  uint32_t max_inflight = 3, inflight = 0;
  std::condition_variable slot_cv;
};

// ZGPU_TRACE=1: one stderr line per coalesced-batch phase (microseconds since the first trace)
static bool co_tracing() {
  static const bool on = [] {
    const char *e = std::getenv("ZGPU_TRACE");
    return e && std::atoi(e) != 0;
  }();
  return on;
}
static void co_trace(const char *what, uint64_t batch, uint64_t a = 0, uint64_t b = 0) {
  if (!co_tracing()) return;
  static const auto t0 = std::chrono::steady_clock::now();
  const long long us =
      std::chrono::duration_cast<std::chrono::microseconds>(std::chrono::steady_clock::now() - t0).count();
  std::fprintf(stderr, "[zgpu-trace] %lld %s %llu %llu %llu\n", us, what, (unsigned long long)batch,
               (unsigned long long)a, (unsigned long long)b);
}

static Coalescer &coalescer(zgpu_ctx *C) {
  std::lock_guard<std::mutex> lk(C->mu);
  if (!C->co) {
    C->co = new Coalescer();
    if (const char *e = std::getenv("ZGPU_COALESCE_US")) C->co->window_us = (uint32_t)std::max(0, std::atoi(e));
    if (const char *e = std::getenv("ZGPU_COALESCE_CALLS")) C->co->max_calls = (uint32_t)std::max(1, std::atoi(e));
    if (const char *e = std::getenv("ZGPU_COALESCE_BYTES")) C->co->max_bytes = std::strtoull(e, nullptr, 10);
    if (const char *e = std::getenv("ZGPU_CO_INFLIGHT")) C->co->max_inflight = (uint32_t)std::max(1, std::atoi(e));
  }
  return *C->co;
}

// The leader's work: one decode of every caller's descriptors; fills each call's results and the
// batch's host pack.
static void co_run(CoBatch &B, Lane *LN) {
  zgpu_ctx *C = B.C;
  CoCall &c0 = *B.calls[0];
  zgpu_chain *ch = c0.ch;
  const uint32_t nd = c0.nd, es = ch->chain->es;
  HIPCHK(hipSetDevice(C->device));
  hipStream_t s = pick_stream(LN, nullptr);
  // stacked output: caller k's window at rows [row0[k], row0[k] + V.shape[0]) of axis 0
  uint64_t stacked[ZG_MAXD] = {0};
  std::vector<uint64_t> row0(B.calls.size());
  for (size_t k = 0; k < B.calls.size(); k++) {
    const zgpu_out_view &V = B.calls[k]->V;
    row0[k] = stacked[0];
    stacked[0] += V.shape[0];
    for (uint32_t d = 1; d < nd; d++) stacked[d] = std::max(stacked[d], V.shape[d]);
  }
  std::vector<zgpu_chunk_desc> all;
  std::vector<std::pair<uint32_t, uint64_t>> owner;  // (call, descriptor)
  std::vector<std::vector<int32_t>> st(B.calls.size());
  for (size_t k = 0; k < B.calls.size(); k++) {
    CoCall &c = *B.calls[k];
    st[k].assign(c.n, 0);
    for (uint64_t i = 0; i < c.n; i++) {
      if (!desc_geometry_ok(c.descs[i], nd, c.V.shape)) {
        st[k][i] = ZGPU_INVALID_ARGUMENT;
        continue;
      }
      zgpu_chunk_desc d = c.descs[i];
      d.out_start[0] += row0[k];
      all.push_back(d);
      owner.push_back({(uint32_t)k, i});
    }
  }
  HostStage H(C);
  std::vector<zgpu_chunk_desc> local;
  co_trace("batch-start", B.id, B.calls.size(), all.size());
  stage_host_inputs(H, all.data(), all.size(), local, s);
  co_trace("h2d-done", B.id);
  uint64_t row_elems = 1;
  for (uint32_t d = 1; d < nd; d++) row_elems *= stacked[d];
  const uint64_t stacked_bytes = stacked[0] * row_elems * es;
  uint64_t pack_bytes = 0;
  for (CoCall *c : B.calls) {
    c->pack_off = pack_bytes;
    pack_bytes += volume(c->V.shape, nd) * es;
  }
  uint8_t *dout = (uint8_t *)C->dev_alloc(stacked_bytes ? stacked_bytes : 1);
  uint8_t *dpack = nullptr;
  try {
    std::vector<int32_t> ast(all.size(), 0);
    decode_device(ch, nd, local.data(), local.size(), dout, stacked, c0.flags, ast.data(), s);
    co_trace("decode-done", B.id);
    const SizeDetail sd = g_size_detail;
    for (size_t j = 0; j < all.size(); j++) st[owner[j].first][owner[j].second] = ast[j];
    if (sd.valid && sd.desc < owner.size()) {
      CoCall &c = *B.calls[owner[sd.desc].first];
      c.sd = sd;
      c.sd.desc = owner[sd.desc].second;
    }
    // The pack kernels and the D2H run on a high-priority stream: the other lanes' decodes hold the
    // CUs with long-running waves, and a normal-priority pack kernel queued behind them waited for
    // their slots (trace: 60 MB packs taking 20+ ms). ZGPU_CO_HIPRIO=0: the lane's own stream.
    static const bool hiprio = [] {
      const char *e = std::getenv("ZGPU_CO_HIPRIO");
      return !e || std::atoi(e) != 0;
    }();
    if (hiprio) {
      if (!LN->out_hi) {
        int least = 0, greatest = 0;
        HIPCHK(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIPCHK(hipStreamCreateWithPriority(&LN->out_hi, hipStreamNonBlocking, greatest));
      }
      HIPCHK(hipStreamSynchronize(s));  // (decode_device has read its statuses back: a no-op)
      s = LN->out_hi;
    }
    // pack: a window whose trailing extents are the stacked ones is already compact in place
    bool compact = true;
    for (CoCall *c : B.calls)
      for (uint32_t d = 1; d < nd; d++)
        if (c->V.shape[d] != stacked[d]) compact = false;
    std::vector<BoxRuns> boxes;
    bool rect = false;  // every window a 3-D box: packed by the copy engines, no kernel
    if (!compact) {
      static const bool rect_on = [] {
        const char *e = std::getenv("ZGPU_CO_PACK_RECT");
        return !e || std::atoi(e) != 0;
      }();
      rect = rect_on;
      for (size_t k = 0; k < B.calls.size(); k++) {
        uint64_t org[ZG_MAXD] = {0};
        org[0] = row0[k];
        boxes.push_back(box_runs(nd, stacked, org, B.calls[k]->V.shape, es));
        if (boxes.back().outer > 2) rect = false;
      }
    }
    // power-of-two size classes (>= 64 MiB): batches of varying size reuse pooled pinned buffers
    // instead of page-locking new ones
    if (compact || rect) co_trace("packed", B.id, compact ? 0 : 2);
    uint64_t cls = 64ull << 20;
    while (cls < pack_bytes) cls <<= 1;
    B.pack = (uint8_t *)C->host_alloc(cls);
    co_trace("pack-alloc", B.id);
    if (compact) {
      if (pack_bytes) HIPCHK(hipMemcpyAsync(B.pack, dout, pack_bytes, hipMemcpyDeviceToHost, s));
    } else if (rect) {
      // Each caller's window straight from the stacked output into its place in the pinned pack as
      // one pitched 3-D copy (DMA): a box-copy kernel queued while other lanes' decode waves hold the
      // CUs waited for their slots (trace: pack median 5 ms at 8 lanes, 20 ms at 2 lanes with bigger
      // batches), and the copy engines need none.
      for (size_t k = 0; k < B.calls.size(); k++) {
        const BoxRuns &R = boxes[k];
        if (!R.n_runs) continue;
        const uint64_t w = R.run_bytes;
        const uint64_t h = R.outer >= 1 ? R.shape[R.outer - 1] : 1, depth = R.outer >= 2 ? R.shape[0] : 1;
        const uint64_t pitch = R.outer >= 1 ? R.stride[R.outer - 1] : w;
        const uint64_t sy = R.outer >= 2 ? R.stride[0] / pitch : h;
        hipMemcpy3DParms p3{};
        p3.srcPtr = make_hipPitchedPtr(dout + R.base, pitch, w, sy);
        p3.dstPtr = make_hipPitchedPtr(B.pack + B.calls[k]->pack_off, w, w, h);
        p3.extent = make_hipExtent(w, h, depth);
        p3.kind = hipMemcpyDeviceToHost;
        HIPCHK(hipMemcpy3DAsync(&p3, s));
      }
    } else {
      dpack = (uint8_t *)C->dev_alloc(pack_bytes ? pack_bytes : 1);
      for (size_t k = 0; k < B.calls.size(); k++) {
        const BoxRuns &R = boxes[k];
        ZgBoxCopy P{};
        P.outer = R.outer;
        for (uint32_t d = 0; d < R.outer; d++) {
          P.shape[d] = R.shape[d];
          P.src_stride[d] = R.stride[d];
        }
        uint64_t cs = R.run_bytes;  // compact strides of the outer axes
        for (int d = (int)R.outer - 1; d >= 0; d--) {
          P.dst_stride[d] = cs;
          cs *= R.shape[d];
        }
        P.src_base = R.base;
        P.dst_base = B.calls[k]->pack_off;
        P.run_bytes = R.run_bytes;
        P.n_runs = R.n_runs;
        HIPCHK(launch_box_copy(dout, dpack, P, s));
      }
      if (co_tracing()) {
        HIPCHK(hipStreamSynchronize(s));
        co_trace("packed", B.id, 1);
      }
      if (pack_bytes) HIPCHK(hipMemcpyAsync(B.pack, dpack, pack_bytes, hipMemcpyDeviceToHost, s));
    }
    HIPCHK(hipStreamSynchronize(s));
    co_trace("d2h-done", B.id, pack_bytes);
  } catch (...) {
    C->dev_free(dout);
    C->dev_free(dpack);
    throw;
  }
  C->dev_free(dout);
  C->dev_free(dpack);
  for (size_t k = 0; k < B.calls.size(); k++) {
    CoCall &c = *B.calls[k];
    c.rc = 0;
    for (uint64_t i = 0; i < c.n; i++) {
      if (c.status) c.status[i] = st[k][i];
      if (!c.rc) c.rc = st[k][i];
    }
  }
}

// A caller's encoded bytes copied into pinned memory by the caller's own thread before it joins a
// batch: a batch's callers pack their inputs in parallel (each on its own thread, overlapping the
// other lanes' GPU work) and the leader's upload is one DMA per contiguous range, instead of the
// leader staging every caller's pageable bytes itself. Ranges (descriptors sorted by address, touching
// ones merged) are placed back to back; local[i].enc points into the pinned copy. Returns nullptr
// (local untouched) when there is nothing to copy or the bytes are pinned already.
static uint8_t *pin_caller_inputs(zgpu_ctx *C, const zgpu_chunk_desc *descs, uint64_t n,
                                  std::vector<zgpu_chunk_desc> &local) {
  std::vector<uint64_t> order;
  for (uint64_t i = 0; i < n; i++)
    if (descs[i].enc && descs[i].enc_len) order.push_back(i);
  if (order.empty()) return nullptr;
  std::sort(order.begin(), order.end(),
            [&](uint64_t a, uint64_t b) { return (uintptr_t)descs[a].enc < (uintptr_t)descs[b].enc; });
  std::vector<HostRange> ranges;
  std::vector<uint64_t> range_of(n, 0);
  uint64_t total = 0;
  for (uint64_t i : order) {
    const uint8_t *p = (const uint8_t *)descs[i].enc;
    if (!ranges.empty() && p <= ranges.back().src + ranges.back().len) {
      HostRange &r = ranges.back();
      const uint64_t end = std::max<uint64_t>((uint64_t)(p - r.src) + descs[i].enc_len, r.len);
      total += end - r.len;
      r.len = end;
    } else {
      ranges.push_back(HostRange{p, descs[i].enc_len, total});
      total += descs[i].enc_len;
    }
    range_of[i] = ranges.size() - 1;
  }
  bool pinned = true;
  for (const HostRange &r : ranges)
    if (!host_is_pinned(r.src) || !host_is_pinned(r.src + r.len - 1)) {
      pinned = false;
      break;
    }
  if (pinned) return nullptr;
  uint64_t cls = 4ull << 20;  // power-of-two classes: the pooled buffers are reused call after call
  while (cls < total) cls <<= 1;
  uint8_t *pin = (uint8_t *)C->host_alloc(cls);
  std::vector<uint8_t *> d;
  std::vector<const uint8_t *> sp;
  std::vector<uint64_t> ln;
  for (const HostRange &r : ranges) {
    d.push_back(pin + r.dev_off);
    sp.push_back(r.src);
    ln.push_back(r.len);
  }
  parallel_memcpy(d, sp, ln, 2);
  local.assign(descs, descs + n);
  for (uint64_t i : order) {
    const HostRange &r = ranges[range_of[i]];
    local[i].enc = pin + r.dev_off + ((const uint8_t *)descs[i].enc - r.src);
  }
  return pin;
}

// zgpu_decode_pinned's result: a pooled pinned buffer of the context, or a slice of a coalesced
// batch's pack (the batch, and with it the pack, lives until every caller released its result)
struct zgpu_result {
  zgpu_ctx *ctx = nullptr;
  uint8_t *own = nullptr;             // pooled pinned buffer (uncoalesced call)
  std::shared_ptr<CoBatch> batch;     // coalesced call: the batch holding the pack
  ~zgpu_result() {
    if (own) ctx->host_free(own);
    batch.reset();
    ctx_unref(ctx);
  }
};

static int coalesced_call(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n,
                          const zgpu_out_view &V, uint32_t flags, int32_t *status,
                          zgpu_result **keep = nullptr, const void **keep_data = nullptr) {
  zgpu_ctx *C = ch->ctx;
  Coalescer &K = coalescer(C);
  static const bool pin_in = [] {
    const char *e = std::getenv("ZGPU_CO_PIN");
    return !e || std::atoi(e) != 0;
  }();
  std::vector<zgpu_chunk_desc> pinned_descs;
  struct PinGuard {
    zgpu_ctx *C;
    uint8_t *p;
    ~PinGuard() { C->host_free(p); }
  } pin{C, pin_in ? pin_caller_inputs(C, descs, n, pinned_descs) : nullptr};
  co_trace("pinned", 0, pin.p ? 1 : 0);
  if (pin.p) descs = pinned_descs.data();
  CoCall me{ch, nd, descs, n, V, flags, status};
  for (uint64_t i = 0; i < n; i++)
    if (descs[i].enc) me.enc_bytes += descs[i].enc_len;
  const CoKey key{ch, flags, nd};
  std::shared_ptr<CoBatch> B;
  bool leader = false;
  std::unique_lock<std::mutex> lk(K.mu);
  K.active++;  // left below, once this call's batch is done (the lock is held there)
  auto it = K.open.find(key);
  if (it == K.open.end()) {
    B = std::make_shared<CoBatch>();
    B->C = C;
    B->id = ++K.seq;
    K.open[key] = B;
    leader = true;
  } else {
    B = it->second;
  }
  B->calls.push_back(&me);
  B->bytes += me.enc_bytes;
  co_trace(leader ? "arrive-lead" : "arrive-join", B->id, me.enc_bytes);
  auto close = [&]() {
    B->closed = true;
    auto jt = K.open.find(key);
    if (jt != K.open.end() && jt->second == B) K.open.erase(jt);
  };
  if (B->calls.size() >= K.max_calls || B->bytes >= K.max_bytes) {
    close();
    B->cv.notify_all();
  }
  if (leader) {
    // the batch takes joiners for the collect window, and then for as long as its leader waits for a
    // free lane: under load (every lane decoding an earlier batch) batches grow by themselves. A lone
    // caller (no other coalescable call in flight on the context) does not wait: a single-threaded
    // reader pays no collect window per chunk.
    if (K.active > 1)
      B->cv.wait_until(lk, std::chrono::steady_clock::now() + std::chrono::microseconds(K.window_us),
                       [&] { return B->closed; });
    K.slot_cv.wait(lk, [&] { return K.inflight < K.max_inflight; });
    K.inflight++;
    lk.unlock();
    int rc = 0;
    std::string err;
    Lane *LN = nullptr;
    try {
      HIPCHK(hipSetDevice(C->device));
      LN = C->acquire_lane();
    } catch (const HipFail &e) {
      rc = ZGPU_HIP_ERROR;
      err = std::string(e.what) + ": " + hipGetErrorString(e.e);
    }
    co_trace("lane", B->id);
    lk.lock();
    if (!B->closed) close();
    K.batches++;
    K.calls += B->calls.size();
    lk.unlock();
    if (!rc) try {
      co_run(*B, LN);
    } catch (const ChainError &e) {
      rc = e.status;
      err = e.msg;
    } catch (const HipFail &e) {
      rc = ZGPU_HIP_ERROR;
      err = std::string(e.what) + ": " + hipGetErrorString(e.e);
    } catch (const std::exception &e) {
      rc = ZGPU_INVALID_ARGUMENT;
      err = e.what();
    }
    if (LN) C->release_lane(LN);
    lk.lock();
    K.inflight--;
    K.slot_cv.notify_one();
    for (CoCall *c : B->calls) {
      if (rc) {
        c->rc = rc;
        c->err = err;
        c->call_error = true;
        c->sd = SizeDetail{};
      }
      c->done = true;
    }
    B->cv.notify_all();
  } else {
    B->cv.wait(lk, [&] { return me.done; });
  }
  K.active--;
  lk.unlock();
  g_size_detail = me.sd;
  if (me.call_error) return set_err(me.rc, me.err);
  if (keep) {  // zgpu_decode_pinned: the caller copies its compact window out of the pack itself
    auto *R = new zgpu_result();
    ctx_ref(C);
    R->ctx = C;
    R->batch = B;
    *keep = R;
    *keep_data = B->pack + me.pack_off;
    if (me.rc) set_err(me.rc, zgpu_status_name(me.rc));
    return me.rc;
  }
  // this caller's window: its rows placed from the pinned pack by this caller's own thread (the
  // batch's callers do this in parallel)
  const BoxRuns R = box_runs(nd, V.array_shape, V.start, V.shape, ch->chain->es);
  const uint64_t nb = R.n_runs * R.run_bytes;
  // the batch's callers place their rows concurrently; each takes its share of the copy threads
  const int share = std::max<int>(1, host_copy_threads() / (int)std::max<size_t>(1, B->calls.size()));
  copy_box_runs(R, (uint8_t *)V.base, B->pack + me.pack_off, 0, nb, true, std::min(share, 4));
  co_trace("copied-out", B->id, nb);
  if (me.rc) set_err(me.rc, zgpu_status_name(me.rc));
  return me.rc;
}

static int decode_entry(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n,
                        const zgpu_out_view &V, uint32_t flags, int32_t *status, void *stream) {
  zgpu_ctx *C = ch->ctx;
  for (uint32_t d = 0; d < nd; d++)
    if (V.start[d] + V.shape[d] > V.array_shape[d]) return set_err(ZGPU_INVALID_ARGUMENT, "view outside its array");
  HIPCHK(hipSetDevice(C->device));
  reset_call_state();
  if ((flags & ZGPU_COALESCE) && !(flags & (ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE)) && n &&
      covered_volume(descs, n, nd) == volume(V.shape, nd))
    return coalesced_call(ch, nd, descs, n, V, flags & ~ZGPU_COALESCE, status);
  LaneScope ls(C);
  hipStream_t s = pick_stream(ls.L, stream);
  const int rc = decode_call(ch, ls.L, s, nd, descs, n, V, flags & ~ZGPU_COALESCE, status);
  if (rc) set_err(rc, zgpu_status_name(rc));
  return rc;
}

static void delete_coalescer(Coalescer *co) { delete co; }

extern "C" {

int zgpu_decode_pinned(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n, const uint64_t *out_shape,
                       uint32_t flags, int32_t *status, const void **data, zgpu_result **result) {
  ABI_GUARD_BEGIN
  if (data) *data = nullptr;
  if (result) *result = nullptr;
  if (!ch || !out_shape || (n && !descs) || !data || !result) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  if (flags & (ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE))
    return set_err(ZGPU_INVALID_ARGUMENT, "zgpu_decode_pinned takes host inputs and returns host memory");
  zgpu_ctx *C = ch->ctx;
  HIPCHK(hipSetDevice(C->device));
  reset_call_state();
  const uint64_t bytes = volume(out_shape, nd) * ch->chain->es;
  if ((flags & ZGPU_COALESCE) && n && covered_volume(descs, n, nd) == volume(out_shape, nd)) {
    zgpu_out_view V{};
    V.base = nullptr;  // never written: the result stays in the pack
    for (uint32_t d = 0; d < nd; d++) V.array_shape[d] = V.shape[d] = out_shape[d];
    zgpu_result *R = nullptr;
    const void *p = nullptr;
    const int rc = coalesced_call(ch, nd, descs, n, V, flags & ~ZGPU_COALESCE, status, &R, &p);
    if (rc) {
      delete R;
      return rc;
    }
    *result = R;
    *data = p;
    return ZGPU_OK;
  }
  // one call: its own pooled pinned buffer (pinned host output takes the overlapped D2H paths)
  std::unique_ptr<zgpu_result> R(new zgpu_result());
  ctx_ref(C);
  R->ctx = C;
  R->own = (uint8_t *)C->host_alloc(bytes ? bytes : 1);
  zgpu_out_view V{};
  V.base = R->own;
  for (uint32_t d = 0; d < nd; d++) V.array_shape[d] = V.shape[d] = out_shape[d];
  if (covered_volume(descs, n, nd) != volume(out_shape, nd) && bytes)  // parts no descriptor covers: zero
    std::memset(R->own, 0, bytes);
  LaneScope ls(C);
  hipStream_t s = pick_stream(ls.L, nullptr);
  const int rc = decode_call(ch, ls.L, s, nd, descs, n, V, flags & ~ZGPU_COALESCE, status);
  if (rc) return set_err(rc, zgpu_status_name(rc));
  *data = R->own;
  *result = R.release();
  return ZGPU_OK;
  ABI_GUARD_END
}

void zgpu_result_release(zgpu_result *r) { delete r; }

int zgpu_decode_batch(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n, void *out,
                      const uint64_t *out_shape, uint32_t flags, int32_t *status, void *stream) {
  ABI_GUARD_BEGIN
  if (!ch || !out_shape || (n && !descs) || !out) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  zgpu_out_view V{};
  V.base = out;
  for (uint32_t d = 0; d < nd; d++) V.array_shape[d] = V.shape[d] = out_shape[d];
  return decode_entry(ch, nd, descs, n, V, flags, status, stream);
  ABI_GUARD_END
}

int zgpu_decode_into(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *descs, uint64_t n, const zgpu_out_view *view,
                     uint32_t flags, int32_t *status, void *stream) {
  ABI_GUARD_BEGIN
  if (!ch || !view || (n && !descs) || !view->base) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  return decode_entry(ch, nd, descs, n, *view, flags, status, stream);
  ABI_GUARD_END
}

int zgpu_ctx_set_coalescing(zgpu_ctx *ctx, uint32_t window_us, uint32_t max_calls, uint64_t max_bytes) {
  if (!ctx) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  Coalescer &K = coalescer(ctx);
  std::lock_guard<std::mutex> lk(K.mu);
  K.window_us = window_us;
  K.max_calls = std::max<uint32_t>(1, max_calls);
  K.max_bytes = max_bytes ? max_bytes : UINT64_MAX;
  return ZGPU_OK;
}

int zgpu_ctx_coalescing_stats(const zgpu_ctx *ctx, uint64_t *batches, uint64_t *calls) {
  if (!ctx) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  Coalescer &K = coalescer(const_cast<zgpu_ctx *>(ctx));
  std::lock_guard<std::mutex> lk(K.mu);
  if (batches) *batches = K.batches;
  if (calls) *calls = K.calls;
  return ZGPU_OK;
}

int zgpu_retrieve_array_subset(zgpu_chain *ch, uint32_t nd, const uint64_t *array_shape, const uint64_t *chunk_shape,
                               const void *const *chunk_ptrs, const uint64_t *chunk_lens, const uint64_t *sel_start,
                               const uint64_t *sel_shape, void *out, uint32_t flags, void *stream) {
  ABI_GUARD_BEGIN
  if (!ch || !array_shape || !chunk_shape || !chunk_ptrs || !chunk_lens || !sel_start || !sel_shape || !out)
    return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  std::vector<zgpu_chunk_desc> descs;
  std::vector<uint64_t> lins;
  const int r = subset_descs(nd, array_shape, chunk_shape, sel_start, sel_shape, descs, lins);
  if (r) return r < 0 ? ZGPU_OK : r;
  for (size_t k = 0; k < descs.size(); k++) {
    descs[k].enc = chunk_ptrs[lins[k]];
    descs[k].enc_len = descs[k].enc ? chunk_lens[lins[k]] : 0;
  }
  return zgpu_decode_batch(ch, nd, descs.data(), descs.size(), out, sel_shape, flags, nullptr, stream);
  ABI_GUARD_END
}

// Filesystem store -> HBM -> decode, pipelined over sub-batches in descriptor order: host threads
// read sub-batch g into pinned slab g%2 (positional reads, O_DIRECT pages with ZGPU_DIRECT_IO) while
// sub-batch g-1's H2D (copy stream 0) and decode (the call's stream) run; slab g%2 is reused once
// sub-batch g-2's H2D has completed.
int zgpu_decode_files(zgpu_chain *ch, uint32_t nd, const zgpu_chunk_desc *descs, const zgpu_file_range *files,
                      uint64_t n, void *out, const uint64_t *out_shape, uint32_t flags, int32_t *status,
                      void *stream) {
  ABI_GUARD_BEGIN
  if (!ch || !out_shape || (n && (!descs || !files)) || !out) return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  zgpu_ctx *C = ch->ctx;
  HIPCHK(hipSetDevice(C->device));
  LaneScope ls(C);
  Lane *LN = ls.L;
  hipStream_t s = pick_stream(LN, stream);
  reset_call_state();
  const int threads = host_copy_threads();
  std::vector<FileRange> fr(n);
  for (uint64_t i = 0; i < n; i++) {
    fr[i].path = files[i].path;
    fr[i].offset = files[i].offset;
    fr[i].len = files[i].len;
  }
  struct Closer {
    std::vector<FileRange> &r;
    ~Closer() { fs_close_all(r); }
  } closer{fr};
  std::string err = fs_open_all(fr, (flags & ZGPU_DIRECT_IO) != 0, threads);
  if (!err.empty()) return set_err(ZGPU_STORAGE_ERROR, err);
  // sub-batches: ~8 of them, 32-512 MiB of reads each
  auto readable = [&](uint64_t i) { return !fr[i].missing && !fr[i].bad_range; };
  uint64_t total = 0;
  for (uint64_t i = 0; i < n; i++)
    if (readable(i)) total += (fr[i].rd_len + 4095) & ~(uint64_t)4095;
  uint64_t target = std::min<uint64_t>(512ull << 20, std::max<uint64_t>(32ull << 20, total / 8));
  if (const char *e = std::getenv("ZGPU_FS_GROUP_BYTES")) target = std::max<uint64_t>(1, std::strtoull(e, nullptr, 10));
  struct Group { uint64_t b, e, base, bytes; };
  std::vector<Group> groups;
  {
    Group g{0, 0, 0, 0};
    for (uint64_t i = 0; i < n; i++) {
      const uint64_t sz = readable(i) ? ((fr[i].rd_len + 4095) & ~(uint64_t)4095) : 0;
      if (i > g.b && g.bytes + sz > target) {
        g.e = i;
        groups.push_back(g);
        g = Group{i, 0, g.base + g.bytes, 0};
      }
      fr[i].slab_off = g.bytes;  // page-aligned (O_DIRECT buffers)
      g.bytes += sz;
    }
    g.e = n;
    if (n) groups.push_back(g);
  }
  uint64_t max_g = 4096;
  for (const Group &g : groups) max_g = std::max(max_g, g.bytes);
  uint64_t out_elems = 1;
  for (uint32_t d = 0; d < nd; d++) out_elems *= out_shape[d];
  const uint64_t out_bytes = out_elems * ch->chain->es;
  const bool host_out = !(flags & ZGPU_OUT_DEVICE);
  for (hipStream_t &cs : LN->copy)
    if (!cs) HIPCHK(hipStreamCreateWithFlags(&cs, hipStreamNonBlocking));
  uint8_t *enc_dev = nullptr, *dout = (uint8_t *)out, *slab[2] = {nullptr, nullptr}, *pin_stage = nullptr;
  const uint64_t stage_slab = 64ull << 20;
  std::vector<hipEvent_t> ev(groups.size(), nullptr);
  std::vector<std::unique_ptr<zgpu_plan>> plans(groups.size());
  auto cleanup = [&]() {
    (void)hipStreamSynchronize(LN->copy[0]);
    (void)hipStreamSynchronize(s);
    plans.clear();
    for (hipEvent_t e : ev)
      if (e) (void)hipEventDestroy(e);
    C->dev_free(enc_dev);
    if (host_out) C->dev_free(dout);
    C->host_free(slab[0]);
    C->host_free(slab[1]);
    C->host_free(pin_stage);
  };
  int rc = 0;
  const bool fused = fused_plannable(*ch->chain) && uniform_shapes(descs, n, nd);
  std::vector<int32_t> all(n, 0);
  try {
    enc_dev = (uint8_t *)C->dev_alloc(total ? total : 1);
    if (host_out) {
      dout = (uint8_t *)C->dev_alloc(out_bytes ? out_bytes : 1);
      uint64_t covered = 0;  // disjoint regions: equal volumes mean full coverage (no upload)
      for (uint64_t i = 0; i < n; i++) {
        uint64_t v = 1;
        for (uint32_t d = 0; d < nd; d++) v *= descs[i].sel_shape[d];
        covered += v;
      }
      if (covered != out_elems) {
        pin_stage = (uint8_t *)C->host_alloc(2 * stage_slab);
        HIPCHK(h2d_bytes(dout, (const uint8_t *)out, out_bytes, pin_stage, stage_slab, threads, s));
      }
    }
    for (int k = 0; k < 2 && k < (int)groups.size(); k++) slab[k] = (uint8_t *)C->host_alloc(max_g);
    for (hipEvent_t &e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    for (size_t g = 0; g < groups.size(); g++) {
      const Group &G = groups[g];
      if (g >= 2) HIPCHK(hipEventSynchronize(ev[g - 2]));  // slab g%2 free again
      uint8_t *sl = slab[g & 1];
      std::vector<uint64_t> idx;
      for (uint64_t i = G.b; i < G.e; i++)
        if (readable(i)) idx.push_back(i);
      err = fs_read_into(fr, idx, sl, threads);
      if (!err.empty()) throw ChainError{ZGPU_STORAGE_ERROR, err};
      if (G.bytes) HIPCHK(hipMemcpyAsync(enc_dev + G.base, sl, G.bytes, hipMemcpyHostToDevice, LN->copy[0]));
      HIPCHK(hipEventRecord(ev[g], LN->copy[0]));
      std::vector<zgpu_chunk_desc> gd(descs + G.b, descs + G.e);
      for (uint64_t i = G.b; i < G.e; i++) {
        zgpu_chunk_desc &d = gd[i - G.b];
        if (readable(i)) {  // an empty object still has a (valid) address
          d.enc = enc_dev + G.base + fr[i].slab_off + (fr[i].offset - fr[i].rd_off);
          d.enc_len = fr[i].len;
        } else {
          d.enc = nullptr;
          d.enc_len = 0;
        }
      }
      if (!fused) {  // the general decode is synchronous: this group is done before the next is read
        HIPCHK(hipStreamWaitEvent(s, ev[g], 0));
        GeneralCall GC{C, ch->validate && !(flags & ZGPU_NO_VALIDATE), nd, dout, out_shape,
                       flags | ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE, s, {}};
        decode_general(GC, ch->chain, gd.data(), gd.size(), all.data() + G.b);
        continue;
      }
      plans[g].reset(plan_new(ch, nd, gd.data(), gd.size(), out_shape, flags | ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE));
      plan_upload(*plans[g], s);
      HIPCHK(hipStreamWaitEvent(s, ev[g], 0));
      plan_enqueue(*plans[g], dout, s);
    }
    for (size_t g = 0; g < groups.size(); g++)
      if (plans[g]) plan_statuses(*plans[g], all.data() + groups[g].b, s);
    for (uint64_t i = 0; i < n; i++) {
      if (fr[i].bad_range) all[i] = ZGPU_INVALID_BYTE_RANGE;
      if (status) status[i] = all[i];
      if (!rc) rc = all[i];
    }
    if (host_out) {
      if (!pin_stage) pin_stage = (uint8_t *)C->host_alloc(2 * stage_slab);
      HIPCHK(d2h_bytes((uint8_t *)out, dout, out_bytes, pin_stage, stage_slab, threads, s));
    }
  } catch (...) {
    cleanup();
    throw;
  }
  cleanup();
  if (rc) set_err(rc, zgpu_status_name(rc));
  return rc;
  ABI_GUARD_END
}

// Encoded size of one chunk for a fixed-size chain (BytesRepresentation::FixedSize), -1 if variable.
int64_t zgpu_chain_encoded_size(const zgpu_chain *ch, uint32_t nd, const uint64_t *chunk_shape) {
  if (!ch || !chunk_shape || nd == 0 || nd > ZGPU_MAX_DIMS) return -1;
  uint64_t n = 1;
  for (uint32_t d = 0; d < nd; d++) n *= chunk_shape[d];
  return chain_fixed_encoded_size(*ch->chain, n);
}

// Upper bound of one chunk's encoded size: the fixed size, a compressing chain's bounded size
// (chain_encoded_bound), or for sharding_indexed every inner chunk at its bound plus the index
// (ShardingCodec::encoded_shard_bounded_size, sharding_codec.rs:924-945, BytesRepresentation::
// BoundedSize); -1 if unbounded.
int64_t zgpu_chain_encoded_bound(const zgpu_chain *ch, uint32_t nd, const uint64_t *chunk_shape) {
  if (!ch || !chunk_shape || nd == 0 || nd > ZGPU_MAX_DIMS) return -1;
  const Chain &c = *ch->chain;
  if (c.a2b.kind != CodecKind::Sharding) {
    uint64_t n = 1;
    for (uint32_t d = 0; d < nd; d++) n *= chunk_shape[d];
    return chain_encoded_bound(c, n);
  }
  if (!c.a2a.empty() || !c.b2b.empty() || c.a2b.inner_shape.size() != nd) return -1;
  uint64_t n_inner = 1, inner_n = 1;
  for (uint32_t d = 0; d < nd; d++) {
    const uint64_t is = c.a2b.inner_shape[d];
    if (chunk_shape[d] % is) return -1;
    n_inner *= chunk_shape[d] / is;
    inner_n *= is;
  }
  const int64_t E = chain_encoded_bound(*c.a2b.inner, inner_n);
  const int64_t X = chain_fixed_encoded_size(*c.a2b.index, n_inner * 2);
  if (E < 0 || X < 0) return -1;
  return (int64_t)n_inner * E + X;
}

}  // extern "C"

// CodecChain::encode (codec_chain.rs:528-555) of a fixed-size chain for n chunks of a device array
// into device buffers h_dst[i] (chunk origins h_starts[i*nd..]): one gather (transposes + endianness +
// innermost shuffle, fill past the array edge), then one k_crc32c_encode launch per crc32c codec.
// Enqueues only (no synchronisation); d_tab: device table of n dst pointers + n*nd origins.
// The gather's parameters: the chain's transposes, bytes endianness and (shuffle) an innermost
// numcodecs.shuffle over the data type size, chunk data at data_off bytes into each destination.
static ZgEncode encode_params(const Chain &c, uint32_t nd, const uint64_t *chunk_shape, const uint64_t *array_shape,
                              bool shuffle, uint64_t data_off) {
  ZgEncode P{};
  P.nd = nd;
  P.es = c.es;
  P.comp = c.comp;
  P.swap = (c.a2b.big_endian && c.comp > 1) ? 1 : 0;
  P.shuffle = shuffle;
  P.nelem = 1;
  for (uint32_t d = 0; d < nd; d++) P.nelem *= chunk_shape[d];
  P.data_off = data_off;
  uint32_t m[ZG_MAXD];
  composed_axes(c, nd, m);
  uint64_t stride = 1;
  for (int d = (int)nd - 1; d >= 0; d--) {
    P.array_shape[d] = array_shape[d];
    P.array_stride[d] = stride;
    stride *= array_shape[d];
  }
  for (uint32_t a = 0; a < nd; a++) {
    P.dec_axis[a] = m[a];
    P.enc_shape[a] = chunk_shape[m[a]];
  }
  {
    uint64_t es_ = 1;
    for (int a = (int)nd - 1; a >= 0; a--) {
      P.enc_stride_of_dec[m[a]] = es_;
      es_ *= P.enc_shape[a];
    }
    for (uint32_t d = 0; d < nd; d++) P.dec_shape[d] = chunk_shape[d];
    // tiled encode: the axis (other than the encoded and the array innermost) with the smallest
    // encoded stride, so the TJ slabs of a block are adjacent encoded rows
    P.tile_b = ZG_MAXD;
    for (uint32_t d = 0; d + 1 < nd; d++) {
      if (d == m[nd - 1]) continue;
      if (P.tile_b == ZG_MAXD || P.enc_stride_of_dec[d] < P.enc_stride_of_dec[P.tile_b]) P.tile_b = d;
    }
  }
  std::memcpy(P.fill, c.fill, sizeof(P.fill));
  P.aligned = 0;
  return P;
}

static int encode_fixed(zgpu_ctx *C, const Chain &c, uint32_t nd, const uint64_t *chunk_shape, const void *array,
                        const uint64_t *array_shape, const std::vector<uint64_t> &h_tab, uint64_t n,
                        std::vector<void *> &owned, hipStream_t s, ZgEncode *out_P = nullptr) {
  if (c.a2b.kind != CodecKind::Bytes) return set_err(ZGPU_UNSUPPORTED, "encode: array->bytes codec must be bytes");
  for (const Codec &k : c.a2a)
    if (k.order.size() != nd) return set_err(ZGPU_INVALID_ARGUMENT, "transpose order rank != ndim");
  bool shuffle = false;
  int n_start = 0;
  for (size_t i = 0; i < c.b2b.size(); i++) {
    const Codec &k = c.b2b[i];
    if (k.kind == CodecKind::Shuffle && i == 0 && k.elementsize == c.es) shuffle = true;
    else if (k.kind == CodecKind::Crc32c) n_start += k.at_start ? 1 : 0;
    else return set_err(ZGPU_UNSUPPORTED, "encode: only transpose / bytes / numcodecs.shuffle (innermost, "
                                          "elementsize = data type size) / crc32c / gzip run on the GPU write path");
  }
  ZgEncode P = encode_params(c, nd, chunk_shape, array_shape, shuffle, 4ull * n_start);
  bool aligned = (P.data_off % c.es) == 0;
  for (uint64_t i = 0; i < n; i++)
    if (h_tab[i] % 16) aligned = false;
  P.aligned = aligned;
  if (out_P) *out_P = P;
  if (!n) return ZGPU_OK;
  uint64_t *d = (uint64_t *)C->dev_alloc(h_tab.size() * 8);
  owned.push_back(d);
  HIPCHK(hipMemcpyAsync(d, h_tab.data(), h_tab.size() * 8, hipMemcpyHostToDevice, s));
  HIPCHK(launch_encode_gather(d, d + n, (const uint8_t *)array, P, (uint32_t)n, s));
  uint64_t lo = P.data_off, len = P.nelem * c.es;
  for (const Codec &k : c.b2b) {
    if (k.kind != CodecKind::Crc32c) continue;
    HIPCHK(launch_crc32c_encode(d, (uint32_t)n, lo, len, k.at_start ? 1 : 0, s));
    if (k.at_start) lo -= 4;
    len += 4;
  }
  return ZGPU_OK;
}

static bool chain_compresses(const Chain &c) {
  for (const Codec &k : c.b2b)
    if (k.kind == CodecKind::Gzip || k.kind == CodecKind::Zstd || k.kind == CodecKind::Blosc) return true;
  return false;  // (blosc is refused by encode_var: its encoder is not on the GPU)
}

// CodecChain::encode (codec_chain.rs:528-555) of a chain with a compressor, for n chunks whose origins
// are origins[i*nd..]: the gather (transposes, endianness, innermost shuffle) into 64 B-headroom
// slots, then the bytes->bytes codecs in metadata order over the items {src, len}: crc32c appended /
// prepended in place, gzip into the other slot pool (k_gzip_encode). Enqueues only; on return the
// device item table and statuses describe every chunk's encoded bytes (inside scratch `owned`), and
// *d_tab_out is the device table [n gather destinations | n*nd origins].
static int encode_var(zgpu_ctx *C, const Chain &c, uint32_t nd, const uint64_t *chunk_shape, const void *array,
                      const uint64_t *array_shape, const uint64_t *origins, uint64_t n, std::vector<void *> &owned,
                      hipStream_t s, ZgItem **d_items_out, uint32_t **d_status_out, uint64_t **d_tab_out,
                      ZgEncode *P_out) {
  if (c.a2b.kind != CodecKind::Bytes) return set_err(ZGPU_UNSUPPORTED, "encode: array->bytes codec must be bytes");
  for (const Codec &k : c.a2a)
    if (k.order.size() != nd) return set_err(ZGPU_INVALID_ARGUMENT, "transpose order rank != ndim");
  uint64_t nelem = 1;
  for (uint32_t d = 0; d < nd; d++) nelem *= chunk_shape[d];
  bool shuffle = false;
  uint64_t size = nelem * c.es, max_size = size;
  uint32_t n_crc = 0;
  for (size_t i = 0; i < c.b2b.size(); i++) {
    const Codec &k = c.b2b[i];
    if (k.kind == CodecKind::Shuffle && i == 0 && k.elementsize == c.es) {
      shuffle = true;
    } else if (k.kind == CodecKind::Crc32c) {
      size += 4;
      n_crc++;
    } else if (k.kind == CodecKind::Gzip) {
      size = gzip_bound(size);
    } else if (k.kind == CodecKind::Zstd) {
      size = zstd_bound(size);
    } else if (k.kind == CodecKind::Blosc) {
      size += 16;
    } else {
      return set_err(ZGPU_UNSUPPORTED, "encode: only transpose / bytes / numcodecs.shuffle (innermost, elementsize = "
                                       "data type size) / crc32c / gzip / zstd / blosc run on the GPU write path");
    }
    max_size = std::max(max_size, size);
  }
  if (n_crc > 14) return set_err(ZGPU_UNSUPPORTED, "encode: too many crc32c codecs");
  constexpr uint64_t HR = 64;  // headroom in front of a slot's bytes (crc32c at the start)
  const uint64_t pitch = (HR + max_size + 4 * n_crc + 16 + 255) & ~(uint64_t)255;
  bool gz = false;  // a compressor: its output goes to the other slot pool
  for (const Codec &k : c.b2b)
    gz = gz || k.kind == CodecKind::Gzip || k.kind == CodecKind::Zstd || k.kind == CodecKind::Blosc;
  uint8_t *pool[2] = {(uint8_t *)C->dev_alloc(std::max<uint64_t>(n * pitch, 1)), nullptr};
  owned.push_back(pool[0]);
  if (gz) {
    pool[1] = (uint8_t *)C->dev_alloc(std::max<uint64_t>(n * pitch, 1));
    owned.push_back(pool[1]);
  }
  // gather into pool 0
  std::vector<uint64_t> tab(n * (1 + nd));
  for (uint64_t i = 0; i < n; i++) tab[i] = (uint64_t)(pool[0] + i * pitch + HR);
  std::memcpy(tab.data() + n, origins, n * nd * 8);
  uint64_t *d_tab = (uint64_t *)C->dev_alloc(std::max<size_t>(tab.size() * 8, 8));
  owned.push_back(d_tab);
  HIPCHK(hipMemcpyAsync(d_tab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice, s));
  ZgEncode P = encode_params(c, nd, chunk_shape, array_shape, shuffle, 0);
  P.aligned = (c.es <= 16 && (HR % 16) == 0 && (pitch % 16) == 0) ? 1u : 0u;
  if (n) HIPCHK(launch_encode_gather(d_tab, d_tab + n, (const uint8_t *)array, P, (uint32_t)n, s));
  // items over the gathered chunks
  std::vector<ZgItem> items(n);
  for (uint64_t i = 0; i < n; i++) items[i] = ZgItem{tab[i], nelem * c.es, (uint32_t)i, 0, 0, 0};
  ZgItem *d_items = (ZgItem *)C->dev_alloc(std::max<uint64_t>(n * sizeof(ZgItem), 1));
  uint32_t *d_status = (uint32_t *)C->dev_alloc(std::max<uint64_t>(n * 4, 4));
  owned.push_back(d_items);
  owned.push_back(d_status);
  HIPCHK(hipMemcpyAsync(d_items, items.data(), n * sizeof(ZgItem), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(d_status, 0, std::max<uint64_t>(n * 4, 4), s));
  int cur = 0;
  uint32_t *sym = nullptr;
  uint8_t *zscr = nullptr;
  uint64_t in_size = nelem * c.es;  // the current stage's input bound
  bool var_len = false;             // an earlier stage made the lengths variable
  for (size_t i = 0; i < c.b2b.size(); i++) {
    const Codec &k = c.b2b[i];
    const uint64_t stage_in = in_size;
    if (k.kind == CodecKind::Blosc) {
      // BloscCodec::encode (blosc_codec_via_blosc_src.rs:113-128): blosclz / lz4 / lz4hc / zlib / zstd
      // streams on the GPU
      const uint32_t comp = (k.cname == "lz4" || k.cname == "lz4hc") ? (uint32_t)BL_COMP_LZ4
                            : k.cname == "zstd"                       ? (uint32_t)BL_COMP_ZSTD
                            : k.cname == "blosclz"                    ? (uint32_t)BL_COMP_BLOSCLZ
                            : k.cname == "zlib"                       ? (uint32_t)BL_COMP_ZLIB
                            : k.cname == "snappy"                     ? (uint32_t)BL_COMP_SNAPPY
                                                                      : UINT32_MAX;
      if (comp == UINT32_MAX)
        return set_err(ZGPU_UNSUPPORTED, "encode: blosc cname '" + k.cname +
                                             "' (the GPU writes blosclz, lz4, lz4hc, snappy, zlib and zstd)");
      if (var_len) return set_err(ZGPU_UNSUPPORTED, "encode: blosc after a variable-length codec");
      const uint32_t ts = std::max<uint32_t>(1, k.elementsize);
      const int sh = k.shuffle >= 0 ? k.shuffle : (k.elementsize > 0 ? 2 : 0);  // zarrs' default (:119-123)
      const BloscEnc E = blosc_enc_params(comp, (uint32_t)sh, ts, stage_in, k.blocksize);
      uint8_t *bscr = (uint8_t *)C->dev_alloc(blosc_encode_scratch(E, (uint32_t)n));
      owned.push_back(bscr);
      cur ^= 1;
      HIPCHK(launch_blosc_encode(d_items, d_status, (uint32_t)n, E, pool[cur], pitch, bscr, k.level, s));
      in_size += 16;
      var_len = true;
      continue;
    }
    if (k.kind == CodecKind::Gzip || k.kind == CodecKind::Zstd) var_len = true;
    in_size = k.kind == CodecKind::Crc32c ? in_size + 4 : k.kind == CodecKind::Gzip ? gzip_bound(in_size)
              : k.kind == CodecKind::Zstd ? zstd_bound(in_size) : in_size;
    if (k.kind == CodecKind::Crc32c) {
      HIPCHK(launch_crc32c_items(d_items, d_status, (uint32_t)n, k.at_start ? 1 : 0, s));
    } else if (k.kind == CodecKind::Gzip) {
      if (!sym) {
        sym = (uint32_t *)C->dev_alloc((uint64_t)gzip_encode_grid((uint32_t)std::max<uint64_t>(n, 1)) * GZE_BLK_SYMS * 4);
        owned.push_back(sym);
      }
      cur ^= 1;
      HIPCHK(launch_gzip_encode(d_items, d_status, (uint32_t)n, pool[cur], pitch, sym, k.level, s));
    } else if (k.kind == CodecKind::Zstd) {
      zscr = (uint8_t *)C->dev_alloc(zstd_encode_scratch((uint32_t)n, stage_in));
      owned.push_back(zscr);
      cur ^= 1;
      HIPCHK(launch_zstd_encode(d_items, d_status, (uint32_t)n, stage_in, pool[cur], pitch, zscr, k.checksum ? 1 : 0,
                                s));
    }
  }
  *d_items_out = d_items;
  *d_status_out = d_status;
  if (d_tab_out) *d_tab_out = d_tab;
  if (P_out) *P_out = P;
  return ZGPU_OK;
}

// first non-zero of n device statuses (read back synchronously), 0 if none
static int first_status(const uint32_t *d_status, uint64_t n, hipStream_t s) {
  std::vector<uint32_t> h(n);
  if (n) HIPCHK(hipMemcpyAsync(h.data(), d_status, n * 4, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (uint32_t v : h)
    if (v) return (int)v;
  return 0;
}

// a chain with a compressor, unsharded: encode_var, then every chunk copied to its destination
static int encode_compressed(zgpu_ctx *C, const Chain &c, uint32_t nd, const uint64_t *chunk_shape, const void *array,
                             const uint64_t *array_shape, const zgpu_encode_desc *descs, uint64_t n, uint64_t *enc_lens,
                             std::vector<void *> &owned, hipStream_t s) {
  uint64_t nelem = 1;
  for (uint32_t d = 0; d < nd; d++) nelem *= chunk_shape[d];
  const int64_t bound = chain_encoded_bound(c, nelem);
  if (bound < 0) return set_err(ZGPU_UNSUPPORTED, "encode: the chain's encoded size is not bounded");
  for (uint64_t i = 0; i < n; i++)
    if (!descs[i].dst || descs[i].dst_cap < (uint64_t)bound)
      return set_err(ZGPU_INVALID_ARGUMENT, "encode: destination missing or smaller than the encoded bound");
  std::vector<uint64_t> org(n * nd), dc(2 * n);
  for (uint64_t i = 0; i < n; i++) {
    for (uint32_t d = 0; d < nd; d++) org[i * nd + d] = descs[i].chunk_start[d];
    dc[i] = (uint64_t)descs[i].dst;
    dc[n + i] = descs[i].dst_cap;
  }
  ZgItem *items = nullptr;
  uint32_t *st = nullptr;
  int rc = encode_var(C, c, nd, chunk_shape, array, array_shape, org.data(), n, owned, s, &items, &st, nullptr, nullptr);
  if (rc) return rc;
  uint64_t *d_dc = (uint64_t *)C->dev_alloc(8 * (3 * n));
  owned.push_back(d_dc);
  HIPCHK(hipMemcpyAsync(d_dc, dc.data(), 16 * n, hipMemcpyHostToDevice, s));
  HIPCHK(launch_encode_place(items, st, d_dc, d_dc + n, d_dc + 2 * n, (uint32_t)n, s));
  std::vector<uint64_t> lens(n);
  HIPCHK(hipMemcpyAsync(lens.data(), d_dc + 2 * n, 8 * n, hipMemcpyDeviceToHost, s));
  rc = first_status(st, n, s);
  if (rc) return set_err(rc, std::string("encode: ") + zgpu_status_name(rc));
  if (enc_lens) std::memcpy(enc_lens, lens.data(), 8 * n);
  return ZGPU_OK;
}

// sharding_indexed over a fixed-size inner chain (ShardingCodecBound::encode_bounded,
// sharding_codec.rs:924-1085, SubchunkWriteOrder::C): all inner chunks of all shards encoded into
// temporary slots in one batch, all-fill inner chunks omitted, the rest laid out in C order with the
// encoded index at the start or the end; shard lengths to enc_lens.
static int encode_sharded(zgpu_ctx *C, const Chain &top, uint32_t nd, const uint64_t *shard_shape, const void *array,
                          const uint64_t *array_shape, const zgpu_encode_desc *descs, uint64_t n, uint64_t *enc_lens,
                          std::vector<void *> &owned, hipStream_t s) {
  const Chain &inner = *top.a2b.inner, &xc = *top.a2b.index;
  if (!top.a2a.empty() || !top.b2b.empty())
    return set_err(ZGPU_UNSUPPORTED, "encode: codecs around sharding_indexed");
  if (top.a2b.inner_shape.size() != nd) return set_err(ZGPU_INVALID_ARGUMENT, "sharding chunk_shape rank");
  if (xc.a2b.kind != CodecKind::Bytes || !xc.a2a.empty())
    return set_err(ZGPU_UNSUPPORTED, "index_codecs must be bytes (+crc32c)");
  for (const Codec &k : xc.b2b)
    if (k.kind != CodecKind::Crc32c) return set_err(ZGPU_UNSUPPORTED, "index_codecs must be bytes (+crc32c)");
  uint64_t cps[ZG_MAXD], n_inner = 1, inner_n = 1;
  for (uint32_t d = 0; d < nd; d++) {
    const uint64_t is = top.a2b.inner_shape[d];
    if (shard_shape[d] % is) return set_err(ZGPU_INVALID_ARGUMENT, "shard shape not a multiple of chunk_shape");
    cps[d] = shard_shape[d] / is;
    n_inner *= cps[d];
    inner_n *= is;
  }
  const int64_t X = chain_fixed_encoded_size(xc, n_inner * 2);
  if (chain_compresses(inner)) {
    // inner chunks of variable length: encode_var over all inner chunks of all shards, then the
    // variable-length layout (C write order, all-fill inner chunks omitted) and the index crc32c
    const int64_t EB = chain_encoded_bound(inner, inner_n);
    if (EB < 0) return set_err(ZGPU_UNSUPPORTED, "encode: the inner chain's encoded size is not bounded");
    const uint64_t bound = n_inner * (uint64_t)EB + (uint64_t)X;
    uint64_t cap = UINT64_MAX;
    for (uint64_t i = 0; i < n; i++) {
      if (!descs[i].dst || descs[i].dst_cap < bound)
        return set_err(ZGPU_INVALID_ARGUMENT, "encode: destination missing or smaller than the shard's bounded size");
      cap = std::min(cap, descs[i].dst_cap);
    }
    const uint64_t n_chunks = n * n_inner;
    std::vector<uint64_t> org(n_chunks * nd);
    for (uint64_t i = 0; i < n; i++)
      for (uint64_t k = 0; k < n_inner; k++) {
        uint64_t rem = k;
        for (int d = (int)nd - 1; d >= 0; d--) {
          org[(i * n_inner + k) * nd + d] = descs[i].chunk_start[d] + (rem % cps[d]) * top.a2b.inner_shape[d];
          rem /= cps[d];
        }
      }
    ZgItem *items = nullptr;
    uint32_t *st = nullptr;
    uint64_t *d_tab = nullptr;
    ZgEncode IP{};
    int rc = encode_var(C, inner, nd, top.a2b.inner_shape.data(), array, array_shape, org.data(), n_chunks, owned, s,
                        &items, &st, &d_tab, &IP);
    if (rc) return rc;
    uint64_t *d_sh = (uint64_t *)C->dev_alloc(8 * (3 * n + n_chunks));
    uint32_t *d_nf = (uint32_t *)C->dev_alloc(4 * std::max<uint64_t>(n_chunks, 1) + 4 * n);
    owned.push_back(d_sh);
    owned.push_back(d_nf);
    std::vector<uint64_t> hd(n);
    for (uint64_t i = 0; i < n; i++) hd[i] = (uint64_t)descs[i].dst;
    HIPCHK(hipMemcpyAsync(d_sh, hd.data(), 8 * n, hipMemcpyHostToDevice, s));
    uint64_t *d_index_ptr = d_sh + n, *d_len = d_sh + 2 * n, *d_off = d_sh + 3 * n;
    uint32_t *d_shst = d_nf + n_chunks;
    int n_pre = 0;
    for (const Codec &k : xc.b2b) n_pre += k.at_start ? 1 : 0;
    ZgShardLayoutArgs A{n_inner, 0, cap, (uint64_t)X, 4ull * n_pre, top.a2b.at_start ? 1u : 0u,
                        xc.a2b.big_endian ? 1u : 0u};
    HIPCHK(launch_shard_encode_var(d_tab + n_chunks, (const uint8_t *)array, IP, (uint32_t)n_chunks, d_nf, items, st, A,
                                   d_sh, d_off, d_index_ptr, d_len, d_shst, (uint32_t)n, s));
    uint64_t lo = 4ull * n_pre, len = n_inner * 16;
    for (const Codec &k : xc.b2b) {
      HIPCHK(launch_crc32c_encode(d_index_ptr, (uint32_t)n, lo, len, k.at_start ? 1 : 0, s));
      if (k.at_start) lo -= 4;
      len += 4;
    }
    HIPCHK(hipMemcpyAsync(enc_lens, d_len, 8 * n, hipMemcpyDeviceToHost, s));
    rc = first_status(st, n_chunks, s);
    if (!rc) rc = first_status(d_shst, n, s);
    if (rc) return set_err(rc == 1 ? ZGPU_HIP_ERROR : rc, std::string("encode: ") + zgpu_status_name(rc));
    return ZGPU_OK;
  }
  const int64_t E = chain_fixed_encoded_size(inner, inner_n);
  if (E < 0) return set_err(ZGPU_UNSUPPORTED, "encode: the inner chain of sharding_indexed must be fixed-size or "
                                              "compressed by gzip");
  const uint64_t bound = n_inner * (uint64_t)E + (uint64_t)X;
  for (uint64_t i = 0; i < n; i++)
    if (!descs[i].dst || descs[i].dst_cap < bound)
      return set_err(ZGPU_INVALID_ARGUMENT, "encode: destination missing or smaller than the shard's bounded size");
  const uint64_t pitch = ((uint64_t)E + 255) & ~(uint64_t)255, n_chunks = n * n_inner;
  uint8_t *tmp = (uint8_t *)C->dev_alloc(std::max<uint64_t>(n_chunks * pitch, 1));
  owned.push_back(tmp);
  // inner chunk k of shard i: dst slot, origin in the array
  std::vector<uint64_t> tab(n_chunks * (1 + nd));
  for (uint64_t i = 0; i < n; i++)
    for (uint64_t k = 0; k < n_inner; k++) {
      const uint64_t g = i * n_inner + k;
      tab[g] = (uint64_t)(tmp + g * pitch);
      uint64_t rem = k;
      for (int d = (int)nd - 1; d >= 0; d--) {
        tab[n_chunks + g * nd + d] = descs[i].chunk_start[d] + (rem % cps[d]) * top.a2b.inner_shape[d];
        rem /= cps[d];
      }
    }
  ZgEncode IP{};
  int rc = encode_fixed(C, inner, nd, top.a2b.inner_shape.data(), array, array_shape, tab, n_chunks, owned, s, &IP);
  if (rc) return rc;
  const uint64_t *d_tab = (const uint64_t *)owned.back();  // [dst slots | origins] on the device
  // per-shard tables: dst pointers, inner offsets, index positions, lengths; fill flags
  uint64_t *d_sh = (uint64_t *)C->dev_alloc(8 * (3 * n + n_chunks));
  uint32_t *d_nf = (uint32_t *)C->dev_alloc(4 * std::max<uint64_t>(n_chunks, 1));
  owned.push_back(d_sh);
  owned.push_back(d_nf);
  std::vector<uint64_t> hd(n);
  for (uint64_t i = 0; i < n; i++) hd[i] = (uint64_t)descs[i].dst;
  HIPCHK(hipMemcpyAsync(d_sh, hd.data(), 8 * n, hipMemcpyHostToDevice, s));
  uint64_t *d_index_ptr = d_sh + n, *d_len = d_sh + 2 * n, *d_off = d_sh + 3 * n;
  int n_pre = 0;
  for (const Codec &k : xc.b2b) n_pre += k.at_start ? 1 : 0;
  ZgShardLayoutArgs A{n_inner, (uint64_t)E, pitch, (uint64_t)X, 4ull * n_pre, top.a2b.at_start ? 1u : 0u,
                      xc.a2b.big_endian ? 1u : 0u};
  HIPCHK(launch_shard_encode(d_tab + n_chunks, (const uint8_t *)array, IP, (uint32_t)n_chunks, d_nf, tmp, A, d_sh, d_off,
                             d_index_ptr, d_len, (uint32_t)n, s));
  uint64_t lo = 4ull * n_pre, len = n_inner * 16;
  for (const Codec &k : xc.b2b) {
    HIPCHK(launch_crc32c_encode(d_index_ptr, (uint32_t)n, lo, len, k.at_start ? 1 : 0, s));
    if (k.at_start) lo -= 4;
    len += 4;
  }
  HIPCHK(hipMemcpyAsync(enc_lens, d_len, 8 * n, hipMemcpyDeviceToHost, s));
  return ZGPU_OK;
}

extern "C" {

int zgpu_encode_chunks(zgpu_chain *ch, uint32_t nd, const uint64_t *chunk_shape, const void *array,
                       const uint64_t *array_shape, const zgpu_encode_desc *descs, uint64_t n, uint32_t flags,
                       uint64_t *enc_lens, void *stream) {
  ABI_GUARD_BEGIN
  if (!ch || !chunk_shape || !array || !array_shape || (n && !descs))
    return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  if ((flags & (ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE)) != (ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE))
    return set_err(ZGPU_INVALID_ARGUMENT, "encode: array and destinations must be device memory");
  const Chain &c = *ch->chain;
  for (uint64_t i = 0; i < n; i++)
    for (uint32_t d = 0; d < nd; d++)
      if (descs[i].chunk_start[d] >= array_shape[d])
        return set_err(ZGPU_INVALID_ARGUMENT, "encode: chunk origin outside the array");
  zgpu_ctx *C = ch->ctx;
  HIPCHK(hipSetDevice(C->device));
  LaneScope ls(C);
  hipStream_t s = pick_stream(ls.L, stream);
  if (!n) return ZGPU_OK;
  std::vector<void *> owned;
  int rc = 0;
  try {
    if (c.a2b.kind == CodecKind::Sharding) {
      uint64_t *hl = (uint64_t *)C->host_alloc(8 * n);
      rc = encode_sharded(C, c, nd, chunk_shape, array, array_shape, descs, n, hl, owned, s);
      HIPCHK(hipStreamSynchronize(s));
      if (!rc && enc_lens) std::memcpy(enc_lens, hl, 8 * n);
      C->host_free(hl);
    } else if (chain_compresses(c)) {
      uint64_t *hl = (uint64_t *)C->host_alloc(8 * n);
      rc = encode_compressed(C, c, nd, chunk_shape, array, array_shape, descs, n, hl, owned, s);
      HIPCHK(hipStreamSynchronize(s));
      if (!rc && enc_lens) std::memcpy(enc_lens, hl, 8 * n);
      C->host_free(hl);
    } else {
      const int64_t enc_size = chain_fixed_encoded_size(c, [&] {
        uint64_t e = 1;
        for (uint32_t d = 0; d < nd; d++) e *= chunk_shape[d];
        return e;
      }());
      if (enc_size < 0 && c.a2b.kind == CodecKind::Bytes)
        rc = set_err(ZGPU_UNSUPPORTED, "encode: only transpose / bytes / numcodecs.shuffle (innermost, elementsize = "
                                       "data type size) / crc32c, or sharding_indexed over such a chain, run on "
                                       "the GPU write path");
      for (uint64_t i = 0; i < n && !rc; i++)
        if (!descs[i].dst || descs[i].dst_cap < (uint64_t)std::max<int64_t>(enc_size, 0))
          rc = set_err(ZGPU_INVALID_ARGUMENT, "encode: destination missing or smaller than the encoded size");
      if (!rc) {
        std::vector<uint64_t> tab(n * (1 + nd));
        for (uint64_t i = 0; i < n; i++) {
          tab[i] = (uint64_t)descs[i].dst;
          for (uint32_t d = 0; d < nd; d++) tab[n + i * nd + d] = descs[i].chunk_start[d];
        }
        rc = encode_fixed(C, c, nd, chunk_shape, array, array_shape, tab, n, owned, s);
        HIPCHK(hipStreamSynchronize(s));
        if (!rc && enc_lens)
          for (uint64_t i = 0; i < n; i++) enc_lens[i] = (uint64_t)enc_size;
      }
    }
  } catch (...) {
    (void)hipStreamSynchronize(s);
    for (void *p : owned) C->dev_free(p);
    throw;
  }
  for (void *p : owned) C->dev_free(p);
  return rc;
  ABI_GUARD_END
}

// One chunk (or shard) from host bytes, encoded on the GPU, the encoded bytes left in pooled pinned
// memory for the caller to copy (the plugin's CodecChain::encode / ShardingCodecBound::encode).
int zgpu_encode_pinned(zgpu_chain *ch, uint32_t nd, const uint64_t *chunk_shape, const void *decoded,
                       const void **enc, uint64_t *enc_len, zgpu_result **result) {
  ABI_GUARD_BEGIN
  if (enc) *enc = nullptr;
  if (result) *result = nullptr;
  if (!ch || !chunk_shape || !decoded || !enc || !enc_len || !result)
    return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  zgpu_ctx *C = ch->ctx;
  HIPCHK(hipSetDevice(C->device));
  const int64_t bound = zgpu_chain_encoded_bound(ch, nd, chunk_shape);
  if (bound < 0) return set_err(ZGPU_UNSUPPORTED, "encode: the chain's encoded size is not bounded");
  const uint64_t nbytes = volume(chunk_shape, nd) * ch->chain->es;
  uint8_t *d_in = (uint8_t *)C->dev_alloc(nbytes ? nbytes : 1);
  uint8_t *d_out = (uint8_t *)C->dev_alloc(bound ? (uint64_t)bound : 1);
  std::unique_ptr<zgpu_result> R(new zgpu_result());
  ctx_ref(C);
  R->ctx = C;
  int rc = 0;
  try {
    hipStream_t s;
    {
      LaneScope ls(C);
      s = pick_stream(ls.L, nullptr);
      HIPCHK(hipMemcpyAsync(d_in, decoded, nbytes, hipMemcpyHostToDevice, s));
      HIPCHK(hipStreamSynchronize(s));
    }
    zgpu_encode_desc D{};
    D.dst = d_out;
    D.dst_cap = (uint64_t)bound;
    uint64_t len = 0;
    rc = zgpu_encode_chunks(ch, nd, chunk_shape, d_in, chunk_shape, &D, 1, ZGPU_ENC_DEVICE | ZGPU_OUT_DEVICE, &len,
                            nullptr);
    if (!rc) {
      R->own = (uint8_t *)C->host_alloc(len ? len : 1);
      LaneScope ls(C);
      s = pick_stream(ls.L, nullptr);
      HIPCHK(hipMemcpyAsync(R->own, d_out, len, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      *enc = R->own;
      *enc_len = len;
    }
  } catch (...) {
    C->dev_free(d_in);
    C->dev_free(d_out);
    throw;
  }
  C->dev_free(d_in);
  C->dev_free(d_out);
  if (rc) return rc;
  *result = R.release();
  return ZGPU_OK;
  ABI_GUARD_END
}

int zgpu_encode_batch(zgpu_chain *ch, uint32_t nd, const uint64_t *chunk_shape, const void *array,
                      const uint64_t *array_shape, const zgpu_encode_desc *descs, uint64_t n, uint32_t flags,
                      void *hip_stream) {
  if (ch && ch->chain->a2b.kind == CodecKind::Sharding)
    return set_err(ZGPU_INVALID_ARGUMENT, "encode: sharding_indexed chunks have variable lengths: zgpu_encode_chunks");
  if (ch && chain_compresses(*ch->chain))
    return set_err(ZGPU_INVALID_ARGUMENT, "encode: compressed chunks have variable lengths: zgpu_encode_chunks");
  return zgpu_encode_chunks(ch, nd, chunk_shape, array, array_shape, descs, n, flags, nullptr, hip_stream);
}

int zgpu_retrieve_array_subset_files(zgpu_chain *ch, uint32_t nd, const uint64_t *array_shape,
                                     const uint64_t *chunk_shape, const char *const *chunk_paths,
                                     const uint64_t *sel_start, const uint64_t *sel_shape, void *out, uint32_t flags,
                                     void *stream) {
  ABI_GUARD_BEGIN
  if (!ch || !array_shape || !chunk_shape || !chunk_paths || !sel_start || !sel_shape || !out)
    return set_err(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return set_err(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  std::vector<zgpu_chunk_desc> descs;
  std::vector<uint64_t> lins;
  const int r = subset_descs(nd, array_shape, chunk_shape, sel_start, sel_shape, descs, lins);
  if (r) return r < 0 ? ZGPU_OK : r;
  std::vector<zgpu_file_range> files(descs.size());
  for (size_t k = 0; k < descs.size(); k++) files[k] = zgpu_file_range{chunk_paths[lins[k]], 0, UINT64_MAX};
  return zgpu_decode_files(ch, nd, descs.data(), files.data(), descs.size(), out, sel_shape, flags, nullptr, stream);
  ABI_GUARD_END
}

}  // extern "C"
