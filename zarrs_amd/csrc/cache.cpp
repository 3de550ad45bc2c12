// HBM-resident decoded-chunk cache and DLPack (kDLROCM) export of device outputs (SURVEY.md §8(f)
// rank 4), on top of the batched decode of zgpu.cpp.
//
// zgpu_cache <- ChunkCacheDecodedLruSizeLimit (zarrs/src/array/chunk_cache/chunk_cache_lru.rs:270) used
//   through ArrayCached::retrieve_array_subset (array_read_ops_array_cached.rs:315-412): decoded WHOLE
//   chunks (the full decode path, checksums verified) are kept, keyed by chunk-grid index; a chunk
//   whose key is missing is cached as "no chunk" (ChunkCacheTypeDecoded = Option<..>: None) and reads
//   as the fill value; least recently used entries are evicted when the byte capacity is reached.
//   Here the entries live in one HBM pool of fixed-size slots: a read decodes all of its misses
//   straight into their slots in ONE batch (the pool viewed as an array [n_slots * c0, c1, ...] whose
//   axis-0 block k is slot k), then gathers the subset from the cached chunks in one more batch
//   (a bytes-only chain over device-resident decoded chunks: the scatter kernels, HBM bound).
// zgpu_*_dlpack <- the reference's DLPack export of retrieved data (zarrs/src/array/array_dlpack_ext.rs:
//   44-70, CPU memory only: Device::CPU): here the decoded subset stays in HBM and is handed over as a
//   DLManagedTensor on kDLROCM, zero copy (torch.utils.dlpack.from_dlpack / any DLPack consumer).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstring>
#include <list>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/zgpu.h"
#include "chain.hpp"
#include "internal.hpp"

using namespace zgpu;

struct zgpu_cache {
  zgpu_ctx *ctx = nullptr;
  int device = 0;  // the context's device, kept so that destroying the cache never reads the context
  uint64_t capacity = 0;
  std::mutex mu;
  // geometry of the cached chunks (one array per cache, as an ArrayCached owns its cache)
  const zgpu_chain *chain = nullptr;
  std::vector<uint64_t> chunk_shape;
  uint32_t es = 0;
  uint64_t slot_bytes = 0, n_slots = 0;
  uint8_t *pool = nullptr;
  zgpu_chain *identity = nullptr;  // [bytes little] over the same data type + fill: the gather
  // LRU: front = most recently used
  struct Entry {
    int64_t slot;  // -1: the chunk's key is missing (cached None -> fill value)
    std::list<uint64_t>::iterator it;
  };
  std::unordered_map<uint64_t, Entry> map;
  std::list<uint64_t> lru;
  std::vector<uint64_t> free_slots;
  uint64_t hits = 0, misses = 0;
  // "no chunk" entries hold no slot, so the byte capacity does not bound them: they are capped by
  // count (sparse arrays would otherwise grow the map, and every eviction scan, without limit)
  uint64_t n_slotless = 0;
  uint64_t slotless_cap() const { return 4 * n_slots + 4096; }
  void trim_slotless(const std::vector<uint64_t> &keep) {
    if (n_slotless <= slotless_cap()) return;
    std::unordered_map<uint64_t, char> in_read;
    for (uint64_t lin : keep) in_read[lin] = 1;
    for (auto it = lru.end(); it != lru.begin() && n_slotless > slotless_cap();) {
      --it;
      auto e = map.find(*it);
      if (e->second.slot >= 0 || in_read.count(*it)) continue;
      map.erase(e);
      it = lru.erase(it);
      n_slotless--;
    }
  }

  void reset() {
    n_slotless = 0;
    map.clear();
    lru.clear();
    free_slots.clear();
    if (pool) (void)hipFree(pool);
    pool = nullptr;
    if (identity) zgpu_chain_destroy(identity);
    identity = nullptr;
    chain = nullptr;
    n_slots = slot_bytes = 0;
  }
  ~zgpu_cache() { reset(); }
};

namespace {

int fail(int st, const std::string &m) { return set_last_error(st, m); }

// (re)bind the cache to a chain + chunk shape: the pool holds floor(capacity / chunk bytes) slots
int bind(zgpu_cache &K, const zgpu_chain *ch, uint32_t nd, const uint64_t *chunk_shape) {
  const Chain &c = chain_model(ch);
  const std::vector<uint64_t> cs(chunk_shape, chunk_shape + nd);
  if (K.chain == ch && K.chunk_shape == cs && K.es == c.es) return ZGPU_OK;
  K.reset();
  K.chain = ch;
  K.chunk_shape = cs;
  K.es = c.es;
  K.slot_bytes = c.es;
  for (uint64_t s : cs) K.slot_bytes *= s;
  K.n_slots = K.slot_bytes ? K.capacity / K.slot_bytes : 0;
  if (hipSetDevice(K.device) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipSetDevice");
  if (K.n_slots) {
    if (hipMalloc(&K.pool, K.n_slots * K.slot_bytes) != hipSuccess) {
      K.pool = nullptr;
      K.n_slots = 0;
      return fail(ZGPU_HIP_ERROR, "zgpu_cache: hipMalloc of the slot pool failed");
    }
    for (uint64_t k = K.n_slots; k-- > 0;) K.free_slots.push_back(k);
  }
  const char *identity = R"([{"name":"bytes","configuration":{"endian":"little"}}])";
  const int rc = zgpu_chain_create(K.ctx, identity, c.data_type.c_str(), c.fill, c.es, 0, &K.identity);
  if (rc) {
    K.reset();
    return rc;
  }
  return ZGPU_OK;
}

}  // namespace

extern "C" {

int zgpu_cache_create(zgpu_ctx *ctx, uint64_t capacity_bytes, zgpu_cache **out) {
  if (!ctx || !out) return fail(ZGPU_INVALID_ARGUMENT, "NULL argument");
  auto K = std::make_unique<zgpu_cache>();
  ctx_ref(ctx);
  K->ctx = ctx;
  K->device = ctx_device(ctx);
  K->capacity = capacity_bytes;
  *out = K.release();
  return ZGPU_OK;
}

void zgpu_cache_destroy(zgpu_cache *cache) {
  if (!cache) return;
  // the cache holds a reference to its context: it is alive here whatever order a garbage-collected
  // binding destroys them in
  zgpu_ctx *ctx = cache->ctx;
  if (hipSetDevice(cache->device) != hipSuccess) (void)hipGetLastError();
  delete cache;
  (void)hipGetLastError();  // a failed free must not surface in the caller's next HIP error check
  ctx_unref(ctx);
}

int zgpu_cache_clear(zgpu_cache *K) {
  if (!K) return fail(ZGPU_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> lk(K->mu);
  K->n_slotless = 0;
  K->map.clear();
  K->lru.clear();
  K->free_slots.clear();
  for (uint64_t k = K->n_slots; k-- > 0;) K->free_slots.push_back(k);
  return ZGPU_OK;
}

int zgpu_cache_stats(zgpu_cache *K, uint64_t *hits, uint64_t *misses, uint64_t *entries, uint64_t *bytes_used) {
  if (!K) return fail(ZGPU_INVALID_ARGUMENT, "NULL argument");
  std::lock_guard<std::mutex> lk(K->mu);
  if (hits) *hits = K->hits;
  if (misses) *misses = K->misses;
  if (entries) *entries = K->map.size();
  if (bytes_used) *bytes_used = (K->n_slots - K->free_slots.size()) * K->slot_bytes;
  return ZGPU_OK;
}

int zgpu_cache_retrieve_array_subset(zgpu_cache *K, zgpu_chain *ch, uint32_t nd, const uint64_t *array_shape,
                                     const uint64_t *chunk_shape, const void *const *chunk_ptrs,
                                     const uint64_t *chunk_lens, const uint64_t *sel_start, const uint64_t *sel_shape,
                                     void *out, uint32_t flags, void *hip_stream) {
  if (!K || !ch || !array_shape || !chunk_shape || !chunk_ptrs || !chunk_lens || !sel_start || !sel_shape || !out)
    return fail(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return fail(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  if (chain_ctx(ch) != K->ctx) return fail(ZGPU_INVALID_ARGUMENT, "zgpu_cache: chain of another context");
  std::lock_guard<std::mutex> lk(K->mu);
  std::vector<zgpu_chunk_desc> descs;
  std::vector<uint64_t> lins;
  int rc = subset_descs(nd, array_shape, chunk_shape, sel_start, sel_shape, descs, lins);
  if (rc) return rc < 0 ? ZGPU_OK : rc;
  if ((rc = bind(*K, ch, nd, chunk_shape))) return rc;
  // the chunks this read needs that hold no slot yet
  std::vector<size_t> need;
  uint64_t present = 0;
  for (size_t k = 0; k < descs.size(); k++) {
    const uint64_t lin = lins[k];
    auto e = K->map.find(lin);
    if (e != K->map.end()) {
      K->lru.splice(K->lru.begin(), K->lru, e->second.it);
      K->hits++;
      if (e->second.slot >= 0) present++;
      continue;
    }
    K->misses++;
    if (chunk_ptrs[lin]) {
      need.push_back(k);
      present++;
    } else {  // missing key: cached as "no chunk" (fill value)
      K->lru.push_front(lin);
      K->map[lin] = zgpu_cache::Entry{-1, K->lru.begin()};
      K->n_slotless++;
    }
  }
  K->trim_slotless(lins);
  if (present > K->n_slots) {  // the read alone exceeds the capacity: decode it directly, cache nothing new
    return zgpu_retrieve_array_subset(ch, nd, array_shape, chunk_shape, chunk_ptrs, chunk_lens, sel_start, sel_shape,
                                      out, flags, hip_stream);
  }
  // slots for the misses: free ones first, then the least recently used entries this read does not use
  std::vector<char> used_now;
  if (!need.empty()) {
    std::unordered_map<uint64_t, char> in_read;
    for (uint64_t lin : lins) in_read[lin] = 1;
    std::vector<zgpu_chunk_desc> md;
    std::vector<int64_t> mslot;
    for (size_t k : need) {
      int64_t slot = -1;
      if (!K->free_slots.empty()) {
        slot = (int64_t)K->free_slots.back();
        K->free_slots.pop_back();
      } else {
        for (auto it = K->lru.end(); it != K->lru.begin();) {
          --it;
          const uint64_t victim = *it;
          if (in_read.count(victim)) continue;
          auto ve = K->map.find(victim);
          if (ve->second.slot < 0) continue;  // holds no slot
          slot = ve->second.slot;
          K->lru.erase(it);
          K->map.erase(ve);
          break;
        }
      }
      if (slot < 0) return fail(ZGPU_INVALID_ARGUMENT, "zgpu_cache: no slot could be freed");
      zgpu_chunk_desc d{};
      d.enc = chunk_ptrs[lins[k]];
      d.enc_len = chunk_lens[lins[k]];
      for (uint32_t a = 0; a < nd; a++) {
        d.chunk_shape[a] = chunk_shape[a];
        d.sel_shape[a] = chunk_shape[a];  // whole chunks: the full decode path
      }
      d.out_start[0] = (uint64_t)slot * chunk_shape[0];
      md.push_back(d);
      mslot.push_back(slot);
    }
    // every miss decoded into its slot in one batch: the pool is an array [n_slots * c0, c1, ...]
    std::vector<uint64_t> pshape(chunk_shape, chunk_shape + nd);
    pshape[0] *= K->n_slots;
    // -1: no status written (a call-level failure returns before the per-chunk statuses exist)
    std::vector<int32_t> st(md.size(), -1);
    // entries hold verified chunks (the header's promise): a caller's ZGPU_NO_VALIDATE does not reach
    // the miss decode, so an entry never depends on which reader decoded it first
    rc = zgpu_decode_batch(ch, nd, md.data(), md.size(), K->pool, pshape.data(),
                           (flags & ZGPU_ENC_DEVICE) | ZGPU_OUT_DEVICE, st.data(), hip_stream);
    // a chunk is cached only with a written status of 0: a call-level error (HIP, argument, or a chain
    // the planner rejects, e.g. UNSUPPORTED, before any status exists) leaves every slot undecoded
    bool any_status = false;
    for (int32_t v : st) any_status = any_status || v >= 0;
    if (rc && !any_status) {
      for (int64_t sl : mslot) K->free_slots.push_back((uint64_t)sl);
      return rc;
    }
    for (size_t j = 0; j < need.size(); j++) {
      if (st[j] != 0) {  // not cached; the error is the call's
        K->free_slots.push_back((uint64_t)mslot[j]);
        continue;
      }
      const uint64_t lin = lins[need[j]];
      K->lru.push_front(lin);
      K->map[lin] = zgpu_cache::Entry{mslot[j], K->lru.begin()};
    }
    if (rc) return fail(rc, zgpu_status_name(rc));
  }
  // gather the subset from the cached chunks (device-resident, decoded): one batch
  for (size_t k = 0; k < descs.size(); k++) {
    const zgpu_cache::Entry &e = K->map.at(lins[k]);
    descs[k].enc = e.slot < 0 ? nullptr : K->pool + (uint64_t)e.slot * K->slot_bytes;
    descs[k].enc_len = e.slot < 0 ? 0 : K->slot_bytes;
  }
  return zgpu_decode_batch(K->identity, nd, descs.data(), descs.size(), out, sel_shape,
                           ZGPU_ENC_DEVICE | (flags & ZGPU_OUT_DEVICE), nullptr, hip_stream);
}

// ---------------------------------------------------------------------------------------------
// DLPack export
// ---------------------------------------------------------------------------------------------
namespace {
struct DlHolder {
  zgpu_dl_managed_tensor mt;
  int64_t shape[ZGPU_MAX_DIMS];
  int device;
};

void dl_deleter(zgpu_dl_managed_tensor *t) {
  if (!t) return;
  DlHolder *h = (DlHolder *)t->manager_ctx;
  (void)hipSetDevice(h->device);
  (void)hipFree(t->dl_tensor.data);
  delete h;
}

bool dl_dtype(const std::string &n, zgpu_dl_data_type &d) {
  struct E { const char *name; uint8_t code, bits; };
  static const E tab[] = {{"bool", 6, 8},      {"int8", 0, 8},       {"int16", 0, 16},    {"int32", 0, 32},
                          {"int64", 0, 64},    {"uint8", 1, 8},      {"uint16", 1, 16},   {"uint32", 1, 32},
                          {"uint64", 1, 64},   {"float16", 2, 16},   {"float32", 2, 32},  {"float64", 2, 64},
                          {"bfloat16", 4, 16}, {"complex64", 5, 64}, {"complex128", 5, 128}};
  for (const E &e : tab)
    if (n == e.name) {
      d = zgpu_dl_data_type{e.code, e.bits, 1};
      return true;
    }
  return false;
}
}  // namespace

int zgpu_retrieve_array_subset_dlpack(zgpu_cache *cache, zgpu_chain *ch, uint32_t nd, const uint64_t *array_shape,
                                      const uint64_t *chunk_shape, const void *const *chunk_ptrs,
                                      const uint64_t *chunk_lens, const uint64_t *sel_start, const uint64_t *sel_shape,
                                      uint32_t flags, void *hip_stream, zgpu_dl_managed_tensor **out) {
  if (!ch || !sel_shape || !out) return fail(ZGPU_INVALID_ARGUMENT, "NULL argument");
  if (nd == 0 || nd > ZGPU_MAX_DIMS) return fail(ZGPU_INVALID_ARGUMENT, "ndim out of range");
  *out = nullptr;
  const Chain &c = chain_model(ch);
  auto h = std::make_unique<DlHolder>();
  if (!dl_dtype(c.data_type, h->mt.dl_tensor.dtype))
    return fail(ZGPU_UNSUPPORTED, "DLPack: data type " + c.data_type);
  uint64_t bytes = c.es;
  for (uint32_t d = 0; d < nd; d++) {
    bytes *= sel_shape[d];
    h->shape[d] = (int64_t)sel_shape[d];
  }
  h->device = ctx_device(chain_ctx(ch));
  if (hipSetDevice(h->device) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipSetDevice");
  void *buf = nullptr;
  if (hipMalloc(&buf, bytes ? bytes : 1) != hipSuccess) return fail(ZGPU_HIP_ERROR, "DLPack: hipMalloc failed");
  const uint32_t f = (flags & ~(uint32_t)ZGPU_OUT_DEVICE) | ZGPU_OUT_DEVICE;
  const int rc = cache ? zgpu_cache_retrieve_array_subset(cache, ch, nd, array_shape, chunk_shape, chunk_ptrs, chunk_lens,
                                                          sel_start, sel_shape, buf, f, hip_stream)
                       : zgpu_retrieve_array_subset(ch, nd, array_shape, chunk_shape, chunk_ptrs, chunk_lens, sel_start,
                                                    sel_shape, buf, f, hip_stream);
  if (rc) {
    (void)hipFree(buf);
    return rc;
  }
  zgpu_dl_tensor &t = h->mt.dl_tensor;
  t.data = buf;
  t.device = zgpu_dl_device{ZGPU_DL_ROCM, h->device};
  t.ndim = (int32_t)nd;
  t.shape = h->shape;
  t.strides = nullptr;  // compact row-major
  t.byte_offset = 0;
  h->mt.manager_ctx = h.get();
  h->mt.deleter = dl_deleter;
  *out = &h.release()->mt;
  return ZGPU_OK;
}

}  // extern "C"
