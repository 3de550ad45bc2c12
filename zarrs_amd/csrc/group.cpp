// Plan groups: one decode call over the independent parts of a batch (one chunk shape and one output
// each: the levels of a multiscale pyramid), laid out on streams of the group's own.
//
// Reference: zarrs decodes each array's chunks in one rayon loop (zarrs/src/array/
// array_read_ops_common.rs:111-179); a pyramid read is one such loop per level, and the levels are
// independent. On the GPU the levels differ in what bounds them: the largest level's entropy decoding
// is throughput-bound, a mid level's LZ77 execution and the small levels' per-block FSE chains are
// latency-bound. Running them concurrently on a few streams, with the throughput-bound literal work of
// some plans overlapping the latency-bound sequence decoding of the others, is what bench.py's C5 did
// by hand in round 5 (profiles/r05/r05lf_zstd_lits_first_ab.txt); the group does it in the library:
//   * parts holding at least 1/(ZGPU_GROUP_SMALL_DIV x lanes) of the group's encoded bytes get a lane
//     each; the other (small) parts share one lane, largest first; the lanes left over go to the
//     largest part, whose descriptors are split into that many pieces of balanced encoded bytes (LPT);
//   * zstd literals-first (ZGPU_ZSTD_LITS_FIRST) on the largest part's first piece and on the
//     small-part lane; the largest part's lanes run at high stream priority;
//   * at most ZGPU_GROUP_LANES lanes (default 4: HIP's default GPU_MAX_HW_QUEUES; more streams than
//     hardware queues share queues and serialise).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <memory>
#include <mutex>
#include <numeric>
#include <string>
#include <vector>

#include "../../include/zgpu.h"
#include "chain.hpp"
#include "internal.hpp"

using namespace zgpu;

struct zgpu_group {
  zgpu_ctx *ctx = nullptr;
  int device = 0;
  struct Piece {
    zgpu_plan *plan = nullptr;
    uint32_t part = 0, lane = 0, lits_first = 0;
    std::vector<uint64_t> idx;  // positions of the piece's descriptors in the group's status order
  };
  std::vector<Piece> pieces;
  std::vector<std::vector<uint32_t>> lanes;  // piece indices per lane, in execution order
  std::vector<hipStream_t> streams;
  hipEvent_t fork = nullptr;
  std::vector<hipEvent_t> joins;
  uint64_t n_descs = 0;
  uint32_t n_parts = 0;
  std::mutex mu;
  ~zgpu_group() {
    for (Piece &p : pieces) zgpu_plan_destroy(p.plan);
    (void)hipSetDevice(device);
    for (hipStream_t s : streams) (void)hipStreamDestroy(s);
    for (hipEvent_t e : joins) (void)hipEventDestroy(e);
    if (fork) (void)hipEventDestroy(fork);
    ctx_unref(ctx);
  }
};

namespace {

uint32_t env_u32(const char *name, uint32_t dflt) {
  const char *s = std::getenv(name);
  return s && *s ? (uint32_t)std::strtoul(s, nullptr, 0) : dflt;
}

// descriptor indices [0, n) split into k lists of balanced weight (longest processing time first), each
// list in ascending index order
std::vector<std::vector<uint64_t>> lpt(const std::vector<uint64_t> &w, uint32_t k) {
  std::vector<uint64_t> order(w.size());
  std::iota(order.begin(), order.end(), 0);
  std::stable_sort(order.begin(), order.end(), [&](uint64_t a, uint64_t b) { return w[a] > w[b]; });
  std::vector<std::vector<uint64_t>> parts(k);
  std::vector<uint64_t> load(k, 0);
  for (uint64_t i : order) {
    const uint32_t j = (uint32_t)(std::min_element(load.begin(), load.end()) - load.begin());
    parts[j].push_back(i);
    load[j] += w[i];
  }
  for (auto &p : parts) std::sort(p.begin(), p.end());
  return parts;
}

int fail(int st, const std::string &m) { return set_last_error(st, m); }

}  // namespace

int zgpu_group_create(zgpu_chain *const *chains, uint32_t nd, uint32_t n_parts, const zgpu_chunk_desc *const *descs,
                      const uint64_t *n_descs, const uint64_t *const *out_shapes, uint32_t flags, zgpu_group **out) {
  try {
    if (!chains || !descs || !n_descs || !out_shapes || !out || n_parts == 0)
      return fail(ZGPU_INVALID_ARGUMENT, "NULL argument");
    for (uint32_t p = 0; p < n_parts; p++)
      if (!chains[p] || !out_shapes[p] || (n_descs[p] && !descs[p])) return fail(ZGPU_INVALID_ARGUMENT, "NULL part");
    zgpu_ctx *ctx = chain_ctx(chains[0]);
    for (uint32_t p = 1; p < n_parts; p++)
      if (chain_ctx(chains[p]) != ctx) return fail(ZGPU_INVALID_ARGUMENT, "zgpu_group: chains of different contexts");
    std::unique_ptr<zgpu_group> G(new zgpu_group);
    ctx_ref(ctx);
    G->ctx = ctx;
    G->device = ctx_device(ctx);
    G->n_parts = n_parts;
    if (hipSetDevice(G->device) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipSetDevice");
    // part weights: encoded bytes
    std::vector<uint64_t> bytes(n_parts, 0), first(n_parts, 0);
    uint64_t total = 0;
    for (uint32_t p = 0; p < n_parts; p++) {
      first[p] = G->n_descs;
      G->n_descs += n_descs[p];
      for (uint64_t i = 0; i < n_descs[p]; i++) bytes[p] += descs[p][i].enc_len;
      total += bytes[p];
    }
    std::vector<uint32_t> live;  // parts with descriptors, largest first
    for (uint32_t p = 0; p < n_parts; p++)
      if (n_descs[p]) live.push_back(p);
    std::stable_sort(live.begin(), live.end(), [&](uint32_t a, uint32_t b) { return bytes[a] > bytes[b]; });
    const uint32_t max_lanes = std::max<uint32_t>(1, std::min<uint32_t>(env_u32("ZGPU_GROUP_LANES", 4), 16));
    const uint32_t small_div = std::max<uint32_t>(1, env_u32("ZGPU_GROUP_SMALL_DIV", 4));
    std::vector<uint32_t> big, small;
    for (uint32_t p : live) (big.empty() || bytes[p] * small_div * max_lanes >= total ? big : small).push_back(p);
    // one lane per big part and one for the small parts: the smallest big parts join the small ones
    // while that is more than max_lanes
    while (!big.empty() && big.size() + (small.empty() ? 0u : 1u) > max_lanes) {
      small.insert(small.begin(), big.back());
      big.pop_back();
    }
    const uint32_t n_lanes_min = (uint32_t)big.size() + (small.empty() ? 0u : 1u);
    const uint32_t extra = live.size() > 1 && max_lanes > n_lanes_min ? max_lanes - n_lanes_min : 0u;
    const uint32_t lf_mask = env_u32("ZGPU_GROUP_LITS_FIRST", ~0u);  // lanes allowed literals-first (A/B)
    const char *lf_force_s = std::getenv("ZGPU_GROUP_LF_FORCE");     // A/B: lane i literals-first iff bit i
    const bool lf_forced = lf_force_s && *lf_force_s;
    const uint32_t lf_force = lf_forced ? (uint32_t)std::strtoul(lf_force_s, nullptr, 0) : 0u;
    const bool multi = n_lanes_min + extra > 1;
    auto add_piece = [&](uint32_t part, const std::vector<uint64_t> &which, uint32_t lane, bool lits_first) -> int {
      std::vector<zgpu_chunk_desc> d;
      d.reserve(which.size());
      zgpu_group::Piece pc;
      pc.part = part;
      pc.lane = lane;
      if (lf_forced) lits_first = (lf_force >> lane) & 1u;
      pc.lits_first = lits_first ? 1u : 0u;
      for (uint64_t i : which) {
        d.push_back(descs[part][i]);
        pc.idx.push_back(first[part] + i);
      }
      const uint32_t pf = flags | (multi ? ZGPU_ONE_STREAM : 0u) | (multi && lits_first ? ZGPU_ZSTD_LITS_FIRST : 0u);
      const int rc = zgpu_plan_create(chains[part], nd, d.data(), d.size(), out_shapes[part], pf, &pc.plan);
      if (rc) return rc;
      if (G->lanes.size() <= lane) G->lanes.resize(lane + 1);
      G->lanes[lane].push_back((uint32_t)G->pieces.size());
      G->pieces.push_back(std::move(pc));
      return ZGPU_OK;
    };
    uint32_t lane = 0;
    std::vector<uint32_t> high_lanes;
    for (size_t b = 0; b < big.size(); b++) {
      const uint32_t part = big[b];
      const uint32_t k = b == 0 ? 1 + extra : 1;
      std::vector<uint64_t> w(n_descs[part]);
      for (uint64_t i = 0; i < n_descs[part]; i++) w[i] = descs[part][i].enc_len;
      auto split = k > 1 ? lpt(w, k) : std::vector<std::vector<uint64_t>>{[&] {
        std::vector<uint64_t> all(n_descs[part]);
        std::iota(all.begin(), all.end(), 0);
        return all;
      }()};
      for (uint32_t j = 0; j < split.size(); j++) {
        if (split[j].empty()) continue;
        const bool lf = b == 0 && j == 0;
        const int rc = add_piece(part, split[j], lane, lf && ((lf_mask >> lane) & 1));
        if (rc) return rc;
        if (b == 0) high_lanes.push_back(lane);
        lane++;
      }
    }
    if (!small.empty()) {
      for (uint32_t part : small) {
        std::vector<uint64_t> all(n_descs[part]);
        std::iota(all.begin(), all.end(), 0);
        const int rc = add_piece(part, all, lane, (lf_mask >> lane) & 1);
        if (rc) return rc;
      }
      lane++;
    }
    int lo_prio = 0, hi_prio = 0;
    if (hipDeviceGetStreamPriorityRange(&lo_prio, &hi_prio) != hipSuccess) lo_prio = hi_prio = 0;
    for (uint32_t l = 0; l < G->lanes.size(); l++) {
      hipStream_t s = nullptr;
      const bool hi = std::find(high_lanes.begin(), high_lanes.end(), l) != high_lanes.end() && multi;
      if (hipStreamCreateWithPriority(&s, hipStreamNonBlocking, hi ? hi_prio : lo_prio) != hipSuccess)
        return fail(ZGPU_HIP_ERROR, "hipStreamCreateWithPriority");
      G->streams.push_back(s);
      hipEvent_t e = nullptr;
      if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipEventCreate");
      G->joins.push_back(e);
    }
    if (hipEventCreateWithFlags(&G->fork, hipEventDisableTiming) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipEventCreate");
    *out = G.release();
    return ZGPU_OK;
  } catch (const std::exception &e) {
    return fail(ZGPU_HIP_ERROR, std::string("zgpu_group_create: ") + e.what());
  }
}

static int group_statuses(zgpu_group *G, int32_t *status) {
  int first_rc = ZGPU_OK;
  std::vector<int32_t> tmp;
  for (zgpu_group::Piece &pc : G->pieces) {
    tmp.assign(pc.idx.size(), 0);
    const int rc = zgpu_plan_status(pc.plan, tmp.data(), G->streams[pc.lane]);
    if (rc && !first_rc) first_rc = rc;
    if (status)
      for (size_t i = 0; i < pc.idx.size(); i++) status[pc.idx[i]] = tmp[i];
  }
  if (first_rc) set_last_error(first_rc, zgpu_status_name(first_rc));
  return first_rc;
}

int zgpu_group_execute(zgpu_group *G, void *const *outs, int32_t *status, void *hip_stream) {
  try {
    if (!G || !outs) return fail(ZGPU_INVALID_ARGUMENT, "NULL argument");
    for (uint32_t p = 0; p < G->n_parts; p++)
      if (!outs[p]) return fail(ZGPU_INVALID_ARGUMENT, "NULL output");
    std::lock_guard<std::mutex> lk(G->mu);
    if (hipSetDevice(G->device) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipSetDevice");
    hipStream_t caller = (hipStream_t)hip_stream;  // NULL: the legacy default stream
    if (hipEventRecord(G->fork, caller) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipEventRecord");
    for (uint32_t l = 0; l < G->lanes.size(); l++) {
      if (hipStreamWaitEvent(G->streams[l], G->fork, 0) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipStreamWaitEvent");
      for (uint32_t pi : G->lanes[l]) {
        zgpu_group::Piece &pc = G->pieces[pi];
        const int rc = zgpu_plan_execute(pc.plan, outs[pc.part], nullptr, G->streams[l]);
        if (rc) return rc;
      }
      if (hipEventRecord(G->joins[l], G->streams[l]) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipEventRecord");
      if (hipStreamWaitEvent(caller, G->joins[l], 0) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipStreamWaitEvent");
    }
    if (!status) return ZGPU_OK;
    return group_statuses(G, status);
  } catch (const std::exception &e) {
    return fail(ZGPU_HIP_ERROR, std::string("zgpu_group_execute: ") + e.what());
  }
}

int zgpu_group_status(zgpu_group *G, int32_t *status, void *hip_stream) {
  (void)hip_stream;  // every piece is waited for on its own lane
  if (!G) return fail(ZGPU_INVALID_ARGUMENT, "NULL argument");
  try {
    std::lock_guard<std::mutex> lk(G->mu);
    if (hipSetDevice(G->device) != hipSuccess) return fail(ZGPU_HIP_ERROR, "hipSetDevice");
    return group_statuses(G, status);
  } catch (const std::exception &e) {
    return fail(ZGPU_HIP_ERROR, std::string("zgpu_group_status: ") + e.what());
  }
}

uint32_t zgpu_group_layout(const zgpu_group *G, uint32_t *lane_of, uint32_t *part_of, uint32_t *lits_first,
                           uint32_t n) {
  if (!G) return 0;
  const uint32_t k = (uint32_t)std::min<size_t>(n, G->pieces.size());
  for (uint32_t i = 0; i < k; i++) {
    if (lane_of) lane_of[i] = G->pieces[i].lane;
    if (part_of) part_of[i] = G->pieces[i].part;
    if (lits_first) lits_first[i] = G->pieces[i].lits_first;
  }
  return (uint32_t)G->pieces.size();
}

uint64_t zgpu_group_algorithmic_bytes(const zgpu_group *G) {
  if (!G) return 0;
  uint64_t b = 0;
  for (const zgpu_group::Piece &pc : G->pieces) b += zgpu_plan_algorithmic_bytes(pc.plan);
  return b;
}

uint32_t zgpu_group_counters(const zgpu_group *G, uint64_t *out, uint32_t n) {
  if (!G || !out) return 0;
  uint32_t k = 0;
  std::vector<uint64_t> c(n, 0), sum(n, 0);
  for (const zgpu_group::Piece &pc : G->pieces) {
    k = zgpu_plan_counters(pc.plan, c.data(), n);
    for (uint32_t i = 0; i < k; i++) sum[i] += c[i];
  }
  std::copy(sum.begin(), sum.begin() + k, out);
  return k;
}

void zgpu_group_destroy(zgpu_group *G) {
  if (!G) return;
  { std::lock_guard<std::mutex> lk(G->mu); }  // no execute of it still running on another thread
  delete G;
}
