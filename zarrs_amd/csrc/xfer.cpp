// Host <-> device transfer engine of the decode call; see xfer.hpp.
#include "xfer.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <thread>

namespace zgpu {

int host_copy_threads() {
  static const int n = [] {
    const char *e = std::getenv("ZGPU_COPY_THREADS");
    int v = e ? std::atoi(e) : 0;
    if (v <= 0) v = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
    return v;
  }();
  return n;
}

bool host_is_pinned(const void *p) {
  hipPointerAttribute_t a;
  if (hipPointerGetAttributes(&a, p) != hipSuccess) {
    (void)hipGetLastError();  // pageable memory: not an error for us
    return false;
  }
  return a.type == hipMemoryTypeHost;
}

void parallel_memcpy(const std::vector<uint8_t *> &dst, const std::vector<const uint8_t *> &src,
                     const std::vector<uint64_t> &len, int threads) {
  uint64_t total = 0;
  for (uint64_t n : len) total += n;
  if (total < (8u << 20) || threads <= 1) {  // small: one thread
    for (size_t i = 0; i < len.size(); i++) std::memcpy(dst[i], src[i], len[i]);
    return;
  }
  // split the byte stream into `threads` equal shares, pieces cut at share boundaries
  const uint64_t share = (total + threads - 1) / threads;
  std::vector<std::thread> pool;
  pool.reserve(threads);
  for (int t = 0; t < threads; t++) {
    const uint64_t b0 = (uint64_t)t * share, b1 = std::min(total, b0 + share);
    if (b0 >= b1) break;
    pool.emplace_back([&, b0, b1] {
      uint64_t off = 0;
      for (size_t i = 0; i < len.size() && off < b1; i++) {
        const uint64_t s0 = off, s1 = off + len[i];
        off = s1;
        const uint64_t lo = std::max(s0, b0), hi = std::min(s1, b1);
        if (lo < hi) std::memcpy(dst[i] + (lo - s0), src[i] + (lo - s0), hi - lo);
      }
    });
  }
  for (auto &th : pool) th.join();
}

hipError_t h2d_ranges(uint8_t *dev, const std::vector<HostRange> &ranges, bool pinned_ok, uint8_t *stage,
                      uint64_t slab_bytes, int threads, hipStream_t s) {
  hipError_t e = hipSuccess;
  if (pinned_ok) {
    for (const HostRange &r : ranges)
      if (r.len && (e = hipMemcpyAsync(dev + r.dev_off, r.src, r.len, hipMemcpyHostToDevice, s)) != hipSuccess)
        return e;
    return hipSuccess;
  }
  // staged: fill slab k on the host while slab k^1's H2D is in flight
  hipEvent_t done[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; k++)
    if ((e = hipEventCreateWithFlags(&done[k], hipEventDisableTiming)) != hipSuccess) return e;
  bool used[2] = {false, false};
  int slab = 0;
  size_t i = 0;
  uint64_t off_in_range = 0;
  while (i < ranges.size() && e == hipSuccess) {
    if (used[slab]) e = hipEventSynchronize(done[slab]);
    if (e != hipSuccess) break;
    uint8_t *buf = stage + (uint64_t)slab * slab_bytes;
    std::vector<uint8_t *> d;
    std::vector<const uint8_t *> sp;
    std::vector<uint64_t> n;
    std::vector<std::pair<uint64_t, uint64_t>> dev_pieces;  // (dev_off, len) mirrored in buf order
    uint64_t fill = 0;
    while (i < ranges.size() && fill < slab_bytes) {
      const HostRange &r = ranges[i];
      const uint64_t take = std::min(r.len - off_in_range, slab_bytes - fill);
      d.push_back(buf + fill);
      sp.push_back(r.src + off_in_range);
      n.push_back(take);
      dev_pieces.push_back({r.dev_off + off_in_range, take});
      fill += take;
      off_in_range += take;
      if (off_in_range == r.len) {
        i++;
        off_in_range = 0;
      }
    }
    parallel_memcpy(d, sp, n, threads);
    // consecutive pieces whose device offsets are contiguous go as one copy
    uint64_t bo = 0;
    for (size_t k = 0; k < dev_pieces.size();) {
      uint64_t dv = dev_pieces[k].first, ln = dev_pieces[k].second;
      size_t j = k + 1;
      while (j < dev_pieces.size() && dev_pieces[j].first == dv + ln) ln += dev_pieces[j++].second;
      if ((e = hipMemcpyAsync(dev + dv, buf + bo, ln, hipMemcpyHostToDevice, s)) != hipSuccess) break;
      bo += ln;
      k = j;
    }
    if (e == hipSuccess) e = hipEventRecord(done[slab], s);
    used[slab] = true;
    slab ^= 1;
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  for (int k = 0; k < 2; k++) (void)hipEventDestroy(done[k]);
  return e;
}

hipError_t h2d_bytes(uint8_t *dst, const uint8_t *src, uint64_t n, uint8_t *stage, uint64_t slab_bytes,
                     int threads, hipStream_t s) {
  std::vector<HostRange> r{{src, n, 0}};
  return h2d_ranges(dst, r, host_is_pinned(src), stage, slab_bytes, threads, s);
}

hipError_t d2h_bytes(uint8_t *dst, const uint8_t *src, uint64_t n, uint8_t *stage, uint64_t slab_bytes,
                     int threads, hipStream_t s) {
  hipError_t e;
  if (host_is_pinned(dst)) {
    if ((e = hipMemcpyAsync(dst, src, n, hipMemcpyDeviceToHost, s)) != hipSuccess) return e;
    return hipStreamSynchronize(s);
  }
  // staged: D2H of slab k+1 overlaps the host copy-out of slab k
  hipEvent_t done[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; k++)
    if ((e = hipEventCreateWithFlags(&done[k], hipEventDisableTiming)) != hipSuccess) return e;
  const uint64_t nslabs = (n + slab_bytes - 1) / slab_bytes;
  auto issue = [&](uint64_t k) {
    const uint64_t o = k * slab_bytes, len = std::min(slab_bytes, n - o);
    hipError_t r = hipMemcpyAsync(stage + (k & 1) * slab_bytes, src + o, len, hipMemcpyDeviceToHost, s);
    if (r == hipSuccess) r = hipEventRecord(done[k & 1], s);
    return r;
  };
  e = nslabs ? issue(0) : hipSuccess;
  for (uint64_t k = 0; k < nslabs && e == hipSuccess; k++) {
    if (k + 1 < nslabs && (e = issue(k + 1)) != hipSuccess) break;
    if ((e = hipEventSynchronize(done[k & 1])) != hipSuccess) break;
    const uint64_t o = k * slab_bytes, len = std::min(slab_bytes, n - o);
    parallel_memcpy({dst + o}, {stage + (k & 1) * slab_bytes}, {len}, threads);
  }
  for (int k = 0; k < 2; k++) (void)hipEventDestroy(done[k]);
  return e;
}

// ------------------------------------------------------------------------------------------------
// Boxes of a larger array (ArrayBytesFixedDisjointView, array_bytes_fixed_disjoint_view.rs:177-206:
// one memcpy per contiguous run of the view's subset)
// ------------------------------------------------------------------------------------------------
bool box_is_whole(uint32_t nd, const uint64_t *array_shape, const uint64_t *start, const uint64_t *shape) {
  for (uint32_t d = 0; d < nd; d++)
    if (start[d] != 0 || shape[d] != array_shape[d]) return false;
  return true;
}

BoxRuns box_runs(uint32_t nd, const uint64_t *array_shape, const uint64_t *start, const uint64_t *shape, uint32_t es) {
  BoxRuns R;
  uint64_t stride[8];
  uint64_t s = es;
  for (int d = (int)nd - 1; d >= 0; d--) {
    stride[d] = s;
    s *= array_shape[d];
  }
  for (uint32_t d = 0; d < nd; d++) R.base += start[d] * stride[d];
  // the run: the innermost axis plus every outer axis the box spans whole, up to (and including) the
  // first axis it does not
  int j = (int)nd - 1;
  uint64_t run = shape[j] * es;
  while (j > 0 && shape[j] == array_shape[j]) {
    j--;
    run *= shape[j];
  }
  R.run_bytes = run;
  R.outer = (uint32_t)j;
  R.n_runs = 1;
  for (int d = 0; d < j; d++) {
    R.shape[d] = shape[d];
    R.stride[d] = stride[d];
    R.n_runs *= shape[d];
  }
  if (run == 0) R.n_runs = 0;
  return R;
}

uint64_t BoxRuns::offset(uint64_t k) const {
  uint64_t off = base;
  for (int d = (int)outer - 1; d >= 0; d--) {
    off += (k % shape[d]) * stride[d];
    k /= shape[d];
  }
  return off;
}

void copy_box_runs(const BoxRuns &R, uint8_t *array, uint8_t *compact, uint64_t lo, uint64_t hi, bool to_array,
                   int threads) {
  if (hi <= lo || !R.run_bytes) return;
  const uint64_t k0 = lo / R.run_bytes, k1 = (hi - 1) / R.run_bytes + 1;
  auto work = [&](uint64_t a, uint64_t b) {
    for (uint64_t k = a; k < b; k++) {
      const uint64_t r0 = std::max(lo, k * R.run_bytes), r1 = std::min(hi, (k + 1) * R.run_bytes);
      uint8_t *arr = array + R.offset(k) + (r0 - k * R.run_bytes);
      uint8_t *cmp = compact + (r0 - lo);
      if (to_array)
        std::memcpy(arr, cmp, r1 - r0);
      else
        std::memcpy(cmp, arr, r1 - r0);
    }
  };
  const uint64_t nk = k1 - k0;
  if (threads <= 1 || hi - lo < (4u << 20) || nk < 2) {
    work(k0, k1);
    return;
  }
  const uint64_t nt = std::min<uint64_t>((uint64_t)threads, nk);
  std::vector<std::thread> pool;
  pool.reserve(nt);
  for (uint64_t t = 0; t < nt; t++) pool.emplace_back(work, k0 + nk * t / nt, k0 + nk * (t + 1) / nt);
  for (auto &th : pool) th.join();
}

hipError_t d2h_box(const BoxRuns &R, uint8_t *host_array, const uint8_t *dev_compact, uint8_t *stage,
                   uint64_t slab_bytes, int threads, hipStream_t s) {
  const uint64_t n = R.n_runs * R.run_bytes;
  if (R.n_runs == 1) return d2h_bytes(host_array + R.base, dev_compact, n, stage, slab_bytes, threads, s);
  hipError_t e;
  hipEvent_t done[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; k++)
    if ((e = hipEventCreateWithFlags(&done[k], hipEventDisableTiming)) != hipSuccess) return e;
  const uint64_t nslabs = (n + slab_bytes - 1) / slab_bytes;
  auto issue = [&](uint64_t k) {
    const uint64_t o = k * slab_bytes, len = std::min(slab_bytes, n - o);
    hipError_t r = hipMemcpyAsync(stage + (k & 1) * slab_bytes, dev_compact + o, len, hipMemcpyDeviceToHost, s);
    if (r == hipSuccess) r = hipEventRecord(done[k & 1], s);
    return r;
  };
  e = nslabs ? issue(0) : hipSuccess;
  for (uint64_t k = 0; k < nslabs && e == hipSuccess; k++) {
    if (k + 1 < nslabs && (e = issue(k + 1)) != hipSuccess) break;
    if ((e = hipEventSynchronize(done[k & 1])) != hipSuccess) break;
    const uint64_t o = k * slab_bytes, len = std::min(slab_bytes, n - o);
    copy_box_runs(R, host_array, stage + (k & 1) * slab_bytes, o, o + len, true, threads);
  }
  for (int k = 0; k < 2; k++) (void)hipEventDestroy(done[k]);
  return e;
}

hipError_t h2d_box(const BoxRuns &R, uint8_t *dev_compact, const uint8_t *host_array, uint8_t *stage,
                   uint64_t slab_bytes, int threads, hipStream_t s) {
  const uint64_t n = R.n_runs * R.run_bytes;
  if (R.n_runs == 1) return h2d_bytes(dev_compact, host_array + R.base, n, stage, slab_bytes, threads, s);
  hipError_t e = hipSuccess;
  hipEvent_t done[2] = {nullptr, nullptr};
  for (int k = 0; k < 2; k++)
    if ((e = hipEventCreateWithFlags(&done[k], hipEventDisableTiming)) != hipSuccess) return e;
  bool used[2] = {false, false};
  for (uint64_t o = 0, k = 0; o < n && e == hipSuccess; o += slab_bytes, k++) {
    const uint64_t len = std::min(slab_bytes, n - o);
    if (used[k & 1] && (e = hipEventSynchronize(done[k & 1])) != hipSuccess) break;
    uint8_t *buf = stage + (k & 1) * slab_bytes;
    copy_box_runs(R, const_cast<uint8_t *>(host_array), buf, o, o + len, false, threads);
    if ((e = hipMemcpyAsync(dev_compact + o, buf, len, hipMemcpyHostToDevice, s)) != hipSuccess) break;
    e = hipEventRecord(done[k & 1], s);
    used[k & 1] = true;
  }
  if (e == hipSuccess) e = hipStreamSynchronize(s);
  for (int k = 0; k < 2; k++) (void)hipEventDestroy(done[k]);
  return e;
}

}  // namespace zgpu
