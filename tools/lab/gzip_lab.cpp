// Lab harness (not product code): times the gzip inflate kernel on C3-like inner chunks
// (32^3 f32, gzip level 1) and prints the per-phase shader-clock profile (ZG_PROFILE build).
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fopenmp -DZG_PROFILE -I../../zarrs_amd/csrc \
//        -x hip -o gzip_lab gzip_lab.cpp -lz
#include <hip/hip_runtime.h>
#include <zlib.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "common.hpp"
#ifdef INFLATE_SRC
#include INFLATE_SRC
#else
#include "kernels/inflate.hip"  // the product kernel source, built here with ZG_PROFILE
#endif

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

static uint64_t mix64(uint64_t x) {
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull; x ^= x >> 27; x *= 0x94d049bb133111ebull; x ^= x >> 31; return x;
}
static float hnorm(uint64_t key) {
  uint64_t h = mix64(key);
  float s = (float)(h & 0xFFFF) + (float)((h >> 16) & 0xFFFF) + (float)((h >> 32) & 0xFFFF) + (float)(h >> 48);
  return (s / 65535.0f - 2.0f) * 1.7320508f;
}
static float c3v(uint64_t x, uint64_t y, uint64_t z) {
  float s = sinf(0.05f * x) + cosf(0.03f * y) + 0.5f * sinf(0.07f * z);
  return rintf(256.0f * s + hnorm((x * 2048ull + y) * 2048ull + z + 7ull * 0x9E3779B97F4A7C15ull)) / 256.0f;
}

int main(int argc, char **argv) {
  setvbuf(stdout, NULL, _IOLBF, 0);
  const int n = argc > 1 ? atoi(argv[1]) : 8192;
  const int level = argc > 2 ? atoi(argv[2]) : 1;
  const int E = 32, NB = E * E * E * 4;
  std::vector<std::vector<uint8_t>> enc(n);
  std::vector<float> dec((size_t)n * E * E * E);
  size_t total = 0;
#pragma omp parallel for reduction(+ : total)
  for (int c = 0; c < n; c++) {
    const uint64_t ox = (c % 64) * E, oy = ((c / 64) % 64) * E, oz = (c / 4096) * E;
    float *d = &dec[(size_t)c * E * E * E];
    for (int i = 0; i < E; i++)
      for (int j = 0; j < E; j++)
        for (int k = 0; k < E; k++) d[(i * E + j) * E + k] = c3v(ox + i, oy + j, oz + k);
    z_stream s;
    memset(&s, 0, sizeof(s));
    deflateInit2(&s, level, Z_DEFLATED, 31, 8, Z_DEFAULT_STRATEGY);
    enc[c].resize(NB + NB / 8 + 1024);
    s.next_in = (Bytef *)d; s.avail_in = NB; s.next_out = enc[c].data(); s.avail_out = enc[c].size();
    deflate(&s, Z_FINISH);
    enc[c].resize(s.total_out);
    deflateEnd(&s);
    total += s.total_out;
  }
  if (getenv("LAB_SAME")) {  // every chunk a copy of chunk LAB_SAME (content variance out of the timing)
    const int src = atoi(getenv("LAB_SAME")) % n;
    total = 0;
    for (int c = 0; c < n; c++) {
      enc[c] = enc[src];
      memcpy(&dec[(size_t)c * E * E * E], &dec[(size_t)src * E * E * E], NB);
      total += enc[c].size();
    }
  }
  printf("%d chunks, %.1f MiB encoded, ratio %.3f\n", n, total / 1048576.0, (double)n * NB / total);
  // pack encoded (256-B aligned) on device
  std::vector<uint64_t> off(n);
  size_t o = 0;
  for (int c = 0; c < n; c++) { off[c] = o; o += (enc[c].size() + 255) & ~255ull; }
  std::vector<uint8_t> packed(o);
  for (int c = 0; c < n; c++) memcpy(&packed[off[c]], enc[c].data(), enc[c].size());
  uint8_t *d_enc, *d_out;
  CK(hipMalloc(&d_enc, o));
  CK(hipMemcpy(d_enc, packed.data(), o, hipMemcpyHostToDevice));
  const uint64_t slot = NB;
  CK(hipMalloc(&d_out, (size_t)n * slot));
  std::vector<ZgItem> items(n);
  for (int c = 0; c < n; c++) items[c] = ZgItem{(uint64_t)(d_enc + off[c]), enc[c].size(), (uint32_t)c, 0, 0, 0};
  ZgItem *d_items;
  uint32_t *d_status;
  uint2 *d_aux;
  CK(hipMalloc(&d_items, n * sizeof(ZgItem)));
  CK(hipMalloc(&d_status, n * 4));
  CK(hipMalloc(&d_aux, n * 8));
  uint32_t *d_seg = nullptr;  // segmented symbol decode scratch (ZGPU_GZIP_SEG=0: the lookahead path)
  if (const uint64_t b = zgpu::gzip_seg_scratch_bytes(n)) CK(hipMalloc(&d_seg, b));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e30f;
  for (int rep = 0; rep < 3; rep++) {
    CK(hipMemcpy(d_items, items.data(), n * sizeof(ZgItem), hipMemcpyHostToDevice));
    CK(hipMemset(d_status, 0, n * 4));
#ifdef ZG_PROFILE
    unsigned long long z[16] = {0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(zgpu::g_prof), z, sizeof(z)));
#endif
    CK(hipEventRecord(e0));
    CK(zgpu::launch_gzip(d_items, d_status, n, d_out, slot, nullptr, d_seg, 0));
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    if (ms < best) best = ms;
  }
  if (getenv("LAB_EACH")) {  // every stream alone: the per-stream latency distribution
    std::vector<std::pair<float, int>> t(n);
    for (int c = 0; c < n; c++) {
      float b1 = 1e30f;
      for (int rep = 0; rep < 2; rep++) {
        CK(hipMemcpy(d_items + c, &items[c], sizeof(ZgItem), hipMemcpyHostToDevice));
        CK(hipMemset(d_status + c, 0, 4));
        CK(hipEventRecord(e0));
        CK(zgpu::launch_gzip(d_items + c, d_status + c, 1, d_out + (size_t)c * slot, slot, nullptr, d_seg, 0));
        CK(hipEventRecord(e1));
        CK(hipEventSynchronize(e1));
        float ms; CK(hipEventElapsedTime(&ms, e0, e1));
        b1 = std::min(b1, ms);
      }
      t[c] = {b1, c};
    }
    std::sort(t.begin(), t.end());
    printf("per-stream latency: min %.3f  p50 %.3f  p90 %.3f  p99 %.3f  max %.3f ms\n", t[0].first, t[n / 2].first,
           t[n * 9 / 10].first, t[n * 99 / 100].first, t[n - 1].first);
    for (int k = n - 1; k >= 0 && k >= n - 6; k--)
      printf("  slow: chunk %d %.3f ms, %zu B encoded\n", t[k].second, t[k].first, enc[t[k].second].size());
  }
  unsigned long long prof[16] = {0, 0, 0, 0, 1};
#ifdef ZG_PROFILE
  CK(hipMemcpyFromSymbol(prof, HIP_SYMBOL(zgpu::g_prof), sizeof(prof)));
#endif
  std::vector<uint32_t> st(n);
  CK(hipMemcpy(st.data(), d_status, n * 4, hipMemcpyDeviceToHost));
  std::vector<float> out((size_t)n * E * E * E);
  CK(hipMemcpy(out.data(), d_out, (size_t)n * slot, hipMemcpyDeviceToHost));
  int bad = 0;
  for (int c = 0; c < n; c++) if (st[c] || memcmp(&out[(size_t)c * E * E * E], &dec[(size_t)c * E * E * E], NB)) bad++;
  printf("k_gzip: %.3f ms  %.2f GB/s decoded  %.2f GB/s encoded  bad=%d\n", best, (double)n * NB / best / 1e6,
         (double)total / best / 1e6, bad);
  const double tot = (double)prof[4];
  const char *names[] = {"hdr+tables", "sym decode", "execute", "repairs", "total"};
  for (int i = 0; i < 5; i++)
    if (i == 3)
      printf("  %-12s %.1f per chunk (segmented decode: lanes re-decoded from their predecessor's exit)\n", names[i],
             (double)prof[i] / n);
    else
      printf("  %-12s %6.1f%%  %.0f cycles/chunk\n", names[i], 100.0 * prof[i] / tot, (double)prof[i] / n);
  if (prof[12])
    printf("  header detail: %.1f blocks/chunk; per chunk cycles: code lengths %.0f, litlen table %.0f, dist table %.0f, "
           "trailer crc %.0f\n", (double)prof[12] / n, (double)prof[8] / n, (double)prof[9] / n, (double)prof[10] / n,
           (double)prof[11] / n);
  if (prof[13])
    printf("  segmented decode: %.1f rounds/chunk, repair loop %.0f cycles/chunk, slow-path fallbacks %.2f/chunk\n",
           (double)prof[13] / n, (double)prof[14] / n, (double)prof[15] / n);
  if (prof[6])
    printf("  per chunk: %.0f batches, %.1f symbols/batch, %.2f match rounds/batch\n", (double)prof[6] / n,
           (double)prof[7] / prof[6], (double)prof[5] / prof[6]);
  return bad ? 1 : 0;
}
