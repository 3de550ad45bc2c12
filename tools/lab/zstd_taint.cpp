// Analysis (not product code): how much of a C5 level-0 zstd frame depends, through match chains,
// on bytes before the start of its own segment when the frame is cut into S segments.
// Build: g++ -O2 -fopenmp zstd_taint.cpp -L../synth -lsynth -Wl,-rpath,$ORIGIN/../synth -l:libzstd.so.1
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
#include <algorithm>
extern "C" {
void synth_c5_level0(uint64_t nz, uint64_t ny, uint64_t nx, int nblobs, const float *cz, const float *cy,
                     const float *cx, const float *sg, const float *amp, uint64_t seed, uint16_t *out, int nt);
typedef struct ZSTD_CCtx_s ZSTD_CCtx;
ZSTD_CCtx *ZSTD_createCCtx(void);
size_t ZSTD_CCtx_setParameter(ZSTD_CCtx *, int, int);
typedef struct { unsigned offset, litLength, matchLength, rep; } ZSTD_Sequence;
size_t ZSTD_generateSequences(ZSTD_CCtx *, ZSTD_Sequence *, size_t, const void *, size_t);
unsigned ZSTD_isError(size_t);
}
int main(int argc, char **argv) {
  const int chunk = argc > 1 ? atoi(argv[1]) : 0;
  std::mt19937_64 g(42);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  float cz[64], cy[64], cx[64], sg[64], amp[64];
  for (int b = 0; b < 64; b++) {
    cz[b] = 512 * u(g); cy[b] = 1024 * u(g); cx[b] = 1024 * u(g);
    sg[b] = 4 + 36 * u(g); amp[b] = 300 + 3700 * u(g);
  }
  std::vector<uint16_t> lvl((size_t)512 * 1024 * 1024);
  synth_c5_level0(512, 1024, 1024, 64, cz, cy, cx, sg, amp, 42, lvl.data(), 8);
  const int level = argc > 2 ? atoi(argv[2]) : 0;  // 1: a chunk [64,256,256] of the 2x2x2 mean level
  const int c = chunk;
  const int ncz = level ? 64 : 32, ncy = level ? 256 : 512;
  const int z0 = (c / 4) * ncz, y0 = ((c / 2) % 2) * ncy, x0 = (c % 2) * ncy;
  const uint64_t cnt = (uint64_t)ncz * ncy * ncy, N = 2 * cnt;
  std::vector<uint8_t> d(N);
  uint64_t i = 0;
  for (int z = 0; z < ncz; z++)
    for (int y = 0; y < ncy; y++)
      for (int x = 0; x < ncy; x++, i++) {
        uint32_t v;
        if (!level) {
          v = lvl[((uint64_t)(z0 + z) * 1024 + (y0 + y)) * 1024 + (x0 + x)];
        } else {
          uint32_t sum = 0;
          for (int k = 0; k < 8; k++)
            sum += lvl[((uint64_t)(2 * (z0 + z) + (k >> 2)) * 1024 + (2 * (y0 + y) + ((k >> 1) & 1))) * 1024 +
                       (2 * (x0 + x) + (k & 1))];
          v = sum / 8;
        }
        d[i] = (uint8_t)v; d[cnt + i] = (uint8_t)(v >> 8);
      }
  ZSTD_CCtx *cc = ZSTD_createCCtx();
  ZSTD_CCtx_setParameter(cc, 100, 3);
  std::vector<ZSTD_Sequence> s(N / 2);
  size_t ns = ZSTD_generateSequences(cc, s.data(), s.size(), d.data(), N);
  if (ZSTD_isError(ns)) { printf("generateSequences failed\n"); return 1; }
  uint64_t nm = 0, mb = 0, lb = 0;
  for (size_t k = 0; k < ns; k++) { lb += s[k].litLength; if (s[k].matchLength) { nm++; mb += s[k].matchLength; } }
  {
    uint64_t p = 0, lo_seq = 0, cross = 0;
    for (size_t k = 0; k < ns; k++) {
      p += s[k].litLength;
      if (p < N / 2) lo_seq++;
      if (s[k].matchLength && p >= N / 2 && p - s[k].offset < N / 2) cross++;
      p += s[k].matchLength;
    }
    printf("sequences starting in the low plane %lu of %zu; matches crossing into it from the high plane %lu\n", lo_seq, ns, cross);
  }
  printf("chunk %d: %zu sequences, %lu matches, match bytes %lu, literal bytes %lu (total %lu)\n", c, ns, nm, mb, lb, N);
  {  // offset / length histogram of the matches
    const uint64_t lim[] = {1, 2, 4, 8, 16, 64, 256, 511, 512, 513, 1024, 4096, 65536, 262144, 1ull << 40};
    uint64_t hc[16] = {}, hb[16] = {}, lc[8] = {};
    for (size_t k = 0; k < ns; k++) {
      if (!s[k].matchLength) continue;
      int b = 0; while (s[k].offset > lim[b]) b++;
      hc[b]++; hb[b] += s[k].matchLength;
      const unsigned ml = s[k].matchLength;
      lc[ml < 8 ? 0 : ml < 16 ? 1 : ml < 32 ? 2 : ml < 64 ? 3 : ml < 256 ? 4 : ml < 1024 ? 5 : ml < 4096 ? 6 : 7]++;
    }
    for (int b = 0; b < 15; b++) if (hc[b]) printf("  offset <= %llu: %lu matches, %lu bytes\n", (unsigned long long)lim[b], hc[b], hb[b]);
    printf("  match length <8 %lu, <16 %lu, <32 %lu, <64 %lu, <256 %lu, <1K %lu, <4K %lu, >=4K %lu\n", lc[0], lc[1], lc[2], lc[3], lc[4], lc[5], lc[6], lc[7]);
  }
  {  // resolution rounds of k_zstd_exec_item's batches: the frontier rule vs exact dependencies
    const uint32_t ZB = 4096, BIG = 2048;
    uint64_t rf = 0, rp = 0, nbat = 0, pos = 0, maxp = 0, maxs = 0, rsp = 0, hist[5] = {};
    size_t k = 0;
    while (k < ns) {
      // one batch: up to 64 sequences, output span <= ZB, stopping before a big one / block end
      std::vector<uint64_t> ms, src;
      std::vector<uint32_t> n;
      uint64_t span = 0;
      size_t k0 = k;
      while (k < ns && ms.size() < 64) {
        const ZSTD_Sequence &q = s[k];
        if (q.litLength >= BIG || q.matchLength >= BIG) break;
        if (span + q.litLength + q.matchLength > ZB) break;
        span += q.litLength + q.matchLength;
        ms.push_back(pos + span - q.matchLength);
        src.push_back(pos + span - q.matchLength - q.offset);
        n.push_back(q.matchLength);
        k++;
        if (!q.matchLength) break;  // block delimiter / last literals
      }
      if (k == k0) { pos += s[k].litLength + s[k].matchLength; k++; continue; }  // single (big) sequence
      pos += span;
      nbat++;
      const int m = (int)ms.size();
      std::vector<bool> pend(m);
      for (int j = 0; j < m; j++) pend[j] = n[j] > 0;
      // frontier rule
      std::vector<bool> pf = pend;
      while (true) {
        int first = -1;
        for (int j = 0; j < m; j++) if (pf[j]) { first = j; break; }
        if (first < 0) break;
        const uint64_t F = ms[first];
        std::vector<bool> rdy(m);
        for (int j = 0; j < m; j++) {
          const uint64_t cl = std::min<uint64_t>(n[j], ms[j] - src[j]);
          rdy[j] = pf[j] && (j == first || src[j] + cl <= F);
        }
        for (int j = 0; j < m; j++) if (rdy[j]) pf[j] = false;
        rf++;
      }
      // exact rule: ready when no pending match's destination overlaps the external source bytes
      std::vector<bool> pe = pend;
      while (true) {
        bool any = false;
        for (int j = 0; j < m; j++) any = any || pe[j];
        if (!any) break;
        std::vector<bool> rdy(m);
        for (int j = 0; j < m; j++) {
          if (!pe[j]) continue;
          const uint64_t a = src[j], b = src[j] + std::min<uint64_t>(n[j], ms[j] - src[j]);
          bool ok = true;
          for (int i = 0; i < j; i++) if (pe[i] && ms[i] < b && ms[i] + n[i] > a) ok = false;
          rdy[j] = ok;
        }
        uint32_t mx = 0, ms_ = 0; bool sp = false;
        for (int j = 0; j < m; j++) if (rdy[j]) {
          const uint32_t d = (uint32_t)(ms[j] - src[j]);
          if (d < n[j] && d < 16) { sp = true; ms_ = std::max(ms_, (n[j] + 15) / 16); }
          else mx = std::max(mx, (n[j] + 15) / 16);
        }
        maxp += mx; maxs += ms_; rsp += sp;
        hist[std::min<uint32_t>(mx, 32) / 8]++;
        for (int j = 0; j < m; j++) if (rdy[j]) pe[j] = false;
        rp++;
      }
    }
    {
      uint64_t c[5] = {}, bsum[5] = {};
      for (size_t q = 0; q < ns; q++) {
        const unsigned n = s[q].matchLength, d = s[q].offset;
        if (!n) continue;
        const int cls = n > 512 ? 4 : (d < n && n > 16 && (d == 1 || d == 2 || d == 4 || d == 8)) ? 0 : d >= n ? 1 : d < 16 ? 2 : 3;
        c[cls]++; bsum[cls] += n;
      }
      printf("  matches: splat %lu (%lu B), straight %lu (%lu B), overlap d<16 %lu (%lu B), overlap d>=16 %lu (%lu B), >512 B %lu (%lu B)\n",
             c[0], bsum[0], c[1], bsum[1], c[2], bsum[2], c[3], bsum[3], c[4], bsum[4]);
    }
    printf("  batches %lu, rounds: frontier rule %lu, exact dependencies %lu\n", nbat, rf, rp);
    printf("  exact rounds: sum of max straight pieces %lu, sum of max period pieces %lu, rounds with a period copy %lu; max pieces <8 %lu, <16 %lu, <24 %lu, <32 %lu, 32 %lu\n",
           maxp, maxs, rsp, hist[0], hist[1], hist[2], hist[3], hist[4]);
  }
  for (int S : {2, 4, 8, 16, 32, 128}) {
    const uint64_t seg = N / S;
    std::vector<uint8_t> t(N, 0);  // taint: derives from before own segment start
    std::vector<uint64_t> first_clean(S, 0), tainted(S, 0), tmatch(S, 0);
    uint64_t p = 0;
    for (size_t k = 0; k < ns; k++) {
      p += s[k].litLength;
      for (unsigned m = 0; m < s[k].matchLength; m++, p++) {
        const uint64_t src = p - s[k].offset, ss = (p / seg) * seg;
        t[p] = src < ss ? 1 : t[src];
      }
    }
    uint64_t tot = 0, lastpos = 0;
    for (uint64_t q = 0; q < N; q++) if (t[q]) { tot++; tainted[q / seg]++; if (q % seg > lastpos) lastpos = q % seg; }
    printf("S=%3d: tainted %.3f%% of bytes; worst segment %.3f%%; deepest tainted offset in a segment %lu of %lu\n", S,
           100.0 * tot / N, 100.0 * [&] { uint64_t w = 0; for (auto x : tainted) w = x > w ? x : w; return w; }() / seg,
           lastpos, seg);
  }
  return 0;
}
