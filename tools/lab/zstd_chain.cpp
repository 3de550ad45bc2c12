// Analysis (not product code): LZ77 dependency chains of C5-like zstd frames, to size an intra-frame
// parallel executor. For every output byte: its chain depth (match hops until a literal byte) and
// whether the chain leaves the byte's 128 KiB block; per block-parallel round count.
// Build: g++ -O2 -fopenmp zstd_chain.cpp -L../synth -lsynth -Wl,-rpath,$ORIGIN/../synth -l:libzstd.so.1 -o zstd_chain
// Run: ./zstd_chain <chunk> <level 0|1> [zstd level]
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>
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
  const int c = argc > 1 ? atoi(argv[1]) : 0;
  const int level = argc > 2 ? atoi(argv[2]) : 0;
  const int zl = argc > 3 ? atoi(argv[3]) : 3;
  std::mt19937_64 g(42);
  std::uniform_real_distribution<float> u(0.f, 1.f);
  float cz[64], cy[64], cx[64], sg[64], amp[64];
  for (int b = 0; b < 64; b++) {
    cz[b] = 512 * u(g); cy[b] = 1024 * u(g); cx[b] = 1024 * u(g);
    sg[b] = 4 + 36 * u(g); amp[b] = 300 + 3700 * u(g);
  }
  std::vector<uint16_t> lvl((size_t)512 * 1024 * 1024);
  synth_c5_level0(512, 1024, 1024, 64, cz, cy, cx, sg, amp, 42, lvl.data(), 8);
  // level L: the 2^L mean of L0 ([512,1024,1024] here); chunk shapes as bench C5
  const int czs[5] = {32, 64, 64, 64, 32}, cys[5] = {512, 256, 128, 64, 64};
  const int ncz = czs[level], ncy = cys[level], f = 1 << level;
  const int gz = (512 / f) / ncz, gy = (1024 / f) / ncy;
  const int z0 = (c / (gy * gy)) % gz * ncz, y0 = (c / gy) % gy * ncy, x0 = c % gy * ncy;
  const uint64_t cnt = (uint64_t)ncz * ncy * ncy, N = 2 * cnt;
  std::vector<uint8_t> d(N);
  uint64_t i = 0;
  for (int z = 0; z < ncz; z++)
    for (int y = 0; y < ncy; y++)
      for (int x = 0; x < ncy; x++, i++) {
        uint64_t sum = 0;
        for (int a = 0; a < f; a++)
          for (int b = 0; b < f; b++)
            for (int e = 0; e < f; e++)
              sum += lvl[((uint64_t)((z0 + z) * f + a) * 1024 + ((y0 + y) * f + b)) * 1024 + ((x0 + x) * f + e)];
        const uint32_t v = (uint32_t)(sum / ((uint64_t)f * f * f));
        d[i] = (uint8_t)v; d[cnt + i] = (uint8_t)(v >> 8);
      }
  ZSTD_CCtx *cc = ZSTD_createCCtx();
  ZSTD_CCtx_setParameter(cc, 100, zl);
  std::vector<ZSTD_Sequence> s(N / 2);
  size_t ns = ZSTD_generateSequences(cc, s.data(), s.size(), d.data(), N);
  if (ZSTD_isError(ns)) { printf("generateSequences failed\n"); return 1; }
  // per byte: source (p - off) or literal; depth; leaves-block
  std::vector<uint32_t> depth(N, 0), exitb(N, 0);  // exitb: 1 if the chain leaves the byte's block
  std::vector<uint32_t> srcp(N, 0xFFFFFFFFu);
  uint64_t p = 0, nm = 0, mb = 0, lb = 0, shortm = 0;
  std::vector<uint64_t> offh(8, 0);  // offsets: 1-3, 4-15, 16-255, 256-4095, 4K-64K, 64K+
  for (size_t k = 0; k < ns; k++) {
    p += s[k].litLength;
    lb += s[k].litLength;
    if (s[k].matchLength) {
      nm++;
      mb += s[k].matchLength;
      if (s[k].matchLength < 16) shortm++;
      const uint32_t o = s[k].offset;
      offh[o < 4 ? 0 : o < 16 ? 1 : o < 256 ? 2 : o < 4096 ? 3 : o < 65536 ? 4 : 5]++;
      for (uint32_t j = 0; j < s[k].matchLength; j++) srcp[p + j] = (uint32_t)(p + j - o);
      p += s[k].matchLength;
    }
  }
  const uint64_t BLK = 131072;
  uint32_t maxd = 0;
  std::vector<uint64_t> dh(32, 0);
  uint64_t nexit = 0, nmatchb = 0;
  std::vector<uint32_t> exit_hops(N, 0);  // block boundaries crossed along the chain
  uint32_t max_hops = 0;
  for (uint64_t q = 0; q < N; q++) {
    if (srcp[q] == 0xFFFFFFFFu) continue;
    nmatchb++;
    const uint32_t sp = srcp[q];
    depth[q] = depth[sp] + 1;
    const bool leaves = sp / BLK != q / BLK;
    exitb[q] = leaves || exitb[sp];
    exit_hops[q] = exit_hops[sp] + (sp / BLK != q / BLK ? (uint32_t)(q / BLK - sp / BLK) : 0);
    max_hops = std::max(max_hops, exit_hops[q]);
    nexit += exitb[q];
    maxd = std::max(maxd, depth[q]);
    int lg = 0;
    while ((1u << lg) <= depth[q]) lg++;
    dh[lg]++;
  }
  printf("chunk %d level %d zstd %d: %llu bytes, %zu sequences, %llu matches (%llu < 16 B), literals %llu (%.1f%%), "
         "mean match %.1f B\n",
         c, level, zl, (unsigned long long)N, ns, (unsigned long long)nm, (unsigned long long)shortm,
         (unsigned long long)lb, 100.0 * lb / N, nm ? (double)mb / nm : 0.0);
  printf("offsets: 1-3 %llu, 4-15 %llu, 16-255 %llu, 256-4095 %llu, 4K-64K %llu, 64K+ %llu\n",
         (unsigned long long)offh[0], (unsigned long long)offh[1], (unsigned long long)offh[2],
         (unsigned long long)offh[3], (unsigned long long)offh[4], (unsigned long long)offh[5]);
  printf("match bytes %llu; max chain depth %u (pointer-doubling rounds %d); chain leaves its 128 KiB block: %llu "
         "bytes (%.1f%% of all); max blocks crossed %u\n",
         (unsigned long long)nmatchb, maxd, [&] { int r = 0; while ((1u << r) <= maxd) r++; return r; }(),
         (unsigned long long)nexit, 100.0 * nexit / N, max_hops);
  printf("depth histogram (by log2 bucket):");
  for (int k = 0; k < 32; k++)
    if (dh[k]) printf(" [<%u]=%llu", 1u << k, (unsigned long long)dh[k]);
  printf("\n");
  // match-granular multi-round resolution: round of a match = 1 + max round of the matches its
  // source bytes lie in (literal bytes: round 0)
  std::vector<uint32_t> round_of(N, 0);
  uint32_t maxr = 0;
  p = 0;
  for (size_t k = 0; k < ns; k++) {
    p += s[k].litLength;
    if (s[k].matchLength) {
      uint32_t r = 0;
      const uint32_t o = s[k].offset;
      for (uint32_t j = 0; j < std::min<uint32_t>(s[k].matchLength, o); j++) r = std::max(r, round_of[p + j - o]);
      r += 1;
      for (uint32_t j = 0; j < s[k].matchLength; j++) round_of[p + j] = r;
      maxr = std::max(maxr, r);
      p += s[k].matchLength;
    }
  }
  printf("match-granular resolution rounds (whole frame): %u\n", maxr);
  {  // sequences per 128 KiB block (by the sequence's start)
    std::vector<uint32_t> per(N / BLK + 1, 0);
    uint64_t q = 0;
    for (size_t k = 0; k < ns; k++) { per[q / BLK]++; q += s[k].litLength + s[k].matchLength; }
    uint32_t mx = 0; uint64_t tot = 0;
    for (uint32_t v : per) { mx = std::max(mx, v); tot += v; }
    printf("sequences per 128 KiB block: mean %.0f max %u (blocks %zu)\n", (double)tot / per.size(), mx, per.size());
  }
  // windowed pointer doubling (the k_zstd_exec_win model): windows of W bytes in order; a match byte
  // whose (period-reduced) source lies before the window takes the final value, else it points into
  // the window; synchronous doubling rounds until every cell holds a value
  for (uint32_t W : {8192u, 16384u, 32768u}) {
    std::vector<uint8_t> out(N, 0);
    std::vector<uint32_t> cell(W), nxt(W);  // bit 31: resolved (value in low 8 bits), else window index
    std::vector<uint32_t> sstart(ns), sml(ns), sof(ns);
    uint64_t pp = 0;
    for (size_t k = 0; k < ns; k++) {
      pp += s[k].litLength;
      sstart[k] = (uint32_t)pp;
      sml[k] = s[k].matchLength;
      sof[k] = s[k].offset;
      pp += s[k].matchLength;
    }
    // per byte: match index or literal
    std::vector<int32_t> mof(N, -1);
    for (size_t k = 0; k < ns; k++)
      for (uint32_t j = 0; j < sml[k]; j++) mof[sstart[k] + j] = (int32_t)k;
    uint64_t rounds_total = 0, nwin = 0, bad = 0;
    uint32_t rounds_max = 0;
    for (uint64_t w0 = 0; w0 < N; w0 += W) {
      const uint32_t wn = (uint32_t)std::min<uint64_t>(W, N - w0);
      uint32_t unres = 0;
      for (uint32_t t = 0; t < wn; t++) {
        const uint64_t q = w0 + t;
        const int32_t k = mof[q];
        if (k < 0) { cell[t] = 0x80000000u | d[q]; continue; }
        const uint64_t ms = sstart[k], of = sof[k];
        uint64_t src = q - of;
        if (of < sml[k]) src = ms - of + ((q - ms) % of);  // period reduction: source before the match
        if (src < w0) cell[t] = 0x80000000u | out[src];
        else { cell[t] = (uint32_t)(src - w0); unres++; }
      }
      uint32_t r = 0;
      while (unres) {
        unres = 0;
        for (uint32_t t = 0; t < wn; t++) {
          const uint32_t c = cell[t];
          if (c & 0x80000000u) { nxt[t] = c; continue; }
          const uint32_t cq = cell[c];
          nxt[t] = (cq & 0x80000000u) ? cq : cq;  // value, or the pointer one hop further
          if (!(nxt[t] & 0x80000000u)) unres++;
        }
        std::swap(cell, nxt);
        r++;
      }
      for (uint32_t t = 0; t < wn; t++) {
        out[w0 + t] = (uint8_t)cell[t];
        bad += out[w0 + t] != d[w0 + t];
      }
      rounds_total += r;
      rounds_max = std::max(rounds_max, r);
      nwin++;
    }
    printf("window %5u: %llu windows, doubling rounds mean %.2f max %u, mismatches %llu\n", W,
           (unsigned long long)nwin, (double)rounds_total / nwin, rounds_max, (unsigned long long)bad);
  }
  return 0;
}
