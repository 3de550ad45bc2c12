// Lab harness (not product code): the block-parallel zstd path on C5-like chunks (byte-shuffled
// uint16 blob field + noise, zstd level 3), per-kernel times and, in a ZG_PROFILE build, the
// per-phase shader-clock profile of k_zstd_exec.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -fopenmp [-DZG_PROFILE] -I../../zarrs_amd/csrc \
//        -x hip -o zstd_lab zstd_lab.cpp -L../synth -lsynth -Wl,-rpath,'$ORIGIN/../synth' -l:libzstd.so.1
// Run: ./zstd_lab <chunks> <MiB per chunk> [level] [c5]   (c5: bench-like data, 16 MiB chunks)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "common.hpp"
#include "kernels/zstd.hip"

typedef struct ZSTD_CCtx_s ZSTD_CCtx;
extern "C" {
void synth_c5_level0(uint64_t nz, uint64_t ny, uint64_t nx, int nblobs, const float *cz, const float *cy,
                     const float *cx, const float *sg, const float *amp, uint64_t seed, uint16_t *out, int nthreads);
unsigned ZSTD_isError(size_t code);
ZSTD_CCtx *ZSTD_createCCtx(void);
size_t ZSTD_freeCCtx(ZSTD_CCtx *);
size_t ZSTD_CCtx_setParameter(ZSTD_CCtx *, int param, int value);
size_t ZSTD_compress2(ZSTD_CCtx *, void *dst, size_t cap, const void *src, size_t n);
size_t ZSTD_compressBound(size_t srcSize);
}

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

int main(int argc, char **argv) {
  setvbuf(stdout, NULL, _IOLBF, 0);
  const int n = argc > 1 ? atoi(argv[1]) : 64;
  // argv[4] == "bz": the blosc-zstd bench's streams: 256 KiB byte-shuffled blocks (2 z-slices of a
  // [64,256,256] chunk of the u16 volume [1024,2048,1024]) at zstd level 9 (c-blosc clevel 5)
  const bool bz = argc > 4 && !strcmp(argv[4], "bz");
  // argv[4] == "c5lL", L = 0..4: chunks of bench C5's level L (the 2^L mean of level 0), as bench.py
  // cuts them: [32,512,512], [64,256,256], [64,128,128], [64,64,64], [32,64,64] (argv[2] ignored)
  const int clev = argc > 4 && !strncmp(argv[4], "c5l", 3) ? atoi(argv[4] + 3) : !(argc > 4 && !strcmp(argv[4], "c5")) ? -1 : 0;
  const int czs[5] = {32, 64, 64, 64, 32}, cys[5] = {512, 256, 128, 64, 64};
  const uint64_t chunk = bz ? 262144ull
                         : clev >= 0 ? 2ull * czs[clev] * cys[clev] * cys[clev]
                                     : (uint64_t)(argc > 2 ? atoll(argv[2]) : 16) << 20;  // bytes
  const int level = bz ? 9 : argc > 3 ? atoi(argv[3]) : 3;
  // argv[4] == "c5": chunks [32,512,512] of a bench-like C5 level 0 ([512,1024,1024], 64 blobs)
  // argv[4] == "c5l1": chunks [64,256,256] of the 2x2x2 mean of that level (8 MiB each)
  const bool c5 = clev >= 0;
  std::vector<uint16_t> lvl;
  if (c5) {
    std::mt19937_64 g(42);
    std::uniform_real_distribution<float> u(0.f, 1.f);
    float cz[64], cy[64], cx[64], sg[64], amp[64];
    for (int b = 0; b < 64; b++) {
      cz[b] = 512 * u(g); cy[b] = 1024 * u(g); cx[b] = 1024 * u(g);
      sg[b] = 4 + 36 * u(g); amp[b] = 300 + 3700 * u(g);
    }
    lvl.resize((size_t)512 * 1024 * 1024);
    synth_c5_level0(512, 1024, 1024, 64, cz, cy, cx, sg, amp, 42, lvl.data(), 16);
  }
  std::vector<std::vector<uint8_t>> dec(n), enc(n);
  // c5 modes: chunks past the 64 distinct ones repeat them (throughput at scale)
  const int gz = c5 ? (512 >> clev) / czs[clev] : 1, gy = c5 ? (1024 >> clev) / cys[clev] : 1;
  const int ndist = c5 ? std::min(n, gz * gy * gy) : n;  // the chunks the level holds
#pragma omp parallel for
  for (int c = 0; c < ndist; c++) {
    if (c5) {
      const int ncz = czs[clev], ncy = cys[clev], f = 1 << clev;
      const int z0 = (c / (gy * gy)) % gz * ncz, y0 = (c / gy) % gy * ncy, x0 = c % gy * ncy;
      const uint64_t cnt = (uint64_t)ncz * ncy * ncy;
      dec[c].resize(2 * cnt);
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
            dec[c][i] = (uint8_t)v;
            dec[c][cnt + i] = (uint8_t)(v >> 8);
          }
      ZSTD_CCtx *cc = ZSTD_createCCtx();
      ZSTD_CCtx_setParameter(cc, 100, level);
      enc[c].resize(ZSTD_compressBound(2 * cnt));
      enc[c].resize(ZSTD_compress2(cc, enc[c].data(), enc[c].size(), dec[c].data(), 2 * cnt));
      ZSTD_freeCCtx(cc);
      continue;
    }
    std::mt19937_64 rng(1234 + c);
    std::normal_distribution<float> nd(0.f, 1.f);
    const uint64_t cnt = chunk / 2;
    std::vector<uint16_t> v(cnt);
    if (bz) {
      const int ci = c / 32, b = c % 32;
      const int z0 = 64 * ((ci / 32) % 16) + 2 * b, y0 = 256 * ((ci / 4) % 8), x0 = 256 * (ci % 4);
      for (uint64_t i = 0; i < cnt; i++) {
        const float z = (float)(z0 + (int)(i >> 16)), y = (float)(y0 + (int)((i >> 8) & 255)), x = (float)(x0 + (int)(i & 255));
        const float m = 100.f + 900.f * fabsf(sinf(z * 0.05f) * cosf(y * 0.013f) * sinf(x * 0.021f));
        v[i] = (uint16_t)fminf(fmaxf(m + nd(rng) * sqrtf(m), 0.f), 65535.f);
      }
    }
    for (uint64_t i = 0; !bz && i < cnt; i++) {
      const float x = (float)(i % 512), y = (float)((i / 512) % 512);
      const float m = 100.f + 3000.f * expf(-((x - 200) * (x - 200) + (y - 300) * (y - 300)) / (2 * 40.f * 40.f));
      float val = rintf(m + sqrtf(m) * nd(rng));
      v[i] = (uint16_t)fminf(fmaxf(val, 0.f), 65535.f);
    }
    dec[c].resize(chunk);
    const uint8_t *b = (const uint8_t *)v.data();
    for (uint64_t i = 0; i < cnt; i++) { dec[c][i] = b[2 * i]; dec[c][cnt + i] = b[2 * i + 1]; }
    ZSTD_CCtx *cc = ZSTD_createCCtx();
    ZSTD_CCtx_setParameter(cc, 100, level);
    enc[c].resize(ZSTD_compressBound(chunk));
    size_t r = ZSTD_compress2(cc, enc[c].data(), enc[c].size(), dec[c].data(), chunk);
    enc[c].resize(r);
    ZSTD_freeCCtx(cc);
  }
  for (int c = ndist; c < n; c++) {
    dec[c] = dec[c % ndist];
    enc[c] = enc[c % ndist];
  }
  uint64_t total = 0;
  std::vector<uint64_t> off(n);
  for (int c = 0; c < n; c++) { off[c] = total; total += (enc[c].size() + 255) & ~255ull; }
  printf("%d chunks of %.1f MiB, %.1f MiB encoded (ratio %.3f)\n", n, chunk / 1048576.0, total / 1048576.0,
         (double)n * chunk / total);
  std::vector<uint8_t> packed(total);
  for (int c = 0; c < n; c++) memcpy(&packed[off[c]], enc[c].data(), enc[c].size());
  uint8_t *d_enc, *d_out;
  CK(hipMalloc(&d_enc, total));
  CK(hipMemcpy(d_enc, packed.data(), total, hipMemcpyHostToDevice));
  CK(hipMalloc(&d_out, (size_t)n * chunk));
  std::vector<ZgItem> items(n);
  for (int c = 0; c < n; c++) items[c] = ZgItem{(uint64_t)(d_enc + off[c]), enc[c].size(), (uint32_t)c, 0, 0, 0};
  ZgItem *d_items;
  uint32_t *d_status;
  CK(hipMalloc(&d_items, n * sizeof(ZgItem)));
  CK(hipMalloc(&d_status, n * 4));
  zgpu::ZstdScratch Z{};
  uint64_t blk_bytes;
  zgpu::zstd_scratch_layout(chunk, Z.blk_cap, blk_bytes, Z.lit_stride, Z.seq_cap);
  CK(hipMalloc(&Z.blks, n * (uint64_t)Z.blk_cap * blk_bytes));
  CK(hipMalloc(&Z.nblk, n * 4));
  CK(hipMalloc(&Z.mode, n * 4));
  CK(hipMalloc(&Z.lit, n * Z.lit_stride));
  CK(hipMalloc(&Z.seq, n * Z.seq_cap * 12));
  if (!getenv("LAB_NONORM")) CK(hipMalloc(&Z.norm, n * (uint64_t)Z.blk_cap * zgpu::zstd_norm_bytes()));
  if (getenv("LAB_EXEC") && !strcmp(getenv("LAB_EXEC"), "par")) {
    CK(hipMalloc(&Z.ext, 2 * (uint64_t)n * chunk * 4));
    CK(hipMalloc(&Z.ext_cnt, zgpu::ZEXT_ROUNDS * 8));
    Z.ext_items = n;
  }

  constexpr int NK = 7;
  const char *kn[NK] = {"scan", "blocks", "huf", "lits", "plan", "direct", "exec_item"};
  hipEvent_t ev[NK + 1];
  for (auto &evk : ev) CK(hipEventCreate(&evk));

  float best[NK];
  for (auto &bk : best) bk = 1e30f;
#ifdef ZG_SQ_PROFILE
  {
    unsigned long long z[20] = {0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(zgpu::g_sqprof), z, sizeof(z)));
  }
#endif
#ifdef ZG_XWIN_PROF
  {
    unsigned long long z[16] = {0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(zgpu::xwin::g_xwprof), z, sizeof(z)));
  }
#endif
#ifdef ZG_PROFILE
  {
    unsigned long long z[13] = {0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(zgpu::g_zprof), z, sizeof(z)));
  }
#endif
#ifdef ZG_LIT_STATS
  {
    unsigned long long z[8] = {0};
    CK(hipMemcpyToSymbol(HIP_SYMBOL(zgpu::g_litstats), z, sizeof(z)));
  }
#endif
  int ncu = 256;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const int reps = getenv("LAB_REPS") ? atoi(getenv("LAB_REPS")) : 3;
  uint8_t *lit_rec = nullptr;  // literal record slots (ZG_LIT_REC; LAB_NOREC=1: none)
  {
    uint32_t wgs = 0;
    const uint64_t rb = zgpu::zstd_lit_rec_bytes(wgs);
    if (rb && !getenv("LAB_NOREC") && wgs >= (uint32_t)ncu * ZG_LIT_GRID_PER_CU) CK(hipMalloc(&lit_rec, rb));
  }
  for (int rep = 0; rep < reps; rep++) {
    CK(hipMemcpy(d_items, items.data(), n * sizeof(ZgItem), hipMemcpyHostToDevice));
    CK(hipMemset(d_status, 0, n * 4));
    CK(hipMemset(d_out, 0xA5, (size_t)n * chunk));
    zgpu::ZBlk *blks = (zgpu::ZBlk *)Z.blks;
    const uint64_t recs = (uint64_t)n * Z.blk_cap;
    const uint32_t grid = (uint32_t)std::min<uint64_t>(recs, (uint64_t)ncu * 16);
    const uint32_t lgrid = (uint32_t)std::min<uint64_t>(recs, (uint64_t)ncu * ZG_LIT_GRID_PER_CU);
    const uint32_t bgrid = (uint32_t)std::min<uint64_t>(recs, std::max<uint64_t>(grid, (uint64_t)ncu * 4 * ZG_BLK_WPE));
    CK(hipEventRecord(ev[0]));
    hipLaunchKernelGGL(zgpu::k_zstd_scan, dim3(n), dim3(64), 0, 0, d_items, d_status, blks, Z.blk_cap, Z.nblk, Z.mode,
                       Z.lit_stride, Z.seq_cap, 0u, (unsigned long long *)nullptr, (uint32_t *)nullptr,
                       (unsigned long long *)nullptr, (unsigned long long *)nullptr, Z.norm);
    CK(hipEventRecord(ev[1]));
    const int seqm = getenv("LAB_SEQLG") ? atoi(getenv("LAB_SEQLG")) : 1;
    if (seqm == 1) {  // the lane-group sequence decoder, as launch_zstd_pass
      const uint64_t per_cu =
          std::max<uint64_t>(1, (160u << 10) / ((sizeof(zgpu::ZDecLgSmem<ZG_SEQ_G>) + 1023) & ~size_t(1023)));
      const uint32_t lg_grid =
          (uint32_t)std::min<uint64_t>((recs + ZG_SEQ_G - 1) / ZG_SEQ_G, (uint64_t)ncu * per_cu);
      hipLaunchKernelGGL(zgpu::k_zstd_blocks_lg<ZG_SEQ_G>, dim3(lg_grid), dim3(64), 0, 0, d_items, d_status, blks,
                         Z.blk_cap, Z.nblk, Z.mode, (uint32_t)n, Z.seq, Z.seq_cap, (const unsigned long long *)nullptr);
    } else {
      hipLaunchKernelGGL(zgpu::k_zstd_blocks, dim3(bgrid), dim3(64), 0, 0, d_items, d_status, blks, Z.blk_cap,
                         Z.nblk, Z.mode, (uint32_t)n, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap,
                         (const unsigned long long *)nullptr, Z.norm);
    }
    CK(hipEventRecord(ev[2]));
    hipLaunchKernelGGL(zgpu::k_zstd_huf, dim3(grid), dim3(64), 0, 0, d_items, d_status, blks, Z.blk_cap, Z.nblk, Z.mode,
                       (uint32_t)n, Z.lit, Z.lit_stride, (const unsigned long long *)nullptr);
    CK(hipEventRecord(ev[3]));
    hipLaunchKernelGGL(zgpu::k_zstd_lits, dim3(lgrid), dim3(zgpu::LIT_THREADS), 0, 0, d_items, d_status, blks, Z.blk_cap,
                       Z.nblk, Z.mode, (uint32_t)n, Z.lit, Z.lit_stride, lit_rec, (const unsigned long long *)nullptr);
    CK(hipEventRecord(ev[4]));
    // executor: LAB_EXEC=win (k_zstd_exec_win, the default), wide, dense; LAB_XSEG segments per item
    const char *lx = getenv("LAB_EXEC");
    const int xk = !lx || !strcmp(lx, "win") ? 2 : !strcmp(lx, "par") ? 3 : !strcmp(lx, "dense") ? 1 : 0;
    const uint32_t xseg = getenv("LAB_XSEG") ? (uint32_t)atoi(getenv("LAB_XSEG")) : xk == 2 ? zgpu::XSEG_WIN : zgpu::XSEG;
    hipLaunchKernelGGL(zgpu::k_zstd_plan, dim3(n), dim3(64), 0, 0, d_items, d_status, blks, Z.blk_cap, Z.nblk, Z.mode,
                       chunk, xseg, (uint64_t *)nullptr, Z.lit, Z.lit_stride);
    CK(hipEventRecord(ev[5]));
    hipLaunchKernelGGL(zgpu::k_zstd_direct, dim3(grid), dim3(256), 0, 0, d_items, d_status, blks, Z.blk_cap, Z.nblk,
                       Z.mode, (uint32_t)n, d_out, chunk, Z.lit, Z.lit_stride, (const uint64_t *)nullptr,
                       (const unsigned long long *)nullptr, 0);
    CK(hipEventRecord(ev[6]));
    if (xk == 3) {  // the latency mode, as launch_zstd_pass runs it
      const uint64_t tot = (uint64_t)n * chunk;
      CK(hipMemsetAsync(Z.ext, 0xFF, tot * 4, 0));
      CK(hipMemsetAsync(Z.ext_cnt, 0, zgpu::ZEXT_ROUNDS * 8, 0));
      hipLaunchKernelGGL(zgpu::k_zstd_exec_win<true>, dim3(ncu), dim3(zgpu::xwin::THREADS), 0, 0, d_items, d_status,
                         blks, Z.blk_cap, Z.nblk, Z.mode, d_out, chunk, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap,
                         (uint32_t)n, Z.ext, (const unsigned long long *)nullptr);
      uint32_t rounds = 2;
      while (rounds < zgpu::ZEXT_ROUNDS && (1ull << (rounds - 2)) < chunk / 1024 + 1) rounds++;
      const uint32_t g2 = (uint32_t)std::min<uint64_t>((tot / 4 + 255) / 256, (uint64_t)ncu * 16);
      uint32_t *ea = Z.ext, *eb = Z.ext + tot;
      for (uint32_t r = 0; r < rounds; r++) {
        hipLaunchKernelGGL(zgpu::k_zstd_ext_round, dim3(g2), dim3(256), 0, 0, ea, eb, d_out, chunk, tot,
                           r ? Z.ext_cnt + r - 1 : (const unsigned long long *)nullptr, Z.ext_cnt + r);
        std::swap(ea, eb);
      }
      hipLaunchKernelGGL(zgpu::k_zstd_par_finish, dim3(n), dim3(64), 0, 0, d_items, d_status, blks, Z.blk_cap, Z.nblk,
                         Z.mode, d_out, chunk);
    } else if (xk == 2)
      hipLaunchKernelGGL(zgpu::k_zstd_exec_win<false>, dim3(n * xseg), dim3(zgpu::xwin::THREADS), 0, 0, d_items,
                         d_status, blks, Z.blk_cap, Z.nblk, Z.mode, d_out, chunk, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap,
                         xseg, (uint32_t *)nullptr, (const unsigned long long *)nullptr);
    else if (xk == 1)
      hipLaunchKernelGGL(zgpu::xdense::k_zstd_exec_item, dim3(n * xseg), dim3(64), 0, 0, d_items, d_status, blks,
                         Z.blk_cap, Z.nblk, Z.mode, d_out, chunk, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap, xseg);
    else
      hipLaunchKernelGGL(zgpu::xwide::k_zstd_exec_item, dim3(n * xseg), dim3(64), 0, 0, d_items, d_status, blks,
                         Z.blk_cap, Z.nblk, Z.mode, d_out, chunk, Z.lit, Z.lit_stride, Z.seq, Z.seq_cap, xseg);
    CK(hipEventRecord(ev[7]));
    CK(hipEventSynchronize(ev[7]));
    for (int k = 0; k < NK; k++) {
      float ms;
      CK(hipEventElapsedTime(&ms, ev[k], ev[k + 1]));
      best[k] = std::min(best[k], ms);
    }

  }
  std::vector<uint32_t> st(n), nblk(n), mode(n);
  CK(hipMemcpy(st.data(), d_status, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(nblk.data(), Z.nblk, n * 4, hipMemcpyDeviceToHost));
  CK(hipMemcpy(mode.data(), Z.mode, n * 4, hipMemcpyDeviceToHost));
  int bad = 0;
  std::vector<uint8_t> out(chunk);
  uint64_t blocks = 0;
  for (int c = 0; c < n; c++) {
    CK(hipMemcpy(out.data(), d_out + (uint64_t)c * chunk, chunk, hipMemcpyDeviceToHost));
    if (st[c] || memcmp(out.data(), dec[c].data(), chunk)) {
      if (bad < 4) {
        uint64_t k = 0;
        while (k < chunk && out[k] == dec[c][k]) k++;
        printf("chunk %d: status %u, first mismatch at %llu (got %u want %u)\n", c, st[c], (unsigned long long)k,
               k < chunk ? out[k] : 0, k < chunk ? dec[c][k] : 0);
      }
      bad++;
    }
    blocks += nblk[c];
  }
  double tot = 0;
  for (int k = 0; k < NK; k++) tot += best[k];
  printf("blocks %llu (%.1f/chunk), mode[0]=%u, bad=%d\n", (unsigned long long)blocks, (double)blocks / n, mode[0], bad);
  for (int k = 0; k < NK; k++) printf("  %-12s %8.3f ms\n", kn[k], best[k]);
#ifdef ZG_LIT_PROF
  {
    unsigned long long z[8];
    CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(zgpu::g_litprof), sizeof(z)));
    const double r = (double)(z[5] ? z[5] : 1);
    printf("lits phases per record (s_memtime ticks, 100 MHz; all reps): pass1 %.0f repairs %.0f prefix %.0f pass2 %.0f | records %llu\n",
           z[0] / r, z[1] / r, z[2] / r, z[3] / r, z[5]);
  }
#endif
#ifdef ZG_LIT_STATS
  {
    unsigned long long z[8];
    CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(zgpu::g_litstats), sizeof(z)));
    printf("lit stats (all reps): huffman blocks %llu, blocks needing repair %llu, repair rounds %llu, lanes re-decoded %llu, "
           "symbols %llu, warm-up symbols %llu, lanes %llu, lanes decoding twice %llu\n", z[0], z[1], z[2], z[3], z[4], z[5], z[6], z[7]);
  }
#endif
#ifdef ZG_PROFILE
  {
    unsigned long long z[13];
    CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(zgpu::g_zprof), sizeof(z)));
    const double nb = z[4] ? (double)z[4] : 1.0;
    const double nbt = z[6] ? (double)z[6] : 1.0;
    const double per = (double)n * 3;  // per frame (3 reps)
    printf("exec_item per frame (Mticks): single-lits %.2f stage %.2f single-matches %.2f resolve %.2f singles %.2f raw/rle/tail %.2f | total %.2f | batches %.0f\n",
           z[0] / per / 1e6, z[1] / per / 1e6, z[2] / per / 1e6, z[3] / per / 1e6, z[4] / per / 1e6, z[5] / per / 1e6,
           z[6] / per / 1e6, (double)(z[7] & 0xFFFFFFFFu) / per);
    printf("single matches with d < 16 per frame: %.0f\n", (double)(z[7] >> 32) / per);
    printf("resolve per frame (Mticks): ready %.2f fast copies %.2f slow copies %.2f | rounds %.0f\n", z[8] / per / 1e6,
           z[9] / per / 1e6, z[10] / per / 1e6, (double)z[11] / per);
    printf("batches with far sources per frame: %.0f\n", z[12] / per);
  }
#endif
#ifdef ZG_XWIN_PROF
  {
    unsigned long long z[16];
    CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(zgpu::xwin::g_xwprof), sizeof(z)));
    const double w = z[6] ? (double)z[6] : 1.0;
    printf("exec_win per window: pointer cells %.0f literal loads %.0f far loads %.0f | classify clocks %.0f | wave-0 "
           "round steps %.2f, wave-0 round clocks (no barrier) %.0f\n", z[8] / w, z[9] / w, z[10] / w, z[5] / w, z[11] / w,
           z[12] / w);
    printf("exec_win per window (clocks, workgroup thread 0): table %.0f rows %.0f expand %.0f rounds %.0f output %.0f | "
           "windows %llu (all reps), rounds/window %.2f\n", z[0] / w, z[1] / w, z[2] / w, z[3] / w, z[4] / w, z[6], z[7] / w);
  }
#endif
#ifdef ZG_SQ_PROFILE
  {
    unsigned long long z[20];
    CK(hipMemcpyFromSymbol(z, HIP_SYMBOL(zgpu::g_sqprof), sizeof(z)));
    for (int t = 0; t < 3; t++)
      printf("table %s modes (predefined / rle / fse / repeat): %llu %llu %llu %llu\n", t == 0 ? "LL" : t == 1 ? "OF" : "ML",
             z[8 + 4 * t] / reps, z[9 + 4 * t] / reps, z[10 + 4 * t] / reps, z[11 + 4 * t] / reps);
    const double nb = z[3] ? (double)z[3] : 1.0;
    printf("sequences: %.0f blocks with sequences, %.1f sequences/block, records visited %llu, epochs %llu | per block "
           "(clocks, wave sums): tables %.0f decode %.0f | per sequence: decode %.1f\n", nb / reps, z[2] / nb,
           z[5] / reps, z[4] / reps, z[0] / nb, z[1] / nb, z[1] / (double)(z[2] ? z[2] : 1));
    printf("tables (k_zstd_blocks, per block with sequences): FSE descriptions parsed %.0f clocks, built %.0f clocks\n",
           z[6] / nb, z[7] / nb);
  }
#endif
  if (Z.ext_cnt) {
    unsigned long long c[zgpu::ZEXT_ROUNDS];
    CK(hipMemcpy(c, Z.ext_cnt, sizeof(c), hipMemcpyDeviceToHost));
    printf("ext references left after each round:");
    for (uint32_t r = 0; r < 16; r++) printf(" %llu", c[r]);
    printf("\n");
  }
  printf("total %.3f ms -> %.2f GB/s decoded\n", tot, (double)n * chunk / tot / 1e6);
  return bad ? 1 : 0;
}
