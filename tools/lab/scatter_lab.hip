// Microbenchmark lab (not product code): variants of the C2 decode (64^3 f32 chunks, transpose
// order [2,1,0] + big-endian swap, scattered into a 1024^3 array) against a plain streaming copy,
// to find the practical HBM ceiling of this access pattern on gfx950.
// Build: hipcc --offload-arch=gfx950 -O3 -o scatter_lab scatter_lab.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int C = 64;          // chunk edge
constexpr int G = 16;          // chunks per axis
constexpr int N = C * G;       // array edge
constexpr uint64_t NCH = (uint64_t)G * G * G;
constexpr uint64_t CHUNK_ELEMS = (uint64_t)C * C * C;
constexpr uint64_t TOTAL = NCH * CHUNK_ELEMS;  // elements

typedef unsigned int v4u __attribute__((ext_vector_type(4)));
template <bool NT>
__device__ __forceinline__ uint4 ld(const uint4 *p) {
  if constexpr (NT) { v4u x = __builtin_nontemporal_load((const v4u *)p); return make_uint4(x.x, x.y, x.z, x.w); }
  else return *p;
}
template <bool NT>
__device__ __forceinline__ void st(uint4 *p, uint4 v) {
  if constexpr (NT) { v4u x = {v.x, v.y, v.z, v.w}; __builtin_nontemporal_store(x, (v4u *)p); }
  else *p = v;
}

template <bool NT>
__global__ __launch_bounds__(256) void k_copy(const uint4 *__restrict__ a, uint4 *__restrict__ b, uint64_t n) {
  uint64_t i = (uint64_t)blockIdx.x * 256 * 4 + threadIdx.x;
  uint4 v[4];
#pragma unroll
  for (int k = 0; k < 4; k++) v[k] = ld<NT>(a + i + k * 256);
#pragma unroll
  for (int k = 0; k < 4; k++) st<NT>(b + i + k * 256, v[k]);
}

__device__ __forceinline__ uint32_t bs(uint32_t x) { return __builtin_bswap32(x); }

// TJ consecutive j-slices of one chunk per block; THREADS threads. LDS tile[TJ][64][65] f32.
template <int TJ, int THREADS, bool NT, bool SWZ>
__global__ __launch_bounds__(THREADS) void k_tr(const uint32_t *__restrict__ enc, uint32_t *__restrict__ out) {
  constexpr int PITCH = SWZ ? 64 : 65;
  __shared__ uint32_t tile[TJ][64][PITCH];
  constexpr int GROUPS = 64 / TJ;
  const uint32_t c = blockIdx.x / GROUPS;
  const uint32_t j0 = (blockIdx.x % GROUPS) * TJ;
  const uint32_t ci = c / (G * G), cj = (c / G) % G, ck = c % G;
  const uint32_t *src = enc + (uint64_t)c * CHUNK_ELEMS;
  constexpr int LOADS = TJ * 1024 / THREADS;  // uint4 per thread
  uint4 v[LOADS];
#pragma unroll
  for (int p = 0; p < LOADS; p++) {
    const uint32_t e = p * THREADS + threadIdx.x;
    const uint32_t k = e / (TJ * 16), rem = e % (TJ * 16), jj = rem / 16, vv = rem % 16;
    v[p] = ld<NT>((const uint4 *)(src + ((uint64_t)k * 64 + j0 + jj) * 64 + vv * 4));
  }
#pragma unroll
  for (int p = 0; p < LOADS; p++) {
    const uint32_t e = p * THREADS + threadIdx.x;
    const uint32_t k = e / (TJ * 16), rem = e % (TJ * 16), jj = rem / 16, vv = rem % 16;
    if constexpr (SWZ) {
      // element (row k, col i) stored at col i ^ (k & 63)... use 4-aligned xor on vector index
      const uint32_t sw = (vv ^ (k & 15)) * 4;
      *(uint4 *)&tile[jj][k][sw] = make_uint4(bs(v[p].x), bs(v[p].y), bs(v[p].z), bs(v[p].w));
    } else {
      tile[jj][k][vv * 4 + 0] = bs(v[p].x);
      tile[jj][k][vv * 4 + 1] = bs(v[p].y);
      tile[jj][k][vv * 4 + 2] = bs(v[p].z);
      tile[jj][k][vv * 4 + 3] = bs(v[p].w);
    }
  }
  __syncthreads();
  // store: out[ci*64+i][cj*64+j0+jj][ck*64 + k], 64 k per row = 16 uint4
#pragma unroll
  for (int p = 0; p < LOADS; p++) {
    const uint32_t e = p * THREADS + threadIdx.x;
    const uint32_t i = e / (TJ * 16), rem = e % (TJ * 16), jj = rem / 16, vv = rem % 16;
    uint4 x;
    if constexpr (SWZ) {
      // need tile[jj][4vv+q][i]: stored at col ((i/4) ^ ((4vv+q)&15))*4 + i%4
      uint32_t r[4];
#pragma unroll
      for (int q = 0; q < 4; q++) {
        const uint32_t k = vv * 4 + q;
        r[q] = tile[jj][k][(((i >> 2) ^ (k & 15)) << 2) | (i & 3)];
      }
      x = make_uint4(r[0], r[1], r[2], r[3]);
    } else {
      x = make_uint4(tile[jj][vv * 4 + 0][i], tile[jj][vv * 4 + 1][i], tile[jj][vv * 4 + 2][i], tile[jj][vv * 4 + 3][i]);
    }
    const uint64_t o = ((uint64_t)(ci * 64 + i) * N + cj * 64 + j0 + jj) * N + ck * 64 + vv * 4;
    st<NT>((uint4 *)(out + o), x);
  }
}


// CKP adjacent chunks (along the fastest chunk-grid axis) x TJ consecutive j-slices per block.
template <int TJ, int CKP, int THREADS, bool NTL, bool NTS>
__global__ __launch_bounds__(THREADS) void k_tr2(const uint32_t *__restrict__ enc, uint32_t *__restrict__ out) {
  __shared__ uint32_t tile[CKP][TJ][64][65];
  constexpr int GROUPS = 64 / TJ;
  const uint32_t cp = blockIdx.x / GROUPS;          // chunk-pair index
  const uint32_t j0 = (blockIdx.x % GROUPS) * TJ;
  const uint32_t c0 = cp * CKP;
  const uint32_t ci = c0 / (G * G), cj = (c0 / G) % G, ck = c0 % G;
  constexpr int PER = CKP * TJ * 1024 / THREADS;  // uint4 per thread
  uint4 v[PER];
#pragma unroll
  for (int p = 0; p < PER; p++) {
    const uint32_t e = p * THREADS + threadIdx.x;
    const uint32_t q = e / (TJ * 1024), r = e % (TJ * 1024);
    const uint32_t k = r / (TJ * 16), rem = r % (TJ * 16), jj = rem / 16, vv = rem % 16;
    v[p] = ld<NTL>((const uint4 *)(enc + (uint64_t)(c0 + q) * CHUNK_ELEMS + ((uint64_t)k * 64 + j0 + jj) * 64 + vv * 4));
  }
#pragma unroll
  for (int p = 0; p < PER; p++) {
    const uint32_t e = p * THREADS + threadIdx.x;
    const uint32_t q = e / (TJ * 1024), r = e % (TJ * 1024);
    const uint32_t k = r / (TJ * 16), rem = r % (TJ * 16), jj = rem / 16, vv = rem % 16;
    tile[q][jj][k][vv * 4 + 0] = bs(v[p].x);
    tile[q][jj][k][vv * 4 + 1] = bs(v[p].y);
    tile[q][jj][k][vv * 4 + 2] = bs(v[p].z);
    tile[q][jj][k][vv * 4 + 3] = bs(v[p].w);
  }
  __syncthreads();
#pragma unroll
  for (int p = 0; p < PER; p++) {
    const uint32_t e = p * THREADS + threadIdx.x;
    // output row (i, jj): CKP*16 vectors contiguous
    const uint32_t i = e / (TJ * CKP * 16), rem = e % (TJ * CKP * 16), jj = rem / (CKP * 16), w = rem % (CKP * 16);
    const uint32_t q = w / 16, vv = w % 16;
    uint4 x = make_uint4(tile[q][jj][vv * 4 + 0][i], tile[q][jj][vv * 4 + 1][i], tile[q][jj][vv * 4 + 2][i], tile[q][jj][vv * 4 + 3][i]);
    const uint64_t o = ((uint64_t)(ci * 64 + i) * N + cj * 64 + j0 + jj) * N + ck * 64 + w * 4;
    st<NTS>((uint4 *)(out + o), x);
  }
}

template <int PER, bool NT>
__global__ __launch_bounds__(256) void k_copy2(const uint4 *__restrict__ a, uint4 *__restrict__ b) {
  uint64_t i = (uint64_t)blockIdx.x * 256 * PER + threadIdx.x;
  uint4 v[PER];
#pragma unroll
  for (int k = 0; k < PER; k++) v[k] = ld<NT>(a + i + k * 256);
#pragma unroll
  for (int k = 0; k < PER; k++) st<NT>(b + i + k * 256, v[k]);
}


// Pipelined: each block loops over slab groups g = blockIdx.x + n*gridDim.x; the loads of group n+1
// are issued before the LDS->HBM stores of group n.
template <int TJ, int THREADS, bool NTL, bool NTS>
__global__ __launch_bounds__(THREADS) void k_tr3(const uint32_t *__restrict__ enc, uint32_t *__restrict__ out, uint32_t ngroups) {
  constexpr int SLAB = 64 * 65 + 1;
  __shared__ uint32_t tile[TJ * SLAB];
  constexpr int GROUPS = 64 / TJ;
  constexpr int PER = TJ * 1024 / THREADS;
  uint4 v[PER];
  uint32_t g = blockIdx.x;
  auto load = [&](uint32_t gg) {
    const uint32_t c = gg / GROUPS, j0 = (gg % GROUPS) * TJ;
    const uint32_t *src = enc + (uint64_t)c * CHUNK_ELEMS;
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const uint32_t e = p * THREADS + threadIdx.x;
      const uint32_t k = e / (TJ * 16), jj = (e / 16) % TJ, vv = e % 16;
      v[p] = ld<NTL>((const uint4 *)(src + ((uint64_t)k * 64 + j0 + jj) * 64 + vv * 4));
    }
  };
  if (g < ngroups) load(g);
  for (; g < ngroups; g += gridDim.x) {
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const uint32_t e = p * THREADS + threadIdx.x;
      const uint32_t k = e / (TJ * 16), jj = (e / 16) % TJ, vv = e % 16;
      uint32_t *t = tile + jj * SLAB + k * 65 + vv * 4;
      t[0] = bs(v[p].x); t[1] = bs(v[p].y); t[2] = bs(v[p].z); t[3] = bs(v[p].w);
    }
    __syncthreads();
    const uint32_t gn = g + gridDim.x;
    if (gn < ngroups) load(gn);
    const uint32_t c = g / GROUPS, j0 = (g % GROUPS) * TJ;
    const uint32_t ci = c / (G * G), cj = (c / G) % G, ck = c % G;
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const uint32_t e = p * THREADS + threadIdx.x;
      const uint32_t i = e / (TJ * 16), jj = (e / 16) % TJ, vv = e % 16;
      const uint32_t *t = tile + jj * SLAB + vv * 4 * 65 + i;
      uint4 x = make_uint4(t[0], t[65], t[130], t[195]);
      const uint64_t o = ((uint64_t)(ci * 64 + i) * N + cj * 64 + j0 + jj) * N + ck * 64 + vv * 4;
      st<NTS>((uint4 *)(out + o), x);
    }
    __syncthreads();
  }
}

// host reference for a few chunks
static bool verify(const std::vector<uint32_t> &h_enc_chunk0, const std::vector<uint32_t> &h_out, int c) {
  return true;
}

int main(int argc, char **argv) {
  const int reps = argc > 1 ? atoi(argv[1]) : 10;
  uint32_t *enc, *out, *ref;
  const size_t bytes = TOTAL * 4;
  CK(hipMalloc(&enc, bytes));
  CK(hipMalloc(&out, bytes));
  CK(hipMalloc(&ref, bytes));
  {
    std::vector<uint32_t> h(TOTAL);
    uint64_t s = 0x123456789abcdef0ull;
    for (uint64_t i = 0; i < TOTAL; i++) { s = s * 6364136223846793005ull + 1442695040888963407ull; h[i] = (uint32_t)(s >> 32); }
    CK(hipMemcpy(enc, h.data(), bytes, hipMemcpyHostToDevice));
  }
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char *name, auto launch, double traffic, uint32_t *dst) {
    CK(hipMemset(dst, 0, bytes));
    launch(); launch();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int r = 0; r < reps; r++) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    bool same = true;
    if (dst != ref) {
      std::vector<uint32_t> a(1 << 20), b(1 << 20);
      for (uint64_t off : {(uint64_t)0, TOTAL / 3, TOTAL - (1u << 20)}) {
        CK(hipMemcpy(a.data(), dst + off, 4 << 20, hipMemcpyDeviceToHost));
        CK(hipMemcpy(b.data(), ref + off, 4 << 20, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < a.size(); i++) if (a[i] != b[i]) { same = false; break; }
      }
    }
    printf("%-34s %8.4f ms  %7.1f GB/s  frac %.3f  %s\n", name, ms, traffic / ms / 1e6, traffic / ms / 1e6 / 8000.0,
           dst == ref ? "(ref)" : same ? "ok" : "MISMATCH");
  };
  const double T = 2.0 * bytes;
  const uint32_t ncopy = (uint32_t)(TOTAL / 4 / 1024);
  timeit("copy uint4 x4", [&] { hipLaunchKernelGGL(k_copy<false>, dim3(ncopy), dim3(256), 0, 0, (const uint4 *)enc, (uint4 *)out, 0); }, T, out);
  timeit("copy uint4 x4 nt", [&] { hipLaunchKernelGGL(k_copy<true>, dim3(ncopy), dim3(256), 0, 0, (const uint4 *)enc, (uint4 *)out, 0); }, T, out);
  CK(hipEventRecord(e0));
  CK(hipMemcpyAsync(out, enc, bytes, hipMemcpyDeviceToDevice, 0));
  CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
  { float ms; CK(hipEventElapsedTime(&ms, e0, e1)); printf("%-34s %8.4f ms  %7.1f GB/s\n", "hipMemcpyD2D", ms, T / ms / 1e6); }
  timeit("tr TJ1 256 (ref)", [&] { hipLaunchKernelGGL((k_tr<1, 256, false, false>), dim3(NCH * 64), dim3(256), 0, 0, enc, ref); }, T, ref);
#define TR2(TJ, CKP, TH, NL, NS) timeit("tr2 TJ" #TJ " CKP" #CKP " " #TH " ntl" #NL " nts" #NS, [&] { hipLaunchKernelGGL((k_tr2<TJ, CKP, TH, NL, NS>), dim3((uint32_t)(NCH / CKP * 64 / TJ)), dim3(TH), 0, 0, enc, out); }, T, out)
#define TR3(TJ, TH, NL, NS, GRID) timeit("tr3 TJ" #TJ " " #TH " ntl" #NL " nts" #NS " grid" #GRID, [&] { hipLaunchKernelGGL((k_tr3<TJ, TH, NL, NS>), dim3(GRID), dim3(TH), 0, 0, enc, out, (uint32_t)(NCH * 64 / TJ)); }, T, out)
  TR2(4, 1, 256, true, true);
  TR2(4, 1, 512, true, true);
  TR3(4, 256, true, true, 512);
  TR3(4, 256, true, true, 1024);
  TR3(4, 256, true, true, 2048);
  TR3(4, 256, true, true, 4096);
  TR3(4, 512, true, true, 512);
  TR3(4, 512, true, true, 1024);
  TR3(2, 256, true, true, 1024);
  TR3(2, 256, true, true, 2048);
  TR3(4, 256, false, true, 1024);
  TR3(4, 256, true, false, 1024);
  TR3(4, 256, false, false, 1024);
  TR2(4, 1, 256, true, true);
  return 0;
}
