// Lab (not product code): cost of 16-B LDS moves on gfx950 by alignment and active lanes, and the
// clock64 tick rate.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef unsigned int v4u __attribute__((ext_vector_type(4)));
__global__ void k(int mis_src, int mis_dst, int iters, int active, int pieces, unsigned long long *cyc, unsigned *sink) {
  __shared__ unsigned char ring[65536];
  for (int i = threadIdx.x; i < 65536; i += 64) ring[i] = (unsigned char)i;
  __syncthreads();
  const unsigned lane = threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
    if ((int)lane < active) {
      const unsigned so = ((it * 2048 + lane * 128) & 16383) + mis_src;
      const unsigned dof = 32768 + ((it * 2048 + lane * 128) & 16383) + mis_dst;
      v4u v0, v1, v2, v3, v4, v5, v6, v7;
      __builtin_memcpy(&v0, &ring[so + 0], 16);
      if (pieces > 1) __builtin_memcpy(&v1, &ring[so + 16], 16);
      if (pieces > 2) __builtin_memcpy(&v2, &ring[so + 32], 16);
      if (pieces > 3) __builtin_memcpy(&v3, &ring[so + 48], 16);
      if (pieces > 4) __builtin_memcpy(&v4, &ring[so + 64], 16);
      if (pieces > 5) __builtin_memcpy(&v5, &ring[so + 80], 16);
      if (pieces > 6) __builtin_memcpy(&v6, &ring[so + 96], 16);
      if (pieces > 7) __builtin_memcpy(&v7, &ring[so + 112], 16);
      __builtin_memcpy(&ring[dof + 0], &v0, 16);
      if (pieces > 1) __builtin_memcpy(&ring[dof + 16], &v1, 16);
      if (pieces > 2) __builtin_memcpy(&ring[dof + 32], &v2, 16);
      if (pieces > 3) __builtin_memcpy(&ring[dof + 48], &v3, 16);
      if (pieces > 4) __builtin_memcpy(&ring[dof + 64], &v4, 16);
      if (pieces > 5) __builtin_memcpy(&ring[dof + 80], &v5, 16);
      if (pieces > 6) __builtin_memcpy(&ring[dof + 96], &v6, 16);
      if (pieces > 7) __builtin_memcpy(&ring[dof + 112], &v7, 16);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  __syncthreads();
  const unsigned long long t1 = clock64();
  if (lane == 0) *cyc = t1 - t0;
  sink[lane] = ring[lane * 7];
}
// destination-aligned variant: aligned 16-B reads of the source, byte-aligned in registers
__device__ __forceinline__ v4u fun(v4u a, v4u b, unsigned sh) {  // bytes [sh, sh+16) of a:b
  v4u r;
  r.x = __builtin_amdgcn_alignbyte(a.y, a.x, sh);
  r.y = __builtin_amdgcn_alignbyte(a.z, a.y, sh);
  r.z = __builtin_amdgcn_alignbyte(a.w, a.z, sh);
  r.w = __builtin_amdgcn_alignbyte(b.x, a.w, sh);
  return r;
}
__global__ void k_al(int mis_src, int iters, int active, int pieces, unsigned long long *cyc, unsigned *sink) {
  __shared__ __attribute__((aligned(16))) unsigned char ring[65536];
  for (int i = threadIdx.x; i < 65536; i += 64) ring[i] = (unsigned char)i;
  __syncthreads();
  const unsigned lane = threadIdx.x;
  const unsigned long long t0 = clock64();
  for (int it = 0; it < iters; it++) {
    if ((int)lane < active) {
      const unsigned so = ((it * 2048 + lane * 144) & 16383) + mis_src;
      const unsigned dof = 32768 + ((it * 2048 + lane * 144) & 16383);
      const unsigned sa = so & ~15u, sh = so & 15;
      const v4u *sv = (const v4u *)&ring[sa];
      v4u *dv = (v4u *)&ring[dof];
      v4u a0 = sv[0], a1 = sv[1], a2, a3, a4, a5, a6, a7, a8;
      if (pieces > 1) a2 = sv[2];
      if (pieces > 2) a3 = sv[3];
      if (pieces > 3) a4 = sv[4];
      if (pieces > 4) a5 = sv[5];
      if (pieces > 5) a6 = sv[6];
      if (pieces > 6) a7 = sv[7];
      if (pieces > 7) a8 = sv[8];
      dv[0] = fun(a0, a1, sh);
      if (pieces > 1) dv[1] = fun(a1, a2, sh);
      if (pieces > 2) dv[2] = fun(a2, a3, sh);
      if (pieces > 3) dv[3] = fun(a3, a4, sh);
      if (pieces > 4) dv[4] = fun(a4, a5, sh);
      if (pieces > 5) dv[5] = fun(a5, a6, sh);
      if (pieces > 6) dv[6] = fun(a6, a7, sh);
      if (pieces > 7) dv[7] = fun(a7, a8, sh);
    }
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  }
  __syncthreads();
  const unsigned long long t1 = clock64();
  if (lane == 0) *cyc = t1 - t0;
  sink[lane] = ring[lane * 7];
}
__global__ void spin(unsigned long long n, unsigned long long *cyc) {
  const unsigned long long t0 = clock64();
  unsigned long long t = t0;
  while (t - t0 < n) t = clock64();
  if (threadIdx.x == 0) *cyc = t - t0;
}
int main() {
  unsigned long long *c; unsigned *s;
  hipMalloc(&c, 8); hipMalloc(&s, 256);
  int cases[][4] = {{0, 0, 64, 1}, {1, 3, 64, 1}, {0, 0, 64, 8}, {1, 3, 64, 8}, {1, 3, 5, 8}, {1, 3, 1, 8}, {0, 0, 1, 8}, {1, 3, 5, 1}};
  for (auto &cs : cases) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, cs[0], cs[1], 1000, cs[2], cs[3], c, s);
    unsigned long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("src+%d dst+%d lanes %d pieces %d: %.1f ticks per iteration\n", cs[0], cs[1], cs[2], cs[3], h / 1000.0);
  }
  int acases[][3] = {{3, 64, 8}, {3, 10, 8}, {3, 5, 8}, {3, 1, 8}, {3, 10, 1}};
  for (auto &cs : acases) {
    hipLaunchKernelGGL(k_al, dim3(1), dim3(64), 0, 0, cs[0], 1000, cs[1], cs[2], c, s);
    unsigned long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("aligned+alignbyte src+%d lanes %d pieces %d: %.1f ticks per iteration\n", cs[0], cs[1], cs[2], h / 1000.0);
  }
  int ucases[][4] = {{1, 3, 10, 8}, {1, 3, 10, 1}};
  for (auto &cs : ucases) {
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, cs[0], cs[1], 1000, cs[2], cs[3], c, s);
    unsigned long long h; hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
    printf("src+%d dst+%d lanes %d pieces %d: %.1f ticks per iteration\n", cs[0], cs[1], cs[2], cs[3], h / 1000.0);
  }
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  hipEventRecord(e0);
  hipLaunchKernelGGL(spin, dim3(1), dim3(64), 0, 0, 100000000ull, c);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1);
  printf("clock64: 1e8 ticks in %.3f ms -> %.3f GHz\n", ms, 1e8 / ms / 1e6);
  return 0;
}
