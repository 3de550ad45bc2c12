// Lab harness (not product code): calibrates rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the
// access widths and patterns the entropy kernels use. MI355X_MICROARCH.md calibrates FETCH_SIZE only
// for 16-B/lane coalesced streaming reads (it reports half the bytes) and says other widths must be
// calibrated on a known byte count. Every kernel here moves exactly BYTES bytes once (1 GiB, far past
// the 256 MiB Infinity Cache, which is flushed between kernels by a 512 MiB streaming write).
// Build: hipcc --offload-arch=gfx950 -O3 -o fetch_calib fetch_calib.hip
// Run:   rocprofv3 --pmc FETCH_SIZE -d out -o pmc --output-format csv -- ./fetch_calib
//        rocprofv3 --pmc WRITE_SIZE ... (a separate pass)
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr uint64_t BYTES = 1ull << 30;
constexpr int TPB = 256;

// coalesced reads of T per lane, grid-stride
template <class T>
__global__ __launch_bounds__(TPB) void rd_coal(const T *p, uint64_t n, uint32_t *sink) {
  uint32_t acc = 0;
  for (uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * TPB) {
    const T v = p[i];
    acc ^= (uint32_t)(sizeof(T) >= 4 ? *(const uint32_t *)&v : (uint32_t)*(const uint8_t *)&v);
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
// each lane reads its own contiguous segment of SEG bytes, W bytes at a time (the gzip / literal
// decoders' lane streams: adjacent lanes' segments are adjacent)
template <int W, int SEG>
__global__ __launch_bounds__(TPB) void rd_seg(const uint8_t *p, uint64_t n, uint32_t *sink) {
  uint32_t acc = 0;
  const uint64_t lanes = (uint64_t)gridDim.x * TPB, lane = blockIdx.x * (uint64_t)TPB + threadIdx.x;
  for (uint64_t base = lane * SEG; base < n; base += lanes * SEG) {
    for (int k = 0; k < SEG; k += W) {
      if (W == 16) {
        const uint4 v = *(const uint4 *)(p + base + k);
        acc ^= v.x ^ v.w;
      } else if (W == 8) {
        const uint2 v = *(const uint2 *)(p + base + k);
        acc ^= v.x ^ v.y;
      } else {
        acc ^= *(const uint32_t *)(p + base + k);
      }
    }
  }
  if (acc == 0x12345678u) sink[0] = acc;
}
// coalesced writes of T per lane
template <class T>
__global__ __launch_bounds__(TPB) void wr_coal(T *p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * TPB) p[i] = (T)i;
}
// stride-2 byte writes: one byte plane of u16 elements (the fused-unshuffle question)
__global__ __launch_bounds__(TPB) void wr_plane(uint8_t *p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x; i < n / 2; i += (uint64_t)gridDim.x * TPB)
    p[2 * i] = (uint8_t)i;
}
__global__ __launch_bounds__(TPB) void flush_l3(uint4 *p, uint64_t n) {
  for (uint64_t i = blockIdx.x * (uint64_t)TPB + threadIdx.x; i < n; i += (uint64_t)gridDim.x * TPB)
    p[i] = make_uint4((uint32_t)i, 0, 0, 0);
}

int main() {
  uint8_t *src, *dst, *fl;
  uint32_t *sink;
  CK(hipMalloc(&src, BYTES));
  CK(hipMalloc(&dst, BYTES));
  CK(hipMalloc(&fl, 512ull << 20));
  CK(hipMalloc(&sink, 64));
  CK(hipMemset(src, 1, BYTES));
  int ncu = 256;
  CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  const dim3 g(ncu * 8), b(TPB);
  auto flush = [&] { hipLaunchKernelGGL(flush_l3, g, b, 0, 0, (uint4 *)fl, (512ull << 20) / 16); };
  flush();
  hipLaunchKernelGGL(rd_coal<uint4>, g, b, 0, 0, (const uint4 *)src, BYTES / 16, sink);
  flush();
  hipLaunchKernelGGL(rd_coal<uint2>, g, b, 0, 0, (const uint2 *)src, BYTES / 8, sink);
  flush();
  hipLaunchKernelGGL(rd_coal<uint32_t>, g, b, 0, 0, (const uint32_t *)src, BYTES / 4, sink);
  flush();
  hipLaunchKernelGGL(rd_coal<uint8_t>, g, b, 0, 0, (const uint8_t *)src, BYTES, sink);
  flush();
  hipLaunchKernelGGL((rd_seg<4, 512>), g, b, 0, 0, src, BYTES, sink);
  flush();
  hipLaunchKernelGGL((rd_seg<16, 512>), g, b, 0, 0, src, BYTES, sink);
  flush();
  hipLaunchKernelGGL((rd_seg<4, 4096>), g, b, 0, 0, src, BYTES, sink);
  flush();
  hipLaunchKernelGGL((rd_seg<8, 4096>), g, b, 0, 0, src, BYTES, sink);
  flush();
  hipLaunchKernelGGL(wr_coal<uint4>, g, b, 0, 0, (uint4 *)dst, BYTES / 16);
  flush();
  hipLaunchKernelGGL(wr_coal<uint32_t>, g, b, 0, 0, (uint32_t *)dst, BYTES / 4);
  flush();
  hipLaunchKernelGGL(wr_coal<uint8_t>, g, b, 0, 0, dst, BYTES);
  flush();
  hipLaunchKernelGGL(wr_plane, g, b, 0, 0, dst, BYTES);
  CK(hipDeviceSynchronize());
  printf("fetch_calib: every rd_*/wr_* kernel moves %llu bytes (wr_plane: %llu bytes, every other byte of %llu)\n",
         (unsigned long long)BYTES, (unsigned long long)(BYTES / 2), (unsigned long long)BYTES);
  return 0;
}
