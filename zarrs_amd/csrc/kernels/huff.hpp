// Length-limited Huffman code lengths, shared by the DEFLATE (deflate_enc.hip) and zstd
// (zstd_enc.hip) encoders; one 64-lane wave per call.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace zgpu {

struct HuffScratch {
  uint16_t sorted[288];
  uint16_t parent[576];
  uint32_t weight[288];
  uint8_t depth[576];
  uint32_t blc[16];
};

__device__ __forceinline__ uint32_t huff_wave_sum(uint32_t v) {
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// Code lengths of a length-limited Huffman code for freq[0..n) (n <= 288) into lens (zlib trees.c
// build_tree + gen_bitlen semantics: fewer than two used symbols are padded to two one-bit codes, so
// every code is complete). Wave-cooperative; freq is only read.
__device__ inline void huff_lengths(HuffScratch &S, const uint32_t *freq, uint32_t n, uint32_t maxlen, uint8_t *lens) {
  const uint32_t lane = threadIdx.x;
  uint32_t cnt = 0;
  for (uint32_t s = lane; s < n; s += 64) {
    lens[s] = 0;
    cnt += freq[s] ? 1u : 0u;
  }
  const uint32_t m = huff_wave_sum(cnt);
  __syncthreads();
  if (m < 2) {
    if (lane == 0) {
      uint32_t a = n, b = n;
      for (uint32_t s = 0; s < n; s++)
        if (freq[s]) a = s;
      if (a == n) a = 0;
      b = a == 0 ? 1 : 0;
      lens[a] = 1;
      lens[b] = 1;
    }
    __syncthreads();
    return;
  }
  // ranks by (frequency, symbol): leaves in ascending order of weight
  for (uint32_t s = lane; s < n; s += 64) {
    const uint32_t f = freq[s];
    if (!f) continue;
    uint32_t r = 0;
    for (uint32_t t = 0; t < n; t++) {
      const uint32_t g = freq[t];
      r += (g && (g < f || (g == f && t < s))) ? 1u : 0u;
    }
    S.sorted[r] = (uint16_t)s;
  }
  __syncthreads();
  if (lane == 0) {
    // two-queue Huffman merge: leaves 0..m-1 (sorted), internal nodes m..2m-2 in creation order
    uint32_t li = 0, ii = 0, ni = 0;
    auto wt = [&](uint32_t node) { return node < m ? freq[S.sorted[node]] : S.weight[node - m]; };
    for (uint32_t k = 0; k + 1 < m; k++) {
      const uint32_t a = (li < m && (ii >= ni || wt(li) <= S.weight[ii])) ? li++ : m + ii++;
      const uint32_t b = (li < m && (ii >= ni || wt(li) <= S.weight[ii])) ? li++ : m + ii++;
      S.weight[ni] = wt(a) + wt(b);
      S.parent[a] = (uint16_t)(m + ni);
      S.parent[b] = (uint16_t)(m + ni);
      ni++;
    }
    // depths top-down (a parent's index is above its children's), each clamped to maxlen from its
    // parent's clamped depth; every clamped node counts as an overflow, internal ones included
    // (zlib gen_bitlen's first pass: counting leaves only leaves the code over-subscribed)
    const uint32_t root = 2 * m - 2;
    S.depth[root] = 0;
    for (uint32_t b = 0; b < 16; b++) S.blc[b] = 0;
    int overflow = 0;
    for (int node = (int)root - 1; node >= 0; node--) {
      uint32_t d = S.depth[S.parent[node]] + 1u;
      if (d > maxlen) {
        d = maxlen;
        overflow++;
      }
      S.depth[node] = (uint8_t)d;
      if (node < (int)m) S.blc[d]++;
    }
    while (overflow > 0) {  // zlib gen_bitlen: move leaves down until the counts fit the limit
      uint32_t bits = maxlen - 1;
      while (S.blc[bits] == 0) bits--;
      S.blc[bits]--;
      S.blc[bits + 1] += 2;
      S.blc[maxlen]--;
      overflow -= 2;
    }
    uint32_t idx = 0;  // the least frequent leaves take the longest codes
    for (uint32_t len = maxlen; len >= 1; len--)
      for (uint32_t c = 0; c < S.blc[len]; c++) lens[S.sorted[idx++]] = (uint8_t)len;
  }
  __syncthreads();
}

}  // namespace zgpu
