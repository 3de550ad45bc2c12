// Fused final decode stage for gfx950: bytes codec (endianness swap) + transpose codec(s) +
// numcodecs.shuffle (innermost position only) + scatter of the chunk selection into the output
// array (ArrayBytesFixedDisjointView::copy_from_slice / fill).
//
// Reference semantics restated (paths relative to the zarrs workspace root):
//   endianness   zarrs_data_type/src/codec_traits/bytes.rs:97-131 (reverse each component)
//   transpose    zarrs/src/array/codec/array_to_array/transpose.rs:110-135,223-266
//                (decoded dec[c] = enc[e], e_a = c[order[a]]; composed over all a2a codecs)
//   unshuffle    zarrs/src/array/codec/bytes_to_bytes/shuffle/shuffle_codec.rs:109-129
//   scatter/fill zarrs_codec/src/array_bytes_fixed_disjoint_view.rs:144-206
//   size check   zarrs_codec/src/array_bytes.rs:376-386 (UnexpectedChunkDecodedSize)
//
// Three kernels, chosen per batch on the host from the chain's composed permutation:
//   k_scatter_rows   the encoded innermost axis is the decoded innermost axis: contiguous rows,
//                    16-B vector copy when every row is 16-B aligned, element copy otherwise.
//   k_scatter_tiled  a true innermost transpose: 64x64-element tiles staged through LDS so both
//                    the encoded read and the output write are row-contiguous (HBM bound).
//   k_scatter_generic anything else (fused shuffle + transpose, odd element sizes): one thread
//                    per output element, coalesced writes.
#include <hip/hip_runtime.h>

#include <algorithm>

#include "../common.hpp"
#include "launch.hpp"
#include "dev.hpp"

namespace zgpu {

// Load one element of `es` bytes (es <= 16) from a possibly unaligned address, apply the
// endianness reversal of each `comp`-byte component, and return it in a 16-byte register.
__device__ __forceinline__ uint4 load_elem(const uint8_t *p, uint32_t es, uint32_t comp, uint32_t swap) {
  uint8_t b[16];
  uintptr_t a = (uintptr_t)p;
  if (es == 4 && (a & 3) == 0) {
    uint32_t w = *(const uint32_t *)p;
    if (swap) w = swap_word(w, comp);
    return make_uint4(w, 0, 0, 0);
  }
  if (es == 2 && (a & 1) == 0) {
    uint32_t w = *(const uint16_t *)p;
    if (swap) w = ((w >> 8) | (w << 8)) & 0xFFFFu;
    return make_uint4(w, 0, 0, 0);
  }
  if (es == 8 && (a & 7) == 0) {
    uint2 w = *(const uint2 *)p;
    uint4 v = make_uint4(w.x, w.y, 0, 0);
    if (swap) {
      if (comp == 8) v = make_uint4(__builtin_bswap32(w.y), __builtin_bswap32(w.x), 0, 0);
      else v = make_uint4(swap_word(w.x, comp), swap_word(w.y, comp), 0, 0);
    }
    return v;
  }
  for (uint32_t i = 0; i < es; i++) b[i] = p[i];
  if (swap && comp > 1)
    for (uint32_t c0 = 0; c0 < es; c0 += comp)
      for (uint32_t x = 0, y = comp - 1; x < y; x++, y--) {
        uint8_t t = b[c0 + x]; b[c0 + x] = b[c0 + y]; b[c0 + y] = t;
      }
  for (uint32_t i = es; i < 16; i++) b[i] = 0;
  uint4 v;
  v.x = b[0] | b[1] << 8 | b[2] << 16 | (uint32_t)b[3] << 24;
  v.y = b[4] | b[5] << 8 | b[6] << 16 | (uint32_t)b[7] << 24;
  v.z = b[8] | b[9] << 8 | b[10] << 16 | (uint32_t)b[11] << 24;
  v.w = b[12] | b[13] << 8 | b[14] << 16 | (uint32_t)b[15] << 24;
  return v;
}

__device__ __forceinline__ void store_elem(uint8_t *p, uint4 v, uint32_t es) {
  uintptr_t a = (uintptr_t)p;
  if (es == 4 && (a & 3) == 0) { *(uint32_t *)p = v.x; return; }
  if (es == 2 && (a & 1) == 0) { *(uint16_t *)p = (uint16_t)v.x; return; }
  if (es == 8 && (a & 7) == 0) { *(uint2 *)p = make_uint2(v.x, v.y); return; }
  if (es == 1) { *p = (uint8_t)v.x; return; }
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  for (uint32_t i = 0; i < es; i++) p[i] = (uint8_t)(w[i >> 2] >> (8 * (i & 3)));
}

__device__ __forceinline__ uint4 fill_elem(const ZgScatter &P) {
  uint4 v;
  v.x = P.fill[0] | P.fill[1] << 8 | P.fill[2] << 16 | (uint32_t)P.fill[3] << 24;
  v.y = P.fill[4] | P.fill[5] << 8 | P.fill[6] << 16 | (uint32_t)P.fill[7] << 24;
  v.z = P.fill[8] | P.fill[9] << 8 | P.fill[10] << 16 | (uint32_t)P.fill[11] << 24;
  v.w = P.fill[12] | P.fill[13] << 8 | P.fill[14] << 16 | (uint32_t)P.fill[15] << 24;
  return v;
}

// Validate the decoded byte count of a non-fill item; returns false if the item is dead.
__device__ __forceinline__ bool item_live(const ZgItem &it, uint32_t *status, uint32_t i,
                                          const ZgScatter &P) {
  if (status[i] || (it.flags & ZG_ITEM_DIRECT)) return false;
  if (!(it.flags & ZG_ITEM_FILL) && it.len != P.nelem * P.es) {
    if (threadIdx.x == 0) status[i] = ZG_DECODED_SIZE_MISMATCH;
    return false;
  }
  return true;
}

__device__ __forceinline__ void store16(bool nt, uint8_t *d, uint4 v) {
  if (nt) nt_store16(d, v);
  else *(uint4 *)d = v;
}

// ---------------------------------------------------------------------------------------------
// Rows: block = (item, group of ROWS rows). Row offsets are computed once per row into LDS.
// ---------------------------------------------------------------------------------------------
constexpr int ROWS_PER_BLOCK = 64;
constexpr int SCATTER_THREADS = 256;

// One (item, group of ROWS_PER_BLOCK rows) unit of the rows scatter; every early exit is block-uniform.
__device__ __forceinline__ void rows_unit(const ZgItem *__restrict__ items, const uint64_t *__restrict__ geom,
                                          uint32_t *__restrict__ status, const ZgScatter &P,
                                          uint8_t *__restrict__ out, uint32_t item, uint32_t blk) {
  const ZgItem it = items[item];
  if (!item_live(it, status, item, P)) return;
  const uint32_t nd = P.nd;
  const uint64_t *g = geom + (uint64_t)item * 3 * nd;  // sel_start | sel_shape | out_start
  uint64_t nrows = 1;
  for (uint32_t d = 0; d + 1 < nd; d++) nrows *= g[nd + d];
  const uint64_t row0 = (uint64_t)blk * ROWS_PER_BLOCK;
  if (row0 >= nrows) return;
  const uint32_t nr = (uint32_t)min<uint64_t>(ROWS_PER_BLOCK, nrows - row0);
  const uint64_t L = g[nd + nd - 1];  // row length (elements)
  const uint32_t es = P.es;

  __shared__ uint64_t s_src[ROWS_PER_BLOCK], s_dst[ROWS_PER_BLOCK];
  __shared__ int s_misaligned;
  if (threadIdx.x == 0) s_misaligned = 0;
  __syncthreads();
  const bool fill = it.flags & ZG_ITEM_FILL;
  if (threadIdx.x < nr) {
    uint64_t r = row0 + threadIdx.x, so = g[nd - 1] * P.enc_stride[nd - 1], dof = g[2 * nd + nd - 1];
    for (int d = (int)nd - 2; d >= 0; d--) {
      const uint64_t ext = g[nd + d], c = r % ext;
      r /= ext;
      so += (g[d] + c) * P.enc_stride[d];
      dof += (g[2 * nd + d] + c) * P.out_stride[d];
    }
    const uint64_t sb = it.src + so * es, db = (uint64_t)out + dof * es;
    s_src[threadIdx.x] = sb;
    s_dst[threadIdx.x] = db;
    if (((fill ? 0 : sb) | db | (L * es)) & 15) s_misaligned = 1;
  }
  __syncthreads();
  const uint32_t swap = P.swap && P.comp > 1;
  if (!s_misaligned && !P.shuffle) {
    // 16-B vectors: every row start and length is 16-B aligned.
    const uint32_t vpr = (uint32_t)(L * es / 16);
    const uint32_t total = nr * vpr;
    const uint4 fv = fill ? fill_elem(P) : make_uint4(0, 0, 0, 0);
    uint4 fvec = fv;
    if (fill) {  // replicate the element over 16 bytes
      uint8_t b[16];
      for (int i = 0; i < 16; i++) b[i] = P.fill[i % es];
      fvec.x = b[0] | b[1] << 8 | b[2] << 16 | (uint32_t)b[3] << 24;
      fvec.y = b[4] | b[5] << 8 | b[6] << 16 | (uint32_t)b[7] << 24;
      fvec.z = b[8] | b[9] << 8 | b[10] << 16 | (uint32_t)b[11] << 24;
      fvec.w = b[12] | b[13] << 8 | b[14] << 16 | (uint32_t)b[15] << 24;
    }
    for (uint32_t v = threadIdx.x; v < total; v += SCATTER_THREADS) {
      const uint32_t r = v / vpr, c = v % vpr;
      uint4 x;
      if (fill) {
        x = fvec;
      } else {
        x = *(const uint4 *)(s_src[r] + (uint64_t)c * 16);
        if (swap) x = swap_vec(x, P.comp);
      }
      *(uint4 *)(s_dst[r] + (uint64_t)c * 16) = x;
    }
    return;
  }
  if (P.shuffle && !fill && (es == 2 || es == 4)) {
    // Fused unshuffle, 16 output bytes per thread: byte plane k of the chunk holds byte k of every
    // element (shuffle_codec.rs:109-129), so 16/es consecutive elements take 16/es bytes from each
    // plane (one 8- or 4-byte load per plane) and are interleaved with byte permutes into one
    // 16-byte store. Needs rows of whole vectors on aligned plane and output addresses.
    const uint32_t epv = 16 / es;  // elements per vector
    const uint64_t s0 = (s_src[0] - it.src) / es;
    bool vec_ok = (L % epv) == 0 && (P.nelem % epv) == 0 && ((it.src & 15) == 0);
    for (uint32_t r = 0; r < nr && vec_ok; r++)
      vec_ok = (((s_src[r] - it.src) / es) % epv) == 0 && (s_dst[r] & 15) == 0;
    (void)s0;
    if (vec_ok && es == 2 && P.pad0) {
      // A/B (ZGPU_UNSHUFFLE_WIDE=1: non-temporal loads, 2: plain loads; off by default): u16 rows of
      // whole 16-element units on 16-B aligned plane offsets, each unit one 16-B load per plane and
      // two 16-B stores, two units per thread in flight. C5 with non-temporal loads: 71.8 ms against
      // 70.8-71.1 with the 8-B plane loads below (profiles/r06/r06us_c5_unshuffle_wide_ab.txt)
      bool wide = (L % 16) == 0 && (P.nelem % 16) == 0;
      for (uint32_t r = 0; r < nr && wide; r++) wide = (((s_src[r] - it.src) / 2) % 16) == 0;
      if (wide) {
        const uint32_t upr = (uint32_t)(L / 16);
        const uint32_t tot = nr * upr;
        const uint8_t *base = (const uint8_t *)it.src;
        for (uint32_t u0 = threadIdx.x; u0 < tot; u0 += 2 * SCATTER_THREADS) {
          uint4 a[2], b[2];
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const uint32_t u = u0 + q * SCATTER_THREADS;
            if (u < tot) {
              const uint32_t r = u / upr, c = u % upr;
              const uint64_t e0 = (s_src[r] - it.src) / 2 + (uint64_t)c * 16;
              if (P.pad0 == 1) {
                a[q] = nt_load16(base + e0);
                b[q] = nt_load16(base + P.nelem + e0);
              } else {
                a[q] = *(const uint4 *)(base + e0);
                b[q] = *(const uint4 *)(base + P.nelem + e0);
              }
            }
          }
#pragma unroll
          for (int q = 0; q < 2; q++) {
            const uint32_t u = u0 + q * SCATTER_THREADS;
            if (u < tot) {
              const uint32_t r = u / upr, c = u % upr;
              const uint4 lo = swap ? b[q] : a[q], hi = swap ? a[q] : b[q];
              uint8_t *d = (uint8_t *)(s_dst[r] + (uint64_t)c * 32);
              store16(P.pad0 == 1, d, make_uint4(__builtin_amdgcn_perm(hi.x, lo.x, 0x05010400u),
                                       __builtin_amdgcn_perm(hi.x, lo.x, 0x07030602u),
                                       __builtin_amdgcn_perm(hi.y, lo.y, 0x05010400u),
                                       __builtin_amdgcn_perm(hi.y, lo.y, 0x07030602u)));
              store16(P.pad0 == 1, d + 16, make_uint4(__builtin_amdgcn_perm(hi.z, lo.z, 0x05010400u),
                                            __builtin_amdgcn_perm(hi.z, lo.z, 0x07030602u),
                                            __builtin_amdgcn_perm(hi.w, lo.w, 0x05010400u),
                                            __builtin_amdgcn_perm(hi.w, lo.w, 0x07030602u)));
            }
          }
        }
        return;
      }
    }
    if (vec_ok) {
      const uint32_t vpr = (uint32_t)(L / epv);
      const uint32_t total = nr * vpr;
      const uint8_t *base = (const uint8_t *)it.src;
      for (uint32_t v = threadIdx.x; v < total; v += SCATTER_THREADS) {
        const uint32_t r = v / vpr, c = v % vpr;
        const uint64_t e0 = (s_src[r] - it.src) / es + (uint64_t)c * epv;  // first element
        uint32_t w[4];
        if (es == 2) {
          const uint2 a = *(const uint2 *)(base + e0), b = *(const uint2 *)(base + P.nelem + e0);
          // bytes of element j: plane 0 byte j, plane 1 byte j (swapped for big-endian u16)
          const uint2 lo = swap ? b : a, hi = swap ? a : b;
          w[0] = __builtin_amdgcn_perm(hi.x, lo.x, 0x05010400u);
          w[1] = __builtin_amdgcn_perm(hi.x, lo.x, 0x07030602u);
          w[2] = __builtin_amdgcn_perm(hi.y, lo.y, 0x05010400u);
          w[3] = __builtin_amdgcn_perm(hi.y, lo.y, 0x07030602u);
        } else {
          uint32_t pl[4];
#pragma unroll
          for (int k = 0; k < 4; k++) pl[k] = *(const uint32_t *)(base + (uint64_t)k * P.nelem + e0);
          // element j = bytes j of planes 0..3; a 4x4 byte transpose
          const uint32_t t0 = __builtin_amdgcn_perm(pl[1], pl[0], 0x05010400u);  // p0b0 p1b0 p0b1 p1b1
          const uint32_t t1 = __builtin_amdgcn_perm(pl[1], pl[0], 0x07030602u);  // p0b2 p1b2 p0b3 p1b3
          const uint32_t t2 = __builtin_amdgcn_perm(pl[3], pl[2], 0x05010400u);
          const uint32_t t3 = __builtin_amdgcn_perm(pl[3], pl[2], 0x07030602u);
          w[0] = __builtin_amdgcn_perm(t2, t0, 0x05040100u);  // e0: p0b0 p1b0 p2b0 p3b0
          w[1] = __builtin_amdgcn_perm(t2, t0, 0x07060302u);  // e1
          w[2] = __builtin_amdgcn_perm(t3, t1, 0x05040100u);  // e2
          w[3] = __builtin_amdgcn_perm(t3, t1, 0x07060302u);  // e3
          if (swap) {
#pragma unroll
            for (int k = 0; k < 4; k++) w[k] = swap_word(w[k], P.comp);
          }
        }
        *(uint4 *)(s_dst[r] + (uint64_t)c * 16) = make_uint4(w[0], w[1], w[2], w[3]);
      }
      return;
    }
  }
  // Element path (unaligned rows, odd sizes, fused unshuffle).
  const uint64_t total = (uint64_t)nr * L;
  const uint4 fv = fill_elem(P);
  for (uint64_t v = threadIdx.x; v < total; v += SCATTER_THREADS) {
    const uint32_t r = (uint32_t)(v / L);
    const uint64_t c = v % L;
    uint4 x;
    if (fill) {
      x = fv;
    } else if (P.shuffle) {
      // element s of the chunk: byte b lives at src[b * nelem + s]
      const uint64_t s = (s_src[r] - it.src) / es + c;
      const uint8_t *base = (const uint8_t *)it.src;
      uint8_t b[16];
      for (uint32_t k = 0; k < es; k++) b[k] = base[(uint64_t)k * P.nelem + s];
      if (swap)
        for (uint32_t c0 = 0; c0 < es; c0 += P.comp)
          for (uint32_t a = 0, bb = P.comp - 1; a < bb; a++, bb--) {
            uint8_t t = b[c0 + a]; b[c0 + a] = b[c0 + bb]; b[c0 + bb] = t;
          }
      uint32_t w[4] = {0, 0, 0, 0};
      for (uint32_t k = 0; k < es; k++) w[k >> 2] |= (uint32_t)b[k] << (8 * (k & 3));
      x = make_uint4(w[0], w[1], w[2], w[3]);
    } else {
      x = load_elem((const uint8_t *)(s_src[r] + c * es), es, P.comp, swap);
    }
    store_elem((uint8_t *)(s_dst[r] + c * es), x, es);
  }
}

__global__ __launch_bounds__(SCATTER_THREADS) void k_scatter_rows(
    const ZgItem *__restrict__ items, const uint64_t *__restrict__ geom, uint32_t *__restrict__ status,
    ZgScatter P, uint8_t *__restrict__ out, uint32_t blocks_per_item, uint64_t block_base) {
  const uint64_t bid = block_base + blockIdx.x;
  rows_unit(items, geom, status, P, out, (uint32_t)(bid / blocks_per_item), (uint32_t)(bid % blocks_per_item));
}

// The items still to scatter after a stage that wrote most of them into the output itself
// (ZG_ITEM_DIRECT: k_gzip's whole chunks): k_live_items lists them, and a grid of a few blocks per CU
// walks their units -- a full grid spent most of its time dispatching blocks that only exit (C3: 195 k
// of 250 k).
__global__ void k_live_items(const ZgItem *__restrict__ items, const uint32_t *__restrict__ status, uint32_t n,
                             uint32_t *__restrict__ list, uint32_t *__restrict__ count) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n && !status[i] && !(items[i].flags & ZG_ITEM_DIRECT)) list[atomicAdd(count, 1u)] = i;
}

__global__ __launch_bounds__(SCATTER_THREADS) void k_scatter_rows_list(
    const ZgItem *__restrict__ items, const uint64_t *__restrict__ geom, uint32_t *__restrict__ status,
    ZgScatter P, uint8_t *__restrict__ out, uint32_t blocks_per_item, const uint32_t *__restrict__ list,
    const uint32_t *__restrict__ count) {
  const uint64_t total = (uint64_t)*count * blocks_per_item;
  for (uint64_t w = blockIdx.x; w < total; w += gridDim.x) {
    __syncthreads();  // the previous unit's row tables are no longer read
    rows_unit(items, geom, status, P, out, list[w / blocks_per_item], (uint32_t)(w % blocks_per_item));
  }
}

// ---------------------------------------------------------------------------------------------
// Tiled transpose: decoded axis A = P.tile_a is innermost (stride 1) in the encoded layout,
// decoded axis Lx = nd-1 is innermost in the output. A slab is a TILE x TILE tile over (A, Lx) for
// fixed values of the other axes; loaded along A (contiguous), stored along Lx (contiguous) via
// LDS. One block moves TJ slabs at consecutive values of axis B = P.tile_b (the other axis with the
// smallest encoded stride), so for a full chunk the TJ encoded rows of one Lx index are ONE
// contiguous run (TJ x 256 B for f32 64^3) and every thread keeps TJ*4 16-B loads in flight.
// Every byte is touched once, so loads and stores are non-temporal (no L2 retention).
// Measured on MI355X (tools/lab/scatter_lab.hip, 4096 x 64^3 f32 chunks): TJ 1 -> 5.19 TB/s,
// TJ 2 -> 5.48, TJ 4 -> 5.81, TJ 4 + nt -> 5.98 TB/s; TJ 8 (1 block/CU) is slower again.
// ---------------------------------------------------------------------------------------------
constexpr int TILE = 64;

template <int ES>
__global__ __launch_bounds__(SCATTER_THREADS) void k_scatter_tiled(
    const ZgItem *__restrict__ items, const uint64_t *__restrict__ geom, uint32_t *__restrict__ status,
    ZgScatter P, uint8_t *__restrict__ out, uint32_t tiles_per_item, uint64_t block_base) {
  using T = typename std::conditional<ES == 1, uint8_t, typename std::conditional<ES == 2, uint16_t,
            typename std::conditional<ES == 4, uint32_t, uint2>::type>::type>::type;
  constexpr int TJ = tiled_slabs(ES);
  constexpr int PITCH = TILE + (ES >= 4 ? 1 : 4 / ES);  // +1 word: column reads conflict-free
  constexpr int SLAB = TILE * PITCH + (ES >= 4 ? 1 : 4 / ES);  // +1 word: slabs on distinct banks
  __shared__ T tile[TJ * SLAB];
  const uint64_t bid = block_base + blockIdx.x;
  const uint32_t item = (uint32_t)(bid / tiles_per_item);
  uint32_t t = (uint32_t)(bid % tiles_per_item);
  const ZgItem it = items[item];
  if (!item_live(it, status, item, P)) return;
  const uint32_t nd = P.nd, A = P.tile_a, Lx = nd - 1, B = P.tile_b;
  const uint64_t *g = geom + (uint64_t)item * 3 * nd;
  const uint64_t *ss = g, *sh = g + nd, *os = g + 2 * nd;
  const bool hasB = B < nd;
  const uint64_t bext = hasB ? sh[B] : 1;
  const uint32_t nta = (uint32_t)((sh[A] + TILE - 1) / TILE), ntl = (uint32_t)((sh[Lx] + TILE - 1) / TILE);
  const uint32_t nbg = (uint32_t)((bext + TJ - 1) / TJ);
  const uint32_t ta = t % nta; t /= nta;
  const uint32_t tl = t % ntl; t /= ntl;
  const uint32_t tb = t % nbg; t /= nbg;
  // remaining index enumerates the other axes (row-major over axes != A, Lx, B)
  uint64_t so = 0, dof = 0, rem = t;
  for (int d = (int)nd - 1; d >= 0; d--) {
    if ((uint32_t)d == A || (uint32_t)d == Lx || (uint32_t)d == B) continue;
    const uint64_t c = rem % sh[d];
    rem /= sh[d];
    so += (ss[d] + c) * P.enc_stride[d];
    dof += (os[d] + c) * P.out_stride[d];
  }
  if (rem) return;  // beyond this item's selection
  const uint64_t a0 = (uint64_t)ta * TILE, l0 = (uint64_t)tl * TILE, b0 = (uint64_t)tb * TJ;
  const uint32_t na = (uint32_t)min<uint64_t>(TILE, sh[A] - a0), nl = (uint32_t)min<uint64_t>(TILE, sh[Lx] - l0);
  const uint32_t nb = (uint32_t)min<uint64_t>(TJ, bext - b0);
  const uint64_t sL = P.enc_stride[Lx], dA = P.out_stride[A];
  const uint64_t sB = hasB ? P.enc_stride[B] : 0, dB = hasB ? P.out_stride[B] : 0;
  so += (ss[A] + a0) * P.enc_stride[A] + (ss[Lx] + l0) * sL + (hasB ? (ss[B] + b0) * sB : 0);
  dof += (os[A] + a0) * dA + (os[Lx] + l0) + (hasB ? (os[B] + b0) * dB : 0);
  T *dst = (T *)(out) + dof;
  constexpr int VPR = TILE * ES / 16;  // 16-B vectors per tile row
  constexpr int EPV = 16 / ES;         // elements per vector
  constexpr int NV = TJ * TILE * VPR;  // vectors per block
  const bool oaligned = (((uint64_t)dst & 15) == 0) && ((dA * ES) % 16 == 0) && ((dB * ES) % 16 == 0) &&
                        nl == TILE;
  if (it.flags & ZG_ITEM_FILL) {
    T fv;
    __builtin_memcpy(&fv, P.fill, ES);
    if (oaligned) {
      uint4 x;
      T *xe = (T *)&x;
#pragma unroll
      for (int k = 0; k < EPV; k++) xe[k] = fv;
      for (uint32_t e = threadIdx.x; e < (uint32_t)NV; e += SCATTER_THREADS) {
        const uint32_t a = e / (TJ * VPR), jj = (e / VPR) % TJ, v = e % VPR;
        if (a < na && jj < nb) nt_store16(dst + jj * dB + (uint64_t)a * dA + v * EPV, x);
      }
    } else {
      for (uint32_t e = threadIdx.x; e < (uint32_t)(TJ * TILE * TILE); e += SCATTER_THREADS) {
        const uint32_t a = e / (TJ * TILE), jj = (e / TILE) % TJ, l = e % TILE;
        if (a < na && jj < nb && l < nl) dst[jj * dB + (uint64_t)a * dA + l] = fv;
      }
    }
    return;
  }
  const T *src = (const T *)(it.src) + so;
  const uint32_t swap = P.swap && P.comp > 1;
  const bool aligned = (((uint64_t)src & 15) == 0) && ((sL * ES) % 16 == 0) && ((sB * ES) % 16 == 0) &&
                       na == TILE;
  if (aligned) {
    // e -> (row l, slab jj, vector v): a wave reads TJ adjacent encoded rows = one contiguous run
    constexpr int PER = NV / SCATTER_THREADS;
    uint4 x[PER];
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const uint32_t e = p * SCATTER_THREADS + threadIdx.x;
      const uint32_t l = e / (TJ * VPR), jj = (e / VPR) % TJ, v = e % VPR;
      if (l < nl && jj < nb) x[p] = nt_load16(src + jj * sB + (uint64_t)l * sL + v * EPV);
    }
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const uint32_t e = p * SCATTER_THREADS + threadIdx.x;
      const uint32_t l = e / (TJ * VPR), jj = (e / VPR) % TJ, v = e % VPR;
      if (l < nl && jj < nb) {
        uint4 y = swap ? swap_vec(x[p], P.comp) : x[p];
        const T *ye = (const T *)&y;
#pragma unroll
        for (int k = 0; k < EPV; k++) tile[jj * SLAB + l * PITCH + v * EPV + k] = ye[k];
      }
    }
  } else {
    for (uint32_t e = threadIdx.x; e < (uint32_t)(TJ * TILE * TILE); e += SCATTER_THREADS) {
      const uint32_t l = e / (TJ * TILE), jj = (e / TILE) % TJ, a = e % TILE;
      if (l < nl && jj < nb && a < na) {
        uint4 y = load_elem((const uint8_t *)(src + jj * sB + (uint64_t)l * sL + a), ES, P.comp, swap);
        T v;
        __builtin_memcpy(&v, &y, ES);
        tile[jj * SLAB + l * PITCH + a] = v;
      }
    }
  }
  __syncthreads();
  if (oaligned) {
#pragma unroll
    for (int p = 0; p < NV / SCATTER_THREADS; p++) {
      const uint32_t e = p * SCATTER_THREADS + threadIdx.x;
      const uint32_t a = e / (TJ * VPR), jj = (e / VPR) % TJ, v = e % VPR;
      if (a < na && jj < nb) {
        uint4 y;
        T *ye = (T *)&y;
#pragma unroll
        for (int k = 0; k < EPV; k++) ye[k] = tile[jj * SLAB + (v * EPV + k) * PITCH + a];
        nt_store16(dst + jj * dB + (uint64_t)a * dA + v * EPV, y);
      }
    }
  } else {
    for (uint32_t e = threadIdx.x; e < (uint32_t)(TJ * TILE * TILE); e += SCATTER_THREADS) {
      const uint32_t a = e / (TJ * TILE), jj = (e / TILE) % TJ, l = e % TILE;
      if (a < na && jj < nb && l < nl) dst[jj * dB + (uint64_t)a * dA + l] = tile[jj * SLAB + l * PITCH + a];
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Generic element gather: one thread per selected element.
// ---------------------------------------------------------------------------------------------
__global__ __launch_bounds__(SCATTER_THREADS) void k_scatter_generic(
    const ZgItem *__restrict__ items, const uint64_t *__restrict__ geom, uint32_t *__restrict__ status,
    ZgScatter P, uint8_t *__restrict__ out, uint32_t blocks_per_item, uint64_t block_base) {
  const uint64_t bid = block_base + blockIdx.x;
  const uint32_t item = (uint32_t)(bid / blocks_per_item);
  const uint32_t blk = (uint32_t)(bid % blocks_per_item);
  const ZgItem it = items[item];
  if (!item_live(it, status, item, P)) return;
  const uint32_t nd = P.nd, es = P.es;
  const uint64_t *g = geom + (uint64_t)item * 3 * nd;
  uint64_t n = 1;
  for (uint32_t d = 0; d < nd; d++) n *= g[nd + d];
  const uint64_t e = (uint64_t)blk * SCATTER_THREADS + threadIdx.x;
  if (e >= n) return;
  uint64_t rem = e, so = 0, dof = 0;
  for (int d = (int)nd - 1; d >= 0; d--) {
    const uint64_t c = rem % g[nd + d];
    rem /= g[nd + d];
    so += (g[d] + c) * P.enc_stride[d];
    dof += (g[2 * nd + d] + c) * P.out_stride[d];
  }
  const uint32_t swap = P.swap && P.comp > 1;
  uint4 x;
  if (it.flags & ZG_ITEM_FILL) {
    x = fill_elem(P);
  } else if (P.shuffle) {
    const uint8_t *base = (const uint8_t *)it.src;
    uint8_t b[16];
    for (uint32_t k = 0; k < es; k++) b[k] = base[(uint64_t)k * P.nelem + so];
    if (swap)
      for (uint32_t c0 = 0; c0 < es; c0 += P.comp)
        for (uint32_t a = 0, bb = P.comp - 1; a < bb; a++, bb--) {
          uint8_t t = b[c0 + a]; b[c0 + a] = b[c0 + bb]; b[c0 + bb] = t;
        }
    uint32_t w[4] = {0, 0, 0, 0};
    for (uint32_t k = 0; k < es; k++) w[k >> 2] |= (uint32_t)b[k] << (8 * (k & 3));
    x = make_uint4(w[0], w[1], w[2], w[3]);
  } else {
    x = load_elem((const uint8_t *)it.src + so * es, es, P.comp, swap);
  }
  store_elem(out + dof * es, x, es);
}

// ---------------------------------------------------------------------------------------------
hipError_t launch_scatter(const ZgItem *items, const uint64_t *geom, uint32_t *status, const ZgScatter &P,
                          uint8_t *out, uint32_t n_items, uint32_t mode, uint64_t units_per_item,
                          hipStream_t s, uint32_t *live_scratch) {
  if (n_items == 0 || units_per_item == 0) return hipSuccess;
  if (units_per_item > 0xFFFFFFFFull) return hipErrorInvalidConfiguration;
  if (live_scratch && mode == SCATTER_ROWS) {  // [count | list of n_items]
    hipError_t e = hipMemsetAsync(live_scratch, 0, 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_live_items, dim3((n_items + 255) / 256), dim3(256), 0, s, items, status, n_items,
                       live_scratch + 1, live_scratch);
    int dev = 0, ncu = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                 hipSuccess || ncu <= 0)
      ncu = 256;
    const uint64_t g = std::min<uint64_t>((uint64_t)n_items * units_per_item, (uint64_t)ncu * 8);
    hipLaunchKernelGGL(k_scatter_rows_list, dim3((uint32_t)g), dim3(SCATTER_THREADS), 0, s, items, geom, status, P,
                       out, (uint32_t)units_per_item, live_scratch + 1, live_scratch);
    return hipGetLastError();
  }
  const uint64_t total = (uint64_t)n_items * units_per_item;
  const uint32_t u = (uint32_t)units_per_item;
  // gridDim.x * blockDim.x must stay below 2^32: launch the block range in slices
  const uint64_t MAXG = max_grid_blocks(SCATTER_THREADS);
  for (uint64_t base = 0; base < total; base += MAXG) {
    const dim3 g((uint32_t)std::min<uint64_t>(MAXG, total - base));
    switch (mode) {
      case SCATTER_ROWS:
        hipLaunchKernelGGL(k_scatter_rows, g, dim3(SCATTER_THREADS), 0, s, items, geom, status, P, out, u, base);
        break;
      case SCATTER_TILED:
        switch (P.es) {
          case 1: hipLaunchKernelGGL(k_scatter_tiled<1>, g, dim3(SCATTER_THREADS), 0, s, items, geom, status, P, out, u, base); break;
          case 2: hipLaunchKernelGGL(k_scatter_tiled<2>, g, dim3(SCATTER_THREADS), 0, s, items, geom, status, P, out, u, base); break;
          case 4: hipLaunchKernelGGL(k_scatter_tiled<4>, g, dim3(SCATTER_THREADS), 0, s, items, geom, status, P, out, u, base); break;
          case 8: hipLaunchKernelGGL(k_scatter_tiled<8>, g, dim3(SCATTER_THREADS), 0, s, items, geom, status, P, out, u, base); break;
          default: return hipErrorInvalidValue;
        }
        break;
      default:
        hipLaunchKernelGGL(k_scatter_generic, g, dim3(SCATTER_THREADS), 0, s, items, geom, status, P, out, u, base);
    }
    const hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  return hipSuccess;
}

uint64_t scatter_units_per_item(uint32_t mode, const ZgScatter &P, const uint64_t *max_sel_shape) {
  const uint32_t nd = P.nd;
  if (mode == SCATTER_ROWS) {
    uint64_t rows = 1;
    for (uint32_t d = 0; d + 1 < nd; d++) rows *= max_sel_shape[d];
    return (rows + ROWS_PER_BLOCK - 1) / ROWS_PER_BLOCK;
  }
  if (mode == SCATTER_TILED) {
    const uint64_t tj = tiled_slabs(P.es);
    uint64_t t = 1;
    for (uint32_t d = 0; d < nd; d++) {
      if (d == P.tile_a || d == nd - 1) t *= (max_sel_shape[d] + TILE - 1) / TILE;
      else if (d == P.tile_b) t *= (max_sel_shape[d] + tj - 1) / tj;
      else t *= max_sel_shape[d];
    }
    return t;
  }
  uint64_t n = 1;
  for (uint32_t d = 0; d < nd; d++) n *= max_sel_shape[d];
  return (n + SCATTER_THREADS - 1) / SCATTER_THREADS;
}

}  // namespace zgpu

namespace zgpu {

// Box copy between two device arrays (coalesced calls: a caller's window of the batch's stacked
// output packed into its compact layout before the one D2H copy). One wave per contiguous run; 16-B
// lanes when both runs and their length allow it, else 4-B, else bytes.
// One-wave workgroups: the coalesced drop-in path launches this while other lanes' decodes hold the
// CUs with long-running one-wave items, and a 4-wave workgroup waited for four free slots on one CU
// (trace: 11 ms median for 30-60 MB packs).
__global__ __launch_bounds__(64) void k_box_copy(const uint8_t *__restrict__ src, uint8_t *__restrict__ dst,
                                                   ZgBoxCopy P) {
  const uint32_t lane = threadIdx.x & 63;
  const uint64_t waves = (uint64_t)gridDim.x * (blockDim.x >> 6);
  for (uint64_t r = (uint64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6); r < P.n_runs; r += waves) {
    uint64_t k = r, so = 0, dof = 0;
    for (int d = (int)P.outer - 1; d >= 0; d--) {
      const uint64_t c = k % P.shape[d];
      k /= P.shape[d];
      so += c * P.src_stride[d];
      dof += c * P.dst_stride[d];
    }
    const uint8_t *s = src + P.src_base + so;
    uint8_t *t = dst + P.dst_base + dof;
    const uint64_t n = P.run_bytes;
    if ((((uintptr_t)s | (uintptr_t)t | n) & 15) == 0) {
      for (uint64_t i = (uint64_t)lane * 16; i < n; i += 64 * 16)
        *(uint4 *)(t + i) = *(const uint4 *)(s + i);
    } else if ((((uintptr_t)s | (uintptr_t)t | n) & 3) == 0) {
      for (uint64_t i = (uint64_t)lane * 4; i < n; i += 64 * 4)
        *(uint32_t *)(t + i) = *(const uint32_t *)(s + i);
    } else {
      for (uint64_t i = lane; i < n; i += 64) t[i] = s[i];
    }
  }
}

hipError_t launch_box_copy(const uint8_t *src, uint8_t *dst, const ZgBoxCopy &P, hipStream_t s) {
  if (!P.n_runs || !P.run_bytes) return hipSuccess;
  const uint64_t blocks = std::min<uint64_t>(P.n_runs, (uint64_t)device_cu_count() * 64);
  hipLaunchKernelGGL(k_box_copy, dim3((uint32_t)blocks), dim3(64), 0, s, src, dst, P);
  return hipGetLastError();
}

}  // namespace zgpu
