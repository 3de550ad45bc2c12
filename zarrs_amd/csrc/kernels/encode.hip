// Chunk encode (the write side of the same chain): array -> encoded chunks
// for fixed-size chains. CodecChain::encode (zarrs/src/array/codec/array_to_bytes/codec_chain.rs:
// 528-555) runs the array->array codecs forward (transpose: encoded shape = permute(shape, order),
// transpose_codec.rs:243-262), the bytes codec (bytes_codec.rs:180-201: element bytes reversed for
// a non-native endianness), then the bytes->bytes codecs in order. Here the transposes, the byte
// order and an innermost numcodecs.shuffle (shuffle_codec.rs:86-107: enc[i*count + j] = dec[j*es + i])
// are one gather from the array into each chunk's encoded layout; crc32c codecs follow as
// k_crc32c_encode launches. Chunk regions past the array edge encode the fill value (zarrs encodes
// the whole chunk, filled: array_write_ops / ArrayBytes::new_fill_value).
#include <algorithm>
#include <type_traits>

#include "dev.hpp"
#include "launch.hpp"

namespace zgpu {

template <int ES>
struct Elem {  // byte-aligned element (any destination offset)
  uint8_t b[ES];
};
template <int ES>
struct alignas(ES) ElemA {  // naturally aligned element: one ES-byte access
  uint8_t b[ES];
};

template <int ES>
__global__ __launch_bounds__(256) void k_encode_gather(const uint64_t *dsts, const uint64_t *starts,
                                                       const uint8_t *array, ZgEncode P, uint64_t total) {
  const uint64_t nd = P.nd;
  for (uint64_t g = (uint64_t)blockIdx.x * 256 + threadIdx.x; g < total; g += (uint64_t)gridDim.x * 256) {
    const uint64_t c = g / P.nelem, e = g - c * P.nelem;
    const uint64_t *st = starts + c * nd;
    // encoded C-order index e -> encoded coords (axis a of the encoded shape is decoded axis m[a])
    uint64_t rem = e, off = 0;
    bool inside = true;
    for (int a = (int)nd - 1; a >= 0; a--) {
      const uint64_t ext = P.enc_shape[a];
      const uint64_t q = rem / ext, x = rem - q * ext;
      rem = q;
      const uint32_t d = P.dec_axis[a];
      const uint64_t ac = st[d] + x;
      inside = inside && ac < P.array_shape[d];
      off += ac * P.array_stride[d];
    }
    Elem<ES> v;
    if (inside) {
      const ElemA<ES> a = *(const ElemA<ES> *)(array + off * ES);  // the array is element-aligned
#pragma unroll
      for (int k = 0; k < ES; k++) v.b[k] = a.b[k];
    } else {
#pragma unroll
      for (int k = 0; k < ES; k++) v.b[k] = P.fill[k];
    }
    if (P.swap) {  // reverse each component (bytes codec, non-native endianness)
      Elem<ES> w = v;
      if (P.comp == ES) {
#pragma unroll
        for (int k = 0; k < ES; k++) w.b[k] = v.b[ES - 1 - k];
      } else {  // multi-component types (complex): per component
        for (uint32_t c0 = 0; c0 < ES; c0 += P.comp)
          for (uint32_t k = 0; k < P.comp; k++) w.b[c0 + k] = v.b[c0 + P.comp - 1 - k];
      }
      v = w;
    }
    uint8_t *o = (uint8_t *)dsts[c] + P.data_off;
    if (P.shuffle) {
#pragma unroll
      for (int k = 0; k < ES; k++) o[(uint64_t)k * P.nelem + e] = v.b[k];
    } else if (P.aligned) {
      ElemA<ES> w;
#pragma unroll
      for (int k = 0; k < ES; k++) w.b[k] = v.b[k];
      *(ElemA<ES> *)(o + e * ES) = w;
    } else {
      *(Elem<ES> *)(o + e * ES) = v;
    }
  }
}


// Transposing chains: the encoded innermost axis (decoded axis A = dec_axis[nd-1]) differs from the
// array's innermost axis Lx = nd-1, so a plain gather reads the array with a stride. The decode
// path's k_scatter_tiled run backwards: a block moves TJ slabs of a 64x64 (A x Lx) tile at
// consecutive values of axis B (the other axis with the smallest encoded stride, so the TJ encoded
// rows of one Lx index are adjacent), reading array rows along Lx with 16-B non-temporal loads into
// a padded LDS tile (row pitch 65 words: conflict-free column reads) and writing encoded rows along
// A with 16-B non-temporal stores. Tiles that cross the array edge or unaligned layouts take an
// element path (fill past the edge). Launched in slices of the block range (grid*256 < 2^32).
constexpr int ETILE = 64;
constexpr int ETHREADS = 256;

template <int ES>
__global__ __launch_bounds__(ETHREADS) void k_encode_tiled(const uint64_t *__restrict__ dsts,
                                                           const uint64_t *__restrict__ starts,
                                                           const uint8_t *__restrict__ array, ZgEncode P,
                                                           uint64_t tiles_per_chunk, uint64_t block_base) {
  using T = typename std::conditional<ES == 1, uint8_t, typename std::conditional<ES == 2, uint16_t,
            typename std::conditional<ES == 4, uint32_t, uint2>::type>::type>::type;
  constexpr int TJ = tiled_slabs(ES);
  constexpr int PITCH = ETILE + (ES >= 4 ? 1 : 4 / ES);
  constexpr int SLAB = ETILE * PITCH + (ES >= 4 ? 1 : 4 / ES);
  __shared__ T tile[TJ * SLAB];
  const uint64_t bid = block_base + blockIdx.x;
  const uint64_t c = bid / tiles_per_chunk;
  uint64_t t = bid % tiles_per_chunk;
  const uint32_t nd = P.nd, A = P.dec_axis[nd - 1], Lx = nd - 1, B = P.tile_b;
  const bool hasB = B < nd;
  const uint64_t extA = P.dec_shape[A], extL = P.dec_shape[Lx], extB = hasB ? P.dec_shape[B] : 1;
  const uint64_t nta = (extA + ETILE - 1) / ETILE, ntl = (extL + ETILE - 1) / ETILE, nbg = (extB + TJ - 1) / TJ;
  const uint64_t ta = t % nta; t /= nta;
  const uint64_t tl = t % ntl; t /= ntl;
  const uint64_t tb = t % nbg; t /= nbg;
  const uint64_t *st = starts + c * nd;
  // the other decoded coordinates (C order over the axes other than A, Lx, B)
  uint64_t arr = 0, enc = 0, rem = t;
  bool inside = true;
  for (int d = (int)nd - 1; d >= 0; d--) {
    if ((uint32_t)d == A || (uint32_t)d == Lx || (uint32_t)d == B) continue;
    const uint64_t x = rem % P.dec_shape[d];
    rem /= P.dec_shape[d];
    const uint64_t ac = st[d] + x;
    inside = inside && ac < P.array_shape[d];
    arr += ac * P.array_stride[d];
    enc += x * P.enc_stride_of_dec[d];
  }
  const uint64_t a0 = ta * ETILE, l0 = tl * ETILE, b0 = tb * TJ;
  const uint32_t na = (uint32_t)min<uint64_t>(ETILE, extA - a0), nl = (uint32_t)min<uint64_t>(ETILE, extL - l0);
  const uint32_t nb = (uint32_t)min<uint64_t>(TJ, extB - b0);
  const uint64_t sA = P.array_stride[A], sB = hasB ? P.array_stride[B] : 0;
  const uint64_t eL = P.enc_stride_of_dec[Lx], eB = hasB ? P.enc_stride_of_dec[B] : 0;
  // array-space origin of the tile and how much of it lies inside the array
  const uint64_t oa = st[A] + a0, ol = st[Lx] + l0, ob = hasB ? st[B] + b0 : 0;
  const bool whole = inside && oa + na <= P.array_shape[A] && ol + nl <= P.array_shape[Lx] &&
                     (!hasB || ob + nb <= P.array_shape[B]);
  const T *src = (const T *)array + arr + oa * sA + ol + (hasB ? ob * sB : 0);
  uint8_t *dst8 = (uint8_t *)dsts[c] + P.data_off + (enc + a0 + l0 * eL + b0 * eB) * ES;
  const uint32_t swap = P.swap && P.comp > 1;
  constexpr int VPR = ETILE * ES / 16;  // 16-B vectors per tile row
  constexpr int EPV = 16 / ES;          // elements per vector
  constexpr int NV = TJ * ETILE * VPR;  // vectors per block
  constexpr int PER = NV / ETHREADS;
  const bool vload = whole && nl == ETILE && (((uint64_t)src & 15) == 0) && ((sA * ES) % 16 == 0) &&
                     ((sB * ES) % 16 == 0);
  if (vload) {
    // e -> (row a, slab jj, vector v along Lx)
    uint4 x[PER];
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const uint32_t e = p * ETHREADS + threadIdx.x;
      const uint32_t a = e / (TJ * VPR), jj = (e / VPR) % TJ, v = e % VPR;
      if (a < na && jj < nb) x[p] = nt_load16(src + jj * sB + (uint64_t)a * sA + v * EPV);
    }
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const uint32_t e = p * ETHREADS + threadIdx.x;
      const uint32_t a = e / (TJ * VPR), jj = (e / VPR) % TJ, v = e % VPR;
      if (a < na && jj < nb) {
        uint4 y = swap ? swap_vec(x[p], P.comp) : x[p];
        const T *ye = (const T *)&y;
#pragma unroll
        for (int k = 0; k < EPV; k++) tile[jj * SLAB + a * PITCH + v * EPV + k] = ye[k];
      }
    }
  } else {
    T fv;
    __builtin_memcpy(&fv, P.fill, ES);
    if (swap) {  // the fill value is stored through the same endianness as the data
      uint8_t b[ES], w[ES];
      __builtin_memcpy(b, &fv, ES);
      for (uint32_t c0 = 0; c0 < (uint32_t)ES; c0 += P.comp)
        for (uint32_t k = 0; k < P.comp; k++) w[c0 + k] = b[c0 + P.comp - 1 - k];
      __builtin_memcpy(&fv, w, ES);
    }
    for (uint32_t e = threadIdx.x; e < (uint32_t)(TJ * ETILE * ETILE); e += ETHREADS) {
      const uint32_t a = e / (TJ * ETILE), jj = (e / ETILE) % TJ, l = e % ETILE;
      if (a >= na || jj >= nb || l >= nl) continue;
      T v = fv;
      if (inside && oa + a < P.array_shape[A] && ol + l < P.array_shape[Lx] &&
          (!hasB || ob + jj < P.array_shape[B])) {
        v = src[jj * sB + (uint64_t)a * sA + l];
        if (swap) {
          uint8_t b[ES], w[ES];
          __builtin_memcpy(b, &v, ES);
          for (uint32_t c0 = 0; c0 < (uint32_t)ES; c0 += P.comp)
            for (uint32_t k = 0; k < P.comp; k++) w[c0 + k] = b[c0 + P.comp - 1 - k];
          __builtin_memcpy(&v, w, ES);
        }
      }
      tile[jj * SLAB + a * PITCH + l] = v;
    }
  }
  __syncthreads();
  const bool vstore = na == ETILE && (((uint64_t)dst8 & 15) == 0) && ((eL * ES) % 16 == 0) && ((eB * ES) % 16 == 0);
  if (vstore) {
    // e -> (row l, slab jj, vector v along A): TJ adjacent encoded rows per Lx index
#pragma unroll
    for (int p = 0; p < PER; p++) {
      const uint32_t e = p * ETHREADS + threadIdx.x;
      const uint32_t l = e / (TJ * VPR), jj = (e / VPR) % TJ, v = e % VPR;
      if (l < nl && jj < nb) {
        uint4 y;
        T *ye = (T *)&y;
#pragma unroll
        for (int k = 0; k < EPV; k++) ye[k] = tile[jj * SLAB + (v * EPV + k) * PITCH + l];
        nt_store16(dst8 + (jj * eB + (uint64_t)l * eL + v * EPV) * ES, y);
      }
    }
  } else {
    for (uint32_t e = threadIdx.x; e < (uint32_t)(TJ * ETILE * ETILE); e += ETHREADS) {
      const uint32_t l = e / (TJ * ETILE), jj = (e / ETILE) % TJ, a = e % ETILE;
      if (l < nl && jj < nb && a < na) {
        const T v = tile[jj * SLAB + a * PITCH + l];
        uint8_t *o = dst8 + (jj * eB + (uint64_t)l * eL + a) * ES;
        if (P.aligned) *(T *)o = v;
        else __builtin_memcpy(o, &v, ES);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// sharding_indexed encode for fixed-size inner chains (ShardingCodecBound::encode_bounded,
// zarrs/src/array/codec/array_to_bytes/sharding/sharding_codec.rs:924-1085 with
// SubchunkWriteOrder::C): every inner chunk is encoded by the inner chain (launch_encode_gather +
// crc32c above) into a temporary slot of E bytes; an inner chunk whose decoded values all equal the
// fill value is omitted (index entry (u64::MAX, u64::MAX), encode_inner_by_chunk_index :883-920);
// the present ones are laid out back to back in C order of the inner grid after (index at start) or
// before (index at end) the encoded index (bytes{endian} + crc32c codecs, compute_index_encoded_size).
// ---------------------------------------------------------------------------------------------
template <int ES>
__global__ __launch_bounds__(256) void k_fill_check(const uint64_t *__restrict__ starts,
                                                    const uint8_t *__restrict__ array, ZgEncode P,
                                                    uint32_t *__restrict__ nonfill) {
  using T = typename std::conditional<ES == 1, uint8_t, typename std::conditional<ES == 2, uint16_t,
            typename std::conditional<ES == 4, uint32_t, typename std::conditional<ES == 8, uint2,
            uint4>::type>::type>::type>::type;
  const uint64_t c = blockIdx.x;
  const uint64_t *st = starts + c * P.nd;
  T fv;
  __builtin_memcpy(&fv, P.fill, ES);
  const uint32_t nd = P.nd, L = nd - 1;
  const uint64_t ext = P.dec_shape[L], rows = P.nelem / ext;
  bool differs = false;
  for (uint64_t r0 = 0; r0 < rows && !differs; r0 += 256 / 64) {
    // a wave per row (64 lanes along the innermost axis), 4 rows per pass
    const uint64_t r = r0 + threadIdx.x / 64;
    if (r < rows) {
      uint64_t rem = r, off = 0;
      bool inside = true;
      for (int d = (int)nd - 2; d >= 0; d--) {
        const uint64_t x = rem % P.dec_shape[d];
        rem /= P.dec_shape[d];
        const uint64_t ac = st[d] + x;
        inside = inside && ac < P.array_shape[d];
        off += ac * P.array_stride[d];
      }
      if (inside)
        for (uint64_t x = threadIdx.x & 63; x < ext; x += 64) {
          if (st[L] + x >= P.array_shape[L]) break;  // past the array edge: fill
          const T v = *(const T *)(array + (off + st[L] + x) * ES);
          uint32_t a[(ES + 3) / 4] = {}, b[(ES + 3) / 4] = {};
          __builtin_memcpy(a, &v, ES);
          __builtin_memcpy(b, &fv, ES);
          bool ne = false;
#pragma unroll
          for (int w = 0; w < (ES + 3) / 4; w++) ne = ne || a[w] != b[w];
          if (ne) {
            differs = true;
            break;
          }
        }
    }
    if (__syncthreads_or(differs)) differs = true;
  }
  if (threadIdx.x == 0) nonfill[c] = differs ? 1u : 0u;
}

struct ZgShardLayout {
  uint64_t n_inner, E, E_pitch;  // inner chunks per shard, encoded inner size, temp slot pitch
  uint64_t index_bytes, pre;     // encoded index size; crc32c bytes before the raw index (start crcs)
  uint32_t at_start, big_endian;
};

// One workgroup per shard: C-order prefix sum of the present inner chunks, index entries written
// (raw u64 pairs, endianness of the index bytes codec) into the shard at the index position; the
// shard's length and the position of its encoded index (for the index crc32c launches) returned.
__global__ __launch_bounds__(256) void k_shard_layout(const uint32_t *__restrict__ nonfill, ZgShardLayout Lo,
                                                      const uint64_t *__restrict__ shard_dst,
                                                      uint64_t *__restrict__ inner_off,
                                                      uint64_t *__restrict__ index_ptr, uint64_t *__restrict__ shard_len) {
  __shared__ uint64_t s_base, s_wsum[4];
  const uint64_t sh = blockIdx.x, n = Lo.n_inner;
  const uint32_t *nf = nonfill + sh * n;
  uint64_t *off = inner_off + sh * n;
  const uint64_t body0 = Lo.at_start ? Lo.index_bytes : 0;
  if (threadIdx.x == 0) s_base = 0;
  __syncthreads();
  for (uint64_t k0 = 0; k0 < n; k0 += 256) {
    const uint64_t k = k0 + threadIdx.x;
    const uint32_t f = k < n ? nf[k] : 0u;
    // block exclusive scan of f
    uint32_t incl = f;
    const uint32_t lane = threadIdx.x & 63;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t u = __shfl_up(incl, o, 64);
      if ((int)lane >= o) incl += u;
    }
    if (lane == 63) s_wsum[threadIdx.x / 64] = incl;
    __syncthreads();
    uint64_t before = s_base;
    for (uint32_t w = 0; w < threadIdx.x / 64; w++) before += s_wsum[w];
    before += incl - f;
    if (k < n) off[k] = f ? body0 + before * Lo.E : ~0ull;
    __syncthreads();
    if (threadIdx.x == 0) s_base += s_wsum[0] + s_wsum[1] + s_wsum[2] + s_wsum[3];
    __syncthreads();
  }
  const uint64_t body = s_base * Lo.E;
  const uint64_t idx0 = Lo.at_start ? 0 : body0 + body;  // encoded index position in the shard
  uint8_t *raw = (uint8_t *)shard_dst[sh] + idx0 + Lo.pre;
  for (uint64_t q = threadIdx.x; q < 2 * n; q += 256) {
    const uint64_t o = off[q / 2];
    const uint64_t v = o == ~0ull ? ~0ull : (q & 1 ? Lo.E : o);
#pragma unroll
    for (int b = 0; b < 8; b++) raw[q * 8 + b] = (uint8_t)(v >> (8 * (Lo.big_endian ? 7 - b : b)));
  }
  if (threadIdx.x == 0) {
    index_ptr[sh] = shard_dst[sh] + idx0;
    shard_len[sh] = body0 + body + (Lo.at_start ? 0 : Lo.index_bytes);
  }
}

// The present inner chunks from their temporary slots to their shard offsets: a workgroup per
// (shard, inner chunk); dword moves when both sides allow, bytes otherwise.
__global__ __launch_bounds__(256) void k_shard_copy(const uint8_t *__restrict__ tmp, ZgShardLayout Lo,
                                                    const uint64_t *__restrict__ shard_dst,
                                                    const uint64_t *__restrict__ inner_off) {
  const uint64_t g = blockIdx.x, sh = g / Lo.n_inner;
  const uint64_t o = inner_off[g];
  if (o == ~0ull) return;
  const uint8_t *src = tmp + g * Lo.E_pitch;
  uint8_t *dst = (uint8_t *)shard_dst[sh] + o;
  if ((((uintptr_t)dst | Lo.E) & 3) == 0) {
    const uint32_t *s4 = (const uint32_t *)src;
    uint32_t *d4 = (uint32_t *)dst;
    for (uint64_t k = threadIdx.x; k < Lo.E / 4; k += 256) d4[k] = s4[k];
  } else {
    for (uint64_t k = threadIdx.x; k < Lo.E; k += 256) dst[k] = src[k];
  }
}

hipError_t launch_fill_check(const uint64_t *starts, const uint8_t *array, const ZgEncode &inner, uint32_t n_chunks,
                             uint32_t *nonfill, hipStream_t s) {
  if (!n_chunks) return hipSuccess;
  switch (inner.es) {
    case 1: hipLaunchKernelGGL(k_fill_check<1>, dim3(n_chunks), dim3(256), 0, s, starts, array, inner, nonfill); break;
    case 2: hipLaunchKernelGGL(k_fill_check<2>, dim3(n_chunks), dim3(256), 0, s, starts, array, inner, nonfill); break;
    case 4: hipLaunchKernelGGL(k_fill_check<4>, dim3(n_chunks), dim3(256), 0, s, starts, array, inner, nonfill); break;
    case 8: hipLaunchKernelGGL(k_fill_check<8>, dim3(n_chunks), dim3(256), 0, s, starts, array, inner, nonfill); break;
    case 16: hipLaunchKernelGGL(k_fill_check<16>, dim3(n_chunks), dim3(256), 0, s, starts, array, inner, nonfill); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

hipError_t launch_shard_encode(const uint64_t *starts, const uint8_t *array, const ZgEncode &inner, uint32_t n_chunks,
                               uint32_t *nonfill, const uint8_t *tmp, const ZgShardLayoutArgs &A,
                               const uint64_t *shard_dst, uint64_t *inner_off, uint64_t *index_ptr,
                               uint64_t *shard_len, uint32_t n_shards, hipStream_t s) {
  if (!n_chunks) return hipSuccess;
  hipError_t e = launch_fill_check(starts, array, inner, n_chunks, nonfill, s);
  if (e != hipSuccess) return e;
  const ZgShardLayout Lo{A.n_inner, A.E, A.E_pitch, A.index_bytes, A.pre, A.at_start, A.big_endian};
  hipLaunchKernelGGL(k_shard_layout, dim3(n_shards), dim3(256), 0, s, nonfill, Lo, shard_dst, inner_off, index_ptr,
                     shard_len);
  hipLaunchKernelGGL(k_shard_copy, dim3(n_chunks), dim3(256), 0, s, tmp, Lo, shard_dst, inner_off);
  return hipGetLastError();
}

hipError_t launch_encode_gather(const uint64_t *dsts, const uint64_t *starts, const uint8_t *array,
                                const ZgEncode &P, uint32_t n_chunks, hipStream_t s) {
  const uint64_t total = (uint64_t)n_chunks * P.nelem;
  if (!total) return hipSuccess;
  const uint32_t A = P.dec_axis[P.nd - 1], Lx = P.nd - 1;
  if (A != Lx && !P.shuffle && (P.es == 1 || P.es == 2 || P.es == 4 || P.es == 8)) {  // transposing: LDS-tiled
    const uint64_t tj = tiled_slabs(P.es);
    uint64_t tpc = 1;
    for (uint32_t d = 0; d < P.nd; d++) {
      if (d == A || d == Lx) tpc *= (P.dec_shape[d] + ETILE - 1) / ETILE;
      else if (d == P.tile_b) tpc *= (P.dec_shape[d] + tj - 1) / tj;
      else tpc *= P.dec_shape[d];
    }
    const uint64_t blocks = (uint64_t)n_chunks * tpc;
    const uint64_t MAXG = max_grid_blocks(ETHREADS);
    for (uint64_t base = 0; base < blocks; base += MAXG) {
      const dim3 g((uint32_t)std::min<uint64_t>(MAXG, blocks - base));
      switch (P.es) {
        case 1: hipLaunchKernelGGL(k_encode_tiled<1>, g, dim3(ETHREADS), 0, s, dsts, starts, array, P, tpc, base); break;
        case 2: hipLaunchKernelGGL(k_encode_tiled<2>, g, dim3(ETHREADS), 0, s, dsts, starts, array, P, tpc, base); break;
        case 4: hipLaunchKernelGGL(k_encode_tiled<4>, g, dim3(ETHREADS), 0, s, dsts, starts, array, P, tpc, base); break;
        default: hipLaunchKernelGGL(k_encode_tiled<8>, g, dim3(ETHREADS), 0, s, dsts, starts, array, P, tpc, base); break;
      }
      const hipError_t e = hipGetLastError();
      if (e != hipSuccess) return e;
    }
    return hipSuccess;
  }
  const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, (uint64_t)device_cu_count() * 64);
  switch (P.es) {
    case 1: hipLaunchKernelGGL(k_encode_gather<1>, dim3(grid), dim3(256), 0, s, dsts, starts, array, P, total); break;
    case 2: hipLaunchKernelGGL(k_encode_gather<2>, dim3(grid), dim3(256), 0, s, dsts, starts, array, P, total); break;
    case 4: hipLaunchKernelGGL(k_encode_gather<4>, dim3(grid), dim3(256), 0, s, dsts, starts, array, P, total); break;
    case 8: hipLaunchKernelGGL(k_encode_gather<8>, dim3(grid), dim3(256), 0, s, dsts, starts, array, P, total); break;
    case 16: hipLaunchKernelGGL(k_encode_gather<16>, dim3(grid), dim3(256), 0, s, dsts, starts, array, P, total); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace zgpu
