// Chunk encode (the write side of the same chain): array -> encoded chunks
// for fixed-size chains. CodecChain::encode (zarrs/src/array/codec/array_to_bytes/codec_chain.rs:
// 528-555) runs the array->array codecs forward (transpose: encoded shape = permute(shape, order),
// transpose_codec.rs:243-262), the bytes codec (bytes_codec.rs:180-201: element bytes reversed for
// a non-native endianness), then the bytes->bytes codecs in order. Here the transposes, the byte
// order and an innermost numcodecs.shuffle (shuffle_codec.rs:86-107: enc[i*count + j] = dec[j*es + i])
// are one gather from the array into each chunk's encoded layout; crc32c codecs follow as
// k_crc32c_encode launches. Chunk regions past the array edge encode the fill value (zarrs encodes
// the whole chunk, filled: array_write_ops / ArrayBytes::new_fill_value).
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
// array's innermost axis B = nd-1, so a plain gather reads the array with a stride. One workgroup
// per (chunk, other coords, 64x64 tile of A x B): coalesced reads along B into a padded LDS tile,
// coalesced writes along A out of it (the decode path's k_scatter_tiled, run backwards).
template <int ES>
__global__ __launch_bounds__(256) void k_encode_tiled(const uint64_t *dsts, const uint64_t *starts,
                                                      const uint8_t *array, ZgEncode P, uint64_t n_other,
                                                      uint32_t tiles_a, uint32_t tiles_b) {
  __shared__ ElemA<ES> tile[64][65];
  const uint32_t nd = P.nd, A = P.dec_axis[nd - 1], Bx = nd - 1;
  uint64_t id = blockIdx.x;
  const uint32_t tb = (uint32_t)(id % tiles_b);
  id /= tiles_b;
  const uint32_t ta = (uint32_t)(id % tiles_a);
  id /= tiles_a;
  const uint64_t o = id % n_other, c = id / n_other;
  const uint64_t *st = starts + c * nd;
  // the other decoded coordinates (C order over the axes other than A and B)
  uint64_t base_arr = 0, base_enc = 0, rem = o;
  bool inside = true;
  for (int d = (int)nd - 1; d >= 0; d--) {
    if ((uint32_t)d == A || (uint32_t)d == Bx) continue;
    const uint64_t ext = P.dec_shape[d], x = rem % ext;
    rem /= ext;
    const uint64_t ac = st[d] + x;
    inside = inside && ac < P.array_shape[d];
    base_arr += ac * P.array_stride[d];
    base_enc += x * P.enc_stride_of_dec[d];
  }
  const uint32_t t = threadIdx.x, lx = t & 63, ly = t >> 6;
  const uint64_t extA = P.dec_shape[A], extB = P.dec_shape[Bx];
  // read: rows along A, columns along B (array-contiguous)
  for (uint32_t r = ly; r < 64; r += 4) {
    const uint64_t a = (uint64_t)ta * 64 + r, b = (uint64_t)tb * 64 + lx;
    if (a >= extA || b >= extB) continue;
    const uint64_t aa = st[A] + a, ab = st[Bx] + b;
    ElemA<ES> v;
    if (inside && aa < P.array_shape[A] && ab < P.array_shape[Bx]) {
      v = *(const ElemA<ES> *)(array + (base_arr + aa * P.array_stride[A] + ab * P.array_stride[Bx]) * ES);
    } else {
#pragma unroll
      for (int k = 0; k < ES; k++) v.b[k] = P.fill[k];
    }
    tile[r][lx] = v;
  }
  __syncthreads();
  uint8_t *out = (uint8_t *)dsts[c] + P.data_off;
  // write: for a fixed b, consecutive a are consecutive encoded elements
  for (uint32_t r = ly; r < 64; r += 4) {
    const uint64_t a = (uint64_t)ta * 64 + lx, b = (uint64_t)tb * 64 + r;
    if (a >= extA || b >= extB) continue;
    ElemA<ES> v = tile[lx][r];
    if (P.swap) {
      ElemA<ES> w = v;
      if (P.comp == ES) {
#pragma unroll
        for (int k = 0; k < ES; k++) w.b[k] = v.b[ES - 1 - k];
      } else {
        for (uint32_t c0 = 0; c0 < ES; c0 += P.comp)
          for (uint32_t k = 0; k < P.comp; k++) w.b[c0 + k] = v.b[c0 + P.comp - 1 - k];
      }
      v = w;
    }
    const uint64_t e = base_enc + a * P.enc_stride_of_dec[A] + b * P.enc_stride_of_dec[Bx];
    if (P.shuffle) {
#pragma unroll
      for (int k = 0; k < ES; k++) out[(uint64_t)k * P.nelem + e] = v.b[k];
    } else if (P.aligned) {
      *(ElemA<ES> *)(out + e * ES) = v;
    } else {
      Elem<ES> w;
#pragma unroll
      for (int k = 0; k < ES; k++) w.b[k] = v.b[k];
      *(Elem<ES> *)(out + e * ES) = w;
    }
  }
}

hipError_t launch_encode_gather(const uint64_t *dsts, const uint64_t *starts, const uint8_t *array,
                                const ZgEncode &P, uint32_t n_chunks, hipStream_t s) {
  const uint64_t total = (uint64_t)n_chunks * P.nelem;
  if (!total) return hipSuccess;
  const uint32_t A = P.dec_axis[P.nd - 1], Bx = P.nd - 1;
  if (A != Bx && P.es <= 8) {  // transposing chain: LDS-tiled
    const uint64_t extA = P.dec_shape[A], extB = P.dec_shape[Bx];
    const uint32_t tiles_a = (uint32_t)((extA + 63) / 64), tiles_b = (uint32_t)((extB + 63) / 64);
    const uint64_t n_other = P.nelem / (extA * extB);
    const uint64_t blocks = (uint64_t)n_chunks * n_other * tiles_a * tiles_b;
    if (blocks < (1ull << 31)) {
      const dim3 g((uint32_t)blocks);
      switch (P.es) {
        case 1: hipLaunchKernelGGL(k_encode_tiled<1>, g, dim3(256), 0, s, dsts, starts, array, P, n_other, tiles_a, tiles_b); break;
        case 2: hipLaunchKernelGGL(k_encode_tiled<2>, g, dim3(256), 0, s, dsts, starts, array, P, n_other, tiles_a, tiles_b); break;
        case 4: hipLaunchKernelGGL(k_encode_tiled<4>, g, dim3(256), 0, s, dsts, starts, array, P, n_other, tiles_a, tiles_b); break;
        case 8: hipLaunchKernelGGL(k_encode_tiled<8>, g, dim3(256), 0, s, dsts, starts, array, P, n_other, tiles_a, tiles_b); break;
        default: return hipErrorInvalidValue;
      }
      return hipGetLastError();
    }
  }
  const uint32_t grid = (uint32_t)std::min<uint64_t>((total + 255) / 256, 256 * 64);
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
