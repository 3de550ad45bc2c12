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

hipError_t launch_encode_gather(const uint64_t *dsts, const uint64_t *starts, const uint8_t *array,
                                const ZgEncode &P, uint32_t n_chunks, hipStream_t s) {
  const uint64_t total = (uint64_t)n_chunks * P.nelem;
  if (!total) return hipSuccess;
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
