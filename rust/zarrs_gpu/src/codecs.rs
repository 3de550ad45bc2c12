//! Per-codec GPU runtime plugins: `bytes` (array->bytes), `transpose` (array->array) and the
//! bytes->bytes codecs `crc32c`, `gzip`, `zstd` and `numcodecs.shuffle`, each registered with
//! `zarrs_codec::register_codec_v3` so that zarrs' unchanged CodecChain (codec_chain.rs:557-646) decodes
//! every stage of an unsharded chunk on the MI355X. The pattern is
//! zarrs/tests/codec_runtime_registration.rs:92-183: a runtime plugin matched by name, creating a codec
//! whose `decode` is the GPU's and whose metadata, representation, encode and partial-encode behaviour
//! is zarrs' own codec, which the plugin wraps.
//!
//! Each decode is one synchronous `zgpu_decode_pinned` of a one-codec chain (n = 1, host bytes in,
//! the decoded bytes copied once out of pinned memory), coalesced with the calls other rayon workers
//! make at the same time (ZGPU_COALESCE: one H2D, one launch sequence, one D2H per batch). A
//! per-codec plugin cannot fuse a chain's stages: every GPU stage is a PCIe round trip, so by default
//! only the entropy stages gzip and blosc (GPU_ENTROPY_CODEC_NAMES) are registered and zarrs' own
//! bytes / transpose / crc32c / shuffle run on the host around them; per-chunk zstd is opt-in
//! (GPU_ZSTD_CODEC_NAMES: bench.py's `secondary.c5.dropin_emulation` measures that split on C5 and
//! finds the host side alone as slow as zarrs' CPU zstd). The batched paths (the `sharding_indexed`
//! plugin, ArrayGpuExt) remain the fast ones.

use std::borrow::Cow;
use std::num::NonZeroU64;
use std::sync::{Arc, OnceLock};

use zarrs::array::codec::{BloscCodec, BytesCodec, Crc32cCodec, GzipCodec, ShuffleCodec, TransposeCodec, ZstdCodec};
use zarrs_chunk_grid::ChunkGridCreateError;
use zarrs_codec::{
    ArrayBytes, ArrayBytesRaw, ArrayCodecTraits, ArrayPartialDecoderTraits, ArrayPartialEncoderTraits,
    ArrayToArrayCodecSubchunkingTraits, ArrayToArrayCodecTraits, ArrayToBytesCodecSubchunkingTraits,
    ArrayToBytesCodecTraits, BytesPartialDecoderTraits, BytesPartialEncoderTraits, BytesRepresentation,
    BytesToBytesCodecTraits, ChunkGridDecoded, ChunkGridDecodedRef, ChunkGridEncoded, ChunkGridEncodedRef, ChunkShape,
    Codec, CodecCreateError, CodecError, CodecMetadataOptions, CodecOptions, CodecSpecificOptions, CodecTraits,
    CodecTraitsV3, PartialDecoderCapability, PartialEncoderCapability, RecommendedConcurrency,
    UnboundArrayToArrayCodecTraits, UnboundArrayToBytesCodecTraits,
};
use zarrs_data_type::{DataType, FillValue};
use zarrs_metadata::Configuration;
use zarrs_metadata::v3::MetadataV3;
use zarrs_plugin::ZarrVersion;

use crate::Chain;

/// Names every per-codec plugin answers to (the v3 names zarrs registers for these codecs).
pub const GPU_CODEC_NAMES: [&str; 8] =
    ["bytes", "transpose", "crc32c", "gzip", "zstd", "blosc", "numcodecs.shuffle", "shuffle"];

/// The codecs [`crate::register_codecs`] sends to the GPU by default: the entropy stages whose
/// per-chunk decode is worth a PCIe round trip (an inflate runs ~0.3 GB/s per host core; the GPU's
/// coalesced call moves only the compressed bytes in and the decoded bytes out). `bytes`,
/// `transpose`, `crc32c` and `numcodecs.shuffle` run near memory speed on the host, where a hop to
/// the GPU and back costs more than the stage: they stay zarrs' own unless
/// [`crate::register_codecs_all`] asks for them.
///
/// `zstd` is not among them: a lone 16 MiB C5 frame decodes in 3.3 ms through the plugin's call
/// (the window executor's latency mode), but zarrs' per-codec chain then copies the result out of
/// pinned memory, unshuffles and places it on the host, and that host work alone is about the CPU
/// codec's whole per-chunk cost (libzstd ~1.5 GB/s per core): C5 read per chunk through the plugin
/// runs at 10.1 GiB/s against 28.7 on 16 host threads (bench.py `secondary.c5.dropin_emulation`,
/// profiles/r06/). Opt in with [`GPU_ZSTD_CODEC_NAMES`] and [`crate::register_codecs_named`]; the
/// batched paths (ArrayGpuExt: 216 GiB/s from HBM on C5) are the ones for zstd arrays.
pub const GPU_ENTROPY_CODEC_NAMES: [&str; 2] = ["gzip", "blosc"];

/// The per-chunk zstd plugin (opt-in, see [`GPU_ENTROPY_CODEC_NAMES`]).
pub const GPU_ZSTD_CODEC_NAMES: [&str; 1] = ["zstd"];

/// The runtime-plugin create function of the per-codec plugins: zarrs' own codec is created from the
/// metadata (never through the registry, which would find this plugin again) and wrapped.
///
/// # Errors
/// Returns [`CodecCreateError`] as zarrs' codec creation does.
pub fn create(metadata: &MetadataV3) -> Result<Codec, CodecCreateError> {
    let cpu = match metadata.name() {
        "bytes" => <BytesCodec as CodecTraitsV3>::create(metadata)?,
        "transpose" => <TransposeCodec as CodecTraitsV3>::create(metadata)?,
        "crc32c" => <Crc32cCodec as CodecTraitsV3>::create(metadata)?,
        "gzip" => <GzipCodec as CodecTraitsV3>::create(metadata)?,
        "zstd" => <ZstdCodec as CodecTraitsV3>::create(metadata)?,
        "blosc" => <BloscCodec as CodecTraitsV3>::create(metadata)?,
        "numcodecs.shuffle" | "shuffle" => <ShuffleCodec as CodecTraitsV3>::create(metadata)?,
        other => return Err(CodecCreateError::Other(format!("zarrs_gpu: no GPU plugin for codec {other}"))),
    };
    let meta_json = serde_json::to_string(metadata).map_err(CodecCreateError::other)?;
    Ok(match cpu {
        Codec::BytesToBytes(cpu) => Codec::BytesToBytes(Arc::new(GpuBytesToBytes {
            cpu,
            name: metadata.name().to_string(),
            meta_json,
            chain: OnceLock::new(),
        })),
        Codec::ArrayToBytes(cpu) => Codec::ArrayToBytes(Arc::new(GpuBytes { cpu, meta_json })),
        Codec::ArrayToArray(cpu) => Codec::ArrayToArray(Arc::new(GpuTranspose { cpu, meta_json })),
        other => other,
    })
}

const BYTES_LE: &str = r#"{"name":"bytes","configuration":{"endian":"little"}}"#;

// ---------------------------------------------------------------------------------------------------
// bytes -> bytes: crc32c, gzip, zstd, numcodecs.shuffle
// ---------------------------------------------------------------------------------------------------

/// A bytes->bytes codec decoded on the GPU: the chain `[bytes, <codec>]` over uint8 elements, one
/// chunk of the decoded representation's size.
#[derive(Debug)]
pub struct GpuBytesToBytes {
    cpu: Arc<dyn BytesToBytesCodecTraits>,
    name: String,
    meta_json: String,
    chain: OnceLock<Result<Chain, String>>,
}

/// The decoded length of a bytes->bytes codec's output when the chain only bounds it
/// (BytesRepresentation::BoundedSize / UnboundedSize, e.g. crc32c after gzip in C3's inner chain):
/// crc32c strips 4 bytes (crc32c_codec.rs:108-141; a shorter input decodes to the GPU's
/// CRC_INPUT_TOO_SHORT), shuffle keeps the length (shuffle_codec.rs:109-129), gzip's trailer ISIZE
/// (RFC 1952, modulo 2^32) and a zstd frame's content size (RFC 8878 frame header) are hints the GPU
/// decode checks (DECODED_SIZE_MISMATCH when a stream lies: the caller then takes zarrs' codec).
fn decoded_len_hint(name: &str, enc: &[u8]) -> Option<u64> {
    match name {
        "crc32c" => Some(enc.len().saturating_sub(4) as u64),
        "numcodecs.shuffle" | "shuffle" => Some(enc.len() as u64),
        "gzip" if enc.len() >= 18 => {
            let t = &enc[enc.len() - 4..];
            Some(u64::from(u32::from_le_bytes([t[0], t[1], t[2], t[3]])))
        }
        "zstd" if enc.len() >= 6 && enc[..4] == [0x28, 0xB5, 0x2F, 0xFD] => {
            let fhd = enc[4];
            let (fcs_flag, single, dict_flag) = (fhd >> 6, (fhd >> 5) & 1, fhd & 3);
            let fcs_len = match fcs_flag {
                0 => usize::from(single),
                1 => 2,
                2 => 4,
                _ => 8,
            };
            if fcs_len == 0 {
                return None;
            }
            let at = 5 + usize::from(single == 0) + [0usize, 1, 2, 4][usize::from(dict_flag)];
            let f = enc.get(at..at + fcs_len)?;
            let mut v = 0u64;
            for (i, b) in f.iter().enumerate() {
                v |= u64::from(*b) << (8 * i);
            }
            Some(if fcs_len == 2 { v + 256 } else { v })
        }
        _ => None,
    }
}

impl GpuBytesToBytes {
    fn chain(&self) -> Result<&Chain, CodecError> {
        self.chain
            .get_or_init(|| {
                let json = format!("[{BYTES_LE},{}]", self.meta_json);
                Chain::new(&json, &zarrs::array::data_type::uint8(), &FillValue::from(0u8)).map_err(|e| e.to_string())
            })
            .as_ref()
            .map_err(|e| CodecError::Other(e.clone()))
    }
}

impl CodecTraits for GpuBytesToBytes {
    fn configuration(&self, version: ZarrVersion, options: &CodecMetadataOptions) -> Option<Configuration> {
        self.cpu.configuration(version, options)
    }
    fn partial_decoder_capability(&self) -> PartialDecoderCapability {
        self.cpu.partial_decoder_capability()
    }
    fn partial_encoder_capability(&self) -> PartialEncoderCapability {
        self.cpu.partial_encoder_capability()
    }
}

impl BytesToBytesCodecTraits for GpuBytesToBytes {
    fn into_dyn(self: Arc<Self>) -> Arc<dyn BytesToBytesCodecTraits> {
        self
    }

    fn with_codec_specific_options(
        self: Arc<Self>,
        opts: &CodecSpecificOptions,
    ) -> Result<Arc<dyn BytesToBytesCodecTraits>, CodecCreateError> {
        let cpu = self.cpu.clone().with_codec_specific_options(opts)?;
        Ok(Arc::new(Self { cpu, name: self.name.clone(), meta_json: self.meta_json.clone(), chain: OnceLock::new() }))
    }

    fn recommended_concurrency(&self, decoded: &BytesRepresentation) -> Result<RecommendedConcurrency, CodecError> {
        self.cpu.recommended_concurrency(decoded)
    }

    fn encoded_representation(&self, decoded: &BytesRepresentation) -> BytesRepresentation {
        self.cpu.encoded_representation(decoded)
    }

    fn encode<'a>(&self, decoded: ArrayBytesRaw<'a>, options: &CodecOptions) -> Result<ArrayBytesRaw<'a>, CodecError> {
        self.cpu.encode(decoded, options)
    }

    /// The GPU decode (crc32c verified per `options.validate_checksums()`, gzip trailer / zstd frame
    /// checks always). A fixed-size decoded representation gives the length; otherwise (crc32c after a
    /// compressor, as in C3's inner chain `[bytes, gzip, crc32c]`) it comes from the stream
    /// (`decoded_len_hint`). zarrs' own codec only when no length is known (a zstd frame without a
    /// content size) or a compressor's hint proves wrong.
    fn decode<'a>(
        &self,
        encoded: ArrayBytesRaw<'a>,
        decoded: &BytesRepresentation,
        options: &CodecOptions,
    ) -> Result<ArrayBytesRaw<'a>, CodecError> {
        let (n, hinted) = match *decoded {
            BytesRepresentation::FixedSize(n) => (n, false),
            _ => match decoded_len_hint(&self.name, &encoded) {
                Some(n) => (n, true),
                None => return self.cpu.decode(encoded, decoded, options),
            },
        };
        let chain = self.chain()?;
        match chain.decode_region(&encoded, &[n], &[0], &[n], options.validate_checksums()) {
            Ok(out) => Ok(Cow::Owned(out)),
            Err(CodecError::UnexpectedChunkDecodedSize(_)) if hinted && !matches!(self.name.as_str(), "crc32c") => {
                self.cpu.decode(encoded, decoded, options)
            }
            Err(e) => Err(e),
        }
    }

    fn partial_decoder(
        self: Arc<Self>,
        input_handle: Arc<dyn BytesPartialDecoderTraits>,
        decoded: &BytesRepresentation,
        options: &CodecOptions,
    ) -> Result<Arc<dyn BytesPartialDecoderTraits>, CodecError> {
        // crc32c's partial decoder strips without verifying (crc32c_codec.rs:143-158) and shuffle's
        // reads byte ranges: zarrs' own partial decoders; gzip / zstd decode the whole chunk through
        // the default partial decoder, which calls the GPU `decode` above
        match self.cpu.partial_decoder_capability().partial_decode {
            true => self.cpu.clone().partial_decoder(input_handle, decoded, options),
            false => Ok(Arc::new(zarrs_codec::BytesToBytesCodecPartialDefault::new_bytes(
                input_handle,
                *decoded,
                self.into_dyn(),
            ))),
        }
    }

    fn partial_encoder(
        self: Arc<Self>,
        input_output_handle: Arc<dyn BytesPartialEncoderTraits>,
        decoded: &BytesRepresentation,
        options: &CodecOptions,
    ) -> Result<Arc<dyn BytesPartialEncoderTraits>, CodecError> {
        self.cpu.clone().partial_encoder(input_output_handle, decoded, options)
    }
}

// ---------------------------------------------------------------------------------------------------
// array -> bytes: bytes (endianness)
// ---------------------------------------------------------------------------------------------------

/// The unbound GPU `bytes` codec.
#[derive(Debug)]
pub struct GpuBytes {
    cpu: Arc<dyn UnboundArrayToBytesCodecTraits>,
    meta_json: String,
}

impl CodecTraits for GpuBytes {
    fn configuration(&self, version: ZarrVersion, options: &CodecMetadataOptions) -> Option<Configuration> {
        self.cpu.configuration(version, options)
    }
    fn partial_decoder_capability(&self) -> PartialDecoderCapability {
        self.cpu.partial_decoder_capability()
    }
    fn partial_encoder_capability(&self) -> PartialEncoderCapability {
        self.cpu.partial_encoder_capability()
    }
}

impl UnboundArrayToBytesCodecTraits for GpuBytes {
    fn into_dyn(self: Arc<Self>) -> Arc<dyn UnboundArrayToBytesCodecTraits> {
        self
    }

    fn with_context(
        &self,
        data_type: DataType,
        fill_value: FillValue,
    ) -> Result<Arc<dyn ArrayToBytesCodecTraits>, CodecCreateError> {
        let cpu = self.cpu.with_context(data_type.clone(), fill_value.clone())?;
        // the GPU chain for fixed-size data types whose stored endianness is not the host's (the only
        // case where the bytes codec does work, zarrs_data_type/src/codec_traits/bytes.rs:111-118)
        let json = format!("[{}]", self.meta_json);
        let native = serde_json::from_str::<serde_json::Value>(&self.meta_json)
            .ok()
            .and_then(|m| m.pointer("/configuration/endian").and_then(|e| e.as_str()).map(str::to_owned))
            .is_none_or(|e| (e == "little") == cfg!(target_endian = "little"));
        let chain = if native || data_type.fixed_size().is_none() {
            None
        } else {
            Some(Arc::new(Chain::new(&json, &data_type, &fill_value)?))
        };
        Ok(Arc::new(GpuBytesBound { cpu, chain, data_type, fill_value }))
    }
}

/// `bytes` bound to a data type: a swap of the element components on the GPU when the stored
/// endianness differs from the host's, zarrs' borrowed passthrough otherwise.
#[derive(Debug)]
pub struct GpuBytesBound {
    cpu: Arc<dyn ArrayToBytesCodecTraits>,
    chain: Option<Arc<Chain>>,
    data_type: DataType,
    fill_value: FillValue,
}

impl ArrayCodecTraits for GpuBytesBound {
    fn as_any(&self) -> &dyn std::any::Any {
        self
    }
    fn data_type(&self) -> &DataType {
        &self.data_type
    }
    fn fill_value(&self) -> &FillValue {
        &self.fill_value
    }
    fn recommended_concurrency(&self, shape: &[NonZeroU64]) -> Result<RecommendedConcurrency, CodecError> {
        self.cpu.recommended_concurrency(shape)
    }
}

impl ArrayToBytesCodecSubchunkingTraits for GpuBytesBound {
    fn decoded_subchunk_grids(
        &self,
        decoded_chunk_grid: ChunkGridDecodedRef<'_>,
    ) -> Result<Vec<ChunkGridDecoded>, ChunkGridCreateError> {
        self.cpu.decoded_subchunk_grids(decoded_chunk_grid)
    }
}

impl ArrayToBytesCodecTraits for GpuBytesBound {
    fn into_dyn(self: Arc<Self>) -> Arc<dyn ArrayToBytesCodecTraits> {
        self
    }

    fn encoded_representation(&self, shape: &[NonZeroU64]) -> Result<BytesRepresentation, CodecError> {
        self.cpu.encoded_representation(shape)
    }

    fn encode<'a>(
        &self,
        bytes: ArrayBytes<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<ArrayBytesRaw<'a>, CodecError> {
        self.cpu.encode(bytes, shape, options)
    }

    /// BytesCodecBound::decode (bytes_codec.rs:203-219): the swap on the GPU (one chunk, full path).
    fn decode<'a>(
        &self,
        bytes: ArrayBytesRaw<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<ArrayBytes<'a>, CodecError> {
        let Some(chain) = &self.chain else {
            return self.cpu.decode(bytes, shape, options);
        };
        let shape: Vec<u64> = shape.iter().map(|s| s.get()).collect();
        let zeros = vec![0u64; shape.len()];
        let out = chain.decode_region(&bytes, &shape, &zeros, &shape, options.validate_checksums())?;
        Ok(ArrayBytes::new_flen(Cow::Owned(out)))
    }

    fn partial_decoder(
        self: Arc<Self>,
        input_handle: Arc<dyn BytesPartialDecoderTraits>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<Arc<dyn ArrayPartialDecoderTraits>, CodecError> {
        // BytesCodecPartial reads only the byte ranges of the requested elements
        // (bytes_codec_partial.rs:85-123): zarrs' own
        self.cpu.clone().partial_decoder(input_handle, shape, options)
    }

    fn partial_encoder(
        self: Arc<Self>,
        input_output_handle: Arc<dyn BytesPartialEncoderTraits>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<Arc<dyn ArrayPartialEncoderTraits>, CodecError> {
        self.cpu.clone().partial_encoder(input_output_handle, shape, options)
    }
}

// ---------------------------------------------------------------------------------------------------
// array -> array: transpose
// ---------------------------------------------------------------------------------------------------

/// The unbound GPU `transpose` codec.
#[derive(Debug)]
pub struct GpuTranspose {
    cpu: Arc<dyn UnboundArrayToArrayCodecTraits>,
    meta_json: String,
}

impl CodecTraits for GpuTranspose {
    fn configuration(&self, version: ZarrVersion, options: &CodecMetadataOptions) -> Option<Configuration> {
        self.cpu.configuration(version, options)
    }
    fn partial_decoder_capability(&self) -> PartialDecoderCapability {
        self.cpu.partial_decoder_capability()
    }
    fn partial_encoder_capability(&self) -> PartialEncoderCapability {
        self.cpu.partial_encoder_capability()
    }
}

impl UnboundArrayToArrayCodecTraits for GpuTranspose {
    fn into_dyn(self: Arc<Self>) -> Arc<dyn UnboundArrayToArrayCodecTraits> {
        self
    }

    fn with_context(
        &self,
        data_type: DataType,
        fill_value: FillValue,
    ) -> Result<Arc<dyn ArrayToArrayCodecTraits>, CodecCreateError> {
        let cpu = self.cpu.with_context(data_type.clone(), fill_value.clone())?;
        // [transpose, bytes(native)]: the permutation alone, element bytes untouched
        let native = if cfg!(target_endian = "little") { "little" } else { "big" };
        let json = format!(r#"[{},{{"name":"bytes","configuration":{{"endian":"{native}"}}}}]"#, self.meta_json);
        let chain = match data_type.fixed_size() {
            Some(_) => Some(Arc::new(Chain::new(&json, &data_type, &fill_value)?)),
            None => None,
        };
        Ok(Arc::new(GpuTransposeBound { cpu, chain, data_type, fill_value }))
    }
}

/// `transpose` bound to a data type: TransposeCodecBound::decode (transpose_codec.rs:264-281) as the
/// GPU's tiled permutation of one chunk.
#[derive(Debug)]
pub struct GpuTransposeBound {
    cpu: Arc<dyn ArrayToArrayCodecTraits>,
    chain: Option<Arc<Chain>>,
    data_type: DataType,
    fill_value: FillValue,
}

impl ArrayCodecTraits for GpuTransposeBound {
    fn as_any(&self) -> &dyn std::any::Any {
        self
    }
    fn data_type(&self) -> &DataType {
        &self.data_type
    }
    fn fill_value(&self) -> &FillValue {
        &self.fill_value
    }
    fn recommended_concurrency(&self, shape: &[NonZeroU64]) -> Result<RecommendedConcurrency, CodecError> {
        self.cpu.recommended_concurrency(shape)
    }
}

impl ArrayToArrayCodecSubchunkingTraits for GpuTransposeBound {
    fn encoded_chunk_grid(
        &self,
        decoded_chunk_grid: ChunkGridDecodedRef<'_>,
    ) -> Result<ChunkGridEncoded, ChunkGridCreateError> {
        self.cpu.encoded_chunk_grid(decoded_chunk_grid)
    }

    fn decoded_subchunk_grid(
        &self,
        decoded_chunk_grid: ChunkGridDecodedRef<'_>,
        encoded_subchunk_grid: ChunkGridEncodedRef<'_>,
    ) -> Result<ChunkGridDecoded, ChunkGridCreateError> {
        self.cpu.decoded_subchunk_grid(decoded_chunk_grid, encoded_subchunk_grid)
    }
}

impl ArrayToArrayCodecTraits for GpuTransposeBound {
    fn into_dyn(self: Arc<Self>) -> Arc<dyn ArrayToArrayCodecTraits> {
        self
    }

    fn encoded_data_type(&self) -> &DataType {
        self.cpu.encoded_data_type()
    }

    fn encoded_fill_value(&self) -> &FillValue {
        self.cpu.encoded_fill_value()
    }

    fn encoded_shape(&self, decoded_shape: &[NonZeroU64]) -> Result<ChunkShape, CodecError> {
        self.cpu.encoded_shape(decoded_shape)
    }

    fn partial_decode_granularity(
        &self,
        decoded_shape: &[NonZeroU64],
        encoded_granularity: &[NonZeroU64],
    ) -> Result<ChunkShape, CodecError> {
        self.cpu.partial_decode_granularity(decoded_shape, encoded_granularity)
    }

    fn encode<'a>(
        &self,
        bytes: ArrayBytes<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<ArrayBytes<'a>, CodecError> {
        self.cpu.encode(bytes, shape, options)
    }

    fn decode<'a>(
        &self,
        bytes: ArrayBytes<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<ArrayBytes<'a>, CodecError> {
        let Some(chain) = &self.chain else {
            return self.cpu.decode(bytes, shape, options);
        };
        let raw = bytes.into_fixed()?;
        let shape: Vec<u64> = shape.iter().map(|s| s.get()).collect();
        let zeros = vec![0u64; shape.len()];
        let out = chain.decode_region(&raw, &shape, &zeros, &shape, options.validate_checksums())?;
        Ok(ArrayBytes::new_flen(Cow::Owned(out)))
    }

    fn partial_decoder(
        self: Arc<Self>,
        input_handle: Arc<dyn ArrayPartialDecoderTraits>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<Arc<dyn ArrayPartialDecoderTraits>, CodecError> {
        self.cpu.clone().partial_decoder(input_handle, shape, options)
    }

    fn partial_encoder(
        self: Arc<Self>,
        input_output_handle: Arc<dyn ArrayPartialEncoderTraits>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<Arc<dyn ArrayPartialEncoderTraits>, CodecError> {
        self.cpu.clone().partial_encoder(input_output_handle, shape, options)
    }
}
