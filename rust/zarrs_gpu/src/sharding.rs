//! GPU `sharding_indexed`: decode on the MI355X, everything else delegated to zarrs' ShardingCodec.
//!
//! Reference: zarrs/src/array/codec/array_to_bytes/sharding/sharding_codec.rs (ShardingCodec,
//! ShardingCodecBound::{decode :378-518, decode_into :617-707}) and sharding_partial_decoder_sync.rs
//! (ShardingPartialDecoder::partial_decode_into :311-400). The trait surface is zarrs_codec's
//! UnboundArrayToBytesCodecTraits / ArrayToBytesCodecTraits (codec_traits/array_to_bytes.rs:77-270).

use std::any::Any;
use std::borrow::Cow;
use std::num::NonZeroU64;
use std::sync::Arc;

use zarrs::array::codec::ShardingCodec;
use zarrs_chunk_grid::{ChunkGridCreateError, Indexer};
use zarrs_codec::{
    ArrayBytes, ArrayBytesRaw, ArrayCodecTraits, ArrayPartialDecoderNoSubchunkingTraits, ArrayPartialDecoderTraits,
    ArrayPartialEncoderTraits, ArrayToBytesCodecSubchunkingTraits, ArrayToBytesCodecTraits, BytesPartialDecoderTraits,
    BytesPartialEncoderTraits, BytesRepresentation, ChunkGridDecoded, ChunkGridDecodedRef, Codec, CodecCreateError,
    CodecError, CodecMetadataOptions, CodecOptions, CodecSpecificOptions, CodecTraits, CodecTraitsV3,
    PartialDecoderCapability, PartialEncoderCapability, RecommendedConcurrency, UnboundArrayToBytesCodecTraits,
};
use zarrs_data_type::{DataType, FillValue};
use zarrs_metadata::Configuration;
use zarrs_metadata::v3::MetadataV3;
use zarrs_plugin::ZarrVersion;
use zarrs_storage::StorageError;

use crate::Chain;

/// The unbound GPU `sharding_indexed` codec: zarrs' own ShardingCodec (for metadata, encoding and
/// subchunk grids) plus the codec metadata the GPU chain is created from at bind time.
#[derive(Debug)]
pub struct GpuShardingCodec {
    cpu: Arc<dyn UnboundArrayToBytesCodecTraits>,
    codecs_json: String,
}

zarrs_plugin::impl_extension_aliases!(GpuShardingCodec, v3: "sharding_indexed");

impl GpuShardingCodec {
    /// The runtime-plugin create function (CodecTraitsV3::create of the reference codec, wrapped).
    ///
    /// # Errors
    /// Returns [`CodecCreateError`] if zarrs' ShardingCodec cannot be created from `metadata`.
    pub fn create(metadata: &MetadataV3) -> Result<Codec, CodecCreateError> {
        let Codec::ArrayToBytes(cpu) = <ShardingCodec as CodecTraitsV3>::create(metadata)? else {
            return Err(CodecCreateError::Other("sharding_indexed is not an array-to-bytes codec".into()));
        };
        // the GPU chain parses the same metadata: a one-codec "codecs" list
        let codecs_json = serde_json::to_string(&[metadata]).map_err(CodecCreateError::other)?;
        Ok(Codec::ArrayToBytes(Arc::new(Self { cpu, codecs_json })))
    }
}

impl CodecTraits for GpuShardingCodec {
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

impl UnboundArrayToBytesCodecTraits for GpuShardingCodec {
    fn into_dyn(self: Arc<Self>) -> Arc<dyn UnboundArrayToBytesCodecTraits> {
        self
    }

    fn with_codec_specific_options(
        self: Arc<Self>,
        opts: &CodecSpecificOptions,
    ) -> Result<Arc<dyn UnboundArrayToBytesCodecTraits>, CodecCreateError> {
        let cpu = self.cpu.clone().with_codec_specific_options(opts)?;
        Ok(Arc::new(Self { cpu, codecs_json: self.codecs_json.clone() }))
    }

    fn with_context(
        &self,
        data_type: DataType,
        fill_value: FillValue,
    ) -> Result<Arc<dyn ArrayToBytesCodecTraits>, CodecCreateError> {
        let cpu = self.cpu.with_context(data_type.clone(), fill_value.clone())?;
        let chain = Chain::new(&self.codecs_json, &data_type, &fill_value)?;
        Ok(Arc::new(GpuShardingCodecBound { cpu, chain: Arc::new(chain), data_type, fill_value }))
    }
}

/// `sharding_indexed` bound to a data type and fill value: decoding runs on the GPU.
#[derive(Debug)]
pub struct GpuShardingCodecBound {
    cpu: Arc<dyn ArrayToBytesCodecTraits>,
    chain: Arc<Chain>,
    data_type: DataType,
    fill_value: FillValue,
}

fn u64s(shape: &[NonZeroU64]) -> Vec<u64> {
    shape.iter().map(|s| s.get()).collect()
}

impl ArrayCodecTraits for GpuShardingCodecBound {
    fn as_any(&self) -> &dyn Any {
        self
    }

    fn data_type(&self) -> &DataType {
        &self.data_type
    }

    fn fill_value(&self) -> &FillValue {
        &self.fill_value
    }

    /// One shard is one GPU batch: no inner (codec) concurrency to hand out to rayon.
    fn recommended_concurrency(&self, _shape: &[NonZeroU64]) -> Result<RecommendedConcurrency, CodecError> {
        Ok(RecommendedConcurrency::new_maximum(1))
    }
}

impl ArrayToBytesCodecSubchunkingTraits for GpuShardingCodecBound {
    fn decoded_subchunk_grids(
        &self,
        decoded_chunk_grid: ChunkGridDecodedRef<'_>,
    ) -> Result<Vec<ChunkGridDecoded>, ChunkGridCreateError> {
        self.cpu.decoded_subchunk_grids(decoded_chunk_grid)
    }
}

impl ArrayToBytesCodecTraits for GpuShardingCodecBound {
    fn into_dyn(self: Arc<Self>) -> Arc<dyn ArrayToBytesCodecTraits> {
        self
    }

    fn encoded_representation(&self, shape: &[NonZeroU64]) -> Result<BytesRepresentation, CodecError> {
        self.cpu.encoded_representation(shape)
    }

    /// The write path stays zarrs' (ShardingCodecBound::encode, sharding_codec.rs:351-376).
    fn encode<'a>(
        &self,
        bytes: ArrayBytes<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<ArrayBytesRaw<'a>, CodecError> {
        self.cpu.encode(bytes, shape, options)
    }

    /// ShardingCodecBound::decode: every inner chunk of the shard in one zgpu_decode_batch call
    /// (index decode + crc32c verify, inner chains, scatter into the shard), checksums verified per
    /// `options.validate_checksums()`. The default `decode_into` copies the result into the view.
    fn decode<'a>(
        &self,
        bytes: ArrayBytesRaw<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<ArrayBytes<'a>, CodecError> {
        let shape = u64s(shape);
        let zeros = vec![0u64; shape.len()];
        let out = self.chain.decode_region(&bytes, &shape, &zeros, &shape, options.validate_checksums())?;
        Ok(ArrayBytes::new_flen(Cow::Owned(out)))
    }

    fn compact<'a>(
        &self,
        bytes: ArrayBytesRaw<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<Option<ArrayBytesRaw<'a>>, CodecError> {
        self.cpu.compact(bytes, shape, options)
    }

    fn partial_decoder(
        self: Arc<Self>,
        input_handle: Arc<dyn BytesPartialDecoderTraits>,
        shape: &[NonZeroU64],
        _options: &CodecOptions,
    ) -> Result<Arc<dyn ArrayPartialDecoderTraits>, CodecError> {
        Ok(Arc::new(GpuShardPartialDecoder { input: input_handle, shape: u64s(shape), codec: self }))
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

/// ShardingPartialDecoder on the GPU: the shard's bytes are read once, and only the inner chunks that
/// intersect the requested subset are decoded (crc32c stripped, not verified: crc32c_codec.rs:143-158),
/// all in one zgpu_decode_batch call. A missing shard reads as the fill value (:329-333).
struct GpuShardPartialDecoder {
    input: Arc<dyn BytesPartialDecoderTraits>,
    shape: Vec<u64>,
    codec: Arc<GpuShardingCodecBound>,
}

impl ArrayPartialDecoderNoSubchunkingTraits for GpuShardPartialDecoder {}

impl ArrayPartialDecoderTraits for GpuShardPartialDecoder {
    fn data_type(&self) -> &DataType {
        &self.codec.data_type
    }

    fn exists(&self) -> Result<bool, StorageError> {
        self.input.exists()
    }

    fn size_held(&self) -> usize {
        self.input.size_held()
    }

    fn partial_decode(&self, indexer: &dyn Indexer, options: &CodecOptions) -> Result<ArrayBytes<'_>, CodecError> {
        let Some(encoded) = self.input.decode(options)? else {
            return Ok(ArrayBytes::new_fill_value(&self.codec.data_type, indexer.len(), &self.codec.fill_value)?);
        };
        let chain = &self.codec.chain;
        if let Some(subset) = indexer.as_array_subset() {
            let (start, shape) = (subset.start(), subset.shape());
            let inside = start.len() == self.shape.len()
                && start.iter().zip(shape.iter()).zip(&self.shape).all(|((s, n), e)| s + n <= *e);
            if !inside {
                return Err(CodecError::Other(format!(
                    "subset {start:?} + {shape:?} is out of the bounds of the shard {:?}",
                    self.shape
                )));
            }
            if shape.iter().any(|&n| n == 0) {
                return Ok(ArrayBytes::new_flen(Cow::Owned(Vec::new())));
            }
            let out = chain.decode_region(&encoded, &self.shape, &start, &shape, options.validate_checksums())?;
            return Ok(ArrayBytes::new_flen(Cow::Owned(out)));
        }
        // arbitrary indexers: the whole shard decoded on the GPU, the indexed elements gathered here
        let zeros = vec![0u64; self.shape.len()];
        let full = chain.decode_region(&encoded, &self.shape, &zeros, &self.shape, options.validate_checksums())?;
        let es = chain.element_size;
        let mut out = Vec::with_capacity(usize::try_from(indexer.len()).unwrap_or(0) * es);
        for i in indexer.iter_linearised_indices(&self.shape)? {
            let o = usize::try_from(i).map_err(|e| CodecError::Other(e.to_string()))? * es;
            out.extend_from_slice(&full[o..o + es]);
        }
        Ok(ArrayBytes::new_flen(Cow::Owned(out)))
    }

    fn supports_partial_decode(&self) -> bool {
        true
    }
}
