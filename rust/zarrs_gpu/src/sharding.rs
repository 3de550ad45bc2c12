//! GPU `sharding_indexed`: decode on the MI355X, everything else delegated to zarrs' ShardingCodec.
//! Whole shards (decode / decode_into) are one zgpu_decode_batch of the sharded chain; the partial
//! decoder reads the index and only the intersecting inner chunks by ranged reads, as zarrs does.
//!
//! Reference: zarrs/src/array/codec/array_to_bytes/sharding/sharding_codec.rs (ShardingCodec,
//! ShardingCodecBound::{decode :378-518, decode_into :617-707}) and sharding_partial_decoder_sync.rs
//! (ShardingPartialDecoder::partial_decode_into :311-400). The trait surface is zarrs_codec's
//! UnboundArrayToBytesCodecTraits / ArrayToBytesCodecTraits (codec_traits/array_to_bytes.rs:77-270).

use std::any::Any;
use std::borrow::Cow;
use std::collections::HashMap;
use std::num::NonZeroU64;
use std::sync::Arc;

use zarrs::array::codec::ShardingCodec;
use zarrs::array::{CodecChain, CodecChainBound, data_type};
use zarrs_metadata_ext::codec::sharding::{ShardingCodecConfiguration, ShardingCodecConfigurationV1, ShardingIndexLocation};
use zarrs_storage::byte_range::ByteRange;
use zarrs_chunk_grid::{ChunkGridCreateError, Indexer, IndexerError};
use zarrs_codec::{
    ArrayBytes, ArrayBytesDecodeIntoTarget, ArrayBytesRaw, ArrayCodecTraits, ArrayPartialDecoderNoSubchunkingTraits, ArrayPartialDecoderTraits,
    ArrayPartialEncoderTraits, ArrayToBytesCodecSubchunkingTraits, ArrayToBytesCodecTraits, BytesPartialDecoderTraits,
    BytesPartialEncoderTraits, BytesRepresentation, ChunkGridDecoded, ChunkGridDecodedRef, Codec, CodecCreateError,
    CodecError, CodecMetadataOptions, CodecOptions, CodecSpecificOptions, CodecTraits, CodecTraitsV3,
    InvalidNumberOfElementsError,
    PartialDecoderCapability, PartialEncoderCapability, RecommendedConcurrency, UnboundArrayToBytesCodecTraits,
    decode_into_array_bytes_target,
};
use zarrs_data_type::{DataType, FillValue};
use zarrs_metadata::Configuration;
use zarrs_metadata::v3::MetadataV3;
use zarrs_plugin::ZarrVersion;
use zarrs_storage::StorageError;

use crate::{Chain, Pinned, ffi};

/// The unbound GPU `sharding_indexed` codec: zarrs' own ShardingCodec (for metadata, encoding and
/// subchunk grids) plus the codec metadata the GPU chain is created from at bind time.
#[derive(Debug)]
pub struct GpuShardingCodec {
    cpu: Arc<dyn UnboundArrayToBytesCodecTraits>,
    codecs_json: String,
    config: ShardingCodecConfigurationV1,
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
        let ShardingCodecConfiguration::V1(config) = metadata.to_typed_configuration::<ShardingCodecConfiguration>()
            .map_err(|e| CodecCreateError::Other(e.to_string()))?;
        Ok(Codec::ArrayToBytes(Arc::new(Self { cpu, codecs_json, config })))
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
        Ok(Arc::new(Self { cpu, codecs_json: self.codecs_json.clone(), config: self.config.clone() }))
    }

    fn with_context(
        &self,
        data_type: DataType,
        fill_value: FillValue,
    ) -> Result<Arc<dyn ArrayToBytesCodecTraits>, CodecCreateError> {
        let cpu = self.cpu.with_context(data_type.clone(), fill_value.clone())?;
        let chain = Chain::new(&self.codecs_json, &data_type, &fill_value)?;
        // the inner chain alone (the partial decoder batches the intersecting inner chunks through
        // it) and zarrs' own index chain, bound to uint64 / u64::MAX (sharding_codec.rs:266-268)
        let inner_json = serde_json::to_string(&self.config.codecs).map_err(CodecCreateError::other)?;
        let inner_chain = Chain::new(&inner_json, &data_type, &fill_value)?;
        let index_chain = CodecChain::from_metadata(&self.config.index_codecs)?
            .with_context(data_type::uint64(), FillValue::from(u64::MAX))?;
        Ok(Arc::new(GpuShardingCodecBound {
            cpu,
            chain: Arc::new(chain),
            inner_chain: Arc::new(inner_chain),
            index_chain,
            subchunk_shape: self.config.chunk_shape.iter().map(|c| c.get()).collect(),
            index_location: self.config.index_location,
            data_type,
            fill_value,
        }))
    }
}

/// `sharding_indexed` bound to a data type and fill value: decoding runs on the GPU.
#[derive(Debug)]
pub struct GpuShardingCodecBound {
    cpu: Arc<dyn ArrayToBytesCodecTraits>,
    chain: Arc<Chain>,
    inner_chain: Arc<Chain>,
    index_chain: Arc<CodecChainBound>,
    subchunk_shape: Vec<u64>,
    index_location: ShardingIndexLocation,
    data_type: DataType,
    fill_value: FillValue,
}

fn u64s(shape: &[NonZeroU64]) -> Vec<u64> {
    shape.iter().map(|s| s.get()).collect()
}

const OOB: &str = "The shard index references out-of-bounds bytes. The chunk may be corrupted.";

impl GpuShardingCodecBound {
    /// Inner chunks per shard along each axis (calculate_chunks_per_shard, sharding.rs:136-154).
    fn chunks_per_shard(&self, shard_shape: &[u64]) -> Result<Vec<u64>, CodecError> {
        if shard_shape.len() != self.subchunk_shape.len() {
            return Err(CodecError::Other("sharding: shard / subchunk dimensionality mismatch".into()));
        }
        shard_shape
            .iter()
            .zip(&self.subchunk_shape)
            .map(|(&s, &c)| {
                if c == 0 || s % c != 0 {
                    Err(CodecError::Other(format!("sharding: subchunk shape {c} does not divide shard shape {s}")))
                } else {
                    Ok(s / c)
                }
            })
            .collect()
    }

    /// decode_shard_index_partial_decoder (sharding.rs:267-288): the encoded index by one ranged
    /// read, decoded (and its crc32c verified) by zarrs' own index chain on the host: it is
    /// 16 B per inner chunk, and the GPU work is the inner chunks. None: the shard does not exist.
    fn read_index(
        &self,
        input: &dyn BytesPartialDecoderTraits,
        shard_shape: &[u64],
        options: &CodecOptions,
    ) -> Result<Option<Vec<u64>>, CodecError> {
        let cps = self.chunks_per_shard(shard_shape)?;
        let mut index_shape: Vec<NonZeroU64> =
            cps.iter().map(|&c| NonZeroU64::new(c).expect("positive")).collect();
        index_shape.push(NonZeroU64::new(2).expect("two"));
        let BytesRepresentation::FixedSize(index_size) = self.index_chain.encoded_representation(&index_shape)? else {
            return Err(CodecError::Other("the array index cannot include a variable size output codec".into()));
        };
        let range = match self.index_location {
            ShardingIndexLocation::Start => ByteRange::FromStart(0, Some(index_size)),
            ShardingIndexLocation::End => ByteRange::Suffix(index_size),
        };
        let Some(encoded) = input.partial_decode(range, options)? else {
            return Ok(None);
        };
        let decoded = self.index_chain.decode(encoded, &index_shape, options)?.into_fixed()?;
        Ok(Some(decoded.chunks_exact(8).map(|b| u64::from_ne_bytes(b.try_into().expect("8 bytes"))).collect()))
    }
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

    /// ShardingCodecBound::encode (sharding_codec.rs:351-376) on the GPU: the shard's inner chunks
    /// encoded by zgpu_encode_pinned (inner chains of fixed-size stages, gzip, zstd, blosc, crc32c; an
    /// inner chunk equal to the fill value everywhere omitted; the index encoded with its chain), the
    /// bytes copied once into the returned buffer. Chains the GPU write path does not take (and
    /// variable-size data types) stay with zarrs' own encoder.
    fn encode<'a>(
        &self,
        bytes: ArrayBytes<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<ArrayBytesRaw<'a>, CodecError> {
        // the reference's length check first (sharding_codec.rs:357-359): a wrong-length input is
        // InvalidBytesLength whichever encoder would have run
        let num_elements = shape.iter().map(|d| d.get()).product::<u64>();
        bytes.validate(num_elements, &self.data_type)?;
        if self.data_type.fixed_size().is_some() {
            if let ArrayBytes::Fixed(raw) = &bytes {
                if let Some(enc) = self.chain.encode_pinned(raw, &u64s(shape))? {
                    return Ok(Cow::Owned(enc.as_slice().to_vec()));
                }
            }
        }
        self.cpu.encode(bytes, shape, options)
    }

    /// ShardingCodecBound::decode: every inner chunk of the shard in one zgpu_decode_batch call
    /// (index decode + crc32c verify, inner chains, scatter into the shard), checksums verified per
    /// `options.validate_checksums()`, coalesced with concurrent calls (ZGPU_COALESCE).
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

    /// ShardingCodecBound::decode_into (sharding_codec.rs:617-707) into the caller's disjoint view
    /// (the shard's place in the retrieve_array_subset output, array_read_ops_common.rs:150-176): the
    /// shard's inner chunks are decoded in one GPU batch, coalesced (ZGPU_COALESCE) with the shards the
    /// other rayon workers hand over at the same time, and the compact result is placed into the view
    /// run by run (ArrayBytesFixedDisjointView::copy_from_slice, array_bytes_fixed_disjoint_view.rs:
    /// 177-206). zarrs_codec exposes no raw pointer of a view, so the rows are placed here; a caller that
    /// holds the raw output array (ArrayGpuExt) passes it to zgpu_decode_into, which places the rows
    /// itself. Optional (masked) targets take the trait default.
    fn decode_into(
        &self,
        bytes: ArrayBytesRaw<'_>,
        shape: &[NonZeroU64],
        output_target: ArrayBytesDecodeIntoTarget<'_>,
        options: &CodecOptions,
    ) -> Result<(), CodecError> {
        match output_target {
            ArrayBytesDecodeIntoTarget::Fixed(view) => {
                let shape = u64s(shape);
                let n: u64 = shape.iter().product();
                if view.num_elements() != n {
                    return Err(CodecError::Other(format!(
                        "decode_into: the view holds {} elements, the shard {n}",
                        view.num_elements()
                    )));
                }
                let nd = shape.len();
                if nd == 0 || nd > ffi::ZGPU_MAX_DIMS {
                    return Err(CodecError::Other(format!("zgpu: unsupported dimensionality {nd}")));
                }
                let mut d = ffi::zgpu_chunk_desc { enc: bytes.as_ptr().cast(), enc_len: bytes.len() as u64, ..Default::default() };
                d.chunk_shape[..nd].copy_from_slice(&shape);
                d.sel_shape[..nd].copy_from_slice(&shape);
                let flags = ffi::ZGPU_COALESCE | if options.validate_checksums() { 0 } else { ffi::ZGPU_NO_VALIDATE };
                // the decoded shard stays in library pinned memory: one copy into the view, no Vec
                let decoded = self.chain.decode_pinned(&[d], &shape, flags)?;
                view.copy_from_slice(decoded.as_slice())?;
                Ok(())
            }
            target => {
                let decoded = self.decode(bytes, shape, options)?;
                decode_into_array_bytes_target(&decoded, target)
            }
        }
    }

    fn compact<'a>(
        &self,
        bytes: ArrayBytesRaw<'a>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<Option<ArrayBytesRaw<'a>>, CodecError> {
        self.cpu.compact(bytes, shape, options)
    }

    /// ShardingPartialDecoder::new (sharding_partial_decoder_sync.rs:47-74): only the shard index is
    /// read here, by a suffix (index at the end) or prefix byte range (sharding.rs:196-207,267-288).
    fn partial_decoder(
        self: Arc<Self>,
        input_handle: Arc<dyn BytesPartialDecoderTraits>,
        shape: &[NonZeroU64],
        options: &CodecOptions,
    ) -> Result<Arc<dyn ArrayPartialDecoderTraits>, CodecError> {
        let shape = u64s(shape);
        let index = self.read_index(&*input_handle, &shape, options)?;
        Ok(Arc::new(GpuShardPartialDecoder { input: input_handle, shape, codec: self, index }))
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

/// ShardingPartialDecoder on the GPU (sharding_partial_decoder_sync.rs:34-400). Created with the
/// shard index only (`index`, read by a ranged read: `None` = the shard does not exist). A partial
/// decode reads the byte ranges of the inner chunks that intersect the subset with ONE
/// `partial_decode_many` call (get_subchunk_partial_decoder's ByteIntervalPartialDecoder reads,
/// :279-308, batched), and decodes all of them in ONE zgpu_decode_batch of the inner chain: each
/// intersecting inner chunk is a descriptor whose selection is its overlap with the subset, decoded
/// on the partial-decoder path (crc32c stripped, not verified: crc32c_codec.rs:143-158); empty inner
/// chunks are fill-value descriptors (:380-381).
struct GpuShardPartialDecoder {
    input: Arc<dyn BytesPartialDecoderTraits>,
    shape: Vec<u64>,
    codec: Arc<GpuShardingCodecBound>,
    index: Option<Vec<u64>>,
}

impl GpuShardPartialDecoder {
    /// The shard index entry of inner chunk `lin` (C order of the inner grid): None = empty.
    fn entry(index: &[u64], lin: usize) -> Result<Option<ByteRange>, CodecError> {
        let (offset, size) = (index[2 * lin], index[2 * lin + 1]);
        if offset == u64::MAX && size == u64::MAX {
            return Ok(None);
        }
        let end = offset.checked_add(size).ok_or_else(|| CodecError::Other(OOB.into()))?;
        Ok(Some(ByteRange::new(offset..end)))
    }

    /// One batched ranged read of every present inner chunk (get_subchunk_partial_decoder's
    /// ByteIntervalPartialDecoder reads, :279-308): the bytes, and each descriptor's pointer set.
    fn read_inner(
        &self,
        ranges: Vec<ByteRange>,
        present: &[usize],
        descs: &mut [ffi::zgpu_chunk_desc],
        options: &CodecOptions,
    ) -> Result<Vec<Vec<u8>>, CodecError> {
        if ranges.is_empty() {
            return Ok(Vec::new());
        }
        let bytes: Vec<Vec<u8>> = match self.input.partial_decode_many(Box::new(ranges.into_iter()), options) {
            Ok(Some(b)) => b.into_iter().map(|x| x.into_owned()).collect(),
            Ok(None) => return Err(CodecError::Other("zarrs_gpu: the shard disappeared during the read".into())),
            Err(CodecError::InvalidByteRangeError(_)) => return Err(CodecError::Other(OOB.into())),
            Err(e) => return Err(e),
        };
        for (b, &k) in bytes.iter().zip(present) {
            descs[k].enc = b.as_ptr().cast();
            descs[k].enc_len = b.len() as u64;
        }
        Ok(bytes)
    }

    /// partial_decode_fixed_array_subset_into (sharding_partial_decoder_sync.rs:311-400): the inner
    /// chunks intersecting [start, start + shape), each a descriptor whose selection is its overlap
    /// (crc32c stripped, not verified: crc32c_codec.rs:143-158; empty inner chunks are fill
    /// descriptors, :380-381), decoded in ONE coalesced zgpu_decode_pinned of the inner chain. None: the
    /// shard does not exist (the caller fills, :329-333).
    fn decode_subset_pinned(&self, start: &[u64], shape: &[u64], options: &CodecOptions) -> Result<Option<Pinned>, CodecError> {
        let Some(index) = &self.index else {
            return Ok(None);
        };
        let codec = &self.codec;
        let cps = codec.chunks_per_shard(&self.shape)?;
        let sub = &codec.subchunk_shape;
        let nd = self.shape.len();
        // the intersecting inner chunks, C order (chunks_in_array_subset of the shard's grid)
        let lo: Vec<u64> = start.iter().zip(sub).map(|(s, c)| s / c).collect();
        let hi: Vec<u64> = start.iter().zip(shape).zip(sub).map(|((s, n), c)| (s + n - 1) / c + 1).collect();
        let mut descs = Vec::new();
        let mut ranges = Vec::new(); // byte range of each present inner chunk, in descriptor order
        let mut present = Vec::new(); // descriptor index of each range
        let total: u64 = hi.iter().zip(&lo).map(|(h, l)| h - l).product();
        for t in 0..total {
            // C-order grid coordinates of the t-th intersecting inner chunk
            let mut idx = vec![0u64; nd];
            let mut rem = t;
            for a in (0..nd).rev() {
                let ext = hi[a] - lo[a];
                idx[a] = lo[a] + rem % ext;
                rem /= ext;
            }
            let lin = idx.iter().zip(&cps).fold(0u64, |acc, (i, c)| acc * c + i) as usize;
            let mut d = ffi::zgpu_chunk_desc::default();
            for a in 0..nd {
                let c0 = idx[a] * sub[a];
                let s0 = start[a].max(c0);
                let s1 = (start[a] + shape[a]).min(c0 + sub[a]);
                d.chunk_shape[a] = sub[a];
                d.sel_start[a] = s0 - c0;
                d.sel_shape[a] = s1 - s0;
                d.out_start[a] = s0 - start[a];
            }
            if let Some(r) = Self::entry(index, lin)? {
                ranges.push(r);
                present.push(descs.len());
            }
            descs.push(d);
        }
        let _bytes = self.read_inner(ranges, &present, &mut descs, options)?;
        // coalesced with the partial shards other rayon workers decode at the same time
        Ok(Some(codec.inner_chain.decode_pinned(&descs, shape, ffi::ZGPU_NO_VALIDATE | ffi::ZGPU_COALESCE)?))
    }

    fn fill_bytes(&self, n: u64) -> Result<Vec<u8>, CodecError> {
        let es = self.codec.inner_chain.element_size;
        let mut out = vec![0u8; usize::try_from(n).map_err(|e| CodecError::Other(e.to_string()))? * es];
        let fill = self.codec.fill_value.as_ne_bytes();
        out.chunks_exact_mut(es).for_each(|c| c.copy_from_slice(fill));
        Ok(out)
    }

    /// partial_decode_fixed_indexer (sharding_partial_decoder_sync.rs:492-560) for indexers that are
    /// not an array subset: only the inner chunks the indices touch are decoded -- each once (the
    /// reference's per-chunk decoder cache), all of them in ONE zgpu_decode_pinned whose output stacks
    /// them along axis 0 -- and the indexed elements gathered from the pinned result in indexer order.
    fn decode_indexer(&self, indexer: &dyn Indexer, options: &CodecOptions) -> Result<Vec<u8>, CodecError> {
        let codec = &self.codec;
        let es = codec.inner_chain.element_size;
        let cps = codec.chunks_per_shard(&self.shape)?;
        let sub = &codec.subchunk_shape;
        let nd = self.shape.len();
        let chunk_elems: u64 = sub.iter().product();
        let mut slot: HashMap<u64, usize> = HashMap::new();
        let mut order: Vec<u64> = Vec::new(); // touched inner chunks, first-touch order
        let mut elems: Vec<(usize, u64)> = Vec::new(); // (slot, element offset inside the inner chunk)
        for indices in indexer.iter_indices() {
            if indices.len() != nd {
                return Err(IndexerError::new_incompatible_dimensionality(indices.len(), nd).into());
            }
            let ci: Vec<u64> = indices.iter().zip(sub).map(|(&i, &c)| i / c).collect();
            if ci.iter().zip(&cps).any(|(a, b)| a >= b) {
                return Err(IndexerError::new_oob(ci, cps.clone()).into());
            }
            let lin = ci.iter().zip(&cps).fold(0u64, |acc, (i, c)| acc * c + i);
            let k = *slot.entry(lin).or_insert_with(|| {
                order.push(lin);
                order.len() - 1
            });
            let within = indices.iter().zip(sub).fold(0u64, |acc, (&i, &c)| acc * c + i % c);
            elems.push((k, within));
        }
        let Some(index) = &self.index else {
            return self.fill_bytes(elems.len() as u64);
        };
        let mut descs = Vec::with_capacity(order.len());
        let mut ranges = Vec::new();
        let mut present = Vec::new();
        for (k, &lin) in order.iter().enumerate() {
            let mut d = ffi::zgpu_chunk_desc::default();
            d.chunk_shape[..nd].copy_from_slice(sub);
            d.sel_shape[..nd].copy_from_slice(sub);
            d.out_start[0] = k as u64 * sub[0];
            if let Some(r) = Self::entry(index, usize::try_from(lin).map_err(|e| CodecError::Other(e.to_string()))?)? {
                ranges.push(r);
                present.push(descs.len());
            }
            descs.push(d);
        }
        let _bytes = self.read_inner(ranges, &present, &mut descs, options)?;
        let mut stacked = sub.clone();
        stacked[0] *= order.len().max(1) as u64;
        let decoded = codec.inner_chain.decode_pinned(&descs, &stacked, ffi::ZGPU_NO_VALIDATE | ffi::ZGPU_COALESCE)?;
        let src = decoded.as_slice();
        let mut out = Vec::with_capacity(elems.len() * es);
        for (k, within) in elems {
            let o = usize::try_from(k as u64 * chunk_elems + within).map_err(|e| CodecError::Other(e.to_string()))? * es;
            out.extend_from_slice(&src[o..o + es]);
        }
        Ok(out)
    }

    /// The reference's checks before any decode (sharding_partial_decoder_sync.rs:118-131).
    fn check(&self, indexer: &dyn Indexer) -> Result<(), CodecError> {
        if indexer.dimensionality() != self.shape.len() {
            return Err(IndexerError::new_incompatible_dimensionality(indexer.dimensionality(), self.shape.len()).into());
        }
        if self.codec.data_type.is_optional() {
            return Err(CodecError::UnsupportedDataType(self.codec.data_type.clone(), "sharding_indexed".to_string()));
        }
        Ok(())
    }

    fn subset_inside(&self, start: &[u64], shape: &[u64]) -> Result<(), CodecError> {
        let inside = start.len() == self.shape.len()
            && start.iter().zip(shape.iter()).zip(&self.shape).all(|((s, n), e)| s + n <= *e);
        if inside {
            Ok(())
        } else {
            Err(CodecError::Other(format!("subset {start:?} + {shape:?} is out of the bounds of the shard {:?}", self.shape)))
        }
    }
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
        self.check(indexer)?;
        if let Some(subset) = indexer.as_array_subset() {
            let (start, shape) = (subset.start(), subset.shape());
            self.subset_inside(&start, &shape)?;
            let n: u64 = shape.iter().product();
            if n == 0 {
                return Ok(ArrayBytes::new_flen(Cow::Owned(Vec::new())));
            }
            let out = match self.decode_subset_pinned(&start, &shape, options)? {
                Some(p) => p.as_slice().to_vec(),
                None => self.fill_bytes(n)?, // a missing shard reads as the fill value (:329-333)
            };
            return Ok(ArrayBytes::new_flen(Cow::Owned(out)));
        }
        Ok(ArrayBytes::new_flen(Cow::Owned(self.decode_indexer(indexer, options)?)))
    }

    /// ShardingPartialDecoder::partial_decode_into (sharding_partial_decoder_sync.rs:241-272): an array
    /// subset into a fixed-size view is decoded into library pinned memory and copied into the view
    /// once (copy_from_slice: no intermediate Vec); a missing shard fills the view. Other indexers and
    /// targets decode, then copy (decode_into_array_bytes_target), as the reference does.
    fn partial_decode_into(
        &self,
        indexer: &dyn Indexer,
        output_target: ArrayBytesDecodeIntoTarget<'_>,
        options: &CodecOptions,
    ) -> Result<(), CodecError> {
        if indexer.len() != output_target.num_elements() {
            return Err(InvalidNumberOfElementsError::new(indexer.len(), output_target.num_elements()).into());
        }
        self.check(indexer)?;
        match (indexer.as_array_subset(), output_target) {
            (Some(subset), ArrayBytesDecodeIntoTarget::Fixed(view)) => {
                let (start, shape) = (subset.start(), subset.shape());
                self.subset_inside(&start, &shape)?;
                if shape.iter().product::<u64>() == 0 {
                    return Ok(());
                }
                match self.decode_subset_pinned(&start, &shape, options)? {
                    Some(decoded) => view.copy_from_slice(decoded.as_slice())?,
                    None => view.fill(self.codec.fill_value.as_ne_bytes())?,
                }
                Ok(())
            }
            (_, target) => {
                let decoded = self.partial_decode(indexer, options)?;
                decode_into_array_bytes_target(&decoded, target)
            }
        }
    }

    fn supports_partial_decode(&self) -> bool {
        self.input.supports_partial_decode()
    }
}
