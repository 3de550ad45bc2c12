//! `zarrs_gpu`: the MI355X chunk-decode pipeline (libzgpu.so, include/zgpu.h) behind zarrs' own
//! codec plugin surface, so that `zarrs/src`'s array read path runs unchanged.
//!
//! Three entry points, all over the C ABI:
//!
//! * [`register_codecs`] adds per-codec runtime plugins for the entropy stages `gzip` and `blosc`
//!   (codecs.rs): zarrs' unchanged per-chunk CodecChain then decodes them on the GPU (one coalesced
//!   zgpu_decode_pinned per chunk) and runs its own `bytes` / `transpose` / `crc32c` /
//!   `numcodecs.shuffle` / `zstd` on the host ([`register_codecs_named`] opts zstd in,
//!   [`register_codecs_all`] puts every stage on the GPU).
//! * [`register`] adds a runtime codec plugin for `sharding_indexed`
//!   (`zarrs_codec::register_codec_v3`, zarrs_codec/src/lib.rs:279-318; runtime plugins are matched
//!   before the compile-time ones, lib.rs:385-414). A shard is the natural GPU batch: its
//!   `decode`/`decode_into` (ShardingCodecBound::decode_into, sharding_codec.rs:617-707) and its
//!   partial decoder (ShardingPartialDecoder, sharding_partial_decoder_sync.rs:311-400) decode every
//!   inner chunk of the shard in one `zgpu_decode_batch` call. Everything that is not decoding
//!   (metadata, encoded representation, encode, partial encode, subchunk grids) is delegated to zarrs'
//!   own `ShardingCodec`, which the plugin wraps. This is the pattern of
//!   zarrs/tests/codec_runtime_registration.rs:92-183.
//! * [`ArrayGpuExt`] adds a batched `retrieve_array_subset` for arrays of any supported chain
//!   (unsharded C2/C5-style arrays): all intersecting chunks go to the GPU in one
//!   `zgpu_retrieve_array_subset` call (Array::retrieve_array_subset_into,
//!   array_read_ops_common.rs:20-179).
//!
//! Status codes map onto `CodecError` variants as include/zgpu.h documents.
//!
//! This crate is not compiled in the build container (no Rust toolchain there); its C side is tested
//! from C++ (tests/c/abi_harness.cpp) and Python ctypes.

mod array_ext;
pub mod codecs;
mod ffi;
mod sharding;

use std::collections::HashMap;
use std::ffi::{CStr, CString, c_int, c_void};
use std::ptr::NonNull;
use std::sync::{Arc, LazyLock, Mutex};

use zarrs_codec::{CodecCreateError, CodecError, InvalidBytesLengthError};
use zarrs_data_type::{DataType, FillValue};
use zarrs_plugin::{ExtensionName, ZarrVersion};

pub use array_ext::ArrayGpuExt;
pub use sharding::{GpuShardingCodec, GpuShardingCodecBound};

/// Register the GPU `sharding_indexed` codec plugin. Keep the handle to unregister it.
pub fn register() -> zarrs_codec::CodecRuntimeRegistryHandleV3 {
    zarrs_codec::register_codec_v3(zarrs_codec::CodecRuntimePluginV3::new(
        |name| name == "sharding_indexed",
        GpuShardingCodec::create,
    ))
}

/// Unregister a plugin registered by [`register`].
pub fn unregister(handle: &zarrs_codec::CodecRuntimeRegistryHandleV3) -> bool {
    zarrs_codec::unregister_codec_v3(handle)
}

/// Register the per-codec GPU plugins of the entropy stages worth a per-chunk PCIe round trip
/// (`gzip`, `blosc`: [`codecs::GPU_ENTROPY_CODEC_NAMES`]): one runtime plugin matching their names,
/// zarrs_codec/src/lib.rs:279-318. zarrs' own codecs keep the near-memory-speed stages, and zstd
/// (see [`codecs::GPU_ENTROPY_CODEC_NAMES`] for the measurement; opt in with
/// [`register_codecs_named`]).
pub fn register_codecs() -> zarrs_codec::CodecRuntimeRegistryHandleV3 {
    register_codecs_named(&codecs::GPU_ENTROPY_CODEC_NAMES)
}

/// Register the per-codec GPU plugins of the codecs `names` (a subset of
/// [`codecs::GPU_CODEC_NAMES`]), e.g. `&["gzip", "blosc", "zstd"]`.
pub fn register_codecs_named(names: &'static [&'static str]) -> zarrs_codec::CodecRuntimeRegistryHandleV3 {
    zarrs_codec::register_codec_v3(zarrs_codec::CodecRuntimePluginV3::new(
        move |name| names.contains(&name) && codecs::GPU_CODEC_NAMES.contains(&name),
        codecs::create,
    ))
}

/// Register a per-codec GPU plugin for every stage (`bytes`, `transpose`, `crc32c`, `gzip`, `zstd`,
/// `blosc`, `numcodecs.shuffle`): each stage of zarrs' per-chunk chain then decodes on the GPU, one
/// PCIe round trip per stage.
pub fn register_codecs_all() -> zarrs_codec::CodecRuntimeRegistryHandleV3 {
    zarrs_codec::register_codec_v3(zarrs_codec::CodecRuntimePluginV3::new(
        |name| codecs::GPU_CODEC_NAMES.contains(&name),
        codecs::create,
    ))
}

/// Both: [`register`] and [`register_codecs`] (the handles, for [`unregister`]).
pub fn register_all() -> [zarrs_codec::CodecRuntimeRegistryHandleV3; 2] {
    [register(), register_codecs()]
}

/// The HIP device the plugin decodes on: `ZARRS_GPU_DEVICE` (default 0).
pub(crate) fn device() -> c_int {
    std::env::var("ZARRS_GPU_DEVICE").ok().and_then(|v| v.parse().ok()).unwrap_or(0)
}

/// One zgpu context per HIP device for the life of the process (zgpu.h: thread-safe, calls on one
/// context are serialised internally).
struct Ctx(NonNull<ffi::zgpu_ctx>);
// SAFETY: every zgpu entry point is thread-safe (include/zgpu.h "Threading").
unsafe impl Send for Ctx {}
unsafe impl Sync for Ctx {}

static CONTEXTS: LazyLock<Mutex<HashMap<c_int, Arc<Ctx>>>> = LazyLock::new(|| Mutex::new(HashMap::new()));

fn context(dev: c_int) -> Result<Arc<Ctx>, String> {
    let mut map = CONTEXTS.lock().map_err(|e| e.to_string())?;
    if let Some(c) = map.get(&dev) {
        return Ok(c.clone());
    }
    let mut p: *mut ffi::zgpu_ctx = std::ptr::null_mut();
    // SAFETY: out-pointer to a local; the library fills it on success.
    let rc = unsafe { ffi::zgpu_ctx_create(dev, &mut p) };
    if rc != ffi::ZGPU_OK {
        return Err(format!("zgpu_ctx_create({dev}): {}", last_error()));
    }
    let c = Arc::new(Ctx(NonNull::new(p).ok_or("zgpu_ctx_create returned NULL")?));
    map.insert(dev, c.clone());
    Ok(c)
}

fn last_error() -> String {
    // SAFETY: zgpu_last_error returns a NUL-terminated thread-local string (never NULL).
    unsafe { CStr::from_ptr(ffi::zgpu_last_error(std::ptr::null())) }.to_string_lossy().into_owned()
}

/// A bound codec chain on the GPU (`zgpu_chain`): CodecChain::from_metadata + with_context.
pub(crate) struct Chain {
    ptr: NonNull<ffi::zgpu_chain>,
    _ctx: Arc<Ctx>,
    pub(crate) element_size: usize,
}
// SAFETY: zgpu chains are immutable after creation and every call on them is thread-safe.
unsafe impl Send for Chain {}
unsafe impl Sync for Chain {}

impl std::fmt::Debug for Chain {
    fn fmt(&self, f: &mut std::fmt::Formatter<'_>) -> std::fmt::Result {
        f.debug_struct("zgpu_chain").field("element_size", &self.element_size).finish()
    }
}

impl Drop for Chain {
    fn drop(&mut self) {
        // SAFETY: created by zgpu_chain_create, destroyed once.
        unsafe { ffi::zgpu_chain_destroy(self.ptr.as_ptr()) }
    }
}

impl Chain {
    /// `codecs_json` is the Zarr V3 "codecs" array; the chain is bound to `data_type` / `fill_value`.
    pub(crate) fn new(codecs_json: &str, data_type: &DataType, fill_value: &FillValue) -> Result<Self, CodecCreateError> {
        Self::new_on(codecs_json, data_type, fill_value, device())
    }

    /// As [`Chain::new`], on HIP device `dev` (its process-wide context).
    pub(crate) fn new_on(
        codecs_json: &str,
        data_type: &DataType,
        fill_value: &FillValue,
        dev: c_int,
    ) -> Result<Self, CodecCreateError> {
        let ctx = context(dev).map_err(CodecCreateError::Other)?;
        let name = data_type
            .name(ZarrVersion::V3)
            .ok_or_else(|| CodecCreateError::Other("data type has no Zarr V3 name".into()))?;
        let json = CString::new(codecs_json).map_err(CodecCreateError::other)?;
        let dt = CString::new(name.as_ref()).map_err(CodecCreateError::other)?;
        let fill = fill_value.as_ne_bytes();
        let mut p: *mut ffi::zgpu_chain = std::ptr::null_mut();
        // SAFETY: valid C strings and fill buffer for the duration of the call; out-pointer to a local.
        let rc = unsafe {
            ffi::zgpu_chain_create(
                ctx.0.as_ptr(),
                json.as_ptr(),
                dt.as_ptr(),
                fill.as_ptr().cast(),
                u32::try_from(fill.len()).map_err(CodecCreateError::other)?,
                1,
                &mut p,
            )
        };
        if rc != ffi::ZGPU_OK {
            return Err(CodecCreateError::Other(format!("zgpu_chain_create: {}", last_error())));
        }
        let ptr = NonNull::new(p).ok_or_else(|| CodecCreateError::Other("zgpu_chain_create returned NULL".into()))?;
        // SAFETY: a live chain.
        let element_size = unsafe { ffi::zgpu_chain_element_size(ptr.as_ptr()) } as usize;
        Ok(Self { ptr, _ctx: ctx, element_size })
    }

    pub(crate) fn as_ptr(&self) -> *mut ffi::zgpu_chain {
        self.ptr.as_ptr()
    }

    /// Decode the region `sel_start`/`sel_shape` of one encoded chunk (host bytes) of `chunk_shape`
    /// into a new host buffer holding the region in C order. A region covering the whole chunk takes
    /// the full decode path (checksums verified unless `validate` is false), any other region the
    /// partial-decoder path (crc32c stripped, not verified), as zarrs does.
    pub(crate) fn decode_region(
        &self,
        encoded: &[u8],
        chunk_shape: &[u64],
        sel_start: &[u64],
        sel_shape: &[u64],
        validate: bool,
    ) -> Result<Vec<u8>, CodecError> {
        let nd = chunk_shape.len();
        if nd == 0 || nd > ffi::ZGPU_MAX_DIMS || sel_start.len() != nd || sel_shape.len() != nd {
            return Err(CodecError::Other(format!("zgpu: unsupported dimensionality {nd}")));
        }
        let mut d = ffi::zgpu_chunk_desc {
            enc: encoded.as_ptr().cast(),
            enc_len: encoded.len() as u64,
            ..Default::default()
        };
        d.chunk_shape[..nd].copy_from_slice(chunk_shape);
        d.sel_start[..nd].copy_from_slice(sel_start);
        d.sel_shape[..nd].copy_from_slice(sel_shape);
        // ZGPU_COALESCE: this call joins the other rayon workers' concurrent calls on the chain in one
        // GPU batch (zarrs decodes one shard per worker, array_read_ops_common.rs:173-176); a lone caller
        // does not wait for the collect window (the library sees no other call in flight)
        let flags = ffi::ZGPU_COALESCE | if validate { 0 } else { ffi::ZGPU_NO_VALIDATE };
        Ok(self.decode_pinned(&[d], sel_shape, flags)?.as_slice().to_vec())
    }
}

/// Library-owned pinned bytes handed back by `zgpu_decode_pinned` / `zgpu_encode_pinned` (a coalesced
/// batch's pack buffer or a pooled pinned block). Dropping it returns the block with
/// `zgpu_result_release`, so a pack shared by several callers is recycled once its last holder drops.
pub(crate) struct Pinned {
    ptr: *const u8,
    len: usize,
    res: NonNull<ffi::zgpu_result>,
}

// SAFETY: the bytes are immutable once the call returned, and zgpu_result_release is thread-safe
// (the library counts a pack's holders under its own lock).
unsafe impl Send for Pinned {}
unsafe impl Sync for Pinned {}

impl Pinned {
    /// The result bytes (empty for a zero-length result or a null data pointer).
    pub(crate) fn as_slice(&self) -> &[u8] {
        if self.len == 0 || self.ptr.is_null() {
            return &[];
        }
        // SAFETY: the library guarantees `len` readable bytes at `ptr` until zgpu_result_release.
        unsafe { std::slice::from_raw_parts(self.ptr, self.len) }
    }
}

impl Drop for Pinned {
    fn drop(&mut self) {
        // SAFETY: `res` came from a successful zgpu_*_pinned call and is released exactly once here.
        unsafe { ffi::zgpu_result_release(self.res.as_ptr()) };
    }
}

impl Chain {
    /// zgpu_decode_pinned over `descs` (host encoded bytes): the C-order output of `out_shape` left in
    /// library pinned memory, for ONE copy into the caller's target (a zarrs view can only be written
    /// by `copy_from_slice`, array_bytes_fixed_disjoint_view.rs:177-206). `flags`: ZGPU_NO_VALIDATE
    /// (partial-decoder semantics), ZGPU_COALESCE (join concurrent calls in one GPU batch).
    pub(crate) fn decode_pinned(
        &self,
        descs: &[ffi::zgpu_chunk_desc],
        out_shape: &[u64],
        flags: u32,
    ) -> Result<Pinned, CodecError> {
        let nd = out_shape.len();
        if nd == 0 || nd > ffi::ZGPU_MAX_DIMS {
            return Err(CodecError::Other(format!("zgpu: unsupported dimensionality {nd}")));
        }
        let len = usize::try_from(out_shape.iter().product::<u64>() * self.element_size as u64)
            .map_err(|e| CodecError::Other(e.to_string()))?;
        let mut status = vec![0i32; descs.len().max(1)];
        let mut data: *const c_void = std::ptr::null();
        let mut res: *mut ffi::zgpu_result = std::ptr::null_mut();
        // SAFETY: the descriptors point at host buffers the caller keeps alive for this synchronous call;
        // out-pointers to locals.
        let rc = unsafe {
            ffi::zgpu_decode_pinned(
                self.as_ptr(),
                nd as u32,
                descs.as_ptr(),
                descs.len() as u64,
                out_shape.as_ptr(),
                flags & (ffi::ZGPU_NO_VALIDATE | ffi::ZGPU_COALESCE),
                status.as_mut_ptr(),
                &mut data,
                &mut res,
            )
        };
        if rc != ffi::ZGPU_OK {
            return Err(status_error(rc));
        }
        let res = NonNull::new(res).ok_or_else(|| CodecError::Other("zgpu_decode_pinned returned no result".into()))?;
        Ok(Pinned { ptr: data.cast(), len, res })
    }

    /// zgpu_encode_pinned: one chunk (or shard) of `chunk_shape` from host bytes, encoded on the GPU.
    /// `Ok(None)`: the library's write path does not take this chain (ZGPU_UNSUPPORTED); the caller
    /// falls back to zarrs' own encoder.
    pub(crate) fn encode_pinned(&self, decoded: &[u8], chunk_shape: &[u64]) -> Result<Option<Pinned>, CodecError> {
        let nd = chunk_shape.len();
        let need = chunk_shape.iter().product::<u64>() * self.element_size as u64;
        if nd == 0 || nd > ffi::ZGPU_MAX_DIMS || decoded.len() as u64 != need {
            return Err(CodecError::Other(format!(
                "zgpu encode: {} bytes for a chunk of {chunk_shape:?} ({need} expected)",
                decoded.len()
            )));
        }
        let mut enc: *const c_void = std::ptr::null();
        let mut len = 0u64;
        let mut res: *mut ffi::zgpu_result = std::ptr::null_mut();
        // SAFETY: `decoded` holds the chunk's bytes for this synchronous call; out-pointers to locals.
        let rc = unsafe {
            ffi::zgpu_encode_pinned(self.as_ptr(), nd as u32, chunk_shape.as_ptr(), decoded.as_ptr().cast(), &mut enc,
                                    &mut len, &mut res)
        };
        if rc == ffi::ZGPU_UNSUPPORTED {
            return Ok(None);
        }
        if rc != ffi::ZGPU_OK {
            return Err(status_error(rc));
        }
        let res = NonNull::new(res).ok_or_else(|| CodecError::Other("zgpu_encode_pinned returned no result".into()))?;
        let len = usize::try_from(len).map_err(|e| CodecError::Other(e.to_string()))?;
        Ok(Some(Pinned { ptr: enc.cast(), len, res }))
    }
}

/// Leaf items (chunks / inner chunks) the calling thread's last zgpu call planned (ZGPU_CTR_ITEMS).
pub fn last_call_items() -> u64 {
    let mut c = [0u64; ffi::ZGPU_N_COUNTERS];
    // SAFETY: a buffer of ZGPU_N_COUNTERS values.
    unsafe { ffi::zgpu_last_counters(c.as_mut_ptr(), ffi::ZGPU_N_COUNTERS as u32) };
    c[ffi::ZGPU_CTR_ITEMS]
}

impl Chain {
    /// One `zgpu_decode_batch` call over `descs` (host encoded bytes, host output of shape
    /// `out_shape` in C order): the batched form every per-shard / per-chunk decode of the plugin
    /// uses. `flags` may add ZGPU_NO_VALIDATE (partial-decoder semantics: crc32c stripped, not
    /// verified). Returns the first failing descriptor's status as a [`CodecError`].
    pub(crate) fn decode_descs(
        &self,
        descs: &[ffi::zgpu_chunk_desc],
        out: &mut [u8],
        out_shape: &[u64],
        flags: u32,
    ) -> Result<(), CodecError> {
        let nd = out_shape.len();
        if nd == 0 || nd > ffi::ZGPU_MAX_DIMS {
            return Err(CodecError::Other(format!("zgpu: unsupported dimensionality {nd}")));
        }
        let need = out_shape.iter().product::<u64>() * self.element_size as u64;
        if (out.len() as u64) < need {
            return Err(CodecError::Other("zgpu: output buffer smaller than its shape".into()));
        }
        let mut status = vec![0i32; descs.len().max(1)];
        // SAFETY: the descriptors point at host buffers the caller keeps alive for this synchronous
        // call (flags carry no ZGPU_ENC_DEVICE / ZGPU_OUT_DEVICE), `out` holds the output shape.
        let rc = unsafe {
            ffi::zgpu_decode_batch(
                self.as_ptr(),
                nd as u32,
                descs.as_ptr(),
                descs.len() as u64,
                out.as_mut_ptr().cast::<c_void>(),
                out_shape.as_ptr(),
                flags & (ffi::ZGPU_NO_VALIDATE | ffi::ZGPU_COALESCE),
                status.as_mut_ptr(),
                std::ptr::null_mut(),
            )
        };
        if rc != ffi::ZGPU_OK {
            return Err(status_error(rc));
        }
        Ok(())
    }
}

/// zgpu status -> CodecError (include/zgpu.h; zarrs_codec/src/lib.rs:617-686).
pub(crate) fn status_error(status: c_int) -> CodecError {
    match status {
        ffi::ZGPU_INVALID_CHECKSUM => CodecError::InvalidChecksum,
        ffi::ZGPU_DECODED_SIZE_MISMATCH => {
            let (mut d, mut len, mut expected) = (0u64, 0u64, 0u64);
            // SAFETY: out-pointers to locals.
            if unsafe { ffi::zgpu_last_size_mismatch(&mut d, &mut len, &mut expected) } == 1 {
                let len = if len == u64::MAX { usize::MAX } else { len as usize };
                CodecError::UnexpectedChunkDecodedSize(InvalidBytesLengthError::new(len, expected as usize))
            } else {
                CodecError::Other(last_error())
            }
        }
        ffi::ZGPU_SHARD_INDEX_OOB => {
            CodecError::Other("The shard index references out-of-bounds bytes. The chunk may be corrupted.".into())
        }
        ffi::ZGPU_CORRUPT_STREAM => {
            CodecError::IOError(Arc::new(std::io::Error::new(std::io::ErrorKind::InvalidData, last_error())))
        }
        ffi::ZGPU_CRC_INPUT_TOO_SHORT => CodecError::Other("crc32c decoder expects a 32 bit input".into()),
        ffi::ZGPU_SHARD_TOO_SMALL => {
            CodecError::Other("The encoded shard is smaller than the expected size of its index.".into())
        }
        ffi::ZGPU_SHUFFLE_LENGTH => CodecError::Other(
            "the shuffle codec expects the input byte length to be an integer multiple of the elementsize".into(),
        ),
        _ => {
            // SAFETY: zgpu_status_name returns a static string.
            let name = unsafe { CStr::from_ptr(ffi::zgpu_status_name(status)) }.to_string_lossy();
            CodecError::Other(format!("zgpu {name}: {}", last_error()))
        }
    }
}
