//! Array-level batched read for any chain the GPU pipeline supports (unsharded arrays included):
//! Array::retrieve_array_subset_into (zarrs/src/array/array_ops/array_read_ops_common.rs:20-179) with
//! every intersecting chunk decoded in ONE zgpu_retrieve_array_subset call instead of a rayon loop of
//! per-chunk CodecChain decodes. Per-codec plugins cannot fuse a chain across codecs or batch across
//! chunks; this extension does both, and is how unsharded arrays (e.g. transpose + big-endian bytes,
//! or bytes + shuffle + zstd) reach the GPU.

use std::ffi::c_void;

use zarrs::array::{Array, ArrayError, ArraySubset};
use zarrs_codec::CodecError;
use zarrs_metadata::ArrayMetadata;
use zarrs_storage::ReadableStorageTraits;

use crate::{Chain, ffi, status_error};

/// GPU reads of a Zarr V3 array with a regular chunk grid (other grids are refused with a
/// CodecError; zarrs' own read path handles them).
pub trait ArrayGpuExt {
    /// Decode `subset` on the GPU into a new host buffer (C order, native-endian element bytes).
    ///
    /// # Errors
    /// Returns [`ArrayError`] on storage errors, unsupported chains or decode failures (the first
    /// failing chunk's status, zarrs' try_for_each semantics).
    fn retrieve_array_subset_gpu(&self, subset: &ArraySubset) -> Result<Vec<u8>, ArrayError>;

    /// Decode `subset` on the GPU into device memory (`out` holds the subset in C order).
    ///
    /// # Safety
    /// `out` must be a device allocation of at least `subset.num_elements() * element size` bytes on
    /// the plugin's device (`ZARRS_GPU_DEVICE`), not accessed by anything else until the call returns;
    /// `hip_stream` is a HIP stream of that device or null.
    unsafe fn retrieve_array_subset_gpu_into_device(
        &self,
        subset: &ArraySubset,
        out: *mut c_void,
        hip_stream: *mut c_void,
    ) -> Result<(), ArrayError>;

    /// Decode `subset` on several GPUs of this process (`devices`, HIP ordinals) into a new host
    /// buffer: the subset's axis-0 chunk rows are cut into one contiguous group per device and every
    /// device writes its rows straight into place (`zgpu_retrieve_array_subset_multi`).
    ///
    /// # Errors
    /// Returns [`ArrayError`] as [`ArrayGpuExt::retrieve_array_subset_gpu`] does.
    fn retrieve_array_subset_gpu_multi(&self, subset: &ArraySubset, devices: &[i32]) -> Result<Vec<u8>, ArrayError>;
}

fn gpu_chain<TStorage: ?Sized + ReadableStorageTraits + 'static>(array: &Array<TStorage>) -> Result<Chain, ArrayError> {
    gpu_chain_on(array, crate::device())
}

fn gpu_chain_on<TStorage: ?Sized + ReadableStorageTraits + 'static>(
    array: &Array<TStorage>,
    device: std::ffi::c_int,
) -> Result<Chain, ArrayError> {
    let ArrayMetadata::V3(meta) = array.metadata() else {
        return Err(CodecError::Other("zarrs_gpu: Zarr V2 arrays are read through the CPU path".into()).into());
    };
    // the batched read lays chunks out on a regular grid (zarrs/src/array/chunk_grid/regular.rs); the
    // rectangular / rectilinear / regular_bounded / repeat grids go through zarrs' own read path
    if meta.chunk_grid.name() != "regular" {
        return Err(CodecError::Other(format!(
            "zarrs_gpu: chunk grid '{}' is not regular: read it through Array::retrieve_array_subset",
            meta.chunk_grid.name()
        ))
        .into());
    }
    let json = serde_json::to_string(&meta.codecs).map_err(|e| CodecError::Other(e.to_string()))?;
    Chain::new_on(&json, array.data_type(), array.fill_value(), device)
        .map_err(|e| CodecError::Other(e.to_string()).into())
}

/// The encoded chunks a subset touches, as (pointer, length) tables over the whole chunk grid
/// (C-order linear grid index; NULL = missing key = fill value), and the regular chunk shape.
fn gpu_tables<TStorage: ?Sized + ReadableStorageTraits + 'static>(
    array: &Array<TStorage>,
    subset: &ArraySubset,
) -> Result<(Vec<u64>, Vec<Vec<u8>>, Vec<u64>), ArrayError> {
    let nd = array.dimensionality();
    let chunk_shape: Vec<u64> = array.chunk_shape(&vec![0; nd])?.iter().map(|c| c.get()).collect();
    let grid: Vec<u64> = array.chunk_grid_shape().to_vec();
    let start = subset.start();
    let shape = subset.shape();
    let mut bufs = Vec::new();
    let mut lins = Vec::new();
    if shape.iter().all(|&n| n > 0) {
        let lo: Vec<u64> = start.iter().zip(&chunk_shape).map(|(s, c)| s / c).collect();
        let hi: Vec<u64> = start.iter().zip(shape.iter()).zip(&chunk_shape).map(|((s, n), c)| (s + n - 1) / c + 1).collect();
        let mut idx = lo.clone();
        loop {
            if let Some(b) = array.retrieve_encoded_chunk(&idx)? {
                let lin = idx.iter().zip(&grid).fold(0u64, |acc, (i, g)| acc * g + i);
                lins.push(lin);
                bufs.push(b);
            }
            let mut d = nd;
            while d > 0 {
                d -= 1;
                idx[d] += 1;
                if idx[d] < hi[d] {
                    break;
                }
                idx[d] = lo[d];
                if d == 0 {
                    return Ok((chunk_shape, bufs, lins));
                }
            }
        }
    }
    Ok((chunk_shape, bufs, lins))
}

/// # Safety
/// `out` is a host buffer (flags without ZGPU_OUT_DEVICE) or a device buffer of the subset's size.
unsafe fn gpu_retrieve<TStorage: ?Sized + ReadableStorageTraits + 'static>(
    array: &Array<TStorage>,
    subset: &ArraySubset,
    out: *mut c_void,
    flags: u32,
    stream: *mut c_void,
) -> Result<(), ArrayError> {
    let nd = array.dimensionality();
    if nd == 0 || nd > ffi::ZGPU_MAX_DIMS {
        return Err(CodecError::Other(format!("zarrs_gpu: unsupported dimensionality {nd}")).into());
    }
    let chain = gpu_chain(array)?;
    let (chunk_shape, bufs, lins) = gpu_tables(array, subset)?;
    let n_grid: u64 = array.chunk_grid_shape().iter().product();
    let n_grid = usize::try_from(n_grid).map_err(|e| CodecError::Other(e.to_string()))?;
    // an empty object is present (not missing): it gets a valid address
    let (ptrs, lens) = grid_tables(n_grid, &bufs, &lins);
    let (start, shape) = (subset.start(), subset.shape());
    // SAFETY: the tables, shapes and host chunk buffers outlive the synchronous call; `out` is the
    // caller's (host buffer, or a device buffer per this function's contract).
    let rc = unsafe {
        ffi::zgpu_retrieve_array_subset(
            chain.as_ptr(),
            nd as u32,
            array.shape().as_ptr(),
            chunk_shape.as_ptr(),
            ptrs.as_ptr(),
            lens.as_ptr(),
            start.as_ptr(),
            shape.as_ptr(),
            out,
            flags,
            stream,
        )
    };
    if rc != ffi::ZGPU_OK {
        return Err(status_error(rc).into());
    }
    Ok(())
}

static EMPTY: [u8; 1] = [0];

/// The pointer tables of [`gpu_retrieve`] over the whole chunk grid (NULL = missing chunk).
fn grid_tables(n_grid: usize, bufs: &[Vec<u8>], lins: &[u64]) -> (Vec<*const c_void>, Vec<u64>) {
    let mut ptrs: Vec<*const c_void> = vec![std::ptr::null(); n_grid];
    let mut lens = vec![0u64; n_grid];
    for (b, &lin) in bufs.iter().zip(lins) {
        ptrs[lin as usize] = if b.is_empty() { EMPTY.as_ptr().cast() } else { b.as_ptr().cast() };
        lens[lin as usize] = b.len() as u64;
    }
    (ptrs, lens)
}

impl<TStorage: ?Sized + ReadableStorageTraits + 'static> ArrayGpuExt for Array<TStorage> {
    fn retrieve_array_subset_gpu(&self, subset: &ArraySubset) -> Result<Vec<u8>, ArrayError> {
        let es = self
            .data_type()
            .fixed_size()
            .ok_or_else(|| CodecError::Other("zarrs_gpu: fixed-size data types only".into()))?;
        let n = usize::try_from(subset.num_elements()).map_err(|e| CodecError::Other(e.to_string()))?;
        let mut out = vec![0u8; n * es];
        // SAFETY: host output buffer of the subset's size; no device flags.
        unsafe { gpu_retrieve(self, subset, out.as_mut_ptr().cast(), 0, std::ptr::null_mut())? };
        Ok(out)
    }

    unsafe fn retrieve_array_subset_gpu_into_device(
        &self,
        subset: &ArraySubset,
        out: *mut c_void,
        hip_stream: *mut c_void,
    ) -> Result<(), ArrayError> {
        // SAFETY: forwarded from this function's contract.
        unsafe { gpu_retrieve(self, subset, out, ffi::ZGPU_OUT_DEVICE, hip_stream) }
    }

    fn retrieve_array_subset_gpu_multi(&self, subset: &ArraySubset, devices: &[i32]) -> Result<Vec<u8>, ArrayError> {
        let nd = self.dimensionality();
        if nd == 0 || nd > ffi::ZGPU_MAX_DIMS || devices.is_empty() {
            return Err(CodecError::Other("zarrs_gpu: unsupported dimensionality or no devices".into()).into());
        }
        let chains = devices.iter().map(|&d| gpu_chain_on(self, d)).collect::<Result<Vec<Chain>, ArrayError>>()?;
        let handles: Vec<*mut ffi::zgpu_chain> = chains.iter().map(Chain::as_ptr).collect();
        let es = self
            .data_type()
            .fixed_size()
            .ok_or_else(|| CodecError::Other("zarrs_gpu: fixed-size data types only".into()))?;
        let n = usize::try_from(subset.num_elements()).map_err(|e| CodecError::Other(e.to_string()))?;
        let mut out = vec![0u8; n * es];
        let (chunk_shape, bufs, lins) = gpu_tables(self, subset)?;
        let n_grid: u64 = self.chunk_grid_shape().iter().product();
        let n_grid = usize::try_from(n_grid).map_err(|e| CodecError::Other(e.to_string()))?;
        let (ptrs, lens) = grid_tables(n_grid, &bufs, &lins);
        let (start, shape) = (subset.start(), subset.shape());
        // SAFETY: tables, shapes, host chunk buffers and the host output outlive the synchronous call.
        let rc = unsafe {
            ffi::zgpu_retrieve_array_subset_multi(
                handles.as_ptr(),
                u32::try_from(handles.len()).map_err(|e| CodecError::Other(e.to_string()))?,
                nd as u32,
                self.shape().as_ptr(),
                chunk_shape.as_ptr(),
                ptrs.as_ptr(),
                lens.as_ptr(),
                start.as_ptr(),
                shape.as_ptr(),
                out.as_mut_ptr().cast(),
                0,
            )
        };
        if rc != ffi::ZGPU_OK {
            return Err(status_error(rc).into());
        }
        Ok(out)
    }
}
