//! Raw bindings of include/zgpu.h (the C ABI of libzgpu.so). Keep in step with the header.
#![allow(non_camel_case_types)]

use std::ffi::{c_char, c_int, c_void};

pub const ZGPU_MAX_DIMS: usize = 8;

pub const ZGPU_OK: c_int = 0;
pub const ZGPU_INVALID_CHECKSUM: c_int = 1;
pub const ZGPU_DECODED_SIZE_MISMATCH: c_int = 2;
pub const ZGPU_SHARD_INDEX_OOB: c_int = 3;
pub const ZGPU_CORRUPT_STREAM: c_int = 4;
pub const ZGPU_INVALID_BYTE_RANGE: c_int = 5;
pub const ZGPU_UNSUPPORTED: c_int = 6;
pub const ZGPU_CRC_INPUT_TOO_SHORT: c_int = 7;
pub const ZGPU_SHARD_TOO_SMALL: c_int = 8;
pub const ZGPU_SHUFFLE_LENGTH: c_int = 9;
pub const ZGPU_INVALID_ARGUMENT: c_int = 10;
pub const ZGPU_HIP_ERROR: c_int = 11;
pub const ZGPU_STORAGE_ERROR: c_int = 12;

pub const ZGPU_ENC_DEVICE: u32 = 0x1;
pub const ZGPU_OUT_DEVICE: u32 = 0x2;
pub const ZGPU_NO_VALIDATE: u32 = 0x4;
pub const ZGPU_DIRECT_IO: u32 = 0x8;
/// Every kernel of the call on the caller's stream (no internal side stream).
pub const ZGPU_ONE_STREAM: u32 = 0x10;
/// With ZGPU_ONE_STREAM: a zstd stage decodes its literals before its sequences (zgpu.h).
pub const ZGPU_ZSTD_LITS_FIRST: u32 = 0x40;
/// Concurrent host-in/host-out calls on one chain share one GPU batch (zgpu.h ZGPU_COALESCE).
pub const ZGPU_COALESCE: u32 = 0x20;

#[repr(C)]
pub struct zgpu_ctx {
    _opaque: [u8; 0],
}
#[repr(C)]
pub struct zgpu_chain {
    _opaque: [u8; 0],
}
/// Library-owned pinned bytes of zgpu_decode_pinned / zgpu_encode_pinned (released by
/// zgpu_result_release).
#[repr(C)]
pub struct zgpu_result {
    _opaque: [u8; 0],
}
/// A plan group (`zgpu_group_create`): the independent parts of one batch decoded by one call.
#[repr(C)]
pub struct zgpu_group {
    _opaque: [u8; 0],
}

/// zgpu_last_counters index: leaf items (chunks / inner chunks) the calling thread's last call planned.
pub const ZGPU_CTR_ITEMS: usize = 5;
pub const ZGPU_N_COUNTERS: usize = 6;

/// zgpu_encode_desc: one chunk of a device-resident array encoded into `dst`.
#[repr(C)]
#[derive(Clone, Copy)]
pub struct zgpu_encode_desc {
    pub dst: *mut c_void,
    pub dst_cap: u64,
    pub chunk_start: [u64; ZGPU_MAX_DIMS],
}

#[repr(C)]
#[derive(Clone, Copy)]
pub struct zgpu_chunk_desc {
    pub enc: *const c_void,
    pub enc_len: u64,
    pub chunk_shape: [u64; ZGPU_MAX_DIMS],
    pub sel_start: [u64; ZGPU_MAX_DIMS],
    pub sel_shape: [u64; ZGPU_MAX_DIMS],
    pub out_start: [u64; ZGPU_MAX_DIMS],
}

impl Default for zgpu_chunk_desc {
    fn default() -> Self {
        Self {
            enc: std::ptr::null(),
            enc_len: 0,
            chunk_shape: [0; ZGPU_MAX_DIMS],
            sel_start: [0; ZGPU_MAX_DIMS],
            sel_shape: [0; ZGPU_MAX_DIMS],
            out_start: [0; ZGPU_MAX_DIMS],
        }
    }
}

/// zgpu_out_view: the box [start, start + shape) of a C-order array of array_shape at base.
#[repr(C)]
#[derive(Clone, Copy)]
pub struct zgpu_out_view {
    pub base: *mut c_void,
    pub array_shape: [u64; ZGPU_MAX_DIMS],
    pub start: [u64; ZGPU_MAX_DIMS],
    pub shape: [u64; ZGPU_MAX_DIMS],
}

unsafe extern "C" {
    pub fn zgpu_ctx_create(hip_device: c_int, out: *mut *mut zgpu_ctx) -> c_int;
    pub fn zgpu_ctx_destroy(ctx: *mut zgpu_ctx);
    pub fn zgpu_last_error(ctx: *const zgpu_ctx) -> *const c_char;
    pub fn zgpu_status_name(status: c_int) -> *const c_char;
    pub fn zgpu_chain_create(
        ctx: *mut zgpu_ctx,
        codecs_json: *const c_char,
        data_type: *const c_char,
        fill: *const c_void,
        fill_len: u32,
        validate_checksums: c_int,
        out: *mut *mut zgpu_chain,
    ) -> c_int;
    pub fn zgpu_chain_destroy(chain: *mut zgpu_chain);
    pub fn zgpu_chain_element_size(chain: *const zgpu_chain) -> u32;
    pub fn zgpu_decode_batch(
        chain: *mut zgpu_chain,
        ndim: u32,
        descs: *const zgpu_chunk_desc,
        n: u64,
        out: *mut c_void,
        out_shape: *const u64,
        flags: u32,
        status: *mut i32,
        hip_stream: *mut c_void,
    ) -> c_int;
    pub fn zgpu_decode_into(
        chain: *mut zgpu_chain,
        ndim: u32,
        descs: *const zgpu_chunk_desc,
        n: u64,
        view: *const zgpu_out_view,
        flags: u32,
        status: *mut i32,
        hip_stream: *mut c_void,
    ) -> c_int;
    pub fn zgpu_ctx_set_coalescing(ctx: *mut zgpu_ctx, window_us: u32, max_calls: u32, max_bytes: u64) -> c_int;
    pub fn zgpu_retrieve_array_subset(
        chain: *mut zgpu_chain,
        ndim: u32,
        array_shape: *const u64,
        chunk_shape: *const u64,
        chunk_ptrs: *const *const c_void,
        chunk_lens: *const u64,
        sel_start: *const u64,
        sel_shape: *const u64,
        out: *mut c_void,
        flags: u32,
        hip_stream: *mut c_void,
    ) -> c_int;
    pub fn zgpu_last_size_mismatch(desc: *mut u64, len: *mut u64, expected_len: *mut u64) -> c_int;
    pub fn zgpu_last_counters(out: *mut u64, n: u32) -> u32;
    pub fn zgpu_decode_pinned(
        chain: *mut zgpu_chain,
        ndim: u32,
        descs: *const zgpu_chunk_desc,
        n: u64,
        out_shape: *const u64,
        flags: u32,
        status: *mut i32,
        data: *mut *const c_void,
        result: *mut *mut zgpu_result,
    ) -> c_int;
    pub fn zgpu_encode_pinned(
        chain: *mut zgpu_chain,
        ndim: u32,
        chunk_shape: *const u64,
        decoded: *const c_void,
        enc: *mut *const c_void,
        enc_len: *mut u64,
        result: *mut *mut zgpu_result,
    ) -> c_int;
    pub fn zgpu_result_release(result: *mut zgpu_result);
    pub fn zgpu_group_create(
        chains: *const *mut zgpu_chain,
        ndim: u32,
        n_parts: u32,
        descs: *const *const zgpu_chunk_desc,
        n_descs: *const u64,
        out_shapes: *const *const u64,
        flags: u32,
        out: *mut *mut zgpu_group,
    ) -> c_int;
    pub fn zgpu_group_execute(
        group: *mut zgpu_group,
        outs: *const *mut c_void,
        status: *mut i32,
        hip_stream: *mut c_void,
    ) -> c_int;
    pub fn zgpu_group_status(group: *mut zgpu_group, status: *mut i32, hip_stream: *mut c_void) -> c_int;
    pub fn zgpu_group_destroy(group: *mut zgpu_group);
    pub fn zgpu_retrieve_array_subset_multi(
        chains: *const *mut zgpu_chain,
        n_dev: u32,
        ndim: u32,
        array_shape: *const u64,
        chunk_shape: *const u64,
        chunk_ptrs: *const *const c_void,
        chunk_lens: *const u64,
        sel_start: *const u64,
        sel_shape: *const u64,
        out: *mut c_void,
        flags: u32,
    ) -> c_int;
}
