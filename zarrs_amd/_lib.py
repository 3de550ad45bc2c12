"""ctypes binding of libzgpu.so (the C ABI declared in include/zgpu.h).

The product path has no CPU fallback: if the HIP library is missing this module raises, and every
decode runs the gfx950 kernels.
"""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# ZGPU_LIB: an alternative build of the same library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("ZGPU_LIB") or os.path.join(HERE, "lib", "libzgpu.so")
MAX_DIMS = 8

STATUS_NAMES = [
    "OK", "INVALID_CHECKSUM", "DECODED_SIZE_MISMATCH", "SHARD_INDEX_OOB", "CORRUPT_STREAM",
    "INVALID_BYTE_RANGE", "UNSUPPORTED", "CRC_INPUT_TOO_SHORT", "SHARD_TOO_SMALL", "SHUFFLE_LENGTH",
    "INVALID_ARGUMENT", "HIP_ERROR", "STORAGE_ERROR",
]
OK, INVALID_CHECKSUM, DECODED_SIZE_MISMATCH, SHARD_INDEX_OOB, CORRUPT_STREAM, INVALID_BYTE_RANGE, \
    UNSUPPORTED, CRC_INPUT_TOO_SHORT, SHARD_TOO_SMALL, SHUFFLE_LENGTH, INVALID_ARGUMENT, HIP_ERROR, \
    STORAGE_ERROR = range(13)

ENC_DEVICE = 0x1
OUT_DEVICE = 0x2
ONE_STREAM = 0x10
ZSTD_LITS_FIRST = 0x40
NO_VALIDATE = 0x4
DIRECT_IO = 0x8
COALESCE = 0x20
WHOLE = (1 << 64) - 1  # zgpu_file_range.len: to the end of the file

# every symbol include/zgpu.h declares (tests/test_abi.py checks the .so exports all of them)
EXPORTS = [
    "zgpu_ctx_create", "zgpu_ctx_destroy", "zgpu_last_error", "zgpu_status_name", "zgpu_version",
    "zgpu_chain_create", "zgpu_chain_destroy", "zgpu_chain_element_size", "zgpu_decode_batch",
    "zgpu_plan_create", "zgpu_plan_execute", "zgpu_plan_status", "zgpu_plan_destroy", "zgpu_plan_algorithmic_bytes",
    "zgpu_retrieve_array_subset", "zgpu_decode_files", "zgpu_retrieve_array_subset_files",
    "zgpu_chain_encoded_size", "zgpu_encode_batch", "zgpu_plan_counters", "zgpu_last_counters",
    "zgpu_last_size_mismatch", "zgpu_cache_create", "zgpu_cache_destroy", "zgpu_cache_clear", "zgpu_cache_stats",
    "zgpu_cache_retrieve_array_subset", "zgpu_retrieve_array_subset_dlpack", "zgpu_chain_encoded_bound",
    "zgpu_encode_chunks", "zgpu_retrieve_array_subset_multi", "zgpu_decode_into", "zgpu_ctx_set_coalescing",
    "zgpu_ctx_coalescing_stats", "zgpu_ctx_refcount", "zgpu_decode_pinned", "zgpu_result_release",
    "zgpu_encode_pinned", "zgpu_ctx_release_cached", "zgpu_ctx_pool_stats",
    "zgpu_group_create", "zgpu_group_execute", "zgpu_group_status", "zgpu_group_layout",
    "zgpu_group_algorithmic_bytes", "zgpu_group_counters", "zgpu_group_destroy",
]
CTR_ENC_BYTES, CTR_ZSTD_SERIAL, CTR_ZSTD_PARALLEL, CTR_BLOSC_RERUN, CTR_BLOSC_BLOCKS, CTR_ITEMS = range(6)
N_COUNTERS = 6


class ChunkDesc(C.Structure):
    _fields_ = [
        ("enc", C.c_void_p),
        ("enc_len", C.c_uint64),
        ("chunk_shape", C.c_uint64 * MAX_DIMS),
        ("sel_start", C.c_uint64 * MAX_DIMS),
        ("sel_shape", C.c_uint64 * MAX_DIMS),
        ("out_start", C.c_uint64 * MAX_DIMS),
    ]


class OutView(C.Structure):
    """zgpu_out_view: the box [start, start + shape) of a C-order array of array_shape at base."""
    _fields_ = [
        ("base", C.c_void_p),
        ("array_shape", C.c_uint64 * MAX_DIMS),
        ("start", C.c_uint64 * MAX_DIMS),
        ("shape", C.c_uint64 * MAX_DIMS),
    ]


class FileRange(C.Structure):
    _fields_ = [("path", C.c_char_p), ("offset", C.c_uint64), ("len", C.c_uint64)]


class EncodeDesc(C.Structure):
    _fields_ = [("dst", C.c_void_p), ("dst_cap", C.c_uint64), ("chunk_start", C.c_uint64 * MAX_DIMS)]


class DLDevice(C.Structure):
    _fields_ = [("device_type", C.c_int32), ("device_id", C.c_int32)]


class DLDataType(C.Structure):
    _fields_ = [("code", C.c_uint8), ("bits", C.c_uint8), ("lanes", C.c_uint16)]


class DLTensor(C.Structure):
    _fields_ = [("data", C.c_void_p), ("device", DLDevice), ("ndim", C.c_int32), ("dtype", DLDataType),
                ("shape", C.POINTER(C.c_int64)), ("strides", C.POINTER(C.c_int64)), ("byte_offset", C.c_uint64)]


class DLManagedTensor(C.Structure):
    pass


DLManagedTensor._fields_ = [("dl_tensor", DLTensor), ("manager_ctx", C.c_void_p),
                            ("deleter", C.CFUNCTYPE(None, C.POINTER(DLManagedTensor)))]
DL_ROCM = 10


class ZgpuError(RuntimeError):
    """Maps zgpu status codes onto the reference's CodecError variants (zarrs_codec/src/lib.rs:617-686)."""

    def __init__(self, status: int, message: str = ""):
        self.status = status
        name = STATUS_NAMES[status] if 0 <= status < len(STATUS_NAMES) else str(status)
        super().__init__(f"{name}{': ' + message if message and message != name else ''}")


_lib = None


def load() -> C.CDLL:
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError(f"{LIB_PATH} is missing: build it with `make -C zarrs_amd/csrc` "
                          "(or __graft_entry__.build()); there is no CPU fallback")
    L = C.CDLL(LIB_PATH)
    vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
    P64 = C.POINTER(C.c_uint64)
    L.zgpu_ctx_create.argtypes = [i32, C.POINTER(vp)]
    L.zgpu_ctx_destroy.argtypes = [vp]
    L.zgpu_decode_pinned.argtypes = [vp, C.c_uint32, vp, C.c_uint64, vp, C.c_uint32, vp, C.POINTER(C.c_void_p),
                                     C.POINTER(C.c_void_p)]
    L.zgpu_result_release.argtypes = [vp]
    L.zgpu_encode_pinned.argtypes = [vp, C.c_uint32, vp, vp, C.POINTER(C.c_void_p), C.POINTER(C.c_uint64),
                                     C.POINTER(C.c_void_p)]
    L.zgpu_result_release.restype = None
    L.zgpu_ctx_release_cached.argtypes = [vp]
    L.zgpu_ctx_pool_stats.argtypes = [vp, P64, P64, P64, P64]
    L.zgpu_ctx_refcount.argtypes = [vp]
    L.zgpu_ctx_refcount.restype = C.c_int64
    L.zgpu_last_error.restype = C.c_char_p
    L.zgpu_last_error.argtypes = [vp]
    L.zgpu_status_name.restype = C.c_char_p
    L.zgpu_status_name.argtypes = [i32]
    L.zgpu_version.restype = C.c_char_p
    L.zgpu_chain_create.argtypes = [vp, C.c_char_p, C.c_char_p, vp, u32, i32, C.POINTER(vp)]
    L.zgpu_chain_destroy.argtypes = [vp]
    L.zgpu_chain_element_size.restype = u32
    L.zgpu_chain_element_size.argtypes = [vp]
    L.zgpu_decode_batch.argtypes = [vp, u32, C.POINTER(ChunkDesc), u64, vp, P64, u32,
                                    C.POINTER(C.c_int32), vp]
    L.zgpu_decode_into.argtypes = [vp, u32, C.POINTER(ChunkDesc), u64, C.POINTER(OutView), u32,
                                   C.POINTER(C.c_int32), vp]
    L.zgpu_ctx_set_coalescing.argtypes = [vp, u32, u32, u64]
    L.zgpu_ctx_coalescing_stats.argtypes = [vp, P64, P64]
    L.zgpu_plan_create.argtypes = [vp, u32, C.POINTER(ChunkDesc), u64, P64, u32, C.POINTER(vp)]
    L.zgpu_plan_execute.argtypes = [vp, vp, C.POINTER(C.c_int32), vp]
    L.zgpu_plan_status.argtypes = [vp, C.POINTER(C.c_int32), vp]
    L.zgpu_plan_destroy.argtypes = [vp]
    L.zgpu_plan_algorithmic_bytes.restype = u64
    L.zgpu_plan_algorithmic_bytes.argtypes = [vp]
    L.zgpu_group_create.argtypes = [C.POINTER(vp), u32, u32, C.POINTER(C.POINTER(ChunkDesc)), P64, C.POINTER(P64),
                                    u32, C.POINTER(vp)]
    L.zgpu_group_execute.argtypes = [vp, C.POINTER(vp), C.POINTER(C.c_int32), vp]
    L.zgpu_group_status.argtypes = [vp, C.POINTER(C.c_int32), vp]
    L.zgpu_group_layout.restype = u32
    L.zgpu_group_layout.argtypes = [vp, C.POINTER(u32), C.POINTER(u32), C.POINTER(u32), u32]
    L.zgpu_group_algorithmic_bytes.restype = u64
    L.zgpu_group_algorithmic_bytes.argtypes = [vp]
    L.zgpu_group_counters.restype = u32
    L.zgpu_group_counters.argtypes = [vp, P64, u32]
    L.zgpu_group_destroy.argtypes = [vp]
    L.zgpu_retrieve_array_subset.argtypes = [vp, u32, P64, P64, C.POINTER(vp), P64, P64, P64, vp,
                                             u32, vp]
    L.zgpu_decode_files.argtypes = [vp, u32, C.POINTER(ChunkDesc), C.POINTER(FileRange), u64, vp, P64,
                                    u32, C.POINTER(C.c_int32), vp]
    L.zgpu_retrieve_array_subset_files.argtypes = [vp, u32, P64, P64, C.POINTER(C.c_char_p), P64, P64,
                                                   vp, u32, vp]
    L.zgpu_chain_encoded_size.restype = C.c_int64
    L.zgpu_chain_encoded_size.argtypes = [vp, u32, P64]
    L.zgpu_encode_batch.argtypes = [vp, u32, P64, vp, P64, C.POINTER(EncodeDesc), u64, u32, vp]
    L.zgpu_chain_encoded_bound.restype = C.c_int64
    L.zgpu_chain_encoded_bound.argtypes = [vp, u32, P64]
    L.zgpu_encode_chunks.argtypes = [vp, u32, P64, vp, P64, C.POINTER(EncodeDesc), u64, u32, P64, vp]
    L.zgpu_retrieve_array_subset_multi.argtypes = [C.POINTER(vp), u32, u32, P64, P64, C.POINTER(vp), P64, P64, P64,
                                                   vp, u32]
    L.zgpu_plan_counters.restype = u32
    L.zgpu_plan_counters.argtypes = [vp, P64, u32]
    L.zgpu_last_counters.restype = u32
    L.zgpu_last_counters.argtypes = [P64, u32]
    L.zgpu_last_size_mismatch.argtypes = [P64, P64, P64]
    L.zgpu_cache_create.argtypes = [vp, u64, C.POINTER(vp)]
    L.zgpu_cache_destroy.argtypes = [vp]
    L.zgpu_cache_clear.argtypes = [vp]
    L.zgpu_cache_stats.argtypes = [vp, P64, P64, P64, P64]
    L.zgpu_cache_retrieve_array_subset.argtypes = [vp, vp, u32, P64, P64, C.POINTER(vp), P64, P64, P64, vp, u32, vp]
    L.zgpu_retrieve_array_subset_dlpack.argtypes = [vp, vp, u32, P64, P64, C.POINTER(vp), P64, P64, P64, u32, vp,
                                                    C.POINTER(C.POINTER(DLManagedTensor))]
    _lib = L
    return L


def last_error() -> str:
    return (load().zgpu_last_error(None) or b"").decode()


def last_counters() -> dict:
    """Device counters of this thread's last decode call (zgpu_last_counters)."""
    buf = (C.c_uint64 * N_COUNTERS)()
    load().zgpu_last_counters(buf, N_COUNTERS)
    return {"enc_bytes": buf[0], "zstd_serial": buf[1], "zstd_parallel": buf[2], "blosc_rerun": buf[3],
            "blosc_blocks": buf[4]}


def last_size_mismatch():
    """(descriptor, len, expected_len) of the last DECODED_SIZE_MISMATCH, or None; len None when a
    decompressor overflowed the expected size (InvalidBytesLengthError, zarrs_codec/src/lib.rs:491)."""
    d, n, e = C.c_uint64(), C.c_uint64(), C.c_uint64()
    if not load().zgpu_last_size_mismatch(C.byref(d), C.byref(n), C.byref(e)):
        return None
    return d.value, (None if n.value == (1 << 64) - 1 else n.value), e.value


def check(status: int) -> None:
    if status:
        raise ZgpuError(status, last_error())


def u64s(vals, n=None):
    vals = [int(v) for v in vals]
    return (C.c_uint64 * (n or max(len(vals), 1)))(*vals)
