"""CPU oracle for the zarrs chunk-decode path — TEST INFRASTRUCTURE ONLY.

ctypes front-end over ``oracle/build/liborc.so`` (a C restatement of zarrs' codec pipeline,
see ``oracle/zarrs_oracle.c`` for the per-function reference citations). Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import this module,
and only as the checker / the timed CPU baseline: the product path (``zarrs_amd``) never
calls it.

``OracleChain.from_metadata`` mirrors ``CodecChain::from_metadata``
(zarrs/src/array/codec/array_to_bytes/codec_chain.rs:192-229): the JSON ``codecs`` list is
split into array->array, exactly one array->bytes, and bytes->bytes codecs.
"""
from __future__ import annotations

import ctypes as C
import json
import math
import os
import struct
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liborc.so")
_lib = None

STATUS_NAMES = [
    "OK", "INVALID_CHECKSUM", "DECODED_SIZE_MISMATCH", "SHARD_INDEX_OOB", "CORRUPT_STREAM",
    "INVALID_BYTE_RANGE", "UNSUPPORTED", "CRC_INPUT_TOO_SHORT", "SHARD_TOO_SMALL",
    "SHUFFLE_LENGTH", "INVALID_ARGUMENT",
]

# zarr V3 core data types: name -> (numpy dtype, component size)
DTYPES = {
    "bool": ("|b1", 1), "int8": ("<i1", 1), "uint8": ("<u1", 1),
    "int16": ("<i2", 2), "uint16": ("<u2", 2), "float16": ("<f2", 2),
    "int32": ("<i4", 4), "uint32": ("<u4", 4), "float32": ("<f4", 4),
    "int64": ("<i8", 8), "uint64": ("<u8", 8), "float64": ("<f8", 8),
    "complex64": ("<c8", 4), "complex128": ("<c16", 8),
}


class OracleError(RuntimeError):
    def __init__(self, status: int, what: str = ""):
        self.status = status
        super().__init__(f"{STATUS_NAMES[status] if 0 <= status < len(STATUS_NAMES) else status}"
                         f"{': ' + what if what else ''}")


def build(force: bool = False) -> str:
    """Compile the oracle with its own Makefile (gcc, no GPU)."""
    if force or not os.path.exists(_LIB_PATH):
        subprocess.check_call(["make", "-s", "-C", _HERE])
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(_LIB_PATH)
        vp, u32, u64, i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int
        P64 = C.POINTER(C.c_uint64)
        L.orc_chain_new.restype = vp
        L.orc_chain_new.argtypes = [u32, u32, vp]
        L.orc_chain_free.argtypes = [vp]
        L.orc_chain_add_transpose.argtypes = [vp, u32, C.POINTER(C.c_uint32)]
        L.orc_chain_add_bytes.argtypes = [vp, i32]
        L.orc_chain_add_sharding.argtypes = [vp, u32, P64, vp, vp, i32]
        L.orc_chain_add_crc32c.argtypes = [vp, i32]
        L.orc_chain_add_gzip.argtypes = [vp, i32]
        L.orc_chain_add_zstd.argtypes = [vp, i32, i32]
        L.orc_chain_add_shuffle.argtypes = [vp, u32]
        L.orc_chain_add_blosc.argtypes = [vp, C.c_char_p, i32, i32, u32, C.c_uint64]
        L.orc_decode_chunk.argtypes = [vp, vp, u64, u32, P64, i32, vp]
        L.orc_encode_chunk.argtypes = [vp, vp, u32, P64, C.POINTER(vp), P64]
        L.orc_free.argtypes = [vp]
        L.orc_retrieve_array_subset.argtypes = [vp, u32, P64, P64, C.POINTER(vp), P64, P64, P64,
                                                vp, i32, i32]
        L.orc_crc32c.restype = u32
        L.orc_crc32c.argtypes = [u32, vp, u64]
        L.orc_crc32_ieee.restype = u32
        L.orc_crc32_ieee.argtypes = [vp, u64]
        _lib = L
    return _lib


def _u64(vals):
    return (C.c_uint64 * max(len(vals), 1))(*[int(v) for v in vals])


def crc32c(data: bytes) -> int:
    b = bytes(data)
    return lib().orc_crc32c(0, b, len(b))


def fill_value_bytes(data_type: str, fill) -> bytes:
    """Native-endian fill value bytes (FillValue::as_ne_bytes) for the core numeric types."""
    dt = np.dtype(DTYPES[data_type][0])
    if isinstance(fill, str):
        special = {"NaN": math.nan, "Infinity": math.inf, "-Infinity": -math.inf}
        if fill in special:
            fill = special[fill]
        elif fill.startswith("0x"):
            return int(fill, 16).to_bytes(dt.itemsize, "little")
    if isinstance(fill, list):  # complex
        return np.array(complex(fill[0], fill[1]), dtype=dt).tobytes()
    return np.array(fill, dtype=dt).tobytes()


class OracleChain:
    """A bound codec chain on the CPU (owns the C handle)."""

    def __init__(self, handle, data_type: str, ndim: int):
        self._h = handle
        self.data_type = data_type
        self.ndim = ndim
        self.dtype = np.dtype(DTYPES[data_type][0])

    def __del__(self):
        if getattr(self, "_h", None) and _lib is not None:
            _lib.orc_chain_free(self._h)
            self._h = None

    A2A = ("transpose",)
    A2B = ("bytes", "endian", "sharding_indexed")
    B2B = ("crc32c", "numcodecs.crc32c", "gzip", "zstd", "numcodecs.zstd", "blosc", "numcodecs.blosc",
           "numcodecs.shuffle", "shuffle")

    @staticmethod
    def _sorted(codecs):
        """CodecChain::from_metadata (codec_chain.rs:192-229): entries sorted by kind (array->array,
        array->bytes, bytes->bytes; metadata order within a kind); an entry whose codec cannot be
        created is skipped if it has "must_understand": false (:197-206). Codec names this restatement
        does not know are the "cannot be created" case."""
        a2a, a2b, b2b = [], [], []
        for m in codecs:
            if isinstance(m, str):
                m = {"name": m}
            name = m["name"]
            if name in OracleChain.A2A:
                a2a.append(m)
            elif name in OracleChain.A2B:
                a2b.append(m)
            elif name in OracleChain.B2B:
                b2b.append(m)
            elif m.get("must_understand", True):
                raise OracleError(6, f"codec {name}")
        if len(a2b) != 1:
            raise OracleError(10, "exactly one array->bytes codec")
        return a2a + a2b + b2b

    @staticmethod
    def _build(codecs, data_type: str, fill: bytes, ndim: int):
        L = lib()
        np_dt, comp = DTYPES[data_type]
        es = np.dtype(np_dt).itemsize
        codecs = OracleChain._sorted(codecs)
        h = L.orc_chain_new(es, comp, fill)
        if not h:
            raise OracleError(10, "bad data type")
        for m in codecs:
            name, cfg = m["name"], m.get("configuration", {}) or {}
            if name == "transpose":
                order = cfg["order"]
                st = L.orc_chain_add_transpose(h, len(order), (C.c_uint32 * len(order))(*order))
            elif name in ("bytes", "endian"):
                st = L.orc_chain_add_bytes(h, 1 if cfg.get("endian", "little") == "big" else 0)
            elif name == "sharding_indexed":
                inner_shape = cfg["chunk_shape"]
                inner = OracleChain._build(cfg["codecs"], data_type, fill, ndim)
                idx = OracleChain._build(cfg.get("index_codecs", [
                    {"name": "bytes", "configuration": {"endian": "little"}},
                    {"name": "crc32c"}]), "uint64", b"\xff" * 8, ndim + 1)
                st = L.orc_chain_add_sharding(h, len(inner_shape), _u64(inner_shape), inner, idx,
                                              1 if cfg.get("index_location", "end") == "start" else 0)
            elif name in ("crc32c", "numcodecs.crc32c"):
                st = L.orc_chain_add_crc32c(h, 1 if cfg.get("location", "end") == "start" else 0)
            elif name == "gzip":
                st = L.orc_chain_add_gzip(h, int(cfg.get("level", 5)))
            elif name in ("zstd", "numcodecs.zstd"):
                st = L.orc_chain_add_zstd(h, int(cfg.get("level", 0)), 1 if cfg.get("checksum") else 0)
            elif name in ("blosc", "numcodecs.blosc"):
                sh = {"noshuffle": 0, "shuffle": 1, "bitshuffle": 2}[cfg.get("shuffle", "noshuffle")]
                st = L.orc_chain_add_blosc(h, cfg.get("cname", "lz4").encode(), int(cfg.get("clevel", 5)), sh,
                                           int(cfg.get("typesize") or 0), int(cfg.get("blocksize") or 0))
            elif name in ("numcodecs.shuffle", "shuffle"):
                st = L.orc_chain_add_shuffle(h, int(cfg.get("elementsize", 4)))
            else:
                L.orc_chain_free(h)
                raise OracleError(6, f"codec {name}")
            if st:
                L.orc_chain_free(h)
                raise OracleError(st, f"adding {name}")
        return h

    @classmethod
    def from_metadata(cls, codecs, data_type: str, fill_value=0, ndim: int = 1):
        if isinstance(codecs, str):
            codecs = json.loads(codecs)
        fill = fill_value if isinstance(fill_value, bytes) else fill_value_bytes(data_type, fill_value)
        return cls(cls._build(codecs, data_type, fill, ndim), data_type, ndim)

    def decode(self, encoded: bytes, shape, validate_checksums: bool = True) -> np.ndarray:
        shape = [int(s) for s in shape]
        out = np.empty(shape, dtype=self.dtype)
        enc = bytes(encoded)
        st = lib().orc_decode_chunk(self._h, enc, len(enc), len(shape), _u64(shape),
                                    1 if validate_checksums else 0, out.ctypes.data)
        if st:
            raise OracleError(st)
        return out

    def encode(self, array: np.ndarray) -> bytes:
        a = np.ascontiguousarray(array, dtype=self.dtype)
        p, n = C.c_void_p(), C.c_uint64()
        st = lib().orc_encode_chunk(self._h, a.ctypes.data, a.ndim, _u64(a.shape), C.byref(p),
                                    C.byref(n))
        if st:
            raise OracleError(st)
        try:
            return C.string_at(p.value, n.value)
        finally:
            lib().orc_free(p)


def retrieve_array_subset(chain: OracleChain, array_shape, chunk_shape, chunks: dict,
                          sel_start, sel_shape, nthreads: int = 1, validate_checksums: bool = True,
                          out: np.ndarray | None = None) -> np.ndarray:
    """Array::retrieve_array_subset on a dict {chunk grid index tuple: encoded bytes}."""
    nd = len(array_shape)
    grid = [-(-int(a) // int(c)) for a, c in zip(array_shape, chunk_shape)]
    n = int(np.prod(grid))
    ptrs = (C.c_void_p * n)()
    lens = (C.c_uint64 * n)()
    keep = []
    for idx, enc in chunks.items():
        lin = int(np.ravel_multi_index(tuple(idx), grid))
        b = C.create_string_buffer(bytes(enc), len(enc)) if len(enc) else C.create_string_buffer(1)
        keep.append(b)
        ptrs[lin] = C.cast(b, C.c_void_p)
        lens[lin] = len(enc)
    if out is None:
        out = np.empty([int(s) for s in sel_shape], dtype=chain.dtype)
    st = lib().orc_retrieve_array_subset(chain._h, nd, _u64(array_shape), _u64(chunk_shape), ptrs,
                                         lens, _u64(sel_start), _u64(sel_shape), out.ctypes.data,
                                         nthreads, 1 if validate_checksums else 0)
    if st:
        raise OracleError(st)
    return out


def retrieve_ptrs(chain: OracleChain, array_shape, chunk_shape, ptrs, lens, sel_start, sel_shape,
                  out: np.ndarray, nthreads: int, validate_checksums: bool = True) -> None:
    """Low-level form with caller-built pointer tables (bench cpu_baseline leg)."""
    st = lib().orc_retrieve_array_subset(chain._h, len(array_shape), _u64(array_shape),
                                         _u64(chunk_shape), ptrs, lens, _u64(sel_start),
                                         _u64(sel_shape), out.ctypes.data, nthreads,
                                         1 if validate_checksums else 0)
    if st:
        raise OracleError(st)


def unpack_u64_le(b: bytes):
    return list(struct.unpack("<%dQ" % (len(b) // 8), b))
