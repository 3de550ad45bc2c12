"""Host-side mirror of the zarrs codec API for the GPU chunk-decode path.

Names and argument meaning follow the reference so the parity tests read like zarrs' own:
  CodecChain.from_metadata  <- CodecChain::from_metadata + with_context (codec_chain.rs:105-229)
  CodecChain.decode         <- CodecChainBound::decode (codec_chain.rs:557-590)
  CodecChain.decode_into    <- CodecChainBound::decode_into (codec_chain.rs:592-646)
  CodecChain.partial_decode <- partial_decoder(..).partial_decode (codec_chain.rs:684-745)
  CodecChain.decode_batch   <- the batched GPU entry point (zgpu_decode_batch)
Errors raise ZgpuError whose .status maps 1:1 onto CodecError variants (see include/zgpu.h).
Every call runs the gfx950 kernels in libzgpu.so; there is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import json
import math
from typing import Sequence

import numpy as np

from . import _lib as L

DTYPES = {
    "bool": "|b1", "int8": "<i1", "uint8": "<u1", "int16": "<i2", "uint16": "<u2", "float16": "<f2",
    "int32": "<i4", "uint32": "<u4", "float32": "<f4", "int64": "<i8", "uint64": "<u8",
    "float64": "<f8", "complex64": "<c8", "complex128": "<c16",
}


def fill_value_bytes(data_type: str, fill) -> bytes:
    """FillValue::as_ne_bytes for the core numeric data types (fill value metadata decoding)."""
    if isinstance(fill, (bytes, bytearray)):
        return bytes(fill)
    dt = np.dtype(DTYPES[data_type])
    if isinstance(fill, str):
        special = {"NaN": math.nan, "Infinity": math.inf, "-Infinity": -math.inf}
        if fill in special:
            fill = special[fill]
        elif fill.startswith("0x"):
            return int(fill, 16).to_bytes(dt.itemsize, "little")
    if isinstance(fill, (list, tuple)):
        return np.array(complex(fill[0], fill[1]), dtype=dt).tobytes()
    return np.array(fill, dtype=dt).tobytes()


class Context:
    """One decode context per GPU (zgpu_ctx): a HIP stream plus cached device scratch."""

    _default = {}

    def __init__(self, device: int = 0):
        lib = L.load()
        h = C.c_void_p()
        L.check(lib.zgpu_ctx_create(int(device), C.byref(h)))
        self._h = h
        self.device = device

    @classmethod
    def default(cls, device: int = 0) -> "Context":
        if device not in cls._default:
            cls._default[device] = cls(device)
        return cls._default[device]

    def set_coalescing(self, window_us: int = 200, max_calls: int = 8, max_bytes: int = 1 << 30):
        """Collect window / batch caps of ZGPU_COALESCE calls on this context (zgpu_ctx_set_coalescing)."""
        L.check(L.load().zgpu_ctx_set_coalescing(self._h, int(window_us), int(max_calls), int(max_bytes)))

    def coalescing_stats(self) -> dict:
        b, c = C.c_uint64(), C.c_uint64()
        L.check(L.load().zgpu_ctx_coalescing_stats(self._h, C.byref(b), C.byref(c)))
        return {"batches": b.value, "calls": c.value}

    def refcount(self) -> int:
        """References the library holds on this context: 1 (this handle) + its live chains, plans and
        caches (zgpu_ctx_refcount); 0 once closed."""
        return int(L.load().zgpu_ctx_refcount(self._h)) if getattr(self, "_h", None) else 0

    def release_cached(self):
        """Return the context's cached free device / pinned buffers to HIP (zgpu_ctx_release_cached)."""
        if getattr(self, "_h", None):
            L.check(L.load().zgpu_ctx_release_cached(self._h))

    def pool_stats(self) -> dict:
        """The context's pooled memory in bytes (zgpu_ctx_pool_stats): device blocks in use / cached
        free, pinned host blocks in use / cached free."""
        v = [C.c_uint64() for _ in range(4)]
        L.check(L.load().zgpu_ctx_pool_stats(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("dev_live", "dev_free", "host_live", "host_free"), (x.value for x in v)))

    def close(self):
        """Drop this handle's reference (zgpu_ctx_destroy). Chains, plans and caches made on the
        context keep it alive until they are destroyed too, in any order."""
        if getattr(self, "_h", None):
            L.load().zgpu_ctx_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def _ptr_len(buf):
    """(address, byte length, is_device, keepalive) of bytes / numpy / torch buffers."""
    if buf is None:
        return None, 0, False, None
    try:
        import torch
        if isinstance(buf, torch.Tensor):
            return buf.data_ptr(), buf.numel() * buf.element_size(), buf.is_cuda, buf
    except ImportError:  # pragma: no cover
        pass
    if isinstance(buf, np.ndarray):
        return buf.ctypes.data, buf.nbytes, False, buf
    b = bytes(buf)
    cb = C.create_string_buffer(b, max(len(b), 1))
    return C.addressof(cb), len(b), False, cb


def default_stream(stream, *bufs):
    """The HIP stream a call runs on: the caller's, else torch's current stream of the first device
    tensor among bufs (so the decode is ordered after the kernels that produced its inputs). A NULL
    stream (torch's default stream) makes the library order its own stream after the legacy default
    stream (zgpu.h)."""
    if stream is not None:
        return stream
    try:
        import torch
    except ImportError:  # pragma: no cover
        return None
    for b in bufs:
        if isinstance(b, torch.Tensor) and b.is_cuda:
            return torch.cuda.current_stream(b.device).cuda_stream or None
    return None


def make_desc(enc, chunk_shape, sel_start=None, sel_shape=None, out_start=None) -> L.ChunkDesc:
    nd = len(chunk_shape)
    d = L.ChunkDesc()
    if isinstance(enc, tuple):
        d.enc, d.enc_len = enc
    else:
        p, n, _, keep = _ptr_len(enc)
        d.enc, d.enc_len = p, n
        d._keep = keep  # the descriptor keeps its buffer alive
    sel_start = sel_start if sel_start is not None else [0] * nd
    sel_shape = sel_shape if sel_shape is not None else chunk_shape
    out_start = out_start if out_start is not None else [0] * nd
    for i in range(nd):
        d.chunk_shape[i] = int(chunk_shape[i])
        d.sel_start[i] = int(sel_start[i])
        d.sel_shape[i] = int(sel_shape[i])
        d.out_start[i] = int(out_start[i])
    return d


class CodecChain:
    """A bound codec chain on the GPU (zgpu_chain)."""

    def __init__(self, handle, ctx: Context, codecs, data_type: str):
        self._h = handle
        self.ctx = ctx
        self.codecs = codecs
        self.data_type = data_type
        self.dtype = np.dtype(DTYPES[data_type])

    @classmethod
    def from_metadata(cls, codecs, data_type: str, fill_value=0, ctx: Context | None = None,
                      validate_checksums: bool = True) -> "CodecChain":
        ctx = ctx or Context.default()
        if not isinstance(codecs, str):
            codecs = json.dumps(codecs)
        fill = fill_value_bytes(data_type, fill_value)
        h = C.c_void_p()
        L.check(L.load().zgpu_chain_create(ctx._h, codecs.encode(), data_type.encode(), fill,
                                           len(fill), 1 if validate_checksums else 0, C.byref(h)))
        return cls(h, ctx, json.loads(codecs), data_type)

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                L.load().zgpu_chain_destroy(self._h)
                self._h = None
        except Exception:
            pass

    # ---- batched entry point -------------------------------------------------------------
    def decode_batch(self, descs: Sequence[L.ChunkDesc], out, out_shape, enc_device: bool,
                     validate_checksums: bool | None = None, stream=None, flags: int = 0) -> list:
        """Decode many chunks into `out` (numpy array or torch tensor); returns per-chunk statuses
        and raises ZgpuError with the first failing status (try_for_each semantics). `flags`: extra
        ZGPU_* decode flags (e.g. ONE_STREAM | ZSTD_LITS_FIRST)."""
        n = len(descs)
        arr = (L.ChunkDesc * max(n, 1))(*descs)
        arr._keep = [getattr(d, "_keep", None) for d in descs]
        st = (C.c_int32 * max(n, 1))()
        op, _, odev, _ = _ptr_len(out)
        flags |= (L.ENC_DEVICE if enc_device else 0) | (L.OUT_DEVICE if odev else 0)
        if validate_checksums is False:
            flags |= L.NO_VALIDATE
        stream = default_stream(stream, out, *[getattr(d, "_keep", None) for d in descs])
        rc = L.load().zgpu_decode_batch(self._h, len(out_shape), arr, n, op, L.u64s(out_shape),
                                        flags, st, stream)
        statuses = [st[i] for i in range(n)]
        if rc:
            raise L.ZgpuError(rc, L.last_error())
        return statuses

    def decode_batch_into(self, descs: Sequence[L.ChunkDesc], array, view_start, view_shape, enc_device: bool,
                          validate_checksums: bool | None = None, coalesce: bool = False, stream=None) -> list:
        """decode_into a window of a larger array (ArrayBytesFixedDisjointView; zgpu_decode_into):
        `array` is the whole C-order output (numpy array or torch tensor), the window the box
        [view_start, view_start + view_shape); descriptors' out_start are relative to the window.
        coalesce: ZGPU_COALESCE (concurrent host-in/host-out calls share one GPU batch)."""
        n = len(descs)
        arr = (L.ChunkDesc * max(n, 1))(*descs)
        arr._keep = [getattr(d, "_keep", None) for d in descs]
        st = (C.c_int32 * max(n, 1))()
        op, _, odev, _ = _ptr_len(array)
        v = L.OutView()
        v.base = op
        for d, (a, s0, s1) in enumerate(zip(array.shape, view_start, view_shape)):
            v.array_shape[d], v.start[d], v.shape[d] = int(a), int(s0), int(s1)
        flags = (L.ENC_DEVICE if enc_device else 0) | (L.OUT_DEVICE if odev else 0) | (L.COALESCE if coalesce else 0)
        if validate_checksums is False:
            flags |= L.NO_VALIDATE
        stream = default_stream(stream, array, *[getattr(d, "_keep", None) for d in descs])
        rc = L.load().zgpu_decode_into(self._h, len(view_shape), arr, n, C.byref(v), flags, st, stream)
        statuses = [st[i] for i in range(n)]
        if rc:
            raise L.ZgpuError(rc, L.last_error())
        return statuses

    def decode_pinned_into(self, descs: Sequence[L.ChunkDesc], array: np.ndarray, view_start, view_shape,
                           validate_checksums: bool | None = None, coalesce: bool = False) -> list:
        """The codec plugin's decode_into (rust/zarrs_gpu): host inputs decoded by zgpu_decode_pinned into
        library-owned pinned memory, then ONE copy of the compact window into the caller's view
        (ArrayBytesFixedDisjointView::copy_from_slice, array_bytes_fixed_disjoint_view.rs:177-206; here
        a numpy slice assignment), then zgpu_result_release. Descriptors' out_start are window-relative."""
        n = len(descs)
        arr = (L.ChunkDesc * max(n, 1))(*descs)
        arr._keep = [getattr(d, "_keep", None) for d in descs]
        st = (C.c_int32 * max(n, 1))()
        flags = (L.COALESCE if coalesce else 0) | (L.NO_VALIDATE if validate_checksums is False else 0)
        data, res = C.c_void_p(), C.c_void_p()
        lib = L.load()
        rc = lib.zgpu_decode_pinned(self._h, len(view_shape), arr, n, L.u64s(view_shape), flags, st, C.byref(data),
                                    C.byref(res))
        statuses = [st[i] for i in range(n)]
        if rc:
            raise L.ZgpuError(rc, L.last_error())
        try:
            count = int(np.prod(view_shape))
            src = np.ctypeslib.as_array((C.c_uint8 * (count * self.dtype.itemsize)).from_address(data.value))
            win = tuple(slice(int(a), int(a) + int(b)) for a, b in zip(view_start, view_shape))
            array[win] = src.view(array.dtype).reshape([int(x) for x in view_shape])
        finally:
            lib.zgpu_result_release(res)
        return statuses

    # ---- per-chunk forms (degenerate batches) ------------------------------------------------
    def decode(self, encoded, shape) -> np.ndarray:
        out = np.empty([int(s) for s in shape], dtype=self.dtype)
        self.decode_into(encoded, shape, out)
        return out

    def decode_into(self, encoded, shape, out, out_start=None):
        dev = _ptr_len(encoded)[2]
        self.decode_batch([make_desc(encoded, shape, out_start=out_start)], out, list(out.shape), dev)

    def encoded_size(self, chunk_shape) -> int:
        """Encoded bytes of one chunk (fixed-size chains), -1 if variable (zgpu_chain_encoded_size)."""
        return int(L.load().zgpu_chain_encoded_size(self._h, len(chunk_shape), L.u64s(chunk_shape)))

    def encoded_bound(self, chunk_shape) -> int:
        """Upper bound of one chunk's encoded size (zgpu_chain_encoded_bound), -1 if unbounded."""
        return int(L.load().zgpu_chain_encoded_bound(self._h, len(chunk_shape), L.u64s(chunk_shape)))

    def encode_chunks(self, array, chunk_shape, chunk_starts, stream=None) -> list:
        """CodecChain::encode of the chunks of a device-resident torch array whose origins are
        chunk_starts (zgpu_encode_chunks; sharding_indexed over a fixed-size inner chain included).
        Returns one uint8 device tensor per chunk."""
        import torch
        assert array.is_cuda and array.is_contiguous()
        if array.numel() * array.element_size() != int(np.prod(array.shape)) * self.dtype.itemsize or \
                array.element_size() != self.dtype.itemsize:
            raise L.ZgpuError(L.INVALID_ARGUMENT, f"encode: {array.dtype} tensor for a {self.data_type} chain")
        size = self.encoded_bound(chunk_shape)
        if size < 0:
            raise L.ZgpuError(L.UNSUPPORTED, "encode: the chain's encoded size is not bounded")
        n = len(chunk_starts)
        flat = torch.empty(max(n, 1) * ((size + 255) // 256 * 256), dtype=torch.uint8, device=array.device)
        pitch = (size + 255) // 256 * 256
        descs = (L.EncodeDesc * max(n, 1))()
        for i, st in enumerate(chunk_starts):
            descs[i].dst = flat.data_ptr() + i * pitch
            descs[i].dst_cap = size
            for d, v in enumerate(st):
                descs[i].chunk_start[d] = int(v)
        stream = default_stream(stream, array)
        lens = (C.c_uint64 * max(n, 1))()
        rc = L.load().zgpu_encode_chunks(self._h, len(chunk_shape), L.u64s(chunk_shape), array.data_ptr(),
                                        L.u64s(list(array.shape)), descs, n, L.ENC_DEVICE | L.OUT_DEVICE, lens,
                                        stream)
        L.check(rc)
        return [flat[i * pitch:i * pitch + lens[i]] for i in range(n)]

    def partial_decode(self, encoded, shape, subset_start, subset_shape) -> np.ndarray:
        out = np.empty([int(s) for s in subset_shape], dtype=self.dtype)
        dev = _ptr_len(encoded)[2]
        self.decode_batch([make_desc(encoded, shape, subset_start, subset_shape)], out,
                          list(subset_shape), dev)
        return out


class PlanGroup:
    """zgpu_group: independent parts of one batch (each part one chunk shape and one output, e.g. the
    levels of a multiscale pyramid) decoded by one call; the library lays the parts out on streams of
    its own and picks each plan's literals-first order (group.cpp). `parts`: (chain, descs,
    out_shape) per part, descriptors with device-resident encoded bytes; `execute(outs)` decodes part
    p into outs[p] (device tensors) behind `stream` (default: torch's current stream of outs[0])."""

    def __init__(self, parts, flags: int = 0):
        lib = L.load()
        self.n_parts = len(parts)
        self.chains = [c for c, _, _ in parts]
        nd = len(parts[0][2])
        self._arrs = [(L.ChunkDesc * max(len(d), 1))(*d) for _, d, _ in parts]
        self.n_descs = [len(d) for _, d, _ in parts]
        chains = (C.c_void_p * self.n_parts)(*[c._h for c in self.chains])
        dptrs = (C.POINTER(L.ChunkDesc) * self.n_parts)(*[C.cast(a, C.POINTER(L.ChunkDesc)) for a in self._arrs])
        ns = (C.c_uint64 * self.n_parts)(*self.n_descs)
        self._shapes = [L.u64s(s) for _, _, s in parts]
        shp = (C.POINTER(C.c_uint64) * self.n_parts)(*[C.cast(s, C.POINTER(C.c_uint64)) for s in self._shapes])
        h = C.c_void_p()
        L.check(lib.zgpu_group_create(chains, nd, self.n_parts, dptrs, ns, shp,
                                      flags | L.ENC_DEVICE | L.OUT_DEVICE, C.byref(h)))
        self._h = h
        self.status = (C.c_int32 * max(1, sum(self.n_descs)))()

    def layout(self) -> list:
        """[(lane, part, literals_first)] of the group's plans."""
        lib = L.load()
        n = lib.zgpu_group_layout(self._h, None, None, None, 0)
        lane, part, lf = (C.c_uint32 * max(n, 1))(), (C.c_uint32 * max(n, 1))(), (C.c_uint32 * max(n, 1))()
        lib.zgpu_group_layout(self._h, lane, part, lf, n)
        return [(lane[i], part[i], bool(lf[i])) for i in range(n)]

    def algorithmic_bytes(self) -> int:
        return int(L.load().zgpu_group_algorithmic_bytes(self._h))

    def counters(self) -> list:
        buf = (C.c_uint64 * L.N_COUNTERS)()
        n = L.load().zgpu_group_counters(self._h, buf, L.N_COUNTERS)
        return list(buf[:n])

    def execute(self, outs, stream=None, wait: bool = True) -> list | None:
        """Enqueue the decode; with wait, read back the per-descriptor statuses (concatenated in part
        order) and raise ZgpuError with the first failing one."""
        lib = L.load()
        ptrs = (C.c_void_p * self.n_parts)(*[_ptr_len(o)[0] for o in outs])
        s = default_stream(stream, *outs)
        L.check(lib.zgpu_group_execute(self._h, ptrs, self.status if wait else None, s))
        return list(self.status[: sum(self.n_descs)]) if wait else None

    def wait(self, stream=None) -> list:
        L.check(L.load().zgpu_group_status(self._h, self.status, stream))
        return list(self.status[: sum(self.n_descs)])

    def close(self):
        if getattr(self, "_h", None):
            L.load().zgpu_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
