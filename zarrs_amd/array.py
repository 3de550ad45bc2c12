"""Array-level read path mirror: Array / MemoryStore / DeviceStore over the GPU codec pipeline.

  Array.retrieve_array_subset  <- Array::retrieve_array_subset (array_read_ops_array.rs:74-154,
                                  array_read_ops_common.rs:20-179): subset -> intersecting chunks ->
                                  one batched GPU decode (full chunks: decode_into with checksum
                                  verification; partial chunks: partial decoder semantics)
  Array.retrieve_chunk         <- Array::retrieve_chunk (array_read_ops_array.rs:265-272)
  MemoryStore                  <- zarrs_storage MemoryStore (encoded chunks in host memory)
  DeviceStore                  <- encoded chunks resident in HBM (torch uint8 tensors)
  FilesystemStore              <- zarrs_filesystem FilesystemStore (zarrs_filesystem/src/lib.rs):
                                  key_to_fspath (:173-179), get / get_partial_many (:323-470);
                                  Array reads it through zgpu_retrieve_array_subset_files (chunk
                                  files read by host threads into pinned staging, overlapped with
                                  the H2D copy and decode of the previous sub-batch)
Chunk keys use the default encoding "c/i/j/k" (chunk_key_encoding/default.rs:79-102) or v2 "i.j".
"""
from __future__ import annotations

import ctypes as C
import itertools
import json

import numpy as np

from . import _lib as L
from .codec import CodecChain, Context, default_stream


class MemoryStore(dict):
    """key -> encoded bytes (host memory)."""
    device = False


class DeviceStore(dict):
    """key -> torch.uint8 device tensor (HBM-resident encoded bytes)."""
    device = True

    @classmethod
    def from_store(cls, store, device="cuda"):
        import torch
        d = cls()
        for k, v in store.items():
            d[k] = torch.frombuffer(bytearray(v), dtype=torch.uint8).to(device) if len(v) else \
                torch.empty(0, dtype=torch.uint8, device=device)
        return d


class FilesystemStore:
    """A directory of Zarr keys. ``direct_io`` mirrors FilesystemStoreOptions::direct_io
    (zarrs_filesystem/src/lib.rs:74-77): O_DIRECT page reads (buffered where unsupported)."""
    device = False

    def __init__(self, base_path, direct_io: bool = False):
        import os
        self.base_path = os.fspath(base_path)
        self.direct_io = direct_io

    def key_to_fspath(self, key: str) -> str:
        import os
        return os.path.join(self.base_path, key.lstrip("/")) if key else self.base_path

    def get(self, key: str):
        try:
            with open(self.key_to_fspath(key), "rb") as f:
                return f.read()
        except (FileNotFoundError, NotADirectoryError):
            return None

    def __getitem__(self, key):
        v = self.get(key)
        if v is None:
            raise KeyError(key)
        return v

    def __contains__(self, key):
        import os
        return os.path.isfile(self.key_to_fspath(key))

    def set(self, key: str, value: bytes) -> None:
        import os
        path = self.key_to_fspath(key)
        os.makedirs(os.path.dirname(path), exist_ok=True)
        with open(path, "wb") as f:
            f.write(value)

    __setitem__ = set

    def decode_files(self, chain, descs, ranges, out, out_shape, status=None):
        """zgpu_decode_files: descs (ChunkDesc array) with their (key, offset, length) ranges
        (length None = to the end of the file)."""
        n = len(ranges)
        fr = (L.FileRange * max(n, 1))()
        keep = []
        for i, (key, off, ln) in enumerate(ranges):
            p = None if key is None else self.key_to_fspath(key).encode()
            keep.append(p)
            fr[i].path, fr[i].offset, fr[i].len = p, int(off), L.WHOLE if ln is None else int(ln)
        odev, op = _out_ptr(out)
        st = (C.c_int32 * max(n, 1))()
        flags = (L.OUT_DEVICE if odev else 0) | (L.DIRECT_IO if self.direct_io else 0)
        rc = L.load().zgpu_decode_files(chain._h, len(out_shape), descs, fr, n, op, L.u64s(out_shape),
                                        flags, st, None)
        if status is not None:
            status[:] = list(st)[:n]
        return rc, list(st)[:n]


def _out_ptr(out):
    try:
        import torch
        if isinstance(out, torch.Tensor):
            return out.is_cuda, out.data_ptr()
    except ImportError:  # pragma: no cover
        pass
    return False, out.ctypes.data


class Array:
    def __init__(self, store, metadata: dict, ctx: Context | None = None,
                 validate_checksums: bool = True):
        if isinstance(metadata, str):
            metadata = json.loads(metadata)
        self.store = store
        self.metadata = metadata
        self.shape = [int(s) for s in metadata["shape"]]
        grid = metadata["chunk_grid"]
        if grid.get("name") != "regular":
            # the batched read plans one regular grid (zarrs/src/array/chunk_grid/regular.rs); the
            # rectangular / rectilinear / regular_bounded grids would place chunks wrongly
            raise L.ZgpuError(L.UNSUPPORTED, f"chunk grid {grid.get('name')!r}: only 'regular' grids are supported")
        self.chunk_shape = [int(c) for c in grid["configuration"]["chunk_shape"]]
        self.data_type = metadata["data_type"]
        kenc = metadata.get("chunk_key_encoding", {"name": "default"})
        cfg = kenc.get("configuration", {}) or {}
        if kenc["name"] == "default":
            self._sep, self._prefix = cfg.get("separator", "/"), "c" + cfg.get("separator", "/")
        else:
            self._sep, self._prefix = cfg.get("separator", "."), ""
        self._validate = validate_checksums
        self.codecs = CodecChain.from_metadata(metadata["codecs"], self.data_type,
                                               metadata.get("fill_value", 0), ctx,
                                               validate_checksums)
        self.dtype = self.codecs.dtype

    @property
    def ndim(self):
        return len(self.shape)

    def chunk_key(self, idx) -> str:
        return self._prefix + self._sep.join(str(int(i)) for i in idx)

    def chunk_grid_shape(self):
        return [-(-s // c) for s, c in zip(self.shape, self.chunk_shape)]

    def _tables(self, start, shape):
        """Pointer tables indexed by the C-order linear chunk-grid index; only the chunks the subset
        intersects are looked up in the store (chunks_in_array_subset, array_ops_array.rs:341-346),
        the others stay NULL. Host bytes are passed zero-copy."""
        grid = self.chunk_grid_shape()
        n = int(np.prod(grid))
        ptrs = (C.c_void_p * n)()
        lens = (C.c_uint64 * n)()
        keep = []
        if any(int(s) == 0 for s in shape):
            return ptrs, lens, keep
        ranges = [range(int(st) // c, (int(st) + int(sh) - 1) // c + 1)
                  for st, sh, c in zip(start, shape, self.chunk_shape)]
        for idx in itertools.product(*ranges):
            v = self.store.get(self.chunk_key(idx))
            if v is None:
                continue
            lin = int(np.ravel_multi_index(idx, grid))
            if self.store.device:
                ptrs[lin] = v.data_ptr() if v.numel() else None
                lens[lin] = v.numel()
                keep.append(v)
                if not v.numel():  # an empty object is still present: give it a valid address
                    import torch
                    t = torch.empty(1, dtype=torch.uint8, device=v.device)
                    keep.append(t)
                    ptrs[lin] = t.data_ptr()
            else:
                b = np.frombuffer(v, dtype=np.uint8) if len(v) else np.zeros(1, np.uint8)
                keep.append(b)
                ptrs[lin] = b.ctypes.data
                lens[lin] = len(v)
        return ptrs, lens, keep

    def retrieve_array_subset_into(self, start, shape, out) -> None:
        if isinstance(self.store, FilesystemStore):
            grid = self.chunk_grid_shape()
            n = int(np.prod(grid))
            paths = (C.c_char_p * n)()
            for lin in range(n):
                paths[lin] = self.store.key_to_fspath(self.chunk_key(np.unravel_index(lin, grid))).encode()
            odev, op = _out_ptr(out)
            flags = (L.OUT_DEVICE if odev else 0) | (L.DIRECT_IO if self.store.direct_io else 0)
            rc = L.load().zgpu_retrieve_array_subset_files(
                self.codecs._h, self.ndim, L.u64s(self.shape), L.u64s(self.chunk_shape), paths,
                L.u64s(start), L.u64s(shape), op, flags, default_stream(None, out))
            L.check(rc)
            return
        ptrs, lens, keep = self._tables(start, shape)
        try:
            import torch
            odev = isinstance(out, torch.Tensor) and out.is_cuda
            op = out.data_ptr() if isinstance(out, torch.Tensor) else out.ctypes.data
        except ImportError:  # pragma: no cover
            odev, op = False, out.ctypes.data
        flags = (L.ENC_DEVICE if self.store.device else 0) | (L.OUT_DEVICE if odev else 0)
        rc = L.load().zgpu_retrieve_array_subset(
            self.codecs._h, self.ndim, L.u64s(self.shape), L.u64s(self.chunk_shape), ptrs, lens,
            L.u64s(start), L.u64s(shape), op, flags, default_stream(None, out, *keep))
        del keep
        L.check(rc)

    @property
    def read_chunk_shape(self):
        """The decode granule: a sharded array's inner chunk shape (sharding_indexed's chunk_shape), else
        its chunk shape."""
        c0 = self.metadata["codecs"][0] if self.metadata.get("codecs") else {}
        if c0.get("name") == "sharding_indexed":
            return [int(c) for c in c0["configuration"]["chunk_shape"]]
        return list(self.chunk_shape)

    def retrieve_boxes_into(self, boxes, out, origin) -> None:
        """Several boxes of the array decoded as ONE batch (one plan: every box's chunks in one launch per
        stage) into `out`, whose first element is array coordinate `origin`; elements of `out` outside
        the boxes are not written. A distributed rank's share (chunk_line_partition's <= 3 boxes) decodes
        in one latency instead of one per box. Stores read by path (FilesystemStore) take one
        retrieve_array_subset_into per box."""
        from .codec import make_desc
        boxes = [([int(a) for a in b0], [int(n) for n in bs]) for b0, bs in boxes]
        boxes = [(b0, bs) for b0, bs in boxes if all(n > 0 for n in bs)]
        if not boxes:
            return
        if isinstance(self.store, FilesystemStore):
            for b0, bs in boxes:
                v = out[tuple(slice(a - o, a - o + n) for a, o, n in zip(b0, origin, bs))]
                self.retrieve_array_subset_into(b0, bs, v)
            return
        descs, keep = [], []
        for b0, bs in boxes:
            ranges = [range(a // c, (a + n - 1) // c + 1) for a, n, c in zip(b0, bs, self.chunk_shape)]
            for idx in itertools.product(*ranges):
                org = [i * c for i, c in zip(idx, self.chunk_shape)]
                s0 = [max(a, o) for a, o in zip(b0, org)]
                s1 = [min(a + n, o + c) for a, n, o, c in zip(b0, bs, org, self.chunk_shape)]
                v = self.store.get(self.chunk_key(idx))
                if v is None:
                    enc = (0, 0)
                elif self.store.device:
                    keep.append(v)
                    enc = (v.data_ptr(), v.numel())
                    if not v.numel():  # an empty object is still present: give it a valid address (_tables)
                        import torch
                        t = torch.empty(1, dtype=torch.uint8, device=v.device)
                        keep.append(t)
                        enc = (t.data_ptr(), 0)
                else:
                    b = np.frombuffer(v, dtype=np.uint8) if len(v) else np.zeros(1, np.uint8)
                    keep.append(b)
                    enc = (b.ctypes.data, len(v))
                descs.append(make_desc(enc, self.chunk_shape, sel_start=[a - o for a, o in zip(s0, org)],
                                       sel_shape=[e - a for a, e in zip(s0, s1)],
                                       out_start=[a - o for a, o in zip(s0, origin)]))
        self.codecs.decode_batch(descs, out, list(out.shape), enc_device=bool(self.store.device),
                                 validate_checksums=self._validate)
        del keep

    def retrieve_array_subset_multi(self, start, shape, out, contexts) -> None:
        """The subset decoded by several GPUs of this process (zgpu_retrieve_array_subset_multi): one
        chain per context in `contexts`, the subset's axis-0 chunk rows cut into one contiguous group
        per device; a device `out` lives on contexts[0]'s device and receives the other devices'
        rows peer-to-peer. Host-resident stores only (each device uploads its own chunks)."""
        if self.store.device:
            raise ValueError("multi-device reads take host-resident encoded chunks")
        chains = [self.codecs if c is self.codecs.ctx else
                  CodecChain.from_metadata(self.metadata["codecs"], self.data_type,
                                           self.metadata.get("fill_value", 0), c, self._validate)
                  for c in contexts]
        hs = (C.c_void_p * len(chains))(*[ch._h.value for ch in chains])
        ptrs, lens, keep = self._tables(start, shape)
        odev, op = _out_ptr(out)
        if odev:
            import torch
            torch.cuda.synchronize(out.device)  # the call has no stream: order torch's work first
        rc = L.load().zgpu_retrieve_array_subset_multi(
            hs, len(chains), self.ndim, L.u64s(self.shape), L.u64s(self.chunk_shape), ptrs, lens,
            L.u64s(start), L.u64s(shape), op, L.OUT_DEVICE if odev else 0)
        del keep, chains
        L.check(rc)

    def retrieve_array_subset_dlpack(self, start=None, shape=None, cache=None):
        """The subset decoded into HBM and handed over zero-copy as a DLPack kDLROCM tensor
        (zgpu_retrieve_array_subset_dlpack; the reference's DLPack export, array_dlpack_ext.rs:44-70,
        is CPU-only). Returns a torch tensor on the context's device that owns the library's buffer.
        `cache`: an optional ChunkCacheDecodedLruSizeLimit. Encoded chunks from any store but the
        filesystem one."""
        import torch
        start = [0] * self.ndim if start is None else [int(v) for v in start]
        shape = list(self.shape) if shape is None else [int(v) for v in shape]
        ptrs, lens, keep = self._tables(start, shape)
        flags = L.ENC_DEVICE if self.store.device else 0
        mt = C.POINTER(L.DLManagedTensor)()
        rc = L.load().zgpu_retrieve_array_subset_dlpack(
            cache._h if cache is not None else None, self.codecs._h, self.ndim, L.u64s(self.shape),
            L.u64s(self.chunk_shape), ptrs, lens, L.u64s(start), L.u64s(shape), flags,
            default_stream(None, *keep), C.byref(mt))
        del keep
        L.check(rc)
        new_capsule = C.pythonapi.PyCapsule_New
        new_capsule.restype = C.py_object
        new_capsule.argtypes = [C.c_void_p, C.c_char_p, C.c_void_p]
        return torch.utils.dlpack.from_dlpack(new_capsule(C.cast(mt, C.c_void_p), b"dltensor", None))

    def retrieve_array_subset(self, start=None, shape=None) -> np.ndarray:
        start = [0] * self.ndim if start is None else list(start)
        shape = self.shape if shape is None else list(shape)
        out = np.zeros([int(s) for s in shape], dtype=self.dtype)
        self.retrieve_array_subset_into(start, shape, out)
        return out

    def retrieve_chunk(self, idx) -> np.ndarray:
        start = [int(i) * c for i, c in zip(idx, self.chunk_shape)]
        shape = [min(c, s - st) for c, s, st in zip(self.chunk_shape, self.shape, start)]
        return self.retrieve_array_subset(start, shape)


class ChunkCacheDecodedLruSizeLimit:
    """A decoded-chunk LRU cache of `capacity` bytes resident in HBM (zgpu_cache): the GPU form of
    zarrs' ChunkCacheDecodedLruSizeLimit (zarrs/src/array/chunk_cache/chunk_cache_lru.rs:270)."""

    def __init__(self, capacity: int, ctx: Context | None = None):
        self.ctx = ctx or Context.default()
        h = C.c_void_p()
        L.check(L.load().zgpu_cache_create(self.ctx._h, int(capacity), C.byref(h)))
        self._h = h
        self.capacity = int(capacity)

    def stats(self) -> dict:
        v = [C.c_uint64() for _ in range(4)]
        L.check(L.load().zgpu_cache_stats(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("hits", "misses", "entries", "bytes_used"), (x.value for x in v)))

    def clear(self) -> None:
        L.check(L.load().zgpu_cache_clear(self._h))

    def __del__(self):
        try:
            if getattr(self, "_h", None):
                L.load().zgpu_cache_destroy(self._h)
                self._h = None
        except Exception:
            pass


class ArrayCached:
    """ArrayCached (zarrs/src/array/array_cached.rs:86-120): an Array with a chunk cache; reads go
    through the HBM cache (ArrayCached::retrieve_array_subset, array_read_ops_array_cached.rs:315)."""

    def __init__(self, array: Array, cache: ChunkCacheDecodedLruSizeLimit):
        if isinstance(array.store, FilesystemStore):
            raise NotImplementedError("ArrayCached over a FilesystemStore: read the chunks into a MemoryStore")
        self.array, self.cache = array, cache

    def retrieve_array_subset_into(self, start, shape, out) -> None:
        a = self.array
        ptrs, lens, keep = a._tables(start, shape)
        odev, op = _out_ptr(out)
        flags = (L.ENC_DEVICE if a.store.device else 0) | (L.OUT_DEVICE if odev else 0)
        rc = L.load().zgpu_cache_retrieve_array_subset(
            self.cache._h, a.codecs._h, a.ndim, L.u64s(a.shape), L.u64s(a.chunk_shape), ptrs, lens,
            L.u64s(start), L.u64s(shape), op, flags, default_stream(None, out, *keep))
        del keep
        L.check(rc)

    def retrieve_array_subset(self, start=None, shape=None) -> np.ndarray:
        start = [0] * self.array.ndim if start is None else list(start)
        shape = self.array.shape if shape is None else list(shape)
        out = np.zeros([int(s) for s in shape], dtype=self.array.dtype)
        self.retrieve_array_subset_into(start, shape, out)
        return out

    def retrieve_array_subset_dlpack(self, start=None, shape=None):
        return self.array.retrieve_array_subset_dlpack(start, shape, cache=self.cache)

    def retrieve_chunk(self, idx) -> np.ndarray:
        a = self.array
        start = [int(i) * c for i, c in zip(idx, a.chunk_shape)]
        shape = [min(c, s - st) for c, s, st in zip(a.chunk_shape, a.shape, start)]
        return self.retrieve_array_subset(start, shape)
