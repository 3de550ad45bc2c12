"""Array-level read path mirror: Array / MemoryStore / DeviceStore over the GPU codec pipeline.

  Array.retrieve_array_subset  <- Array::retrieve_array_subset (array_read_ops_array.rs:74-154,
                                  array_read_ops_common.rs:20-179): subset -> intersecting chunks ->
                                  one batched GPU decode (full chunks: decode_into with checksum
                                  verification; partial chunks: partial decoder semantics)
  Array.retrieve_chunk         <- Array::retrieve_chunk (array_read_ops_array.rs:265-272)
  MemoryStore                  <- zarrs_storage MemoryStore (encoded chunks in host memory)
  DeviceStore                  <- encoded chunks resident in HBM (torch uint8 tensors)
Chunk keys use the default encoding "c/i/j/k" (chunk_key_encoding/default.rs:79-102) or v2 "i.j".
"""
from __future__ import annotations

import ctypes as C
import json

import numpy as np

from . import _lib as L
from .codec import CodecChain, Context


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


class Array:
    def __init__(self, store, metadata: dict, ctx: Context | None = None,
                 validate_checksums: bool = True):
        if isinstance(metadata, str):
            metadata = json.loads(metadata)
        self.store = store
        self.metadata = metadata
        self.shape = [int(s) for s in metadata["shape"]]
        self.chunk_shape = [int(c) for c in metadata["chunk_grid"]["configuration"]["chunk_shape"]]
        self.data_type = metadata["data_type"]
        kenc = metadata.get("chunk_key_encoding", {"name": "default"})
        cfg = kenc.get("configuration", {}) or {}
        if kenc["name"] == "default":
            self._sep, self._prefix = cfg.get("separator", "/"), "c" + cfg.get("separator", "/")
        else:
            self._sep, self._prefix = cfg.get("separator", "."), ""
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

    def _tables(self):
        grid = self.chunk_grid_shape()
        n = int(np.prod(grid))
        ptrs = (C.c_void_p * n)()
        lens = (C.c_uint64 * n)()
        keep = []
        for lin in range(n):
            idx = np.unravel_index(lin, grid)
            v = self.store.get(self.chunk_key(idx))
            if v is None:
                continue
            if self.store.device:
                ptrs[lin] = v.data_ptr() if v.numel() else None
                lens[lin] = v.numel()
                if not v.numel():  # an empty object is still present: give it a valid address
                    import torch
                    t = torch.empty(1, dtype=torch.uint8, device=v.device)
                    keep.append(t)
                    ptrs[lin] = t.data_ptr()
            else:
                b = C.create_string_buffer(bytes(v), max(len(v), 1))
                keep.append(b)
                ptrs[lin] = C.addressof(b)
                lens[lin] = len(v)
        return ptrs, lens, keep

    def retrieve_array_subset_into(self, start, shape, out) -> None:
        ptrs, lens, keep = self._tables()
        try:
            import torch
            odev = isinstance(out, torch.Tensor) and out.is_cuda
            op = out.data_ptr() if isinstance(out, torch.Tensor) else out.ctypes.data
        except ImportError:  # pragma: no cover
            odev, op = False, out.ctypes.data
        flags = (L.ENC_DEVICE if self.store.device else 0) | (L.OUT_DEVICE if odev else 0)
        rc = L.load().zgpu_retrieve_array_subset(
            self.codecs._h, self.ndim, L.u64s(self.shape), L.u64s(self.chunk_shape), ptrs, lens,
            L.u64s(start), L.u64s(shape), op, flags, None)
        del keep
        L.check(rc)

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
