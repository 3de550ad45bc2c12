"""zarrs_amd — MI355X-native (gfx950) Zarr chunk-decode codec pipeline.

The product is libzgpu.so (hand-written HIP kernels + C++ orchestration behind include/zgpu.h).
This package is the host-side mirror of the zarrs read-path interface used by tests and bench.py.
"""
from ._lib import ZgpuError, load as load_library  # noqa: F401
from .codec import CodecChain, Context, PlanGroup, fill_value_bytes, make_desc  # noqa: F401
from .array import (Array, ArrayCached, ChunkCacheDecodedLruSizeLimit, DeviceStore,  # noqa: F401
                    FilesystemStore, MemoryStore)

__version__ = "0.1.0"
