import sys, numpy as np
sys.path.insert(0, ".")
from zarrs_amd import Array, ArrayCached, ChunkCacheDecodedLruSizeLimit, MemoryStore, Context, ZgpuError
ctx = Context(0)
codecs = [{"name": "sharding_indexed", "configuration": {
    "chunk_shape": [4], "codecs": [{"name": "bytes", "configuration": {"endian": "little"}}],
    "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}]}},
    {"name": "crc32c"}]
meta = {"shape": [16], "data_type": "uint16", "fill_value": 0, "codecs": codecs,
        "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": [8]}}}
store = MemoryStore({"c/0": bytes(64), "c/1": bytes(64)})
arr = Array(store, meta, ctx)
try:
    print("direct", arr.retrieve_array_subset())
except ZgpuError as e:
    print("direct err", e.status, e)
ca = ArrayCached(arr, ChunkCacheDecodedLruSizeLimit(1 << 20, ctx))
for i in range(2):
    try:
        print("cached", ca.retrieve_array_subset(), ca.cache.stats())
    except ZgpuError as e:
        print("cached err", e.status, e, ca.cache.stats())
