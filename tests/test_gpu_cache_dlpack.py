"""the HBM-resident decoded-chunk cache (zgpu_cache: ChunkCacheDecodedLruSizeLimit
+ ArrayCached, zarrs/src/array/chunk_cache/chunk_cache_lru.rs, array_cached.rs) and the DLPack kDLROCM
export of decoded subsets (the reference's DLPack export is CPU-only: array_dlpack_ext.rs:44-70).
Every read is checked bit-exactly against the CPU oracle's retrieve_array_subset."""
import numpy as np
import pytest

import oracle as O
from test_gpu_parity import CHAINS, _encode_grid

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    return Context(0)


def _setup(ctx, name, store="hbm", shape=(45, 70, 33), cs=(16, 32, 32), drop=((1, 1, 0),)):
    import torch  # noqa: F401
    from zarrs_amd import Array, DeviceStore, MemoryStore
    codecs, dt = CHAINS[name]
    rng = np.random.default_rng(len(name))
    npdt = np.dtype(O.DTYPES[dt][0])
    a = (rng.standard_normal(shape) * 100).astype(npdt)
    co = O.OracleChain.from_metadata(codecs, dt, 3, len(shape))
    chunks = _encode_grid(co, a, list(cs), drop=set(drop))
    ms = MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in chunks.items()})
    meta = {"shape": list(shape), "data_type": dt, "fill_value": 3, "codecs": codecs,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": list(cs)}}}
    arr = Array(DeviceStore.from_store(ms) if store == "hbm" else ms, meta, ctx)
    return arr, co, chunks, list(shape), list(cs)


SUBSETS = [([0, 0, 0], [45, 70, 33]), ([5, 17, 3], [30, 40, 29]), ([16, 32, 0], [16, 32, 32]), ([44, 69, 32], [1, 1, 1])]


@pytest.mark.parametrize("name", ["c2_transpose_be", "shuffle2_zstd_u16", "sharded_crc"])
@pytest.mark.parametrize("store", ["hbm", "host"])
def test_dlpack_export(ctx, name, store):
    import torch
    arr, co, chunks, shape, cs = _setup(ctx, name, store)
    for start, sub in SUBSETS:
        t = arr.retrieve_array_subset_dlpack(start, sub)
        assert t.is_cuda and list(t.shape) == sub and t.is_contiguous()
        exp = O.retrieve_array_subset(co, shape, cs, chunks, start, sub, nthreads=4)
        assert t.cpu().numpy().tobytes() == exp.tobytes(), (start, sub)
        assert t.dtype == torch.from_numpy(exp[:0]).dtype
        del t  # the library's deleter frees the buffer
    torch.cuda.synchronize()


@pytest.mark.parametrize("name", ["c2_transpose_be", "shuffle2_zstd_u16", "sharded_crc"])
def test_hbm_chunk_cache(ctx, name):
    from zarrs_amd import ArrayCached, ChunkCacheDecodedLruSizeLimit
    arr, co, chunks, shape, cs = _setup(ctx, name)
    chunk_bytes = int(np.prod(cs)) * arr.dtype.itemsize
    cache = ChunkCacheDecodedLruSizeLimit(6 * chunk_bytes, ctx)
    ca = ArrayCached(arr, cache)
    # a small window swept over the array: hits, misses and LRU evictions (6 slots, 3x3x2 grid)
    rng = np.random.default_rng(1)
    for it in range(25):
        start = [int(rng.integers(0, s - 1)) for s in shape]
        sub = [int(rng.integers(1, min(20, s - st) + 1)) for s, st in zip(shape, start)]
        exp = O.retrieve_array_subset(co, shape, cs, chunks, start, sub, nthreads=4)
        assert ca.retrieve_array_subset(start, sub).tobytes() == exp.tobytes(), (it, start, sub)
    st = cache.stats()
    assert st["hits"] > 0 and st["misses"] > 0 and st["bytes_used"] <= 6 * chunk_bytes, st
    # the same chunk read twice: the second read is all hits
    before = cache.stats()["hits"]
    for _ in range(2):
        got = ca.retrieve_chunk([0, 0, 0])
        assert got.tobytes() == O.retrieve_array_subset(co, shape, cs, chunks, [0, 0, 0], cs, nthreads=4).tobytes()
    assert cache.stats()["hits"] >= before + 1
    # a read needing more chunks than the cache holds is decoded directly, and is still exact
    exp = O.retrieve_array_subset(co, shape, cs, chunks, [0, 0, 0], shape, nthreads=4)
    assert ca.retrieve_array_subset().tobytes() == exp.tobytes()
    # DLPack through the cache
    t = ca.retrieve_array_subset_dlpack([5, 17, 3], [10, 10, 10])
    exp = O.retrieve_array_subset(co, shape, cs, chunks, [5, 17, 3], [10, 10, 10], nthreads=4)
    assert t.cpu().numpy().tobytes() == exp.tobytes()
    cache.clear()
    assert cache.stats()["entries"] == 0


def test_cache_does_not_keep_failed_chunks(ctx):
    """A chunk whose checksum fails is reported (INVALID_CHECKSUM) and not cached."""
    from zarrs_amd import Array, ArrayCached, ChunkCacheDecodedLruSizeLimit, MemoryStore, ZgpuError
    codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}]
    co = O.OracleChain.from_metadata(codecs, "uint16", 0, 1)
    a = np.arange(300, dtype=np.uint16)
    chunks = {(i,): co.encode(a[i * 100:(i + 1) * 100]) for i in range(3)}
    bad = bytearray(chunks[(1,)])
    bad[5] ^= 1
    store = MemoryStore({"c/0": chunks[(0,)], "c/1": bytes(bad), "c/2": chunks[(2,)]})
    meta = {"shape": [300], "data_type": "uint16", "fill_value": 0, "codecs": codecs,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": [100]}}}
    ca = ArrayCached(Array(store, meta, ctx), ChunkCacheDecodedLruSizeLimit(10 * 200, ctx))
    with pytest.raises(ZgpuError) as ei:
        ca.retrieve_array_subset()
    assert ei.value.status == 1
    assert ca.cache.stats()["entries"] == 2
    assert np.array_equal(ca.retrieve_array_subset([200], [100]), a[200:])


def test_cache_call_level_error_is_not_cached(ctx):
    """A chain the planner rejects before any chunk status exists (a shard index compressed with gzip:
    the index must have a fixed encoded size, UNSUPPORTED) fails on every read through the cache; no
    slot is kept."""
    from zarrs_amd import Array, ArrayCached, ChunkCacheDecodedLruSizeLimit, MemoryStore, ZgpuError
    idx = [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "gzip", "configuration": {"level": 1}}]
    codecs = [{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [4], "codecs": [{"name": "bytes", "configuration": {"endian": "little"}}],
        "index_codecs": idx}}]
    meta = {"shape": [16], "data_type": "uint16", "fill_value": 0, "codecs": codecs,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": [8]}}}
    store = MemoryStore({"c/0": bytes(64), "c/1": bytes(64)})
    ca = ArrayCached(Array(store, meta, ctx), ChunkCacheDecodedLruSizeLimit(1 << 20, ctx))
    for _ in range(2):
        with pytest.raises(ZgpuError) as ei:
            ca.retrieve_array_subset()
        assert ei.value.status == 6
    assert ca.cache.stats()["entries"] == 0
