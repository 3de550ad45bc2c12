"""The drop-in boundary's call pattern: decode_into a window of a larger array
(ArrayBytesFixedDisjointView, zarrs_codec/src/array_bytes_fixed_disjoint_view.rs:12-207 -- the target
ShardingCodecBound::decode_into writes into, sharding_codec.rs:617-707) and ZGPU_COALESCE, which merges
concurrent per-shard calls from a thread pool (zarrs' rayon loop, array_read_ops_common.rs:173-176)
into one GPU batch while every caller keeps its own statuses and first error.

Checked against the oracle's decode of the same shards; bytes of the output array outside each
caller's window must keep their sentinel value.
"""
import struct
import threading
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

BYTES_LE = {"name": "bytes", "configuration": {"endian": "little"}}
INNER_CODECS = [BYTES_LE, {"name": "gzip", "configuration": {"level": 1}}, {"name": "crc32c"}]
CODECS = [{"name": "sharding_indexed", "configuration": {
    "chunk_shape": [16, 16, 16], "codecs": INNER_CODECS,
    "index_codecs": [BYTES_LE, {"name": "crc32c"}], "index_location": "end"}}]
SH = 64
SHAPE = [128, 128, 256]  # 2 x 2 x 4 = 16 shards
SENTINEL = np.float32(-7.25)


def _values(shape):
    rng = np.random.default_rng(11)
    x = np.arange(shape[0], dtype=np.float32)[:, None, None]
    y = np.arange(shape[1], dtype=np.float32)[None, :, None]
    z = np.arange(shape[2], dtype=np.float32)[None, None, :]
    v = np.rint(64 * (np.sin(0.1 * x) + np.cos(0.07 * y) + np.sin(0.05 * z)) + rng.standard_normal(shape)) / 64
    return v.astype(np.float32)


@pytest.fixture(scope="module")
def data():
    a = _values(SHAPE)
    co = O.OracleChain.from_metadata(CODECS, "float32", 0.0, 3)
    keys = [(i, j, k) for i in range(2) for j in range(2) for k in range(4)]
    shards = {}
    for key in keys:
        sl = tuple(slice(c * SH, (c + 1) * SH) for c in key)
        shards[key] = np.frombuffer(co.encode(np.ascontiguousarray(a[sl])), np.uint8).copy()
    return a, shards


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    c = Context(0)
    yield c
    c.close()


def _corrupt(shard: np.ndarray, inner: int) -> np.ndarray:
    """Flip a byte of inner chunk `inner`'s stored crc32c (InvalidChecksum on the full path)."""
    n_inner = (SH // 16) ** 3
    tail = shard[len(shard) - (n_inner * 16 + 4):len(shard) - 4].tobytes()
    idx = struct.unpack("<%dQ" % (2 * n_inner), tail)
    off, nb = idx[2 * inner], idx[2 * inner + 1]
    bad = shard.copy()
    bad[off + nb - 2] ^= 0x10
    return bad


def _origin(key):
    return [c * SH for c in key]


def test_decode_into_host_window(ctx, data):
    from zarrs_amd import CodecChain, make_desc
    a, shards = data
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    out = np.full(SHAPE, SENTINEL, np.float32)
    key = (1, 0, 2)
    o = _origin(key)
    st = ch.decode_batch_into([make_desc(shards[key], [SH] * 3)], out, o, [SH] * 3, enc_device=False)
    assert st == [0]
    win = tuple(slice(s, s + SH) for s in o)
    assert np.array_equal(out[win], a[win])
    mask = np.ones(SHAPE, bool)
    mask[win] = False
    assert np.all(out[mask] == SENTINEL)


def test_decode_into_host_window_partial(ctx, data):
    """A partial selection of one shard into a window of a larger host array (the partial decoder's
    partial_decode_into, sharding_partial_decoder_sync.rs:241-272), crc32c stripped."""
    from zarrs_amd import CodecChain, make_desc
    a, shards = data
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    out = np.full(SHAPE, SENTINEL, np.float32)
    key = (0, 1, 3)
    o = _origin(key)
    ss, sz = [5, 17, 3], [40, 33, 61]
    ws = [a_ + b_ for a_, b_ in zip(o, ss)]
    st = ch.decode_batch_into([make_desc(shards[key], [SH] * 3, ss, sz)], out, ws, sz, enc_device=False)
    assert st == [0]
    win = tuple(slice(s, s + n) for s, n in zip(ws, sz))
    assert np.array_equal(out[win], a[win])
    mask = np.ones(SHAPE, bool)
    mask[win] = False
    assert np.all(out[mask] == SENTINEL)


def test_decode_into_device_window(ctx, data):
    import torch
    from zarrs_amd import CodecChain, make_desc
    a, shards = data
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    out = torch.full(SHAPE, float(SENTINEL), dtype=torch.float32, device="cuda")
    keys = [(0, 0, 0), (1, 1, 3)]
    for key in keys:
        d = torch.from_numpy(shards[key]).cuda()
        st = ch.decode_batch_into([make_desc(d, [SH] * 3)], out, _origin(key), [SH] * 3, enc_device=True)
        assert st == [0]
    torch.cuda.synchronize()
    h = out.cpu().numpy()
    mask = np.ones(SHAPE, bool)
    for key in keys:
        win = tuple(slice(s, s + SH) for s in _origin(key))
        assert np.array_equal(h[win], a[win])
        mask[win] = False
    assert np.all(h[mask] == SENTINEL)


def test_decode_into_rejects_view_outside_array(ctx, data):
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    _, shards = data
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    out = np.zeros(SHAPE, np.float32)
    with pytest.raises(ZgpuError) as e:
        ch.decode_batch_into([make_desc(shards[(0, 0, 0)], [SH] * 3)], out, [100, 0, 0], [SH] * 3, enc_device=False)
    assert e.value.status == 10  # INVALID_ARGUMENT


def _coalesced_full(ctx, data, bad_key=None, threads=16):
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    a, shards = data
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    out = np.full(SHAPE, SENTINEL, np.float32)
    src = dict(shards)
    if bad_key is not None:
        src[bad_key] = _corrupt(shards[bad_key], 9)
    barrier = threading.Barrier(threads)

    def one(key):
        barrier.wait()
        try:
            return ch.decode_batch_into([make_desc(src[key], [SH] * 3)], out, _origin(key), [SH] * 3,
                                        enc_device=False, coalesce=True)
        except ZgpuError as e:
            return e.status
    keys = sorted(src)
    with ThreadPoolExecutor(threads) as ex:
        res = dict(zip(keys, ex.map(one, keys)))
    return a, out, res


def test_lone_coalesced_caller_does_not_wait_the_window(ctx, data):
    """A coalesced call with no other call in flight closes its batch at once (the collect window is
    for concurrent callers): with a 300 ms window a lone shard call must not take 300 ms."""
    import time
    from zarrs_amd import CodecChain, make_desc
    a, shards = data
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    out = np.full(SHAPE, SENTINEL, np.float32)
    key = (0, 1, 3)
    o = _origin(key)
    call = lambda co: ch.decode_batch_into([make_desc(shards[key], [SH] * 3)], out, o, [SH] * 3,  # noqa: E731
                                           enc_device=False, coalesce=co)
    call(False)  # warm the chain's plan and pools
    ctx.set_coalescing(window_us=300000, max_calls=16)
    try:
        t0 = time.perf_counter()
        st = call(True)
        dt = time.perf_counter() - t0
    finally:
        ctx.set_coalescing(window_us=200, max_calls=8)
    assert st == [0]
    win = tuple(slice(s, s + SH) for s in o)
    assert np.array_equal(out[win], a[win])
    assert dt < 0.15, dt


def test_coalesced_full_shards(ctx, data):
    ctx.set_coalescing(window_us=50000, max_calls=16)
    before = ctx.coalescing_stats()
    a, out, res = _coalesced_full(ctx, data)
    after = ctx.coalescing_stats()
    assert all(v == [0] for v in res.values()), res
    assert np.array_equal(out, a)
    calls = after["calls"] - before["calls"]
    batches = after["batches"] - before["batches"]
    assert calls == 16 and batches < 16, (calls, batches)


def test_coalesced_one_corrupt_caller(ctx, data):
    """16 threads, one shard with a corrupt inner checksum: only that caller gets INVALID_CHECKSUM
    (its own first error); every other caller's window is decoded bit-exactly."""
    ctx.set_coalescing(window_us=50000, max_calls=16)
    bad = (1, 0, 1)
    a, out, res = _coalesced_full(ctx, data, bad_key=bad)
    for key, v in res.items():
        if key == bad:
            assert v == 1, (key, v)  # INVALID_CHECKSUM
        else:
            assert v == [0], (key, v)
            win = tuple(slice(s, s + SH) for s in _origin(key))
            assert np.array_equal(out[win], a[win]), key


@pytest.mark.parametrize("max_calls", [3, 16])
def test_coalesced_partial_windows_of_different_shapes(ctx, data, max_calls):
    """Partial selections of different shapes (the batch's stacked output is padded to the largest
    trailing extents and packed per caller on the device), one per thread, with the inner chain's
    partial path (crc32c stripped)."""
    from zarrs_amd import CodecChain, make_desc
    a, shards = data
    ctx.set_coalescing(window_us=50000, max_calls=max_calls)
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    out = np.full(SHAPE, SENTINEL, np.float32)
    rng = np.random.default_rng(3)
    keys = sorted(shards)
    sels = {}
    for key in keys:
        ss = [int(rng.integers(0, 40)) for _ in range(3)]
        sz = [int(rng.integers(1, SH - s + 1)) for s in ss]
        sels[key] = (ss, sz)
    barrier = threading.Barrier(len(keys))

    def one(key):
        ss, sz = sels[key]
        ws = [o + s for o, s in zip(_origin(key), ss)]
        barrier.wait()
        return ch.decode_batch_into([make_desc(shards[key], [SH] * 3, ss, sz)], out, ws, sz, enc_device=False,
                                    coalesce=True)
    with ThreadPoolExecutor(len(keys)) as ex:
        res = list(ex.map(one, keys))
    assert all(r == [0] for r in res)
    mask = np.ones(SHAPE, bool)
    for key in keys:
        ss, sz = sels[key]
        win = tuple(slice(o + s, o + s + n) for o, s, n in zip(_origin(key), ss, sz))
        assert np.array_equal(out[win], a[win]), key
        mask[win] = False
    assert np.all(out[mask] == SENTINEL)


def test_coalesced_two_chains_and_inner_chunk_calls(ctx, data):
    """Concurrent coalesced calls on two chains (the sharded chain for whole shards, the inner chain
    for partial shards' inner chunks, as the plugin's partial decoder issues them) batch per chain."""
    from zarrs_amd import CodecChain, make_desc
    a, shards = data
    ctx.set_coalescing(window_us=20000, max_calls=8)
    sharded = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    inner = CodecChain.from_metadata(INNER_CODECS, "float32", 0.0, ctx)
    out = np.full(SHAPE, SENTINEL, np.float32)
    keys = sorted(shards)
    n_inner = (SH // 16) ** 3
    barrier = threading.Barrier(len(keys))

    def one(key):
        o = _origin(key)
        barrier.wait()
        if sum(key) % 2 == 0:
            return sharded.decode_batch_into([make_desc(shards[key], [SH] * 3)], out, o, [SH] * 3,
                                             enc_device=False, coalesce=True)
        # inner chunks of rows 16..48 along axis 0 of this shard, through the inner chain
        host = shards[key]
        idx = np.frombuffer(host[len(host) - (n_inner * 16 + 4):len(host) - 4].tobytes(), np.uint64).reshape(-1, 2)
        descs = []
        for ci in range(1, 3):
            for cj in range(4):
                for ck in range(4):
                    off, ln = idx[(ci * 4 + cj) * 4 + ck]
                    descs.append(make_desc((host.ctypes.data + int(off), int(ln)), [16] * 3,
                                           out_start=[(ci - 1) * 16, cj * 16, ck * 16]))
        return inner.decode_batch_into(descs, out, [o[0] + 16, o[1], o[2]], [32, SH, SH], enc_device=False,
                                       validate_checksums=False, coalesce=True)
    with ThreadPoolExecutor(len(keys)) as ex:
        res = list(ex.map(one, keys))
    assert all(all(v == 0 for v in r) for r in res)
    for key in keys:
        o = _origin(key)
        if sum(key) % 2 == 0:
            win = tuple(slice(s, s + SH) for s in o)
        else:
            win = (slice(o[0] + 16, o[0] + 48), slice(o[1], o[1] + SH), slice(o[2], o[2] + SH))
        assert np.array_equal(out[win], a[win]), key


def test_coalesce_flag_with_uncovered_window_takes_direct_path(ctx, data):
    """A window the descriptors do not cover keeps its other bytes: such a call is not coalesced."""
    from zarrs_amd import CodecChain, make_desc
    a, shards = data
    ctx.set_coalescing(window_us=1000, max_calls=8)
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    out = np.full(SHAPE, SENTINEL, np.float32)
    key = (0, 0, 1)
    o = _origin(key)
    # window of [SH, SH, 2*SH]; only its first half is decoded
    st = ch.decode_batch_into([make_desc(shards[key], [SH] * 3)], out, o, [SH, SH, 2 * SH], enc_device=False,
                              coalesce=True)
    assert st == [0]
    win = tuple(slice(s, s + SH) for s in o)
    assert np.array_equal(out[win], a[win])
    rest = (slice(o[0], o[0] + SH), slice(o[1], o[1] + SH), slice(o[2] + SH, o[2] + 2 * SH))
    assert np.all(out[rest] == SENTINEL)


@pytest.mark.parametrize("coalesce", [False, True])
def test_decode_pinned_plugin_pattern(ctx, data, coalesce):
    """zgpu_decode_pinned (the Rust plugin's decode_into: the decoded window stays in library pinned
    memory and the caller copies it once into its view) from 16 threads: full shards and partial
    selections, one corrupt caller that gets its own INVALID_CHECKSUM and no data."""
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    a, shards = data
    ctx.set_coalescing(window_us=2000, max_calls=6)
    ch = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    inner = CodecChain.from_metadata(INNER_CODECS, "float32", 0.0, ctx)
    out = np.full(SHAPE, SENTINEL, np.float32)
    bad = (0, 1, 2)
    src = dict(shards)
    src[bad] = _corrupt(shards[bad], 5)
    keys = sorted(src)
    barrier = threading.Barrier(len(keys))

    def one(key):
        barrier.wait()
        o = _origin(key)
        try:
            if sum(key) % 2:  # full shard: the sharded chain, index verified
                return ch.decode_pinned_into([make_desc(src[key], [SH] * 3)], out, o, [SH] * 3, coalesce=coalesce)
            return ch.decode_pinned_into([make_desc(src[key], [SH] * 3, [0, 0, 0], [SH, SH, 40])], out, o,
                                         [SH, SH, 40], coalesce=coalesce)
        except ZgpuError as e:
            return e.status
    with ThreadPoolExecutor(len(keys)) as ex:
        res = dict(zip(keys, ex.map(one, keys)))
    mask = np.ones(SHAPE, bool)
    for key, v in res.items():
        o = _origin(key)
        full = sum(key) % 2 == 1
        if key == bad and full:
            assert v == 1, (key, v)
            continue
        assert v == [0], (key, v)
        win = tuple(slice(s_, s_ + n_) for s_, n_ in zip(o, [SH] * 3 if full else [SH, SH, 40]))
        assert np.array_equal(out[win], a[win]), key
        mask[win] = False
    assert np.all(out[mask] == SENTINEL)  # the corrupt caller's window and the unselected parts
