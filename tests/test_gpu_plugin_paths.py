"""The C-ABI calls behind the Rust plugin's partial-decoder and encode paths (rust/zarrs_gpu/src/sharding.rs),
each mirrored here through ctypes and checked against the oracle:

  partial_decode_into  ShardingPartialDecoder::partial_decode_into (sharding_partial_decoder_sync.rs:241-272):
                       the intersecting inner chunks in one zgpu_decode_pinned, one copy into the view
  generic indexer      partial_decode_fixed_indexer (:492-560): only the inner chunks the indices touch are
                       decoded (each once, stacked along axis 0), counted by ZGPU_CTR_ITEMS
  encode               ShardingCodecBound::encode (sharding_codec.rs:351-376) through zgpu_encode_pinned
"""
import ctypes as C

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

BYTES_LE = {"name": "bytes", "configuration": {"endian": "little"}}
INNER = [BYTES_LE, {"name": "gzip", "configuration": {"level": 1}}, {"name": "crc32c"}]
CODECS = [{"name": "sharding_indexed", "configuration": {
    "chunk_shape": [8, 8, 8], "codecs": INNER, "index_codecs": [BYTES_LE, {"name": "crc32c"}],
    "index_location": "end"}}]
SH = [32, 32, 32]


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    c = Context(0)
    yield c
    c.close()


@pytest.fixture(scope="module")
def shard():
    rng = np.random.default_rng(5)
    a = (np.round(rng.standard_normal(SH) * 32) / 32).astype(np.float32)
    a[8:16, 0:8, 16:24] = 0.0  # an inner chunk equal to the fill value: omitted from the shard (empty entry)
    co = O.OracleChain.from_metadata(CODECS, "float32", 0.0, 3)
    return a, np.frombuffer(co.encode(a), np.uint8).copy()


def _index(enc):
    n = (SH[0] // 8) ** 3
    return np.frombuffer(enc[len(enc) - (16 * n + 4):len(enc) - 4].tobytes(), np.uint64).reshape(-1, 2)


def _inner_desc(enc, index, ci, sel_start, sel_shape, out_start):
    from zarrs_amd import make_desc
    lin = (ci[0] * 4 + ci[1]) * 4 + ci[2]
    off, nb = index[lin]
    src = None if off == 2 ** 64 - 1 else (enc.ctypes.data + int(off), int(nb))
    return make_desc(src, [8, 8, 8], sel_start, sel_shape, out_start)


def test_partial_decode_into_view(ctx, shard):
    from zarrs_amd import CodecChain
    a, enc = shard
    inner = CodecChain.from_metadata(INNER, "float32", 0.0, ctx)
    index = _index(enc)
    start, shape = [3, 5, 9], [20, 17, 14]
    descs = []
    for ci in np.ndindex(*[(s + n - 1) // 8 + 1 - s // 8 for s, n in zip(start, shape)]):
        ci = [c + s // 8 for c, s in zip(ci, start)]
        s0 = [max(s, c * 8) for s, c in zip(start, ci)]
        s1 = [min(s + n, c * 8 + 8) for s, n, c in zip(start, shape, ci)]
        descs.append(_inner_desc(enc, index, ci, [x - c * 8 for x, c in zip(s0, ci)], [b - x for x, b in zip(s0, s1)],
                                 [x - s for x, s in zip(s0, start)]))
    view = np.full([40, 40, 40], -1.0, np.float32)  # the caller's array; the view is a window of it
    w0 = [7, 1, 20]
    st = inner.decode_pinned_into(descs, view, w0, shape, validate_checksums=False)
    assert st == [0] * len(descs)
    sl = tuple(slice(s, s + n) for s, n in zip(start, shape))
    win = tuple(slice(s, s + n) for s, n in zip(w0, shape))
    assert np.array_equal(view[win], a[sl])
    mask = np.ones(view.shape, bool)
    mask[win] = False
    assert np.all(view[mask] == -1.0)


def test_generic_indexer_decodes_touched_inner_chunks_only(ctx, shard):
    from zarrs_amd import CodecChain
    from zarrs_amd import _lib as L
    a, enc = shard
    inner = CodecChain.from_metadata(INNER, "float32", 0.0, ctx)
    index = _index(enc)
    rng = np.random.default_rng(9)
    pts = rng.integers(0, 32, size=(50, 3))
    pts[:5] = [[9, 3, 17], [10, 4, 18], [0, 0, 0], [31, 31, 31], [9, 3, 17]]  # repeats + the empty inner chunk
    order, slot, elems = [], {}, []
    for p in pts:
        ci = tuple(int(x) // 8 for x in p)
        if ci not in slot:
            slot[ci] = len(order)
            order.append(ci)
        elems.append((slot[ci], ((int(p[0]) % 8) * 8 + int(p[1]) % 8) * 8 + int(p[2]) % 8))
    descs = [_inner_desc(enc, index, ci, [0, 0, 0], [8, 8, 8], [k * 8, 0, 0]) for k, ci in enumerate(order)]
    stacked = np.empty([8 * len(order), 8, 8], np.float32)
    st = inner.decode_pinned_into(descs, stacked, [0, 0, 0], list(stacked.shape), validate_checksums=False)
    assert st == [0] * len(descs)
    ctr = (C.c_uint64 * L.N_COUNTERS)()
    L.load().zgpu_last_counters(ctr, L.N_COUNTERS)
    assert ctr[L.CTR_ITEMS] == len(order) < 50  # each touched inner chunk once, nothing else
    flat = stacked.reshape(len(order), -1)
    got = np.array([flat[k, w] for k, w in elems], np.float32)
    assert np.array_equal(got, a[pts[:, 0], pts[:, 1], pts[:, 2]])


def test_encode_pinned_shard_and_zstd_chunk(ctx, shard):
    from zarrs_amd import CodecChain
    from zarrs_amd import _lib as L
    lib = L.load()
    a, _ = shard
    for codecs, x, dt in ((CODECS, a, "float32"),
                          ([BYTES_LE, {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
                            {"name": "zstd", "configuration": {"level": 3, "checksum": False}}],
                           (np.arange(16 * 64 * 64) % 977).astype(np.uint16).reshape(16, 64, 64), "uint16")):
        ch = CodecChain.from_metadata(codecs, dt, 0, ctx)
        p, n, r = C.c_void_p(), C.c_uint64(), C.c_void_p()
        L.check(lib.zgpu_encode_pinned(ch._h, 3, L.u64s(list(x.shape)), x.ctypes.data, C.byref(p), C.byref(n),
                                       C.byref(r)))
        try:
            enc = bytes((C.c_uint8 * n.value).from_address(p.value))
        finally:
            lib.zgpu_result_release(r)
        co = O.OracleChain.from_metadata(codecs, dt, 0, 3)
        assert np.array_equal(co.decode(enc, x.shape), x)
