"""GPU parity of the write path: zgpu_encode_batch (CodecChain::encode,
codec_chain.rs:528-555) for fixed-size chains against the oracle's encoder (the restatement of
zarrs' encode, pinned by round trips through the reference fixtures' decode path), bit-exact,
including edge chunks that extend past the array (encoded with the fill value)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    return torch


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    return Context(0)


B = lambda e: {"name": "bytes", "configuration": {"endian": e}}  # noqa: E731
T = lambda o: {"name": "transpose", "configuration": {"order": o}}  # noqa: E731
CHAINS = {
    "c2_transpose_be_f32": ([T([2, 1, 0]), B("big")], "float32"),
    "bytes_le_u8": ([B("little")], "uint8"),
    "transpose_021_be_u16": ([T([0, 2, 1]), B("big")], "uint16"),
    "two_transposes_be_i64": ([T([1, 2, 0]), T([2, 0, 1]), B("big")], "int64"),
    "crc_end_f64": ([B("little"), {"name": "crc32c"}], "float64"),
    "shuffle_crc_f32": ([B("big"), {"name": "numcodecs.shuffle", "configuration": {"elementsize": 4}},
                         {"name": "crc32c"}], "float32"),
    "crc_start_end_i32": ([T([2, 0, 1]), B("little"), {"name": "crc32c", "configuration": {"location": "start"}},
                           {"name": "crc32c"}], "int32"),
    "complex64_be": ([B("big")], "complex64"),
    # transposing chains through the LDS-tiled encoder's less common branches
    "transpose_shuffle_crc_f32": ([T([2, 1, 0]), B("big"), {"name": "numcodecs.shuffle", "configuration":
                                   {"elementsize": 4}}, {"name": "crc32c"}], "float32"),
    "transpose_crc_start_f64": ([T([2, 1, 0]), B("little"), {"name": "crc32c", "configuration":
                                 {"location": "start"}}], "float64"),
    "transpose_complex64_be": ([T([1, 2, 0]), B("big")], "complex64"),
}
# (array shape, chunk shape): small ragged chunks, and 64-wide tiles (the vectorised tiled path)
# whose edge chunks cross the array boundary (element path with fill)
GEOMS = {"ragged": ([45, 70, 33], [16, 32, 32]), "tiles64": ([130, 12, 100], [64, 8, 64])}


@pytest.mark.parametrize("geom", list(GEOMS))
@pytest.mark.parametrize("name", list(CHAINS))
def test_encode_vs_oracle(ctx, torch_cuda, name, geom):
    from zarrs_amd import CodecChain
    codecs, dt = CHAINS[name]
    rng = np.random.default_rng(3)
    shape, cs = GEOMS[geom]
    npdt = np.dtype(O.DTYPES[dt][0])
    a = (rng.standard_normal(shape) * 100).astype(npdt) if npdt.kind != "c" else \
        (rng.standard_normal(shape) + 1j * rng.standard_normal(shape)).astype(npdt)
    co = O.OracleChain.from_metadata(codecs, dt, 5, 3)
    ch = CodecChain.from_metadata(codecs, dt, 5, ctx)
    grid = [-(-s // c) for s, c in zip(shape, cs)]
    starts = [[i * c for i, c in zip(idx, cs)] for idx in np.ndindex(*grid)]
    t = torch_cuda.from_numpy(a.view(np.uint8).reshape(-1)).cuda()
    arr = t.view(torch_cuda.uint8)
    # the library takes an untyped device array: pass the bytes with the element shape
    arr_t = arr.view(-1)
    got = ch.encode_chunks(_Typed(arr_t, shape, npdt.itemsize), cs, starts)
    fill = np.array(5, npdt)
    for st, g in zip(starts, got):
        blk = np.full(cs, fill, npdt)
        sl = tuple(slice(s0, min(s0 + c, s)) for s0, c, s in zip(st, cs, shape))
        src = a[sl]
        blk[tuple(slice(0, n) for n in src.shape)] = src
        exp = co.encode(blk)
        assert g.cpu().numpy().tobytes() == exp, (name, st)


class _Typed:
    """A device byte buffer presented with the array's element shape (what encode_chunks reads)."""
    def __init__(self, t, shape, itemsize):
        self._t, self.shape, self._itemsize = t, shape, itemsize
        self.is_cuda, self.device = True, t.device
        assert t.numel() == int(np.prod(shape)) * itemsize

    def is_contiguous(self):
        return True

    def numel(self):
        return int(np.prod(self.shape))

    def element_size(self):
        return self._itemsize

    def data_ptr(self):
        return self._t.data_ptr()


def test_encode_round_trip_and_unsupported(ctx, torch_cuda):
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    from zarrs_amd import _lib as L
    codecs = [T([2, 1, 0]), B("big")]
    ch = CodecChain.from_metadata(codecs, "float32", 0, ctx)
    x = torch_cuda.rand((128, 128, 128), device="cuda")
    starts = [[i, j, k] for i in (0, 64) for j in (0, 64) for k in (0, 64)]
    enc = ch.encode_chunks(x, [64, 64, 64], starts)
    out = torch_cuda.empty_like(x)
    descs = [make_desc((e.data_ptr(), e.numel()), [64] * 3, out_start=s) for e, s in zip(enc, starts)]
    assert ch.decode_batch(descs, out, [128] * 3, enc_device=True) == [0] * 8
    assert torch_cuda.equal(out, x)
    gz = CodecChain.from_metadata([B("little"), {"name": "gzip", "configuration": {"level": 1}}], "float32", 0, ctx)
    with pytest.raises(ZgpuError) as ei:
        gz.encode_chunks(x, [64, 64, 64], starts)
    assert ei.value.status == L.UNSUPPORTED
    # a tensor whose element size does not match the chain's data type is refused up front
    with pytest.raises(ZgpuError) as ei:
        ch.encode_chunks(x.to(torch_cuda.float16), [64, 64, 64], starts)
    assert ei.value.status == L.INVALID_ARGUMENT


def test_sliced_launches(ctx, torch_cuda, monkeypatch):
    """Block ranges beyond one launch's grid limit (gridDim.x * 256 < 2^32) run as several launches
    with a block offset: forced here with a tiny ZGPU_MAX_GRID, for the tiled encoder and the
    tiled / rows scatter kernels, bit-exact against the unsliced result."""
    from zarrs_amd import CodecChain, make_desc
    monkeypatch.setenv("ZGPU_MAX_GRID", "7")
    for codecs in ([T([2, 1, 0]), B("big")], [B("big"), {"name": "crc32c"}]):
        ch = CodecChain.from_metadata(codecs, "float32", 0, ctx)
        x = torch_cuda.rand((128, 72, 128), device="cuda")
        starts = [[i, j, k] for i in (0, 64) for j in (0, 64) for k in (0, 64)]
        enc = ch.encode_chunks(x, [64, 64, 64], starts)
        co = O.OracleChain.from_metadata(codecs, "float32", 0, 3)
        xh = x.cpu().numpy()
        for s, e in zip(starts, enc):
            blk = np.zeros([64] * 3, np.float32)
            src = xh[s[0]:s[0] + 64, s[1]:s[1] + 64, s[2]:s[2] + 64]
            blk[:src.shape[0], :src.shape[1], :src.shape[2]] = src
            assert e.cpu().numpy().tobytes() == co.encode(blk)
        out = torch_cuda.empty_like(x)
        descs = [make_desc((e.data_ptr(), e.numel()), [64] * 3, sel_shape=[min(64, n - s0) for n, s0 in
                                                                            zip(x.shape, s)], out_start=s)
                 for e, s in zip(enc, starts)]
        assert ch.decode_batch(descs, out, list(x.shape), enc_device=True) == [0] * 8
        assert torch_cuda.equal(out, x)


SHARDED = {
    "c3_fixed_inner": ([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [8, 16, 8], "codecs": [B("little"), {"name": "crc32c"}],
        "index_codecs": [B("little"), {"name": "crc32c"}], "index_location": "end"}}], "float32"),
    "transposed_inner_index_start": ([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [4, 8, 16], "codecs": [T([2, 0, 1]), B("big"),
                                              {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
                                              {"name": "crc32c", "configuration": {"location": "start"}}],
        "index_codecs": [B("big"), {"name": "crc32c"}, {"name": "crc32c", "configuration": {"location": "start"}}],
        "index_location": "start"}}], "uint16"),
}


@pytest.mark.parametrize("name", list(SHARDED))
def test_sharding_encode_vs_oracle(ctx, torch_cuda, name):
    """ShardingCodecBound::encode_bounded on the GPU (SubchunkWriteOrder::C; all-fill inner chunks
    omitted; shards crossing the array edge) byte-for-byte against the oracle's shard encoder, and
    decoded back through the GPU read path."""
    from zarrs_amd import CodecChain, make_desc
    codecs, dt = SHARDED[name]
    rng = np.random.default_rng(9)
    npdt = np.dtype(O.DTYPES[dt][0])
    shape, cs = [40, 50, 36], [16, 32, 16]
    a = (rng.standard_normal(shape) * 100).astype(npdt)
    a[:16, :32, :16] = 5             # shard (0,0,0) entirely fill
    a[16:24, 0:16, 0:8] = 5          # one inner chunk of shard (1,0,0) fill
    co = O.OracleChain.from_metadata(codecs, dt, 5, 3)
    ch = CodecChain.from_metadata(codecs, dt, 5, ctx)
    grid = [-(-s // c) for s, c in zip(shape, cs)]
    starts = [[i * c for i, c in zip(idx, cs)] for idx in np.ndindex(*grid)]
    t = torch_cuda.from_numpy(a.view(np.uint8).reshape(-1)).cuda()
    got = ch.encode_chunks(_Typed(t, shape, npdt.itemsize), cs, starts)
    exps = []
    for st, g in zip(starts, got):
        blk = np.full(cs, 5, npdt)
        sl = tuple(slice(s0, min(s0 + c, s)) for s0, c, s in zip(st, cs, shape))
        blk[tuple(slice(0, n) for n in a[sl].shape)] = a[sl]
        exp = co.encode(blk)
        exps.append(exp)
        assert g.cpu().numpy().tobytes() == exp, (name, st)
    assert len(got[0]) < len(got[1])  # the all-fill shard holds only its index
    # round trip through the GPU decode (full and partial shards)
    out = np.zeros(shape, npdt)
    descs = [make_desc(g, cs, sel_shape=[min(c, s - s0) for c, s, s0 in zip(cs, shape, st)], out_start=st)
             for g, st in zip(got, starts)]
    assert ch.decode_batch(descs, out, shape, enc_device=True) == [0] * len(descs)
    assert np.array_equal(out, a)
