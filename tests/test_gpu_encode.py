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
    # blosc behind a variable-length codec (its frame needs a fixed typesize layout) is refused loudly
    bl = CodecChain.from_metadata([B("little"), {"name": "gzip", "configuration": {"level": 1}},
                                   {"name": "blosc", "configuration": {"cname": "lz4", "clevel": 5, "shuffle": "shuffle",
                                                                       "typesize": 4, "blocksize": 0}}],
                                  "float32", 0, ctx)
    with pytest.raises(ZgpuError) as ei:
        bl.encode_chunks(x, [64, 64, 64], starts)
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


# ---- compressing chains (gzip) -------------------------------------------------------------------
GZ = {"name": "gzip", "configuration": {"level": 1}}
CRC = {"name": "crc32c"}
CRC_S = {"name": "crc32c", "configuration": {"location": "start"}}


def _c3_values(shape, seed=7):
    rng = np.random.default_rng(seed)
    z, y, x = np.meshgrid(*[np.arange(n) for n in shape], indexing="ij")
    v = np.round((np.sin(0.05 * x) + np.cos(0.03 * y) + 0.5 * np.sin(0.07 * z)) * 256) / 256
    return (v + rng.standard_normal(v.shape) / 256).astype(np.float32)


def _contents(shape):
    """f32 volumes of the kinds an encoder must get right: SURVEY C3's quantised smooth field,
    white noise (incompressible: stored blocks), constant runs (258-byte matches), a ramp, and a
    mix of regions."""
    rng = np.random.default_rng(3)
    n = int(np.prod(shape))
    mixed = _c3_values(shape, 9).reshape(-1).copy()
    mixed[: n // 3] = 0
    mixed[n // 3: n // 2] = rng.standard_normal(n // 2 - n // 3)
    return {"c3": _c3_values(shape), "noise": rng.standard_normal(shape).astype(np.float32),
            "zeros": np.zeros(shape, np.float32), "ramp": np.arange(n, dtype=np.float32).reshape(shape),
            "mixed": mixed.reshape(shape)}


@pytest.mark.parametrize("chain", ["gzip", "gzip_crc", "crc_start_gzip_crc", "be_shuffle_gzip"])
def test_gzip_encode_decodes_with_zlib(ctx, torch_cuda, chain):
    """GzipCodec::encode on the GPU (k_gzip_encode): every member inflates with zlib (the reference's
    own decoder family) to the exact chunk bytes, the crc32c codecs around it are the oracle's, and
    the GPU decode reads it back bit-exactly."""
    import zlib
    from zarrs_amd import CodecChain, make_desc
    codecs = {"gzip": [B("little"), GZ], "gzip_crc": [B("little"), GZ, CRC],
              "crc_start_gzip_crc": [B("little"), CRC_S, GZ, CRC],
              "be_shuffle_gzip": [T([2, 1, 0]), B("big"), {"name": "numcodecs.shuffle",
                                                           "configuration": {"elementsize": 4}}, GZ]}[chain]
    co = O.OracleChain.from_metadata(codecs, "float32", 0, 3)
    ch = CodecChain.from_metadata(codecs, "float32", 0, ctx)
    cs = [32, 32, 32]
    for kind, a in _contents([64, 64, 32]).items():
        x = torch_cuda.from_numpy(a).cuda()
        starts = [[i, j, 0] for i in (0, 32) for j in (0, 32)]
        enc = ch.encode_chunks(x, cs, starts)
        bound = ch.encoded_bound(cs)
        for st, e in zip(starts, enc):
            got = e.cpu().numpy().tobytes()
            assert len(got) <= bound
            blk = np.ascontiguousarray(a[st[0]:st[0] + 32, st[1]:st[1] + 32, :])
            # the member itself, unwrapped from the crc32c codecs the oracle would write around it
            plain = co.decode(got, cs)
            assert np.array_equal(plain, blk), (chain, kind, st)
            if chain == "gzip":
                assert zlib.decompress(got, 31) == blk.tobytes()
        out = torch_cuda.zeros_like(x)
        descs = [make_desc((e.data_ptr(), e.numel()), cs, out_start=st) for e, st in zip(enc, starts)]
        assert ch.decode_batch(descs, out, list(x.shape), enc_device=True) == [0] * len(enc)
        assert torch_cuda.equal(out, x), (chain, kind)


def test_gzip_encode_ratio_vs_zlib_level1(ctx, torch_cuda):
    """The GPU encoder's compression on SURVEY C3 data against zlib level 1 (the configured level):
    within 30 % of its size (LZ77 parsing is an encoder choice, gzip_codec.rs:126-128)."""
    import zlib
    from zarrs_amd import CodecChain
    a = _c3_values([128, 64, 64])
    ch = CodecChain.from_metadata([B("little"), GZ], "float32", 0, ctx)
    x = torch_cuda.from_numpy(a).cuda()
    starts = [[i, j, k] for i in range(0, 128, 32) for j in (0, 32) for k in (0, 32)]
    enc = ch.encode_chunks(x, [32, 32, 32], starts)
    gpu = sum(e.numel() for e in enc)
    ref = 0
    for st in starts:
        blk = np.ascontiguousarray(a[st[0]:st[0] + 32, st[1]:st[1] + 32, st[2]:st[2] + 32])
        c = zlib.compressobj(1, zlib.DEFLATED, 31)
        ref += len(c.compress(blk.tobytes()) + c.flush())
    print(f"gzip encode on C3 data: GPU {gpu} B, zlib-1 {ref} B, ratio {gpu / ref:.3f}")
    assert gpu <= 1.3 * ref


def test_gzip_encode_small_and_ragged_chunks(ctx, torch_cuda):
    """Chunks of 1..9 elements (shorter than a hash window) and chunks crossing the array edge
    (fill value past it), u8 and u16."""
    import zlib
    from zarrs_amd import CodecChain
    for dt, npdt in (("uint8", np.uint8), ("uint16", np.uint16)):
        codecs = [B("little"), GZ]
        for n in (1, 2, 3, 4, 5, 9, 63, 64, 65, 200):
            a = (np.arange(n * 3) % 7).astype(npdt)
            ch = CodecChain.from_metadata(codecs, dt, 5, ctx)
            x = torch_cuda.from_numpy(a.view(np.uint8).copy()).cuda()
            x = x.view(torch_cuda.uint8 if dt == "uint8" else torch_cuda.int16)
            starts = [[0], [n], [2 * n], [3 * n - 1]]
            enc = ch.encode_chunks(x, [n], starts)
            for st, e in zip(starts, enc):
                blk = np.full(n, 5, npdt)
                src = a[st[0]:st[0] + n]
                blk[:len(src)] = src
                assert zlib.decompress(e.cpu().numpy().tobytes(), 31) == blk.tobytes(), (dt, n, st)


def test_gzip_encode_huffman_length_limits(ctx, torch_cuda):
    """Length-limited Huffman codes (zlib gen_bitlen: every node clamped to the limit counts as an
    overflow, internal ones included): the code-length code at its 7-bit limit on the C3 inner chunk
    where counting clamped leaves only left it over-subscribed (zlib: "invalid code lengths set";
    the C3 synth volume at [0:32, 352:384, 1024:1056], tools/synth), and literal codes at the 15-bit
    limit on bytes with Fibonacci-distributed frequencies (optimal depth ~24), through zlib."""
    import ctypes as C
    import os
    import zlib
    from zarrs_amd import CodecChain
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    syn = C.CDLL(os.path.join(root, "tools", "synth", "libsynth.so"))
    P64 = C.POINTER(C.c_uint64)
    syn.synth_c3_values.argtypes = [P64, P64, C.c_void_p, C.c_int]
    u64 = lambda v: (C.c_uint64 * 3)(*v)  # noqa: E731
    a = np.empty([32, 32, 32], np.float32)
    syn.synth_c3_values(u64([0, 352, 1024]), u64([32, 32, 32]), a.ctypes.data, 4)
    ch = CodecChain.from_metadata([B("little"), GZ], "float32", 0, ctx)
    e = ch.encode_chunks(torch_cuda.from_numpy(a).cuda(), [32, 32, 32], [[0, 0, 0]])[0]
    assert zlib.decompress(e.cpu().numpy().tobytes(), 31) == a.tobytes()
    fib = [1, 1]
    while len(fib) < 26:
        fib.append(fib[-1] + fib[-2])
    rng = np.random.default_rng(11)
    b = rng.permutation(np.repeat(np.arange(26, dtype=np.uint8) * 7, fib))
    chb = CodecChain.from_metadata([B("little"), GZ], "uint8", 0, ctx)
    n = len(b)
    e = chb.encode_chunks(torch_cuda.from_numpy(b).cuda(), [n], [[0]])[0]
    assert zlib.decompress(e.cpu().numpy().tobytes(), 31) == b.tobytes()


def test_sharding_gzip_encode_c3_chain(ctx, torch_cuda):
    """ShardingCodecBound::encode over SURVEY C3's exact inner chain ([bytes, gzip 1, crc32c], index
    [bytes, crc32c] at the end) on the GPU: shards decode through the oracle (zlib) and the GPU to
    the array; an all-fill inner chunk is omitted from the shard."""
    from zarrs_amd import CodecChain, make_desc
    codecs = [{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [16, 16, 16], "codecs": [B("little"), GZ, CRC],
        "index_codecs": [B("little"), CRC], "index_location": "end"}}]
    shape, cs = [64, 64, 48], [32, 32, 48]
    a = _c3_values(shape)
    a[0:16, 0:16, 0:16] = 0  # fill value: omitted inner chunk
    co = O.OracleChain.from_metadata(codecs, "float32", 0.0, 3)
    ch = CodecChain.from_metadata(codecs, "float32", 0.0, ctx)
    x = torch_cuda.from_numpy(a).cuda()
    grid = [-(-s // c) for s, c in zip(shape, cs)]
    starts = [[i * c for i, c in zip(idx, cs)] for idx in np.ndindex(*grid)]
    enc = ch.encode_chunks(x, cs, starts)
    for st, e in zip(starts, enc):
        blk = a[st[0]:st[0] + 32, st[1]:st[1] + 32, :]
        assert np.array_equal(co.decode(e.cpu().numpy().tobytes(), cs), blk), st
    idx = np.frombuffer(enc[0].cpu().numpy().tobytes()[-(12 * 16 + 4):-4], np.uint64).reshape(-1, 2)
    assert idx[0].tolist() == [2 ** 64 - 1] * 2  # the all-fill inner chunk
    out = torch_cuda.zeros_like(x)
    descs = [make_desc(e, cs, out_start=st) for e, st in zip(enc, starts)]
    assert ch.decode_batch(descs, out, shape, enc_device=True) == [0] * len(enc)
    assert torch_cuda.equal(out, x)


# ---- zstd ----------------------------------------------------------------------------------------
ZS = {"name": "zstd", "configuration": {"level": 3, "checksum": False}}
ZS_CK = {"name": "zstd", "configuration": {"level": 3, "checksum": True}}
SHUF2 = {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}}


def _c5_level(shape, seed=42):
    rng = np.random.default_rng(seed)
    z, y, x = np.meshgrid(*[np.arange(n) for n in shape], indexing="ij")
    img = 100 + 3000 * np.exp(-((y - shape[1] / 2) ** 2 + (x - shape[2] / 3) ** 2) / (2 * 20.0 ** 2)) * (1 + 0 * z)
    img = img + np.sqrt(img) * rng.standard_normal(shape)
    return np.clip(img, 0, 65535).astype(np.uint16)


@pytest.mark.parametrize("chain", ["zstd", "zstd_checksum", "zstd_crc", "c5_shuffle_zstd"])
def test_zstd_encode_decodes_with_libzstd(ctx, torch_cuda, chain):
    """ZstdCodec::encode on the GPU (k_zstd_encode): every frame decodes through the oracle (libzstd,
    the reference's zstd-sys) to the exact chunk, and back through the GPU decoder."""
    from zarrs_amd import CodecChain, make_desc
    if chain == "c5_shuffle_zstd":
        codecs, dt = [B("little"), SHUF2, ZS], "uint16"
        shape, cs = [32, 128, 96], [16, 64, 96]
        contents = {"c5": _c5_level(shape), "zeros": np.zeros(shape, np.uint16),
                    "noise": np.random.default_rng(1).integers(0, 65536, shape).astype(np.uint16)}
    else:
        codecs = {"zstd": [B("little"), ZS], "zstd_checksum": [B("little"), ZS_CK],
                  "zstd_crc": [B("little"), ZS, CRC]}[chain]
        dt = "float32"
        shape, cs = [64, 64, 32], [32, 32, 32]
        contents = _contents(shape)
    co = O.OracleChain.from_metadata(codecs, dt, 0, 3)
    ch = CodecChain.from_metadata(codecs, dt, 0, ctx)
    for kind, a in contents.items():
        x = torch_cuda.from_numpy(a.view(np.int16) if dt == "uint16" else a).cuda()
        grid = [s // c for s, c in zip(shape, cs)]
        starts = [[i * c for i, c in zip(idx, cs)] for idx in np.ndindex(*grid)]
        enc = ch.encode_chunks(x, cs, starts)
        for st, e in zip(starts, enc):
            assert e.numel() <= ch.encoded_bound(cs)
            blk = a[tuple(slice(s0, s0 + c) for s0, c in zip(st, cs))]
            assert np.array_equal(co.decode(e.cpu().numpy().tobytes(), cs), blk), (chain, kind, st)
        out = torch_cuda.zeros_like(x)
        descs = [make_desc((e.data_ptr(), e.numel()), cs, out_start=st) for e, st in zip(enc, starts)]
        assert ch.decode_batch(descs, out, shape, enc_device=True) == [0] * len(enc)
        assert torch_cuda.equal(out, x), (chain, kind)


def test_zstd_encode_large_chunk_and_small_chunks(ctx, torch_cuda):
    """A 4 MiB chunk (16 superblocks of 64 blocks, matches reaching back across blocks and
    superblocks) and chunks of 1..600 bytes."""
    from zarrs_amd import CodecChain
    co = O.OracleChain.from_metadata([B("little"), ZS], "uint8", 0, 1)
    ch = CodecChain.from_metadata([B("little"), ZS], "uint8", 0, ctx)
    rng = np.random.default_rng(5)
    blk = rng.integers(0, 256, 3000, dtype=np.uint8)
    big = np.concatenate([np.tile(blk, 933), np.zeros(1 << 20, np.uint8), rng.integers(0, 4, 300000, dtype=np.uint8)])
    n = len(big)
    x = torch_cuda.from_numpy(big).cuda()
    enc = ch.encode_chunks(x, [n], [[0]])
    assert co.decode(enc[0].cpu().numpy().tobytes(), [n]).tobytes() == big.tobytes()
    assert enc[0].numel() < n // 2
    for m in (1, 2, 3, 4, 5, 7, 64, 255, 256, 257, 600):
        a = (np.arange(3 * m) % 5).astype(np.uint8)
        x = torch_cuda.from_numpy(a).cuda()
        enc = ch.encode_chunks(x, [m], [[0], [m], [2 * m]])
        for i, e in enumerate(enc):
            assert co.decode(e.cpu().numpy().tobytes(), [m]).tobytes() == a[i * m:(i + 1) * m].tobytes(), m


def test_zstd_encode_many_segmented_chunks(ctx, torch_cuda):
    """32 chunks of 16 MiB (16 one-wave segments each, 512 segment units): every frame, assembled
    from its segments, decodes through libzstd. Half the chunks have an all-zero high byte plane
    (RLE-literal blocks whose matches reach back across segment cuts)."""
    from zarrs_amd import CodecChain
    codecs = [B("little"), SHUF2, ZS]
    co = O.OracleChain.from_metadata(codecs, "uint16", 0, 3)
    ch = CodecChain.from_metadata(codecs, "uint16", 0, ctx)
    g = torch_cuda.Generator(device="cuda").manual_seed(7)
    x = torch_cuda.randint(0, 200, [32 * 32, 512, 512], device="cuda", generator=g, dtype=torch_cuda.int32)
    x[16 * 32:] += 3000
    x = x.to(torch_cuda.int16)
    starts = [[i * 32, 0, 0] for i in range(32)]
    enc = ch.encode_chunks(x, [32, 512, 512], starts)
    for i, e in enumerate(enc):
        d = co.decode(e.cpu().numpy().tobytes(), [32, 512, 512])
        assert np.array_equal(d.view(np.int16), x[i * 32:(i + 1) * 32].cpu().numpy()), i


def test_zstd_encode_ratio_vs_libzstd_level3(ctx, torch_cuda):
    """Compression of SURVEY C5-like data ([bytes, shuffle 2, zstd 3] u16) against libzstd level 3:
    reported; the GPU frames use Huffman literals and predefined FSE sequence tables (an encoder
    choice, zstd_codec.rs:100-111)."""
    from zarrs_amd import CodecChain
    codecs = [B("little"), SHUF2, ZS]
    co = O.OracleChain.from_metadata(codecs, "uint16", 0, 3)
    ch = CodecChain.from_metadata(codecs, "uint16", 0, ctx)
    a = _c5_level([64, 128, 128])
    cs = [32, 128, 128]
    x = torch_cuda.from_numpy(a.view(np.int16)).cuda()
    enc = ch.encode_chunks(x, cs, [[0, 0, 0], [32, 0, 0]])
    gpu = sum(e.numel() for e in enc)
    ref = sum(len(co.encode(np.ascontiguousarray(a[i:i + 32]))) for i in (0, 32))
    print(f"zstd encode on C5-like data: GPU {gpu} B, libzstd-3 {ref} B, ratio {gpu / ref:.3f}, "
          f"raw {a.nbytes} B")
    assert gpu < a.nbytes


def BL(cname, shuffle, typesize, blocksize=0, clevel=5):
    return {"name": "blosc", "configuration": {"cname": cname, "clevel": clevel, "shuffle": shuffle,
                                               "typesize": typesize, "blocksize": blocksize}}


BLOSC_CHAINS = {
    "lz4_shuffle_f32": ([B("little"), BL("lz4", "shuffle", 4)], "float32"),
    "lz4_noshuffle_f32": ([B("little"), BL("lz4", "noshuffle", 4)], "float32"),
    "lz4_bitshuffle_f32": ([B("little"), BL("lz4", "bitshuffle", 4)], "float32"),
    "lz4hc_shuffle_blocks_f32": ([B("little"), BL("lz4hc", "shuffle", 4, blocksize=10000)], "float32"),
    "zstd_shuffle_f32": ([B("little"), BL("zstd", "shuffle", 4)], "float32"),
    "zstd_bitshuffle_blocks_f32": ([B("little"), BL("zstd", "bitshuffle", 4, blocksize=24000)], "float32"),
    "lz4_shuffle_crc_f32": ([B("little"), BL("lz4", "shuffle", 4), {"name": "crc32c"}], "float32"),
    "blosclz_shuffle_f32": ([B("little"), BL("blosclz", "shuffle", 4)], "float32"),
    "blosclz_noshuffle_blocks_f32": ([B("little"), BL("blosclz", "noshuffle", 4, blocksize=100000)], "float32"),
    "zlib_shuffle_f32": ([B("little"), BL("zlib", "shuffle", 4)], "float32"),
    "zlib_bitshuffle_blocks_f32": ([B("little"), BL("zlib", "bitshuffle", 4, blocksize=24000)], "float32"),
    "zlib_noshuffle_crc_f32": ([B("little"), BL("zlib", "noshuffle", 4), {"name": "crc32c"}], "float32"),
}


@pytest.mark.parametrize("name", sorted(BLOSC_CHAINS))
def test_blosc_encode_decodes_with_c_blosc(ctx, torch_cuda, name):
    """BloscCodec::encode on the GPU (blosc_enc.hip: shuffle / bitshuffle, blosclz / lz4 / zlib / zstd streams,
    zlib / zstd / blosclz streams, stored streams and memcpyed frames where compression does not help): every frame decodes
    through the oracle (c-blosc 1.21, the library zarrs' blosc codec wraps) to the exact chunk, and
    back through the GPU decoder. Block sizes that leave a short last block exercise split and
    unsplit blocks and bitshuffle's unshuffled tail."""
    from zarrs_amd import CodecChain, make_desc
    codecs, dt = BLOSC_CHAINS[name]
    co = O.OracleChain.from_metadata(codecs, dt, 0, 3)
    ch = CodecChain.from_metadata(codecs, dt, 0, ctx)
    cs = [32, 32, 32]
    for kind, a in _contents([64, 64, 32]).items():
        x = torch_cuda.from_numpy(a).cuda()
        starts = [[i, j, 0] for i in (0, 32) for j in (0, 32)]
        enc = ch.encode_chunks(x, cs, starts)
        for st, e in zip(starts, enc):
            got = e.cpu().numpy().tobytes()
            assert len(got) <= ch.encoded_bound(cs)
            blk = np.ascontiguousarray(a[st[0]:st[0] + 32, st[1]:st[1] + 32, :])
            assert np.array_equal(co.decode(got, cs), blk), (name, kind, st)
        out = torch_cuda.zeros_like(x)
        descs = [make_desc((e.data_ptr(), e.numel()), cs, out_start=st) for e, st in zip(enc, starts)]
        assert ch.decode_batch(descs, out, list(x.shape), enc_device=True) == [0] * len(enc)
        assert torch_cuda.equal(out, x), (name, kind)


def test_blosc_encode_u16_ratio_and_small_chunks(ctx, torch_cuda):
    """u16 C5-like data through blosc lz4 + byte shuffle (numcodecs' Blosc defaults): the size
    against c-blosc's own encoding is reported; 1..600-byte chunks round-trip (memcpyed / short
    frames)."""
    from zarrs_amd import CodecChain
    codecs = [B("little"), BL("lz4", "shuffle", 2)]
    co = O.OracleChain.from_metadata(codecs, "uint16", 0, 3)
    ch = CodecChain.from_metadata(codecs, "uint16", 0, ctx)
    a = _c5_level([64, 128, 128])
    cs = [32, 128, 128]
    x = torch_cuda.from_numpy(a.view(np.int16)).cuda()
    enc = ch.encode_chunks(x, cs, [[0, 0, 0], [32, 0, 0]])
    for i, e in enumerate(enc):
        assert np.array_equal(co.decode(e.cpu().numpy().tobytes(), cs), a[32 * i:32 * (i + 1)])
    gpu = sum(e.numel() for e in enc)
    ref = sum(len(co.encode(np.ascontiguousarray(a[i:i + 32]))) for i in (0, 32))
    print(f"blosc lz4 encode on C5-like data: GPU {gpu} B, c-blosc {ref} B, ratio {gpu / ref:.3f}, raw {a.nbytes} B")
    assert gpu < a.nbytes
    co8 = O.OracleChain.from_metadata([B("little"), BL("lz4", "shuffle", 1)], "uint8", 0, 1)
    ch8 = CodecChain.from_metadata([B("little"), BL("lz4", "shuffle", 1)], "uint8", 0, ctx)
    for m in (1, 5, 12, 13, 64, 600):
        v = (np.arange(3 * m) % 7).astype(np.uint8)
        enc = ch8.encode_chunks(torch_cuda.from_numpy(v).cuda(), [m], [[0], [m], [2 * m]])
        for i, e in enumerate(enc):
            assert co8.decode(e.cpu().numpy().tobytes(), [m]).tobytes() == v[i * m:(i + 1) * m].tobytes(), m


def _snappy_decode(z: bytes) -> bytes:
    """google/snappy format_description.txt (the same decoder tests/test_snappy_writer.py pins)."""
    import test_snappy_writer as W
    return W._snappy_decode(z)


def _blosc_snappy_frame_decode(f: bytes) -> bytes:
    """A c-blosc 1.x frame with snappy streams, decoded here (the host c-blosc has no snappy):
    header, bstarts, per block its split streams ({csize, snappy stream} or stored when csize == the
    stream's size), then byte- or bit-unshuffle (blosc.c blosc_d / shuffle.c)."""
    import struct
    ver, vlz, flags, ts = f[0], f[1], f[2], f[3]
    nbytes, bsize, cbytes = struct.unpack_from("<3I", f, 4)
    assert ver == 2 and cbytes == len(f)
    if flags & 2:  # memcpyed
        return bytes(f[16:16 + nbytes])
    assert (flags >> 5) == 2, "snappy streams"
    nblk = (nbytes + bsize - 1) // bsize
    bstarts = struct.unpack_from("<%di" % nblk, f, 16)
    out = bytearray()
    for b in range(nblk):
        bs = min(bsize, nbytes - b * bsize)
        leftover = bs < bsize
        nsplit = ts if (not (flags & 0x10) and not leftover) else 1
        ne = bs // nsplit
        p = bstarts[b]
        blk = bytearray()
        for _ in range(nsplit):
            (cs,) = struct.unpack_from("<i", f, p)
            p += 4
            z = f[p:p + cs]
            p += cs
            blk += z if cs == ne else _snappy_decode(bytes(z))
        assert len(blk) == bs
        v = np.frombuffer(bytes(blk), np.uint8)
        if flags & 1 and ts > 1:  # byte shuffle
            neb = bs // ts
            body = v[:neb * ts].reshape(ts, neb).T.reshape(-1)
            v = np.concatenate([body, v[neb * ts:]])
        elif flags & 4 and ts >= 1 and bs >= ts:  # bitshuffle (element count a multiple of 8)
            n = bs // ts
            if n % 8 == 0:
                bits = np.unpackbits(v[:n * ts].reshape(8 * ts, n // 8), axis=1, bitorder="little")
                v = np.packbits(bits.reshape(ts, 8, n).transpose(2, 0, 1), axis=2, bitorder="little").reshape(-1)
                v = np.concatenate([v, np.frombuffer(bytes(blk), np.uint8)[n * ts:]])
        out += v.tobytes()
    return bytes(out)


SNAPPY_CHAINS = {
    "snappy_shuffle_f32": ([B("little"), BL("snappy", "shuffle", 4)], "float32"),
    "snappy_noshuffle_blocks_f32": ([B("little"), BL("snappy", "noshuffle", 4, blocksize=10000)], "float32"),
    "snappy_bitshuffle_f32": ([B("little"), BL("snappy", "bitshuffle", 4)], "float32"),
    "snappy_shuffle_crc_u16": ([B("little"), BL("snappy", "shuffle", 2), {"name": "crc32c"}], "uint16"),
}


@pytest.mark.parametrize("name", sorted(SNAPPY_CHAINS))
def test_blosc_snappy_encode(ctx, torch_cuda, name):
    """BloscCodec::encode with snappy streams (blosc_via_blosc_src.rs:57 maps BloscCompressor::Snappy):
    k_lz4_encode's LZ77 parse emitted as snappy elements (literals, 1- and 2-byte-offset copies,
    long matches as several copies). Parity unpinned (no snappy library or fixture in the image):
    every frame is decoded here from the format description and by the GPU decoder, to the exact
    chunk."""
    import struct
    from zarrs_amd import CodecChain, make_desc
    codecs, dt = SNAPPY_CHAINS[name]
    ch = CodecChain.from_metadata(codecs, dt, 0, ctx)
    crc = codecs[-1]["name"] == "crc32c"
    cs = [32, 32, 32]
    for kind, a in _contents([64, 64, 32]).items():
        if dt == "uint16":
            a = (a.view(np.uint32) & 0xFFFF).astype(np.uint16)
        x = torch_cuda.from_numpy(a.view(np.int16) if dt == "uint16" else a).cuda()
        starts = [[i, j, 0] for i in (0, 32) for j in (0, 32)]
        enc = ch.encode_chunks(x, cs, starts)
        for st, e in zip(starts, enc):
            got = e.cpu().numpy().tobytes()
            if crc:
                assert struct.unpack("<I", got[-4:])[0] == O.crc32c(got[:-4])
                got = got[:-4]
            blk = np.ascontiguousarray(a[st[0]:st[0] + 32, st[1]:st[1] + 32, :])
            assert _blosc_snappy_frame_decode(got) == blk.tobytes(), (name, kind, st)
        out = torch_cuda.zeros_like(x)
        descs = [make_desc((e.data_ptr(), e.numel()), cs, out_start=st) for e, st in zip(enc, starts)]
        assert ch.decode_batch(descs, out, list(x.shape), enc_device=True) == [0] * len(enc)
        assert torch_cuda.equal(out, x), (name, kind)
