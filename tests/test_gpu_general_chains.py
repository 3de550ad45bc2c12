"""GPU parity of the chains one fused plan does not take, against the CPU oracle (bit-exact):
bytes->bytes codecs after sharding_indexed (a checksum / compressor over the whole shard), sharding
nested three deep, codecs around a nested sharding_indexed, and batches mixing chunk shapes.
zarrs composes any chain (codec_chain.rs:192-229) and decodes each chunk with its own shape;
libzgpu composes them from fused plans (zgpu.cpp decode_general)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

LEAF = [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "gzip", "configuration": {"level": 1}}]
IDX = [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}]


def sh(cs, inner, loc="end"):
    return {"name": "sharding_indexed",
            "configuration": {"chunk_shape": cs, "codecs": inner, "index_codecs": IDX, "index_location": loc}}


CHAINS = {
    "shard_gzip": [sh([4, 8, 8], LEAF), {"name": "gzip", "configuration": {"level": 5}}],
    "shard_crc": [sh([4, 8, 8], LEAF, "start"), {"name": "crc32c"}],
    "shard_crc_zstd": [sh([4, 8, 8], LEAF), {"name": "crc32c"},
                       {"name": "zstd", "configuration": {"level": 3, "checksum": True}}],
    "shard_blosc": [sh([4, 8, 8], [{"name": "bytes", "configuration": {"endian": "little"}}]),
                    {"name": "blosc", "configuration": {"cname": "lz4", "clevel": 5, "shuffle": "noshuffle",
                                                        "typesize": 1, "blocksize": 0}}],
    "deep3": [sh([8, 16, 16], [sh([4, 8, 8], [sh([2, 4, 4], LEAF)])])],
    "deep3_zstd_outer": [sh([8, 16, 16], [sh([4, 8, 8], [sh([2, 4, 4], LEAF)])]),
                         {"name": "zstd", "configuration": {"level": 1}}],
    "around_nested": [sh([8, 16, 16], [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
                                        sh([4, 8, 8], LEAF), {"name": "crc32c"}])],
    # transposes before a sharding the fused plan does not take: decoded in the encoded frame, then
    # transposed and scattered (zgpu.cpp transposed_general)
    "transpose_nested_zstd": [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
                              sh([8, 16, 8], [sh([4, 8, 4], LEAF)]),
                              {"name": "zstd", "configuration": {"level": 3, "checksum": False}}],
    "transpose_deep3": [{"name": "transpose", "configuration": {"order": [1, 2, 0]}},
                        {"name": "transpose", "configuration": {"order": [0, 2, 1]}},
                        sh([16, 8, 16], [sh([8, 4, 8], [sh([4, 2, 4], LEAF)])])],
    "transpose_around_nested": [{"name": "transpose", "configuration": {"order": [2, 0, 1]}},
                                sh([16, 8, 16], [{"name": "transpose", "configuration": {"order": [1, 0, 2]}},
                                                  sh([8, 4, 8], LEAF), {"name": "crc32c"}])],
}
SHAPE = [16, 32, 32]


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    return torch


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    return Context(0)


def _array(seed):
    rng = np.random.default_rng(seed)
    a = np.round(rng.standard_normal(SHAPE) * 20).astype(np.float32)
    a[8:16, 0:16, 16:32] = 3  # all-fill regions: omitted inner chunks / middle shards
    a[0:2, 0:4, 0:4] = 3
    return a


def _src(enc, torch, hbm):
    return torch.frombuffer(bytearray(enc), dtype=torch.uint8).cuda() if hbm else enc


@pytest.mark.parametrize("hbm", [True, False], ids=["hbm", "host"])
@pytest.mark.parametrize("name", sorted(CHAINS))
def test_general_chain_vs_oracle(ctx, torch_cuda, name, hbm):
    from zarrs_amd import CodecChain, make_desc
    codecs = CHAINS[name]
    a = _array(sorted(CHAINS).index(name))
    oc = O.OracleChain.from_metadata(codecs, "float32", 3, 3)
    enc = oc.encode(a)
    assert np.array_equal(oc.decode(enc, SHAPE), a)
    ch = CodecChain.from_metadata(codecs, "float32", 3, ctx)
    src = _src(enc, torch_cuda, hbm)
    for start, sub in (([0, 0, 0], SHAPE), ([3, 5, 7], [11, 20, 22]), ([9, 17, 1], [1, 1, 1])):
        out = np.zeros(sub, np.float32)
        st = ch.decode_batch([make_desc(src, SHAPE, start, sub)], out, sub, enc_device=hbm)
        assert st == [0]
        exp = a[tuple(slice(s, s + n) for s, n in zip(start, sub))]
        assert out.tobytes() == exp.tobytes(), (name, start, sub)


def test_general_chain_batch_two_shards_and_missing(ctx, torch_cuda):
    """Two shards of a [32,32,32] array plus a missing one in one batch, each with its own selection,
    into one output (the array read path: one descriptor per shard)."""
    from zarrs_amd import CodecChain, make_desc
    codecs = CHAINS["shard_crc_zstd"]
    oc = O.OracleChain.from_metadata(codecs, "float32", 3, 3)
    ch = CodecChain.from_metadata(codecs, "float32", 3, ctx)
    a0, a1 = _array(1), _array(2)
    e0, e1 = oc.encode(a0), oc.encode(a1)
    out = np.zeros([48, 32, 32], np.float32)
    descs = [make_desc(_src(e0, torch_cuda, True), SHAPE, [0, 0, 0], SHAPE, [0, 0, 0]),
             make_desc(_src(e1, torch_cuda, True), SHAPE, [4, 0, 0], [12, 32, 32], [16, 0, 0]),
             make_desc(None, SHAPE, [0, 0, 0], [4, 32, 32], [28, 0, 0])]
    assert ch.decode_batch(descs, out, [48, 32, 32], enc_device=True) == [0, 0, 0]
    assert out[:16].tobytes() == a0.tobytes()
    assert out[16:28].tobytes() == a1[4:].tobytes()
    assert np.all(out[28:32] == 3)


def test_whole_shard_checksum_full_vs_partial(ctx, torch_cuda):
    """crc32c over the whole shard: a corrupt checksum fails a full read (INVALID_CHECKSUM) and is
    stripped unverified on a partial read (Crc32cPartialDecoder, crc32c_codec.rs:108-158)."""
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    from zarrs_amd import _lib as L
    codecs = [sh([4, 8, 8], LEAF), {"name": "crc32c"}]
    a = _array(5)
    enc = bytearray(O.OracleChain.from_metadata(codecs, "float32", 3, 3).encode(a))
    enc[-1] ^= 0x5A
    ch = CodecChain.from_metadata(codecs, "float32", 3, ctx)
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch([make_desc(bytes(enc), SHAPE)], np.zeros(SHAPE, np.float32), SHAPE, enc_device=False)
    assert ei.value.status == L.INVALID_CHECKSUM
    sub = [8, 16, 16]
    out = np.zeros(sub, np.float32)
    assert ch.decode_batch([make_desc(bytes(enc), SHAPE, [2, 3, 4], sub)], out, sub, enc_device=False) == [0]
    assert out.tobytes() == a[2:10, 3:19, 4:20].tobytes()


def test_whole_shard_corrupt_stream(ctx, torch_cuda):
    """A corrupt whole-shard gzip stream fails like the oracle does, and only its descriptor."""
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    codecs = CHAINS["shard_gzip"]
    oc = O.OracleChain.from_metadata(codecs, "float32", 3, 3)
    a = _array(6)
    good = oc.encode(a)
    bad = bytearray(good)
    bad[len(bad) // 2] ^= 0xFF
    bad[len(bad) // 2 + 1] ^= 0xFF
    with pytest.raises(O.OracleError) as oe:
        oc.decode(bytes(bad), SHAPE)
    ch = CodecChain.from_metadata(codecs, "float32", 3, ctx)
    out = np.zeros([32, 32, 32], np.float32)
    descs = [make_desc(good, SHAPE, out_start=[0, 0, 0]), make_desc(bytes(bad), SHAPE, out_start=[16, 0, 0])]
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch(descs, out, [32, 32, 32], enc_device=False)
    assert ei.value.status == oe.value.status
    assert out[:16].tobytes() == a.tobytes()


def test_deep_nesting_index_errors(ctx, torch_cuda):
    """Three-deep sharding: an outer index entry past the shard -> SHARD_INDEX_OOB; a corrupt outer
    index -> INVALID_CHECKSUM (the host-resolved path keeps the fused path's statuses)."""
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    from zarrs_amd import _lib as L
    codecs = CHAINS["deep3"]
    a = _array(7)
    enc = O.OracleChain.from_metadata(codecs, "float32", 3, 3).encode(a)
    ch = CodecChain.from_metadata(codecs, "float32", 3, ctx)
    n1 = 8
    ib = len(enc) - 4 - 16 * n1
    bad = bytearray(enc)
    bad[ib:ib + 8] = (len(enc) + 100).to_bytes(8, "little")
    bad[-4:] = O.crc32c(bytes(bad[ib:-4])).to_bytes(4, "little")
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch([make_desc(bytes(bad), SHAPE)], np.zeros(SHAPE, np.float32), SHAPE, enc_device=False)
    assert ei.value.status == L.SHARD_INDEX_OOB
    bad2 = bytearray(enc)
    bad2[ib + 3] ^= 1
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch([make_desc(bytes(bad2), SHAPE)], np.zeros(SHAPE, np.float32), SHAPE, enc_device=False)
    assert ei.value.status == L.INVALID_CHECKSUM


@pytest.mark.parametrize("sharded", [False, True], ids=["chunks", "shards"])
def test_mixed_chunk_shapes_one_batch(ctx, torch_cuda, sharded):
    """Descriptors of different chunk shapes in one batch (zarrs decodes each chunk with its own
    shape, e.g. a rectilinear grid): one plan per shape, statuses in caller order."""
    from zarrs_amd import CodecChain, make_desc
    codecs = ([sh([2, 4, 4], LEAF)] if sharded else LEAF)
    oc = O.OracleChain.from_metadata(codecs, "float32", 0, 3)
    ch = CodecChain.from_metadata(codecs, "float32", 0, ctx)
    rng = np.random.default_rng(9)
    full = np.round(rng.standard_normal([24, 24, 24]) * 50).astype(np.float32)
    # a rectilinear split of [24,24,24]: axis 0 in [8, 16], the others whole
    parts = [(0, 8), (8, 16)]
    descs, exp_out = [], np.zeros([24, 24, 24], np.float32)
    for z0, zn in parts:
        c = full[z0:z0 + zn]
        e = oc.encode(c)
        descs.append(make_desc(_src(e, torch_cuda, True), list(c.shape), [0, 0, 0], list(c.shape), [z0, 0, 0]))
        exp_out[z0:z0 + zn] = oc.decode(e, c.shape)
    out = np.zeros([24, 24, 24], np.float32)
    assert ch.decode_batch(descs, out, [24, 24, 24], enc_device=True) == [0, 0]
    assert out.tobytes() == exp_out.tobytes() == full.tobytes()


def test_whole_shard_gzip_isize_hint_retried_alone(ctx, torch_cuda):
    """gzip's ISIZE (the decoded size mod 2^32, RFC 1952) only sizes the whole-shard slot: a member
    whose ISIZE understates it outgrows the slot and is re-run alone with 8x larger slots until it
    decodes; a member whose ISIZE then disagrees with its decoded size is corrupt (zlib and flate2
    reject it too), while the shards beside it decode normally."""
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    from zarrs_amd import _lib as L
    codecs = CHAINS["shard_gzip"]
    oc = O.OracleChain.from_metadata(codecs, "float32", 3, 3)
    a0, a1 = _array(11), _array(12)
    e0, e1 = oc.encode(a0), bytearray(oc.encode(a1))
    e1[-4:] = (64).to_bytes(4, "little")  # ISIZE understated
    with pytest.raises(O.OracleError) as oe:
        oc.decode(bytes(e1), SHAPE)
    ch = CodecChain.from_metadata(codecs, "float32", 3, ctx)
    out = np.zeros([32, 32, 32], np.float32)
    descs = [make_desc(e0, SHAPE, out_start=[0, 0, 0]), make_desc(bytes(e1), SHAPE, out_start=[16, 0, 0])]
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch(descs, out, [32, 32, 32], enc_device=False)
    assert ei.value.status == oe.value.status == L.CORRUPT_STREAM
    assert out[:16].tobytes() == a0.tobytes()
    # both members with understated ISIZE hints but intact streams are not possible (the trailer holds
    # ISIZE); a good member alone decodes from its own hint
    out2 = np.zeros(SHAPE, np.float32)
    assert ch.decode_batch([make_desc(e0, SHAPE)], out2, SHAPE, enc_device=False) == [0]
    assert out2.tobytes() == a0.tobytes()
