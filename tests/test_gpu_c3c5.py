"""GPU parity for the exact BASELINE chains at reduced size, against the
CPU oracle on the same seeded inputs.

C3: sharding_indexed{chunk_shape [32]^3, codecs [bytes, gzip 1, crc32c], index [bytes, crc32c] at the
end} over a [512]^3 f32 array of [256]^3 shards, read whole and through partial subsets (full shards take
ShardingCodecBound::decode_into with inner crc32c verified, sharding_codec.rs:617-707; partial shards
take ShardingPartialDecoder, whose inner crc32c is stripped, not verified,
sharding_partial_decoder_sync.rs:311-400 + crc32c_codec.rs:143-158), with one empty inner chunk and one
corrupted inner checksum.

C5: [32,512,512] u16 chunks (16 MiB) through [bytes, numcodecs.shuffle{2}, zstd{3}], on the
block-parallel zstd path and forced onto the serial one-wave fallback decoder (zstd_codec.rs:113-130).
"""
import os
import struct
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

BYTES_LE = {"name": "bytes", "configuration": {"endian": "little"}}
C3_CODECS = [{"name": "sharding_indexed", "configuration": {
    "chunk_shape": [32, 32, 32],
    "codecs": [BYTES_LE, {"name": "gzip", "configuration": {"level": 1}}, {"name": "crc32c"}],
    "index_codecs": [BYTES_LE, {"name": "crc32c"}],
    "index_location": "end"}}]
SHARD, INNER, N = 256, 32, 512


def _c3_values(shape):
    """round(256*(sin .05x + cos .03y + .5 sin .07z) + N(0,1))/256, quantised like bench C3."""
    rng = np.random.default_rng(7)
    x = np.arange(shape[0], dtype=np.float32)[:, None, None]
    y = np.arange(shape[1], dtype=np.float32)[None, :, None]
    z = np.arange(shape[2], dtype=np.float32)[None, None, :]
    s = np.sin(0.05 * x) + np.cos(0.03 * y) + 0.5 * np.sin(0.07 * z)
    v = np.rint(256.0 * s + rng.standard_normal(shape, dtype=np.float32)) / 256.0
    return v.astype(np.float32)


def _index(shard: bytes, n_inner: int):
    tail = shard[len(shard) - (n_inner * 16 + 4):]
    return list(struct.unpack("<%dQ" % (2 * n_inner), tail[:-4]))


def _with_index(shard: bytes, n_inner: int, idx):
    body = shard[:len(shard) - (n_inner * 16 + 4)]
    raw = struct.pack("<%dQ" % (2 * n_inner), *idx)
    return body + raw + struct.pack("<I", O.crc32c(raw))


@pytest.fixture(scope="module")
def c3():
    a = _c3_values([N, N, N])
    co = O.OracleChain.from_metadata(C3_CODECS, "float32", 0.0, 3)
    keys = [(i, j, k) for i in range(2) for j in range(2) for k in range(2)]

    def enc(key):
        sl = tuple(slice(c * SHARD, (c + 1) * SHARD) for c in key)
        return co.encode(np.ascontiguousarray(a[sl]))
    with ThreadPoolExecutor(8) as ex:
        shards = dict(zip(keys, ex.map(enc, keys)))
    n_inner = (SHARD // INNER) ** 3
    # shard (0,0,1): inner chunk 5 empty (u64::MAX, u64::MAX) -> fill value (sharding_codec.rs:680-681)
    idx = _index(shards[(0, 0, 1)], n_inner)
    idx[10] = idx[11] = (1 << 64) - 1
    shards[(0, 0, 1)] = _with_index(shards[(0, 0, 1)], n_inner, idx)
    # shard (1,1,0): inner chunk 7's stored crc32c flipped -> InvalidChecksum on the full path only
    idx = _index(shards[(1, 1, 0)], n_inner)
    off, nb = idx[14], idx[15]
    bad = bytearray(shards[(1, 1, 0)])
    bad[off + nb - 2] ^= 0x10
    shards[(1, 1, 0)] = bytes(bad)
    return a, co, shards


def _array(shards, ctx, store, validate=True):
    from zarrs_amd import Array, DeviceStore, MemoryStore
    ms = MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in shards.items()})
    meta = {"shape": [N] * 3, "data_type": "float32", "fill_value": 0.0, "codecs": C3_CODECS,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": [SHARD] * 3}}}
    return Array(DeviceStore.from_store(ms) if store == "hbm" else ms, meta, ctx, validate_checksums=validate)


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    return Context(0)


@pytest.mark.parametrize("gz_direct", ["1", "0"], ids=["direct_rows", "slot_scatter"])
@pytest.mark.parametrize("gzip_kernel", ["pipelined", "one_wave"])
@pytest.mark.parametrize("store", ["hbm", "host"])
def test_c3_chain_full_and_partial(ctx, c3, store, gzip_kernel, gz_direct, monkeypatch):
    """Both k_gzip kernels: batches of <= 2048 streams take the two-wave pipelined one unless
    ZGPU_GZIP_PIPE_MAX (read per launch) lowers the threshold; 0 forces the one-wave kernel.
    gz_direct: whole inner chunks written into the output rows by k_gzip (ZGPU_GZIP_DIRECT, read per
    plan) or through the slot and the rows scatter."""
    from zarrs_amd import ZgpuError
    monkeypatch.setenv("ZGPU_GZIP_DIRECT", gz_direct)
    if gzip_kernel == "one_wave":
        monkeypatch.setenv("ZGPU_GZIP_PIPE_MAX", "0")
    a, co, shards = c3
    arr = _array(shards, ctx, store)
    # the whole array: shard (1,1,0) is fully covered -> its corrupted inner crc32c is verified
    with pytest.raises(ZgpuError) as ei:
        arr.retrieve_array_subset()
    assert ei.value.status == 1  # INVALID_CHECKSUM
    with pytest.raises(O.OracleError) as eo:
        O.retrieve_array_subset(co, [N] * 3, [SHARD] * 3, shards, [0] * 3, [N] * 3, nthreads=8)
    assert eo.value.status == 1
    subsets = [
        ([0, 0, 0], [N, SHARD, N]),            # shards (*,0,*) fully covered, incl. the empty inner chunk
        ([200, 300, 100], [268, 180, 300]),    # partial shards incl. (1,1,0): crc stripped, not verified
        ([256, 256, 0], [256, 256, 255]),      # (1,1,0) nearly whole: still the partial path
        ([0, 0, 256], [SHARD, SHARD, SHARD]),  # exactly shard (0,0,1): full path with an empty inner chunk
        ([37, 5, 290], [1, 1, 1]),             # one voxel
        ([250, 250, 250], [12, 12, 12]),       # straddles all 8 shards
    ]
    for start, sub in subsets:
        exp = O.retrieve_array_subset(co, [N] * 3, [SHARD] * 3, shards, start, sub, nthreads=8)
        got = arr.retrieve_array_subset(start, sub)
        assert got.tobytes() == exp.tobytes(), (start, sub)
    # the empty inner chunk reads as the fill value; the corrupted one reads as the original data
    sub = arr.retrieve_array_subset([0, 0, 256], [SHARD] * 3)
    assert not sub[0:32, 0:32, 160:192].any()
    assert np.array_equal(sub[:, :, :160], a[:SHARD, :SHARD, 256:416])
    got = arr.retrieve_array_subset([256, 256, 0], [256, 256, 255])
    assert np.array_equal(got, a[256:, 256:, :255])
    # shard (1,1,0) fully covered: the full path verifies -> error; validate_checksums=false decodes it
    with pytest.raises(ZgpuError) as ei:
        arr.retrieve_array_subset([256, 256, 0], [SHARD] * 3)
    assert ei.value.status == 1
    nov = _array(shards, ctx, store, validate=False)
    # the lone shard (512 streams: the pipelined kernel's latency mode unless forced off) without
    # validation: its corrupt inner crc32c is stripped, not checked (crc32c_codec.rs:108-141)
    got = nov.retrieve_array_subset([256, 256, 0], [SHARD] * 3)
    exp = O.retrieve_array_subset(co, [N] * 3, [SHARD] * 3, shards, [256, 256, 0], [SHARD] * 3, nthreads=8,
                                  validate_checksums=False)
    assert got.tobytes() == exp.tobytes()
    assert np.array_equal(got, a[256:, 256:, :256])
    exp = O.retrieve_array_subset(co, [N] * 3, [SHARD] * 3, shards, [0] * 3, [N] * 3, nthreads=8,
                                  validate_checksums=False)
    got = nov.retrieve_array_subset()
    assert got.tobytes() == exp.tobytes()
    exp_a = a.copy()
    exp_a[0:32, 0:32, 256 + 160:256 + 192] = 0
    assert np.array_equal(got, exp_a)


@pytest.mark.parametrize("gzip_kernel", ["pipelined", "one_wave", "one_wave_crc_fork"])
def test_c3_corrupt_gzip_header_checksum_first(ctx, c3, gzip_kernel, monkeypatch):
    """A corrupt gzip header inside an inner chunk: the chain decodes crc32c before gzip, so with the
    stored CRC-32C left as it was the full path reports INVALID_CHECKSUM (crc32c_codec.rs:108-141) on
    both gzip kernels (the pipelined one folds the check in); with the CRC-32C recomputed over the
    corrupt stream the gzip decoder's CORRUPT_STREAM (gzip_codec.rs:110-120); the partial path strips
    the CRC-32C unverified and reports CORRUPT_STREAM either way."""
    from zarrs_amd import ZgpuError
    if gzip_kernel.startswith("one_wave"):
        monkeypatch.setenv("ZGPU_GZIP_PIPE_MAX", "0")
    if gzip_kernel == "one_wave_crc_fork":  # the check on a side stream beside the decode (opt-in A/B)
        monkeypatch.setenv("ZGPU_GZIP_CRC_FORK", "1")
    a, co, shards = c3
    n_inner = (SHARD // INNER) ** 3
    key = (0, 1, 0)
    idx = _index(shards[key], n_inner)
    off, nb = idx[6], idx[7]  # inner chunk 3
    for fix_crc, full_status in ((False, 1), (True, 4)):
        bad = bytearray(shards[key])
        bad[off] ^= 0xFF  # gzip ID1 0x1f
        if fix_crc:
            bad[off + nb - 4:off + nb] = struct.pack("<I", O.crc32c(bytes(bad[off:off + nb - 4])))
        sh = dict(shards)
        sh[key] = bytes(bad)
        arr = _array(sh, ctx, "hbm")
        start = [0, SHARD, 0]
        with pytest.raises(ZgpuError) as ei:
            arr.retrieve_array_subset(start, [SHARD] * 3)
        assert ei.value.status == full_status, (fix_crc, ei.value.status)
        with pytest.raises(O.OracleError) as eo:
            O.retrieve_array_subset(co, [N] * 3, [SHARD] * 3, sh, start, [SHARD] * 3, nthreads=8)
        assert eo.value.status == full_status
        with pytest.raises(ZgpuError) as ei:  # partial: crc stripped, the gzip header fails
            arr.retrieve_array_subset([0, SHARD, 0], [SHARD - 1, SHARD, SHARD])
        assert ei.value.status == 4


def _c5_chunk(seed, shape=(32, 512, 512)):
    """Background 100 + Gaussian blobs + sqrt(mean) noise, u16 (bench C5 values)."""
    rng = np.random.default_rng(seed)
    z, y, x = (np.arange(n, dtype=np.float32) for n in shape)
    m = np.full(shape, 100.0, np.float32)
    for _ in range(6):
        cz, cy, cx = rng.uniform(0, shape[0]), rng.uniform(0, shape[1]), rng.uniform(0, shape[2])
        s, amp = rng.uniform(8, 60), rng.uniform(300, 4000)
        m += (amp * np.exp(-(z - cz) ** 2 / (2 * s * s))[:, None, None]
              * np.exp(-(y - cy) ** 2 / (2 * s * s))[None, :, None]
              * np.exp(-(x - cx) ** 2 / (2 * s * s))[None, None, :])
    v = np.rint(m + np.sqrt(m) * rng.standard_normal(shape, dtype=np.float32))
    return np.clip(v, 0, 65535).astype(np.uint16)


C5_CODECS = [BYTES_LE, {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
             {"name": "zstd", "configuration": {"level": 3, "checksum": False}}]


@pytest.mark.parametrize("force_serial,lits_first,xwin", [(False, False, 1), (False, False, 0), (True, False, 1),
                                                          (False, True, 1), (False, True, 0)],
                         ids=["block_parallel", "block_parallel_wave_exec", "serial_fallback",
                              "lits_first_one_stream", "lits_first_wave_exec"])
def test_c5_16mib_frames(ctx, force_serial, lits_first, xwin, monkeypatch):
    """Full-size C5 L0 chunks (16 MiB shuffled-u16 zstd frames): bit-exact vs libzstd through the oracle,
    and the path taken is the one asked for (device counters of the call). lits_first: one stream, the
    Huffman literals decoded before the sequences (ZGPU_ONE_STREAM | ZGPU_ZSTD_LITS_FIRST). xwin: the
    windowed workgroup executor (k_zstd_exec_win, default) or the per-segment wave executor."""
    import torch
    monkeypatch.setenv("ZGPU_ZSTD_XWIN", str(xwin))
    from zarrs_amd import CodecChain, make_desc
    from zarrs_amd import _lib as L
    co = O.OracleChain.from_metadata(C5_CODECS, "uint16", 0, 3)
    cs = [32, 512, 512]
    blocks = [_c5_chunk(s) for s in range(3)]
    encs = [co.encode(b) for b in blocks]
    for b, e in zip(blocks, encs):
        assert np.array_equal(co.decode(e, cs), b)
    devs = [torch.frombuffer(bytearray(e), dtype=torch.uint8).cuda() for e in encs]
    ch = CodecChain.from_metadata(C5_CODECS, "uint16", 0, ctx)
    out = torch.zeros([96, 512, 512], dtype=torch.int16, device="cuda")
    descs = [make_desc(d, cs, out_start=[32 * i, 0, 0]) for i, d in enumerate(devs)]
    old = os.environ.get("ZGPU_ZSTD_FORCE_SERIAL")
    os.environ["ZGPU_ZSTD_FORCE_SERIAL"] = "1" if force_serial else "0"
    try:
        extra = (L.ONE_STREAM | L.ZSTD_LITS_FIRST) if lits_first else 0
        st = ch.decode_batch(descs, out, [96, 512, 512], enc_device=True, flags=extra)
        ctr = L.last_counters()
    finally:
        if old is None:
            del os.environ["ZGPU_ZSTD_FORCE_SERIAL"]
        else:
            os.environ["ZGPU_ZSTD_FORCE_SERIAL"] = old
    assert st == [0, 0, 0]
    got = out.cpu().numpy().view(np.uint16)
    for i, b in enumerate(blocks):
        assert np.array_equal(got[32 * i:32 * (i + 1)], b), i
    if force_serial:
        assert ctr["zstd_serial"] == 3 and ctr["zstd_parallel"] == 0, ctr
    else:
        assert ctr["zstd_serial"] == 0 and ctr["zstd_parallel"] == 3, ctr


def test_size_mismatch_detail(ctx):
    """DECODED_SIZE_MISMATCH carries InvalidBytesLengthError{len, expected_len} (lib.rs:491-501,632)."""
    import gzip
    from zarrs_amd import CodecChain, ZgpuError
    from zarrs_amd import _lib as L
    ch = CodecChain.from_metadata([BYTES_LE, {"name": "gzip"}], "uint8", 0, ctx)
    with pytest.raises(ZgpuError) as ei:
        ch.decode(gzip.compress(b"x" * 100), [101])
    assert ei.value.status == 2
    assert L.last_size_mismatch() == (0, 100, 101)
    with pytest.raises(ZgpuError):  # within the slot's 256-B rounding: the decoded length is exact
        ch.decode(gzip.compress(b"x" * 100), [99])
    assert L.last_size_mismatch() == (0, 100, 99)
    with pytest.raises(ZgpuError):  # far beyond it: inflate stops at the slot, the total is unknown
        ch.decode(gzip.compress(b"x" * 5000), [99])
    assert L.last_size_mismatch() == (0, None, 99)
    raw = CodecChain.from_metadata([BYTES_LE, {"name": "crc32c"}], "uint16", 0, ctx)
    enc = np.arange(10, dtype=np.uint16).tobytes()
    enc += struct.pack("<I", O.crc32c(enc))
    with pytest.raises(ZgpuError):
        raw.decode(enc, [12])
    assert L.last_size_mismatch() == (0, 20, 24)
    assert raw.decode(enc, [10]).tolist() == list(range(10))
    assert L.last_size_mismatch() is None
