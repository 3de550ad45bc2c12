"""GPU stress parity for the entropy stages: many gzip / zstd streams of varied content decoded in
one batch, compared byte-for-byte with the oracle (zlib / libzstd restatement of flate2 / zstd-sys)."""
import zlib

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

BYTES_LE = {"name": "bytes", "configuration": {"endian": "little"}}


def _content(rng, n, kind):
    if kind == "random":
        return rng.integers(0, 256, n, dtype=np.uint8)
    if kind == "text":
        words = [b"zarr", b"chunk", b"shard", b"decode", b"gpu", b"mi355x", b"codec", b" ", b"\n"]
        out = b"".join(words[i] for i in rng.integers(0, len(words), n))
        return np.frombuffer(out[:n], dtype=np.uint8).copy()
    if kind == "smooth":  # quantised smooth float field
        x = np.arange(n // 4, dtype=np.float32)
        f = np.round((np.sin(0.05 * x) + np.cos(0.003 * x)) * 256) / 256
        return f.astype(np.float32).view(np.uint8)[:n].copy()
    if kind == "runs":
        v = rng.integers(0, 4, n // 100 + 1, dtype=np.uint8)
        return np.repeat(v, 100)[:n].copy()
    if kind == "far":  # repeats at distances near the 32 KiB window limit
        blk = rng.integers(0, 256, 30000, dtype=np.uint8)
        return np.tile(blk, n // 30000 + 1)[:n].copy()
    if kind == "vfar":  # repeats 100,000 bytes back: zstd sources beyond the 64 KiB LDS ring
        blk = rng.integers(0, 256, 100000, dtype=np.uint8)
        return np.tile(blk, n // 100000 + 1)[:n].copy()
    if kind == "periods":  # runs of short odd / even periods and lengths: overlapping copies
        out, size = [], 0
        while size < n:
            p = int(rng.choice([1, 2, 3, 5, 7, 12, 17, 24, 40]))
            ln = int(rng.integers(20, 3000))
            pat = rng.integers(0, 256, p, dtype=np.uint8)
            out.append(np.tile(pat, ln // p + 1)[:ln])
            out.append(rng.integers(0, 256, int(rng.integers(0, 40)), dtype=np.uint8))
            size += ln + len(out[-1])
        return np.concatenate(out)[:n].copy()
    if kind == "direct":  # raw, rle and literal-only blocks, then matches reaching back into them
        r = rng.integers(0, 256, 150000, dtype=np.uint8)
        sk = np.minimum(rng.geometric(0.3, 150000), 255).astype(np.uint8)  # skewed: Huffman literals
        parts = [r, r[-5000:], r[60000:61000], np.zeros(300000, np.uint8), sk, sk[-3000:], r[:2000],
                 sk[1000:1500], r[140000:149000]]
        out = np.concatenate(parts)
        return np.tile(out, n // len(out) + 1)[:n].copy()
    if kind == "direct_period":  # a raw block ending a block boundary, then a long period-2/1 run from it
        r = rng.integers(0, 256, 131072, dtype=np.uint8)
        parts = [r, np.tile(r[-2:], 3000), rng.integers(0, 256, 131072 - 6000, dtype=np.uint8),
                 np.full(5000, r[-1], np.uint8), rng.integers(0, 256, 200000, dtype=np.uint8)]
        out = np.concatenate(parts)
        return np.tile(out, n // len(out) + 1)[:n].copy()
    raise ValueError(kind)


@pytest.mark.parametrize("level", [1, 6, 9])
def test_gzip_batch_vs_zlib(level):
    from zarrs_amd import CodecChain, Context, make_desc
    import torch
    rng = np.random.default_rng(level)
    codecs = [BYTES_LE, {"name": "gzip", "configuration": {"level": level}}]
    n = 131072
    kinds = ["random", "text", "smooth", "runs", "far", "periods"] * 8
    data = [_content(rng, n, k) for k in kinds]
    encs = []
    for d in data:
        c = zlib.compressobj(level, zlib.DEFLATED, 31)
        encs.append(c.compress(d.tobytes()) + c.flush())
    blob = b"".join(encs)
    dev = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    descs, off = [], 0
    for i, e in enumerate(encs):
        descs.append(make_desc((dev.data_ptr() + off, len(e)), [n], out_start=[i * n]))
        off += len(e)  # unaligned stream starts on purpose
    ch = CodecChain.from_metadata(codecs, "uint8", 0, Context.default())
    out = torch.zeros(len(encs) * n, dtype=torch.uint8, device="cuda")
    st = ch.decode_batch(descs, out, [len(encs) * n], enc_device=True)
    assert st == [0] * len(encs)
    got = out.cpu().numpy().reshape(len(encs), n)
    for i, d in enumerate(data):
        assert np.array_equal(got[i], d), (i, kinds[i])


@pytest.mark.parametrize("strategy", ["stored", "fixed", "rle", "huffman_only", "filtered"])
def test_gzip_block_types_vs_zlib(strategy):
    """Every DEFLATE block type and symbol mix the decoder's paths distinguish: stored blocks (level
    0), fixed-Huffman blocks (Z_FIXED), run-length matches at distance 1 (Z_RLE: overlapping copies,
    long matches), literal-only dynamic blocks (Z_HUFFMAN_ONLY), and Z_FILTERED; varied content and
    lengths, unaligned stream starts, one batch per strategy."""
    from zarrs_amd import CodecChain, Context, make_desc
    import torch
    rng = np.random.default_rng(zlib.crc32(strategy.encode()))
    level, strat = {"stored": (0, zlib.Z_DEFAULT_STRATEGY), "fixed": (6, zlib.Z_FIXED), "rle": (6, zlib.Z_RLE),
                    "huffman_only": (6, zlib.Z_HUFFMAN_ONLY), "filtered": (6, zlib.Z_FILTERED)}[strategy]
    kinds = ["random", "text", "smooth", "runs", "far", "periods"] * 3
    sizes = [int(v) for v in rng.integers(1, 200000, len(kinds))]
    n = max(sizes)
    data = [_content(rng, max(sz, 200), k)[:sz] for sz, k in zip(sizes, kinds)]
    encs = []
    for d in data:
        c = zlib.compressobj(level, zlib.DEFLATED, 31, 8, strat)
        encs.append(c.compress(d.tobytes()) + c.flush())
    blob = b"".join(encs)
    dev = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    ch = CodecChain.from_metadata([BYTES_LE, {"name": "gzip", "configuration": {"level": max(level, 1)}}], "uint8",
                                  0, Context.default())
    off = 0
    for i, (d, e) in enumerate(zip(data, encs)):  # one decode per stream (each has its own length)
        out = torch.zeros(len(d), dtype=torch.uint8, device="cuda")
        st = ch.decode_batch([make_desc((dev.data_ptr() + off, len(e)), [len(d)])], out, [len(d)], enc_device=True)
        off += len(e)
        assert st == [0], (i, kinds[i], len(d))
        assert np.array_equal(out.cpu().numpy(), d), (i, kinds[i], len(d))


def test_gzip_header_fields_and_trailing_member():
    """FEXTRA/FNAME/FCOMMENT headers; a second member after the first is ignored (GzDecoder)."""
    from zarrs_amd import CodecChain
    import gzip
    import struct
    rng = np.random.default_rng(3)
    d = _content(rng, 5000, "text")
    raw = zlib.compressobj(6, zlib.DEFLATED, -15)
    body = raw.compress(d.tobytes()) + raw.flush()
    hdr = b"\x1f\x8b\x08" + bytes([4 | 8 | 16]) + b"\0\0\0\0\0\xff"
    hdr += struct.pack("<H", 5) + b"extra" + b"name.bin\0" + b"a comment\0"
    trailer = struct.pack("<II", zlib.crc32(d.tobytes()), len(d))
    enc = hdr + body + trailer + gzip.compress(b"second member")
    assert O.OracleChain.from_metadata([BYTES_LE, {"name": "gzip"}], "uint8", 0, 1).decode(enc, [5000]).tobytes() \
        == d.tobytes()
    ch = CodecChain.from_metadata([BYTES_LE, {"name": "gzip"}], "uint8", 0)
    assert np.array_equal(ch.decode(enc, [5000]), d)


def test_gzip_size_mismatch():
    from zarrs_amd import CodecChain, ZgpuError
    import gzip
    ch = CodecChain.from_metadata([BYTES_LE, {"name": "gzip"}], "uint8", 0)
    with pytest.raises(ZgpuError) as ei:
        ch.decode(gzip.compress(b"x" * 100), [99])
    assert ei.value.status == 2
    with pytest.raises(ZgpuError) as ei:
        ch.decode(gzip.compress(b"x" * 100), [101])
    assert ei.value.status == 2


@pytest.mark.parametrize("level", [1, 3, 19])
def test_zstd_batch_vs_libzstd(level):
    from zarrs_amd import CodecChain, Context, make_desc
    import torch
    rng = np.random.default_rng(100 + level)
    codecs = [BYTES_LE, {"name": "zstd", "configuration": {"level": level, "checksum": level == 3}}]
    oc = O.OracleChain.from_metadata(codecs, "uint8", 0, 1)
    n = 131072
    kinds = ["random", "text", "smooth", "runs", "far"] * 4
    data = [_content(rng, n, k) for k in kinds]
    encs = [oc.encode(d) for d in data]
    blob = b"".join(encs)
    dev = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    descs, off = [], 0
    for i, e in enumerate(encs):
        descs.append(make_desc((dev.data_ptr() + off, len(e)), [n], out_start=[i * n]))
        off += len(e)
    ch = CodecChain.from_metadata(codecs, "uint8", 0, Context.default())
    out = torch.zeros(len(encs) * n, dtype=torch.uint8, device="cuda")
    st = ch.decode_batch(descs, out, [len(encs) * n], enc_device=True)
    assert st == [0] * len(encs)
    got = out.cpu().numpy().reshape(len(encs), n)
    for i, d in enumerate(data):
        assert np.array_equal(got[i], d), (i, kinds[i])


def _zstd_batch(codecs, encs, n_each, nd_shape=None):
    from zarrs_amd import CodecChain, Context, make_desc
    import torch
    blob = b"".join(encs)
    dev = torch.frombuffer(bytearray(blob), dtype=torch.uint8).cuda()
    descs, off = [], 0
    for i, e in enumerate(encs):
        descs.append(make_desc((dev.data_ptr() + off, len(e)), [n_each], out_start=[i * n_each]))
        off += len(e)
    ch = CodecChain.from_metadata(codecs, "uint8", 0, Context.default())
    out = torch.zeros(len(encs) * n_each, dtype=torch.uint8, device="cuda")
    try:
        st = ch.decode_batch(descs, out, [len(encs) * n_each], enc_device=True)
    except Exception as e:  # noqa: BLE001
        return getattr(e, "status", -1), None
    return st, out.cpu().numpy().reshape(len(encs), n_each)


@pytest.mark.parametrize("level", [1, 3, 19])
def test_zstd_multiblock_frames(level):
    """MiB-sized frames: many blocks per frame, treeless literals and repeat-mode FSE tables that
    the block-parallel path resolves to earlier blocks, repeat offsets across block boundaries."""
    rng = np.random.default_rng(200 + level)
    codecs = [BYTES_LE, {"name": "zstd", "configuration": {"level": level, "checksum": level != 1}}]
    oc = O.OracleChain.from_metadata(codecs, "uint8", 0, 1)
    n = 3 << 20
    kinds = ["random", "text", "smooth", "runs", "far", "vfar", "periods", "direct", "direct_period"]
    data = [_content(rng, n, k) for k in kinds]
    # C5-like: byte-shuffled u16 blobs + noise
    z = np.arange(n // 2, dtype=np.float32)
    u16 = np.clip(100 + 3000 * np.exp(-((z % 65536) - 30000) ** 2 / 2e7) + rng.normal(0, 10, n // 2), 0,
                  65535).astype(np.uint16)
    data.append(np.concatenate([u16.view(np.uint8)[0::2], u16.view(np.uint8)[1::2]]))
    kinds.append("shuffled_u16")
    encs = [oc.encode(d) for d in data]
    st, got = _zstd_batch(codecs, encs, n)
    assert st == [0] * len(encs)
    for i, d in enumerate(data):
        assert np.array_equal(got[i], d), (i, kinds[i])


@pytest.mark.parametrize("level", [3, 9])
def test_zstd_frames_beyond_the_scan_lds(level):
    """20 MiB frames: 160 blocks, more than k_zstd_scan's three-pass path holds in LDS (144 block
    records), so the frame is walked by the uniform scan and the sequence decoder parses the FSE table
    descriptions itself (no scan-parsed counts for these blocks); bit-exact vs libzstd."""
    rng = np.random.default_rng(300 + level)
    codecs = [BYTES_LE, {"name": "zstd", "configuration": {"level": level, "checksum": True}}]
    oc = O.OracleChain.from_metadata(codecs, "uint8", 0, 1)
    n = 20 << 20
    z = np.arange(n // 2, dtype=np.float32)
    u16 = np.clip(100 + 3000 * np.exp(-((z % 65536) - 30000) ** 2 / 2e7) + rng.normal(0, 10, n // 2), 0,
                  65535).astype(np.uint16)
    data = [_content(rng, n, "text"), np.concatenate([u16.view(np.uint8)[0::2], u16.view(np.uint8)[1::2]])]
    encs = [oc.encode(d) for d in data]
    st, got = _zstd_batch(codecs, encs, n)
    assert st == [0] * len(encs)
    for i, d in enumerate(data):
        assert np.array_equal(got[i], d), i


def test_zstd_concatenated_and_skippable_frames():
    """Several frames (and a skippable frame) in one chunk decode to the concatenation
    (zstd bulk decompress semantics, zstd_codec.rs:113-130)."""
    import struct
    rng = np.random.default_rng(5)
    codecs = [BYTES_LE, {"name": "zstd", "configuration": {"level": 3, "checksum": True}}]
    oc = O.OracleChain.from_metadata(codecs, "uint8", 0, 1)
    parts = [_content(rng, 300000, "text"), _content(rng, 70000, "smooth"), _content(rng, 500000, "runs")]
    skip = struct.pack("<II", 0x184D2A53, 7) + b"ignored"
    enc = oc.encode(parts[0]) + skip + oc.encode(parts[1]) + oc.encode(parts[2])
    n = sum(len(p) for p in parts)
    st, got = _zstd_batch(codecs, [enc], n)
    assert st == [0]
    assert np.array_equal(got[0], np.concatenate(parts))


def test_zstd_corruption_detected():
    """A flipped byte inside a checksummed multi-block frame is reported as CORRUPT_STREAM, and the
    other chunks of the batch still decode."""
    rng = np.random.default_rng(6)
    codecs = [BYTES_LE, {"name": "zstd", "configuration": {"level": 3, "checksum": True}}]
    oc = O.OracleChain.from_metadata(codecs, "uint8", 0, 1)
    n = 1 << 20
    data = [_content(rng, n, "text"), _content(rng, n, "smooth")]
    encs = [oc.encode(d) for d in data]
    bad = bytearray(encs[0])
    bad[len(bad) // 2] ^= 0x40
    from zarrs_amd import CodecChain, Context, make_desc
    import torch
    ch = CodecChain.from_metadata(codecs, "uint8", 0, Context.default())
    out = np.zeros(2 * n, np.uint8)
    descs = [make_desc(bytes(bad), [n], out_start=[0]), make_desc(encs[1], [n], out_start=[n])]
    from zarrs_amd import ZgpuError
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch(descs, out, [2 * n], enc_device=False)
    assert ei.value.status in (2, 4)  # CORRUPT_STREAM (or a size mismatch it causes)
    assert np.array_equal(out[n:], data[1])


def _raw_block_frame(data: bytes, block: int) -> bytes:
    """A zstd frame of raw blocks of `block` bytes (RFC 8878: single segment, 2-byte content size),
    built by hand: more blocks than the block-parallel scratch holds send it to the serial decoder."""
    import struct
    n = len(data)
    assert 256 <= n < 65536 + 256
    out = bytearray(struct.pack("<IB", 0xFD2FB528, 0x60) + struct.pack("<H", n - 256))
    for off in range(0, n, block):
        part = data[off:off + block]
        last = 1 if off + block >= n else 0
        out += struct.pack("<I", last | (len(part) << 3))[:3] + part
    return bytes(out)


def _skippable(n: int) -> bytes:
    import struct
    return struct.pack("<II", 0x184D2A50, n - 8) + b"\0" * (n - 8)


def test_plan_reruns_when_input_needs_the_serial_decoder():
    """A plan whose executions had no item for the serial zstd decoder stops launching it; when the
    input bytes change so that one item needs it, zgpu_plan_status re-runs the execution with the
    kernel launched (both results exact, the serial counter reports the item)."""
    import ctypes as C
    import torch
    from zarrs_amd import CodecChain, Context, make_desc
    from zarrs_amd import _lib as L
    lib = L.load()
    rng = np.random.default_rng(11)
    codecs = [BYTES_LE, {"name": "zstd", "configuration": {"level": 3, "checksum": False}}]
    oc = O.OracleChain.from_metadata(codecs, "uint8", 0, 1)
    n, k = 4096, 3
    data = [_content(rng, n, "text") for _ in range(k)]
    serial = _raw_block_frame(data[1].tobytes(), 40)  # 103 raw blocks > the 64-record scratch
    encs = [oc.encode(d) for d in data]
    L_item = max(len(serial), *[len(e) for e in encs]) + 16
    pad = [e + _skippable(L_item - len(e)) for e in encs]
    blob = torch.frombuffer(bytearray(b"".join(pad)), dtype=torch.uint8).cuda()
    descs = [make_desc((blob.data_ptr() + i * L_item, L_item), [n], out_start=[i * n]) for i in range(k)]
    ch = CodecChain.from_metadata(codecs, "uint8", 0, Context.default())
    arr = (L.ChunkDesc * k)(*descs)
    plan = C.c_void_p()
    L.check(lib.zgpu_plan_create(ch._h, 1, arr, k, L.u64s([k * n]), L.ENC_DEVICE | L.OUT_DEVICE, C.byref(plan)))
    try:
        out = torch.zeros(k * n, dtype=torch.uint8, device="cuda")
        st = (C.c_int32 * k)()
        ctr = (C.c_uint64 * L.N_COUNTERS)()
        for _ in range(2):  # all items on the block-parallel path; the second execution skips the fallback
            out.zero_()
            assert lib.zgpu_plan_execute(plan, out.data_ptr(), st, None) == 0
            assert np.array_equal(out.cpu().numpy(), np.concatenate(data))
            lib.zgpu_plan_counters(plan, ctr, L.N_COUNTERS)
            assert ctr[1] == 0 and ctr[2] == k
        # item 1 now holds the many-block frame (same padded length)
        blob[L_item:2 * L_item] = torch.frombuffer(bytearray(serial + _skippable(L_item - len(serial))),
                                                   dtype=torch.uint8).cuda()
        out.zero_()
        assert lib.zgpu_plan_execute(plan, out.data_ptr(), None, None) == 0  # asynchronous
        assert lib.zgpu_plan_status(plan, st, None) == 0
        assert list(st) == [0] * k
        assert np.array_equal(out.cpu().numpy(), np.concatenate(data))
        lib.zgpu_plan_counters(plan, ctr, L.N_COUNTERS)
        assert ctr[1] == 1 and ctr[2] == k - 1
    finally:
        lib.zgpu_plan_destroy(plan)
