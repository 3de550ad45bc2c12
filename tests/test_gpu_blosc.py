"""GPU parity of the blosc codec against the reference's blosc fixtures
(zstd + bitshuffle, written by zarrs and zarr-python) and the CPU oracle (c-blosc 1.21, the library
zarrs' blosc-src binds) on seeded inputs: blosclz (c-blosc's default) / lz4 / lz4hc / zlib / zstd streams
(snappy: frames written by the test's own encoder, the host c-blosc has no snappy),
byte shuffle / bitshuffle / none, typesizes 1-8, forced block sizes (split streams, leftover blocks,
bitshuffle skipped for element counts that are not a multiple of 8), memcpyed frames, blosc inside
sharding. Bit-exact."""
import numpy as np
import pytest

import fixtures as F
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


@pytest.mark.parametrize("store", ["host", "hbm"])
@pytest.mark.parametrize("fixture", F.BLOSC)
def test_blosc_reference_fixture(ctx, torch_cuda, fixture, store):
    from zarrs_amd import Array, DeviceStore, MemoryStore
    m, chunks = F.load_array(fixture)
    meta = {"shape": m["shape"], "data_type": m["data_type"], "fill_value": m["fill_value"],
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": m["chunk_shape"]}},
            "codecs": m["codecs"]}
    ms = MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in chunks.items()})
    arr = Array(DeviceStore.from_store(ms) if store == "hbm" else ms, meta, ctx)
    exp = np.arange(100).reshape(10, 10).astype(np.float32)
    assert np.array_equal(arr.retrieve_array_subset(), exp)
    assert np.array_equal(arr.retrieve_array_subset([1, 2], [6, 5]), exp[1:7, 2:7])


def _blosc(cname, shuffle, ts, blocksize=0, clevel=5):
    return {"name": "blosc", "configuration": {"cname": cname, "clevel": clevel, "shuffle": shuffle,
                                               "typesize": ts, "blocksize": blocksize}}


DT = {1: "uint8", 2: "uint16", 4: "float32", 8: "float64"}
CASES = []
for cname in ("lz4", "zstd", "lz4hc", "blosclz", "zlib"):
    for sh in ("noshuffle", "shuffle", "bitshuffle"):
        for ts in (1, 2, 4, 8):
            CASES.append((cname, sh, ts))


def _data(rng, n, ts):
    a = rng.standard_normal(n) * 40
    a[: n // 2] = np.round(a[: n // 2])  # half compressible
    if ts == 1:
        return (a % 200).astype(np.uint8)
    if ts == 2:
        return np.abs(a).astype(np.uint16)
    return a.astype(DT[ts])


@pytest.mark.parametrize("cname,shuffle,ts", CASES, ids=[f"{c}-{s}-{t}" for c, s, t in CASES])
def test_blosc_batch_vs_oracle(ctx, torch_cuda, cname, shuffle, ts):
    """Batches of 3 chunks (one decode call per chunk shape: a plan has one leaf chunk shape)
    through the GPU stage, bytes vs the c-blosc oracle, device-resident inputs."""
    from zarrs_amd import CodecChain, make_desc
    rng = np.random.default_rng(ts * 7 + len(cname) + len(shuffle))
    # (elements, blocksize): single block, forced small blocks with a leftover, element counts that
    # are not a multiple of 8, a large chunk with automatic blocks
    specs = [(1, 0), (100, 0), (1000, 256), (4099, 1024), (33333, 0), (262147, 0), (5000, 4096)]
    # the GPU chain is parsed once; the decoder reads cname/shuffle/blocksize from each frame
    ch = CodecChain.from_metadata([{"name": "bytes", "configuration": {"endian": "little"}},
                                   _blosc(cname, shuffle, ts)], DT[ts], 0, ctx)
    for n, bsz in specs:
        codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc(cname, shuffle, ts, bsz)]
        co = O.OracleChain.from_metadata(codecs, DT[ts], 0, 1)
        descs, keep, exp = [], [], []
        for k in range(3):
            a = _data(rng, n, ts)
            enc = co.encode(a)
            assert np.array_equal(co.decode(enc, (n,)), a)
            d = torch_cuda.frombuffer(bytearray(enc), dtype=torch_cuda.uint8).cuda()
            keep.append(d)
            descs.append(make_desc(d, [n], out_start=[k * n]))
            exp.append(a)
        out = np.zeros(3 * n, DT[ts])
        st = ch.decode_batch(descs, out, [3 * n], enc_device=True)
        assert st == [0] * 3, (n, bsz)
        assert out.tobytes() == np.concatenate(exp).tobytes(), (n, bsz)


def test_blosc_memcpyed_and_errors(ctx, torch_cuda):
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    from zarrs_amd import _lib as L
    rng = np.random.default_rng(5)
    a = rng.random(3000).astype(np.float32)  # clevel 0 -> memcpyed frame
    codecs0 = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc("lz4", "shuffle", 4, clevel=0)]
    enc0 = O.OracleChain.from_metadata(codecs0, "float32", 0, 1).encode(a)
    assert enc0[2] & 0x2  # memcpyed
    ch = CodecChain.from_metadata(codecs0, "float32", 0, ctx)
    out = np.zeros(3000, np.float32)
    assert ch.decode_batch([make_desc(enc0, [3000])], out, [3000], enc_device=False) == [0]
    assert np.array_equal(out, a)
    # compressor formats 5-7 are not defined by c-blosc 1.x: UNSUPPORTED, loudly (a relabelled frame)
    codecs1 = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc("lz4", "shuffle", 4)]
    enc1 = bytearray(O.OracleChain.from_metadata(codecs1, "float32", 0, 1).encode(np.zeros(3000, np.float32) + 1))
    assert not enc1[2] & 0x2
    enc1[2] = (enc1[2] & 0x1F) | (5 << 5)
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch([make_desc(bytes(enc1), [3000])], out, [3000], enc_device=False)
    assert ei.value.status == L.UNSUPPORTED
    # zlib streams: a flipped Adler-32 trailer byte / a corrupt zlib header -> CORRUPT_STREAM
    codecs3 = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc("zlib", "shuffle", 4)]
    z = np.round(rng.standard_normal(3000) * 10).astype(np.float32)
    enc3 = bytearray(O.OracleChain.from_metadata(codecs3, "float32", 0, 1).encode(z))
    assert not enc3[2] & 0x2 and enc3[2] >> 5 == 3
    ch3 = CodecChain.from_metadata(codecs3, "float32", 0, ctx)
    assert ch3.decode_batch([make_desc(bytes(enc3), [3000])], out, [3000], enc_device=False) == [0]
    assert np.array_equal(out, z)
    # the first block's first compressed (not stored) stream: {csize i32, zlib stream}
    bsize = int.from_bytes(enc3[8:12], "little")
    nsplit = 1 if enc3[2] & 0x10 else 4
    p, tgt = int.from_bytes(enc3[16:20], "little"), None
    for _ in range(nsplit):
        cs = int.from_bytes(enc3[p:p + 4], "little")
        if cs != bsize // nsplit:
            tgt = (p + 4, cs)
            break
        p += 4 + cs
    assert tgt is not None
    for off in (tgt[0] + tgt[1] - 1, tgt[0]):  # last Adler-32 byte, CMF
        bad3 = bytearray(enc3)
        bad3[off] ^= 0x5A
        with pytest.raises(ZgpuError) as ei:
            ch3.decode_batch([make_desc(bytes(bad3), [3000])], out, [3000], enc_device=False)
        assert ei.value.status == L.CORRUPT_STREAM
    # corrupt lz4 stream / truncated frame / wrong decoded size
    codecs2 = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc("lz4", "shuffle", 4)]
    b = np.round(rng.standard_normal(3000) * 10).astype(np.float32)
    enc2 = bytearray(O.OracleChain.from_metadata(codecs2, "float32", 0, 1).encode(b))
    assert not enc2[2] & 0x2
    bad = bytearray(enc2)  # the first stream's compressed size points past the frame
    p0 = int.from_bytes(enc2[16:20], "little")
    bad[p0:p0 + 4] = (0x7FFFFFF0).to_bytes(4, "little")
    for e, want in ((bytes(bad), (L.CORRUPT_STREAM,)), (bytes(enc2[:10]), (L.CORRUPT_STREAM,)),
                    (bytes(enc2[:-5]), (L.CORRUPT_STREAM,))):
        with pytest.raises(ZgpuError) as ei:
            ch.decode_batch([make_desc(e, [3000])], out, [3000], enc_device=False)
        assert ei.value.status in want
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch([make_desc(bytes(enc2), [2000])], out[:2000], [2000], enc_device=False)
    assert ei.value.status == L.DECODED_SIZE_MISMATCH


@pytest.mark.parametrize("cname,shuffle,clevel", [("lz4", "shuffle", 5), ("blosclz", "shuffle", 9),
                                                  ("zstd", "bitshuffle", 3), ("lz4", "noshuffle", 0),
                                                  ("zlib", "shuffle", 1)])
def test_blosc_direct_output_rows(ctx, torch_cuda, cname, shuffle, clevel):
    """Whole chunks of a 3-D u16 array: blosc is the chain's last stage and the scatter would copy
    the rows unchanged, so k_blosc_finish writes the unshuffled rows straight into the output
    (ZG_ITEM_DIRECT, fast u16 path and the bitshuffle / memcpyed byte paths, forced small blocks);
    a missing chunk still takes the scatter's fill, a partial subset the slot path. vs the oracle."""
    from zarrs_amd import CodecChain, make_desc
    rng = np.random.default_rng(len(cname) + clevel)
    shape, cs = [4, 96, 512], [2, 48, 256]
    z, y, x = np.meshgrid(*[np.arange(n) for n in shape], indexing="ij")
    a = (500 + 300 * np.sin(y * 0.07) * np.cos(x * 0.05) + rng.integers(0, 40, shape)).astype(np.uint16)
    for bsz in (0, 4096):
        codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc(cname, shuffle, 2, bsz, clevel)]
        co = O.OracleChain.from_metadata(codecs, "uint16", 7, 1)
        ch = CodecChain.from_metadata(codecs, "uint16", 7, ctx)
        exp = a.copy()
        descs, keep = [], []
        for idx in np.ndindex(2, 2, 2):
            sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(idx, cs))
            o = [i * c for i, c in zip(idx, cs)]
            if idx == (1, 1, 0):  # missing chunk: fill value
                exp[sl] = 7
                descs.append(make_desc((0, 0), cs, out_start=o))
                continue
            d = torch_cuda.frombuffer(bytearray(co.encode(np.ascontiguousarray(a[sl]))), dtype=torch_cuda.uint8).cuda()
            keep.append(d)
            descs.append(make_desc(d, cs, out_start=o))
        out = torch_cuda.zeros(shape, dtype=torch_cuda.int16, device="cuda")
        assert ch.decode_batch(descs, out, shape, enc_device=True) == [0] * 8
        assert np.array_equal(out.cpu().numpy().view(np.uint16), exp), bsz
        # a partial selection of every chunk: the slot + scatter path
        sub = [make_desc((dd.enc, dd.enc_len), cs, sel_start=[1, 5, 16], sel_shape=[1, 40, 224],
                         out_start=[i * 1, 0, 0]) for i, dd in enumerate(descs[:4])]
        out2 = torch_cuda.zeros([4, 40, 224], dtype=torch_cuda.int16, device="cuda")
        assert ch.decode_batch(sub, out2, [4, 40, 224], enc_device=True) == [0] * 4
        for i in range(4):
            idx = list(np.ndindex(2, 2, 2))[i]
            src = exp[tuple(slice(j * c, (j + 1) * c) for j, c in zip(idx, cs))]
            assert np.array_equal(out2[i].cpu().numpy().view(np.uint16), src[1, 5:45, 16:240]), (bsz, i)


@pytest.mark.parametrize("clevel", [1, 5, 9])
def test_blosclz_streams_vs_cblosc(ctx, torch_cuda, clevel):
    """blosclz (c-blosc's default compressor, the one zarrs benchmarks: benches/codecs.rs:52): long
    runs, periodic data at distances past the 13-bit window (16-bit far matches, > 8191 back),
    random literals, u16 image-like data; byte-exact vs c-blosc 1.21 through the oracle."""
    from zarrs_amd import CodecChain, make_desc
    rng = np.random.default_rng(clevel)
    n = 1 << 20
    datas = [np.repeat(rng.integers(0, 6, n // 64, dtype=np.uint8), 64),
             np.tile(rng.integers(0, 256, 20000, dtype=np.uint8), n // 20000 + 1)[:n],
             np.tile(rng.integers(0, 256, 9000, dtype=np.uint8), n // 9000 + 1)[:n],
             rng.integers(0, 256, n, dtype=np.uint8),
             (100 + rng.poisson(30, n // 2)).astype(np.uint16).view(np.uint8),
             np.zeros(n, np.uint8)]
    for sh in ("noshuffle", "shuffle"):
        codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc("blosclz", sh, 2, clevel=clevel)]
        co = O.OracleChain.from_metadata(codecs, "uint16", 0, 1)
        encs = [co.encode(d.view(np.uint16)) for d in datas]
        ch = CodecChain.from_metadata(codecs, "uint16", 0, ctx)
        devs = [torch_cuda.frombuffer(bytearray(e), dtype=torch_cuda.uint8).cuda() for e in encs]
        descs = [make_desc(d, [n // 2], out_start=[k * (n // 2)]) for k, d in enumerate(devs)]
        out = np.zeros(len(datas) * n // 2, np.uint16)
        assert ch.decode_batch(descs, out, [out.size], enc_device=True) == [0] * len(datas)
        assert out.view(np.uint8).tobytes() == np.concatenate(datas).tobytes(), sh


@pytest.mark.parametrize("cname", ["lz4", "zstd", "blosclz"])
def test_blosc_inside_sharding_vs_oracle(ctx, torch_cuda, cname):
    from zarrs_amd import Array, DeviceStore, MemoryStore
    from test_gpu_parity import _encode_grid
    codecs = [{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [16, 16, 16],
        "codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc(cname, "shuffle", 2)],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}]}}]
    rng = np.random.default_rng(11)
    shape, cs = [70, 64, 50], [32, 32, 32]
    a = (np.abs(rng.standard_normal(shape)) * 300).astype(np.uint16)
    co = O.OracleChain.from_metadata(codecs, "uint16", 7, 3)
    chunks = _encode_grid(co, a, cs, drop={(1, 1, 0)})
    ms = MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in chunks.items()})
    meta = {"shape": shape, "data_type": "uint16", "fill_value": 7, "codecs": codecs,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": cs}}}
    arr = Array(DeviceStore.from_store(ms), meta, ctx)
    for start, sub in (([0, 0, 0], shape), ([5, 17, 3], [60, 40, 29])):
        exp = O.retrieve_array_subset(co, shape, cs, chunks, start, sub, nthreads=4)
        assert arr.retrieve_array_subset(start, sub).tobytes() == exp.tobytes(), (start, sub)


@pytest.mark.parametrize("cname", ["lz4", "zstd", "blosclz"])
def test_blosc_plan_cached_layout_and_rerun(ctx, torch_cuda, cname):
    """A plan's first execution reads the blosc headers back and records the stream-table sizes; later
    executions lay the table out on the device (no host round trip). Rewriting the device inputs in
    place with frames of more blocks / streams (smaller blocksize, shuffle split) makes the recorded
    layout too small: that execution is re-run with a read-back layout (ZGPU_CTR_BLOSC_RERUN = 1)
    and is still bit-exact; a smaller layout afterwards fits the larger capacities (inert tails)."""
    import ctypes as C
    from zarrs_amd import CodecChain, make_desc
    from zarrs_amd import _lib as L
    rng = np.random.default_rng(3)
    n, nchunk = 1 << 18, 4
    datas = [_data(rng, n, 2) for _ in range(nchunk)]
    # (shuffle, clevel) -> c-blosc's automatic blocksize: clevel 9 one 512 KiB block; clevel 1 8-16
    # blocks of 32-64 KiB; clevel 5 two blocks (blosclz: a memcpyed frame)
    variants = []
    for sh, cl in (("noshuffle", 9), ("shuffle", 1), ("noshuffle", 5)):
        codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc(cname, sh, 2, clevel=cl)]
        co = O.OracleChain.from_metadata(codecs, "uint16", 0, 1)
        variants.append([co.encode(d) for d in datas])
    cap = max(len(e) for v in variants for e in v)
    bufs = [torch_cuda.zeros(cap, dtype=torch_cuda.uint8, device="cuda") for _ in range(nchunk)]
    ch = CodecChain.from_metadata([{"name": "bytes", "configuration": {"endian": "little"}},
                                   _blosc(cname, "shuffle", 2)], "uint16", 0, ctx)
    descs = [make_desc(b, [n], out_start=[k * n]) for k, b in enumerate(bufs)]
    arr = (L.ChunkDesc * nchunk)(*descs)
    plan = C.c_void_p()
    L.check(L.load().zgpu_plan_create(ch._h, 1, arr, nchunk, L.u64s([nchunk * n]), L.ENC_DEVICE | L.OUT_DEVICE,
                                      C.byref(plan)))
    out = torch_cuda.empty(nchunk * n, dtype=torch_cuda.int16, device="cuda")
    st = (C.c_int32 * nchunk)()
    ctr = (C.c_uint64 * L.N_COUNTERS)()
    exp = np.concatenate(datas).view(np.int16)
    try:
        # (variant, expected rerun flag): first run reads back; same layout cached; grows -> rerun;
        # shrinks -> fits; back to the first -> fits
        for v, rerun in ((0, 0), (0, 0), (1, 1), (1, 0), (2, 0), (0, 0)):
            for b, e in zip(bufs, variants[v]):
                b.zero_()
                b[: len(e)] = torch_cuda.frombuffer(bytearray(e), dtype=torch_cuda.uint8).cuda()
            out.fill_(-1)
            torch_cuda.cuda.synchronize()
            L.check(L.load().zgpu_plan_execute(plan, out.data_ptr(), st, None))
            assert list(st) == [0] * nchunk, v
            assert np.array_equal(out.cpu().numpy(), exp), v
            L.load().zgpu_plan_counters(plan, ctr, L.N_COUNTERS)
            assert ctr[L.CTR_BLOSC_RERUN] == rerun, (v, list(ctr))
    finally:
        L.load().zgpu_plan_destroy(plan)


# ---- snappy streams (c-blosc compressor format 2) ------------------------------------------------
# The host c-blosc is built without snappy, so these frames are written here: a small snappy encoder
# (raw format, google/snappy format_description.txt) that emits every element form — inline and
# 1-4-byte literal lengths, copies with 1-, 2- and 4-byte offsets, overlapping copies — inside c-blosc
# 1.x frames (16-B header, bstarts, {csize, stream} per split; a stream whose compressed size would
# reach the split's size is stored). Parity unpinned (no snappy library in the image): checked by
# round trip against the encoded data.
def _varint(v):
    out = bytearray()
    while True:
        b = v & 127
        v >>= 7
        out.append(b | (128 if v else 0))
        if not v:
            return bytes(out)


def _snappy_literal(out, lit, rng):
    while lit:
        n = len(lit) if len(lit) <= 200 else int(rng.integers(1, len(lit) + 1))
        if n <= 60 and rng.random() < 0.7:
            out.append((n - 1) << 2)
        else:  # 60..63: the length - 1 in 1..4 little-endian bytes (any width that holds it is valid)
            nb = max(1, ((n - 1).bit_length() + 7) // 8)
            nb = min(4, nb + int(rng.integers(0, 2)))
            out.append((59 + nb) << 2)
            out += (n - 1).to_bytes(nb, "little")
        out += lit[:n]
        lit = lit[n:]


def _snappy_copy(out, off, n, rng):
    while n:
        if 4 <= n <= 11 and off < 2048 and rng.random() < 0.6:
            out.append(1 | ((n - 4) << 2) | ((off >> 8) << 5))
            out.append(off & 255)
            return
        m = min(n, 64)
        if n - m and n - m < 4:  # keep the remainder encodable (a copy of >= 1 byte is fine too)
            m = n - 4 if n > 4 else n
        if off < 65536 and rng.random() < 0.7:
            out.append(2 | ((m - 1) << 2))
            out += off.to_bytes(2, "little")
        else:
            out.append(3 | ((m - 1) << 2))
            out += off.to_bytes(4, "little")
        n -= m


def _snappy_compress(data, rng):
    out = bytearray(_varint(len(data)))
    table, i, lit0, n = {}, 0, 0, len(data)
    while i + 4 <= n:
        key = data[i:i + 4]
        j = table.get(key)
        table[key] = i
        if j is not None:
            m = 4
            while i + m < n and data[j + m] == data[i + m] and m < 300:
                m += 1
            _snappy_literal(out, data[lit0:i], rng)
            _snappy_copy(out, i - j, m, rng)
            i += m
            lit0 = i
        else:
            i += 1
    _snappy_literal(out, data[lit0:], rng)
    return bytes(out)


def _blosc_snappy_frame(data, ts, shuffle, blocksize, split, rng):
    nbytes = len(data)
    nblk = -(-nbytes // blocksize)
    left = nbytes % blocksize
    flags = (1 if shuffle else 0) | (0 if split else 0x10) | (2 << 5)
    body, starts = bytearray(), []
    hdr_len = 16 + 4 * nblk
    for b in range(nblk):
        src = data[b * blocksize:(b + 1) * blocksize]
        bsize = len(src)
        if shuffle and ts > 1:  # c-blosc shuffle: byte i of element j -> i * neb + j; the tail as is
            neb = bsize // ts
            a = np.frombuffer(src[:neb * ts], np.uint8).reshape(neb, ts).T.reshape(-1).tobytes()
            src = a + src[neb * ts:]
        nsplit = ts if (split and not (left and b == nblk - 1)) else 1
        ne = bsize // nsplit
        starts.append(hdr_len + len(body))
        for j in range(nsplit):
            part = src[j * ne:(j + 1) * ne]
            z = _snappy_compress(part, rng)
            if len(z) >= ne:
                z = part  # stored
            body += len(z).to_bytes(4, "little") + z
    cbytes = hdr_len + len(body)
    hdr = bytes([2, 1, flags, ts]) + nbytes.to_bytes(4, "little") + blocksize.to_bytes(4, "little") + \
        cbytes.to_bytes(4, "little")
    return hdr + b"".join(s.to_bytes(4, "little") for s in starts) + bytes(body)


@pytest.mark.parametrize("ts,shuffle,split", [(1, False, False), (2, True, True), (4, True, False),
                                              (4, False, True), (8, True, True)])
def test_blosc_snappy_streams(ctx, torch_cuda, ts, shuffle, split):
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    from zarrs_amd import _lib as L
    rng = np.random.default_rng(ts * 11 + shuffle + 2 * split)
    ch = CodecChain.from_metadata([{"name": "bytes", "configuration": {"endian": "little"}},
                                   _blosc("snappy", "shuffle" if shuffle else "noshuffle", ts)], DT[ts], 0, ctx)
    for n, bsz in ((1000, 4096), (40000, 8192), (30001, 4096), (70000, 65536)):
        n -= n % 1 if ts == 1 else n % ts
        descs, keep, exp = [], [], []
        for k in range(3):
            a = _data(rng, n // ts, ts)
            if k == 1:  # long runs and a period past the 2-byte offsets (4-byte copies)
                a = np.resize(np.repeat(a[: max(1, len(a) // 64)], 64), n // ts)
            raw = a.tobytes()
            enc = _blosc_snappy_frame(raw, ts, shuffle, bsz, split, rng)
            d = torch_cuda.frombuffer(bytearray(enc), dtype=torch_cuda.uint8).cuda()
            keep.append(d)
            descs.append(make_desc(d, [n // ts], out_start=[k * (n // ts)]))
            exp.append(a)
        out = np.zeros(3 * (n // ts), DT[ts])
        st = ch.decode_batch(descs, out, [3 * (n // ts)], enc_device=True)
        assert st == [0] * 3, (n, bsz)
        assert out.tobytes() == np.concatenate(exp).tobytes(), (n, bsz)
    # a copy reaching before the stream start / a truncated stream -> CORRUPT_STREAM
    a = _data(rng, 4096 // ts, ts)
    enc = bytearray(_blosc_snappy_frame(a.tobytes(), ts, False, 4096, False, rng))
    p = int.from_bytes(enc[16:20], "little")
    cs = int.from_bytes(enc[p:p + 4], "little")
    if cs != 4096:
        z = bytearray(_varint(4096)) + bytes([2 | (3 << 2)]) + (9).to_bytes(2, "little")  # copy 4 at offset 9
        bad = enc[:p] + len(z).to_bytes(4, "little") + z
        bad[12:16] = len(bad).to_bytes(4, "little")
        for e in (bytes(bad), bytes(enc[:p + 4 + cs // 2])):
            with pytest.raises(ZgpuError) as ei:
                ch.decode_batch([make_desc(e, [4096 // ts])], np.zeros(4096 // ts, DT[ts]), [4096 // ts],
                                enc_device=False)
            assert ei.value.status == L.CORRUPT_STREAM


@pytest.mark.parametrize("cname,shuffle", [("lz4", "shuffle"), ("lz4", "bitshuffle"), ("blosclz", "shuffle"),
                                           ("blosclz", "bitshuffle")])
def test_blosc_lz_corrupt_stream_beside_good_ones(ctx, torch_cuda, cname, shuffle):
    """Streams are decoded two per wave (k_lz4m / k_blosclzm, bitshuffled ones one per wave): a
    stream that fails (a match before the output start) reports CORRUPT_STREAM for its own chunk
    only, and the chunks decoded beside it in the same waves are exact (per-chunk statuses of
    zgpu_decode_batch)."""
    import ctypes as C
    from zarrs_amd import CodecChain, make_desc
    from zarrs_amd import _lib as L
    from zarrs_amd.codec import default_stream
    rng = np.random.default_rng(11)
    n, nch, badk = 5000, 8, 3
    codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc(cname, shuffle, 4, 4096)]
    co = O.OracleChain.from_metadata(codecs, "float32", 0, 1)
    ch = CodecChain.from_metadata(codecs, "float32", 0, ctx)
    data = [np.round(rng.standard_normal(n) * 10).astype(np.float32) for _ in range(nch)]
    encs = [bytearray(co.encode(a)) for a in data]
    e = encs[badk]
    assert not e[2] & 0x2
    nblk = (int.from_bytes(e[4:8], "little") + int.from_bytes(e[8:12], "little") - 1) // int.from_bytes(e[8:12], "little")
    bsize = int.from_bytes(e[8:12], "little")
    nsplit = 1 if e[2] & 0x10 else 4
    hit = False
    for b in range(nblk):  # the first compressed (not stored) stream of any full block
        p = int.from_bytes(e[16 + 4 * b:20 + 4 * b], "little")
        for _ in range(nsplit):
            cs = int.from_bytes(e[p:p + 4], "little")
            if cs != bsize // nsplit and not hit:
                s0 = p + 4
                if cname == "lz4":
                    e[s0] = 0x0F  # no literals, then a match at output offset 0
                else:
                    r = (e[s0] & 31) + 1
                    e[s0 + 1 + r] = 0xFF  # a match reaching 7937+ bytes back after <= 32 literals
                hit = True
            p += 4 + cs
        if hit:
            break
    assert hit
    keep = [torch_cuda.frombuffer(bytearray(x), dtype=torch_cuda.uint8).cuda() for x in encs]
    descs = [make_desc(d, [n], out_start=[k * n]) for k, d in enumerate(keep)]
    out = torch_cuda.zeros(nch * n, dtype=torch_cuda.float32, device="cuda")
    arr = (L.ChunkDesc * nch)(*descs)
    st = (C.c_int32 * nch)()
    rc = L.load().zgpu_decode_batch(ch._h, 1, arr, nch, C.c_void_p(out.data_ptr()), L.u64s([nch * n]),
                                    L.ENC_DEVICE | L.OUT_DEVICE, st, default_stream(None, out))
    assert rc == L.CORRUPT_STREAM
    got = out.cpu().numpy()
    for k in range(nch):
        if k == badk:
            assert st[k] == L.CORRUPT_STREAM
        else:
            assert st[k] == 0, k
            assert np.array_equal(got[k * n:(k + 1) * n], data[k]), k


@pytest.mark.parametrize("cname,shuffle", [("lz4", "shuffle"), ("zstd", "bitshuffle"), ("blosclz", "noshuffle")])
def test_blosc_partial_decodes_only_covering_blocks(ctx, torch_cuda, cname, shuffle):
    """A partial selection of a blosc chunk decodes only the blocks that cover the bytes it reads, as
    zarrs' blosc partial decoder does (blosc_partial_decoder.rs:33-60 -> blosc_decompress_bytes_partial,
    c-blosc's blosc_getitem): ZGPU_CTR_BLOSC_BLOCKS counts the decoded blocks; the values equal the
    oracle's."""
    from zarrs_amd import CodecChain, make_desc
    from zarrs_amd import _lib as L
    codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc(cname, shuffle, 4, blocksize=8192)]
    co = O.OracleChain.from_metadata(codecs, "float32", 0, 3)
    ch = CodecChain.from_metadata(codecs, "float32", 0, ctx)
    rng = np.random.default_rng(5)
    cs = [32, 32, 32]  # 128 KiB
    x = np.arange(32, dtype=np.float32)
    a = (np.round(rng.standard_normal(cs) * 2) + x[:, None, None] * 3 + x[None, :, None]).astype(np.float32)
    enc = co.encode(a)
    flags, bs = enc[2], int.from_bytes(enc[8:12], "little")  # c-blosc may round the requested block size
    assert not flags & 2, "a compressed (not memcpyed) frame"
    nblk = -(-a.nbytes // bs)
    assert nblk >= 2
    for hbm in (True, False):
        src = torch_cuda.frombuffer(bytearray(enc), dtype=torch_cuda.uint8).cuda() if hbm else enc
        for start, sub in (([0, 0, 0], cs), ([0, 0, 0], [2, 32, 32]), ([10, 5, 0], [2, 4, 32]), ([3, 0, 7], [9, 32, 3]),
                           ([31, 31, 31], [1, 1, 1]), ([0, 0, 0], [32, 1, 1])):
            out = np.zeros(sub, np.float32)
            assert ch.decode_batch([make_desc(src, cs, start, sub)], out, sub, enc_device=hbm) == [0]
            exp = co.decode(enc, cs)[tuple(slice(s, s + n) for s, n in zip(start, sub))]
            assert out.tobytes() == exp.tobytes(), (start, sub)
            # the blocks covering [first selected byte, last selected byte]
            lo = 4 * sum(s * st for s, st in zip(start, (1024, 32, 1)))
            hi = 4 * sum((s + n - 1) * st for s, n, st in zip(start, sub, (1024, 32, 1))) + 4
            blocks = nblk if sub == cs else (hi - 1) // bs - lo // bs + 1
            assert L.last_counters()["blosc_blocks"] == blocks, (start, sub, bs, L.last_counters())


def _zstd_block_kinds(frame):
    """(type, nseq) per block of one zstd frame (RFC 8878 3.1.1.2; nseq None for raw / rle)."""
    fhd = frame[4]
    single = (fhd >> 5) & 1
    p = 5 + (0 if single else 1) + [0, 1, 2, 4][fhd & 3] + [1 if single else 0, 2, 4, 8][fhd >> 6]
    out = []
    while True:
        h = frame[p] | frame[p + 1] << 8 | frame[p + 2] << 16
        p += 3
        t, sz = (h >> 1) & 3, h >> 3
        nseq = None
        if t == 2:
            b = frame[p]
            lt, sf = b & 3, (b >> 2) & 3
            if lt < 2:
                lh = [1, 2, 1, 3][sf]
                regen = (b >> 3) if sf in (0, 2) else ((b >> 4) | (frame[p + 1] << 4) if sf == 1 else
                                                       (b >> 4) | (frame[p + 1] << 4) | (frame[p + 2] << 12))
                csz = regen if lt == 0 else 1
            else:
                lh = [3, 3, 4, 5][sf]
                v = int.from_bytes(frame[p:p + lh], "little")
                csz = v >> [14, 14, 18, 22][sf]
            c0 = frame[p + lh + csz]
            nseq = c0 if c0 < 128 else (((c0 - 128) << 8) + frame[p + lh + csz + 1] if c0 < 255 else 1 << 15)
        out.append((t, nseq))
        p += sz if t != 1 else 1
        if h & 1:
            return out


def test_blosc_zstd_block_aliases_vs_oracle(ctx, torch_cuda):
    """k_blosc_finish reads zstd blocks that need no execution where they lie (ZstdScratch::alias):
    raw (noise) and rle (constant) byte planes, literal-only blocks, and raw blocks that a later
    block's matches copy from (those must stay in the slot). Bytes vs the c-blosc oracle; the test
    asserts the frames really hold each block kind."""
    from zarrs_amd import CodecChain, make_desc
    rng = np.random.default_rng(77)
    n = 1 << 17  # u16 elements: one 256 KiB blosc block per chunk, two 128 KiB zstd blocks
    cases = []
    noise = rng.integers(0, 256, n, dtype=np.uint16)
    cases.append(noise)  # low plane raw, high plane rle (0)
    cases.append(noise | np.uint16(0x0700))  # rle 7
    cases.append((noise % 180).astype(np.uint16))  # low plane literal-only (Huffman), high plane rle
    cases.append(noise | (np.arange(n, dtype=np.uint16) // 512 % 5 << 8).astype(np.uint16))  # raw, then matches
    half = rng.integers(0, 65536, n // 2, dtype=np.uint16)
    cases.append(np.concatenate([half, half]))  # shuffled planes with a repeat (matches)
    kinds = set()
    for shuffle in ("shuffle", "noshuffle"):
        codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc("zstd", shuffle, 2, 0, 5)]
        co = O.OracleChain.from_metadata(codecs, "uint16", 0, 1)
        ch = CodecChain.from_metadata(codecs, "uint16", 0, ctx)
        descs, keep = [], []
        for k, a in enumerate(cases):
            enc = bytes(co.encode(a))
            nb = int.from_bytes(enc[8:12], "little")
            for bi in range((2 * n + nb - 1) // nb):
                s0 = int.from_bytes(enc[16 + 4 * bi:20 + 4 * bi], "little")
                cs = int.from_bytes(enc[s0:s0 + 4], "little", signed=True)
                if enc[2] & 0x10 and cs != nb:  # not split: one zstd frame per block
                    kinds.update((shuffle,) + kb for kb in _zstd_block_kinds(enc[s0 + 4:s0 + 4 + cs]))
            d = torch_cuda.frombuffer(bytearray(enc), dtype=torch_cuda.uint8).cuda()
            keep.append(d)
            descs.append(make_desc(d, [n], out_start=[k * n]))
        out = np.zeros(len(cases) * n, np.uint16)
        assert ch.decode_batch(descs, out, [len(cases) * n], enc_device=True) == [0] * len(cases)
        assert out.tobytes() == np.concatenate(cases).tobytes(), shuffle
    assert ("shuffle", 0, None) in kinds and ("shuffle", 1, None) in kinds, kinds  # raw and rle planes
    assert ("shuffle", 2, 0) in kinds, kinds  # literal-only
    assert ("noshuffle", 0, None) in kinds, kinds


@pytest.mark.parametrize("knobs", [{"ZGPU_ZSTD_SPLIT": "1", "ZGPU_ZSTD_SPLIT_MIN": "1"}, {"ZGPU_ZSTD_XDENSE": "1"},
                                   {"ZGPU_ZSTD_XDENSE": "0"}, {"ZGPU_BLOSC_ALIAS": "0"},
                                   {"ZGPU_ZSTD_SPLIT": "1", "ZGPU_ZSTD_SPLIT_MIN": "1", "ZGPU_ZSTD_XDENSE": "1"}],
                         ids=["split", "xdense", "xwide", "noalias", "split-xdense"])
def test_blosc_zstd_pipeline_knobs_vs_oracle(ctx, torch_cuda, knobs):
    """The zstd pipeline's run-time choices change no byte: two pipelined halves on a second stream
    (opt-in ZGPU_ZSTD_SPLIT, forced for small batches by ZGPU_ZSTD_SPLIT_MIN), either executor configuration, and slot copies
    instead of block aliases. A batch of shuffled u16 chunks (several blosc blocks each: raw, rle,
    literal-only and sequence blocks) plus a corrupt one, vs the c-blosc oracle."""
    import ctypes as C
    import os
    from zarrs_amd import CodecChain, make_desc
    from zarrs_amd import _lib as L
    from zarrs_amd.codec import default_stream
    rng = np.random.default_rng(91)
    n = 3 << 17  # three 256 KiB blosc blocks per chunk
    codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, _blosc("zstd", "shuffle", 2, 0, 5)]
    co = O.OracleChain.from_metadata(codecs, "uint16", 0, 1)
    x = np.arange(n)
    chunks = [rng.integers(0, 256, n).astype(np.uint16),
              (100 + 900 * np.abs(np.sin(x * 0.001)) + rng.standard_normal(n) * 8).astype(np.uint16),
              (rng.integers(0, 256, n) % 180).astype(np.uint16),
              np.tile(rng.integers(0, 65536, n // 3, dtype=np.uint16), 3),
              (x // 700 % 9).astype(np.uint16)]
    encs = [bytes(co.encode(a)) for a in chunks]
    bad = bytearray(encs[1])
    b1 = int.from_bytes(bad[20:24], "little")  # blosc block 1: 4-byte size, then its zstd frame
    bad[b1 + 4] ^= 0x5A  # the frame's magic number
    encs.append(bytes(bad))
    saved = {k: os.environ.get(k) for k in knobs}
    os.environ.update(knobs)
    try:
        ch = CodecChain.from_metadata(codecs, "uint16", 0, ctx)
        descs, keep = [], []
        for k, e in enumerate(encs):
            d = torch_cuda.frombuffer(bytearray(e), dtype=torch_cuda.uint8).cuda()
            keep.append(d)
            descs.append(make_desc(d, [n], out_start=[k * n]))
        nch = len(encs)
        out = torch_cuda.zeros(nch * n, dtype=torch_cuda.int16, device="cuda")
        arr = (L.ChunkDesc * nch)(*descs)
        stc = (C.c_int32 * nch)()
        rc = L.load().zgpu_decode_batch(ch._h, 1, arr, nch, C.c_void_p(out.data_ptr()), L.u64s([nch * n]),
                                        L.ENC_DEVICE | L.OUT_DEVICE, stc, default_stream(None, out))
        st = list(stc)
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    assert rc == L.CORRUPT_STREAM and st[:5] == [0] * 5 and st[5] == L.CORRUPT_STREAM, (rc, st)
    assert out.cpu().numpy()[:5 * n].tobytes() == np.concatenate(chunks).tobytes()
