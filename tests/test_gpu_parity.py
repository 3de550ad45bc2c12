"""GPU parity: the HIP pipeline (libzgpu.so through the C ABI) against the committed goldens, the
reference's own fixtures, and the CPU oracle on seeded inputs. Bit-exact everywhere (every stage on
this path is lossless: SURVEY 8(a))."""
import json
import os

import numpy as np
import pytest

import fixtures as F
import oracle as O

pytestmark = pytest.mark.gpu

CASES = json.load(open(os.path.join(F.GOLDEN, "cases.json")))


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    return torch


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    return Context(0)


def _gpu_decode(ctx, case, enc: bytes, device_input: bool, torch):
    from zarrs_amd import CodecChain, make_desc
    ch = CodecChain.from_metadata(case["codecs"], case["data_type"], case["fill_value"], ctx)
    shape = case["shape"]
    sel = case["sel"] or [[0] * len(shape), shape]
    src = torch.frombuffer(bytearray(enc), dtype=torch.uint8).cuda() if (device_input and len(enc)) else enc
    out = np.zeros(sel[1], dtype=ch.dtype)
    d = make_desc(src, shape, sel[0], sel[1])
    return ch.decode_batch([d], out, list(sel[1]), enc_device=device_input and len(enc) > 0), out


@pytest.mark.parametrize("device_input", [True, False], ids=["hbm", "host"])
@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_golden(ctx, torch_cuda, case, device_input):
    from zarrs_amd import ZgpuError
    g = np.load(os.path.join(F.GOLDEN, "synthetic.npz"), allow_pickle=False)
    enc = g[case["name"] + "/enc"].tobytes()
    if case["status"]:
        with pytest.raises(ZgpuError) as ei:
            _gpu_decode(ctx, case, enc, device_input, torch_cuda)
        assert ei.value.status == case["status"]
        return
    st, out = _gpu_decode(ctx, case, enc, device_input, torch_cuda)
    assert st == [0]
    assert out.tobytes() == g[case["name"] + "/dec"].tobytes()


@pytest.mark.parametrize("fixture", F.FLOAT_0_99 + [F.SHARDED])
@pytest.mark.parametrize("store", ["host", "hbm"])
def test_reference_fixture_array(ctx, torch_cuda, fixture, store):
    from zarrs_amd import Array, DeviceStore, MemoryStore
    m, chunks = F.load_array(fixture)
    meta = {"shape": m["shape"], "data_type": m["data_type"], "fill_value": m["fill_value"],
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": m["chunk_shape"]}},
            "chunk_key_encoding": {"name": "default", "configuration": {"separator": "/"}},
            "codecs": m["codecs"]}
    ms = MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in chunks.items()})
    st = DeviceStore.from_store(ms) if store == "hbm" else ms
    arr = Array(st, meta, ctx)
    exp = np.arange(int(np.prod(m["shape"]))).reshape(m["shape"]).astype(arr.dtype)
    assert np.array_equal(arr.retrieve_array_subset(), exp)
    # partial subsets crossing chunk boundaries (partial-decoder path)
    assert np.array_equal(arr.retrieve_array_subset([1, 2], [6, 5]), exp[1:7, 2:7])
    assert np.array_equal(arr.retrieve_chunk([1, 0]), exp[m["chunk_shape"][0]:2 * m["chunk_shape"][0],
                                                          :m["chunk_shape"][1]])


def _encode_grid(chain_o, a, cs, drop=()):
    chunks = {}
    grid = [-(-s // c) for s, c in zip(a.shape, cs)]
    for idx in np.ndindex(*grid):
        if idx in drop:
            continue
        blk = np.zeros(cs, a.dtype)
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, cs, a.shape))
        src = a[sl]
        blk[tuple(slice(0, n) for n in src.shape)] = src
        chunks[idx] = chain_o.encode(blk)
    return chunks


CHAINS = {
    "c2_transpose_be": ([{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
                         {"name": "bytes", "configuration": {"endian": "big"}}], "float32"),
    "bytes_le": ([{"name": "bytes", "configuration": {"endian": "little"}}], "float32"),
    "transpose_021_u16": ([{"name": "transpose", "configuration": {"order": [0, 2, 1]}},
                           {"name": "bytes", "configuration": {"endian": "big"}}], "uint16"),
    "crc_shuffle": ([{"name": "bytes", "configuration": {"endian": "little"}},
                     {"name": "numcodecs.shuffle", "configuration": {"elementsize": 8}},
                     {"name": "crc32c"}], "float64"),
    "shuffle2_zstd_u16": ([{"name": "bytes", "configuration": {"endian": "little"}},
                           {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
                           {"name": "zstd", "configuration": {"level": 3, "checksum": False}}], "uint16"),
    "shuffle4_be_f32": ([{"name": "bytes", "configuration": {"endian": "big"}},
                         {"name": "numcodecs.shuffle", "configuration": {"elementsize": 4}}], "float32"),
    "shuffle2_be_gzip_i16": ([{"name": "bytes", "configuration": {"endian": "big"}},
                              {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
                              {"name": "gzip", "configuration": {"level": 1}}], "int16"),
    "sharded_crc": ([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [8, 8, 8], "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                                             {"name": "crc32c"}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "end"}}], "float32"),
    "sharded_transpose_inner": ([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [8, 4, 16], "codecs": [{"name": "transpose", "configuration": {"order": [2, 0, 1]}},
                                              {"name": "bytes", "configuration": {"endian": "big"}}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "big"}}, {"name": "crc32c"}],
        "index_location": "start"}}], "int32"),
    # transpose codecs before sharding_indexed: the shard and its inner grid are in the transposed frame
    "transpose_then_sharded": ([{"name": "transpose", "configuration": {"order": [1, 2, 0]}},
                                {"name": "sharding_indexed", "configuration": {
        "chunk_shape": [8, 8, 4], "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                                             {"name": "crc32c"}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "end"}}], "float32"),
    "transpose_then_sharded_inner_transpose_gzip": ([{"name": "transpose", "configuration": {"order": [2, 0, 1]}},
                                                     {"name": "sharding_indexed", "configuration": {
        "chunk_shape": [8, 8, 16], "codecs": [{"name": "transpose", "configuration": {"order": [1, 2, 0]}},
                                              {"name": "bytes", "configuration": {"endian": "big"}},
                                              {"name": "gzip", "configuration": {"level": 1}}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}],
        "index_location": "start"}}], "int16"),
    "transpose_keep_inner_then_sharded": ([{"name": "transpose", "configuration": {"order": [1, 0, 2]}},
                                           {"name": "sharding_indexed", "configuration": {
        "chunk_shape": [8, 16, 8], "codecs": [{"name": "bytes", "configuration": {"endian": "big"}}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "end"}}], "float64"),
    # nested sharding: [16,32,32] shards of [8,16,16] middle shards of [4,8,8] (or [8,4,16]) leaves
    "nested_sharded_crc": ([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [8, 16, 16],
        "codecs": [{"name": "sharding_indexed", "configuration": {
            "chunk_shape": [4, 8, 8], "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                                                 {"name": "crc32c"}],
            "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
            "index_location": "end"}}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "end"}}], "float32"),
    "nested_sharded_zstd_transpose": ([{"name": "transpose", "configuration": {"order": [2, 0, 1]}},
                                       {"name": "sharding_indexed", "configuration": {
        "chunk_shape": [16, 8, 16],
        "codecs": [{"name": "sharding_indexed", "configuration": {
            "chunk_shape": [8, 4, 16], "codecs": [{"name": "transpose", "configuration": {"order": [1, 0, 2]}},
                                                  {"name": "bytes", "configuration": {"endian": "big"}},
                                                  {"name": "zstd", "configuration": {"level": 1, "checksum": False}}],
            "index_codecs": [{"name": "bytes", "configuration": {"endian": "big"}}],
            "index_location": "start"}}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "start"}}], "uint16"),
}


@pytest.mark.parametrize("name", list(CHAINS))
@pytest.mark.parametrize("store", ["host", "hbm"])
def test_random_arrays_vs_oracle(ctx, torch_cuda, name, store):
    from zarrs_amd import Array, DeviceStore, MemoryStore
    codecs, dt = CHAINS[name]
    rng = np.random.default_rng(abs(hash(name)) % 2**32)
    shape, cs = [45, 70, 33], [16, 32, 32]
    npdt = np.dtype(O.DTYPES[dt][0])
    a = (rng.standard_normal(shape) * 100).astype(npdt)
    co = O.OracleChain.from_metadata(codecs, dt, 3, 3)
    chunks = _encode_grid(co, a, cs, drop={(1, 1, 0)})
    ms = MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in chunks.items()})
    meta = {"shape": shape, "data_type": dt, "fill_value": 3, "codecs": codecs,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": cs}}}
    arr = Array(DeviceStore.from_store(ms) if store == "hbm" else ms, meta, ctx)
    for start, sub in (([0, 0, 0], shape), ([5, 17, 3], [30, 40, 29]), ([16, 32, 0], [16, 32, 32]),
                       ([44, 69, 32], [1, 1, 1])):
        exp = O.retrieve_array_subset(co, shape, cs, chunks, start, sub, nthreads=4)
        got = arr.retrieve_array_subset(start, sub)
        assert got.tobytes() == exp.tobytes(), (start, sub)


def test_device_output_and_plan(ctx, torch_cuda):
    """Device-resident encoded chunks -> device output through the prepared-plan API (bench path)."""
    import ctypes as C
    torch = torch_cuda
    from zarrs_amd import CodecChain, make_desc
    from zarrs_amd import _lib as L
    codecs, dt = CHAINS["c2_transpose_be"]
    rng = np.random.default_rng(5)
    cs, grid = [64, 64, 64], [2, 3, 2]
    a = rng.standard_normal([g * c for g, c in zip(grid, cs)]).astype(np.float32)
    co = O.OracleChain.from_metadata(codecs, dt, 0, 3)
    chunks = _encode_grid(co, a, cs)
    dev = {k: torch.frombuffer(bytearray(v), dtype=torch.uint8).cuda() for k, v in chunks.items()}
    ch = CodecChain.from_metadata(codecs, dt, 0, ctx)
    descs = [make_desc(dev[k], cs, out_start=[i * c for i, c in zip(k, cs)]) for k in sorted(dev)]
    out = torch.empty(a.shape, dtype=torch.float32, device="cuda")
    arr = (L.ChunkDesc * len(descs))(*descs)
    plan = C.c_void_p()
    L.check(L.load().zgpu_plan_create(ch._h, 3, arr, len(descs), L.u64s(a.shape),
                                      L.ENC_DEVICE | L.OUT_DEVICE, C.byref(plan)))
    st = (C.c_int32 * len(descs))()
    for _ in range(3):
        out.zero_()
        L.check(L.load().zgpu_plan_execute(plan, out.data_ptr(), st, None))
        assert np.array_equal(out.cpu().numpy(), a)
    assert L.load().zgpu_plan_algorithmic_bytes(plan) == 2 * a.nbytes
    L.load().zgpu_plan_destroy(plan)


def test_error_first_status_per_descriptor(ctx, torch_cuda):
    """A corrupt chunk reports INVALID_CHECKSUM for its descriptor only; the others decode."""
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    codecs = [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}]
    co = O.OracleChain.from_metadata(codecs, "uint16", 0, 1)
    a = np.arange(300, dtype=np.uint16)
    encs = [co.encode(a[i * 100:(i + 1) * 100]) for i in range(3)]
    bad = bytearray(encs[1])
    bad[10] ^= 1
    encs[1] = bytes(bad)
    ch = CodecChain.from_metadata(codecs, "uint16", 0, ctx)
    out = np.zeros(300, np.uint16)
    descs = [make_desc(e, [100], out_start=[100 * i]) for i, e in enumerate(encs)]
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch(descs, out, [300], enc_device=False)
    assert ei.value.status == 1
    assert np.array_equal(out[:100], a[:100]) and np.array_equal(out[200:], a[200:])
    # validate_checksums = false -> decodes (the flipped byte shows through)
    ch2 = CodecChain.from_metadata(codecs, "uint16", 0, ctx, validate_checksums=False)
    out2 = np.zeros(300, np.uint16)
    assert ch2.decode_batch(descs, out2, [300], enc_device=False) == [0, 0, 0]


def test_pipelined_host_to_host(ctx, torch_cuda):
    """Pinned host chunks -> pinned host array covering it: the overlapped sub-batch path (H2D,
    decode and D2H of axis-0 row ranges on three streams). Bit-exact vs the oracle; a corrupt chunk
    in a middle sub-batch fails its descriptor only; a partial cover falls back to the serial path."""
    import torch
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    codecs = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
              {"name": "bytes", "configuration": {"endian": "big"}}, {"name": "crc32c"}]
    cs, grid = [16, 32, 32], [16, 2, 2]
    rng = np.random.default_rng(11)
    a = rng.standard_normal([g * c for g, c in zip(grid, cs)]).astype(np.float32)
    co = O.OracleChain.from_metadata(codecs, "float32", 0, 3)
    chunks = _encode_grid(co, a, cs)
    keys = sorted(chunks)
    offs = np.cumsum([0] + [len(chunks[k]) for k in keys])
    host = torch.from_numpy(np.frombuffer(b"".join(chunks[k] for k in keys), np.uint8).copy()).pin_memory()
    base = host.data_ptr()
    descs = [make_desc((base + int(offs[j]), len(chunks[k])), cs, out_start=[i * c for i, c in zip(k, cs)])
             for j, k in enumerate(keys)]
    ch = CodecChain.from_metadata(codecs, "float32", 0, ctx)
    out = torch.zeros(a.shape, dtype=torch.float32).pin_memory()
    assert ch.decode_batch(descs, out, list(a.shape), enc_device=False) == [0] * len(descs)
    assert np.array_equal(out.numpy(), a)
    # a flipped byte in the chunk at rows 128..143 (sub-batch 5 of 8)
    bad = keys.index((8, 1, 0))
    host[int(offs[bad]) + 7] ^= 1
    out.zero_()
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch(descs, out, list(a.shape), enc_device=False)
    assert ei.value.status == 1
    got = out.numpy()
    assert np.array_equal(got[:128], a[:128]) and np.array_equal(got[144:], a[144:])
    host[int(offs[bad]) + 7] ^= 1
    # partial cover (the last chunk row left out): serial path, uncovered bytes keep their values
    part = [d for d, k in zip(descs, keys) if k[0] < 15]
    out.fill_(7.0)
    ch.decode_batch(part, out, list(a.shape), enc_device=False)
    assert np.array_equal(out.numpy()[:240], a[:240]) and bool((out[240:] == 7.0).all())


TILED = [  # (data type, transpose order, chunk shape, array shape): full 64-wide tiles, ragged slab groups
    ("float32", [2, 1, 0], [64, 6, 64], [128, 12, 192]),
    ("float64", [2, 1, 0], [64, 5, 64], [128, 10, 128]),
    ("uint16", [2, 1, 0], [64, 7, 64], [192, 14, 128]),
    ("uint8", [1, 2, 0], [64, 3, 64], [128, 6, 128]),
    ("float32", [1, 0], [64, 128], [128, 256]),
    ("int32", [3, 1, 0, 2], [2, 64, 5, 64], [4, 128, 10, 128]),
]


@pytest.mark.parametrize("dt,order,cs,shape", TILED, ids=[f"{t[0]}_{''.join(map(str, t[1]))}" for t in TILED])
def test_tiled_transpose_paths(ctx, torch_cuda, dt, order, cs, shape):
    """The slab-batched LDS transpose (k_scatter_tiled): aligned 16-B paths, ragged slab groups,
    fill (missing chunk), partial selections, unaligned output offsets -- vs the oracle."""
    from zarrs_amd import Array, DeviceStore, MemoryStore
    codecs = [{"name": "transpose", "configuration": {"order": order}},
              {"name": "bytes", "configuration": {"endian": "big"}}]
    rng = np.random.default_rng(len(shape) * 100 + cs[1])
    npdt = np.dtype(O.DTYPES[dt][0])
    a = (rng.standard_normal(shape) * 1000).astype(npdt)
    co = O.OracleChain.from_metadata(codecs, dt, 7, len(shape))
    chunks = _encode_grid(co, a, cs, drop={tuple([1] + [0] * (len(shape) - 1))})
    ms = MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in chunks.items()})
    meta = {"shape": shape, "data_type": dt, "fill_value": 7, "codecs": codecs,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": cs}}}
    arr = Array(DeviceStore.from_store(ms), meta, ctx)
    subsets = [([0] * len(shape), shape),
               ([1] * len(shape), [s - 2 for s in shape]),
               ([c // 2 for c in cs], [max(1, c) for c in cs])]
    for start, sub in subsets:
        exp = O.retrieve_array_subset(co, shape, cs, chunks, start, sub, nthreads=4)
        got = arr.retrieve_array_subset(start, sub)
        assert got.tobytes() == exp.tobytes(), (start, sub)


@pytest.mark.parametrize("out_dev", [False, True])
def test_retrieve_array_subset_multi_device(ctx, torch_cuda, out_dev):
    """zgpu_retrieve_array_subset_multi: the subset's axis-0 chunk rows cut over several contexts
    (on this 1-GPU box: three contexts on device 0, so the partitioning, the per-device uploads, the
    device-slab + peer-copy gather and the status order are exercised; the 8-GPU node runs the same
    code with one context per device), vs the oracle. A corrupt chunk in the middle group is reported."""
    from zarrs_amd import Array, Context, MemoryStore
    codecs = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
              {"name": "bytes", "configuration": {"endian": "big"}},
              {"name": "gzip", "configuration": {"level": 1}}, {"name": "crc32c"}]
    rng = np.random.default_rng(21)
    shape, cs = [70, 40, 33], [16, 16, 16]
    a = np.round(rng.standard_normal(shape) * 50).astype(np.float32)
    co = O.OracleChain.from_metadata(codecs, "float32", 0, 3)
    chunks = _encode_grid(co, a, cs, drop={(1, 1, 1)})
    ms = MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in chunks.items()})
    meta = {"shape": shape, "data_type": "float32", "fill_value": 0, "codecs": codecs,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": cs}}}
    arr = Array(ms, meta, ctx)
    extra = [Context(0), Context(0)]
    try:
        for n_dev in (1, 2, 3):
            for start, sub in (([0, 0, 0], shape), ([5, 3, 2], [60, 30, 31]), ([17, 0, 0], [5, 40, 33])):
                exp = O.retrieve_array_subset(co, shape, cs, chunks, start, sub, nthreads=4)
                if out_dev:
                    out = torch_cuda.full(sub, -7.0, dtype=torch_cuda.float32, device="cuda")
                else:
                    out = np.full(sub, -7.0, np.float32)
                arr.retrieve_array_subset_multi(start, sub, out, [ctx] + extra[: n_dev - 1])
                got = out.cpu().numpy() if out_dev else out
                assert got.tobytes() == exp.tobytes(), (n_dev, start, sub)
        # a corrupt chunk in the middle group: its status, not a later one's
        bad = dict(chunks)
        k = (2, 0, 0)
        b = bytearray(bad[k])
        b[-1] ^= 0xFF  # its crc32c
        bad[k] = bytes(b)
        arr_bad = Array(MemoryStore({"c/" + "/".join(map(str, kk)): v for kk, v in bad.items()}), meta, ctx)
        out = np.zeros(shape, np.float32)
        from zarrs_amd import ZgpuError
        from zarrs_amd import _lib as L
        with pytest.raises(ZgpuError) as ei:
            arr_bad.retrieve_array_subset_multi([0, 0, 0], shape, out, [ctx] + extra)
        assert ei.value.status == L.INVALID_CHECKSUM
    finally:
        for c in extra:
            c.close()


def test_nested_sharding_fill_and_errors(ctx, torch_cuda):
    """Nested sharding: an all-fill middle shard (an empty outer index entry) decodes to the fill
    value; a corrupt middle-shard index fails with INVALID_CHECKSUM (middle indexes are verified like
    the outer one, SH:178-194); an out-of-range middle index entry fails with SHARD_INDEX_OOB."""
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    from zarrs_amd import _lib as L
    codecs, dt = CHAINS["nested_sharded_crc"]
    shape = [16, 32, 32]
    rng = np.random.default_rng(11)
    a = (rng.standard_normal(shape) * 100).astype(np.float32)
    a[8:16, 0:16, 16:32] = 3  # middle shard (1, 0, 1): all fill -> omitted by the encoder
    a[0:4, 0:8, 0:8] = 3      # a leaf of middle shard (0, 0, 0): all fill -> omitted
    co = O.OracleChain.from_metadata(codecs, dt, 3, 3)
    enc = co.encode(a)
    n1 = 8  # middle shards per shard
    idx = np.frombuffer(enc[len(enc) - 4 - 16 * n1:len(enc) - 4], "<u8").reshape(n1, 2)
    assert tuple(idx[5]) == (2**64 - 1, 2**64 - 1)  # (1, 0, 1) in C order
    ch = CodecChain.from_metadata(codecs, dt, 3, ctx)
    for start, sub in (([0, 0, 0], shape), ([3, 5, 7], [11, 20, 22])):
        out = np.zeros(sub, np.float32)
        desc = make_desc(enc, shape, sel_start=start, sel_shape=sub)
        assert ch.decode_batch([desc], out, sub, enc_device=False) == [0]
        exp = a[tuple(slice(s, s + n) for s, n in zip(start, sub))]
        assert out.tobytes() == exp.tobytes(), (start, sub)
    # middle shard 0: its own index (8 entries + crc32c) sits at its end
    off, nb = (int(x) for x in idx[0])
    bad = bytearray(enc)
    bad[off + nb - 10] ^= 0x40
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch([make_desc(bytes(bad), shape)], np.zeros(shape, np.float32), shape, enc_device=False)
    assert ei.value.status == L.INVALID_CHECKSUM
    # an outer index entry pointing past the shard -> SHARD_INDEX_OOB (the outer index crc is
    # recomputed so only the range is wrong)
    import zlib  # noqa: F401  (crc32c comes from the oracle)
    bad2 = bytearray(enc)
    ib = len(enc) - 4 - 16 * n1
    bad2[ib:ib + 8] = (len(enc) + 100).to_bytes(8, "little")
    bad2[len(enc) - 4:] = O.crc32c(bytes(bad2[ib:len(enc) - 4])).to_bytes(4, "little")
    with pytest.raises(ZgpuError) as ei:
        ch.decode_batch([make_desc(bytes(bad2), shape)], np.zeros(shape, np.float32), shape, enc_device=False)
    assert ei.value.status == L.SHARD_INDEX_OOB
