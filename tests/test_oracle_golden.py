"""Pin the CPU oracle (oracle/) against the reference's own fixtures and known-answer tests,
and against the committed synthetic goldens (tests/golden/make_golden.py). CPU only."""
import json
import os

import numpy as np
import pytest

import fixtures as F
import oracle as O

GOLD = os.path.join(F.GOLDEN, "synthetic.npz")
CASES = json.load(open(os.path.join(F.GOLDEN, "cases.json")))


def test_crc32c_kat():
    # zarrs/src/array/codec/bytes_to_bytes/crc32c.rs:100-127: bytes 0..6 -> LE checksum [20,133,9,65]
    assert O.crc32c(bytes(range(6))).to_bytes(4, "little") == bytes([20, 133, 9, 65])
    # RFC 3720 / iSCSI check value of "123456789"
    assert O.crc32c(b"123456789") == 0xE3069283


@pytest.mark.parametrize("fixture", F.FLOAT_0_99 + F.BLOSC)
def test_reference_fixture_float(fixture):
    # zarrs/src/array.rs:1684-1788: every array_* fixture decodes to float32 0..99
    m, chunks = F.load_array(fixture)
    ch = O.OracleChain.from_metadata(m["codecs"], m["data_type"], m["fill_value"], 2)
    out = O.retrieve_array_subset(ch, m["shape"], m["chunk_shape"], chunks, [0, 0], m["shape"])
    assert np.array_equal(out, np.arange(100, dtype=np.float32).reshape(10, 10))


def test_reference_fixture_sharded():
    # written by zarrs/examples/sharded_array_write_read.rs: uint16 8x8 = 0..63, gzip inner, crc index
    m, chunks = F.load_array(F.SHARDED)
    ch = O.OracleChain.from_metadata(m["codecs"], m["data_type"], m["fill_value"], 2)
    out = O.retrieve_array_subset(ch, m["shape"], m["chunk_shape"], chunks, [0, 0], [8, 8])
    assert np.array_equal(out, np.arange(64, dtype=np.uint16).reshape(8, 8))
    # partial-decoder path across both shards (sharding_partial_decoder_sync.rs:311-400)
    out = O.retrieve_array_subset(ch, m["shape"], m["chunk_shape"], chunks, [1, 2], [6, 5])
    assert np.array_equal(out, np.arange(64, dtype=np.uint16).reshape(8, 8)[1:7, 2:7])


def test_reference_fixture_shard_index_layout():
    # c/0/0 is 140 B, index entries (52,52),(0,52) -> chunk 1 stored before chunk 0
    enc = F.load_array(F.SHARDED)[1][(0, 0)]
    assert len(enc) == 140
    idx = O.unpack_u64_le(enc[-36:-4])
    assert idx == [52, 52, 0, 52]
    assert O.crc32c(enc[-36:-4]).to_bytes(4, "little") == enc[-4:]


@pytest.mark.parametrize("case", CASES, ids=[c["name"] for c in CASES])
def test_synthetic_golden(case):
    g = np.load(GOLD, allow_pickle=False)
    enc = g[case["name"] + "/enc"].tobytes()
    shape = case["shape"]
    if case["status"]:
        with pytest.raises(O.OracleError) as ei:
            ch = O.OracleChain.from_metadata(case["codecs"], case["data_type"], case["fill_value"], len(shape))
            if case["sel"]:
                O.retrieve_array_subset(ch, shape, shape, {tuple([0] * len(shape)): enc}, *case["sel"])
            else:
                ch.decode(enc, shape)
        assert ei.value.status == case["status"]
        return
    ch = O.OracleChain.from_metadata(case["codecs"], case["data_type"], case["fill_value"], len(shape))
    if case["sel"]:
        got = O.retrieve_array_subset(ch, shape, shape, {tuple([0] * len(shape)): enc}, *case["sel"])
    else:
        got = ch.decode(enc, shape)
    exp = g[case["name"] + "/dec"]
    assert got.tobytes() == exp.tobytes()


@pytest.mark.parametrize("codecs,dt", [
    ([{"name": "transpose", "configuration": {"order": [2, 0, 1]}},
      {"name": "bytes", "configuration": {"endian": "big"}},
      {"name": "numcodecs.shuffle", "configuration": {"elementsize": 4}},
      {"name": "gzip", "configuration": {"level": 3}}, {"name": "crc32c"}], "float32"),
    ([{"name": "bytes", "configuration": {"endian": "little"}},
      {"name": "zstd", "configuration": {"level": 2, "checksum": True}}], "int16"),
    ([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [2, 3, 4], "codecs": [{"name": "bytes", "configuration": {"endian": "big"}},
                                             {"name": "gzip", "configuration": {"level": 1}}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "start"}}], "uint32"),
    # transpose before sharding, and nested sharding (the GPU parity tests' expected values)
    ([{"name": "transpose", "configuration": {"order": [1, 2, 0]}},
      {"name": "sharding_indexed", "configuration": {
          "chunk_shape": [3, 4, 2], "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                                               {"name": "crc32c"}],
          "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
          "index_location": "end"}}], "float32"),
    ([{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [2, 6, 4],
        "codecs": [{"name": "sharding_indexed", "configuration": {
            "chunk_shape": [2, 3, 2], "codecs": [{"name": "bytes", "configuration": {"endian": "big"}},
                                                 {"name": "zstd", "configuration": {"level": 1, "checksum": False}}],
            "index_codecs": [{"name": "bytes", "configuration": {"endian": "big"}}],
            "index_location": "start"}}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "end"}}], "int32"),
])
def test_oracle_roundtrip(codecs, dt):
    rng = np.random.default_rng(1)
    a = rng.integers(0, 1000, size=(4, 6, 8)).astype(np.dtype(O.DTYPES[dt][0]))
    a[:2, :3, :4] = 0  # an all-fill inner chunk when sharded -> empty index entry
    ch = O.OracleChain.from_metadata(codecs, dt, 0, 3)
    enc = ch.encode(a)
    assert np.array_equal(ch.decode(enc, a.shape), a)


def test_oracle_threads_match_serial():
    rng = np.random.default_rng(2)
    a = rng.standard_normal((40, 30, 20)).astype(np.float32)
    codecs = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
              {"name": "bytes", "configuration": {"endian": "big"}}]
    ch = O.OracleChain.from_metadata(codecs, "float32", 0, 3)
    cs = [16, 16, 16]
    chunks = {}
    for i in range(3):
        for j in range(2):
            for k in range(2):
                blk = np.zeros(cs, np.float32)
                src = a[i * 16:(i + 1) * 16, j * 16:(j + 1) * 16, k * 16:(k + 1) * 16]
                blk[:src.shape[0], :src.shape[1], :src.shape[2]] = src
                chunks[(i, j, k)] = ch.encode(blk)
    del chunks[(1, 1, 0)]  # missing -> fill
    exp = a.copy()
    exp[16:32, 16:30, 0:16] = 0
    for nt in (1, 4):
        out = O.retrieve_array_subset(ch, a.shape, cs, chunks, [0, 0, 0], a.shape, nthreads=nt)
        assert np.array_equal(out, exp)
    out = O.retrieve_array_subset(ch, a.shape, cs, chunks, [3, 5, 7], [30, 20, 10], nthreads=3)
    assert np.array_equal(out, exp[3:33, 5:25, 7:17])
