"""The bench's synthetic workload writer (tools/synth) produces valid zarrs encodings: its sharded
gzip+crc32c shards decode through the CPU oracle to exactly the values it generated."""
import ctypes as C
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import oracle as O  # noqa: E402


@pytest.fixture(scope="module")
def syn():
    import bench
    try:
        return bench._synth()
    except RuntimeError as e:
        pytest.skip(str(e))


def test_c3_shard_writer_matches_oracle(syn):
    import bench
    S, I = 64, 16
    dec = np.empty([S] * 3, np.float32)
    org = [256, 512, 1024]
    syn.synth_c3_values(bench._u64(org), bench._u64([S] * 3), dec.ctypes.data, 4)
    p, n = C.c_void_p(), C.c_uint64()
    assert syn.synth_gzip_crc_shard(dec.ctypes.data, 4, bench._u64([S] * 3), bench._u64([I] * 3), 1, 4,
                                    C.byref(p), C.byref(n)) == 0
    enc = C.string_at(p.value, n.value)
    syn.synth_free(p)
    codecs = [dict(bench.C3.CODECS[0])]
    codecs[0] = {"name": "sharding_indexed", "configuration": dict(codecs[0]["configuration"], chunk_shape=[I] * 3)}
    chain = O.OracleChain.from_metadata(codecs, "float32", 0.0, 3)
    got = chain.decode(enc, [S] * 3)
    assert np.array_equal(got, dec)
    # values are quantised to 1/256 -> compressible
    assert np.all(np.round(dec * 256) == dec * 256)
    assert len(enc) < dec.nbytes
