"""GPU parity of the filesystem-store read path: chunk files read by host threads
(buffered or O_DIRECT) into pinned staging, overlapped with H2D + decode, against the reference's
fixtures and the CPU oracle. Mirrors zarrs_filesystem's FilesystemStore semantics
(zarrs_filesystem/src/lib.rs:173-179 key -> path, :339-343/:428-430 missing key -> fill value,
:437-447 byte range past the end -> InvalidByteRangeError)."""
import numpy as np
import pytest

import fixtures as F
import oracle as O
from test_gpu_parity import CHAINS, _encode_grid

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def torch_cuda():
    import torch
    return torch


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    return Context(0)


def _meta(shape, dt, cs, codecs, fill=0):
    return {"shape": list(shape), "data_type": dt, "fill_value": fill, "codecs": codecs,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": list(cs)}},
            "chunk_key_encoding": {"name": "default", "configuration": {"separator": "/"}}}


@pytest.mark.parametrize("direct_io", [False, True], ids=["buffered", "direct"])
@pytest.mark.parametrize("fixture", F.FLOAT_0_99 + [F.SHARDED])
def test_fs_reference_fixture(ctx, torch_cuda, tmp_path, fixture, direct_io):
    from zarrs_amd import Array, FilesystemStore
    m, chunks = F.load_array(fixture)
    st = FilesystemStore(tmp_path, direct_io=direct_io)
    for k, v in chunks.items():
        st["c/" + "/".join(map(str, k))] = v
    arr = Array(st, _meta(m["shape"], m["data_type"], m["chunk_shape"], m["codecs"], m["fill_value"]), ctx)
    exp = np.arange(int(np.prod(m["shape"]))).reshape(m["shape"]).astype(arr.dtype)
    assert np.array_equal(arr.retrieve_array_subset(), exp)
    assert np.array_equal(arr.retrieve_array_subset([1, 2], [6, 5]), exp[1:7, 2:7])
    out = torch_cuda.zeros(m["shape"], dtype=getattr(torch_cuda, arr.dtype.name), device="cuda")
    arr.retrieve_array_subset_into([0, 0], m["shape"], out)
    assert np.array_equal(out.cpu().numpy(), exp)


@pytest.mark.parametrize("group_bytes", [None, "1"], ids=["default_groups", "one_chunk_groups"])
@pytest.mark.parametrize("name", ["c2_transpose_be", "shuffle2_zstd_u16", "shuffle2_be_gzip_i16", "sharded_crc"])
def test_fs_random_arrays_vs_oracle(ctx, torch_cuda, tmp_path, monkeypatch, name, group_bytes):
    """Many sub-batches (ZGPU_FS_GROUP_BYTES=1: every chunk its own read/H2D/decode step), missing
    chunk files, full and partial subsets, host and device outputs."""
    from zarrs_amd import Array, FilesystemStore
    if group_bytes:
        monkeypatch.setenv("ZGPU_FS_GROUP_BYTES", group_bytes)
    codecs, dt = CHAINS[name]
    rng = np.random.default_rng(7)
    shape, cs = [45, 70, 33], [16, 32, 32]
    a = (rng.standard_normal(shape) * 100).astype(np.dtype(O.DTYPES[dt][0]))
    co = O.OracleChain.from_metadata(codecs, dt, 3, 3)
    chunks = _encode_grid(co, a, cs, drop={(1, 1, 0), (2, 0, 1)})
    st = FilesystemStore(tmp_path, direct_io=True)
    for k, v in chunks.items():
        st["c/" + "/".join(map(str, k))] = v
    arr = Array(st, _meta(shape, dt, cs, codecs, 3), ctx)
    for start, sub in (([0, 0, 0], shape), ([5, 17, 3], [30, 40, 29]), ([44, 69, 32], [1, 1, 1])):
        exp = O.retrieve_array_subset(co, shape, cs, chunks, start, sub, nthreads=4)
        assert arr.retrieve_array_subset(start, sub).tobytes() == exp.tobytes(), (start, sub)
    out = torch_cuda.empty(shape, dtype=getattr(torch_cuda, arr.dtype.name), device="cuda")
    arr.retrieve_array_subset_into([0, 0, 0], shape, out)
    exp = O.retrieve_array_subset(co, shape, cs, chunks, [0, 0, 0], shape, nthreads=4)
    assert out.cpu().numpy().tobytes() == exp.tobytes()


@pytest.mark.parametrize("direct_io", [False, True], ids=["buffered", "direct"])
def test_fs_packed_byte_ranges_and_errors(ctx, torch_cuda, tmp_path, monkeypatch, direct_io):
    """Byte ranges at unaligned offsets of one packed file (get_partial_many), a range past the end
    of the file, a missing file, an empty object, and a hard I/O error (a directory)."""
    from zarrs_amd import CodecChain, FilesystemStore, make_desc
    from zarrs_amd import _lib as L
    monkeypatch.setenv("ZGPU_FS_GROUP_BYTES", "5000")
    codecs = [{"name": "bytes", "configuration": {"endian": "little"}},
              {"name": "gzip", "configuration": {"level": 5}}, {"name": "crc32c"}]
    co = O.OracleChain.from_metadata(codecs, "int32", 0, 2)
    rng = np.random.default_rng(3)
    blocks = [rng.integers(0, 50, (16, 16), dtype=np.int32) for _ in range(6)]
    encs = [co.encode(b) for b in blocks]
    packed, offs = b"\x07" * 13, []
    for e in encs:
        offs.append(len(packed))
        packed += e
    st = FilesystemStore(tmp_path, direct_io=direct_io)
    st["packed.bin"] = packed
    st["empty.bin"] = b""
    (tmp_path / "adir").mkdir()
    ch = CodecChain.from_metadata(codecs, "int32", 0, ctx)

    def run(ranges):
        descs = (L.ChunkDesc * len(ranges))()
        for i in range(len(ranges)):
            descs[i] = make_desc((None, 0), [16, 16], out_start=[16 * i, 0])
        out = np.full((16 * len(ranges), 16), -1, np.int32)
        rc, st_ = st.decode_files(ch, descs, ranges, out, list(out.shape))
        return rc, st_, out

    rc, sts, out = run([("packed.bin", offs[i], len(encs[i])) for i in (3, 0, 5, 1)])
    assert rc == 0 and sts == [0] * 4
    assert np.array_equal(out, np.concatenate([blocks[i] for i in (3, 0, 5, 1)]))
    # the last range to the end of the file (length None); a missing key -> fill value 0
    rc, sts, out = run([("packed.bin", offs[5], None), ("nope/c/0", 0, None), ("packed.bin", offs[2], len(encs[2]))])
    assert rc == 0 and sts == [0, 0, 0]
    assert np.array_equal(out, np.concatenate([blocks[5], np.zeros((16, 16), np.int32), blocks[2]]))
    # past the end of the file -> INVALID_BYTE_RANGE for that descriptor only
    rc, sts, out = run([("packed.bin", offs[4], len(encs[4])), ("packed.bin", len(packed) - 10, 11)])
    assert rc == L.INVALID_BYTE_RANGE and sts == [0, L.INVALID_BYTE_RANGE]
    assert np.array_equal(out[:16], blocks[4])
    # an empty object is present (not a missing key): the crc32c codec rejects it
    rc, sts, _ = run([("empty.bin", 0, None)])
    assert sts == [L.CRC_INPUT_TOO_SHORT]
    # reading a directory is a storage error for the whole call
    rc, _, _ = run([("packed.bin", offs[0], len(encs[0])), ("adir", 0, None)])
    assert rc == L.STORAGE_ERROR
