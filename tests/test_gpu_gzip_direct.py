"""k_gzip writing whole chunks straight into the output rows (GzDirect, ZGPU_GZIP_DIRECT): the gzip
stage last before the rows scatter, so the scatter (ArrayBytesFixedDisjointView::copy_from_slice,
array_bytes_fixed_disjoint_view.rs:177-206) takes only partial selections. Every case decodes into a
window of a larger array whose bytes outside the window are sentinels, with the direct path on and
off: whole chunks on aligned rows (direct), whole chunks on misaligned rows and partial selections
(slot + scatter), chunk shapes the planner refuses (a non-power-of-two row axis), the trailing crc32c
of C3's inner chain in both gzip kernels, and a stream of the wrong decoded size
(InvalidBytesLengthError, array_bytes.rs:376-386)."""
import gzip
import struct

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

BYTES_LE = {"name": "bytes", "configuration": {"endian": "little"}}
GZ1 = {"name": "gzip", "configuration": {"level": 1}}


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    return Context(0)


def _enc(chunk, crc):
    e = gzip.compress(np.ascontiguousarray(chunk).tobytes(), 1)
    return e + struct.pack("<I", O.crc32c(e)) if crc else e


CASES = {  # name: dtype, chunk shape, window shape, whole array shape, window start
    "3d_f32": (np.float32, [8, 16, 32], [20, 40, 120], [24, 44, 136], [2, 3, 8]),
    "3d_f32_odd_axis": (np.float32, [8, 12, 32], [20, 30, 120], [22, 32, 128], [1, 1, 4]),
    "2d_u16": (np.uint16, [16, 64], [60, 220], [64, 240], [2, 8]),
    "1d_u8": (np.uint8, [4096], [30000], [30048], [16]),
}


def _cells(cs, win, align):
    """Disjoint placements: a grid of cells of chunk size plus a gap (innermost: `align` elements, so a
    cell start can be 16-B aligned or one element off it)."""
    nd = len(cs)
    gap = [1] * (nd - 1) + [align]
    n = [(w - c - 1) // (c + g) + 1 for c, w, g in zip(cs, win, gap)]
    return [[i * (c + g) for i, c, g in zip(np.unravel_index(k, n), cs, gap)] for k in range(int(np.prod(n)))]


@pytest.mark.parametrize("direct", ["1", "0"])
@pytest.mark.parametrize("crc", [False, True], ids=["gzip", "gzip_crc32c"])
@pytest.mark.parametrize("pipe", ["pipelined", "one_wave"])
@pytest.mark.parametrize("case", list(CASES))
def test_gzip_direct_rows(ctx, case, crc, pipe, direct, monkeypatch):
    import torch
    from zarrs_amd import CodecChain, make_desc
    monkeypatch.setenv("ZGPU_GZIP_DIRECT", direct)
    if pipe == "one_wave":
        monkeypatch.setenv("ZGPU_GZIP_PIPE_MAX", "0")
    dt, cs, win, full, ws = CASES[case]
    nd = len(cs)
    rng = np.random.default_rng(7)
    codecs = [BYTES_LE, GZ1] + ([{"name": "crc32c"}] if crc else [])
    ch = CodecChain.from_metadata(codecs, np.dtype(dt).name, 0, ctx)
    sentinel = np.iinfo(np.uint8).max
    exp = np.full(np.prod(full) * np.dtype(dt).itemsize, sentinel, np.uint8).view(dt).reshape(full)
    exp[tuple(slice(s, s + w) for s, w in zip(ws, win))] = 0
    descs, keep = [], []
    isz = np.dtype(dt).itemsize
    cells = _cells(cs, win, 16 // isz)
    assert len(cells) >= 7
    # six whole chunks: even ones on 16-B aligned output rows (direct), odd ones one element off (slot +
    # scatter); every third one constant (long matches)
    for k in range(6):
        vals = (rng.random(cs) * 1000).astype(dt) if dt == np.float32 else rng.integers(0, 250, cs).astype(dt)
        if k % 3 == 2:
            vals = np.zeros(cs, dt) + k
        dev = torch.frombuffer(bytearray(_enc(vals, crc)), dtype=torch.uint8).cuda()
        keep.append(dev)
        o = list(cells[k])
        o[-1] += k % 2
        descs.append(make_desc(dev, cs, out_start=o))
        exp[tuple(slice(ws[d] + o[d], ws[d] + o[d] + cs[d]) for d in range(nd))] = vals
    # a partial selection of one more chunk (the scatter path)
    vals = (np.arange(np.prod(cs)) % 251).astype(dt).reshape(cs)
    dev = torch.frombuffer(bytearray(_enc(vals, crc)), dtype=torch.uint8).cuda()
    keep.append(dev)
    ss = [c // 4 for c in cs]
    sz = [c // 2 for c in cs]
    o = cells[6]
    descs.append(make_desc(dev, cs, sel_start=ss, sel_shape=sz, out_start=o))
    exp[tuple(slice(ws[d] + o[d], ws[d] + o[d] + sz[d]) for d in range(nd))] = \
        vals[tuple(slice(s_, s_ + z) for s_, z in zip(ss, sz))]
    out = torch.empty(full, dtype={np.float32: torch.float32, np.uint16: torch.int16, np.uint8: torch.uint8}[dt],
                      device="cuda")
    out.view(torch.uint8).fill_(sentinel)
    out[tuple(slice(s_, s_ + w) for s_, w in zip(ws, win))] = 0
    st = ch.decode_batch_into(descs, out, ws, win, enc_device=True)
    assert st == [0] * len(descs)
    got = out.cpu().numpy().view(np.uint8).view(dt).reshape(full)
    assert got.tobytes() == exp.tobytes()


@pytest.mark.parametrize("pipe", ["pipelined", "one_wave"])
def test_gzip_direct_size_mismatch(ctx, pipe, monkeypatch):
    """A whole-chunk item on the direct path whose stream decodes short reports
    DECODED_SIZE_MISMATCH with its exact length; one that decodes long stops at the chunk."""
    import torch
    from zarrs_amd import CodecChain, ZgpuError, make_desc
    from zarrs_amd import _lib as L
    monkeypatch.setenv("ZGPU_GZIP_DIRECT", "1")
    if pipe == "one_wave":
        monkeypatch.setenv("ZGPU_GZIP_PIPE_MAX", "0")
    cs = [4, 8, 32]
    ch = CodecChain.from_metadata([BYTES_LE, GZ1], "float32", 0, ctx)
    nb = int(np.prod(cs)) * 4
    for n, exact in ((nb - 128, True), (nb + 4096, False)):
        dev = torch.frombuffer(bytearray(gzip.compress(bytes(range(256)) * (n // 256) + bytes(n % 256), 1)),
                               dtype=torch.uint8).cuda()
        out = torch.zeros([8, 8, 64], dtype=torch.float32, device="cuda")
        with pytest.raises(ZgpuError) as ei:
            ch.decode_batch([make_desc(dev, cs, out_start=[4, 0, 32])], out, [8, 8, 64], enc_device=True)
        assert ei.value.status == L.DECODED_SIZE_MISMATCH
        assert L.last_size_mismatch() == (0, n if exact else None, nb)
        # nothing outside the chunk's box was written
        o = out.cpu().numpy()
        assert not o[:4].any() and not o[4:, :, :32].any()
