"""Plan groups (zgpu_group): the independent levels of a multiscale pyramid decoded by ONE library call,
which lays the levels out on streams of its own (group.cpp). Every level must equal libzstd through the
oracle (zarrs decodes each array in its own rayon loop, array_read_ops_common.rs:111-179), statuses come
back per descriptor in part order, and the layout follows the documented policy (largest part split
over the lanes left over, small parts sharing one lane, literals-first on the largest part's first
piece and on the small-part lane)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

BYTES_LE = {"name": "bytes", "configuration": {"endian": "little"}}
C5_CODECS = [BYTES_LE, {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
             {"name": "zstd", "configuration": {"level": 3, "checksum": False}}]


def _level0(shape, seed=3):
    """Background 100 + Gaussian blobs + sqrt(mean) noise, u16 (bench C5 values)."""
    rng = np.random.default_rng(seed)
    z, y, x = (np.arange(n, dtype=np.float32) for n in shape)
    m = np.full(shape, 100.0, np.float32)
    for _ in range(5):
        cz, cy, cx = rng.uniform(0, shape[0]), rng.uniform(0, shape[1]), rng.uniform(0, shape[2])
        s, amp = rng.uniform(6, 30), rng.uniform(300, 4000)
        m += (amp * np.exp(-(z - cz) ** 2 / (2 * s * s))[:, None, None]
              * np.exp(-(y - cy) ** 2 / (2 * s * s))[None, :, None]
              * np.exp(-(x - cx) ** 2 / (2 * s * s))[None, None, :])
    v = np.rint(m + np.sqrt(m) * rng.standard_normal(shape, dtype=np.float32))
    return np.clip(v, 0, 65535).astype(np.uint16)


def _mean2(a):
    s = a.shape
    return (a.reshape(s[0] // 2, 2, s[1] // 2, 2, s[2] // 2, 2).astype(np.uint32).sum(axis=(1, 3, 5)) // 8) \
        .astype(np.uint16)


@pytest.fixture(scope="module")
def pyramid():
    """Four levels of a [64,256,256] u16 volume, chunked [16,128,128] / [16,64,64] / [16,32,32] /
    [8,32,32] (mixed chunk shapes across parts), each chunk a shuffled-u16 zstd frame."""
    levels = [_level0((64, 256, 256))]
    for _ in range(3):
        levels.append(_mean2(levels[-1]))
    chunks = [[16, 128, 128], [16, 64, 64], [16, 32, 32], [8, 32, 32]]
    co = O.OracleChain.from_metadata(C5_CODECS, "uint16", 0, 3)
    enc = []
    for a, cs in zip(levels, chunks):
        lv = []
        for i in range(a.shape[0] // cs[0]):
            for j in range(a.shape[1] // cs[1]):
                for k in range(a.shape[2] // cs[2]):
                    blk = np.ascontiguousarray(a[i * cs[0]:(i + 1) * cs[0], j * cs[1]:(j + 1) * cs[1],
                                                 k * cs[2]:(k + 1) * cs[2]])
                    lv.append(((i * cs[0], j * cs[1], k * cs[2]), co.encode(blk)))
        enc.append(lv)
    return levels, chunks, enc


@pytest.fixture(scope="module")
def ctx():
    from zarrs_amd import Context
    return Context(0)


def _parts(ctx, pyramid, corrupt=None):
    import torch
    from zarrs_amd import CodecChain, make_desc
    levels, chunks, enc = pyramid
    ch = CodecChain.from_metadata(C5_CODECS, "uint16", 0, ctx)
    keep, parts, outs = [], [], []
    for li, (a, cs, lv) in enumerate(zip(levels, chunks, enc)):
        descs = []
        for ci, (start, e) in enumerate(lv):
            b = bytearray(e)
            if corrupt == (li, ci):  # the frame magic: CORRUPT_STREAM whatever the frame holds
                b[0] ^= 0xFF
            t = torch.frombuffer(b, dtype=torch.uint8).cuda()
            keep.append(t)
            descs.append(make_desc(t, cs, out_start=list(start)))
        parts.append((ch, descs, list(a.shape)))
        outs.append(torch.zeros(a.shape, dtype=torch.int16, device="cuda"))
    return ch, keep, parts, outs


@pytest.mark.parametrize("lanes", ["4", "2", "1"])
def test_group_pyramid_vs_oracle(ctx, pyramid, lanes, monkeypatch):
    """Every level bit-exact vs the oracle whatever the lane count; every status 0."""
    monkeypatch.setenv("ZGPU_GROUP_LANES", lanes)
    from zarrs_amd import PlanGroup
    levels = pyramid[0]
    ch, keep, parts, outs = _parts(ctx, pyramid)
    g = PlanGroup(parts)
    try:
        for rep in range(2):  # the group re-executes (plans reused)
            for o in outs:
                o.fill_(0x5A5A)
            st = g.execute(outs)
            assert st == [0] * sum(len(p[1]) for p in parts)
            for li, (a, o) in enumerate(zip(levels, outs)):
                assert np.array_equal(o.cpu().numpy().view(np.uint16), a), (lanes, rep, li)
        layout = g.layout()
        used = {lane for lane, _, _ in layout}
        assert len(used) <= int(lanes)
        assert {p for _, p, _ in layout} == set(range(len(parts)))
        assert g.algorithmic_bytes() > 0
    finally:
        g.close()


def test_group_layout_policy(ctx, pyramid, monkeypatch):
    """4 lanes: level 0 (the bulk of the encoded bytes) split over the lanes left over, level 1 on a
    lane of its own, the two small levels sharing the last lane, largest first; literals-first on level
    0's first piece and on the small-part lane."""
    monkeypatch.setenv("ZGPU_GROUP_LANES", "4")
    from zarrs_amd import PlanGroup
    ch, keep, parts, outs = _parts(ctx, pyramid)
    total = sum(d.enc_len for p in parts for d in p[1])
    share = [sum(d.enc_len for d in p[1]) / total for p in parts]
    assert share[0] > 0.5 and share[1] >= 1 / 16 and share[2] < 1 / 16 and share[3] < 1 / 16, share
    g = PlanGroup(parts)
    try:
        layout = g.layout()  # (lane, part, literals-first) per plan, in creation order
        assert layout == [(0, 0, True), (1, 0, False), (2, 1, False), (3, 2, True), (3, 3, True)], layout
    finally:
        g.close()


def test_group_status_order(ctx, pyramid):
    """A corrupt frame in one level: its status lands at its place in the concatenated (part order)
    status list, the other levels still decode, and the call raises the first failing status."""
    from zarrs_amd import PlanGroup, ZgpuError
    levels = pyramid[0]
    bad = (2, 2)
    ch, keep, parts, outs = _parts(ctx, pyramid, corrupt=bad)
    g = PlanGroup(parts)
    try:
        with pytest.raises(ZgpuError) as ei:
            g.execute(outs)
        assert ei.value.status == 4
        st = list(g.status[: sum(len(p[1]) for p in parts)])
        pos = sum(len(p[1]) for p in parts[:bad[0]]) + bad[1]
        assert st[pos] == 4 and sum(1 for s in st if s) == 1, [i for i, s in enumerate(st) if s]
        for li in (0, 1, 3):
            assert np.array_equal(outs[li].cpu().numpy().view(np.uint16), levels[li]), li
    finally:
        g.close()
