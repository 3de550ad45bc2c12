"""CPU check of the synchronisation logic of k_gzip's segmented symbol decode (tools/gzip_seg_model.py
restates kernels/inflate.hip's ZG_INFLATE_SEG path): lanes decode stream regions from an early start,
validate against their predecessor's exit, re-decode when out of sync; the records of the valid lanes,
executed in order, must reproduce zlib's output exactly (dynamic, fixed and stored blocks; levels
1/6/9; tight overlaps that force repairs and record caps that end rounds early)."""
import os
import sys
import zlib

import numpy as np
import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import gzip_seg_model as M  # noqa: E402


def _gz(raw, level):
    co = zlib.compressobj(level, zlib.DEFLATED, 31)
    return co.compress(raw) + co.flush()


def _data(kind, n=4096):
    rng = np.random.default_rng(1)
    x = np.arange(n, dtype=np.float32)
    if kind == "smooth":
        return (np.rint(256 * np.sin(0.01 * x) + rng.standard_normal(n)) / 256).astype(np.float32).tobytes()
    if kind == "noise":
        return rng.integers(0, 256, n * 4, dtype=np.uint8).tobytes()
    if kind == "runs":
        return np.repeat(rng.integers(0, 4, n // 16, dtype=np.uint8), 64).tobytes()
    return b"ab" * 40  # tiny: a fixed-Huffman block


@pytest.mark.parametrize("kind", ["smooth", "noise", "runs", "tiny"])
@pytest.mark.parametrize("level", [1, 6, 9])
def test_segmented_decode_matches_zlib(kind, level):
    raw = _data(kind)
    gz = _gz(raw, level)
    st = {}
    assert M.inflate_seg(gz, stats=st) == raw == zlib.decompress(gz, 31)


def test_segmented_decode_repairs_and_caps():
    """Tiny overlaps (lanes start out of sync: repairs) and small record caps (rounds end early)."""
    raw = _data("smooth", 8192)
    gz = _gz(raw, 1)
    st = {}
    assert M.inflate_seg(gz, segb=256, ovl=32, cap=24, maxrep=3, stats=st) == raw
    assert st["repairs"] > 0
