"""CPU check of the snappy stream writer the blosc GPU tests use (tests/test_gpu_blosc.py: the host
c-blosc has no snappy, so those tests write their own frames): every stream it emits decodes, with a
decoder written from google/snappy's format_description.txt, back to its input."""
import importlib.util
import os

import numpy as np


def _writer():
    spec = importlib.util.spec_from_file_location(
        "gpu_blosc_helpers", os.path.join(os.path.dirname(__file__), "test_gpu_blosc.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _snappy_decode(z: bytes) -> bytes:
    i = n = sh = 0
    while True:
        b = z[i]
        i += 1
        n |= (b & 127) << sh
        sh += 7
        if not b & 128:
            break
    out = bytearray()
    while i < len(z):
        t = z[i]
        i += 1
        if t & 3 == 0:
            ln = (t >> 2) + 1
            if ln > 60:
                nb = ln - 60
                ln = int.from_bytes(z[i:i + nb], "little") + 1
                i += nb
            out += z[i:i + ln]
            i += ln
            continue
        if t & 3 == 1:
            ln, off = 4 + ((t >> 2) & 7), ((t >> 5) << 8) | z[i]
            i += 1
        elif t & 3 == 2:
            ln, off = 1 + (t >> 2), int.from_bytes(z[i:i + 2], "little")
            i += 2
        else:
            ln, off = 1 + (t >> 2), int.from_bytes(z[i:i + 4], "little")
            i += 4
        assert 0 < off <= len(out)
        for _ in range(ln):
            out.append(out[-off])
    assert len(out) == n
    return bytes(out)


def test_snappy_writer_round_trip():
    m = _writer()
    rng = np.random.default_rng(3)
    forms = set()
    for k in range(24):
        a = m._data(rng, int(rng.integers(1, 30000)), 4).tobytes()
        if k % 3 == 0:
            a = bytes(np.repeat(np.frombuffer(a, np.uint8)[:200], 40))
        z = m._snappy_compress(a, rng)
        assert _snappy_decode(z) == a
        forms.update(b & 3 for b in z[1:])  # approximate: tag bytes and payload together
    assert {0, 1, 2, 3} <= forms
