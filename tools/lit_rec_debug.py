"""Lab (not product code): where the zstd literal record path differs on the blosc test data."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))  # oracle/oracle.py (the checker)
import oracle as O  # noqa: E402
from zarrs_amd import CodecChain, Context, make_desc  # noqa: E402

ctx = Context(0)
cname, shuffle, ts = sys.argv[1], sys.argv[2], int(sys.argv[3])
DT = {1: "uint8", 2: "uint16", 4: "float32", 8: "float64"}
rng = np.random.default_rng(ts * 7 + len(cname) + len(shuffle))


def _data(n):
    a = rng.standard_normal(n) * 40
    a[: n // 2] = np.round(a[: n // 2])
    if ts == 1:
        return (a % 200).astype(np.uint8)
    if ts == 2:
        return np.abs(a).astype(np.uint16)
    return a.astype(DT[ts])


def blosc(bsz):
    return {"name": "blosc", "configuration": {"cname": cname, "clevel": 5, "shuffle": shuffle, "typesize": ts,
                                               "blocksize": bsz}}


ch = CodecChain.from_metadata([{"name": "bytes", "configuration": {"endian": "little"}}, blosc(0)], DT[ts], 0, ctx)
for n, bsz in [(1, 0), (100, 0), (1000, 256), (4099, 1024), (33333, 0), (262147, 0), (5000, 4096)]:
    co = O.OracleChain.from_metadata([{"name": "bytes", "configuration": {"endian": "little"}}, blosc(bsz)], DT[ts], 0, 1)
    descs, keep, exp = [], [], []
    for k in range(3):
        a = _data(n)
        enc = co.encode(a)
        d = torch.frombuffer(bytearray(enc), dtype=torch.uint8).cuda()
        keep.append(d)
        descs.append(make_desc(d, [n], out_start=[k * n]))
        exp.append(a)
        if len(sys.argv) > 4:
            open(f"{sys.argv[4]}_{n}_{k}.bin", "wb").write(enc)
    out = np.zeros(3 * n, DT[ts])
    try:
        st = ch.decode_batch(descs, out, [3 * n], enc_device=True)
    except Exception as ex:  # noqa: BLE001
        st = repr(ex)
    e = np.concatenate(exp).view(np.uint8)
    o = out.view(np.uint8)
    bad = np.nonzero(e != o)[0]
    print(n, bsz, st, "mismatched bytes", len(bad), (bad[:8].tolist(), bad[-3:].tolist()) if len(bad) else "")
