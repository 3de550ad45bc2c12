"""Latency floor of one drop-in call: one C3 shard (or a few of its inner chunks) decoded from HBM,
repeated; run under rocprofv3 --kernel-trace --stats to split the call into its kernels."""
import ctypes as C
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

import bench  # noqa: E402
from zarrs_amd import CodecChain, Context, make_desc  # noqa: E402

ctx = Context(0)
syn = bench._synth()
S, I = 256, 32
dec = np.empty([S] * 3, np.float32)
syn.synth_c3_values(bench._u64([256, 256, 256]), bench._u64([S] * 3), dec.ctypes.data, 16)
p, n = C.c_void_p(), C.c_uint64()
assert not syn.synth_gzip_crc_shard(dec.ctypes.data, 4, bench._u64([S] * 3), bench._u64([I] * 3), 1, 16,
                                    C.byref(p), C.byref(n))
host = np.ctypeslib.as_array((C.c_uint8 * n.value).from_address(p.value)).copy()
dev = torch.from_numpy(host).cuda()
chain = CodecChain.from_metadata(bench.C3.CODECS, "float32", 0.0, ctx)
out = torch.empty([S] * 3, dtype=torch.float32, device="cuda")
for name, sel in (("full shard (512 streams)", [S] * 3), ("16 rows: 8x8x8 inner = 512", [S] * 3),
                  ("partial 32x256x256 (64 streams)", [32, S, S]), ("partial 32x32x256 (8 streams)", [32, 32, S]),
                  ("one inner chunk", [32, 32, 32])):
    d = make_desc(dev, [S] * 3, [0, 0, 0], sel)
    o = out if sel == [S] * 3 else torch.empty(sel, dtype=torch.float32, device="cuda")
    for _ in range(3):
        chain.decode_batch([d], o, sel, enc_device=True)
    torch.cuda.synchronize()
    ts = []
    for _ in range(20):
        t0 = time.perf_counter()
        chain.decode_batch([d], o, sel, enc_device=True)
        ts.append(time.perf_counter() - t0)
    print(f"{name}: median {np.median(ts) * 1e3:.2f} ms, min {min(ts) * 1e3:.2f} ms", flush=True)
    assert torch.equal(o.cpu(), torch.from_numpy(dec[tuple(slice(0, k) for k in sel)]))
