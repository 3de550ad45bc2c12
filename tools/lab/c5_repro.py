"""Lab (not product code): decode selected C5 chunks of a given --c5-scale pyramid on the GPU, one
batch per case and all cases in one batch, and report mismatches against the source data.
Usage: python tools/lab/c5_repro.py SCALE [variant libzgpu.so ...]   (runs on the GPU box)"""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402  (data generation helpers)

scale = int(sys.argv[1]) if len(sys.argv) > 1 else 2
variants = sys.argv[2:] or [None]
CHUNKS = bench.C5.CHUNKS
shape0 = [512, 4096 // scale, 4096 // scale]
syn = bench._synth()
syn.synth_c5_level0.argtypes = [C.c_uint64] * 3 + [C.c_int] + [C.c_void_p] * 5 + [C.c_uint64, C.c_void_p, C.c_int]
syn.synth_shuffle_zstd_chunks.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                          C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
rng = np.random.default_rng(42)
nb = 64
cz, cy, cx = (rng.uniform(0, s, nb).astype(np.float32) for s in shape0)
sg = rng.uniform(4, 40, nb).astype(np.float32)
amp = rng.uniform(300, 4000, nb).astype(np.float32)
lvl = np.empty(shape0, np.uint16)
nt = bench._threads()
syn.synth_c5_level0(*shape0, nb, cz.ctypes.data, cy.ctypes.data, cx.ctypes.data, sg.ctypes.data, amp.ctypes.data,
                    42, lvl.ctypes.data, nt)
levels = [lvl]
for _ in range(2):
    a = levels[-1].astype(np.uint32)
    z, y, x = a.shape
    m = a.reshape(z // 2, 2, y // 2, 2, x // 2, 2).sum(axis=(1, 3, 5))
    levels.append(((m + 4) // 8).astype(np.uint16))
cases = [(0, (7, 0, 1)), (0, (8, 0, 1)), (0, (11, 3, 1)), (2, (1, 1, 2)), (2, (1, 0, 1)), (0, (0, 0, 0))]
if os.environ.get("C5_CASES"):  # "level:i,j,k;level:i,j,k..."
    cases = [(int(c.split(":")[0]), tuple(int(x) for x in c.split(":")[1].split(",")))
             for c in os.environ["C5_CASES"].split(";")]
blks, encs = [], []
for li, idx in cases:
    cs = CHUNKS[li]
    sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(idx, cs))
    blk = np.ascontiguousarray(levels[li][sl])
    flat = blk.reshape(-1).view(np.uint8)
    offs = np.zeros(1, np.uint64)
    lens = np.array([flat.nbytes], np.uint64)
    outs = (C.c_void_p * 1)()
    olens = (C.c_uint64 * 1)()
    assert syn.synth_shuffle_zstd_chunks(flat.ctypes.data, 2, offs.ctypes.data, lens.ctypes.data, 1, 3, 0, 1,
                                         outs, olens) == 0
    encs.append(bytes((C.c_uint8 * olens[0]).from_address(outs[0])))
    syn.synth_free(C.c_void_p(outs[0]))
    blks.append(blk)
print("encoded", [len(e) for e in encs], flush=True)
for v in variants:
    import zarrs_amd._lib as L
    if v:
        L.LIB_PATH = os.path.abspath(v)
    L._lib = None
    import torch
    from zarrs_amd import CodecChain, Context, make_desc
    ctx = Context(0)
    ch = CodecChain.from_metadata(bench.C5.CODECS, "uint16", 0, ctx)
    devs = [torch.frombuffer(bytearray(e), dtype=torch.uint8).cuda() for e in encs]
    res = []
    reps = int(os.environ.get("C5_REPS", "1"))
    for (li, idx), blk, d in [c for c in zip(cases, blks, devs) for _ in range(reps)]:
        out = torch.zeros(blk.shape, dtype=torch.int16, device="cuda")
        st = ch.decode_batch([make_desc(d, list(blk.shape))], out, list(blk.shape), enc_device=True)
        got = out.cpu().numpy().view(np.uint16)
        res.append((li, idx, st[0], int((got != blk).sum())))
    print(v or "libzgpu.so", "single:", res, flush=True)
    # all cases of one level in one batch, side by side along axis 0
    for li0 in (0, 2):
        sel = [k for k, (li, _) in enumerate(cases) if li == li0]
        if not sel:
            continue
        cs = CHUNKS[li0]
        out = torch.zeros([cs[0] * len(sel)] + cs[1:], dtype=torch.int16, device="cuda")
        descs = [make_desc(devs[k], cs, out_start=[j * cs[0], 0, 0]) for j, k in enumerate(sel)]
        st = ch.decode_batch(descs, out, list(out.shape), enc_device=True)
        got = out.cpu().numpy().view(np.uint16)
        bad = [int((got[j * cs[0]:(j + 1) * cs[0]] != blks[k]).sum()) for j, k in enumerate(sel)]
        print(v or "libzgpu.so", f"batch level {li0}:", st, bad, flush=True)

# byte-level view of the first failing case: zstd alone on the shuffled bytes, block table
if os.environ.get("C5_BYTES"):
    import torch
    from zarrs_amd import CodecChain, Context, make_desc
    import zarrs_amd._lib as L
    L.LIB_PATH = os.path.join(ROOT, "zarrs_amd", "lib", "libzgpu.so")
    L._lib = None
    k = 0
    e = encs[k]
    raw = np.ascontiguousarray(blks[k]).reshape(-1).view(np.uint8)
    sh = np.concatenate([raw[0::2], raw[1::2]])
    ch = CodecChain.from_metadata([{"name": "bytes", "configuration": {"endian": "little"}},
                                   {"name": "zstd", "configuration": {"level": 3, "checksum": False}}],
                                  "uint8", 0, Context(0))
    d = torch.frombuffer(bytearray(e), dtype=torch.uint8).cuda()
    out = torch.zeros(sh.size, dtype=torch.uint8, device="cuda")
    ch.decode_batch([make_desc(d, [sh.size])], out, [sh.size], enc_device=True)
    got = out.cpu().numpy()
    bad = np.nonzero(got != sh)[0]
    print("bytes: bad", bad.size, "first", bad[:8].tolist(), "last", bad[-4:].tolist() if bad.size else None)
    # frame header (RFC 8878 3.1.1.1) then block headers
    p = 4
    fhd = e[p]; p += 1
    fcs_flag, single = fhd >> 6, (fhd >> 5) & 1
    if not single:
        p += 1
    p += [0, 1, 2, 4][fhd & 3]
    p += [1 if single else 0, 2, 4, 8][fcs_flag]
    pos, bi = 0, 0
    while True:
        h = e[p] | (e[p + 1] << 8) | (e[p + 2] << 16)
        last, typ, size = h & 1, (h >> 1) & 3, h >> 3
        p += 3
        osz = size if typ != 2 else None
        info = ""
        if typ == 2:
            lh = e[p]
            ltype, sf = lh & 3, (lh >> 2) & 3
            if ltype in (0, 1):
                regen = lh >> 3 if sf in (0, 2) else ((lh >> 4) | (e[p + 1] << 4) if sf == 1 else (lh >> 4) | (e[p + 1] << 4) | (e[p + 2] << 12))
            else:
                b = int.from_bytes(e[p:p + 5], "little")
                regen = (b >> 4) & ((1 << [10, 10, 14, 18][sf]) - 1)
            info = f"ltype {ltype} regen {regen}"
        lo = pos
        print(f"block {bi} type {typ} size {size} {info} out_start {lo if osz is not None or bi == 0 else '?'}")
        p += size if typ != 1 else 1
        bi += 1
        if typ != 2:
            pos += size
        else:
            pos = None if pos is None else pos
        if last or bi > 200:
            break
