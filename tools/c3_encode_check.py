"""Lab check (not product code): GPU gzip-encode C3 inner chunks (32^3 f32 of the C3 synth data) with
[bytes, gzip 1, crc32c], decode every one with the oracle (zlib) and with the GPU decoder, report
the chunks that fail and save the first failing input / encoded pair under gpurun_out/c3enc/.
Usage: python tools/c3_encode_check.py [n_shards]"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import bench  # noqa: E402
import oracle as O  # noqa: E402
from zarrs_amd import CodecChain, Context, make_desc  # noqa: E402

INNER = [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "gzip", "configuration": {"level": 1}},
         {"name": "crc32c"}]


def main():
    ns = int(sys.argv[1]) if len(sys.argv) > 1 else 1
    out_dir = os.path.join(ROOT, "gpurun_out", "c3enc")
    os.makedirs(out_dir, exist_ok=True)
    ctx = Context(0)
    ch = CodecChain.from_metadata(INNER, "float32", 0.0, ctx)
    co = O.OracleChain.from_metadata(INNER, "float32", 0.0, 3)
    S, I = 256, 32
    host = np.empty([S, S, S * ns], np.float32)
    bench._synth().synth_c3_values(bench._u64([0, 256, 768]), bench._u64(host.shape), host.ctypes.data, 16)
    x = torch.from_numpy(host).cuda()
    starts = [[a * I, b * I, c * I] for a in range(S // I) for b in range(S // I) for c in range(S * ns // I)]
    enc = ch.encode_chunks(x, [I] * 3, starts)
    torch.cuda.synchronize()
    bad = []
    for k, (e, st) in enumerate(zip(enc, starts)):
        b = e.cpu().numpy().tobytes()
        ref = np.ascontiguousarray(host[st[0]:st[0] + I, st[1]:st[1] + I, st[2]:st[2] + I])
        try:
            got = co.decode(b, [I] * 3)
            ok = np.array_equal(got.view(np.int32), ref.view(np.int32))
        except Exception as ex:  # noqa: BLE001
            ok, got = False, repr(ex)
        if not ok:
            bad.append(k)
            if len(bad) == 1:
                np.save(os.path.join(out_dir, "input.npy"), ref)
                with open(os.path.join(out_dir, "encoded.bin"), "wb") as f:
                    f.write(b)
                print("first bad chunk", k, "start", st, "enc bytes", len(b), "oracle:", str(got)[:200])
    print(f"{len(enc)} chunks, {len(bad)} fail the oracle decode: {bad[:20]}")
    print("sizes: min", min(int(e.numel()) for e in enc), "max", max(int(e.numel()) for e in enc),
          "raw", I ** 3 * 4)
    # the same through the sharded chain: whole shards, oracle decode per shard, then the GPU decode
    sh = [{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [I] * 3, "codecs": INNER,
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "end"}}]
    chs = CodecChain.from_metadata(sh, "float32", 0.0, ctx)
    cos = O.OracleChain.from_metadata(sh, "float32", 0.0, 3)
    sst = [[0, 0, k * S] for k in range(ns)]
    encs = chs.encode_chunks(x, [S] * 3, sst)
    for k, e in enumerate(encs):
        b = e.cpu().numpy().tobytes()
        try:
            got = cos.decode(b, [S] * 3)
            ok = np.array_equal(got.view(np.int32), host[:, :, k * S:(k + 1) * S].view(np.int32))
        except Exception as ex:  # noqa: BLE001
            ok, got = False, repr(ex)
        print("shard", k, "bytes", len(b), "oracle ok" if ok else f"oracle FAIL {str(got)[:200]}")
        if not ok and k == 0:
            with open(os.path.join(out_dir, "shard0.bin"), "wb") as f:
                f.write(b)
    out = torch.empty_like(x)
    try:
        r = chs.decode_batch([make_desc((e.data_ptr(), int(e.numel())), [S] * 3, out_start=st)
                              for e, st in zip(encs, sst)], out, list(x.shape), enc_device=True)
        print("GPU decode statuses", r, "equal", bool(torch.equal(out.view(torch.int32), x.view(torch.int32))))
    except Exception as ex:  # noqa: BLE001
        print("GPU decode error", repr(ex))


if __name__ == "__main__":
    main()
