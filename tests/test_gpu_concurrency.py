"""Concurrent calls on one context (zarrs calls a codec from many rayon workers at once: the
boundary is thread-safe and calls run side by side on the context's lanes, include/zgpu.h
"Threading"). Host-in / host-out and device-in / device-out decodes of different chunk sets from
12 threads at once, each checked against the CPU oracle."""
import threading

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

CHAINS = {
    "gzip_crc": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "gzip", "configuration": {"level": 1}},
                 {"name": "crc32c"}],
    "shuffle_zstd": [{"name": "bytes", "configuration": {"endian": "little"}},
                     {"name": "numcodecs.shuffle", "configuration": {"elementsize": 4}},
                     {"name": "zstd", "configuration": {"level": 3, "checksum": False}}],
    "transpose_be": [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
                     {"name": "bytes", "configuration": {"endian": "big"}}],
}


@pytest.mark.parametrize("name", list(CHAINS))
def test_concurrent_calls_one_context(name):
    import torch
    from zarrs_amd import CodecChain, Context, make_desc
    codecs = CHAINS[name]
    ctx = Context(0)
    ch = CodecChain.from_metadata(codecs, "float32", 0.0, ctx)
    co = O.OracleChain.from_metadata(codecs, "float32", 0.0, 3)
    cs = [16, 32, 32]
    jobs = []
    for t in range(12):
        rng = np.random.default_rng(100 + t)
        a = np.round(rng.standard_normal((48, 32, 64)) * 64).astype(np.float32) / 64
        chunks = {}
        for i in range(3):
            for k in range(2):
                chunks[(i, k)] = co.encode(np.ascontiguousarray(a[i * 16:(i + 1) * 16, :, k * 32:(k + 1) * 32]))
        jobs.append((a, chunks, t % 2 == 1))
    results = [None] * len(jobs)
    errors = []

    def run(j):
        a, chunks, on_device = jobs[j]
        try:
            for _ in range(3):
                if on_device:
                    encs = {k: torch.frombuffer(bytearray(v), dtype=torch.uint8).cuda() for k, v in chunks.items()}
                    out = torch.zeros(a.shape, dtype=torch.float32, device="cuda")
                    descs = [make_desc(e, cs, out_start=[i * 16, 0, k * 32]) for (i, k), e in encs.items()]
                    s = torch.cuda.Stream()
                    # the inputs' H2D copies and the output's zero fill ran on this thread's current
                    # stream: the decode's stream waits for them (a caller stream is not ordered
                    # after other streams by the library, zgpu.h "Stream ordering")
                    s.wait_stream(torch.cuda.current_stream())
                    with torch.cuda.stream(s):
                        st = ch.decode_batch(descs, out, list(a.shape), enc_device=True, stream=s.cuda_stream)
                    s.synchronize()
                    got = out.cpu().numpy()
                else:
                    out = np.zeros(a.shape, np.float32)
                    descs = [make_desc(e, cs, out_start=[i * 16, 0, k * 32]) for (i, k), e in chunks.items()]
                    st = ch.decode_batch(descs, out, list(a.shape), enc_device=False)
                    got = out
                if st != [0] * len(descs) or not np.array_equal(got, a):
                    results[j] = False
                    return
            results[j] = True
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    threads = [threading.Thread(target=run, args=(j,)) for j in range(len(jobs))]
    for t in threads:
        t.start()
    for t in threads:
        t.join(timeout=120)
    assert not errors, errors
    assert all(results), results
