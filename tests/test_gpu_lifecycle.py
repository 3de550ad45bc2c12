"""Object lifetimes across the C ABI: a context outlives the chains, plans and caches made on it, in
whatever order a garbage-collected binding (Python here, Rust's Drop in rust/zarrs_gpu) destroys them
(zgpu_ctx_refcount, include/zgpu.h). The round-4 bench died with SIGSEGV in __cxa_finalize after its
line was printed when contexts were closed while their chains and plans were still alive; the
subprocess cases below end the interpreter in exactly those states and require a clean exit."""
import ctypes as C
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CODECS = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
          {"name": "bytes", "configuration": {"endian": "big"}}]


def _chunk():
    a = np.random.default_rng(3).standard_normal((16, 16, 16)).astype(np.float32)
    return a, O.OracleChain.from_metadata(CODECS, "float32", 0.0, 3).encode(a)


def test_context_closed_before_chain_and_plan():
    import torch
    from zarrs_amd import CodecChain, Context, make_desc
    from zarrs_amd import _lib as L
    lib = L.load()
    a, enc = _chunk()
    ctx = Context(0)
    assert ctx.refcount() == 1
    chain = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    assert ctx.refcount() == 2
    d = torch.frombuffer(bytearray(enc), dtype=torch.uint8).cuda()
    descs = (L.ChunkDesc * 1)(make_desc(d, [16, 16, 16]))
    plan = C.c_void_p()
    L.check(lib.zgpu_plan_create(chain._h, 3, descs, 1, L.u64s([16, 16, 16]), L.ENC_DEVICE | L.OUT_DEVICE,
                                 C.byref(plan)))
    assert ctx.refcount() == 3
    raw = ctx._h
    ctx.close()  # the caller's reference only: the chain and the plan keep the context alive
    assert lib.zgpu_ctx_refcount(raw) == 2
    out = torch.empty((16, 16, 16), dtype=torch.float32, device="cuda")
    st = (C.c_int32 * 1)()
    L.check(lib.zgpu_plan_execute(plan, out.data_ptr(), st, None))
    assert st[0] == 0 and np.array_equal(out.cpu().numpy(), a)
    out.zero_()
    assert chain.decode_batch([make_desc(d, [16, 16, 16])], out, [16, 16, 16], enc_device=True) == [0]
    assert np.array_equal(out.cpu().numpy(), a)
    h = np.empty((16, 16, 16), np.float32)  # host in / host out, coalesced, on the closed handle's context
    assert chain.decode_batch_into([make_desc(np.frombuffer(enc, np.uint8), [16, 16, 16])], h, [0, 0, 0],
                                   [16, 16, 16], enc_device=False, coalesce=True) == [0]
    assert np.array_equal(h, a)
    lib.zgpu_plan_destroy(plan)
    assert lib.zgpu_ctx_refcount(raw) == 1
    del chain  # the last reference: the context is freed here


def test_cache_holds_its_context():
    from zarrs_amd import Context
    from zarrs_amd import _lib as L
    lib = L.load()
    ctx = Context(0)
    cache = C.c_void_p()
    L.check(lib.zgpu_cache_create(ctx._h, 1 << 20, C.byref(cache)))
    raw = ctx._h
    assert ctx.refcount() == 2
    ctx.close()
    assert lib.zgpu_ctx_refcount(raw) == 1
    lib.zgpu_cache_destroy(cache)


EXIT_CASES = {
    # contexts never closed, chains / plans alive at interpreter exit
    "leak_all": "pass",
    # context closed first, chain and plan dropped by the interpreter's teardown
    "ctx_first": "ctx.close()",
    # everything closed explicitly in the worst order
    "ordered_worst": "ctx.close(); lib.zgpu_plan_destroy(plan); del chain",
}


@pytest.mark.parametrize("case", sorted(EXIT_CASES))
def test_clean_interpreter_exit(case, tmp_path):
    a, enc = _chunk()
    np.save(tmp_path / "a.npy", a)
    (tmp_path / "enc.bin").write_bytes(enc)
    src = textwrap.dedent(f"""
        import ctypes as C, sys
        import numpy as np, torch
        sys.path.insert(0, {ROOT!r})
        from zarrs_amd import CodecChain, Context, make_desc
        from zarrs_amd import _lib as L
        from concurrent.futures import ThreadPoolExecutor
        lib = L.load()
        a = np.load({str(tmp_path / "a.npy")!r})
        enc = open({str(tmp_path / "enc.bin")!r}, "rb").read()
        ctx = Context(0)
        chain = CodecChain.from_metadata({CODECS!r}, "float32", 0.0, ctx)
        d = torch.frombuffer(bytearray(enc), dtype=torch.uint8).cuda()
        descs = (L.ChunkDesc * 1)(make_desc(d, [16, 16, 16]))
        plan = C.c_void_p()
        L.check(lib.zgpu_plan_create(chain._h, 3, descs, 1, L.u64s([16, 16, 16]), L.ENC_DEVICE | L.OUT_DEVICE,
                                     C.byref(plan)))
        out = torch.empty((16, 16, 16), dtype=torch.float32, device="cuda")
        L.check(lib.zgpu_plan_execute(plan, out.data_ptr(), None, None))
        def call(_):
            h = np.empty((16, 16, 16), np.float32)
            chain.decode_batch_into([make_desc(np.frombuffer(enc, np.uint8), [16, 16, 16])], h, [0, 0, 0],
                                    [16, 16, 16], enc_device=False, coalesce=True)
            return bool(np.array_equal(h, a))
        with ThreadPoolExecutor(8) as ex:
            assert all(ex.map(call, range(32)))
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), a)
        {EXIT_CASES[case]}
        print("done", flush=True)
    """)
    p = subprocess.run([sys.executable, "-c", src], capture_output=True, text=True, timeout=110)
    assert p.returncode == 0, f"rc={p.returncode}\n{p.stderr[-2000:]}"
    assert p.stdout.strip().endswith("done")


C5_CODECS = [{"name": "bytes", "configuration": {"endian": "little"}},
             {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
             {"name": "zstd", "configuration": {"level": 3, "checksum": False}}]


def test_pinned_calls_keep_pools_bounded(monkeypatch):
    """200 zgpu_decode_pinned calls of varying batch and chunk sizes (the per-codec plugin's pattern that
    exhausted device memory in the round-5 C5 drop-in leg): every result bit-exact, the device and pinned
    pools' free blocks within their caps (ZGPU_POOL_CAP_MB / ZGPU_PINNED_CAP_MB, read at context
    creation), and the blocks in use back to the same level after every call (zgpu_ctx_pool_stats)."""
    from zarrs_amd import CodecChain, Context, make_desc
    monkeypatch.setenv("ZGPU_POOL_CAP_MB", "256")
    monkeypatch.setenv("ZGPU_PINNED_CAP_MB", "128")
    ctx = Context(0)
    chain = CodecChain.from_metadata(C5_CODECS, "uint16", 0, ctx)
    co = O.OracleChain.from_metadata(C5_CODECS, "uint16", 0, 3)
    rng = np.random.default_rng(11)
    lives, frees, hfrees, hlives = [], [], [], []
    for i in range(200):
        n, rows = 1 + (i * 7) % 8, 1 + (i * 13) % 48
        base = rng.integers(0, 64, size=(1, 64, 64), dtype=np.uint16)
        chunks = [(base + rng.integers(0, 3, size=(rows, 64, 64), dtype=np.uint16) * (k + 1)).astype(np.uint16)
                  for k in range(n)]
        encs = [co.encode(c) for c in chunks]
        descs = [make_desc(np.frombuffer(e, np.uint8), [rows, 64, 64], out_start=[k * rows, 0, 0])
                 for k, e in enumerate(encs)]
        out = np.empty((n * rows, 64, 64), np.uint16)
        st = chain.decode_pinned_into(descs, out, [0, 0, 0], [n * rows, 64, 64], coalesce=(i % 2 == 0))
        assert st == [0] * n, (i, st)
        assert np.array_equal(out, np.concatenate(chunks)), i
        s = ctx.pool_stats()
        lives.append(s["dev_live"])
        frees.append(s["dev_free"])
        hlives.append(s["host_live"])
        hfrees.append(s["host_free"])
    assert max(frees) <= 256 << 20, max(frees)
    assert max(hfrees) <= 128 << 20, max(hfrees)
    # nothing accumulates in use: the second half of the calls holds no more than the first half did
    assert max(lives[100:]) <= max(lives[:100]), (max(lives[:100]), max(lives[100:]))
    assert max(hlives[100:]) <= max(hlives[:100]), (max(hlives[:100]), max(hlives[100:]))
    ctx.release_cached()
    s = ctx.pool_stats()
    assert s["dev_free"] == 0 and s["host_free"] == 0, s
    del chain
    ctx.close()
