#!/usr/bin/env python3
"""bench.py — decoded-array GiB/s of the MI355X chunk-decode pipeline on device-resident chunks.

Workload (BASELINE.json configs[1]): 4096 independent 64^3 float32 chunks per GPU
(a [1024,1024,1024] array, 4 GiB encoded + 4 GiB decoded), codecs
[transpose{order:[2,1,0]}, bytes{endian:big}], encoded chunks resident in HBM, decoded into one
device output array. One step = one zgpu_plan_execute over the whole 4096-chunk batch, per-chunk
statuses read back (the full decode, nothing skipped). N GPUs: one process per GPU, each decodes its
own 4096 chunks (weak scaling, no data-path collective); time = max over ranks.

Prints ONE JSON line (rank 0). Extra objects:
  roofline      dominant kernel (k_scatter_tiled<4>): algorithmic bytes per launch / average step
                time from HIP events on the launch stream, against 8.0 TB/s HBM3E
  cpu_baseline  the oracle (C restatement of zarrs' per-chunk pipeline, oracle/) on the host cores,
                rank 0 only, on a bounded sample of the same workload
"""
from __future__ import annotations

import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "decoded-array GiB/s, device-resident chunks, 1/2/4/8 MI355X; % HBM roofline"
CODECS = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
          {"name": "bytes", "configuration": {"endian": "big"}}]
CHUNK = 64


def gen_decoded(shape, seed, device):
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return torch.rand(shape, generator=g, device=device, dtype=torch.float32) * 2 - 1


def encode_c2(dec: torch.Tensor) -> torch.Tensor:
    """[G0*64, G1*64, G2*64] f32 -> encoded chunks [n_chunks, 64,64,64] (transpose [2,1,0], big endian),
    chunk-major in C order of the chunk grid, as uint8 [n_chunks * 1 MiB]."""
    g0, g1, g2 = (s // CHUNK for s in dec.shape)
    t = dec.view(g0, CHUNK, g1, CHUNK, g2, CHUNK).permute(0, 2, 4, 5, 3, 1)  # chunk(i,j,k), enc(k,j,i)
    t = t.contiguous().view(torch.uint8).view(-1, 4).flip(1)  # big endian
    return t.contiguous().view(-1)


def run_gpu(args, rank, world, dev):
    from zarrs_amd import CodecChain, Context, make_desc
    from zarrs_amd import _lib as L
    grid = args.grid
    shape = [g * CHUNK for g in grid]
    n_chunks = grid[0] * grid[1] * grid[2]
    chunk_bytes = CHUNK ** 3 * 4
    dec_ref = gen_decoded(shape, 1234 + rank, dev)
    enc = encode_c2(dec_ref)
    torch.cuda.synchronize()
    ctx = Context(dev.index)
    chain = CodecChain.from_metadata(CODECS, "float32", 0.0, ctx)
    descs = []
    base = enc.data_ptr()
    for c in range(n_chunks):
        i, r = divmod(c, grid[1] * grid[2])
        j, k = divmod(r, grid[2])
        descs.append(make_desc((base + c * chunk_bytes, chunk_bytes), [CHUNK] * 3,
                               out_start=[i * CHUNK, j * CHUNK, k * CHUNK]))
    arr = (L.ChunkDesc * n_chunks)(*descs)
    out = torch.empty(shape, dtype=torch.float32, device=dev)
    plan = C.c_void_p()
    lib = L.load()
    L.check(lib.zgpu_plan_create(chain._h, 3, arr, n_chunks, L.u64s(shape), L.ENC_DEVICE | L.OUT_DEVICE,
                                 C.byref(plan)))
    status = (C.c_int32 * n_chunks)()
    stream = torch.cuda.Stream(dev)  # the library launches on this stream; events are recorded on it
    sp = C.c_void_p(stream.cuda_stream)

    def step():
        rc = lib.zgpu_plan_execute(plan, out.data_ptr(), status, sp)
        if rc:
            raise RuntimeError(f"decode failed: {L.STATUS_NAMES[rc]} {L.last_error()}")

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # round-trip property at full size: decode(encode(x)) == x, bit for bit
    ok = bool(torch.equal(out.view(torch.int32), dec_ref.view(torch.int32)))
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.barrier()
    elapsed = time.perf_counter() - t0
    if args.child:  # rocprofv3 --pmc pass: only the dispatches matter
        lib.zgpu_plan_destroy(plan)
        return None
    # Device time of one decode launch sequence (ctl memset + k_scatter_tiled), HIP events on the
    # stream the library launches on; enqueue-only executes (status=NULL), back to back.
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps):
        rc = lib.zgpu_plan_execute(plan, out.data_ptr(), None, sp)
        if rc:
            raise RuntimeError(f"decode failed: {L.STATUS_NAMES[rc]} {L.last_error()}")
    ev1.record(stream)
    torch.cuda.synchronize()
    ev_ms = ev0.elapsed_time(ev1) / args.steps
    # algorithmic bytes per launch of the dominant kernel: 1 MiB read + 1 MiB written per chunk
    alg_bytes = lib.zgpu_plan_algorithmic_bytes(plan)
    # host planning + upload included (zgpu_decode_batch form), for DESIGN.md
    t1 = time.perf_counter()
    reps = max(1, min(5, args.steps))
    for _ in range(reps):
        chain.decode_batch(descs, out, shape, enc_device=True, stream=sp)
    torch.cuda.synchronize()
    batch_ms = (time.perf_counter() - t1) / reps * 1e3
    lib.zgpu_plan_destroy(plan)
    host = None
    if args.host_leg and rank == 0:
        host = host_leg(chain, enc, shape, grid, chunk_bytes, n_chunks, dec_ref, sp)
    return dict(elapsed=elapsed, ev_ms=ev_ms, alg_bytes=alg_bytes, ok=ok, n_chunks=n_chunks,
                decoded_bytes=n_chunks * chunk_bytes, batch_ms=batch_ms, host=host)


def host_leg(chain, enc, shape, grid, chunk_bytes, n_chunks, dec_ref, sp):
    """PCIe-inclusive rates: encoded chunks in pinned host memory -> zgpu_decode_batch
    (H2D + decode) -> device array, and -> host array (+ D2H). Not the headline value."""
    from zarrs_amd import make_desc
    h_enc = enc.cpu().pin_memory()
    base = h_enc.data_ptr()
    descs = []
    for c in range(n_chunks):
        i, r = divmod(c, grid[1] * grid[2])
        j, k = divmod(r, grid[2])
        descs.append(make_desc((base + c * chunk_bytes, chunk_bytes), [CHUNK] * 3,
                               out_start=[i * CHUNK, j * CHUNK, k * CHUNK]))
    out = torch.empty(shape, dtype=torch.float32, device=enc.device)
    res = {}
    chain.decode_batch(descs, out, shape, enc_device=False, stream=sp)  # warm-up
    torch.cuda.synchronize()
    reps = 3
    t0 = time.perf_counter()
    for _ in range(reps):
        chain.decode_batch(descs, out, shape, enc_device=False, stream=sp)
    torch.cuda.synchronize()
    t = (time.perf_counter() - t0) / reps
    res["host_enc_to_device_out_GiBps"] = round(n_chunks * chunk_bytes / t / 2 ** 30, 2)
    ok = bool(torch.equal(out.view(torch.int32), dec_ref.view(torch.int32)))
    h_out = torch.empty(shape, dtype=torch.float32).pin_memory()
    chain.decode_batch(descs, h_out.numpy(), shape, enc_device=False, stream=sp)
    t0 = time.perf_counter()
    for _ in range(reps):
        chain.decode_batch(descs, h_out.numpy(), shape, enc_device=False, stream=sp)
    t = (time.perf_counter() - t0) / reps
    res["host_enc_to_host_out_GiBps"] = round(n_chunks * chunk_bytes / t / 2 ** 30, 2)
    res["roundtrip_ok"] = ok and bool(torch.equal(h_out.view(torch.int32), dec_ref.cpu().view(torch.int32)))
    return res


KERNEL = "k_scatter_tiled"


def pmc_traffic(args):
    """HBM traffic of the dominant kernel per launch from rocprofv3 PMC counters, in two separate
    passes (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950), corrected as
    /opt/skills/guides/MI355X_MICROARCH.md (HBM) prescribes: counters are in KiB; FETCH_SIZE counts
    exactly half the bytes of a wide (16 B/lane) coalesced streaming read on gfx950 -> x2;
    WRITE_SIZE is exact for 16-B streaming stores. Runs bench.py itself as a child under rocprofv3."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None, "rocprofv3 not found"
    vals = {}
    tmp = tempfile.mkdtemp(prefix="zgpu_pmc_")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = ["rocprofv3", "--pmc", ctr, "--kernel-include-regex", KERNEL, "-d", d, "-o", "pmc",
                   "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "--child",
                   "--steps", "2", "--warmup", "1", "--no-cpu", "--grid", *map(str, args.grid)]
            r = subprocess.run(cmd, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, timeout=240)
            if r.returncode:
                return None, f"rocprofv3 --pmc {ctr} rc={r.returncode}: {r.stderr.decode()[-200:]}"
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            v = [float(row["Counter_Value"]) for f in files for row in csv.DictReader(open(f))
                 if KERNEL in row["Kernel_Name"] and row["Counter_Name"] == ctr]
            if not v:
                return None, f"no {ctr} samples for {KERNEL}"
            vals[ctr] = sum(v) / len(v)
    except Exception as e:  # noqa: BLE001 - report, never fail the bench line on the profiler
        return None, f"pmc pass failed: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch = vals["FETCH_SIZE"] * 1024 * 2
    write = vals["WRITE_SIZE"] * 1024
    return {"bytes": int(fetch + write), "fetch_bytes": int(fetch), "write_bytes": int(write)}, None


def cpu_baseline(args):
    """Oracle (oracle/, C restatement of zarrs' per-chunk pipeline) on host cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    threads = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count() or 1
    g = args.cpu_grid
    shape = [x * CHUNK for x in g]
    n = g[0] * g[1] * g[2]
    rng = np.random.default_rng(7)
    dec = (rng.random(shape, dtype=np.float32) * 2 - 1)
    # encode exactly as the GPU workload: transpose [2,1,0] + big endian, chunk-major
    enc = np.ascontiguousarray(dec.reshape(g[0], CHUNK, g[1], CHUNK, g[2], CHUNK)
                               .transpose(0, 2, 4, 5, 3, 1)).astype(">f4")
    enc = enc.reshape(n, -1)
    chain = O.OracleChain.from_metadata(CODECS, "float32", 0.0, 3)
    ptrs = (C.c_void_p * n)(*[enc[c].ctypes.data for c in range(n)])
    lens = (C.c_uint64 * n)(*([CHUNK ** 3 * 4] * n))
    out = np.empty(shape, np.float32)
    O.retrieve_ptrs(chain, shape, [CHUNK] * 3, ptrs, lens, [0, 0, 0], shape, out, threads)  # warm-up
    assert np.array_equal(out, dec)
    times = []
    t_end = time.perf_counter() + args.cpu_seconds
    while len(times) < 5 or (time.perf_counter() < t_end and len(times) < 50):
        t0 = time.perf_counter()
        O.retrieve_ptrs(chain, shape, [CHUNK] * 3, ptrs, lens, [0, 0, 0], shape, out, threads)
        times.append(time.perf_counter() - t0)
    t = float(np.median(times))
    return {"value": round(n * CHUNK ** 3 * 4 / t / 2 ** 30, 3), "unit": "GiB/s", "cores": threads,
            "kind": "port",
            "sample": f"{n} of the 4096 chunks ({shape[0]}x{shape[1]}x{shape[2]} f32 subset), "
                      f"median of {len(times)} reps, oracle retrieve_array_subset with {threads} threads"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--grid", type=int, nargs=3, default=[16, 16, 16], help="chunk grid per GPU")
    ap.add_argument("--cpu-grid", type=int, nargs=3, default=[8, 8, 8], help="CPU baseline sample grid")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--no-host-leg", dest="host_leg", action="store_false",
                    help="skip the PCIe-inclusive (host input/output) leg")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    dev = torch.device("cuda", local)
    r = run_gpu(args, rank, world, dev)
    if args.child:
        return

    elapsed = torch.tensor([r["elapsed"]], dtype=torch.float64, device=dev)
    ok = torch.tensor([1 if r["ok"] else 0], dtype=torch.int32, device=dev)
    if world > 1:
        torch.distributed.all_reduce(elapsed, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
    t = float(elapsed.item())
    total_bytes = r["decoded_bytes"] * world * args.steps
    value = total_bytes / t / 2 ** 30
    cpu = None
    if rank == 0 and not args.no_cpu:
        cpu = cpu_baseline(args)
    traffic, traffic_note = None, "skipped (--no-pmc or N>1)"
    if rank == 0 and world == 1 and not args.no_pmc:
        traffic, traffic_note = pmc_traffic(args)
    if rank == 0:
        achieved = r["alg_bytes"] / (r["ev_ms"] * 1e-3) / 1e9
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (uniform [-1,1) f32, encoded on device; decode(encode(x)) == x checked)",
            "config": {"workload": "C2: 4096 independent 64^3 f32 chunks per GPU, "
                                   "[transpose{order:[2,1,0]}, bytes{endian:big}], device-resident",
                       "chunks_per_gpu": r["n_chunks"], "array_shape_per_gpu": [g * CHUNK for g in args.grid],
                       "parallelism": f"chunk-partitioned x{world}"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic["bytes"] if traffic else None,
                         "traffic_detail": traffic or traffic_note,
                         "kernel": "k_scatter_tiled<4>",
                         "alg_bytes_per_launch": r["alg_bytes"],
                         "avg_launch_ms_hip_events": round(r["ev_ms"], 4)},
            "cpu_baseline": cpu,
            "roundtrip_ok": bool(ok.item()),
            "decode_batch_ms_incl_host_planning": round(r["batch_ms"], 3),
            "host_leg": r["host"],
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
