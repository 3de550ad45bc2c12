"""N>1 read paths with the HIP decode on every rank (configs C4 and C5's 8-GPU leg).

Two ranks share the box's one GPU (device 0): each rank decodes its share through libzgpu (the HIP
kernels, not the oracle) and the results are gathered to rank 0 over gloo, staged through host
memory (RCCL cannot pair two ranks on one device; the exchange logic is the same code path that
runs over RCCL/xGMI on an 8-GPU node). Rank 0 compares the gathered subset with the CPU oracle.

  C4 pattern: C3's exact chain ([bytes, gzip 1, crc32c] inner chunks, [bytes, crc32c] index at the
              end), subset split into axis-0 slabs, slabs gathered into rank 0's subset; and split
              into stream-balanced inner-chunk lines (partition="lines", each rank's boxes decoded
              as one batch by Array.retrieve_boxes_into), boxes gathered with gather_regions
  C5 pattern: u16 [bytes, numcodecs.shuffle{2}, zstd{3}] chunks LPT-partitioned by encoded size,
              each rank decodes its chunks into its own level array (one zgpu_decode_batch), one
              cross-rank subset gathered with gather_regions (packed boxes and in-place boxes)
"""
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

C3_CODECS = [{"name": "sharding_indexed", "configuration": {
    "chunk_shape": [8, 8, 8],
    "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
               {"name": "gzip", "configuration": {"level": 1}}, {"name": "crc32c"}],
    "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
    "index_location": "end"}}]
C5_CODECS = [{"name": "bytes", "configuration": {"endian": "little"}},
             {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
             {"name": "zstd", "configuration": {"level": 3, "checksum": False}}]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _c3_array():
    rng = np.random.default_rng(3)
    z, y, x = np.meshgrid(np.arange(64), np.arange(48), np.arange(48), indexing="ij")
    v = np.round((np.sin(0.05 * x) + np.cos(0.03 * y) + 0.5 * np.sin(0.07 * z)) * 256) / 256
    return (v + rng.standard_normal(v.shape) / 256).astype(np.float32)


def _c5_level():
    rng = np.random.default_rng(42)
    lvl = (100 + rng.poisson(50, (16, 96, 80))).astype(np.uint16)
    lvl[2:12, 10:70, 8:60] += 3000
    return lvl


def _encode_chunks(co, a, cs):
    out = {}
    for idx in np.ndindex(*[-(-s // c) for s, c in zip(a.shape, cs)]):
        blk = np.zeros(cs, a.dtype)
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, cs, a.shape))
        blk[tuple(slice(0, n) for n in a[sl].shape)] = a[sl]
        out[idx] = co.encode(blk)
    return out


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import torch
    import torch.distributed as dist
    import oracle as O
    from zarrs_amd import Array, CodecChain, Context, DeviceStore, MemoryStore, make_desc
    from zarrs_amd.distributed import chunk_boxes, gather_regions, lpt_partition, retrieve_array_subset_distributed
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        ctx = Context(0)
        dev = torch.device("cuda", 0)
        # ---- C4: sharded gzip+crc32c array, axis-0 slabs decoded on the GPU, gathered to rank 0
        a = _c3_array()
        shard = [16, 16, 16]
        co = O.OracleChain.from_metadata(C3_CODECS, "float32", 0.0, 3)
        shards = _encode_chunks(co, a, shard)
        store = DeviceStore.from_store(MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in shards.items()}))
        meta = {"shape": list(a.shape), "data_type": "float32", "fill_value": 0.0, "codecs": C3_CODECS,
                "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": shard}}}
        arr = Array(store, meta, ctx)
        for name, (start, shape) in {"c4_even": ([5, 3, 7], [50, 40, 33]),
                                     "c4_ragged": ([1, 0, 0], [63, 48, 48]),
                                     "c4_thin": ([30, 2, 2], [3, 5, 40])}.items():
            got = retrieve_array_subset_distributed(arr, start, shape, device=dev)
            lines = retrieve_array_subset_distributed(arr, start, shape, device=dev, partition="lines")
            if rank == 0:
                exp = O.retrieve_array_subset(co, list(a.shape), shard, shards, start, shape, nthreads=4)
                res[name] = got is not None and got.is_cuda and got.cpu().numpy().tobytes() == exp.tobytes()
                # bench.py's C4 cut: stream-balanced inner-chunk lines, each rank's boxes in one batch
                res[name + "_lines"] = (lines is not None and lines.is_cuda and
                                        lines.cpu().numpy().tobytes() == exp.tobytes())
            else:
                res[name] = got is None
                res[name + "_lines"] = lines is None
        # ---- C5: zstd+shuffle u16 chunks LPT-partitioned, each rank decodes its own on the GPU
        lvl = _c5_level()
        cs = [8, 32, 32]
        co5 = O.OracleChain.from_metadata(C5_CODECS, "uint16", 0, 3)
        chunks = _encode_chunks(co5, lvl, cs)
        keys = sorted(chunks)
        parts = lpt_partition([len(chunks[k]) for k in keys], world)
        owner = {keys[i]: r for r, p in enumerate(parts) for i in p}
        chain = CodecChain.from_metadata(C5_CODECS, "uint16", 0, ctx)
        local = torch.zeros(lvl.shape, dtype=torch.int16, device=dev)
        bufs, descs = [], []
        for k in keys:
            if owner[k] != rank:
                continue
            st = [i * c for i, c in zip(k, cs)]
            sel = [min(c, s - o) for c, s, o in zip(cs, lvl.shape, st)]
            t = torch.frombuffer(bytearray(chunks[k]), dtype=torch.uint8).to(dev)
            bufs.append(t)
            descs.append(make_desc(t, cs, [0, 0, 0], sel, st))
        status = chain.decode_batch(descs, local, list(lvl.shape), enc_device=True)
        res["c5_decode_ok"] = all(v == 0 for v in status)
        host = local.cpu()  # gloo: staged through host memory
        for name, (sub0, subn) in {"c5_gather_packed": ([3, 20, 10], [10, 60, 65]),
                                   "c5_gather_in_place": ([0, 32, 0], [16, 32, 80])}.items():
            boxes = [[] for _ in range(world)]
            for idx, b0, bs in chunk_boxes(list(lvl.shape), cs, sub0, subn):
                boxes[owner[idx]].append((b0, bs))
            res[name + "_spans_ranks"] = all(len(b) > 0 for b in boxes)
            got = gather_regions(host, boxes, sub0, subn)
            if rank == 0:
                sl = tuple(slice(o, o + n) for o, n in zip(sub0, subn))
                res[name] = bool(np.array_equal(got.numpy().view(np.uint16), lvl[sl]))
            else:
                res[name] = got is None
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 - reported through the queue
        res["error"] = repr(e)
    finally:
        q.put((rank, res))
        dist.destroy_process_group()


def test_two_ranks_hip_decode_and_gather():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 2
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in range(world):
        assert "error" not in out[r], out
        assert out[r] and all(out[r].values()), out


def _overlap_worker(rank, world, port, q):
    """C4 with the gather overlapped with the decode (gather_slabs_overlapped): each rank decodes its
    axis-0 slab on the GPU in pieces of whole shard rows and sends each piece while the next decodes;
    rank 0 receives every piece straight into place and checks EVERY slab against the oracle."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    import time
    import torch
    import torch.distributed as dist
    import oracle as O
    from zarrs_amd import Array, Context, DeviceStore, MemoryStore
    from zarrs_amd.distributed import retrieve_array_subset_distributed, slab_mismatches, slab_partition
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    try:
        ctx = Context(0)
        dev = torch.device("cuda", 0)
        a = _c3_array()
        shard = [16, 16, 16]
        co = O.OracleChain.from_metadata(C3_CODECS, "float32", 0.0, 3)
        shards = _encode_chunks(co, a, shard)
        store = DeviceStore.from_store(MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in shards.items()}))
        meta = {"shape": list(a.shape), "data_type": "float32", "fill_value": 0.0, "codecs": C3_CODECS,
                "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": shard}}}
        arr = Array(store, meta, ctx)
        for name, (start, shape, rows) in {"shard_rows": ([5, 3, 7], [57, 40, 33], 16),
                                          "inner_rows": ([1, 0, 0], [63, 48, 48], 8)}.items():
            dist.barrier()
            t0 = time.perf_counter()
            got = retrieve_array_subset_distributed(arr, start, shape, device=dev, piece_rows=rows)
            torch.cuda.synchronize()
            res[name + "_ms"] = (time.perf_counter() - t0) * 1e3
            if rank == 0:
                exp = O.retrieve_array_subset(co, list(a.shape), shard, shards, start, shape, nthreads=4)
                bad = slab_mismatches(got.cpu(), torch.from_numpy(exp), slab_partition(start, shape, world))
                res[name] = got.is_cuda and not bad
            else:
                res[name] = got is None
        torch.cuda.synchronize()
    except Exception as e:  # noqa: BLE001 - reported through the queue
        res["error"] = repr(e)
    finally:
        q.put((rank, res))
        dist.destroy_process_group()


def test_three_ranks_overlapped_gather_hip_decode():
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    world = 3
    procs = [ctx.Process(target=_overlap_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=100) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for r in range(world):
        assert "error" not in out[r], out
        assert all(v for k, v in out[r].items() if not k.endswith("_ms")), out
    print({r: {k: round(v, 2) for k, v in out[r].items() if k.endswith("_ms")} for r in out})


def test_retrieve_boxes_into_one_batch():
    """Array.retrieve_boxes_into: a rank's chunk_line_partition boxes decoded as one batch into its slab
    (the HIP decode), equal to the oracle inside the boxes and untouched (sentinel) outside them; an
    absent shard reads as the fill value."""
    import torch
    import oracle as O
    from zarrs_amd import Array, Context, DeviceStore, MemoryStore
    from zarrs_amd.distributed import chunk_line_partition
    a = _c3_array()
    shard = [16, 16, 16]
    co = O.OracleChain.from_metadata(C3_CODECS, "float32", 0.0, 3)
    shards = _encode_chunks(co, a, shard)
    del shards[(1, 1, 1)]  # absent: the fill value
    a[16:32, 16:32, 16:32] = 0
    meta = {"shape": list(a.shape), "data_type": "float32", "fill_value": 0.0, "codecs": C3_CODECS,
            "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": shard}}}
    arr = Array(DeviceStore.from_store(MemoryStore({"c/" + "/".join(map(str, k)): v for k, v in shards.items()})),
                meta, Context(0))
    assert arr.read_chunk_shape == [8, 8, 8]
    start, shape = [3, 5, 1], [50, 40, 45]
    for boxes in chunk_line_partition(start, shape, arr.read_chunk_shape, 3):
        r0 = min(b0[0] for b0, _ in boxes)
        r1 = max(b0[0] + bs[0] for b0, bs in boxes)
        origin = [r0] + start[1:]
        out = torch.full([r1 - r0] + shape[1:], -7.0, device="cuda")
        arr.retrieve_boxes_into(boxes, out, origin)
        got = out.cpu().numpy()
        exp = np.full(got.shape, -7.0, np.float32)
        for b0, bs in boxes:
            sl = tuple(slice(x - o, x - o + n) for x, o, n in zip(b0, origin, bs))
            exp[sl] = a[tuple(slice(x, x + n) for x, n in zip(b0, bs))]
        assert got.tobytes() == exp.tobytes()
