#!/usr/bin/env python3
"""bench.py — decoded-array GiB/s of the MI355X chunk-decode pipeline on device-resident chunks.

Default workload (BASELINE.json configs[1]): 4096 independent 64^3 float32
chunks per GPU (a [1024,1024,1024] array, 4 GiB encoded + 4 GiB decoded), codecs
[transpose{order:[2,1,0]}, bytes{endian:big}], encoded chunks resident in HBM, decoded into one
device output array. One step = one zgpu_plan_execute over the whole batch with per-chunk statuses
read back (the full decode, nothing skipped). N GPUs: one process per GPU, each decodes its own
4096 chunks (chunks are independent: weak scaling, no data-path collective); time = max over ranks.

--workload c3: sharded [2048]^3 f32 array, 256^3 shards of 32^3 inner chunks,
[bytes, gzip 1, crc32c] + [bytes, crc32c] index; read the subset [200:968, 300:1068, 1000:1768]
(64 shards touched, 8 fully covered, 56 partial). With N GPUs the subset is split into N slabs along
axis 0 (each rank decodes the inner chunks its slab touches) and gathered to rank 0 over RCCL
inside the timed step (C4).

Prints ONE JSON line (rank 0). Extra objects:
  roofline      dominant kernel: algorithmic bytes per launch / device time per launch (HIP events on
                the stream the library launches on), against 8.0 TB/s HBM3E; traffic = HBM bytes
                per launch from rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE) of this same script
  cpu_baseline  the oracle (oracle/, C restatement of zarrs' per-chunk pipeline) on the host cores,
                rank 0 only, on a bounded sample of the same workload
  host_leg      (C2) PCIe-inclusive rates: encoded chunks in pinned host memory
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
# HIP runs with the environment's hardware-queue count (GPU_MAX_HW_QUEUES; HIP's default is 4): the
# line records the value it ran with (`hip_env`). Round 4 forced 8 here for the drop-in leg; that is a
# setting a zarrs user does not get, so the line is measured at the box's default.
import numpy as np  # noqa: E402
import torch  # noqa: E402

L_CTR_ZSTD_SERIAL, L_CTR_ZSTD_PARALLEL = 1, 2  # zgpu.h ZGPU_CTR_*
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec, /opt/skills/guides/MI355X_MICROARCH.md
METRIC = "decoded-array GiB/s, device-resident chunks, 1/2/4/8 MI355X; % HBM roofline"


def _threads():
    return int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or os.cpu_count() or 1


def _synth():
    path = os.path.join(ROOT, "tools", "synth", "libsynth.so")
    if not os.path.exists(path):
        raise RuntimeError(f"{path} missing: make -C tools/synth (or __graft_entry__.build())")
    L = C.CDLL(path)
    P64 = C.POINTER(C.c_uint64)
    L.synth_c3_values.argtypes = [P64, P64, C.c_void_p, C.c_int]
    L.synth_gzip_crc_shard.argtypes = [C.c_void_p, C.c_uint64, P64, P64, C.c_int, C.c_int,
                                       C.POINTER(C.c_void_p), P64]
    L.synth_free.argtypes = [C.c_void_p]
    L.synth_unshuffle.argtypes = [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64]
    L.synth_unshuffle.restype = None
    return L


def _emulated_rank(args, rank, world):
    """--emulate-rank R/N (one process, one GPU): the step decodes rank R's share of an N-GPU run (C3:
    its stream-balanced inner-chunk lines, C5: its LPT chunk part) with the single-GPU code path -- for profiling a rank's
    step (the rank_share legs time every rank this way from their own plans)."""
    spec = getattr(args, "emulate_rank", "")
    if not spec or world > 1:
        return rank, world
    r, n = (int(x) for x in spec.split("/"))
    return r, n


def _u64(v):
    return (C.c_uint64 * len(v))(*[int(x) for x in v])


# ------------------------------------------------------------------------------------------------
# C2
# ------------------------------------------------------------------------------------------------
class C2:
    CODECS = [{"name": "transpose", "configuration": {"order": [2, 1, 0]}},
              {"name": "bytes", "configuration": {"endian": "big"}}]
    CHUNK = 64
    kernel = "k_scatter_tiled"
    dtype = "f32"

    def __init__(self, args, rank, world, dev):
        from zarrs_amd import CodecChain, make_desc
        self.args, self.rank, self.world, self.dev = args, rank, world, dev
        grid = args.grid
        K = self.CHUNK
        self.shape = [g * K for g in grid]
        self.n_chunks = grid[0] * grid[1] * grid[2]
        self.chunk_bytes = K ** 3 * 4
        g = torch.Generator(device=dev)
        g.manual_seed(1234 + rank)
        self.dec_ref = torch.rand(self.shape, generator=g, device=dev, dtype=torch.float32) * 2 - 1
        self.enc = self.encode(self.dec_ref)
        self.chain = CodecChain.from_metadata(self.CODECS, "float32", 0.0, args.ctx)
        base = self.enc.data_ptr()
        self.descs = []
        for c in range(self.n_chunks):
            i, r = divmod(c, grid[1] * grid[2])
            j, k = divmod(r, grid[2])
            self.descs.append(make_desc((base + c * self.chunk_bytes, self.chunk_bytes), [K] * 3,
                                        out_start=[i * K, j * K, k * K]))
        self.out = torch.empty(self.shape, dtype=torch.float32, device=dev)
        self.out_shape = self.shape
        self.decoded_bytes = self.n_chunks * self.chunk_bytes  # per rank per step
        self.parts = [(self.chain, self.descs, self.out, self.out_shape)]
        self.step_bytes = self.decoded_bytes * world  # all ranks, one step
        self.config = {"workload": "C2: 4096 independent 64^3 f32 chunks per GPU, "
                                   "[transpose{order:[2,1,0]}, bytes{endian:big}], device-resident",
                       "chunks_per_gpu": self.n_chunks, "array_shape_per_gpu": self.shape,
                       "parallelism": f"chunk-partitioned x{world}"}
        self.data = "synthetic (uniform [-1,1) f32, encoded on device; decode(encode(x)) == x checked)"
        self.scaling = "weak"

    @classmethod
    def encode(cls, dec: torch.Tensor) -> torch.Tensor:
        """[G0*64, G1*64, G2*64] f32 -> encoded chunks (transpose [2,1,0], big endian), chunk-major
        in C order of the chunk grid, as uint8 [n_chunks * 1 MiB]."""
        K = cls.CHUNK
        g0, g1, g2 = (s // K for s in dec.shape)
        t = dec.view(g0, K, g1, K, g2, K).permute(0, 2, 4, 5, 3, 1)  # chunk(i,j,k), enc(k,j,i)
        t = t.contiguous().view(torch.uint8).view(-1, 4).flip(1)  # big endian
        return t.contiguous().view(-1)

    def after_decode(self):
        pass

    def check(self) -> bool:
        return bool(torch.equal(self.out.view(torch.int32), self.dec_ref.view(torch.int32)))

    def cpu_baseline(self):
        """Oracle (C restatement of zarrs' per-chunk pipeline) on host cores, bounded sample."""
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        K, threads, g = self.CHUNK, _threads(), self.args.cpu_grid
        shape = [x * K for x in g]
        n = g[0] * g[1] * g[2]
        rng = np.random.default_rng(7)
        dec = (rng.random(shape, dtype=np.float32) * 2 - 1)
        enc = np.ascontiguousarray(dec.reshape(g[0], K, g[1], K, g[2], K)
                                   .transpose(0, 2, 4, 5, 3, 1)).astype(">f4").reshape(n, -1)
        chain = O.OracleChain.from_metadata(self.CODECS, "float32", 0.0, 3)
        ptrs = (C.c_void_p * n)(*[enc[c].ctypes.data for c in range(n)])
        lens = (C.c_uint64 * n)(*([K ** 3 * 4] * n))
        out = np.empty(shape, np.float32)
        O.retrieve_ptrs(chain, shape, [K] * 3, ptrs, lens, [0, 0, 0], shape, out, threads)
        assert np.array_equal(out, dec)
        times = _time_reps(lambda: O.retrieve_ptrs(chain, shape, [K] * 3, ptrs, lens, [0, 0, 0], shape,
                                                   out, threads), self.args.cpu_seconds)
        t = float(np.median(times))
        return {"value": round(n * K ** 3 * 4 / t / 2 ** 30, 3), "unit": "GiB/s", "cores": threads,
                "kind": "port",
                "sample": f"{n} of the 4096 chunks ({shape[0]}x{shape[1]}x{shape[2]} f32 subset), median of "
                          f"{len(times)} reps, oracle retrieve_array_subset with {threads} threads"}

    def host_leg(self, sp):
        """PCIe-inclusive rates: encoded chunks in pinned host memory -> zgpu_decode_batch
        (H2D + decode) -> device array, and -> host array (+ D2H). Not the headline value."""
        from zarrs_amd import make_desc
        K, grid = self.CHUNK, self.args.grid
        h_enc = self.enc.cpu().pin_memory()
        base = h_enc.data_ptr()
        descs = []
        for c in range(self.n_chunks):
            i, r = divmod(c, grid[1] * grid[2])
            j, k = divmod(r, grid[2])
            descs.append(make_desc((base + c * self.chunk_bytes, self.chunk_bytes), [K] * 3,
                                   out_start=[i * K, j * K, k * K]))
        res = {}
        out = self.out
        self.chain.decode_batch(descs, out, self.shape, enc_device=False, stream=sp)  # warm-up
        torch.cuda.synchronize()
        reps = 3
        t0 = time.perf_counter()
        for _ in range(reps):
            self.chain.decode_batch(descs, out, self.shape, enc_device=False, stream=sp)
        torch.cuda.synchronize()
        t = (time.perf_counter() - t0) / reps
        res["host_enc_to_device_out_GiBps"] = round(self.decoded_bytes / t / 2 ** 30, 2)
        ok = self.check()
        h_out = torch.empty(self.shape, dtype=torch.float32).pin_memory()
        self.chain.decode_batch(descs, h_out, self.shape, enc_device=False, stream=sp)
        t0 = time.perf_counter()
        for _ in range(reps):
            self.chain.decode_batch(descs, h_out, self.shape, enc_device=False, stream=sp)
        t = (time.perf_counter() - t0) / reps
        res["host_enc_to_host_out_GiBps"] = round(self.decoded_bytes / t / 2 ** 30, 2)
        res["roundtrip_ok"] = ok and bool(torch.equal(h_out.view(torch.int32), self.dec_ref.cpu().view(torch.int32)))
        res.update(self.fs_leg(h_enc))
        res["encode"] = self.encode_leg(sp)
        return res

    def encode_leg(self, sp):
        """Write path: zgpu_encode_batch of the same 4096 chunks from the
        decoded device array into chunk buffers (transpose [2,1,0] + big endian), checked byte for
        byte against the bench's own encoding; the oracle's per-chunk encoder on the host beside it."""
        from concurrent.futures import ThreadPoolExecutor
        from zarrs_amd import _lib as L
        lib = L.load()
        K, grid = self.CHUNK, self.args.grid
        dst = torch.empty_like(self.enc)
        descs = (L.EncodeDesc * self.n_chunks)()
        for c in range(self.n_chunks):
            i, r = divmod(c, grid[1] * grid[2])
            j, k = divmod(r, grid[2])
            descs[c].dst = dst.data_ptr() + c * self.chunk_bytes
            descs[c].dst_cap = self.chunk_bytes
            descs[c].chunk_start[0], descs[c].chunk_start[1], descs[c].chunk_start[2] = i * K, j * K, k * K

        def run():
            L.check(lib.zgpu_encode_batch(self.chain._h, 3, L.u64s([K] * 3), self.dec_ref.data_ptr(),
                                          L.u64s(self.shape), descs, self.n_chunks, L.ENC_DEVICE | L.OUT_DEVICE, sp))
        run()
        ok = bool(torch.equal(dst, self.enc))
        reps = 10
        t0 = time.perf_counter()
        for _ in range(reps):
            run()
        t = (time.perf_counter() - t0) / reps
        res = {"gpu_GiBps": round(self.decoded_bytes / t / 2 ** 30, 1), "ms": round(t * 1e3, 3),
               "hbm_frac_incl_launch": round(2 * self.decoded_bytes / t / 1e9 / HBM_PEAK_GBS, 3),
               "bytes_equal_to_reference_encoding": ok}
        if self.args.no_cpu:
            return res
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        co = O.OracleChain.from_metadata(self.CODECS, "float32", 0.0, 3)
        host = self.dec_ref[:8 * K].cpu().numpy()  # 8 x 16 x 16 = 2048 chunk sample
        blocks = [np.ascontiguousarray(host[i * K:(i + 1) * K, j * K:(j + 1) * K, k * K:(k + 1) * K])
                  for i in range(8) for j in range(grid[1]) for k in range(grid[2])][:512]
        with ThreadPoolExecutor(_threads()) as ex:
            list(ex.map(co.encode, blocks))
            times = _time_reps(lambda: list(ex.map(co.encode, blocks)), 3.0)
        tc = float(np.median(times))
        res["cpu_oracle_GiBps"] = round(len(blocks) * self.chunk_bytes / tc / 2 ** 30, 2)
        res["cpu_cores"] = _threads()
        return res

    def fs_leg(self, h_enc):
        """Filesystem store -> device array: the 4096 chunks as files c/i/j/k
        of a FilesystemStore, read by zgpu_retrieve_array_subset_files (host-thread preads into
        pinned staging overlapped with H2D + decode). Buffered reads hit the page cache (the files
        were just written); direct_io reads the device (O_DIRECT, buffered where unsupported)."""
        import shutil
        import tempfile
        from zarrs_amd import Array, FilesystemStore
        K, grid = self.CHUNK, self.args.grid
        root = tempfile.mkdtemp(prefix="zgpu_fs_", dir=os.environ.get("TMPDIR", "/tmp"))
        res = {}
        try:
            raw = h_enc.numpy()
            st = FilesystemStore(root)
            for c in range(self.n_chunks):
                i, r = divmod(c, grid[1] * grid[2])
                j, k = divmod(r, grid[2])
                st[f"c/{i}/{j}/{k}"] = raw[c * self.chunk_bytes:(c + 1) * self.chunk_bytes].tobytes()
            meta = {"shape": self.shape, "data_type": "float32", "fill_value": 0.0, "codecs": self.CODECS,
                    "chunk_grid": {"name": "regular", "configuration": {"chunk_shape": [K] * 3}}}
            for name, direct in (("fs_enc_to_device_out_GiBps", False),
                                 ("fs_direct_enc_to_device_out_GiBps", True)):
                arr = Array(FilesystemStore(root, direct_io=direct), meta, self.args.ctx)
                self.out.zero_()
                arr.retrieve_array_subset_into([0, 0, 0], self.shape, self.out)  # warm-up
                torch.cuda.synchronize()
                ok = self.check()
                reps = 3
                t0 = time.perf_counter()
                for _ in range(reps):
                    arr.retrieve_array_subset_into([0, 0, 0], self.shape, self.out)
                torch.cuda.synchronize()
                t = (time.perf_counter() - t0) / reps
                res[name] = round(self.decoded_bytes / t / 2 ** 30, 2) if ok else "MISMATCH"
        finally:
            shutil.rmtree(root, ignore_errors=True)
        return res


# ------------------------------------------------------------------------------------------------
# C1 (BASELINE configs[0])
# ------------------------------------------------------------------------------------------------
class C1:
    """Round trip of one 256^3 f32 chunk through the bytes-only chain: a step is
    zgpu_encode_batch of the chunk from the device array into the device "store" buffer (the write
    half, CodecChain::encode, codec_chain.rs:528-555) followed by its decode into the output array
    (retrieve_chunk, array_read_ops_array.rs:265-310). On a little-endian host both halves are copies
    (bytes codec passthrough, zarrs_data_type/src/codec_traits/bytes.rs:111-112): HBM-bound plumbing.
    value = decoded bytes per step / step time."""
    CODECS = [{"name": "bytes", "configuration": {"endian": "little"}}]
    N = 256
    kernel = "k_scatter_rows"
    dtype = "f32"

    def __init__(self, args, rank, world, dev):
        from zarrs_amd import _lib as L
        from zarrs_amd import CodecChain, make_desc
        self.args, self.rank, self.world, self.dev = args, rank, world, dev
        n = self.N
        self.shape = [n, n, n]
        g = torch.Generator(device=dev)
        g.manual_seed(4321 + rank)
        self.dec_ref = torch.rand(self.shape, generator=g, device=dev, dtype=torch.float32) * 2 - 1
        self.chain = CodecChain.from_metadata(self.CODECS, "float32", 0.0, args.ctx)
        self.nbytes = n ** 3 * 4
        self.store = torch.empty(self.nbytes, dtype=torch.uint8, device=dev)  # the in-memory store
        self.edesc = (L.EncodeDesc * 1)()
        self.edesc[0].dst, self.edesc[0].dst_cap = self.store.data_ptr(), self.nbytes
        self.out = torch.empty(self.shape, dtype=torch.float32, device=dev)
        self.parts = [(self.chain, [make_desc((self.store.data_ptr(), self.nbytes), self.shape)], self.out,
                       self.shape)]
        self.decoded_bytes = self.nbytes
        self.step_bytes = self.nbytes * world
        self.extra_alg_bytes = 2 * self.nbytes  # the encode half: chunk read + encoded bytes written
        self.config = {"workload": "C1: round trip (encode + decode) of one 256^3 f32 chunk, [bytes{endian:little}], "
                                   "device-resident store", "chunk_shape": self.shape,
                       "parallelism": f"one chunk per GPU x{world}"}
        self.data = "synthetic (uniform [-1,1) f32 on device; decode(encode(x)) == x checked)"
        self.scaling = "weak"

    def pre_step(self, sp):
        from zarrs_amd import _lib as L
        L.check(L.load().zgpu_encode_batch(self.chain._h, 3, L.u64s(self.shape), self.dec_ref.data_ptr(),
                                           L.u64s(self.shape), self.edesc, 1, L.ENC_DEVICE | L.OUT_DEVICE, sp))

    def after_decode(self):
        pass

    def check(self) -> bool:
        return bool(torch.equal(self.out.view(torch.int32), self.dec_ref.view(torch.int32)))

    def cpu_baseline(self):
        """The oracle's encode + decode of the chunk (one chunk: zarrs runs it on one thread)."""
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        co = O.OracleChain.from_metadata(self.CODECS, "float32", 0.0, 3)
        a = self.dec_ref.cpu().numpy()

        def run():
            return co.decode(co.encode(a), self.shape)
        assert np.array_equal(run(), a)
        times = _time_reps(run, min(self.args.cpu_seconds, 5.0))
        t = float(np.median(times))
        return {"value": round(self.nbytes / t / 2 ** 30, 3), "unit": "GiB/s", "cores": 1, "kind": "port",
                "sample": f"the whole workload (one 256^3 f32 chunk encoded + decoded), median of {len(times)} reps, "
                          "oracle encode/decode on one thread"}

    def host_leg(self, sp):
        return None


# ------------------------------------------------------------------------------------------------
# C3 / C4
# ------------------------------------------------------------------------------------------------
class C3:
    SHARD, INNER = 256, 32
    ARRAY = [2048, 2048, 2048]
    SUB_START, SUB_SHAPE = [200, 300, 1000], [768, 768, 768]
    CODECS = [{"name": "sharding_indexed", "configuration": {
        "chunk_shape": [32, 32, 32],
        "codecs": [{"name": "bytes", "configuration": {"endian": "little"}},
                   {"name": "gzip", "configuration": {"level": 1}}, {"name": "crc32c"}],
        "index_codecs": [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}],
        "index_location": "end"}}]
    # the roofline covers the step (k_shard_index, k_item_resolve, k_crc32c_strip, k_order_by_len,
    # k_gzip ~96 %, k_scatter_rows); PMC counters summed over the step's dispatches
    kernel = "C3 decode step (k_gzip ~96 % + k_shard_index/k_item_resolve/k_crc32c_strip/k_scatter_rows)"
    pmc_regex = "zgpu::k_"
    dtype = "f32"

    def __init__(self, args, rank, world, dev):
        from zarrs_amd import CodecChain, make_desc
        self.args, self.rank, self.world, self.dev = args, rank, world, dev
        from zarrs_amd.distributed import chunk_line_partition, slab_partition
        S = self.SHARD
        er, ew = _emulated_rank(args, rank, world)
        if ew > 1:
            # C4: the subset's inner-chunk lines (axis-0 x axis-1 inner chunks) cut into stream-balanced runs
            # (chunk_line_partition: <= 3 boxes per rank, 1,950-1,975 inner chunks each at N = 8, inside the
            # pipelined gzip kernel's 2,048; axis-0 slabs cut through inner-chunk rows and gave a rank 2,500);
            # a rank decodes its boxes into its slab, the rows they span (array coordinates)
            self.boxes_by_rank = chunk_line_partition(self.SUB_START, self.SUB_SHAPE, [self.INNER] * 3, ew)
            self.slabs = [self._box_slab(b) for b in self.boxes_by_rank]
        else:
            self.slabs = slab_partition(self.SUB_START, self.SUB_SHAPE, ew)
            self.boxes_by_rank = [[sl] for sl in self.slabs]
        self.boxes = self.boxes_by_rank[er]
        self.start, self.shape = self.slabs[er]
        syn = _synth()
        self.chain = CodecChain.from_metadata(self.CODECS, "float32", 0.0, args.ctx)
        lo = [s // S for s in self.start]
        hi = [(s + n - 1) // S + 1 for s, n in zip(self.start, self.shape)]
        self.shards, self.descs, enc_total = {}, [], 0
        dec = np.empty([S] * 3, np.float32)
        nt = _threads()
        for si in range(lo[0], hi[0]):
            for sj in range(lo[1], hi[1]):
                for sk in range(lo[2], hi[2]):
                    org = [si * S, sj * S, sk * S]
                    syn.synth_c3_values(_u64(org), _u64([S] * 3), dec.ctypes.data, nt)
                    p, n = C.c_void_p(), C.c_uint64()
                    if syn.synth_gzip_crc_shard(dec.ctypes.data, 4, _u64([S] * 3), _u64([self.INNER] * 3), 1,
                                                nt, C.byref(p), C.byref(n)):
                        raise RuntimeError("shard encode failed")
                    host = np.ctypeslib.as_array((C.c_uint8 * n.value).from_address(p.value)).copy()
                    syn.synth_free(p)
                    t = torch.from_numpy(host).to(dev)
                    self.shards[(si, sj, sk)] = (t, host)
                    enc_total += n.value
        self.descs = self._box_descs(self.boxes, self.start)
        self.enc_total = enc_total
        n_sh = len(self.shards)
        self.ratio = n_sh * S ** 3 * 4 / enc_total
        exp = np.empty(self.shape, np.float32)
        syn.synth_c3_values(_u64(self.start), _u64(self.shape), exp.ctypes.data, nt)
        self.expected = torch.from_numpy(exp).to(dev)
        self.full = None
        self.gather_s = []
        if world > 1 and rank == 0:  # the root decodes its boxes in place inside the gathered subset
            self.full = torch.empty(self.SUB_SHAPE, dtype=torch.float32, device=dev)
            self.out = self.full.narrow(0, self.start[0] - self.SUB_START[0], self.shape[0])
            ef = np.empty(self.SUB_SHAPE, np.float32)  # the whole subset: the root checks every slab
            syn.synth_c3_values(_u64(self.SUB_START), _u64(self.SUB_SHAPE), ef.ctypes.data, nt)
            self.expected_full = torch.from_numpy(ef).to(dev)
            del ef
        else:
            self.out = torch.empty(self.shape, dtype=torch.float32, device=dev)
        self.out_shape = self.shape
        self.decoded_bytes = sum(int(np.prod(bs)) for _, bs in self.boxes) * 4  # per rank per step
        # one plan: at N > 1 the rank's boxes in one launch (C4), sent to the root once decoded
        self.parts = [(self.chain, self.descs, self.out, self.out_shape)]
        self.step_bytes = int(np.prod(self.SUB_SHAPE)) * 4  # the whole subset, all ranks
        if getattr(args, "emulate_rank", ""):
            self.step_bytes = self.decoded_bytes
        self.gathered = None
        self.config = {"workload": "C3" + ("/C4" if world > 1 else "") +
                                   ": sharded [2048]^3 f32, 256^3 shards / 32^3 inner chunks, "
                                   "[bytes, gzip 1, crc32c] + [bytes, crc32c] index at end, read subset "
                                   "[200:968, 300:1068, 1000:1768]",
                       "shards_touched_per_gpu": n_sh, "subset_shape": self.SUB_SHAPE,
                       "slab_per_gpu": self.shape, "gzip_ratio": round(self.ratio, 3),
                       "encoded_bytes_resident_per_gpu": enc_total,
                       "parallelism": ("axis-0 slabs x1" if world == 1 else
                                       f"stream-balanced inner-chunk lines x{world} (<= 3 boxes per rank), peers' "
                                       "boxes sent to rank 0 over RCCL in the step (whole-row boxes received in "
                                       "place)")}
        if world > 1:
            self.config["boxes_this_gpu"] = [[list(b0), list(bs)] for b0, bs in self.boxes]
        self.data = ("synthetic (round(256*(sin(.05x)+cos(.03y)+.5sin(.07z))+N(0,1))/256 f32, shards "
                     "written by tools/synth; decode(encode(x)) == x checked on device)")
        self.scaling = "strong"

    def _box_slab(self, boxes):
        """The slab (rows of the subset, whole on the other axes) that a rank's boxes span (empty: none)."""
        if not boxes:
            return list(self.SUB_START), [0] + list(self.SUB_SHAPE[1:])
        r0 = min(b0[0] for b0, _ in boxes)
        r1 = max(b0[0] + bs[0] for b0, bs in boxes)
        return [r0] + list(self.SUB_START[1:]), [r1 - r0] + list(self.SUB_SHAPE[1:])

    def _box_descs(self, boxes, origin):
        """Chunk descriptors of the shards' parts inside `boxes` (array coordinates), placed relative to
        `origin` (the output's first element)."""
        from zarrs_amd import make_desc
        S = self.SHARD
        pd = []
        for b0, bs in boxes:
            for (si, sj, sk), (t, _) in self.shards.items():
                org = [si * S, sj * S, sk * S]
                s0 = [max(a, o) for a, o in zip(b0, org)]
                s1 = [min(a + n, o + S) for a, n, o in zip(b0, bs, org)]
                if any(b <= a for a, b in zip(s0, s1)):
                    continue
                pd.append(make_desc((t.data_ptr(), int(t.numel())), [S] * 3,
                                    sel_start=[a - o for a, o in zip(s0, org)],
                                    sel_shape=[b - a for a, b in zip(s0, s1)],
                                    out_start=[a - o for a, o in zip(s0, origin)]))
        return pd

    def rank_share(self, n1_ms):
        """SURVEY §8(e) C4 at N = 8, predicted on this GPU: rank r's share of the subset (its stream-
        balanced inner-chunk lines, chunk_line_partition, as --gpus 8 cuts it) decoded alone as the N = 8
        step decodes it (its boxes in one plan into its slab, statuses read back), for every r; its boxes
        then travel to the root over one xGMI link, beside the other peers' on theirs (the exposed exchange:
        the largest rank share at one link's rate). The axis-0 slabs of rounds 5-6 are measured beside it
        (`alt`: 2,500 inner chunks per rank, the one-wave gzip kernel)."""
        from zarrs_amd.distributed import chunk_line_partition, slab_partition
        N = RANK_SHARE_N

        def measure(boxes_by_rank):
            rank_ms, biggest = [], 0
            for boxes in boxes_by_rank:
                start, shape = self._box_slab(boxes)
                buf = torch.empty(shape, dtype=torch.float32, device=self.dev)
                groups = [(self.chain, self._box_descs(boxes, start), buf, shape)]
                rank_ms.append(_time_plan_groups(self.args.ctx, groups, [[0]], set(), self.dev, status_each=True))
                biggest = max(biggest, sum(int(np.prod(bs)) for _, bs in boxes) * 4)
                del buf
            return rank_ms, biggest / (XGMI_LINK_GBS * 1e9) * 1e3

        gb = int(np.prod(self.SUB_SHAPE)) * 4 * (N - 1) // N
        rank_ms, gms = measure(chunk_line_partition(self.SUB_START, self.SUB_SHAPE, [self.INNER] * 3, N))
        rep = rank_share_report(rank_ms, n1_ms, self.step_bytes, gb, gms,
                                "each rank's stream-balanced inner-chunk lines (chunk_line_partition: <= 3 boxes, "
                                "1,950-1,975 inner chunks) decoded alone on this GPU in one plan, as the N = 8 step "
                                "does (5 reps, median); its boxes then go to the root over one xGMI link (at "
                                f"{XGMI_LINK_GBS:.0f} GB/s) beside the other peers'; the slowest rank sets the step")
        alt_ms, alt_g = measure([[sl] for sl in slab_partition(self.SUB_START, self.SUB_SHAPE, N)])
        rep["alt"] = {"partition": "axis-0 slabs (rounds 5-6)",
                      "max_rank_ms": round(max(alt_ms), 3), "gather_ms_model": round(alt_g, 3),
                      "predicted_speedup_vs_n1": round(n1_ms / (max(alt_ms) + alt_g), 3)}
        return rep

    def run_step(self, execute):
        """C4 (N > 1): decode this rank's boxes (one plan on the bench stream, statuses read back), then
        send them to the root (RCCL point-to-point; whole-row boxes land in place, the others packed
        into one message per peer: gather_regions). gather_s records the step's exchange: the time from
        this rank's decode to the completion of its sends (peers) or receives (root)."""
        from zarrs_amd.distributed import gather_regions
        execute(0)
        t0 = time.perf_counter()
        rel = [[([a - o for a, o in zip(b0, self.SUB_START)], bs) for b0, bs in boxes] for boxes in self.boxes_by_rank]
        self.gathered = gather_regions(self.out, rel, [0, 0, 0], self.SUB_SHAPE, dst=0, out=self.full,
                                       local_origin=[a - o for a, o in zip(self.start, self.SUB_START)])
        torch.cuda.synchronize()
        self.gather_s.append(time.perf_counter() - t0)

    def after_decode(self):
        pass

    def _box_views(self, t, origin, boxes):
        return [t[tuple(slice(a - o, a - o + n) for a, o, n in zip(b0, origin, bs))] for b0, bs in boxes]

    def check(self) -> bool:
        # this rank's boxes (its slab holds other ranks' boxes too, which it does not write)
        ok = all(bool(torch.equal(g.contiguous().view(torch.int32), e.contiguous().view(torch.int32)))
                 for g, e in zip(self._box_views(self.out, self.start, self.boxes),
                                 self._box_views(self.expected, self.start, self.boxes)))
        if self.gathered is not None:  # rank 0 holds the whole subset: every rank's boxes are checked
            bad = [r for r, boxes in enumerate(self.boxes_by_rank)
                   if not all(bool(torch.equal(g.contiguous().view(torch.int32), e.contiguous().view(torch.int32)))
                              for g, e in zip(self._box_views(self.gathered, self.SUB_START, boxes),
                                              self._box_views(self.expected_full, self.SUB_START, boxes)))]
            if bad:
                print(f"C4 check: boxes of ranks {bad} differ from the expected subset", file=sys.stderr)
            ok = ok and not bad
        return ok

    def gather_stats(self):
        """The xGMI gather inside the step (N > 1): median wall time of the grouped P2P receives /
        sends, and the bytes the root receives (every peer's boxes)."""
        if self.world == 1 or not self.gather_s:
            return None
        peer_bytes = sum(int(np.prod(bs)) * 4 for r, boxes in enumerate(self.boxes_by_rank) if r != 0
                         for _, bs in boxes)
        return {"ms": float(np.median(self.gather_s)) * 1e3, "bytes_to_root": peer_bytes}

    def cpu_baseline(self):
        """The oracle's retrieve_array_subset of this rank's whole slab (the full C3 subset at N=1, all
        64 shards): shards fan out over the host threads (16 threads -> 16 shards in flight, one thread
        each: zarrs' outer/inner split, concurrency.rs:23-48, with no thread spawned per shard)."""
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        threads = _threads()
        chain = O.OracleChain.from_metadata(self.CODECS, "float32", 0.0, 3)
        grid = [a // self.SHARD for a in self.ARRAY]
        ptrs = (C.c_void_p * int(np.prod(grid)))()
        lens = (C.c_uint64 * int(np.prod(grid)))()
        for (si, sj, sk), (_, host) in self.shards.items():
            lin = (si * grid[1] + sj) * grid[2] + sk
            ptrs[lin] = host.ctypes.data
            lens[lin] = host.nbytes
        out = np.empty(self.shape, np.float32)
        O.retrieve_ptrs(chain, self.ARRAY, [self.SHARD] * 3, ptrs, lens, self.start, self.shape, out, threads)
        assert np.array_equal(out, self.expected.cpu().numpy())
        times = _time_reps(lambda: O.retrieve_ptrs(chain, self.ARRAY, [self.SHARD] * 3, ptrs, lens,
                                                   self.start, self.shape, out, threads), self.args.cpu_seconds)
        t = float(np.median(times))
        return {"value": round(out.nbytes / t / 2 ** 30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
                "sample": f"the whole workload: subset {self.shape} at {self.start} ({len(self.shards)} shards), "
                          f"median of {len(times)} reps, oracle retrieve_array_subset (zlib inflate) with "
                          f"{threads} threads"}

    def host_leg(self, sp):
        return {"dropin_emulation": self.dropin_leg(), "encode": self.encode_leg()}

    def encode_leg(self):
        """Write path: CodecChain::encode of the 64 whole shards this subset touches
        (ShardingCodecBound::encode_bounded over [bytes, gzip 1, crc32c] inner chunks + the crc32c'd
        index, sharding_codec.rs:924-1085) from a device-resident array, on the GPU (k_gzip_encode,
        gzip_codec.rs:96-107): decoded GiB/s, the compressed size against the workload's own zlib-1
        shards, a round trip through the GPU decoder, and the oracle's encoder (zlib deflate level 1,
        one shard per host thread) on a 16-shard sample beside it."""
        from concurrent.futures import ThreadPoolExecutor
        from zarrs_amd import make_desc
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        S = self.SHARD
        keys = sorted(self.shards)
        lo = [min(k[d] for k in keys) for d in range(3)]
        shape = [(max(k[d] for k in keys) - lo[d] + 1) * S for d in range(3)]
        host = np.empty(shape, np.float32)
        _synth().synth_c3_values(_u64([l * S for l in lo]), _u64(shape), host.ctypes.data, _threads())
        x = torch.from_numpy(host).to(self.dev)
        starts = [[(k[d] - lo[d]) * S for d in range(3)] for k in keys]
        enc = self.chain.encode_chunks(x, [S] * 3, starts)  # warm-up (pools, scratch)
        torch.cuda.synchronize()

        def run():
            r = self.chain.encode_chunks(x, [S] * 3, starts)
            torch.cuda.synchronize()
            return r
        times = _time_reps(run, 3.0)
        enc = run()
        gpu_bytes = sum(int(e.numel()) for e in enc)
        zlib_bytes = sum(int(self.shards[k][1].nbytes) for k in keys)
        out = torch.empty_like(x)
        descs = [make_desc((e.data_ptr(), int(e.numel())), [S] * 3, out_start=st) for e, st in zip(enc, starts)]
        ok = self.chain.decode_batch(descs, out, shape, enc_device=True) == [0] * len(keys)
        ok = ok and bool(torch.equal(out.view(torch.int32), x.view(torch.int32)))
        del out
        t = float(np.median(times))
        nbytes = host.nbytes
        # CPU: the oracle's sharding encoder, 16 shards (one per thread)
        co = O.OracleChain.from_metadata(self.CODECS, "float32", 0.0, 3)
        sample = [np.ascontiguousarray(host[tuple(slice(a, a + S) for a in st)]) for st in starts[:16]]
        threads = _threads()
        with ThreadPoolExecutor(threads) as ex:
            tc = float(np.median(_time_reps(lambda: list(ex.map(co.encode, sample)), 5.0)))
        return {"GiBps": round(nbytes / t / 2 ** 30, 2), "ms": round(t * 1e3, 1), "shards": len(keys),
                "decoded_bytes": nbytes, "encoded_bytes": gpu_bytes,
                "size_vs_zlib1": round(gpu_bytes / zlib_bytes, 4), "roundtrip_ok": ok,
                "cpu_oracle_GiBps": round(sum(b.nbytes for b in sample) / tc / 2 ** 30, 3), "cpu_threads": threads,
                "note": "zgpu_encode_chunks of whole 256^3 shards from HBM (host-synchronous call incl. its result "
                        "read-back); size_vs_zlib1 = GPU shard bytes / zlib-1 shard bytes (tools/synth); CPU: "
                        "oracle encode (zlib deflate level 1 + crc32c + index), one shard per thread, 16 shards"}

    def dropin_leg(self):
        """The drop-in boundary's real call pattern (rust/zarrs_gpu with its sharding_indexed plugin
        under zarrs' unchanged read path, array_read_ops_common.rs:173-176): zarrs calls the codec once
        per shard from its rayon workers (here a pool of the host's threads), each call synchronous,
        host bytes in and host bytes out. A fully covered shard is one decode of the sharded chain (its
        index verified) into its window of the output array (ShardingCodecBound::decode_into,
        sharding_codec.rs:617-707); a partial shard reads its index (a suffix range), then decodes only
        the intersecting inner chunks through the inner chain, crc32c stripped, not verified (the
        plugin's GpuShardPartialDecoder) into its window. Each call's descriptor table is built before
        the timed passes (the plugin builds it in native code; Python would time its own loops), so a
        timed call is one zgpu_decode_into through ctypes, which releases the GIL. Measured two ways:
        the plugin's calls with ZGPU_COALESCE into their output windows (concurrent calls become one
        GPU batch, rows placed straight into the array), and isolated calls (no coalescing) into a
        per-call buffer copied into the array by the caller (round 3's pattern)."""
        from concurrent.futures import ThreadPoolExecutor
        from zarrs_amd import _lib as L
        from zarrs_amd import CodecChain, make_desc
        lib = L.load()
        torch.cuda.empty_cache()
        self.args.ctx.release_cached()
        S, I = self.SHARD, self.INNER
        inner = CodecChain.from_metadata(self.CODECS[0]["configuration"]["codecs"], "float32", 0.0, self.args.ctx)
        out = np.empty(self.shape, np.float32)
        cps = S // I
        n_idx = cps ** 3
        expected = self.expected.cpu().numpy()

        def prepare(item):
            (si, sj, sk), (_, host) = item
            org = [si * S, sj * S, sk * S]
            s0 = [max(a, o) for a, o in zip(self.start, org)]
            s1 = [min(a + b, o + S) for a, b, o in zip(self.start, self.shape, org)]
            sel = [b - a for a, b in zip(s0, s1)]
            w0 = [a - b for a, b in zip(s0, self.start)]
            if sel == [S] * 3:  # full shard: ShardingCodecBound::decode_into
                chain, descs, flags = self.chain, [make_desc((host.ctypes.data, host.nbytes), [S] * 3)], 0
            else:  # partial: index by a suffix range, then the intersecting inner chunks' byte ranges
                index = np.frombuffer(host[len(host) - (n_idx * 16 + 4):len(host) - 4].tobytes(),
                                      np.uint64).reshape(-1, 2)
                lo = [(a - o) // I for a, o in zip(s0, org)]
                hi = [(b - o - 1) // I + 1 for b, o in zip(s1, org)]
                descs = []
                for ci in range(lo[0], hi[0]):
                    for cj in range(lo[1], hi[1]):
                        for ck in range(lo[2], hi[2]):
                            off, ln = index[(ci * cps + cj) * cps + ck]
                            c0 = [org[0] + ci * I, org[1] + cj * I, org[2] + ck * I]
                            a0 = [max(a, c) for a, c in zip(s0, c0)]
                            a1 = [min(b, c + I) for b, c in zip(s1, c0)]
                            enc = None if off == 2 ** 64 - 1 else (host.ctypes.data + int(off), int(ln))
                            descs.append(make_desc(enc, [I] * 3, [a - c for a, c in zip(a0, c0)],
                                                   [b - a for a, b in zip(a0, a1)], [a - b for a, b in zip(a0, s0)]))
                chain, flags = inner, L.NO_VALIDATE
            arr = (L.ChunkDesc * len(descs))(*descs)
            view = L.OutView()
            view.base = out.ctypes.data
            for d in range(3):
                view.array_shape[d], view.start[d], view.shape[d] = self.shape[d], w0[d], sel[d]
            buf = np.empty(sel, np.float32)
            dst = tuple(slice(a, a + n) for a, n in zip(w0, sel))
            return chain, arr, len(descs), view, flags, (C.c_int32 * len(descs))(), buf, dst, sel, host

        calls = [prepare(it) for it in self.shards.items()]

        def coalesced(c):
            chain, arr, n, view, flags, st = c[:6]
            rc = lib.zgpu_decode_into(chain._h, 3, arr, n, C.byref(view), flags | L.COALESCE, st, None)
            if rc:
                raise L.ZgpuError(rc, L.last_error())

        def plugin(c):  # the Rust plugin's decode_into: zgpu_decode_pinned, one copy into the view, release
            chain, arr, n, _, flags, st, _, dst, sel, _ = c
            data, res_h = C.c_void_p(), C.c_void_p()
            rc = lib.zgpu_decode_pinned(chain._h, 3, arr, n, L.u64s(sel), flags | L.COALESCE, st, C.byref(data),
                                        C.byref(res_h))
            if rc:
                raise L.ZgpuError(rc, L.last_error())
            try:
                nb = int(np.prod(sel)) * 4
                out[dst] = np.ctypeslib.as_array((C.c_uint8 * nb).from_address(data.value)).view(np.float32).reshape(sel)
            finally:
                lib.zgpu_result_release(res_h)

        def isolated(c):
            chain, arr, n, _, flags, st, buf, dst, sel, _ = c
            rc = lib.zgpu_decode_batch(chain._h, 3, arr, n, buf.ctypes.data, L.u64s(sel), flags, st, None)
            if rc:
                raise L.ZgpuError(rc, L.last_error())
            out[dst] = buf

        res = {"threads": _threads(), "calls": len(calls)}
        sweep = [int(x) for x in str(getattr(self.args, "dropin_sweep", "") or "").split(",") if x]
        best = None
        with ThreadPoolExecutor(_threads()) as ex:
            def measure(fn, key):
                out.fill(0)
                list(ex.map(fn, calls))  # warm-up (pools, scratch)
                ok = bool(np.array_equal(out, expected))
                st0 = self.args.ctx.coalescing_stats()
                times = _time_reps(lambda: list(ex.map(fn, calls)), 4.0)
                st1 = self.args.ctx.coalescing_stats()
                t = float(np.median(times))
                nb = st1["batches"] - st0["batches"]
                return {"GiBps": round(out.nbytes / t / 2 ** 30, 2), "ms": round(t * 1e3, 1), "roundtrip_ok": ok,
                        "batches_per_pass": round(nb / len(times), 2),
                        "calls_per_batch": round((st1["calls"] - st0["calls"]) / max(1, nb), 2)}
            for mc in sweep:
                self.args.ctx.set_coalescing(window_us=200, max_calls=mc)
                r = measure(coalesced, mc)
                res.setdefault("sweep_max_calls", {})[str(mc)] = r
            self.args.ctx.set_coalescing(window_us=getattr(self.args, "dropin_window_us", 200),
                                         max_calls=self.args.dropin_calls)
            best = measure(coalesced, self.args.dropin_calls)
            res.update(best)
            res["max_calls_per_batch"] = self.args.dropin_calls
            plug = measure(plugin, self.args.dropin_calls)
            res["plugin_pattern_GiBps"], res["plugin_pattern_ms"] = plug["GiBps"], plug["ms"]
            res["plugin_pattern_roundtrip_ok"] = plug["roundtrip_ok"]
            iso = measure(isolated, None)
            res["uncoalesced_GiBps"], res["uncoalesced_ms"] = iso["GiBps"], iso["ms"]
            res["uncoalesced_roundtrip_ok"] = iso["roundtrip_ok"]
        # a rayon pool sized to a many-core host (zarrs' default: one worker per logical CPU) keeps
        # every shard's call in flight at once; the calls mostly wait on the GPU
        with ThreadPoolExecutor(len(calls)) as ex:
            self.args.ctx.set_coalescing(window_us=200, max_calls=16)
            wide = measure(coalesced, 16)
            res["threads_one_per_shard"] = {"threads": len(calls), "max_calls_per_batch": 16, **wide}
        res["note"] = ("one synchronous host-in/host-out call per shard from a thread pool (zarrs' rayon loop), "
                       "descriptor tables built before timing; GiBps: ZGPU_COALESCE + zgpu_decode_into the output window "
                       "(rows placed by the library: the C ABI's best case, what ArrayGpuExt-style callers holding the "
                       "raw array get); plugin_pattern_GiBps: the Rust plugin's decode_into (zarrs' view exposes only "
                       "copy_from_slice): ZGPU_COALESCE + zgpu_decode_pinned, one copy of the window into the array, "
                       "zgpu_result_release; uncoalesced_GiBps: isolated zgpu_decode_batch calls into a per-call buffer "
                       "copied into the output. Measured at the process's GPU_MAX_HW_QUEUES (hip_env)")
        return res

# ------------------------------------------------------------------------------------------------
# C5
# ------------------------------------------------------------------------------------------------
class C5:
    """OME-Zarr-style uint16 pyramid: five levels, each the 2x2x2 mean of the one
    above, chunk shapes per level as listed there, [bytes, numcodecs.shuffle{2}, zstd{3}] chunks.
    --c5-scale divides the L0 y/x extents (default 1: the full L0 [512,4096,4096], 16 GiB, 1488 chunks,
    ~1.5 min with data generation; 4: L0 [512,1024,1024], 93 chunks, for quick iterations); chunk
    shapes are unchanged. N GPUs: the chunks
    of all levels are LPT-partitioned by encoded size (strong scaling, no collective)."""
    L0 = [512, 4096, 4096]
    CHUNKS = [[32, 512, 512], [64, 256, 256], [64, 128, 128], [64, 64, 64], [32, 64, 64]]
    CODECS = [{"name": "bytes", "configuration": {"endian": "little"}},
              {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
              {"name": "zstd", "configuration": {"level": 3, "checksum": False}}]
    # a step is a kernel pipeline on 4 streams: the roofline covers the whole step (HIP events around
    # it; PMC counters summed over its dispatches). DESIGN.md §3 has the per-kernel split.
    kernel = "zstd decode step (k_zstd_scan/lits/blocks/plan/direct/exec_item + k_scatter_rows)"
    pmc_regex = "k_zstd|k_scatter"
    dtype = "u16"

    def __init__(self, args, rank, world, dev):
        from zarrs_amd import CodecChain, make_desc
        from zarrs_amd.distributed import lpt_partition
        self.args, self.rank, self.world, self.dev = args, rank, world, dev
        sc = args.c5_scale
        shape0 = [self.L0[0], self.L0[1] // sc, self.L0[2] // sc]
        self.chain = CodecChain.from_metadata(self.CODECS, "uint16", 0, args.ctx)
        cache = getattr(args, "c5_cache", "")
        if args.child and cache and os.path.exists(cache + ".json"):
            # a rocprofv3 PMC pass: the parent's encoded frames, no data generation and no check
            self._init_from_cache(cache, shape0, make_desc)
            return
        syn = _synth()
        syn.synth_c5_level0.argtypes = [C.c_uint64] * 3 + [C.c_int] + [C.c_void_p] * 5 + [C.c_uint64, C.c_void_p,
                                                                                         C.c_int]
        syn.synth_shuffle_zstd_chunks.argtypes = [C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p, C.c_uint64,
                                                  C.c_int, C.c_int, C.c_int, C.c_void_p, C.c_void_p]
        rng = np.random.default_rng(42)
        nb = 64
        cz = rng.uniform(0, shape0[0], nb).astype(np.float32)
        cy = rng.uniform(0, shape0[1], nb).astype(np.float32)
        cx = rng.uniform(0, shape0[2], nb).astype(np.float32)
        sg = rng.uniform(4, 40, nb).astype(np.float32)
        amp = rng.uniform(300, 4000, nb).astype(np.float32)
        lvl = np.empty(shape0, np.uint16)
        nt = _threads()
        syn.synth_c5_level0(*shape0, nb, cz.ctypes.data, cy.ctypes.data, cx.ctypes.data, sg.ctypes.data,
                            amp.ctypes.data, 42, lvl.ctypes.data, nt)
        levels = [lvl]
        for _ in range(4):  # 2x2x2 mean (rounded half up), the usual OME-Zarr downsampling
            a = levels[-1].astype(np.uint32)
            z, y, x = a.shape
            m = a.reshape(z // 2, 2, y // 2, 2, x // 2, 2).sum(axis=(1, 3, 5))
            levels.append(((m + 4) // 8).astype(np.uint16))
        # every chunk of every level, zero-padded to the full chunk shape (zarrs writes edge chunks whole)
        chunks = []  # (level, chunk index, decoded bytes)
        for li, (a, cs) in enumerate(zip(levels, self.CHUNKS)):
            grid = [-(-s // c) for s, c in zip(a.shape, cs)]
            for idx in np.ndindex(*grid):
                blk = np.zeros(cs, np.uint16)
                sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, cs, a.shape))
                src = a[sl]
                blk[tuple(slice(0, n) for n in src.shape)] = src
                chunks.append((li, idx, blk))
        n = len(chunks)
        flat = np.concatenate([b.reshape(-1).view(np.uint8) for _, _, b in chunks])
        offs = np.zeros(n, np.uint64)
        lens = np.array([b.nbytes for _, _, b in chunks], np.uint64)
        offs[1:] = np.cumsum(lens)[:-1]
        outs = (C.c_void_p * n)()
        olens = (C.c_uint64 * n)()
        if syn.synth_shuffle_zstd_chunks(flat.ctypes.data, 2, offs.ctypes.data, lens.ctypes.data, n, 3, 0, nt,
                                         outs, olens):
            raise RuntimeError("zstd encode failed")
        enc_sizes = [int(olens[i]) for i in range(n)]
        # host copies of every encoded chunk (the CPU baseline decodes them all)
        self.enc_host = [np.ctypeslib.as_array((C.c_uint8 * olens[i]).from_address(outs[i])).copy()
                         for i in range(n)]
        for i in range(n):
            syn.synth_free(C.c_void_p(outs[i]))
        self.levels_host = levels
        self.all_chunks = chunks
        self._setup(shape0, [list(a.shape) for a in levels], [(li, idx) for li, idx, _ in chunks], enc_sizes,
                    make_desc, levels)

    def _init_from_cache(self, path, shape0, make_desc):
        meta = json.load(open(path + ".json"))
        raw = np.fromfile(path + ".bin", dtype=np.uint8)
        sizes = meta["enc_sizes"]
        offs = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        self.enc_host = [raw[offs[i]:offs[i + 1]] for i in range(len(sizes))]
        self.levels_host, self.all_chunks = None, None
        self._setup(shape0, meta["level_shapes"], [(li, tuple(idx)) for li, idx in meta["chunks"]], sizes,
                    make_desc, None)

    def save_cache(self, path):
        """The encoded frames and chunk table, for the rocprofv3 PMC passes' children (bench.py --child
        --c5-cache): they profile the same frames without regenerating the pyramid."""
        with open(path + ".bin", "wb") as f:
            for e in self.enc_host:
                f.write(memoryview(e))
        json.dump({"level_shapes": self.level_shapes, "enc_sizes": self.enc_sizes,
                   "chunks": [[li, list(idx)] for li, idx in self.chunk_meta]}, open(path + ".json", "w"))

    def _setup(self, shape0, level_shapes, chunk_meta, enc_sizes, make_desc, levels):
        from zarrs_amd.distributed import lpt_partition
        dev, rank, world, sc = self.dev, self.rank, self.world, self.args.c5_scale
        n = len(chunk_meta)
        self.level_shapes, self.chunk_meta, self.enc_sizes = level_shapes, chunk_meta, enc_sizes
        er, ew = _emulated_rank(self.args, rank, world)
        mine = lpt_partition(enc_sizes, ew)[er]
        self.outs = [torch.zeros(s, dtype=torch.int16, device=dev) for s in level_shapes]
        self.expected = None if levels is None else [torch.from_numpy(a.view(np.int16)).to(dev) for a in levels]
        self.masks = [torch.zeros(s, dtype=torch.bool, device=dev) for s in level_shapes]
        per_level = [[] for _ in level_shapes]
        mine = set(mine)
        self.enc_bufs, enc_total, dec_total, all_bytes, raw_bytes = [], 0, 0, 0, 0
        for i, (li, idx) in enumerate(chunk_meta):
            cs, shp = self.CHUNKS[li], level_shapes[li]
            start = [k * c for k, c in zip(idx, cs)]
            sel = [min(c, s - st) for c, s, st in zip(cs, shp, start)]
            all_bytes += int(np.prod(sel)) * 2
            raw_bytes += int(np.prod(cs)) * 2
            if i not in mine:
                continue
            t = torch.from_numpy(self.enc_host[i]).to(dev)
            self.enc_bufs.append(t)
            enc_total += enc_sizes[i]
            dec_total += int(np.prod(sel)) * 2
            per_level[li].append(make_desc((t.data_ptr(), enc_sizes[i]), cs, [0, 0, 0], sel, start))
            self.masks[li][tuple(slice(st, st + n_) for st, n_ in zip(start, sel))] = True
        # plans (chunk batches) and the streams they run on: the largest level is split in two halves
        # on streams of their own (its entropy-decode kernels are throughput-bound, its per-chunk
        # sequence execution is not, so halving the batch shortens its chain), the next level on a
        # third stream, the small levels one after another on a fourth (HIP's default GPU_MAX_HW_QUEUES is 4)
        l0 = per_level[0]
        halves = lpt_partition([int(dsc.enc_len) for dsc in l0], 2)  # balanced by encoded size
        groups = [[l0[i] for i in hv] for hv in halves] + per_level[1:]
        outs_g = [self.outs[0], self.outs[0]] + self.outs[1:]
        self.parts, lane_of = [], []
        for gi, (d, o) in enumerate(zip(groups, outs_g)):
            if d:
                self.parts.append((self.chain, d, o, list(o.shape)))
                lane_of.append(min(gi, 3))
        self.lanes = [[p for p, l in enumerate(lane_of) if l == k] for k in range(4)]
        self.lanes = [ln for ln in self.lanes if ln]
        # the first L0 half and the small levels decode their literals first (ZGPU_ZSTD_LITS_FIRST)
        # while the second L0 half and L1 decode sequences, so throughput-bound literal work overlaps
        # latency-bound sequence decoding: C5 88.2-88.5 -> 83.2 ms (profiles/r05/r05lf_zstd_lits_first_ab.txt)
        self.lits_first_parts = [p for p, l in enumerate(lane_of) if l in (0, 3)]
        # the same levels as one library plan group (zgpu_group, the default; --bench-lanes: the lanes above)
        self.level_parts = [(self.chain, d, o, list(o.shape)) for d, o in zip(per_level, self.outs) if d]
        self.decoded_bytes = dec_total
        self.step_bytes = dec_total if getattr(self.args, "emulate_rank", "") else all_bytes
        self.ratio = raw_bytes / max(1, sum(enc_sizes))
        self.config = {"workload": f"C5: OME-Zarr-style u16 pyramid, 5 levels, L0 {shape0} (y/x scaled 1/{sc}), "
                                   "chunks [32,512,512] [64,256,256] [64,128,128] [64,64,64] [32,64,64], "
                                   "[bytes, numcodecs.shuffle{2}, zstd{3}]",
                       "chunks_total": n, "chunks_this_gpu": len(mine), "zstd_ratio": round(self.ratio, 3),
                       "encoded_bytes_this_gpu": enc_total,
                       "parallelism": f"LPT chunk partition x{world}"}
        self.data = ("synthetic (background 100 + 64 Gaussian blobs amplitude <= 4000 + sqrt(mean)*N(0,1) noise, "
                     "u16, seed 42; 2x2x2 mean pyramid; decode(encode(x)) == x checked on device)")
        self.scaling = "strong"
        # N > 1: one cross-GPU L0 subset gathered to rank 0 in every step: the middle
        # [64, H/2, W/2] box of L0, whose chunks the LPT partition spreads over the ranks
        self.gathered = None
        self.gather_s = []
        if world > 1:
            from zarrs_amd.distributed import chunk_boxes
            owner = {}
            for r, part in enumerate(lpt_partition(enc_sizes, world)):
                for i in part:
                    owner[i] = r
            lin0 = {idx: i for i, (li, idx) in enumerate(chunk_meta) if li == 0}
            self.g_start = [0, shape0[1] // 4, shape0[2] // 4]
            self.g_shape = [min(64, shape0[0]), shape0[1] // 2, shape0[2] // 2]
            self.g_boxes = [[] for _ in range(world)]
            for idx, b0, bs in chunk_boxes(shape0, self.CHUNKS[0], self.g_start, self.g_shape):
                self.g_boxes[owner[lin0[idx]]].append((b0, bs))
            self.config["gather"] = {"l0_subset_start": self.g_start, "l0_subset_shape": self.g_shape,
                                     "bytes": int(np.prod(self.g_shape)) * 2}

    def rank_share(self, n1_ms):
        """SURVEY §8(e) C5 at N = 8, predicted on this GPU: rank r's LPT share of the pyramid
        (lpt_partition over encoded sizes, as --gpus 8 assigns it) decoded alone with the N = 8 run's
        plan and lane layout (its L0 chunks in two halves, L1, the small levels; literals-first parts),
        for every r; the L0 subset gather priced at the root's 7 direct xGMI links."""
        from zarrs_amd import make_desc
        from zarrs_amd.distributed import lpt_partition
        N = RANK_SHARE_N
        parts = lpt_partition(self.enc_sizes, N)
        if len(self.enc_bufs) != len(self.chunk_meta):
            raise RuntimeError("rank share needs every chunk resident (N = 1)")
        rank_ms = []
        for r in range(N):
            per_level = [[] for _ in self.level_shapes]
            for i in sorted(parts[r]):
                li, idx = self.chunk_meta[i]
                cs, shp = self.CHUNKS[li], self.level_shapes[li]
                start = [k * c for k, c in zip(idx, cs)]
                sel = [min(c, s_ - st) for c, s_, st in zip(cs, shp, start)]
                per_level[li].append(make_desc((self.enc_bufs[i].data_ptr(), self.enc_sizes[i]), cs, [0, 0, 0],
                                               sel, start))
            if not getattr(self.args, "bench_lanes", False):  # the library plan group, as the step runs it
                rank_ms.append(_time_group([(self.chain, d, list(o.shape)) for d, o in zip(per_level, self.outs) if d],
                                           [o for d, o in zip(per_level, self.outs) if d], self.dev))
                continue
            l0 = per_level[0]
            halves = lpt_partition([int(d.enc_len) for d in l0], 2)
            groups_d = [[l0[i] for i in hv] for hv in halves] + per_level[1:]
            outs_g = [self.outs[0], self.outs[0]] + self.outs[1:]
            groups, lane_of = [], []
            for gi, (d, o) in enumerate(zip(groups_d, outs_g)):
                if d:
                    groups.append((self.chain, d, o, list(o.shape)))
                    lane_of.append(min(gi, 3))
            lanes = [[g for g, l in enumerate(lane_of) if l == k] for k in range(4)]
            lanes = [ln for ln in lanes if ln]
            lf = {g for g, l in enumerate(lane_of) if l in (0, 3)}
            rank_ms.append(_time_plan_groups(self.args.ctx, groups, lanes, lf, self.dev))
        s0 = self.level_shapes[0]
        g_shape = [min(64, s0[0]), s0[1] // 2, s0[2] // 2]
        gb = int(np.prod(g_shape)) * 2 * (N - 1) // N
        gms = gb / ((N - 1) * XGMI_LINK_GBS * 1e9) * 1e3
        return rank_share_report(rank_ms, n1_ms, self.step_bytes, gb, gms,
                                 "each rank's LPT chunk share decoded alone on this GPU (its levels as the N = 8 "
                                 "run decodes them: one library plan group, or --bench-lanes' lanes; 5 reps, "
                                 "median); the L0 subset gather (7/8 of it to rank 0) at "
                                 f"7 x {XGMI_LINK_GBS:.0f} GB/s; the slowest rank sets the step")

    def after_decode(self):
        if self.world > 1:
            from zarrs_amd.distributed import gather_regions
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            self.gathered = gather_regions(self.outs[0], self.g_boxes, self.g_start, self.g_shape)
            torch.cuda.synchronize()
            self.gather_s.append(time.perf_counter() - t0)

    def gather_stats(self):
        if self.world == 1 or not self.gather_s:
            return None
        peer_bytes = sum(int(np.prod(bs)) * 2 for r, boxes in enumerate(self.g_boxes) if r != 0 for _, bs in boxes)
        return {"ms": float(np.median(self.gather_s)) * 1e3, "bytes_to_root": peer_bytes}

    def check(self) -> bool:
        if self.expected is None:  # a PMC child on cached frames: the parent checked them
            return True
        ok = True
        if self.gathered is not None:
            sl = tuple(slice(a, a + n) for a, n in zip(self.g_start, self.g_shape))
            ok = bool(torch.equal(self.gathered, self.expected[0][sl]))
        for o, e, m in zip(self.outs, self.expected, self.masks):
            if bool(m.all()):
                ok = ok and bool(torch.equal(o, e))
            else:  # this rank's chunks only; per axis-0 slab (masked indexing of >2^31 elements fails)
                for z in range(o.shape[0]):
                    ok = ok and bool(torch.equal(o[z][m[z]], e[z][m[z]]))
        if not ok:  # diagnostics: the chunks that differ (stderr)
            for li, (o, e, cs) in enumerate(zip(self.outs, self.expected, self.CHUNKS)):
                grid = [-(-s_ // c) for s_, c in zip(o.shape, cs)]
                shown = 0
                for idx in np.ndindex(*grid):
                    sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(idx, cs))
                    if torch.equal(o[sl], e[sl]):
                        continue
                    d = (o[sl] != e[sl])
                    first = d.nonzero()[0].tolist()
                    print(f"C5 check: level {li} chunk {list(idx)}: {int(d.sum())} elements differ, first at {first}",
                          file=sys.stderr)
                    shown += 1
                    if shown >= 6:
                        break
        return ok

    def cpu_baseline(self):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        threads = _threads()
        chain = O.OracleChain.from_metadata(self.CODECS, "uint16", 0, 3)
        # sample: all levels' chunks through the oracle's retrieve (chunk-parallel, libzstd)
        tables = []
        for li, (a, cs) in enumerate(zip(self.levels_host, self.CHUNKS)):
            grid = [-(-s // c) for s, c in zip(a.shape, cs)]
            ptrs = (C.c_void_p * int(np.prod(grid)))()
            lens = (C.c_uint64 * int(np.prod(grid)))()
            tables.append((li, a.shape, cs, ptrs, lens))
        for i, (li, idx, blk) in enumerate(self.all_chunks):
            _, shp, cs, ptrs, lens = tables[li]
            grid = [-(-s // c) for s, c in zip(shp, cs)]
            lin = int(np.ravel_multi_index(idx, grid))
            ptrs[lin] = self.enc_host[i].ctypes.data
            lens[lin] = self.enc_host[i].nbytes
        outs_np = [np.empty(a.shape, np.uint16) for a in self.levels_host]

        def run():
            for (li, shp, cs, ptrs, lens), o in zip(tables, outs_np):
                O.retrieve_ptrs(chain, list(shp), cs, ptrs, lens, [0, 0, 0], list(shp), o, threads)
        run()
        assert all(np.array_equal(o, a) for o, a in zip(outs_np, self.levels_host))
        times = _time_reps(run, self.args.cpu_seconds)
        t = float(np.median(times))
        return {"value": round(self.step_bytes / t / 2 ** 30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
                "sample": f"the whole pyramid ({len(self.all_chunks)} chunks), median of {len(times)} reps, "
                          f"oracle retrieve_array_subset per level (libzstd) with {threads} threads"}

    def host_leg(self, sp):
        return {"encode": self.encode_leg(), "dropin_emulation": self.dropin_leg()}

    def dropin_leg(self):
        """zarrs' unchanged per-chunk read path with the per-codec GPU plugins (rust/zarrs_gpu
        register_codecs: the entropy stage on the GPU, zarrs' own CPU codecs around it). CodecChain::
        decode_into (codec_chain.rs:592-646) of a [bytes, numcodecs.shuffle{2}, zstd] chunk calls, per
        chunk, from a rayon worker: ZstdCodec::decode -> the plugin: one coalesced zgpu_decode_pinned of
        the host frame, copied into a new Vec; ShuffleCodec::decode (shuffle_codec.rs:109-129) on the
        CPU into a new Vec; BytesCodec (little endian: passthrough) decode_into the array's view
        (array_bytes_fixed_disjoint_view.rs:177-206). Emulated for every chunk of the pyramid from a
        pool of the host's threads (numpy copies release the GIL); value = the pyramid's decoded
        bytes / pass time, the same unit as the leg's cpu_baseline."""
        from concurrent.futures import ThreadPoolExecutor
        from zarrs_amd import _lib as L
        from zarrs_amd import CodecChain, make_desc
        lib = L.load()
        syn = _synth()
        zs_meta = self.CODECS[2]
        chain = CodecChain.from_metadata([self.CODECS[0], zs_meta], "uint8", 0, self.args.ctx)
        outs = [np.empty(s_, np.uint16) for s_ in self.level_shapes]
        calls = []
        for i, (li, idx) in enumerate(self.chunk_meta):
            cs = self.CHUNKS[li]
            nb = int(np.prod(cs)) * 2
            enc = self.enc_host[i]
            d = (L.ChunkDesc * 1)(make_desc((enc.ctypes.data, enc.nbytes), [nb]))
            start = [k * c for k, c in zip(idx, cs)]
            sel = [min(c, s_ - st) for c, s_, st in zip(cs, self.level_shapes[li], start)]
            dst = tuple(slice(a, a + n_) for a, n_ in zip(start, sel))
            calls.append((d, nb, cs, li, dst, tuple(slice(0, n_) for n_ in sel), enc))

        def one(c):
            d, nb, cs, li, dst, src_sel, _ = c
            st = (C.c_int32 * 1)()
            data, res_h = C.c_void_p(), C.c_void_p()
            rc = lib.zgpu_decode_pinned(chain._h, 1, d, 1, L.u64s([nb]), L.COALESCE, st, C.byref(data), C.byref(res_h))
            if rc:
                raise L.ZgpuError(rc, L.last_error())
            try:  # the plugin's decode returns an owned Vec: one copy out of the pinned result
                zs = np.ctypeslib.as_array((C.c_uint8 * nb).from_address(data.value)).copy()
            finally:
                lib.zgpu_result_release(res_h)
            # ShuffleCodec::decode (elementsize 2): dec[j*2 + i] = enc[i*count + j], into a new buffer
            # (zarrs' loop compiled natively: tools/synth synth_unshuffle; ctypes drops the GIL)
            dec = np.empty(nb, np.uint8)
            syn.synth_unshuffle(zs.ctypes.data, dec.ctypes.data, nb, 2)
            # BytesCodec decode_into the array's view (little endian: the bytes as they are)
            outs[li][dst] = dec.view(np.uint16).reshape(cs)[src_sel]

        threads = _threads()
        self.args.ctx.set_coalescing(window_us=200, max_calls=8)
        # the encode leg left torch's cache and the context's pools full: the per-call batches need room
        torch.cuda.empty_cache()
        self.args.ctx.release_cached()
        with ThreadPoolExecutor(threads) as ex:
            list(ex.map(one, calls))  # warm-up (pools, pinned buffers)
            ok = all(np.array_equal(o, a) for o, a in zip(outs, self.levels_host))
            st0 = self.args.ctx.coalescing_stats()
            times = _time_reps(lambda: list(ex.map(one, calls)), 4.0)
            st1 = self.args.ctx.coalescing_stats()
        t = float(np.median(times))
        nb_ = st1["batches"] - st0["batches"]
        # one call alone (the latency a lone rayon worker sees): an L0 chunk's frame from host memory,
        # decoded into pinned memory, median of 10 (the plugin's zgpu_decode_pinned, no copies after it)
        lone = []
        d0, nb0 = calls[0][0], calls[0][1]
        for _ in range(11):
            st = (C.c_int32 * 1)()
            data, res_h = C.c_void_p(), C.c_void_p()
            t0 = time.perf_counter()
            rc = lib.zgpu_decode_pinned(chain._h, 1, d0, 1, L.u64s([nb0]), L.COALESCE, st, C.byref(data),
                                        C.byref(res_h))
            lone.append(time.perf_counter() - t0)
            if rc:
                raise L.ZgpuError(rc, L.last_error())
            lib.zgpu_result_release(res_h)
        return {"GiBps": round(self.step_bytes / t / 2 ** 30, 2), "ms": round(t * 1e3, 1), "roundtrip_ok": ok,
                "lone_frame_call_ms": round(float(np.median(lone[1:])) * 1e3, 3), "lone_frame_bytes": nb0,
                "threads": threads, "calls": len(calls), "batches_per_pass": round(nb_ / len(times), 1),
                "calls_per_batch": round((st1["calls"] - st0["calls"]) / max(1, nb_), 2),
                "hip_env_GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default: 4)"),
                "note": "per-chunk CodecChain::decode_into with the per-codec GPU plugins (zstd on the GPU through "
                        "a coalesced zgpu_decode_pinned + one copy into a Vec; shuffle on the CPU by zarrs' loop "
                        "compiled in C (tools/synth synth_unshuffle), bytes as a numpy copy into the array), one call "
                        "per chunk from a thread pool; compare with the leg's cpu_baseline (the whole chain on the "
                        "CPU)"}

    def encode_leg(self):
        """Write path: CodecChain::encode of level 0's whole chunks ([32,512,512]
        u16; 1024 chunks, 16 GiB at full scale) from HBM on the GPU (numcodecs.shuffle + k_zstd_encode: ZstdCodec::encode,
        zstd_codec.rs:100-111): decoded GiB/s, the compressed size against the workload's libzstd
        level-3 chunks, a round trip through the GPU decoder, and the oracle's encoder (libzstd level 3)
        on 32 of those chunks, one per host thread, beside it."""
        from concurrent.futures import ThreadPoolExecutor
        from zarrs_amd import make_desc
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        cs = self.CHUNKS[0]
        x = self.expected[0]
        l0 = [(i, idx) for i, (li, idx, _) in enumerate(self.all_chunks) if li == 0]
        l0 = [(i, idx) for i, idx in l0
              if all((k + 1) * c <= s_ for k, c, s_ in zip(idx, cs, x.shape))]  # whole chunks only
        starts = [[k * c for k, c in zip(idx, cs)] for _, idx in l0]
        self.chain.encode_chunks(x, cs, starts)  # warm-up
        torch.cuda.synchronize()

        def run():
            r = self.chain.encode_chunks(x, cs, starts)
            torch.cuda.synchronize()
            return r
        times = _time_reps(run, 3.0)
        enc = run()
        gpu_bytes = sum(int(e.numel()) for e in enc)
        ref_bytes = sum(int(self.enc_host[i].nbytes) for i, _ in l0)
        out = torch.zeros_like(x)
        descs = [make_desc((e.data_ptr(), int(e.numel())), cs, out_start=st) for e, st in zip(enc, starts)]
        ok = self.chain.decode_batch(descs, out, list(x.shape), enc_device=True) == [0] * len(l0)
        for st in starts:
            sl = tuple(slice(a, a + c) for a, c in zip(st, cs))
            ok = ok and bool(torch.equal(out[sl], x[sl]))
        del out, enc
        t = float(np.median(times))
        nbytes = len(l0) * int(np.prod(cs)) * 2
        co = O.OracleChain.from_metadata(self.CODECS, "uint16", 0, 3)
        sample = [self.all_chunks[i][2] for i, _ in l0[:32]]
        threads = _threads()
        with ThreadPoolExecutor(threads) as ex:
            tc = float(np.median(_time_reps(lambda: list(ex.map(co.encode, sample)), 5.0)))
        return {"GiBps": round(nbytes / t / 2 ** 30, 2), "ms": round(t * 1e3, 1), "chunks": len(l0),
                "decoded_bytes": nbytes, "encoded_bytes": gpu_bytes,
                "size_vs_libzstd3": round(gpu_bytes / ref_bytes, 4), "roundtrip_ok": ok,
                "cpu_oracle_GiBps": round(sum(b.nbytes for b in sample) / tc / 2 ** 30, 3), "cpu_threads": threads,
                "note": "zgpu_encode_chunks of whole L0 chunks from HBM (host-synchronous call incl. its result "
                        "read-back); size_vs_libzstd3 = GPU bytes / libzstd level-3 bytes of the same chunks; "
                        "CPU: oracle encode (shuffle + libzstd level 3), one chunk per thread, 32 chunks"}


# ------------------------------------------------------------------------------------------------
# blosc
# ------------------------------------------------------------------------------------------------
class Blosc:
    """u16 microscopy-style volume [1024,2048,1024] (4 GiB), chunks [64,256,256] (512 chunks of 8 MiB), codecs
    [bytes, blosc{lz4, clevel 5, shuffle, typesize 2}] -- numcodecs' Blosc defaults, the most common
    compressor in existing OME-Zarr data. Chunks encoded on the host by c-blosc 1.21 (the oracle's
    library), decoded on the GPU from HBM; per-rank chunk partition, no collective."""
    SHAPE, CHUNK = [1024, 2048, 1024], [64, 256, 256]
    CNAME = "lz4"
    SHUFFLE = "shuffle"
    kernel = "blosc decode step (k_blosc_info/streams, stream decoders, k_blosc_finish, k_scatter_rows)"
    pmc_regex = "k_blosc|k_lz4|k_zstd|k_scatter"
    dtype = "u16"

    def codecs(self):
        return [{"name": "bytes", "configuration": {"endian": "little"}},
                {"name": "blosc", "configuration": {"cname": self.CNAME, "clevel": 5, "shuffle": self.SHUFFLE,
                                                    "typesize": 2, "blocksize": 0}}]

    def __init__(self, args, rank, world, dev):
        from concurrent.futures import ThreadPoolExecutor
        from zarrs_amd import CodecChain, make_desc
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        self.args, self.rank, self.world, self.dev = args, rank, world, dev
        shape, cs = self.SHAPE, self.CHUNK
        g = torch.Generator(device=dev)
        g.manual_seed(42 + rank)
        z, y, x = (torch.arange(n, device=dev, dtype=torch.float32) for n in shape)
        img = 100 + 900 * (torch.sin(z[:, None, None] * 0.05) * torch.cos(y[None, :, None] * 0.013)
                           * torch.sin(x[None, None, :] * 0.021)).abs()
        img = img + torch.randn(shape, generator=g, device=dev) * img.sqrt()
        self.dec_ref = img.clamp(0, 65535).to(torch.int32).to(torch.uint16)
        host = self.dec_ref.cpu().numpy()
        grid = [s_ // c for s_, c in zip(shape, cs)]
        idxs = list(np.ndindex(*grid))
        co = O.OracleChain.from_metadata(self.codecs(), "uint16", 0, 3)

        def enc(idx):
            sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(idx, cs))
            return co.encode(np.ascontiguousarray(host[sl]))
        with ThreadPoolExecutor(_threads()) as ex:
            self.enc_host = list(ex.map(enc, idxs))
        self.host = host
        self.idxs = idxs
        self.chain = CodecChain.from_metadata(self.codecs(), "uint16", 0, args.ctx)
        self.enc_bufs, descs = [], []
        for idx, e in zip(idxs, self.enc_host):
            t = torch.frombuffer(bytearray(e), dtype=torch.uint8).to(dev)
            self.enc_bufs.append(t)
            descs.append(make_desc((t.data_ptr(), len(e)), cs, out_start=[i * c for i, c in zip(idx, cs)]))
        self.out = torch.empty(shape, dtype=torch.uint16, device=dev)
        self.parts = [(self.chain, descs, self.out, shape)]
        self.decoded_bytes = int(np.prod(shape)) * 2
        self.step_bytes = self.decoded_bytes * world
        enc_total = sum(len(e) for e in self.enc_host)
        self.config = {"workload": f"blosc: u16 volume {shape} per GPU, chunks {cs}, [bytes, blosc{{{self.CNAME}, "
                                   f"clevel 5, {self.SHUFFLE}, typesize 2, blocksize auto}}]"
                                   + (" (numcodecs Blosc defaults)" if self.SHUFFLE == "shuffle" else ""),
                       "chunks_per_gpu": len(idxs), "blosc_ratio": round(self.decoded_bytes / enc_total, 3),
                       "parallelism": f"chunk-partitioned x{world}"}
        self.data = ("synthetic (100 + 900|sin z cos y sin x| + sqrt-scaled N(0,1) noise, u16, seed 42; "
                     "encoded by c-blosc 1.21; decode(encode(x)) == x checked on device)")
        self.scaling = "weak"

    def after_decode(self):
        pass

    def check(self) -> bool:
        return bool(torch.equal(self.out, self.dec_ref))

    def cpu_baseline(self):
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        threads = _threads()
        chain = O.OracleChain.from_metadata(self.codecs(), "uint16", 0, 3)
        grid = [s_ // c for s_, c in zip(self.SHAPE, self.CHUNK)]
        n = int(np.prod(grid))
        ptrs = (C.c_void_p * n)()
        lens = (C.c_uint64 * n)()
        bufs = [np.frombuffer(e, np.uint8) for e in self.enc_host]
        for idx, b in zip(self.idxs, bufs):
            lin = int(np.ravel_multi_index(idx, grid))
            ptrs[lin], lens[lin] = b.ctypes.data, b.nbytes
        out = np.empty(self.SHAPE, np.uint16)
        O.retrieve_ptrs(chain, self.SHAPE, self.CHUNK, ptrs, lens, [0, 0, 0], self.SHAPE, out, threads)
        assert np.array_equal(out, self.host)
        times = _time_reps(lambda: O.retrieve_ptrs(chain, self.SHAPE, self.CHUNK, ptrs, lens, [0, 0, 0],
                                                   self.SHAPE, out, threads), self.args.cpu_seconds)
        t = float(np.median(times))
        return {"value": round(out.nbytes / t / 2 ** 30, 3), "unit": "GiB/s", "cores": threads, "kind": "port",
                "sample": f"the whole volume ({n} chunks), median of {len(times)} reps, oracle "
                          f"retrieve_array_subset (c-blosc 1.21 blosc_decompress_ctx) with {threads} threads"}

    def host_leg(self, sp):
        if self.CNAME not in ("blosclz", "lz4", "lz4hc", "zlib", "zstd"):
            return None  # snappy streams are not written on the GPU
        return {"encode": self.encode_leg()}

    def encode_leg(self):
        """Write path: BloscCodec::encode (blosc_codec_via_blosc_src.rs:113-128)
        of every chunk from HBM on the GPU (blosc_enc.hip: shuffle + lz4 / zstd streams): decoded GiB/s,
        the size against c-blosc's encoding of the same chunks, a round trip through the GPU decoder,
        and the oracle's encoder (c-blosc 1.21, one chunk per host thread) on 64 chunks beside it."""
        from concurrent.futures import ThreadPoolExecutor
        from zarrs_amd import make_desc
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import oracle as O
        cs = self.CHUNK
        x = self.dec_ref.view(torch.int16)
        starts = [[i * c for i, c in zip(idx, cs)] for idx in self.idxs]
        self.chain.encode_chunks(x, cs, starts)  # warm-up
        torch.cuda.synchronize()

        def run():
            r = self.chain.encode_chunks(x, cs, starts)
            torch.cuda.synchronize()
            return r
        times = _time_reps(run, 3.0)
        enc = run()
        gpu_bytes = sum(int(e.numel()) for e in enc)
        ref_bytes = sum(len(e) for e in self.enc_host)
        out = torch.zeros_like(x)
        descs = [make_desc((e.data_ptr(), int(e.numel())), cs, out_start=st) for e, st in zip(enc, starts)]
        ok = self.chain.decode_batch(descs, out, list(x.shape), enc_device=True) == [0] * len(enc)
        ok = ok and bool(torch.equal(out, x))
        del out, enc
        t = float(np.median(times))
        co = O.OracleChain.from_metadata(self.codecs(), "uint16", 0, 3)
        sample = []
        for idx in self.idxs[:64]:
            sl = tuple(slice(i * c, (i + 1) * c) for i, c in zip(idx, cs))
            sample.append(np.ascontiguousarray(self.host[sl]))
        threads = _threads()
        with ThreadPoolExecutor(threads) as ex:
            tc = float(np.median(_time_reps(lambda: list(ex.map(co.encode, sample)), 5.0)))
        return {"GiBps": round(self.decoded_bytes / t / 2 ** 30, 2), "ms": round(t * 1e3, 1),
                "chunks": len(starts), "encoded_bytes": gpu_bytes, "size_vs_c_blosc": round(gpu_bytes / ref_bytes, 4),
                "roundtrip_ok": ok, "cpu_oracle_GiBps": round(sum(b.nbytes for b in sample) / tc / 2 ** 30, 3),
                "cpu_threads": threads,
                "note": "zgpu_encode_chunks of every chunk from HBM (host-synchronous call incl. its result "
                        "read-back); size_vs_c_blosc = GPU bytes / c-blosc 1.21 bytes of the same chunks "
                        "(same cname / clevel / shuffle); CPU: oracle encode (c-blosc), one chunk per thread"}


class BloscZstd(Blosc):
    """Same volume, blosc{zstd, clevel 5, shuffle}: zarr-python 3's BloscCodec default compressor."""
    CNAME = "zstd"


class BloscLZ(Blosc):
    """Same volume, blosc{blosclz, clevel 5, shuffle}: c-blosc's default compressor, the one zarrs'
    own blosc benchmark uses (zarrs/benches/codecs.rs:52)."""
    CNAME = "blosclz"


class BloscZlib(Blosc):
    """Same volume, blosc{zlib, clevel 5, shuffle}: DEFLATE streams (k_gzip's decoder in its RFC 1950
    mode + k_adler32_check; the encoder's zlib mode)."""
    CNAME = "zlib"


class BloscBit(Blosc):
    """Same volume, blosc{lz4, clevel 5, bitshuffle}: the bit-transposed layout (zarrs' BloscCodec
    default shuffle when a typesize is set; k_blosc_finish's bit-transpose path)."""
    SHUFFLE = "bitshuffle"


WORKLOADS = {"c1": C1, "c2": C2, "c3": C3, "c5": C5, "blosc": Blosc, "blosc-zstd": BloscZstd,
             "blosc-blosclz": BloscLZ, "blosc-zlib": BloscZlib,
             "blosc-bitshuffle": BloscBit}


def _time_reps(fn, seconds):
    times = []
    t_end = time.perf_counter() + seconds
    while len(times) < 5 or (time.perf_counter() < t_end and len(times) < 50):
        t0 = time.perf_counter()
        fn()
        times.append(time.perf_counter() - t0)
    return times


RANK_SHARE_N = 8


def _time_plan_groups(ctx, groups, lanes, lits_first, dev, reps=5, status_each=False):
    """Median wall ms of one decode of `groups` ((chain, descs, out tensor, out_shape) per plan) laid out
    as a step is: `lanes` lists of group indices, each lane's plans in order on a stream of its own, the
    lanes concurrent (ZGPU_ONE_STREAM; ZGPU_ZSTD_LITS_FIRST for the groups in `lits_first`). Statuses
    are read back once after the timing and must be 0 (status_each: every plan's statuses read back
    after it, as C4's piece-wise decode does)."""
    from zarrs_amd import _lib as L
    lib = L.load()
    plans = []
    multi = len(lanes) > 1
    for gi, (chain, descs, out, out_shape) in enumerate(groups):
        n = len(descs)
        arr = (L.ChunkDesc * n)(*descs)
        plan = C.c_void_p()
        flags = L.ENC_DEVICE | L.OUT_DEVICE | (L.ONE_STREAM if multi else 0) | \
            (L.ZSTD_LITS_FIRST if multi and gi in lits_first else 0)
        L.check(lib.zgpu_plan_create(chain._h, len(out_shape), arr, n, L.u64s(out_shape), flags, C.byref(plan)))
        plans.append((plan, out, (C.c_int32 * n)()))
    streams = [torch.cuda.Stream(dev) for _ in lanes]
    sps = [C.c_void_p(st.cuda_stream) for st in streams]

    def once():
        main = torch.cuda.current_stream(dev)
        ev = torch.cuda.Event()
        ev.record(main)
        for li, ln in enumerate(lanes):
            streams[li].wait_event(ev)
            for gi in ln:
                plan, out, st = plans[gi]
                rc = lib.zgpu_plan_execute(plan, out.data_ptr(), st if status_each else None, sps[li])
                if rc:
                    raise RuntimeError(f"decode failed: {L.STATUS_NAMES[rc]} {L.last_error()}")
        for st in streams:
            done = torch.cuda.Event()
            done.record(st)
            main.wait_event(done)
        torch.cuda.synchronize(dev)
    try:
        once()
        once()
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            once()
            ts.append(time.perf_counter() - t0)
        for li, ln in enumerate(lanes):
            for gi in ln:
                plan, _, st = plans[gi]
                rc = lib.zgpu_plan_status(plan, st, sps[li])
                if rc or any(st[k] for k in range(len(st))):
                    raise RuntimeError(f"rank share decode failed: {L.STATUS_NAMES[rc]}")
        return float(np.median(ts)) * 1e3
    finally:
        for plan, _, _ in plans:
            lib.zgpu_plan_destroy(plan)


def _time_group(parts, outs, dev, reps=5):
    """Median wall ms of one decode of `parts` ((chain, descs, out_shape) per part) as ONE library plan
    group (zgpu_group) into `outs`; statuses read back after the timing must be 0."""
    from zarrs_amd import PlanGroup
    g = PlanGroup(parts)
    try:
        main = torch.cuda.current_stream(dev)
        for _ in range(2):
            g.execute(outs, stream=main.cuda_stream, wait=True)
        ts = []
        for _ in range(reps):
            t0 = time.perf_counter()
            g.execute(outs, stream=main.cuda_stream, wait=False)
            torch.cuda.synchronize(dev)
            ts.append(time.perf_counter() - t0)
        if any(g.wait()):
            raise RuntimeError("rank share decode failed")
        return float(np.median(ts)) * 1e3
    finally:
        g.close()


def rank_share_report(rank_ms, n1_ms, step_bytes, gather_bytes, gather_ms, note):
    """The N = RANK_SHARE_N prediction from one GPU: each rank's share of the step decoded alone (the
    same kernels, plans and lane layout as that rank runs), the exchange priced at the root's direct xGMI
    links, aggregate = the step's bytes over the slowest rank's time."""
    worst = max(rank_ms)
    t = worst + gather_ms
    return {"ranks": RANK_SHARE_N, "rank_ms": [round(x, 3) for x in rank_ms], "max_rank_ms": round(worst, 3),
            "rank_of_max": int(np.argmax(rank_ms)), "gather_bytes_to_root": gather_bytes,
            "gather_ms_model": round(gather_ms, 3), "n1_ms": round(n1_ms, 3),
            "predicted_step_ms": round(t, 3), "predicted_speedup_vs_n1": round(n1_ms / t, 3),
            "predicted_value_GiBps": round(step_bytes / (t * 1e-3) / 2 ** 30, 2),
            "status": "predicted, unmeasured on 8 GPUs", "note": note}


# ------------------------------------------------------------------------------------------------
def world_info(world, dev):
    """The process world this line was measured in: backend, size and every rank's device (gathered
    over the process group at N > 1)."""
    p = torch.cuda.get_device_properties(dev)
    me = f"{p.name} (cuda:{dev.index}, pci {p.pci_domain_id:04x}:{p.pci_bus_id:02x}:{p.pci_device_id:02x})"
    if world == 1:
        return {"backend": None, "world_size": 1, "devices": [me]}
    devs = [None] * world
    torch.distributed.all_gather_object(devs, me)
    return {"backend": torch.distributed.get_backend(), "world_size": world, "devices": devs}


def run_gpu(args, rank, world, dev):
    from zarrs_amd import Context
    from zarrs_amd import _lib as L
    args.ctx = Context(dev.index)
    W = WORKLOADS[args.workload](args, rank, world, dev)
    lib = L.load()
    plans = []  # one prepared plan per part (e.g. per pyramid level: one chunk shape per plan)
    part_plan = {}
    lits_first = set(getattr(W, "lits_first_parts", []))
    if args.lits_first is not None:
        lits_first = {int(x) for x in args.lits_first.split(",") if x.strip()}
    # independent parts (pyramid levels) as ONE library plan group (zgpu_group: the library lays them out
    # on streams of its own); --bench-lanes (and the profiling / A/B options) keep the bench-side lanes
    group = None
    if getattr(W, "level_parts", None) and not (args.bench_lanes or args.serial_lanes or args.fork or
                                                args.lits_first is not None or args.lane_priorities):
        from zarrs_amd import PlanGroup
        group = PlanGroup([(c, d, shp) for c, d, _, shp in W.level_parts])
        group_outs = [o for _, _, o, _ in W.level_parts]
        W.config["plan_layout"] = {"kind": "library plan group (zgpu_group)",
                                   "plans_lane_part_litsfirst": group.layout()}
    for pi, (chain, descs, out, out_shape) in enumerate([] if group else W.parts):
        n = len(descs)
        if not n:
            continue
        arr = (L.ChunkDesc * n)(*descs)
        plan = C.c_void_p()
        # plans run concurrently on lanes of their own stay on their lane's stream (ZGPU_ONE_STREAM)
        one = L.ONE_STREAM if len(getattr(W, "lanes", [[0]])) > 1 and not args.serial_lanes and not args.fork else 0
        # zstd plans that decode their literals before their sequences (ZGPU_ZSTD_LITS_FIRST)
        lf = L.ZSTD_LITS_FIRST if one and pi in lits_first else 0
        L.check(lib.zgpu_plan_create(chain._h, len(out_shape), arr, n, L.u64s(out_shape),
                                     L.ENC_DEVICE | L.OUT_DEVICE | one | lf, C.byref(plan)))
        part_plan[pi] = len(plans)
        plans.append((plan, out, (C.c_int32 * n)()))
    # stream lanes: lists of plans executed in order on one stream; lanes run concurrently
    lanes = getattr(W, "lanes", [[i] for i in range(len(W.parts))])
    if args.serial_lanes:  # profiling: every plan on one stream, so kernel durations do not overlap
        lanes = [[i for ln in lanes for i in ln]]
    lanes = [[part_plan[i] for i in ln if i in part_plan] for ln in lanes]
    lanes = [ln for ln in lanes if ln]
    # the library launches on this stream; events are recorded on it. Independent parts (pyramid
    # levels) run concurrently, one stream each: part 0 (the largest level, the longest serial chain)
    # on `stream` at high priority, so its kernels take CUs first
    prio = W.lane_priorities if hasattr(W, "lane_priorities") else [-1, -1] + [0] * max(0, len(lanes) - 2)
    if args.lane_priorities:
        prio = [int(x) for x in args.lane_priorities.split(",")]
    prio = (prio + [0] * len(lanes))[:len(lanes)]
    stream = torch.cuda.Stream(dev, priority=prio[0]) if len(lanes) > 1 else torch.cuda.Stream(dev)
    sp = C.c_void_p(stream.cuda_stream)
    side = [torch.cuda.Stream(dev, priority=prio[li]) for li in range(1, len(lanes))]
    lane_sp = [sp] + [C.c_void_p(st.cuda_stream) for st in side]
    plan_sp = {pi: lane_sp[li] for li, ln in enumerate(lanes) for pi in ln}

    def enqueue_all():
        if group:
            group.execute(group_outs, stream=sp.value, wait=False)
            return
        start = torch.cuda.Event()
        start.record(stream)
        for st in side:
            st.wait_event(start)
        for li, ln in enumerate(lanes):
            for pi in ln:
                plan, out, _ = plans[pi]
                rc = lib.zgpu_plan_execute(plan, out.data_ptr(), None, lane_sp[li])
                if rc:
                    raise RuntimeError(f"decode failed: {L.STATUS_NAMES[rc]} {L.last_error()}")
        for st in side:
            done = torch.cuda.Event()
            done.record(st)
            stream.wait_event(done)

    pre = getattr(W, "pre_step", None)

    def execute_part(pi):
        plan, out, status = plans[part_plan[pi]]
        rc = lib.zgpu_plan_execute(plan, out.data_ptr(), status, sp)
        if rc:
            raise RuntimeError(f"decode failed: {L.STATUS_NAMES[rc]} {L.last_error()}")

    def step():
        if pre:
            pre(sp)
        if hasattr(W, "run_step") and world > 1:  # the workload drives its plans (C4: overlapped gather)
            with torch.cuda.stream(stream):
                W.run_step(execute_part)
            W.after_decode()
            return
        if group:
            enqueue_all()
            group.wait()
            rc = 0
        elif len(plans) == 1:
            plan, out, status = plans[0]
            rc = lib.zgpu_plan_execute(plan, out.data_ptr(), status, sp)
        else:
            enqueue_all()
            rc = 0
            for pi, (plan, _, status) in enumerate(plans):
                rc = rc or lib.zgpu_plan_status(plan, status, plan_sp[pi])
        if rc:
            raise RuntimeError(f"decode failed: {L.STATUS_NAMES[rc]} {L.last_error()}")
        W.after_decode()

    if args.lane_times and len(lanes) > 1:  # diagnostics: each lane alone (stderr)
        for li, ln in enumerate(lanes):
            for _ in range(2):
                t0 = time.perf_counter()
                for pi in ln:
                    plan, out, status = plans[pi]
                    lib.zgpu_plan_execute(plan, out.data_ptr(), status, sp)
                dt = time.perf_counter() - t0
            print(f"lane {li} (plans {ln}) alone: {dt * 1e3:.2f} ms", file=sys.stderr)
    torch.cuda.synchronize()
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    ok = W.check()  # decode(encode(x)) == x, bit for bit, at full size
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
        for plan, _, _ in plans:
            lib.zgpu_plan_destroy(plan)
        if group:
            group.close()
        return None
    # Device time of one decode launch sequence, HIP events on the stream the library launches on;
    # enqueue-only executes (status=NULL), back to back.
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)
    ev0.record(stream)
    for _ in range(args.steps):
        if pre:
            pre(sp)
        enqueue_all()
    ev1.record(stream)
    torch.cuda.synchronize()
    ev_ms = ev0.elapsed_time(ev1) / args.steps
    alg_bytes = sum(lib.zgpu_plan_algorithmic_bytes(plan) for plan, _, _ in plans) + getattr(W, "extra_alg_bytes", 0)
    alg_bytes += group.algorithmic_bytes() if group else 0
    counters = group.counters() if group else [0] * L.N_COUNTERS
    for plan, _, _ in plans:  # device counters of each plan's last execute (statuses read in step())
        buf = (C.c_uint64 * L.N_COUNTERS)()
        lib.zgpu_plan_counters(plan, buf, L.N_COUNTERS)
        counters = [a + b for a, b in zip(counters, buf)]
    # host planning + upload included (zgpu_decode_batch form), for DESIGN.md
    t1 = time.perf_counter()
    reps = max(1, min(5, args.steps))
    for _ in range(reps):
        for chain, descs, out, out_shape in W.parts:
            if descs:
                chain.decode_batch(descs, out, out_shape, enc_device=True, stream=sp)
    torch.cuda.synchronize()
    batch_ms = (time.perf_counter() - t1) / reps * 1e3
    for plan, _, _ in plans:
        lib.zgpu_plan_destroy(plan)
    if group:
        group.close()
    host = W.host_leg(sp) if (args.host_leg and rank == 0) else None
    gather = W.gather_stats() if hasattr(W, "gather_stats") else None
    return dict(W=W, elapsed=elapsed, ev_ms=ev_ms, alg_bytes=alg_bytes, ok=ok, batch_ms=batch_ms, host=host,
                counters=counters, world_info=world_info(world, dev), gather=gather)


XGMI_LINK_GBS = 153.0  # one MI355X xGMI link, per direction (/opt/skills/guides/MI355X_MICROARCH.md)


def gather_report(r, world, dev):
    """The gather to rank 0, reported apart from the decode: the max over ranks of
    each rank's median gather time, the bytes rank 0 receives, and their rate against the direct
    links into the root (one per peer, at most 7, 153 GB/s each)."""
    if world == 1 or r.get("gather") is None:
        return None
    ms = torch.tensor([r["gather"]["ms"]], dtype=torch.float64, device=dev)
    torch.distributed.all_reduce(ms, op=torch.distributed.ReduceOp.MAX)
    t = float(ms.item())
    nbytes = r["gather"]["bytes_to_root"]
    peak = min(world - 1, 7) * XGMI_LINK_GBS
    gbs = nbytes / (t * 1e-3) / 1e9 if t > 0 else 0.0
    return {"gather_ms": round(t, 3), "bytes_to_root": nbytes, "xgmi_GBps": round(gbs, 1), "peak_GBps": peak,
            "frac": round(gbs / peak, 4), "included_in_step": True,
            "note": "P2P receives straight into the root's output (RCCL over xGMI) inside the step; C3/C4: the "
                    "slab is decoded in pieces of whole inner-chunk rows and each piece is sent while the next "
                    "decodes, so gather_ms is only the exchange left after a rank's last piece (exposed time)"}


def secondary_legs(args, rank, world, dev, r_primary):
    """The other §8(d) configs measured in the same run as the headline (C2): C3 (C4 at N > 1: the
    subset's axis-0 slabs gathered to rank 0 over RCCL inside the step) and C5 at --secondary-c5-scale
    (default 1: the full L0 [512,4096,4096]; LPT chunk partition, plus the cross-GPU L0 subset gather
    at N > 1). Each leg: value, ms/step, the roofline frac of its step (HIP events, algorithmic bytes),
    decode(encode(x)) == x on device, and (rank 0, N = 1) a short CPU baseline of the oracle, the
    step's HBM traffic from two rocprofv3 PMC passes (C5's child profiles the parent's cached frames)
    and, for C3, the drop-in boundary's per-shard call pattern (dropin_emulation)."""
    import copy
    import gc
    out = {}
    r_primary["W"] = None
    for name in [w for w in args.secondary.split(",") if w]:
        if name not in WORKLOADS:
            out[name] = {"error": "unknown workload"}
            continue
        t_leg = time.perf_counter()
        a = copy.copy(args)
        a.workload, a.steps, a.warmup = name, max(2, min(args.steps, 5)), 1
        a.host_leg, a.cpu_seconds, a.c5_scale = False, 5.0, args.secondary_c5_scale
        a.lane_priorities, a.serial_lanes, a.lane_times, a.fork = "", False, False, False
        a.lits_first = None
        a.bench_lanes = args.bench_lanes
        gc.collect()
        torch.cuda.empty_cache()
        args.ctx.release_cached()  # the previous leg's pooled device / pinned blocks back to the driver
        print(f"[bench] secondary leg {name} ...", file=sys.stderr, flush=True)
        try:
            r = run_gpu(a, rank, world, dev)
        except Exception as e:  # noqa: BLE001 - a secondary leg never voids the headline line
            out[name] = {"error": repr(e)[:300]}
            continue
        W = r["W"]
        el = torch.tensor([r["elapsed"]], dtype=torch.float64, device=dev)
        okt = torch.tensor([1 if r["ok"] else 0], dtype=torch.int32, device=dev)
        if world > 1:
            torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
            torch.distributed.all_reduce(okt, op=torch.distributed.ReduceOp.MIN)
        t = float(el.item())
        achieved = r["alg_bytes"] / (r["ev_ms"] * 1e-3) / 1e9
        leg = {"metric": METRIC, "value": round(W.step_bytes * a.steps / t / 2 ** 30, 2), "unit": "GiB/s",
               "n_gpus": world, "steps": a.steps, "warmup": a.warmup,
               "ms_per_step": round(t / a.steps * 1e3, 3), "scaling": W.scaling, "dtype": W.dtype,
               "config": W.config,
               "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                            "frac": round(achieved / HBM_PEAK_GBS, 4), "kernel": W.kernel,
                            "alg_bytes_per_launch": r["alg_bytes"],
                            "avg_launch_ms_hip_events": round(r["ev_ms"], 4),
                            "traffic": None, "traffic_detail": "skipped (--no-pmc or N>1)"},
               "roundtrip_ok": bool(okt.item())}
        if r["counters"][L_CTR_ZSTD_SERIAL] or r["counters"][L_CTR_ZSTD_PARALLEL]:
            leg["zstd_items_per_step"] = {"block_parallel": r["counters"][L_CTR_ZSTD_PARALLEL],
                                          "serial_fallback": r["counters"][L_CTR_ZSTD_SERIAL]}
        g = gather_report(r, world, dev)
        if g:
            leg["gather"] = g
        if rank == 0 and world == 1 and not args.no_cpu:
            try:
                leg["cpu_baseline"] = W.cpu_baseline()
            except Exception as e:  # noqa: BLE001
                leg["cpu_baseline"] = {"error": repr(e)[:300]}
        if name in ("c3", "c5") and rank == 0 and world == 1 and args.host_leg:
            try:  # the drop-in boundary's own rate (zarrs' per-shard / per-chunk calls from a thread pool)
                leg["dropin_emulation"] = W.dropin_leg()
            except Exception as e:  # noqa: BLE001
                leg["dropin_emulation"] = {"error": repr(e)[:300]}
        if name in ("c3", "c5") and rank == 0 and world == 1 and args.rank_share:
            try:  # one rank's share at N = 8 on this GPU (C4: the slabs; C5: the LPT parts)
                leg["c4_rank_share" if name == "c3" else "c5_rank_share"] = W.rank_share(t / a.steps * 1e3)
            except Exception as e:  # noqa: BLE001
                leg["rank_share"] = {"error": repr(e)[:300]}
        pmc = rank == 0 and world == 1 and not args.no_pmc
        cache = None
        if pmc and hasattr(W, "save_cache"):
            import tempfile
            cache = os.path.join(tempfile.mkdtemp(prefix="zgpu_c5_", dir=os.environ.get("TMPDIR", "/tmp")), "frames")
            W.save_cache(cache)
        import types
        meta = types.SimpleNamespace(**{k: getattr(W, k) for k in ("kernel", "pmc_regex") if hasattr(W, k)})
        r["W"] = W = None
        a.ctx.close()
        gc.collect()
        torch.cuda.empty_cache()
        if pmc:  # HBM traffic of the leg's step: two rocprofv3 --pmc passes of a child on the same data
            a.c5_cache = cache or ""
            try:
                traffic, note = pmc_traffic(a, meta)
            finally:
                if cache:
                    import shutil
                    shutil.rmtree(os.path.dirname(cache), ignore_errors=True)
            leg["roofline"]["traffic"] = traffic["bytes"] if traffic else None
            leg["roofline"]["traffic_detail"] = traffic or note
            if traffic:
                leg["roofline"]["traffic_over_alg"] = round(traffic["bytes"] / r["alg_bytes"], 3)
        leg["leg_seconds"] = round(time.perf_counter() - t_leg, 1)
        out[name] = leg
        if world > 1:
            torch.distributed.barrier()
    return out


def pmc_traffic(args, W):
    """HBM traffic of the dominant kernel from rocprofv3 PMC counters, in two separate passes
    (FETCH_SIZE and WRITE_SIZE cannot share one pass on gfx950), corrected as
    /opt/skills/guides/MI355X_MICROARCH.md (HBM) prescribes: counters are in KiB; FETCH_SIZE counts
    exactly half the bytes of a wide (16 B/lane) coalesced streaming read on gfx950 -> x2 (and, measured
    with tools/lab/fetch_calib.hip, of 4- and 8-B coalesced and per-lane segment reads too); WRITE_SIZE
    is exact for 16-B streaming stores. Runs bench.py itself as a child under rocprofv3. A workload
    whose step is a kernel pipeline (W.pmc_regex, e.g. C5) reports the sum over one step's dispatches;
    otherwise the average per launch of W.kernel."""
    import csv
    import glob
    import shutil
    import subprocess
    import tempfile
    if not shutil.which("rocprofv3"):
        return None, "rocprofv3 not found"
    regex = getattr(W, "pmc_regex", W.kernel)
    per_step = hasattr(W, "pmc_regex")
    warm, steps = 1, 2
    vals = {}
    tmp = tempfile.mkdtemp(prefix="zgpu_pmc_")
    try:
        for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
            d = os.path.join(tmp, ctr)
            cmd = ["rocprofv3", "--pmc", ctr, "--kernel-include-regex", regex, "-d", d, "-o", "pmc",
                   "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "--child",
                   "--workload", args.workload, "--steps", str(steps), "--warmup", str(warm), "--no-cpu",
                   "--grid", *map(str, args.grid), "--c5-scale", str(args.c5_scale)] + \
                  (["--lane-priorities", args.lane_priorities] if args.lane_priorities else []) + \
                  (["--c5-cache", args.c5_cache] if getattr(args, "c5_cache", "") else [])
            # the child's stderr goes to a file; a heartbeat on ours shows the pass is alive
            elog = os.path.join(tmp, ctr + ".err")
            t0 = time.time()
            with open(elog, "wb") as ef:
                proc = subprocess.Popen(cmd, stdout=subprocess.DEVNULL, stderr=ef)
                while True:
                    try:
                        rc = proc.wait(timeout=20)
                        break
                    except subprocess.TimeoutExpired:
                        print(f"[bench] rocprofv3 --pmc {ctr} pass running {time.time() - t0:.0f} s",
                              file=sys.stderr, flush=True)
                        if time.time() - t0 > 600:
                            proc.kill()
                            proc.wait()
                            return None, f"rocprofv3 --pmc {ctr} timed out"
            if rc:
                err = [ln for ln in open(elog, errors="replace").read().splitlines()
                       if "simple_timer" not in ln and ln.strip()]
                return None, f"rocprofv3 --pmc {ctr} rc={rc}: {' | '.join(err[-6:])[-600:]}"
            files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
            import re
            rx = re.compile(regex)
            v = [float(row["Counter_Value"]) for f in files for row in csv.DictReader(open(f))
                 if rx.search(row["Kernel_Name"]) and row["Counter_Name"] == ctr]
            if not v:
                return None, f"no {ctr} samples for {regex}"
            vals[ctr] = sum(v) / (warm + steps) if per_step else sum(v) / len(v)
    except Exception as e:  # noqa: BLE001 - report, never fail the bench line on the profiler
        return None, f"pmc pass failed: {e}"
    finally:
        shutil.rmtree(tmp, ignore_errors=True)
    fetch = vals["FETCH_SIZE"] * 1024 * 2
    write = vals["WRITE_SIZE"] * 1024
    out = {"bytes": int(fetch + write), "fetch_bytes": int(fetch), "write_bytes": int(write),
           "per": "step (all dispatches matching " + regex + ")" if per_step else "launch of " + regex,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes (KiB; FETCH x2 on gfx950)"}
    if per_step:
        out["note"] = ("the x2 FETCH correction, which the guide calibrates for 16-B/lane streaming reads, was "
                       "calibrated here for the entropy kernels' narrower loads too (4/8-B coalesced and per-lane "
                       "segment reads also report half: profiles/r05/r05cal_pmc_calibration_and_crc_fold_ab.txt)")
    return out, None


def launcher_cmd(args, argv, port):
    """torch.distributed.run over N local processes (one per GPU, rendezvous on 127.0.0.1), each
    running this script with the same flags."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + \
        [a for a in argv if a != "--dry-launch"]


def launch_workers(args):
    import socket
    import subprocess
    n_dev = torch.cuda.device_count()  # counts devices without initialising HIP (this image)
    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = launcher_cmd(args, sys.argv[1:], port)
    if args.dry_launch:
        print(json.dumps({"launch": cmd, "visible_devices": n_dev, "fields_at_n_gt_1": {
            "value": "units all ranks processed per step / the max over ranks of the step time",
            "roundtrip_ok": "MIN over ranks; the root checks EVERY received slab (C3/C4, slab_mismatches) and the "
                            "gathered L0 box (C5) against the synthesised values, plus its own decode",
            "gather": "gather_ms (max over ranks of the median in-step gather time), bytes_to_root, xgmi_GBps, "
                      "peak_GBps = min(N-1, 7) x 153 GB/s direct links into the root, frac",
            "world": "backend, world_size and every rank's device"}}))
        return 0
    if n_dev < args.gpus:
        print(f"bench.py: --gpus {args.gpus} but {n_dev} GPU(s) visible", file=sys.stderr)
        return 2
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    return subprocess.call(cmd, env=env)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--grid", type=int, nargs=3, default=[16, 16, 16], help="C2 chunk grid per GPU")
    ap.add_argument("--cpu-grid", type=int, nargs=3, default=[8, 8, 8], help="C2 CPU baseline sample grid")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--c5-scale", type=int, default=1, help="C5: divide the L0 y/x extents by this (1: the full [512,4096,4096] L0)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--lane-times", action="store_true", help="print each stream lane's solo time (stderr)")
    ap.add_argument("--bench-lanes", action="store_true",
                    help="C5: the bench-side stream lanes (round 5) instead of the library plan group (A/B)")
    ap.add_argument("--no-pmc", action="store_true", help="skip the rocprofv3 PMC traffic passes")
    ap.add_argument("--lane-priorities", default="",
                    help="comma-separated HIP stream priorities of the stream lanes (-1 high, 0 normal)")
    ap.add_argument("--lits-first", default=None,
                    help="comma-separated parts whose zstd plans decode literals before sequences (ZGPU_ZSTD_LITS_FIRST; "
                         "default: the workload's choice, '' for none)")
    ap.add_argument("--fork", action="store_true", help=argparse.SUPPRESS)  # A/B: concurrent plans keep their side streams
    ap.add_argument("--serial-lanes", action="store_true",
                    help="run every plan on one stream (profiling: per-kernel durations without overlap)")
    ap.add_argument("--emulate-rank", default="", help="R/N: decode rank R's share of an N-GPU C3/C5 run "
                    "on this one GPU (profiling; the line then covers that share only)")
    ap.add_argument("--no-rank-share", dest="rank_share", action="store_false",
                    help="skip the C3/C5 legs' predicted N = 8 rank shares (SURVEY 8(e))")
    ap.add_argument("--no-host-leg", dest="host_leg", action="store_false",
                    help="skip the PCIe-inclusive (host input/output) leg")
    ap.add_argument("--child", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--secondary", default="c3,c5",
                    help="workloads measured after the headline and reported in its line's `secondary` object "
                         "(comma-separated; '' for none)")
    ap.add_argument("--c5-cache", default="", help=argparse.SUPPRESS)
    ap.add_argument("--dropin-calls", type=int, default=8,
                    help="C3 drop-in leg: most calls one coalesced GPU batch takes (zgpu_ctx_set_coalescing)")
    ap.add_argument("--dropin-sweep", default="", help="C3 drop-in leg: also measure these max_calls values (a,b,...)")
    ap.add_argument("--secondary-c5-scale", type=int, default=1,
                    help="C5 scale of the secondary leg (L0 y/x divided by this)")
    ap.add_argument("--dry-launch", action="store_true",
                    help="print the launcher command --gpus N > 1 would start, and exit (no GPU touched)")
    args = ap.parse_args()

    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        # N processes, one per GPU: started here as a child launcher BEFORE anything touches the GPU
        # (this process never initialises HIP; it waits for the launcher and exits with its code)
        return launch_workers(args)
    world = int(env_world or "1")
    if world != args.gpus:
        print(f"bench.py: WORLD_SIZE={world} but --gpus {args.gpus}: refusing to report a line for a "
              f"world the flags do not name", file=sys.stderr)
        return 2
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
    W = r["W"]
    elapsed = torch.tensor([r["elapsed"]], dtype=torch.float64, device=dev)
    ok = torch.tensor([1 if r["ok"] else 0], dtype=torch.int32, device=dev)
    if world > 1:
        torch.distributed.all_reduce(elapsed, op=torch.distributed.ReduceOp.MAX)
        torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
    t = float(elapsed.item())
    value = W.step_bytes * args.steps / t / 2 ** 30
    gather = gather_report(r, world, dev)
    cpu = W.cpu_baseline() if (rank == 0 and not args.no_cpu) else None
    share = None
    if args.workload in ("c3", "c5") and world == 1 and args.rank_share and not args.emulate_rank:
        try:  # one rank's share at N = 8 on this GPU
            share = W.rank_share(t / args.steps * 1e3)
        except Exception as e:  # noqa: BLE001
            share = {"error": repr(e)[:300]}
    traffic, traffic_note = None, "skipped (--no-pmc or N>1)"
    if rank == 0 and world == 1 and not args.no_pmc:
        # the profiled child needs the HBM this process holds (C5: ~30 GB of frames, outputs and
        # scratch): keep the line's fields, drop the workload's tensors and the zgpu context's pools
        import gc
        import types
        W = types.SimpleNamespace(**{k: getattr(W, k) for k in ("scaling", "dtype", "data", "config", "kernel",
                                                                 "pmc_regex") if hasattr(W, k)})
        r["W"] = None
        gc.collect()
        args.ctx.close()
        torch.cuda.empty_cache()
        traffic, traffic_note = pmc_traffic(args, W)
    if rank == 0:
        achieved = r["alg_bytes"] / (r["ev_ms"] * 1e-3) / 1e9
        line = {
            "metric": METRIC, "value": round(value, 2), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(t / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": W.scaling, "vs_baseline": None, "dtype": W.dtype,
            "data": W.data, "config": W.config,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic["bytes"] if traffic else None,
                         "traffic_detail": traffic or traffic_note,
                         "kernel": W.kernel,
                         "alg_bytes_per_launch": r["alg_bytes"],
                         "avg_launch_ms_hip_events": round(r["ev_ms"], 4)},
            "cpu_baseline": cpu,
            "roundtrip_ok": bool(ok.item()),
            "world": r["world_info"],
            "decode_batch_ms_incl_host_planning": round(r["batch_ms"], 3),
            "host_leg": r["host"],
            "hip_env": {"GPU_MAX_HW_QUEUES": os.environ.get("GPU_MAX_HW_QUEUES", "unset (HIP default: 4)")},
        }
        if r["counters"][L_CTR_ZSTD_SERIAL] or r["counters"][L_CTR_ZSTD_PARALLEL]:
            line["zstd_items_per_step"] = {"block_parallel": r["counters"][L_CTR_ZSTD_PARALLEL],
                                           "serial_fallback": r["counters"][L_CTR_ZSTD_SERIAL]}
        if gather:
            line["gather"] = gather
        if share:
            line["c4_rank_share" if args.workload == "c3" else "c5_rank_share"] = share
    sec = secondary_legs(args, rank, world, dev, r) if args.secondary and not args.child else None
    if rank == 0:
        if sec:
            line["secondary"] = sec
        print(json.dumps(line), flush=True)
    # explicit teardown before the interpreter's: the workload's tensors, then the context (plans were
    # destroyed in run_gpu; chains keep their context alive until they go, zgpu_ctx_refcount)
    r["W"] = None
    import gc
    gc.collect()
    args.ctx.close()
    torch.cuda.synchronize()
    if world > 1:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    sys.exit(main() or 0)
