"""N>1 read path on CPU (gloo, world_size 2 and 3): slab partition + gather assemble exactly the
subset rank 0 would have read alone (the root's slab decoded in place, peers received straight into
their rows); the C5 pattern (chunks LPT-partitioned by encoded size, one cross-rank subset gathered)
on zstd-shuffle chunks; gathers inside a process subgroup. The per-rank decode is the CPU oracle
(the GPU decode itself is covered by the -m gpu parity tests)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle as O
from zarrs_amd.distributed import (_contiguous_in, chunk_boxes, chunk_line_partition, gather_regions, gather_slabs,
                                   lpt_partition,
                                   slab_mismatches, slab_pieces,
                                   retrieve_array_subset_distributed, slab_partition)

CODECS = [{"name": "bytes", "configuration": {"endian": "little"}}, {"name": "crc32c"}]
C5_CODECS = [{"name": "bytes", "configuration": {"endian": "little"}},
             {"name": "numcodecs.shuffle", "configuration": {"elementsize": 2}},
             {"name": "zstd", "configuration": {"level": 3, "checksum": False}}]


def _encode_grid(co, a, cs):
    chunks = {}
    for idx in np.ndindex(*[-(-s // c) for s, c in zip(a.shape, cs)]):
        blk = np.zeros(cs, a.dtype)
        sl = tuple(slice(i * c, min((i + 1) * c, s)) for i, c, s in zip(idx, cs, a.shape))
        blk[tuple(slice(0, n) for n in a[sl].shape)] = a[sl]
        chunks[idx] = co.encode(blk)
    return chunks


class OracleArray:
    """retrieve_array_subset_into through the CPU oracle (the per-rank decode stand-in), counting
    the output buffers it was handed (the root must decode into its view of the gathered subset)."""
    def __init__(self, a, cs, codecs, data_type):
        self.shape, self.cs = list(a.shape), cs
        self.co = O.OracleChain.from_metadata(codecs, data_type, 0, a.ndim)
        self.chunks = _encode_grid(self.co, a, cs)
        self.dtype = a.dtype
        self.outs = []

    def retrieve_array_subset_into(self, start, shape, out):
        self.outs.append(out)
        got = O.retrieve_array_subset(self.co, self.shape, self.cs, self.chunks, start, shape)
        out.copy_(torch.from_numpy(got))

    @property
    def read_chunk_shape(self):
        return self.cs

    def retrieve_boxes_into(self, boxes, out, origin):
        for b0, bs in boxes:
            got = O.retrieve_array_subset(self.co, self.shape, self.cs, self.chunks, b0, bs)
            out[tuple(slice(a - o, a - o + n) for a, o, n in zip(b0, origin, bs))].copy_(torch.from_numpy(got))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = (np.arange(37 * 11 * 5, dtype=np.float32) * 1.5).reshape(37, 11, 5)
        arr = OracleArray(a, [4, 4, 2], CODECS, "float32")
        res = {}
        for name, (start, shape) in {"even": ([2, 1, 0], [20, 9, 5]), "ragged": ([3, 0, 1], [31, 11, 3]),
                                     "tiny": ([5, 5, 2], [1, 2, 2])}.items():
            lines = retrieve_array_subset_distributed(arr, start, shape, device="cpu", partition="lines")
            got = retrieve_array_subset_distributed(arr, start, shape, device="cpu")
            if rank == 0:
                sl = tuple(slice(s, s + n) for s, n in zip(start, shape))
                res[name] = bool(np.array_equal(got.numpy(), a[sl]))
                res[name + "_lines"] = bool(np.array_equal(lines.numpy(), a[sl]))
                # the root's slab was decoded in place, inside the returned subset (no temporary)
                own = arr.outs[-1] if arr.outs else None
                res[name + "_inplace"] = own is None or own.data_ptr() == got.data_ptr()
            else:
                res[name] = got is None
                res[name + "_lines"] = lines is None
        # C5 pattern: u16 chunks [bytes, shuffle 2, zstd 3] LPT-partitioned by encoded size; every rank
        # decodes its chunks into its own level array; one subset spanning ranks gathered to rank 0
        rng = np.random.default_rng(42)
        lvl = (100 + rng.poisson(50, (8, 24, 40))).astype(np.uint16)
        lvl[2:6, 4:20, 8:30] += 3000
        cs = [4, 8, 8]
        src = OracleArray(lvl, cs, C5_CODECS, "uint16")
        keys = sorted(src.chunks)
        parts = lpt_partition([len(src.chunks[k]) for k in keys], world)
        owner = {keys[i]: r for r, p in enumerate(parts) for i in p}
        local = torch.zeros(lvl.shape, dtype=torch.int16)
        for k in keys:
            if owner[k] != rank:
                continue
            st = [i * c for i, c in zip(k, cs)]
            sh = [min(c, s - o) for c, s, o in zip(cs, lvl.shape, st)]
            blk = src.co.decode(src.chunks[k], cs)
            local[tuple(slice(o, o + n) for o, n in zip(st, sh))] = torch.from_numpy(
                blk[tuple(slice(0, n) for n in sh)].view(np.int16))
        sub0, subn = [1, 3, 5], [6, 19, 30]
        boxes = [[] for _ in range(world)]
        for idx, b0, bs in chunk_boxes(list(lvl.shape), cs, sub0, subn):
            boxes[owner[idx]].append((b0, bs))
        res["c5_spans_ranks"] = all(len(b) > 0 for b in boxes)
        got = gather_regions(local, boxes, sub0, subn)
        if rank == 0:
            res["c5_gather"] = bool(np.array_equal(got.numpy().view(np.uint16), lvl[1:7, 3:22, 5:35]))
        else:
            res["c5_gather"] = got is None
        # a subset whose chunk boxes are contiguous runs of it: received in place (no packing)
        sub0, subn = [1, 8, 16], [6, 8, 8]
        boxes = [[] for _ in range(world)]
        for idx, b0, bs in chunk_boxes(list(lvl.shape), cs, sub0, subn):
            boxes[owner[idx]].append((b0, bs))
        got = gather_regions(local, boxes, sub0, subn)
        if rank == 0:
            res["c5_gather_direct"] = bool(np.array_equal(got.numpy().view(np.uint16), lvl[1:7, 8:16, 16:24]))
        else:
            res["c5_gather_direct"] = got is None
        # C4 pattern (bench.py at N > 1): stream-balanced chunk lines, each rank decoding its boxes into
        # its slab (the rows its boxes span; the root's slab is a view of the gathered subset), the boxes
        # gathered with the slab as local's origin
        sub0, subn = [2, 1, 0], [33, 10, 5]
        parts = chunk_line_partition(sub0, subn, arr.cs, world)
        rel = [[([x - o for x, o in zip(b0, sub0)], bs) for b0, bs in boxes] for boxes in parts]
        mine = rel[rank]
        r0 = min(b0[0] for b0, _ in mine)
        r1 = max(b0[0] + bs[0] for b0, bs in mine)
        full = torch.zeros(subn, dtype=torch.float32) if rank == 0 else None
        slab = full.narrow(0, r0, r1 - r0) if rank == 0 else torch.full([r1 - r0] + subn[1:], -1.0)
        for b0, bs in mine:
            arr.retrieve_array_subset_into([x + o for x, o in zip(b0, sub0)], bs,
                                           slab[b0[0] - r0:b0[0] - r0 + bs[0], b0[1]:b0[1] + bs[1], b0[2]:b0[2] + bs[2]])
        got = gather_regions(slab, rel, [0, 0, 0], subn, out=full, local_origin=[r0, 0, 0])
        if rank == 0:
            res["c4_lines_gather"] = bool(np.array_equal(got.numpy(), a[2:35, 1:11, 0:5]))
        else:
            res["c4_lines_gather"] = got is None
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _subgroup_worker(rank, world, port, q):
    """world 3, a subgroup of global ranks [1, 2]: group rank 0 (global 1) is the gather root."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = dist.new_group([1, 2])
        res = {}
        if rank in (1, 2):
            a = (np.arange(19 * 6, dtype=np.float32) - 7).reshape(19, 6)
            arr = OracleArray(a, [5, 4], CODECS, "float32")
            got = retrieve_array_subset_distributed(arr, [2, 1], [15, 5], group=g, device="cpu")
            if rank == 1:
                res["root"] = got is not None and bool(np.array_equal(got.numpy(), a[2:17, 1:6]))
            else:
                res["peer"] = got is None
        dist.barrier()
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _verify_worker(rank, world, port, q):
    """bench.py's N > 1 check (C3/C4): the root compares EVERY received slab with the expected subset,
    not only its own, and the verdict (roundtrip_ok) is the MIN over ranks. Rank 1 corrupts one
    element of its slab: the root names slab 1 and every rank sees roundtrip_ok false. Also a gather
    into a non-contiguous root output (a transposed view), which is received through a temporary."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        res = {}
        shape = [13, 7, 5]
        full = torch.arange(int(np.prod(shape)), dtype=torch.float32).reshape(shape) * 0.25 - 3
        slabs = slab_partition([0, 0, 0], shape, world)
        for corrupt in (False, True):
            s0, sh = slabs[rank]
            local = full[s0[0]:s0[0] + sh[0]].clone()
            if corrupt and rank == 1:
                local[1, 2, 3] += 1.0
            got = gather_slabs(local, slabs, dst=0)
            ok = torch.tensor([1], dtype=torch.int32)
            if rank == 0:
                bad = slab_mismatches(got, full, slabs)
                res[f"bad_{corrupt}"] = bad
                ok[0] = 0 if bad else 1
            dist.all_reduce(ok, op=dist.ReduceOp.MIN)
            res[f"roundtrip_ok_{corrupt}"] = bool(ok.item())
        # non-contiguous root output
        s0, sh = slabs[rank]
        local = full[s0[0]:s0[0] + sh[0]].clone()
        out = torch.empty([shape[2], shape[1], shape[0]]).permute(2, 1, 0) if rank == 0 else None
        got = gather_slabs(local, slabs, dst=0, out=out)
        if rank == 0:
            res["noncontig"] = got is out and bool(torch.equal(out, full))
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _overlap_worker(rank, world, port, q):
    """C4's overlapped gather (gather_slabs_overlapped through retrieve_array_subset_distributed with
    piece_rows): every rank decodes its slab in pieces of whole chunk rows and sends each piece while the
    next decodes; the root receives straight into place. Checked against the whole subset for even and
    ragged slabs, pieces not aligned with the slab starts, and a slab thinner than one piece."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        a = (np.arange(37 * 11 * 5, dtype=np.float32) * 0.75 - 9).reshape(37, 11, 5)
        arr = OracleArray(a, [4, 4, 2], CODECS, "float32")
        res = {}
        for name, (start, shape, rows) in {"even": ([2, 1, 0], [24, 9, 5], 4), "ragged": ([3, 0, 1], [31, 11, 3], 4),
                                          "coarse": ([1, 2, 0], [35, 7, 5], 8),
                                          "thin": ([17, 0, 0], [2, 11, 5], 4)}.items():
            arr.outs.clear()
            got = retrieve_array_subset_distributed(arr, start, shape, device="cpu", piece_rows=rows)
            slabs = slab_partition(start, shape, world)
            # one decode per piece: whole chunk rows, never a row decoded twice inside a rank
            res[name + "_pieces"] = len(arr.outs) == len(slab_pieces(*slabs[rank], rows)) or not slabs[rank][1][0]
            if rank == 0:
                sl = tuple(slice(s, s + n) for s, n in zip(start, shape))
                res[name] = bool(np.array_equal(got.numpy(), a[sl]))
            else:
                res[name] = got is None
        q.put((rank, res))
    finally:
        dist.destroy_process_group()


def _spawn(target, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    return out


def test_slab_partition_covers_subset():
    for ext, world in ((768, 8), (10, 3), (2, 4)):
        slabs = slab_partition([200, 5, 7], [ext, 3, 4], world)
        assert sum(sh[0] for _, sh in slabs) == ext
        assert slabs[0][0][0] == 200
        for (s0, sh0), (s1, _) in zip(slabs, slabs[1:]):
            assert s0[0] + sh0[0] == s1[0]
        assert max(sh[0] for _, sh in slabs) - min(sh[0] for _, sh in slabs) <= 1


def test_lpt_partition_balanced_and_deterministic():
    rng = np.random.default_rng(0)
    costs = rng.integers(1000, 100000, size=500).tolist()
    parts = lpt_partition(costs, 8)
    assert sorted(i for p in parts for i in p) == list(range(500))
    loads = [sum(costs[i] for i in p) for p in parts]
    assert max(loads) - min(loads) <= max(costs)
    assert parts == lpt_partition(costs, 8)


def test_gather_single_rank_passthrough():
    t = torch.arange(6).reshape(2, 3)
    assert gather_slabs(t, slab_partition([0, 0], [2, 3], 1)) is t


def test_two_rank_gloo_gather():
    out = _spawn(_worker, 2)
    assert all(out[0].values()), out
    assert all(out[1].values()), out


def test_subgroup_gather_root_is_group_rank():
    out = _spawn(_subgroup_worker, 3)
    assert out[1] == {"root": True} and out[2] == {"peer": True}, out


def test_chunk_boxes_cover_subset():
    boxes = chunk_boxes([10, 13], [4, 5], [3, 2], [6, 11])
    assert sum(bs[0] * bs[1] for _, _, bs in boxes) == 66
    assert [i for i, _, _ in boxes] == [(0, 0), (0, 1), (0, 2), (1, 0), (1, 1), (1, 2), (2, 0), (2, 1), (2, 2)]


def test_contiguous_box_rule():
    assert _contiguous_in([3, 8, 8], [6, 8, 8])
    assert _contiguous_in([1, 1, 5], [6, 8, 8])
    assert _contiguous_in([1, 3, 8], [6, 8, 8])
    assert not _contiguous_in([1, 3, 7], [6, 8, 8])
    assert not _contiguous_in([2, 4, 8], [6, 8, 8])


def test_world3_root_verifies_every_slab():
    out = _spawn(_verify_worker, 3)
    assert out[0]["bad_False"] == [] and out[0]["bad_True"] == [1]
    for r in range(3):
        assert out[r]["roundtrip_ok_False"] is True
        assert out[r]["roundtrip_ok_True"] is False
    assert out[0]["noncontig"]


def test_slab_mismatches_one_byte_float():
    """Floating dtypes compare bit for bit at every element size, 1-byte floats included."""
    if not hasattr(torch, "float8_e4m3fn"):
        pytest.skip("no float8 dtype in this torch")
    full = torch.arange(24, dtype=torch.uint8).view(torch.float8_e4m3fn).reshape(6, 4)
    slabs = slab_partition([0, 0], [6, 4], 2)
    assert slab_mismatches(full.clone(), full, slabs) == []
    bad = full.clone()
    bad.view(torch.uint8)[4, 1] ^= 1
    assert slab_mismatches(bad, full, slabs) == [1]


def test_slab_pieces_cut_at_chunk_rows():
    assert slab_pieces([3, 0], [10, 4], 4) == [(0, 1), (1, 4), (5, 4), (9, 1)]
    assert slab_pieces([8, 0], [8, 4], 4) == [(0, 4), (4, 4)]
    assert slab_pieces([5, 0], [0, 4], 4) == []


@pytest.mark.parametrize("world", [2, 3])
def test_overlapped_slab_gather(world):
    out = _spawn(_overlap_worker, world)
    for r, res in out.items():
        assert all(res.values()), (r, res)


@pytest.mark.parametrize("world", [1, 2, 3, 8, 13])
def test_chunk_line_partition_balanced_and_exact(world):
    """C4's partition: every voxel of the subset in exactly one rank's boxes, at most three boxes per
    rank, chunk counts per rank within one chunk line of each other, no chunk split between ranks."""
    start, shape, cs = [200, 300, 1000], [768, 768, 768], [32, 32, 32]
    parts = chunk_line_partition(start, shape, cs, world)
    assert len(parts) == world
    cover = np.zeros([25, 25], np.int32)  # chunk lines (axis-0 chunk, axis-1 chunk) of the subset
    vol = 0
    owner = {}
    for r, boxes in enumerate(parts):
        assert len(boxes) <= 3
        for b0, bs in boxes:
            assert b0[2] == start[2] and bs[2] == shape[2]
            vol += int(np.prod(bs))
            for ci in range(b0[0] // 32, (b0[0] + bs[0] - 1) // 32 + 1):
                for cj in range(b0[1] // 32, (b0[1] + bs[1] - 1) // 32 + 1):
                    cover[ci - 6, cj - 9] += 1
                    assert owner.setdefault((ci, cj), r) == r
    assert vol == int(np.prod(shape))
    assert (cover == 1).all()
    counts = [sum(1 for v in owner.values() if v == r) for r in range(world)]
    assert max(counts) - min(counts) <= 1
    # small and 2-d subsets; a 1-d subset falls back to slabs
    parts = chunk_line_partition([3, 1], [10, 7], [4, 3], 3)
    got = np.zeros([10, 7], np.int32)
    for boxes in parts:
        for b0, bs in boxes:
            got[b0[0] - 3:b0[0] - 3 + bs[0], b0[1] - 1:b0[1] - 1 + bs[1]] += 1
    assert (got == 1).all()
    assert chunk_line_partition([5], [10], [4], 2) == [[([5], [5])], [([10], [5])]]
