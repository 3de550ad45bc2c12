"""Multi-GPU read of one array subset: one process per GPU, RCCL only for the gather.

Chunks are independent decode units (zarrs runs them as a rayon loop,
zarrs/src/array/array_ops/array_read_ops_common.rs:173-176; sharding_codec.rs:702-704), so the
read is partitioned and each rank decodes its share on its own GPU with no data-path collective:

  slab_partition   the requested subset split into contiguous slabs along one axis (axis 0 by
                   default) -- each rank's result is a C-contiguous block of the subset; chunks that
                   straddle a slab boundary are decoded by both ranks (only their overlaps are written)
  lpt_partition    independent chunks assigned by longest-processing-time on encoded bytes (C2/C5
                   style batches with uneven compressed sizes)
  gather_slabs     the only exchange step: every rank's slab to the root, received directly into
                   its rows of the root's output (grouped send/recv: RCCL over xGMI on GPUs, gloo
                   on CPU), skipped at N=1

  gather_slabs_overlapped  the same exchange overlapped with the decode: slabs decoded in pieces of
                   whole chunk rows, each piece sent while the next one decodes (C4)
  gather_regions   chunk-partitioned ranks (LPT): every rank's chunk boxes of one subset; boxes that are
                   contiguous runs of the subset are received straight into place, the others are
                   packed into one message per rank and unpacked on the root

A process group whose backend cannot move device tensors (gloo) gets device data staged through
host memory (tests put two ranks on one GPU that way; RCCL/xGMI moves HBM directly).

retrieve_array_subset_distributed ties them together for a zarrs_amd.Array (or anything with the
same retrieve_array_subset_into(start, shape, out) method).
"""
from __future__ import annotations

import heapq
from typing import Sequence


def slab_partition(start: Sequence[int], shape: Sequence[int], world: int, axis: int = 0):
    """[(slab_start, slab_shape)] per rank; slabs differ by at most one row along `axis`
    (the first `extent % world` ranks take one more), empty slabs allowed when world > extent."""
    start, shape = [int(s) for s in start], [int(s) for s in shape]
    ext = shape[axis]
    base, extra = divmod(ext, world)
    out, pos = [], start[axis]
    for r in range(world):
        n = base + (1 if r < extra else 0)
        s, sh = list(start), list(shape)
        s[axis], sh[axis] = pos, n
        out.append((s, sh))
        pos += n
    return out


def chunk_line_partition(start: Sequence[int], shape: Sequence[int], chunk_shape: Sequence[int], world: int):
    """Stream-balanced partition of an array subset over `world` ranks (C4): the subset's
    chunk lines -- (chunk row, chunk column) pairs along axes 0 and 1, each spanning the subset on the
    other axes -- in C order, cut into `world` contiguous runs whose counts differ by at most one. A rank
    decodes the chunks of its lines only, so every chunk is decoded by exactly one rank and every rank
    gets the same number of chunks (+- one line) -- unlike axis-0 slabs, whose boundaries cut through
    chunk rows (the chunks there decoded by two ranks) and whose chunk counts step by whole rows.
    Returns [[(box_start, box_shape), ...] per rank] in array coordinates: at most three boxes per rank
    (a partial chunk row, whole chunk rows, a partial chunk row); 1-d subsets fall back to slabs."""
    start, shape, cs = [int(x) for x in start], [int(x) for x in shape], [int(x) for x in chunk_shape]
    nd = len(shape)
    if nd < 2 or any(n == 0 for n in shape):
        return [[(s, sh)] if all(n > 0 for n in sh) else [] for s, sh in slab_partition(start, shape, world)]
    lo = [s // c for s, c in zip(start, cs)]
    hi = [(s + n - 1) // c + 1 for s, n, c in zip(start, shape, cs)]
    nr, ny = hi[0] - lo[0], hi[1] - lo[1]
    total = nr * ny
    out = []
    for r in range(world):
        l0, l1 = r * total // world, (r + 1) * total // world
        boxes = []  # [b0, b1] per box, merged along axis 1 within a chunk row, then along axis 0
        for ln in range(l0, l1):
            ci, cj = lo[0] + ln // ny, lo[1] + ln % ny
            b0 = [max(start[0], ci * cs[0]), max(start[1], cj * cs[1])] + start[2:]
            b1 = [min(start[0] + shape[0], (ci + 1) * cs[0]), min(start[1] + shape[1], (cj + 1) * cs[1])] + \
                 [a + n for a, n in zip(start[2:], shape[2:])]
            if boxes and boxes[-1][0][0] == b0[0] and boxes[-1][1][1] == b0[1]:
                boxes[-1][1][1] = b1[1]
            else:
                boxes.append([b0, b1])
        merged = []
        for b0, b1 in boxes:
            if merged and merged[-1][1][0] == b0[0] and merged[-1][0][1:] == b0[1:] and merged[-1][1][1:] == b1[1:]:
                merged[-1][1][0] = b1[0]
            else:
                merged.append([list(b0), list(b1)])
        out.append([(b0, [e - b for b, e in zip(b0, b1)]) for b0, b1 in merged])
    return out


def lpt_partition(costs: Sequence[int], world: int):
    """Greedy LPT: items sorted by cost (ties by index) go to the least-loaded rank.
    Returns [[item indices] per rank], each list in ascending index order (deterministic)."""
    order = sorted(range(len(costs)), key=lambda i: (-int(costs[i]), i))
    heap = [(0, r) for r in range(world)]
    parts = [[] for _ in range(world)]
    for i in order:
        load, r = heapq.heappop(heap)
        parts[r].append(i)
        heapq.heappush(heap, (load + int(costs[i]), r))
    return [sorted(p) for p in parts]


def gather_slabs(local, slabs, axis: int = 0, dst: int = 0, group=None, out=None):
    """Gather every rank's slab (this rank's is `local`, shapes from `slab_partition`) to group rank
    `dst`. Returns the assembled subset on dst and None elsewhere.

    Axis-0 slabs of a C-order subset are contiguous byte ranges of it, so on the root every peer's
    slab is received straight into its place in the output (grouped point-to-point receives; RCCL
    has no gather, and a root gather over xGMI should use the direct links, not a ring) and the
    root's own slab is one device copy -- no padding, no temporaries, no concatenation. `out` may be
    given (the root's preallocated subset; `local` may already be its own view into it). Other axes
    fall back to a padded torch.distributed.gather. `dst` is a rank of `group`."""
    import torch
    import torch.distributed as dist
    world = len(slabs)
    if world == 1:
        return local
    rank = dist.get_rank(group)
    g_dst = dist.get_global_rank(group, dst) if group is not None else dst
    if axis == 0:
        if rank != dst:
            if local.numel():
                dist.send(local.contiguous(), g_dst, group=group)
            return None
        if out is not None and not out.is_contiguous():  # P2P receives need contiguous targets
            got = gather_slabs(local, slabs, axis, dst, group)
            out.copy_(got)
            return out
        if out is None:
            shape = list(local.shape)
            shape[0] = sum(sh[0] for _, sh in slabs)
            out = torch.empty(shape, dtype=local.dtype, device=local.device)
        ops, row = [], 0
        for r, (_, sh) in enumerate(slabs):
            part = out.narrow(0, row, sh[0])
            row += sh[0]
            if r == dst:
                if part.data_ptr() != local.data_ptr():
                    part.copy_(local)
            elif part.numel():
                g_r = dist.get_global_rank(group, r) if group is not None else r
                ops.append(dist.P2POp(dist.irecv, part, g_r, group=group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return out
    mx = max(sh[axis] for _, sh in slabs)
    send = local
    if local.shape[axis] != mx:
        pad_shape = list(local.shape)
        pad_shape[axis] = mx
        send = torch.zeros(pad_shape, dtype=local.dtype, device=local.device)
        send.narrow(axis, 0, local.shape[axis]).copy_(local)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send.contiguous(), bufs, dst=g_dst, group=group)
    if rank != dst:
        return None
    parts = [b.narrow(axis, 0, sh[axis]) for b, (_, sh) in zip(bufs, slabs)]
    return torch.cat(parts, dim=axis)


def slab_pieces(slab_start, slab_shape, piece_rows: int, axis: int = 0):
    """A slab cut along `axis` at array-coordinate multiples of `piece_rows` (the chunk or inner-chunk
    extent: a piece's decode touches only its own chunk rows, so no chunk is decoded twice inside a
    rank): [(row offset within the slab, rows)], in order."""
    s0, n = int(slab_start[axis]), int(slab_shape[axis])
    out, r = [], s0
    while r < s0 + n:
        e = min(s0 + n, (r // piece_rows + 1) * piece_rows)
        out.append((r - s0, e - r))
        r = e
    return out


def gather_slabs_overlapped(decode_piece, local, slabs, piece_rows: int, dst: int = 0, group=None, out=None):
    """gather_slabs with the exchange overlapped with the decode (C4): every rank's slab is
    decoded piece by piece (slab_pieces), and a peer sends each piece to the root as soon as it is
    decoded, while its next piece decodes -- over RCCL the send is queued on the communicator's stream
    behind the decode already on the caller's stream, so the xGMI transfer of piece k runs beside the
    kernels of piece k+1. The root posts every receive first (straight into place in `out`) and then
    decodes its own pieces into its rows. decode_piece(k, view) decodes piece k of this rank's slab into
    `view` (its rows of `local`, or of the root's `out`). Axis 0 only. Returns the subset on dst."""
    import torch
    import torch.distributed as dist
    world = len(slabs)
    rank = dist.get_rank(group) if world > 1 else 0
    pieces = [slab_pieces(s, sh, piece_rows) for s, sh in slabs]
    if world == 1:
        for k, (r0, n) in enumerate(pieces[0]):
            decode_piece(k, local.narrow(0, r0, n))
        return local
    staged = _host_staged(group) and local.is_cuda  # gloo: device pieces staged through host memory
    g_dst = dist.get_global_rank(group, dst) if group is not None else dst
    if rank != dst:
        works = []
        for k, (r0, n) in enumerate(pieces[rank]):
            part = local.narrow(0, r0, n)
            decode_piece(k, part)
            if part.numel():
                t = part.cpu() if staged else part  # (the staging copy waits for the decode)
                works.append((dist.isend(t, g_dst, group=group), t))
        for w, _ in works:
            w.wait()
        return None
    if out is None:
        shape = list(local.shape)
        shape[0] = sum(sh[0] for _, sh in slabs)
        out = torch.empty(shape, dtype=local.dtype, device=local.device)
    recvs, row, own = [], 0, 0
    for r, (_, sh) in enumerate(slabs):
        if r == dst:
            own = row
        else:
            g_r = dist.get_global_rank(group, r) if group is not None else r
            for r0, n in pieces[r]:
                tgt = out.narrow(0, row + r0, n)
                if not tgt.numel():
                    continue
                buf = torch.empty(tgt.shape, dtype=tgt.dtype) if staged else tgt
                recvs.append((dist.irecv(buf, g_r, group=group), buf, tgt))
        row += sh[0]
    for k, (r0, n) in enumerate(pieces[dst]):
        decode_piece(k, out.narrow(0, own + r0, n))
    for w, buf, tgt in recvs:
        w.wait()
        if buf is not tgt:
            tgt.copy_(buf)
    return out


def slab_mismatches(gathered, expected, slabs, axis: int = 0):
    """The ranks whose slab of a gathered subset differs from `expected` (bit for bit; the root's
    check of every received slab, not only its own). Both tensors hold the whole subset."""
    import torch
    bad, row = [], 0
    for r, (_, sh) in enumerate(slabs):
        n = int(sh[axis])
        a, b = gathered.narrow(axis, row, n), expected.narrow(axis, row, n)
        row += n
        if a.element_size() in (1, 2, 4, 8) and a.is_floating_point():
            iv = {1: torch.int8, 2: torch.int16, 4: torch.int32, 8: torch.int64}[a.element_size()]
            a, b = a.contiguous().view(iv), b.contiguous().view(iv)
        if not torch.equal(a, b):
            bad.append(r)
    return bad


def chunk_boxes(array_shape, chunk_shape, start, shape):
    """[(chunk grid index, box start, box shape)] for every chunk of a regular grid that intersects
    the subset (chunks_in_array_subset, array_ops_array.rs:341-346), boxes in array coordinates."""
    import itertools
    lo = [int(s) // c for s, c in zip(start, chunk_shape)]
    hi = [(int(s) + int(n) - 1) // c + 1 for s, n, c in zip(start, shape, chunk_shape)]
    out = []
    if any(int(n) == 0 for n in shape):
        return out
    for idx in itertools.product(*[range(a, b) for a, b in zip(lo, hi)]):
        b0 = [max(int(s), i * c) for s, i, c in zip(start, idx, chunk_shape)]
        b1 = [min(int(s) + int(n), (i + 1) * c, a) for s, n, i, c, a in zip(start, shape, idx, chunk_shape,
                                                                              array_shape)]
        out.append((tuple(idx), b0, [e - b for b, e in zip(b0, b1)]))
    return out


def _host_staged(group) -> bool:
    """True when the group's backend moves host tensors only (gloo): device data is staged."""
    import torch.distributed as dist
    return dist.is_initialized() and dist.get_backend(group) == "gloo"


def _contiguous_in(bs, shape) -> bool:
    """A box of shape `bs` inside a C-order array of shape `shape` is one contiguous run: after the
    leading extent-1 axes, every axis but the first non-unit one spans the whole array."""
    i = 0
    while i < len(bs) - 1 and int(bs[i]) == 1:
        i += 1
    return all(int(b) == int(s) for b, s in zip(bs[i + 1:], shape[i + 1:]))


def gather_regions(local, boxes_by_rank, sub_start, sub_shape, dst: int = 0, group=None, out=None,
                   local_origin=None):
    """Assemble an array subset on group rank `dst` from chunk-partitioned ranks (C5: chunks
    LPT-partitioned over the GPUs, one cross-GPU subset gathered). `local` is this
    rank's copy of the whole array holding the chunks it decoded; boxes_by_rank[r] lists the
    (start, shape) array boxes rank r contributes. Each peer packs its boxes into one contiguous
    buffer and sends it with a single point-to-point message; the root receives every peer's buffer
    (grouped receives, all links at once) and unpacks the boxes into the subset. Returns the subset
    on dst and None elsewhere. local_origin: the coordinates of local's first element (default the
    origin: local is the whole array; C4 passes its rank's slab)."""
    import torch
    import torch.distributed as dist
    world = len(boxes_by_rank)
    rank = dist.get_rank(group) if world > 1 else 0

    def view(t, b0, bs, origin):
        sl = tuple(slice(a - o, a - o + n) for a, n, o in zip(b0, bs, origin))
        return t[sl]

    def split(boxes):  # (packed boxes, boxes received in place): the same on sender and root
        packed = [b for b in boxes if not _contiguous_in(b[1], sub_shape)]
        direct = [b for b in boxes if _contiguous_in(b[1], sub_shape)]
        return packed, direct

    def numel(bs):
        return int(torch.Size([int(x) for x in bs]).numel())
    zero = [0] * len(sub_start) if local_origin is None else [int(x) for x in local_origin]
    if rank != dst:
        packed, direct = split(boxes_by_rank[rank])
        peer = dist.get_global_rank(group, dst) if group is not None else dst
        n = sum(numel(bs) for _, bs in packed)
        ops = []
        if n:
            flat = torch.empty(n, dtype=local.dtype, device=local.device)
            off = 0
            for b0, bs in packed:
                k = numel(bs)
                flat.narrow(0, off, k).view(bs).copy_(view(local, b0, bs, zero))
                off += k
            ops.append(dist.P2POp(dist.isend, flat, peer, group=group))
        for b0, bs in direct:  # one message per box, landing in place on the root
            if numel(bs):
                ops.append(dist.P2POp(dist.isend, view(local, b0, bs, zero).contiguous(), peer, group=group))
        if ops:
            for w in dist.batch_isend_irecv(ops):
                w.wait()
        return None
    if out is not None and not out.is_contiguous():  # boxes are received in place: a contiguous target
        got = gather_regions(local, boxes_by_rank, sub_start, sub_shape, dst, group, local_origin=local_origin)
        out.copy_(got)
        return out
    if out is None:
        out = torch.empty([int(x) for x in sub_shape], dtype=local.dtype, device=local.device)
    for b0, bs in boxes_by_rank[dst]:
        o, l_ = view(out, b0, bs, sub_start), view(local, b0, bs, zero)
        if o.data_ptr() != l_.data_ptr() or o.stride() != l_.stride():  # the root decoded in place: no copy
            o.copy_(l_)
    ops, bufs = [], []
    for r in range(world):
        if r == dst:
            continue
        packed, direct = split(boxes_by_rank[r])
        g_r = dist.get_global_rank(group, r) if group is not None else r
        n = sum(numel(bs) for _, bs in packed)
        if n:
            flat = torch.empty(n, dtype=local.dtype, device=local.device)
            bufs.append((packed, flat))
            ops.append(dist.P2POp(dist.irecv, flat, g_r, group=group))
        for b0, bs in direct:
            if numel(bs):
                ops.append(dist.P2POp(dist.irecv, view(out, b0, bs, sub_start), g_r, group=group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for packed, flat in bufs:
        off = 0
        for b0, bs in packed:
            k = numel(bs)
            view(out, b0, bs, sub_start).copy_(flat.narrow(0, off, k).view(bs))
            off += k
    return out


def _retrieve_lines_distributed(array, start, shape, group, dst, device, tdtype, world, rank):
    """retrieve_array_subset_distributed(partition="lines"): this rank's chunk_line_partition boxes of
    the subset (the array's read granule: a sharded array's inner chunks) decoded as one batch into
    its slab (the root's: a view of the gathered subset), then gathered with gather_regions."""
    import torch
    parts = chunk_line_partition(start, shape, array.read_chunk_shape, world)
    mine = parts[rank]
    rel = [[([a - o for a, o in zip(b0, start)], bs) for b0, bs in boxes] for boxes in parts]
    if mine:
        r0 = min(b0[0] for b0, _ in mine)
        r1 = max(b0[0] + bs[0] for b0, bs in mine)
    else:
        r0 = r1 = int(start[0])
    slab0 = [r0] + [int(s) for s in start[1:]]
    slab_shape = [r1 - r0] + [int(n) for n in shape[1:]]
    staged = device.type == "cuda" and world > 1 and _host_staged(group)
    out = None
    if rank == dst and not staged:  # the root decodes its boxes in place inside the gathered subset
        out = torch.empty([int(n) for n in shape], dtype=tdtype, device=device)
        local = out.narrow(0, r0 - int(start[0]), r1 - r0)
    else:
        local = torch.empty(slab_shape, dtype=tdtype, device=device)
    if mine:
        array.retrieve_boxes_into(mine, local, slab0)
    origin = [a - o for a, o in zip(slab0, start)]
    if staged:  # gloo moves host tensors only: the slab staged through host memory
        got = gather_regions(local.cpu(), rel, [0] * len(shape), shape, dst, group, local_origin=origin)
        return None if got is None else got.to(device)
    return gather_regions(local, rel, [0] * len(shape), shape, dst, group, out=out, local_origin=origin)


def retrieve_array_subset_distributed(array, start, shape, group=None, dst: int = 0, axis: int = 0,
                                      device=None, piece_rows: int | None = None, partition: str = "slabs"):
    """Array::retrieve_array_subset over all ranks of `group`: this rank decodes its slab on its own
    device, then the slabs are gathered to `dst` (the assembled subset there, None elsewhere).
    piece_rows (axis 0): decode and send the slab in pieces of that many array rows (the chunk extent
    along axis 0, or a multiple), the sends overlapping the next piece's decode
    (gather_slabs_overlapped). partition="lines": each rank decodes its stream-balanced chunk lines
    (chunk_line_partition over the array's read granule, <= 3 boxes, one batch) instead of a slab --
    every chunk decoded by exactly one rank (bench.py's C4)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    tdtype = torch.from_numpy(np.zeros(1, dtype=array.dtype)).dtype
    device = torch.device(device)
    if partition == "lines" and world > 1 and len(shape) >= 2:
        return _retrieve_lines_distributed(array, start, shape, group, dst, device, tdtype, world, rank)
    if partition not in ("slabs", "lines"):
        raise ValueError(f"partition {partition!r}: 'slabs' or 'lines'")
    slabs = slab_partition(start, shape, world, axis)
    s, sh = slabs[rank]
    if piece_rows and axis == 0:
        pieces = slab_pieces(s, sh, piece_rows)

        def decode_piece(k, view):
            r0, n = pieces[k]
            if n and all(x > 0 for x in sh):
                array.retrieve_array_subset_into([s[0] + r0] + list(s[1:]), [n] + list(sh[1:]), view)
        out = None
        if rank == dst:  # the root's pieces decode in place inside the gathered subset
            out = torch.empty([int(n) for n in shape], dtype=tdtype, device=device)
            local = out.narrow(0, sum(slabs[r][1][0] for r in range(rank)), sh[0])
        else:
            local = torch.empty(sh, dtype=tdtype, device=device)
        return gather_slabs_overlapped(decode_piece, local, slabs, piece_rows, dst, group, out=out)
    if device.type == "cuda" and world > 1 and _host_staged(group):
        # gloo moves host tensors only: decode on the device, stage the slab through host memory
        local = torch.empty(sh, dtype=tdtype, device=device)
        if all(n > 0 for n in sh):
            array.retrieve_array_subset_into(s, sh, local)
        got = gather_slabs(local.cpu(), slabs, axis, dst, group)
        return None if got is None else got.to(device)
    out = None
    if rank == dst and axis == 0:  # the root decodes its slab in place inside the gathered subset
        out = torch.empty([int(n) for n in shape], dtype=tdtype, device=device)
        row0 = sum(slabs[r][1][0] for r in range(rank))
        local = out.narrow(0, row0, sh[0])
    else:
        local = torch.empty(sh, dtype=tdtype, device=device)
    if all(n > 0 for n in sh):
        array.retrieve_array_subset_into(s, sh, local)
    return gather_slabs(local, slabs, axis, dst, group, out=out)
