"""Multi-GPU read of one array subset: one process per GPU, RCCL only for the gather.

Chunks are independent decode units (zarrs runs them as a rayon loop,
zarrs/src/array/array_ops/array_read_ops_common.rs:173-176; sharding_codec.rs:702-704), so the
read is partitioned and each rank decodes its share on its own GPU with no data-path collective:

  slab_partition   the requested subset split into contiguous slabs along one axis (axis 0 by
                   default) -- each rank's result is a C-contiguous block of the subset; chunks that
                   straddle a slab boundary are decoded by both ranks (only their overlaps are written)
  lpt_partition    independent chunks assigned by longest-processing-time on encoded bytes (C2/C5
                   style batches with uneven compressed sizes)
  gather_slabs     the only exchange step: every rank's slab to the root in one
                   torch.distributed.gather (RCCL over xGMI on GPUs, gloo on CPU), skipped at N=1

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


def gather_slabs(local, slabs, axis: int = 0, dst: int = 0, group=None):
    """Gather every rank's slab (this rank's is `local`, shapes from `slab_partition`) to `dst`.
    Returns the assembled subset on dst and None elsewhere. Unequal slabs are padded to the largest
    one for the collective and trimmed after it."""
    import torch
    import torch.distributed as dist
    world = len(slabs)
    if world == 1:
        return local
    rank = dist.get_rank(group)
    mx = max(sh[axis] for _, sh in slabs)
    send = local
    if local.shape[axis] != mx:
        pad_shape = list(local.shape)
        pad_shape[axis] = mx
        send = torch.zeros(pad_shape, dtype=local.dtype, device=local.device)
        send.narrow(axis, 0, local.shape[axis]).copy_(local)
    bufs = [torch.empty_like(send) for _ in range(world)] if rank == dst else None
    dist.gather(send.contiguous(), bufs, dst=dst, group=group)
    if rank != dst:
        return None
    parts = [b.narrow(axis, 0, sh[axis]) for b, (_, sh) in zip(bufs, slabs)]
    return torch.cat(parts, dim=axis)


def retrieve_array_subset_distributed(array, start, shape, group=None, dst: int = 0, axis: int = 0,
                                      device=None):
    """Array::retrieve_array_subset over all ranks of `group`: this rank decodes its slab on its own
    device, then the slabs are gathered to `dst` (the assembled subset there, None elsewhere)."""
    import numpy as np
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group) if dist.is_initialized() else 1
    rank = dist.get_rank(group) if dist.is_initialized() else 0
    slabs = slab_partition(start, shape, world, axis)
    s, sh = slabs[rank]
    if device is None:
        device = torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else "cpu"
    tdtype = torch.from_numpy(np.zeros(1, dtype=array.dtype)).dtype
    local = torch.empty(sh, dtype=tdtype, device=device)
    if all(n > 0 for n in sh):
        array.retrieve_array_subset_into(s, sh, local)
    return gather_slabs(local, slabs, axis, dst, group)
