"""C4 rank-share probe (one GPU): how long a rank's share of the C3 subset takes to decode as a function
of its inner-chunk streams, for shares cut along inner-chunk boundaries -- axis-0 slabs of whole
inner-chunk rows (625 streams each) and stream-balanced shares of whole inner-chunk lines (rank r of 8
takes lines [r * L / 8, (r + 1) * L / 8) of the subset's L = 625 (chunk row, chunk y) lines, 25 streams
each: <= 1,975 streams, inside the pipelined gzip kernel's 2,048). Prints one line per share."""
import argparse
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench as B  # noqa: E402


def boxes_for_lines(start, shape, inner, l0, l1):
    """Array boxes of the subset covering (chunk row, chunk y) lines [l0, l1) (C order), full x extent."""
    lo = [s // inner for s in start]
    hi = [(s + n - 1) // inner + 1 for s, n in zip(start, shape)]
    ny = hi[1] - lo[1]
    boxes = []
    for ln in range(l0, l1):
        ci, cj = lo[0] + ln // ny, lo[1] + ln % ny
        b0 = [max(start[0], ci * inner), max(start[1], cj * inner), start[2]]
        b1 = [min(start[0] + shape[0], (ci + 1) * inner), min(start[1] + shape[1], (cj + 1) * inner),
              start[2] + shape[2]]
        if boxes and boxes[-1][0][0] == b0[0] and boxes[-1][1][0] == b1[0] and boxes[-1][1][1] == b0[1]:
            boxes[-1] = (boxes[-1][0], [b1[0], b1[1], b1[2]])  # extend along y
        else:
            boxes.append((b0, b1))
    return boxes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=5)
    a = ap.parse_args()
    from zarrs_amd import Context, make_desc
    args = argparse.Namespace(ctx=Context(0), emulate_rank="", c5_scale=1)
    dev = torch.device("cuda", 0)
    c3 = B.C3(args, 0, 1, dev)
    S, I = c3.SHARD, c3.INNER
    st, sh = c3.SUB_START, c3.SUB_SHAPE

    def time_boxes(boxes, label):
        r0 = min(b0[0] for b0, _ in boxes)
        r1 = max(b1[0] for _, b1 in boxes)
        bb0, bshape = [r0, st[1], st[2]], [r1 - r0, sh[1], sh[2]]
        buf = torch.empty(bshape, dtype=torch.float32, device=dev)
        pd, streams = [], 0
        for b0, b1 in boxes:
            for (si, sj, sk), (t, _) in c3.shards.items():
                org = [si * S, sj * S, sk * S]
                s0 = [max(x, o) for x, o in zip(b0, org)]
                s1 = [min(x, o + S) for x, o in zip(b1, org)]
                if any(q <= p for p, q in zip(s0, s1)):
                    continue
                streams += int(np.prod([(q - 1) // I - p // I + 1 for p, q in zip(s0, s1)]))
                pd.append(make_desc((t.data_ptr(), int(t.numel())), [S] * 3,
                                    sel_start=[p - o for p, o in zip(s0, org)],
                                    sel_shape=[q - p for p, q in zip(s0, s1)],
                                    out_start=[p - o for p, o in zip(s0, bb0)]))
        ms = B._time_plan_groups(args.ctx, [(c3.chain, pd, buf, bshape)], [[0]], set(), dev, reps=a.reps,
                                 status_each=True)
        print(f"{label:40s} boxes {len(boxes):2d} streams {streams:5d} descs {len(pd):3d} {ms:8.3f} ms", flush=True)
        del buf
        return ms, streams

    lo0 = st[0] // I
    # axis-0 slabs of whole inner-chunk rows: 2, 3 and 4 rows (the current 96-row slabs touch 4)
    for rows in (2, 3, 4):
        c0 = (lo0 + 1) * I
        time_boxes([([c0, st[1], st[2]], [c0 + rows * I, st[1] + sh[1], st[2] + sh[2]])], f"slab {rows} chunk rows")
    ny = (st[1] + sh[1] - 1) // I - st[1] // I + 1
    nz = (st[0] + sh[0] - 1) // I - st[0] // I + 1
    L = ny * nz
    worst = 0.0
    for r in range(8):
        ms, n = time_boxes(boxes_for_lines(st, sh, I, r * L // 8, (r + 1) * L // 8), f"balanced rank {r}/8")
        worst = max(worst, ms)
    print(f"balanced: slowest rank {worst:.3f} ms")


if __name__ == "__main__":
    main()
