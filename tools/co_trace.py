"""Summarise a ZGPU_TRACE=1 stderr log of coalesced drop-in calls (zgpu.cpp co_trace): per-batch
phase times and how busy the lanes were. Usage: python tools/co_trace.py <stderr file>"""
import collections
import statistics as st
import sys

ev = collections.defaultdict(lambda: collections.defaultdict(list))
for line in open(sys.argv[1]):
    if not line.startswith("[zgpu-trace]"):
        continue
    _, t, what, bid, a, b = line.split()[:6]
    ev[int(bid)][what].append((int(t), int(a)))
rows = []
for bid, d in sorted(ev.items()):
    if not all(k in d for k in ("arrive-lead", "lane", "batch-start", "h2d-done", "decode-done", "d2h-done")):
        continue
    t0 = d["arrive-lead"][0][0]
    lane, bs, h, dc, dd = (d[k][0][0] for k in ("lane", "batch-start", "h2d-done", "decode-done", "d2h-done"))
    co = max(t for t, _ in d.get("copied-out", [(dd, 0)]))
    pk = d["packed"][0][0] if "packed" in d else dc
    pa = d["pack-alloc"][0][0] if "pack-alloc" in d else pk
    rows.append(dict(pack=pk - dc, alloc=pa - pk, copy=dd - pa, boxed=d["packed"][0][1] if "packed" in d else -1,t0=t0, wait=lane - t0, setup=bs - lane, h2d=h - bs, decode=dc - h, d2h=dd - h - (dc - h),
                     copyout=co - dd, calls=d["batch-start"][0][1], busy=(lane, dd), end=co,
                     enc=sum(a for _, a in d["arrive-lead"] + d.get("arrive-join", []))))
print(f"{len(rows)} batches, {st.mean(r['calls'] for r in rows):.2f} calls each")
for k in ("wait", "setup", "h2d", "decode", "d2h", "pack", "alloc", "copy", "copyout"):
    v = [r[k] / 1e3 for r in rows]
    print(f"  {k:8s} median {st.median(v):7.2f} ms  mean {st.mean(v):7.2f}  max {max(v):7.2f}")
span = (min(r["t0"] for r in rows), max(r["end"] for r in rows))
busy = sum(b - a for a, b in (r["busy"] for r in rows))
print(f"span {(span[1] - span[0]) / 1e3:.1f} ms, lane-busy {busy / 1e3:.1f} ms = {busy / (span[1] - span[0]):.2f} lanes on average")
for boxed in (0, 1, 2):
    v = [r for r in rows if r["boxed"] == boxed]
    if v:
        name = ("compact", "box-copied (kernel)", "rect-copied (3-D DMA)")[boxed]
        print(f"  {name} batches {len(v)}: pack median {st.median(r['pack'] for r in v) / 1e3:.2f} ms, "
              f"D2H median {st.median(r['copy'] for r in v) / 1e3:.2f} ms")
