#!/usr/bin/env python3
"""Per-kernel HBM traffic from separate rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes.

usage: pmc_per_kernel.py <fetch_dir> <write_dir> <dispatches_per_kernel_divisor> [label]

Both counters are KiB per dispatch (summed over the TCC instances by rocprofv3); FETCH_SIZE is
doubled as MI355X_MICROARCH.md prescribes for gfx950 (calibrated for 16-B/lane streaming reads).
The divisor is the number of bench steps the child ran (warmup + timed), so the figures are per step.
"""
import collections
import csv
import glob
import os
import sys


def load(d, ctr):
    acc = collections.defaultdict(float)
    cnt = collections.Counter()
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row["Counter_Name"] != ctr:
                continue
            k = row["Kernel_Name"].split("(")[0]
            acc[k] += float(row["Counter_Value"])
            cnt[k] += 1
    return acc, cnt


def main():
    fd, wd, div = sys.argv[1], sys.argv[2], float(sys.argv[3])
    label = sys.argv[4] if len(sys.argv) > 4 else ""
    fa, fc = load(fd, "FETCH_SIZE")
    wa, _ = load(wd, "WRITE_SIZE")
    names = sorted(set(fa) | set(wa), key=lambda k: -(fa.get(k, 0) * 2 + wa.get(k, 0)))
    print(f"# per-step HBM traffic by kernel {label} (FETCH x2, KiB->bytes; {div:g} steps per pass)")
    print(f"{'kernel':48s} {'disp/step':>9s} {'fetch MB':>10s} {'write MB':>10s} {'total MB':>10s}")
    tf = tw = 0.0
    for k in names:
        f = fa.get(k, 0) * 1024 * 2 / div
        w = wa.get(k, 0) * 1024 / div
        tf += f
        tw += w
        print(f"{k[:48]:48s} {fc.get(k, 0) / div:9.1f} {f / 1e6:10.1f} {w / 1e6:10.1f} {(f + w) / 1e6:10.1f}")
    print(f"{'TOTAL':48s} {'':9s} {tf / 1e6:10.1f} {tw / 1e6:10.1f} {(tf + tw) / 1e6:10.1f}")


if __name__ == "__main__":
    main()
