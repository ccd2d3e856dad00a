#!/usr/bin/env python3
"""Per-dispatch view of one training step from a rocprofv3 kernel trace.

    python tools/trace_step.py TRACE_CSV [--marker augment] [--steps 3]

Splits the dispatch sequence at every kernel whose name contains ``--marker`` (the batch augment kernel
starts each ddpx step), and prints the last ``--steps`` complete steps as (order, kernel, us), plus the median
duration of every position over all complete steps.  Used for the per-layer VGG breakdowns in profiles/.
"""
import argparse
import csv
import re
import statistics


def short(name):
    name = re.sub(r"\.kd$", "", name)
    m = re.match(r"_ZN4ddpx(.*)", name)
    if m:
        # strip the mangling enough to read: namespace::kernel<template args>
        s = m.group(1)
        parts = []
        while s and s[0].isdigit():
            n = int(re.match(r"\d+", s).group(0))
            d = len(str(n))
            parts.append(s[d:d + n])
            s = s[d + n:]
        tmpl = re.findall(r"Li(-?\d+)E|Lb([01])E", s)
        args = ",".join(a or b for a, b in tmpl)
        return "::".join(parts) + (f"<{args}>" if args else "")
    return name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="augment")
    ap.add_argument("--steps", type=int, default=1)
    ap.add_argument("--exclude", default=None, help="drop steps containing a kernel with this substring")
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    steps, cur = [], None
    for s, e, n in rows:
        if a.marker in n:
            if cur:
                steps.append(cur)
            cur = []
        if cur is not None:
            cur.append((short(n), (e - s) / 1000.0))
    if a.exclude:
        steps = [st for st in steps if not any(a.exclude in k for k, _ in st)]
    if not steps:
        print("no complete step found")
        return
    L = len(steps[-1])
    same = [st for st in steps if len(st) == L and [k for k, _ in st] == [k for k, _ in steps[-1]]]
    print(f"{len(steps)} steps, {len(same)} with the last step's dispatch sequence ({L} kernels)")
    tot = 0.0
    for i, (k, _) in enumerate(steps[-1]):
        med = statistics.median(st[i][1] for st in same)
        tot += med
        print(f"{i:3d} {med:9.1f} us  {k}")
    print(f"sum of medians {tot:.1f} us")


if __name__ == "__main__":
    main()
