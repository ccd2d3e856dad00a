#!/usr/bin/env python3
"""Per-dispatch view of one training step from a rocprofv3 kernel trace.

    python tools/trace_step.py TRACE_CSV [--marker augment] [--steps 3]

Splits the dispatch sequence at every kernel whose name contains ``--marker`` (the batch augment kernel
starts each ddpx step) and prints the step's dispatch sequence with the median duration of every position.
The step shown is the MODAL one — the dispatch sequence most segments share (the graph-replayed training
step) — not the last segment: a segment that ends at the next marker can also hold whatever ran between two
steps (round 4's VGG table took the segment before the stock recipe's first augment, so it showed the bench's
digest copies and the stock model's initialisation kernels as part of a step).  Segments
with any other sequence are counted and listed by kernel count, never mixed into the medians.
Used for the per-layer breakdowns in profiles/.
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
    from collections import Counter
    sigs = Counter(tuple(k for k, _ in st) for st in steps)
    modal, count = sigs.most_common(1)[0]
    same = [st for st in steps if tuple(k for k, _ in st) == modal]
    others = sorted(len(sig) for sig in sigs if sig != modal)
    print(f"{len(steps)} segments; the modal dispatch sequence ({len(modal)} kernels) in {count} of them; "
          f"{len(steps) - count} other segments (kernel counts {others}) excluded")
    tot = 0.0
    for i, k in enumerate(modal):
        med = statistics.median(st[i][1] for st in same)
        tot += med
        print(f"{i:3d} {med:9.1f} us  {k}")
    print(f"sum of medians {tot:.1f} us")


if __name__ == "__main__":
    main()
