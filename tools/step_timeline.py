#!/usr/bin/env python3
"""One training step's kernel timeline from a rocprofv3 kernel-trace CSV.

Usage: python tools/step_timeline.py TRACE.csv [--anchor augment_kernel] [--nth -3] [--out FILE]

A step is the span between two consecutive launches of the anchor kernel (the batch gather that
opens every captured step).  Prints start offset, duration and name of every kernel in the chosen
step (``--nth``: index into the list of anchor launches; negative counts from the end) plus the
step's wall time and the sum of kernel durations.
"""
from __future__ import annotations

import argparse
import csv
import sys


def load(path):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            try:
                rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
            except (KeyError, ValueError):
                continue
    rows.sort()
    return rows


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--anchor", default="augment_kernel")
    ap.add_argument("--nth", type=int, default=-3)
    ap.add_argument("--out", default=None)
    a = ap.parse_args(argv)
    rows = load(a.trace)
    starts = [i for i, r in enumerate(rows) if a.anchor in r[2]]
    if len(starts) < 2:
        print("fewer than two anchor launches", file=sys.stderr)
        return 1
    k = a.nth if a.nth >= 0 else len(starts) - 1 + a.nth
    k = max(0, min(k, len(starts) - 2))
    i0, i1 = starts[k], starts[k + 1]
    t0 = rows[i0][0]
    lines = ["start_us dur_us kernel"]
    busy = 0
    for s, e, n in rows[i0:i1]:
        busy += e - s
        lines.append(f"{(s - t0) / 1e3:8.1f} {(e - s) / 1e3:7.1f}  {n[:110]}")
    wall = rows[i1][0] - t0
    lines.append(f"step wall {wall / 1e3:.1f} us, kernels {i1 - i0}, kernel time {busy / 1e3:.1f} us")
    txt = "\n".join(lines)
    print(txt)
    if a.out:
        with open(a.out, "w") as f:
            f.write(txt + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
