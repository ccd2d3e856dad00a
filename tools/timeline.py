#!/usr/bin/env python3
"""Kernel timeline of one training step from a rocprofv3 kernel trace (start offsets, durations, queues).

    python tools/timeline.py TRACE_CSV [--marker augment] [--skip 8] [--count 1]

Picks the ``--skip``-th complete step (segments between two ``--marker`` kernels, default: the batch augment
kernel that opens every ddpx step) and prints every kernel of it in start order: start offset from the step's
first kernel, duration, queue id, and gaps where no kernel ran.  Shows what overlaps (comm / optimizer side
streams next to backward) and where the GPU idles.
"""
import argparse
import csv

from trace_step import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--marker", default="augment")
    ap.add_argument("--skip", type=int, default=8)
    ap.add_argument("--count", type=int, default=1)
    a = ap.parse_args()
    rows = []
    with open(a.csv) as f:
        for r in csv.DictReader(f):
            q = r.get("Queue_Id") or r.get("Stream_Id") or "?"
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], q))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if a.marker in r[2]]
    if len(starts) < a.skip + a.count + 1:
        print(f"only {len(starts)} markers")
        return
    for n in range(a.count):
        i0, i1 = starts[a.skip + n], starts[a.skip + n + 1]
        seg = rows[i0:i1]
        t0 = seg[0][0]
        busy_end = t0
        print(f"step {a.skip + n}: {len(seg)} kernels, span {(rows[i1][0] - t0) / 1000:.1f} us to the next marker")
        for s, e, name, q in seg:
            gap = (s - busy_end) / 1000.0
            if gap > 1.0:
                print(f"{'':>9}   ... idle {gap:.1f} us")
            print(f"{(s - t0) / 1000:9.1f} {(e - s) / 1000:8.1f} us  q{q:<4} {short(name)[:90]}")
            busy_end = max(busy_end, e)


if __name__ == "__main__":
    main()
