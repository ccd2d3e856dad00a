"""Per-kernel statistics from a rocprofv3 ``*_results.db`` (rocpd SQLite): calls, total / mean time, share.

    python tools/rocpd_stats.py gpurun_out/f32/prof/vgg_results.db [--csv out.csv] [--top 40] [--grid]

``--grid`` adds the grid / workgroup sizes and VGPR counts of each kernel symbol (tile and occupancy
checks).  Used to commit kernel tables under ``profiles/``.
"""
from __future__ import annotations

import argparse
import csv
import sqlite3


def kernel_stats(db: str, with_grid: bool = False):
    c = sqlite3.connect(db)
    q = ("select s.kernel_name, count(*), sum(d.end - d.start), min(d.end - d.start), max(d.end - d.start), "
         "max(d.grid_size_x), max(d.workgroup_size_x), max(s.arch_vgpr_count), max(s.accum_vgpr_count), "
         "max(d.group_segment_size) "
         "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id "
         "group by s.kernel_name order by sum(d.end - d.start) desc")
    rows = list(c.execute(q))
    total = sum(r[2] for r in rows) or 1
    out = []
    for name, n, tot, mn, mx, grid, wg, vgpr, agpr, lds in rows:
        d = {"kernel": name, "calls": n, "total_us": round(tot / 1e3, 1), "mean_us": round(tot / n / 1e3, 2),
             "min_us": round(mn / 1e3, 2), "max_us": round(mx / 1e3, 2), "pct": round(100.0 * tot / total, 2)}
        if with_grid:
            d.update({"grid": grid, "wg": wg, "vgpr": vgpr, "agpr": agpr, "lds": lds})
        out.append(d)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--csv")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--grid", action="store_true")
    a = ap.parse_args()
    rows = kernel_stats(a.db, a.grid)
    for r in rows[:a.top]:
        extra = f" grid={r['grid']} wg={r['wg']} v={r['vgpr']} a={r['agpr']} lds={r['lds']}" if a.grid else ""
        print(f"{r['pct']:6.2f}% {r['total_us']:10.1f}us {r['calls']:5d}x {r['mean_us']:9.2f}us  "
              f"{r['kernel'][:110]}{extra}")
    if a.csv:
        with open(a.csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=list(rows[0].keys()))
            w.writeheader()
            w.writerows(rows)


if __name__ == "__main__":
    main()
