#!/usr/bin/env python3
"""RCCL protocol x channel sweep at the toy MLP's bucket sizes.

    python benchmarks/rccl_sweep.py --nproc 8 [--protos default,Simple,LL128,LL] [--channels 0,4,8,16,32]
                                    [--dtype fp32] [--out gpurun_out/rccl_sweep.json]

RCCL reads ``NCCL_PROTO`` once per process, so every protocol gets its own ``torch.distributed.run`` job
(a child process, one rank per GPU); inside a job every channel setting gets its own communicator
(``ncclConfig_t.minCTAs/maxCTAs`` through ``RcclComm(channels=...)``).  Sizes: the DDP buckets of the toy MLP
(fp32 gradients: 1 MB head/bias bucket, 48.0 MB fc0, 64.2 MB fc1), all-reduce for the replicated plan,
reduce-scatter + all-gather for ZeRO-1.  The winner per (op, size) is printed; pass it to ``bench.py`` /
``multigpu.py`` as ``--rccl_proto`` / ``--rccl_channels``.

On a fully connected 8 x MI355X node each ring channel drives one xGMI link direction (7 links per GPU): fewer
than 7 channels leave links idle on the large buckets, while every channel is a CU taken from the backward GEMMs
the collectives overlap.  LL / LL128 trade bandwidth for latency and only pay on the small head bucket.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))


def free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def best_rows(rows):
    """(op, bytes) -> the fastest row."""
    best = {}
    for r in rows:
        k = (r["op"], r["bytes"])
        if k not in best or r["us"] < best[k]["us"]:
            best[k] = r
    return best


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nproc", type=int, default=8)
    ap.add_argument("--protos", default="default,Simple,LL128,LL")
    ap.add_argument("--channels", default="0,4,8,16,32")
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--sizes", default="toy")
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--timeout", type=float, default=600.0, help="per-protocol job limit (seconds)")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    rows = []
    for proto in a.protos.split(","):
        env = dict(os.environ)
        env.pop("NCCL_PROTO", None)
        if proto != "default":
            env["NCCL_PROTO"] = proto
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        with tempfile.NamedTemporaryFile(suffix=".json", delete=False) as f:
            tmp = f.name
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.nproc}",
               "--master-addr", "127.0.0.1", "--master-port", str(free_port()),
               os.path.join(HERE, "rccl_bench.py"), "--sizes", a.sizes, "--dtype", a.dtype,
               "--channels", a.channels, "--iters", str(a.iters), "--out", tmp]
        print(f"[sweep] NCCL_PROTO={proto}: {' '.join(cmd[3:])}", flush=True)
        rc = subprocess.call(cmd, env=env, timeout=a.timeout)
        if rc != 0:
            print(f"[sweep] protocol {proto} failed (exit {rc}); stopping", flush=True)
            break
        with open(tmp) as f:
            rows += json.load(f)["rows"]
        os.unlink(tmp)
    best = best_rows(rows)
    print(f"\n{'op':15s} {'bytes':>12s}  best: {'proto':>8s} {'chan':>6s} {'us':>9s} {'busbw':>7s}   default us")
    for (op, nb), r in sorted(best.items()):
        dflt = [x["us"] for x in rows if x["op"] == op and x["bytes"] == nb and x["proto"] == "default"
                and x["channels"] == "0"]
        print(f"{op:15s} {nb:12d}        {r['proto']:>8s} {r['channels']:>6s} {r['us']:9.1f} {r['busbw_GBps']:7.1f}"
              f"   {dflt[0] if dflt else float('nan'):9.1f}")
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"nproc": a.nproc, "dtype": a.dtype, "rows": rows,
                       "best": [dict(r) for r in best.values()]}, f, indent=1)


if __name__ == "__main__":
    main()
