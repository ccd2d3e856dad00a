#!/usr/bin/env python3
"""rccl-tests-style microbenchmark of the ddpx native communicator.

    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 benchmarks/rccl_bench.py --out gpurun_out/rccl.json

For each collective (all-reduce, reduce-scatter, all-gather) and message size it reports the
time per call and the bus bandwidth as rccl-tests defines it:

    all-reduce     busbw = bytes / t * 2 (n-1) / n
    reduce-scatter busbw = bytes / t * (n-1) / n      (bytes = full input)
    all-gather     busbw = bytes / t * (n-1) / n      (bytes = full output)

which is what the DDP bucket size and the ZeRO-1 reduce-scatter / all-gather pair are tuned
against (7 xGMI links per MI355X).  Collectives run on the communicator's own high-priority
stream exactly as the DDP reducer issues them.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


# the toy MLP's DDP buckets (fp32 gradients): head weight + biases, fc0 weight (48.0 MB), fc1 weight (64.2 MB)
TOY_BUCKETS = [1 << 20, 12582912 * 4, 16777216 * 4]


def sizes_of(a):
    if a.sizes == "toy":
        return list(TOY_BUCKETS)
    if a.sizes:
        return [int(float(v)) for v in a.sizes.split(",")]
    out, n = [], a.min_bytes
    while n <= a.max_bytes:
        out.append(n)
        n *= 4
    return out


def time_ops(comm, world, rank, dev, dt, esz, nbytes, iters, ops_wanted):
    n = nbytes // esz // world * world
    buf = torch.randn(n, device=dev).to(dt)
    shard = buf[rank * (n // world):(rank + 1) * (n // world)]
    ops = {
        "all_reduce": (lambda: comm.allreduce_(buf, "avg", stream=comm.stream), 2.0 * (world - 1) / world),
        "reduce_scatter": (lambda: comm.reduce_scatter(shard, buf, "avg", stream=comm.stream),
                           (world - 1) / world),
        "all_gather": (lambda: comm.allgather(buf, shard, stream=comm.stream), (world - 1) / world),
    }
    rows = []
    for name, (fn, factor) in ops.items():
        if name not in ops_wanted:
            continue
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        dist.barrier()
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record(comm.stream)
        for _ in range(iters):
            fn()
        e.record(comm.stream)
        e.synchronize()
        t_us = s.elapsed_time(e) * 1000.0 / iters
        # the slowest rank's time is the collective's time
        t = torch.tensor([t_us], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        t_us = float(t[0])
        busbw = (n * esz) / (t_us * 1e-6) * factor / 1e9 if world > 1 else 0.0
        rows.append({"op": name, "bytes": n * esz, "us": round(t_us, 2), "busbw_GBps": round(busbw, 1)})
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min_bytes", type=int, default=1 << 16)
    ap.add_argument("--max_bytes", type=int, default=1 << 28)
    ap.add_argument("--sizes", default=None, help="comma list of message bytes, or 'toy' (the toy MLP's buckets)")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--ops", default="all_reduce,reduce_scatter,all_gather")
    ap.add_argument("--channels", default="0",
                    help="comma list of channel bounds, one communicator each: 0 (RCCL's choice), N, or MIN:MAX")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    from ddpx.parallel.comm import RcclComm
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    if "MASTER_PORT" not in os.environ:
        import socket
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            os.environ["MASTER_PORT"] = str(s.getsockname()[1])
    torch.cuda.set_device(local)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    dev = torch.device("cuda", local)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    esz = torch.tensor([], dtype=dt).element_size()
    ops_wanted = set(a.ops.split(","))
    proto = os.environ.get("NCCL_PROTO", "default")
    rows = []
    for ch in a.channels.split(","):
        comm = RcclComm(dev, channels=ch if ch not in ("0", "") else "")
        for nbytes in sizes_of(a):
            for r in time_ops(comm, world, rank, dev, dt, esz, nbytes, a.iters, ops_wanted):
                r.update(channels=ch, proto=proto)
                rows.append(r)
        comm.check()
        torch.cuda.synchronize()
        comm.close()
    if rank == 0:
        print(f"{'op':15s} {'proto':>8s} {'chan':>6s} {'bytes':>12s} {'us':>10s} {'busbw GB/s':>11s}   "
              f"(world {world}, {a.dtype})")
        for r in rows:
            print(f"{r['op']:15s} {r['proto']:>8s} {r['channels']:>6s} {r['bytes']:12d} {r['us']:10.2f} "
                  f"{r['busbw_GBps']:11.1f}")
        if a.out:
            with open(a.out, "w") as f:
                json.dump({"world": world, "dtype": a.dtype, "rows": rows}, f, indent=1)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
