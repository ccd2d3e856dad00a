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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--min_bytes", type=int, default=1 << 16)
    ap.add_argument("--max_bytes", type=int, default=1 << 28)
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--iters", type=int, default=20)
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
    comm = RcclComm(dev)
    dt = torch.bfloat16 if a.dtype == "bf16" else torch.float32
    esz = torch.tensor([], dtype=dt).element_size()
    rows = []
    nbytes = a.min_bytes
    while nbytes <= a.max_bytes:
        n = nbytes // esz // world * world
        buf = torch.randn(n, device=dev).to(dt)
        shard = buf[rank * (n // world):(rank + 1) * (n // world)]
        ops = {
            "all_reduce": (lambda: comm.allreduce_(buf, "avg", stream=comm.stream), 2.0 * (world - 1) / world),
            "reduce_scatter": (lambda: comm.reduce_scatter(shard, buf, "avg", stream=comm.stream),
                               (world - 1) / world),
            "all_gather": (lambda: comm.allgather(buf, shard, stream=comm.stream), (world - 1) / world),
        }
        for name, (fn, factor) in ops.items():
            for _ in range(3):
                fn()
            torch.cuda.synchronize()
            dist.barrier()
            s = torch.cuda.Event(enable_timing=True)
            e = torch.cuda.Event(enable_timing=True)
            s.record(comm.stream)
            for _ in range(a.iters):
                fn()
            e.record(comm.stream)
            e.synchronize()
            t_us = s.elapsed_time(e) * 1000.0 / a.iters
            busbw = (n * esz) / (t_us * 1e-6) * factor / 1e9 if world > 1 else 0.0
            rows.append({"op": name, "bytes": n * esz, "us": round(t_us, 2), "busbw_GBps": round(busbw, 1)})
        nbytes *= 4
    comm.check()
    if rank == 0:
        print(f"{'op':15s} {'bytes':>12s} {'us':>10s} {'busbw GB/s':>11s}   (world {world}, {a.dtype})")
        for r in rows:
            print(f"{r['op']:15s} {r['bytes']:12d} {r['us']:10.2f} {r['busbw_GBps']:11.1f}")
        if a.out:
            with open(a.out, "w") as f:
                json.dump({"world": world, "dtype": a.dtype, "rows": rows}, f, indent=1)
    torch.cuda.synchronize()
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
