"""Cost of the wide MLP's MX-FP8 weight copy: written by the fused weight-gradient + SGD pair's stream waves
vs a separate quantiser pass over the bf16 copy (the fp8 forward's per-step weight operand).

    python benchmarks/fp8_copy_bench.py [--hidden 16384]

Median microseconds of 20 back-to-back launches (CUDA events) for: the pair without / with the fp8 outputs,
and the two weight quantisations it replaces.
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    ts.sort()
    return round(ts[len(ts) // 2], 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=16384)
    ap.add_argument("--inp", type=int, default=3072)
    ap.add_argument("--batch", type=int, default=512)
    a = ap.parse_args()
    from ddpx.ops import fp8 as F8
    from ddpx.ops import gemm as G
    dev = torch.device("cuda", 0)
    H, I, B = a.hidden, a.inp, a.batch
    torch.manual_seed(0)
    shapes = [(H, H), (H, I)]  # (out, in): fc1, fc0
    dys = [((torch.rand(B, m, device=dev) * 2 - 1) * 1e-3).to(torch.bfloat16) for m, _ in shapes]
    xs = [torch.rand(B, n, device=dev).to(torch.bfloat16) for _, n in shapes]
    lr = torch.full((), 1e-3, device=dev)
    st = [(torch.randn(m * n, device=dev) * 0.01, torch.zeros(m * n, device=dev),
           torch.empty(m * n, dtype=torch.bfloat16, device=dev)) for m, n in shapes]
    spec = [(p, b, s, lr, 0.9, 5e-4) for p, b, s in st]
    mx = [(torch.empty(m, n, dtype=torch.uint8, device=dev), torch.empty(m, n // 32, dtype=torch.uint8, device=dev))
          for m, n in shapes]
    row = {"pair_bf16_only_us": timeit(lambda: G.wgrad_sgd_pair(dys[0], xs[0], spec[0], dys[1], xs[1], spec[1])),
           "pair_with_fp8_us": timeit(lambda: G.wgrad_sgd_pair(dys[0], xs[0], spec[0], dys[1], xs[1], spec[1],
                                                               mx[0], mx[1])),
           "quant_both_weights_us": timeit(lambda: [F8.quant(s.view(m, n), F8.E4M3, out=q)
                                                    for (_, _, s), (m, n), q in zip(st, shapes, mx)])}
    row["fp8_copy_net_us"] = round(row["pair_with_fp8_us"] - row["pair_bf16_only_us"] - row["quant_both_weights_us"], 1)
    print(json.dumps(row))


if __name__ == "__main__":
    main()
