#!/usr/bin/env python3
"""Do a compute-bound GEMM and the HBM-bound optimizer stream overlap when launched on two streams?

Toy-MLP backward pieces (batch 512, H 4096): wgrad / dgrad of the 4096x4096 layer and the SGD stream
of the 4096x3072 layer.  Each case is timed alone, back-to-back on one stream, and concurrently on two
streams (fork/join with events), eagerly and inside a captured HIP graph.  If "concurrent" approaches
max(alone) instead of sum(alone), scheduling the backward as two branches pays.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.sgd_bw import timeit  # noqa: E402
from ddpx.ops import gemm as G  # noqa: E402
from ddpx.ops.elementwise import sgd_flat_  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    B, H, D = 512, 4096, 3072
    lr = torch.full((), 0.01, device=dev)
    dy = (torch.randn(B, H, device=dev) * 0.1).to(torch.bfloat16)
    h1 = torch.randn(B, H, device=dev).to(torch.bfloat16)
    w1 = (torch.randn(H, H, device=dev) * 0.01).to(torch.bfloat16)
    out_bf = torch.empty(H, H, dtype=torch.bfloat16, device=dev)
    n0 = H * D
    p0 = torch.randn(n0, device=dev) * 0.01
    m0 = torch.zeros(n0, device=dev)
    s0 = torch.empty(n0, dtype=torch.bfloat16, device=dev)
    g0 = torch.zeros(n0, dtype=torch.float32, device=dev)
    n1 = H * H
    p1 = torch.randn(n1, device=dev) * 0.01
    m1 = torch.zeros(n1, device=dev)
    s1 = torch.empty(n1, dtype=torch.bfloat16, device=dev)

    cases = {
        "wgrad1_bf16": lambda: G.linear_wgrad(dy, h1, out_bf),
        "dgrad1": lambda: G.linear_dgrad(dy, w1),
        "sgd0_stream": lambda: sgd_flat_(p0, m0, g0, s0, lr, 0.9, 5e-4),
        "wgrad1_fused_sgd": lambda: G.linear_wgrad(dy, h1, None, sgd=(p1, m1, s1, lr, 0.9, 5e-4)),
    }
    res = {k: timeit(f, reps=7, inner=5) for k, f in cases.items()}
    side = torch.cuda.Stream()

    def pair(a, b):
        def run():
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            a()
            with torch.cuda.stream(side):
                b()
            cur.wait_stream(side)
        return run

    def serial(a, b):
        def run():
            a()
            b()
        return run

    for x, y in (("wgrad1_bf16", "sgd0_stream"), ("dgrad1", "wgrad1_fused_sgd"), ("dgrad1", "sgd0_stream")):
        res[f"{x}+{y}_serial"] = timeit(serial(cases[x], cases[y]), reps=7, inner=5)
        res[f"{x}+{y}_2streams"] = timeit(pair(cases[x], cases[y]), reps=7, inner=5)
        # same pair inside a captured graph (branches as two parallel graph nodes)
        g = torch.cuda.CUDAGraph()
        fn = pair(cases[x], cases[y])
        fn()
        torch.cuda.synchronize()
        with torch.cuda.graph(g):
            fn()
        res[f"{x}+{y}_graph"] = timeit(g.replay, reps=7, inner=5)
    print(json.dumps(res, indent=1))
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/overlap_probe.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
