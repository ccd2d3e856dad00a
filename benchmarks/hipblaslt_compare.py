"""The toy MLP's M = 512 GEMMs on hipBLASLt (torch) vs the ddpx pipe core, same process, graph-captured.

    python benchmarks/hipblaslt_compare.py

hipBLASLt cases: plain bf16 GEMM (`x @ w.t()`), the fused bias+ReLU epilogue (`torch._addmm_activation`),
and the data gradient `dy @ w`.  ddpx cases: the bias+ReLU forward and the ReLU-masked data gradient the step
actually runs.  Prints {case: median us}.
"""
from __future__ import annotations

import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import gemm as G  # noqa: E402


def timeit(fn, inner=20, reps=7):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(inner):
            fn()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0 / inner)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    B, I, H = 512, 3072, 4096
    x = (torch.rand(B, I, device=dev) * 2 - 1).to(torch.bfloat16)
    h1 = torch.relu(torch.randn(B, H, device=dev)).to(torch.bfloat16)
    w0 = (torch.randn(H, I, device=dev) * 0.02).to(torch.bfloat16)
    w1 = (torch.randn(H, H, device=dev) * 0.02).to(torch.bfloat16)
    b0 = torch.randn(H, device=dev) * 0.1
    b0h = b0.to(torch.bfloat16)
    dy = (torch.randn(B, H, device=dev) * 0.01).to(torch.bfloat16)
    row = {
        "hipblaslt_fc0_gemm": timeit(lambda: x @ w0.t()),
        "hipblaslt_fc0_bias_relu": timeit(lambda: torch._addmm_activation(b0h, x, w0.t())),
        "ddpx_fc0_bias_relu": timeit(lambda: G.linear_fwd(x, w0, b0, relu=True)),
        "hipblaslt_fc1_gemm": timeit(lambda: h1 @ w1.t()),
        "hipblaslt_fc1_bias_relu": timeit(lambda: torch._addmm_activation(b0h, h1, w1.t())),
        "ddpx_fc1_bias_relu": timeit(lambda: G.linear_fwd(h1, w1, b0, relu=True)),
        "hipblaslt_dgrad_gemm": timeit(lambda: dy @ w1),
        "ddpx_dgrad_relumask": timeit(lambda: G.linear_dgrad(dy, w1, relu_mask_of=h1)),
    }
    print(json.dumps(row, indent=1))


if __name__ == "__main__":
    main()
