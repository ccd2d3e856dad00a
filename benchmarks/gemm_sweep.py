#!/usr/bin/env python3
"""Time every ddpx GEMM tile config against hipBLASLt (torch.matmul) on the MLP shapes.

    python benchmarks/gemm_sweep.py [--hidden 4096] [--batch 512] [--out gpurun_out/gemm_sweep.json]

Shapes are the five products of one toy-MLP step (forward of layers 1-2, dgrad of
layer 2, wgrad of layers 1-2) in their real operand layouts.  Random data
(uniform [-1,1) bf16): zero-filled operands would inflate MFMA clocks.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import gemm as G  # noqa: E402


def timeit(fn, iters=50, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--hidden", type=int, default=4096)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--inp", type=int, default=3072)
    ap.add_argument("--out", default=None)
    ap.add_argument("--cfgs", default="0,1,2,3,4,5,6,7", help="comma-separated tile configs")
    ap.add_argument("--cases", default="", help="comma-separated subset of fwd1,fwd2,dgrad2,wgrad1,wgrad2")
    ap.add_argument("--iters", type=int, default=50)
    a = ap.parse_args()
    cfgs = [int(c) for c in a.cfgs.split(",") if c.strip()]
    dev = torch.device("cuda", 0)
    B, H, I = a.batch, a.hidden, a.inp

    def rnd(*s):
        return (torch.rand(*s, device=dev) * 2 - 1).to(torch.bfloat16)

    x, h1 = rnd(B, I), rnd(B, H)
    w1, w2 = rnd(H, I), rnd(H, H)
    b = torch.randn(H, device=dev)
    dy = rnd(B, H)
    dw1, dw2 = torch.empty(H, I, device=dev), torch.empty(H, H, device=dev)
    dyT, h1T = dy.t().contiguous(), h1.t().contiguous()
    cases = {
        "fwd1": (2 * B * H * I, lambda t: G.gemm_raw(x, w1, torch.empty(B, H, dtype=torch.bfloat16, device=dev),
                 M=B, N=H, K=I, lda=I, ldb=I, ldc=H, a_kcontig=True, b_kcontig=True, epi=G.EPI_BIAS_RELU_BF16,
                 bias=b, tile=t), lambda: torch.relu(torch.nn.functional.linear(x, w1, b.to(torch.bfloat16)))),
        "fwd2": (2 * B * H * H, lambda t: G.gemm_raw(h1, w2, torch.empty(B, H, dtype=torch.bfloat16, device=dev),
                 M=B, N=H, K=H, lda=H, ldb=H, ldc=H, a_kcontig=True, b_kcontig=True, epi=G.EPI_BIAS_RELU_BF16,
                 bias=b, tile=t), lambda: torch.relu(torch.nn.functional.linear(h1, w2, b.to(torch.bfloat16)))),
        "dgrad2": (2 * B * H * H, lambda t: G.gemm_raw(dy, w2, torch.empty(B, H, dtype=torch.bfloat16, device=dev),
                   M=B, N=H, K=H, lda=H, ldb=H, ldc=H, a_kcontig=True, b_kcontig=False, epi=G.EPI_RELUMASK_BF16,
                   aux=h1, ldaux=H, tile=t), lambda: (dy @ w2) * (h1 > 0)),
        "wgrad1": (2 * B * H * I, lambda t: G.gemm_raw(dy, x, dw1, M=H, N=I, K=B, lda=H, ldb=I, ldc=I,
                   a_kcontig=False, b_kcontig=False, epi=G.EPI_F32, tile=t), lambda: dy.t() @ x),
        "wgrad2": (2 * B * H * H, lambda t: G.gemm_raw(dy, h1, dw2, M=H, N=H, K=B, lda=H, ldb=H, ldc=H,
                   a_kcontig=False, b_kcontig=False, epi=G.EPI_F32, tile=t), lambda: dy.t() @ h1),
        # the same weight gradient from K-contiguous (transposed) copies of dY and X: the forward GEMMs' layout
        "wgrad2kk": (2 * B * H * H, lambda t: G.gemm_raw(dyT, h1T, dw2, M=H, N=H, K=B, lda=B, ldb=B, ldc=H,
                     a_kcontig=True, b_kcontig=True, epi=G.EPI_F32, tile=t), lambda: dy.t() @ h1),
    }
    res = {}
    want = [c for c in a.cases.split(",") if c] or list(cases)
    for name, (flop, ours, ref) in cases.items():
        if name not in want:
            continue
        row = {}
        t = timeit(ref, iters=a.iters)
        row["hipblaslt"] = round(t, 2)
        r = ref().float()
        for cfg in cfgs:
            row[f"pipe{cfg}"] = round(timeit(lambda: ours(cfg), iters=a.iters), 2)
            err = ((ours(cfg).float() - r).norm() / r.norm()).item()
            if err > 2e-2:
                row[f"pipe{cfg}_ERR"] = err
        best = min((v, k) for k, v in row.items() if k != "hipblaslt")
        row["best"] = best[1]
        row["best_tflops"] = round(flop / best[0] / 1e6, 1)
        row["hipblaslt_tflops"] = round(flop / row["hipblaslt"] / 1e6, 1)
        res[name] = row
        print(name, json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"batch": B, "hidden": H, "inp": I, "us": res}, f, indent=1)


if __name__ == "__main__":
    main()
