#!/usr/bin/env python3
"""MX-FP8 vs bf16 GEMMs of the wide MLP (3072-16384-16384-10, batch 512; BASELINE config 5), per kernel.

    python benchmarks/fp8_gemm_table.py [--out FILE]

Each product is timed as a HIP graph of back-to-back launches (host launch cost out), interleaved rounds in one
process, median microseconds.  fp8 operands are quantised once outside the timed region (the step produces them
in the kernels that write the activations / weights); the quantisation passes are timed separately.

products (M x N x K):
  fc1 fwd    512 x 16384 x 16384   Y = X W^T            (bf16: linear_fwd;      fp8: MX A=X rows, B=W rows)
  fc0 fwd    512 x 16384 x 3072
  fc1 dgrad  512 x 16384 x 16384   dX = dY W            (bf16: linear_dgrad;    fp8: A=dY rows, B=W^T blocks on out)
  fc1 wgrad  16384 x 16384 x 512   dW = dY^T X (fp32)   (bf16: linear_wgrad;    fp8: A=dY^T, B=X^T)
  fc0 wgrad  16384 x 3072 x 512
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import fp8 as F8  # noqa: E402
from ddpx.ops import gemm as G  # noqa: E402


def graph_of(fn, inner):
    fn()
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(inner):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    return g


def time_graph(g, inner, reps=5):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000 / inner)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--inner", type=int, default=5)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    bf = torch.bfloat16
    B, D0, H = 512, 3072, 16384
    x = torch.rand(B, D0, device=dev).to(bf)
    h1 = torch.relu(torch.randn(B, H, device=dev)).to(bf)
    w0 = (torch.randn(H, D0, device=dev) * 0.02).to(bf)
    w1 = (torch.randn(H, H, device=dev) * 0.01).to(bf)
    b0, b1 = torch.randn(H, device=dev), torch.randn(H, device=dev)
    dy = (torch.randn(B, H, device=dev) * 0.01).to(bf)
    out_bf = torch.empty(B, H, dtype=bf, device=dev)
    dw1 = torch.empty(H, H, device=dev)
    dw0 = torch.empty(H, D0, device=dev)
    # fp8 operands
    xq, xqt = F8.quant(x, F8.E4M3, rows=True, cols=True)
    hq, hqt = F8.quant(h1, F8.E4M3, rows=True, cols=True)
    w0q = F8.quant(w0, F8.E4M3)
    w1q = F8.quant(w1, F8.E4M3)
    w1qt = F8.quant(w1, F8.E4M3, rows=False, cols=True)  # W1^T [in][out], blocks along out (dgrad's K)
    dyq = F8.quant(dy, F8.E4M3)
    dyqt = F8.quant(dy, F8.E4M3, rows=False, cols=True)  # dY^T [out][batch]
    cases = {
        "fc1_fwd_bf16": lambda: G.linear_fwd(h1, w1, b1, relu=True, out=out_bf),
        "fc1_fwd_mx8": lambda: F8.gemm(hq, w1q, out=out_bf, epi=G.EPI_BIAS_RELU_BF16, bias=b1),
        "fc0_fwd_bf16": lambda: G.linear_fwd(x, w0, b0, relu=True, out=out_bf),
        "fc0_fwd_mx8": lambda: F8.gemm(xq, w0q, out=out_bf, epi=G.EPI_BIAS_RELU_BF16, bias=b0),
        "fc1_dgrad_bf16": lambda: G.linear_dgrad(dy, w1, relu_mask_of=h1, out=out_bf),
        "fc1_dgrad_mx8": lambda: F8.gemm(dyq, w1qt, out=out_bf, epi=G.EPI_RELUMASK_BF16, aux=h1),
        "fc1_wgrad_bf16": lambda: G.linear_wgrad(dy, h1, dw1),
        "fc1_wgrad_mx8": lambda: F8.gemm(dyqt, hqt, out=dw1, epi=G.EPI_F32),
        "fc0_wgrad_bf16": lambda: G.linear_wgrad(dy, x, dw0),
        "fc0_wgrad_mx8": lambda: F8.gemm(dyqt, xqt, out=dw0, epi=G.EPI_F32),
        "quant_rows_dy": lambda: F8.quant(dy, F8.E4M3),
        "quant_rows_cols_h1": lambda: F8.quant(h1, F8.E4M3, rows=True, cols=True),
        "quant_cols_w1": lambda: F8.quant(w1, F8.E4M3, rows=False, cols=True),
    }
    flops = {"fc1_fwd": 2 * B * H * H, "fc0_fwd": 2 * B * H * D0, "fc1_dgrad": 2 * B * H * H,
             "fc1_wgrad": 2 * B * H * H, "fc0_wgrad": 2 * B * H * D0}
    graphs = {k: graph_of(f, a.inner) for k, f in cases.items()}
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, g in graphs.items():
            res[k].append(time_graph(g, a.inner))
    out = {}
    for k, v in res.items():
        us = sorted(v)[len(v) // 2]
        base = k.rsplit("_", 1)[0]
        row = {"us": round(us, 2)}
        if base in flops:
            row["pflops"] = round(flops[base] / us / 1e9, 3)
        out[k] = row
        print(f"{k:22s} {us:9.2f} us" + (f"  {row['pflops']:.3f} PF/s" if "pflops" in row else ""), flush=True)
    for base in flops:
        if f"{base}_bf16" in out and f"{base}_mx8" in out:
            sp = out[f"{base}_bf16"]["us"] / out[f"{base}_mx8"]["us"]
            out[f"{base}_speedup"] = round(sp, 3)
            print(f"{base:22s} mx8 speed-up {sp:.3f}x", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
