#!/usr/bin/env python3
"""Run ONE GEMM configuration repeatedly (for rocprofv3 --pmc counter collection / kernel timing).

    rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... -d DIR -- python3 benchmarks/kernel_probe.py --case fwd1_t7
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddpx.ops import gemm as G  # noqa: E402

CASES = ["fwd1_t7", "fwd1_t0", "fwd1_t8", "dgrad1_t3", "wgrad1_t5", "wgrad1_t8", "wgrad1sgd_t5", "mx8_fwd_wide",
         "mx8_wgrad_wide", "bf16_fwd_wide"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", required=True,
                    help="one of CASES, or KIND_tT with KIND in fwd0 (fc0: K = 3072) / fwd1 / dgrad1 / wgrad1 / "
                         "wgrad1sgd and T a dispatch tile (-1: the default plan)")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M, H = 512, 4096
    c = a.case
    if c.startswith("mx8") or c.startswith("bf16_fwd_wide"):
        from ddpx.ops import fp8 as F8
        H = 16384
        x = torch.randn(M, H, device=dev).to(torch.bfloat16)
        w = (torch.randn(H, H, device=dev) * 0.01).to(torch.bfloat16)
        b = torch.randn(H, device=dev)
        if c == "mx8_fwd_wide":
            xq, wq = F8.quant(x), F8.quant(w)
            fn = lambda: F8.gemm(xq, wq, epi=G.EPI_BIAS_RELU_BF16, bias=b)  # noqa: E731
        elif c == "mx8_wgrad_wide":
            dq = F8.quant(x, rows=False, cols=True)
            hq = F8.quant(x, rows=False, cols=True)
            out = torch.empty(H, H, dtype=torch.bfloat16, device=dev)
            fn = lambda: F8.gemm(dq, hq, out=out, epi=G.EPI_BF16)  # noqa: E731
        else:
            fn = lambda: G.linear_fwd(x, w, b, relu=True)  # noqa: E731
    else:
        kind, tile = c.split("_t")
        tile = int(tile)
        K = 3072 if kind == "fwd0" else H
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(H, K, device=dev) * 0.02).to(torch.bfloat16)
        b = torch.randn(H, device=dev)
        dy = torch.randn(M, H, device=dev).to(torch.bfloat16)
        if kind in ("fwd0", "fwd1"):
            # tile -1: the default plan (in-launch split-K on 128x128 tiles for this shape)
            fn = lambda: G.linear_fwd(x, w, b, relu=True, tile=tile)  # noqa: E731
        elif kind == "dgrad1":
            fn = lambda: G.linear_dgrad(dy, w, relu_mask_of=x, tile=tile)  # noqa: E731
        elif kind == "wgrad1":
            out = torch.empty(H, H, dtype=torch.bfloat16, device=dev)
            fn = lambda: G.linear_wgrad(dy, x, out, tile=tile)  # noqa: E731
        else:
            p = torch.randn(H * H, device=dev) * 0.01
            mb = torch.zeros(H * H, device=dev)
            sh = torch.empty(H * H, dtype=torch.bfloat16, device=dev)
            lr = torch.full((), 0.01, device=dev)
            fn = lambda: G.linear_wgrad(dy, x, None, tile=tile, sgd=(p, mb, sh, lr, 0.9, 5e-4))  # noqa: E731
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()


if __name__ == "__main__":
    main()
