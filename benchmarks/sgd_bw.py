#!/usr/bin/env python3
"""Optimizer-traffic microbenchmark: the toy MLP's per-step SGD is HBM-bound (18 B/param fused).

Times (HIP events, median of reps):
  * copy of the same bytes with torch (bandwidth reference),
  * ddpx_sgd_flat over all 29.4 M params (fp32 / bf16 grad),
  * wgrad GEMM alone (fp32 / bf16 out) and wgrad with the SGD epilogue, per tile config,
for the MLP's two big layers (fc0: 4096x3072, fc1: 4096x4096, batch 512).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import gemm as G
from ddpx.ops.elementwise import sgd_flat_


def timeit(fn, reps=20, inner=10):
    """Median over reps of (time of `inner` back-to-back calls) / inner, in µs: back-to-back launches
    keep the GPU busy, so host launch overhead does not inflate short kernels."""
    for _ in range(3):
        fn()
    ts = []
    for _ in range(reps):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(inner):
            fn()
        e.record()
        e.synchronize()
        ts.append(s.elapsed_time(e) * 1000 / inner)
    ts.sort()
    return round(ts[len(ts) // 2], 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    n = 4096 * 3072 + 4096 * 4096
    src = torch.empty(n * 18 // 8, dtype=torch.float64, device=dev)  # 18 B/param moved
    dst = torch.empty_like(src)
    res["copy_18Bpp_us"] = timeit(lambda: dst.copy_(src))
    res["copy_18Bpp_GBps"] = round(n * 18 * 2 / 2 / res["copy_18Bpp_us"] / 1e3, 1)
    p = torch.randn(n, device=dev) * 0.01
    buf = torch.zeros(n, device=dev)
    sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
    lr = torch.full((), 0.01, device=dev)
    for gd in (torch.float32, torch.bfloat16):
        g = (torch.randn(n, device=dev) * 1e-3).to(gd)
        t = timeit(lambda: sgd_flat_(p, buf, g, sh, lr, 0.9, 5e-4))
        bpp = 4 * 4 + 2 + g.element_size()
        res[f"sgd_flat_{str(gd)[6:]}_us"] = t
        res[f"sgd_flat_{str(gd)[6:]}_GBps"] = round(n * bpp / t / 1e3, 1)
    for name, (N, K) in {"fc0": (4096, 3072), "fc1": (4096, 4096)}.items():
        M = 512
        dy = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = torch.randn(N * K, device=dev) * 0.01
        mb = torch.zeros(N * K, device=dev)
        ws = torch.empty(N * K, dtype=torch.bfloat16, device=dev)
        o32 = torch.empty(N, K, device=dev)
        o16 = torch.empty(N, K, dtype=torch.bfloat16, device=dev)
        row = {}
        for tile in range(14):
            try:
                row[f"f32_t{tile}"] = timeit(lambda: G.linear_wgrad(dy, x, o32, tile=tile))
                row[f"bf16_t{tile}"] = timeit(lambda: G.linear_wgrad(dy, x, o16, tile=tile))
                row[f"sgd_t{tile}"] = timeit(lambda: G.linear_wgrad(dy, x, None, tile=tile,
                                                                     sgd=(w, mb, ws, lr, 0.9, 5e-4)))
            except Exception as ex:  # tile not valid for this shape
                row[f"err_t{tile}"] = str(ex)[:80]
        row["sgd_auto"] = timeit(lambda: G.linear_wgrad(dy, x, None, sgd=(w, mb, ws, lr, 0.9, 5e-4)))
        row["sgd_auto_GBps"] = round(N * K * 18 / row["sgd_auto"] / 1e3, 1)
        res[name] = row
    print(json.dumps(res, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
