#!/usr/bin/env python3
"""Is the fused wgrad+SGD kernel stream-bound or serialisation-bound?

Times linear_wgrad(..., sgd=...) for a 16384 x 16384 (wide) and 4096 x 4096 (toy) weight with the
batch (GEMM K) varied from 64 (GEMM negligible: pure optimizer-epilogue stream) to 512, for several
tile configs, and the plain sgd_flat stream of the same parameter count for reference.
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
    res = {}
    lr = torch.full((), 0.01, device=dev)
    for name, (N, K) in {"toy": (4096, 4096), "wide": (16384, 16384)}.items():
        n = N * K
        p = torch.randn(n, device=dev) * 0.01
        mb = torch.zeros(n, device=dev)
        sh = torch.empty(n, dtype=torch.bfloat16, device=dev)
        g = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        row = {"sgd_flat_bf16g_us": timeit(lambda: sgd_flat_(p, mb, g, sh, lr, 0.9, 5e-4), reps=5, inner=3)}
        row["sgd_flat_TBps"] = round(n * 20 / row["sgd_flat_bf16g_us"] / 1e6, 2)
        for M in (64, 512):
            dy = (torch.randn(M, N, device=dev) * 0.1).to(torch.bfloat16)
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            for t in (3, 5, 7, 8, 12):
                us = timeit(lambda: G.linear_wgrad(dy, x, None, tile=t, sgd=(p, mb, sh, lr, 0.9, 5e-4)), reps=5,
                            inner=3)
                row[f"B{M}_t{t}_us"] = us
                row[f"B{M}_t{t}_TBps"] = round(n * 18 / us / 1e6, 2)
            out = torch.empty(N, K, dtype=torch.bfloat16, device=dev)
            row[f"B{M}_wgrad_bf16_t8_us"] = timeit(lambda: G.linear_wgrad(dy, x, out, tile=8), reps=5, inner=3)
        res[name] = row
        print(name, json.dumps(row))
    with open("gpurun_out/sgd_epilogue_probe.json", "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
