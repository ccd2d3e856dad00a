#!/usr/bin/env python3
"""Forward / dgrad GEMMs of the toy MLP at batch 512: default plan (in-launch split-K) vs fixed tiles (µs)."""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddpx.ops import gemm as G  # noqa: E402
from benchmarks.sgd_bw import timeit  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda")
    res = {}
    for name, (K, N) in {"fc0": (3072, 4096), "fc1": (4096, 4096)}.items():
        M = 512
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
        b = torch.randn(N, device=dev)
        dy = torch.randn(M, N, device=dev).to(torch.bfloat16)
        row = {}
        row["fwd_auto"] = timeit(lambda: G.linear_fwd(x, w, b, relu=True))
        row["dgrad_auto"] = timeit(lambda: G.linear_dgrad(dy, w, relu_mask_of=x))
        for t in range(14):
            row[f"fwd_t{t}"] = timeit(lambda: G.linear_fwd(x, w, b, relu=True, tile=t))
            row[f"dgrad_t{t}"] = timeit(lambda: G.linear_dgrad(dy, w, relu_mask_of=x, tile=t))
        res[name] = row
        print(name, json.dumps(row))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
