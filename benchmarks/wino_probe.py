#!/usr/bin/env python3
"""Eager launches of the fp32 Winograd kernels on one VGG layer, for rocprofv3 --pmc passes.

    rocprofv3 --pmc <counters> -- python3 benchmarks/wino_probe.py [--layer 16,256,256] [--iters 3]
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import f32  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--layer", default="16,256,256", help="H,Ci,Co")
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--iters", type=int, default=3)
    a = ap.parse_args()
    H, Ci, Co = (int(v) for v in a.layer.split(","))
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N = a.batch
    x = torch.randn(N, H, H, Ci, device=dev)
    w = torch.randn(Co, Ci, 3, 3, device=dev) / (9 * Ci) ** 0.5
    uf = torch.empty(16 * Ci * Co, device=dev)
    ud = torch.empty(16 * Co * Ci, device=dev)
    f32.wino_wprep(w, uf, ud)
    dy = torch.randn(N * H * H, Co, device=dev)
    gw = torch.empty(Co, Ci, 3, 3, device=dev)
    for _ in range(a.iters):
        f32.wino_conv(x, uf, Co, stats=True)
        f32.wino_conv(dy.view(N, H, H, Co), ud, Ci)
        f32.wino_wgrad(dy, x, Co, Ci, gw)
    torch.cuda.synchronize()
    print("ok")


if __name__ == "__main__":
    main()
