#!/usr/bin/env python3
"""Run ONE fp32 convolution kernel repeatedly, for rocprofv3 --pmc counter passes.

    rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES ... -d DIR -- python3 benchmarks/f32_probe.py --case wino_fwd_h8

cases: wino_fwd_{h32,h16,h8,h4}, wgrad_{h32,h16,h8,h4} (the VGG layer at that resolution with the most work).
"""
import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import f32  # noqa: E402

LAYER = {"h32": (32, 64, 128), "h16": (16, 256, 256), "h8": (8, 512, 512), "h4": (4, 512, 512)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", required=True)
    ap.add_argument("--iters", type=int, default=10)
    a = ap.parse_args()
    kind, res = a.case.rsplit("_", 1)
    H, Ci, Co = LAYER[res]
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N = 512
    x = torch.randn(N, H, H, Ci, device=dev)
    w = torch.randn(Co, Ci, 3, 3, device=dev) / (9 * Ci) ** 0.5
    if kind == "wino_fwd":
        uf = torch.empty(16 * Ci * Co, device=dev)
        f32.wino_wprep(w, uf, None)
        fn = lambda: f32.wino_conv(x, uf, Co, stats=True)  # noqa: E731
    elif kind == "wgrad":
        dy = torch.randn(N * H * H, Co, device=dev)
        out = torch.empty(Co, Ci, 3, 3, device=dev)
        fn = lambda: f32.conv_wgrad(dy, x, Co, Ci, out)  # noqa: E731
    else:
        raise SystemExit(f"unknown case {a.case}")
    for _ in range(a.iters):
        fn()
    torch.cuda.synchronize()
    print("done", a.case, flush=True)


if __name__ == "__main__":
    main()
