#!/usr/bin/env python3
"""Tile configs of the f32 core on the first convolution (3 -> Co channels, image padded to 4: K = 36) at 32x32,
batch 512, with the bias + ReLU epilogue (DeepNN: Co = 128; VGG: Co = 64).

    python benchmarks/f32_first_conv_probe.py

One JSON line per (Co, tile): median of 20 CUDA-event-bracketed launches, us.  tile: 0 = 128x128, 1 = 128x64,
2 = 64x64, 3 = 64x128, -1 = auto_tile's pick.
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import f32 as F  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000.0)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N, H, W, C = 512, 32, 32, 4
    P = N * H * W
    x = torch.randn(N, H, W, C, device=dev)
    x[..., 3] = 0.0
    for Co in (128, 64):
        w = torch.randn(Co, 3, 3, 3, device=dev) * 0.1
        bias = torch.randn(Co, device=dev) * 0.1
        wf = torch.empty(9 * C * Co, device=dev)
        F.conv_wprep(w, wf, None)
        ref = None
        for tile in (-1, 0, 1, 2, 3):
            y = torch.empty(P, Co, device=dev)

            def run():
                F.gemm(F.IM2COL_KC, x, 0, F.DENSE_OC, wf, Co, P, Co, 9 * C, y, geom=(C, H, W, 1), bias=bias,
                       relu=True, tile=tile)
            us = timed(run)
            if ref is None:
                ref = y.clone()
            same = bool(torch.equal(y, ref))
            gb = (P * Co * 4 + P * C * 4) / 1e9
            print(json.dumps({"Co": Co, "tile": tile, "us": round(us, 2), "eff_TBps": round(gb / (us * 1e-6) / 1e3, 2),
                              "bitwise_vs_auto": same}), flush=True)


if __name__ == "__main__":
    main()
