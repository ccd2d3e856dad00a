#!/usr/bin/env python3
"""Split count and tile of the f32 core's direct weight gradient for the first convolution (3 -> 128 channels at
32x32, batch 512: M = 128, N = 36, K = 524288), split GEMM + fixed-order reduce.

    python benchmarks/f32_first_wgrad_probe.py

One JSON line per (splits, tile): median of 20 CUDA-event-bracketed runs (us) of the GEMM and of GEMM + reduce.
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
    N, H, W, Cp, Ci, Co = 512, 32, 32, 4, 3, 128
    P = N * H * W
    ncol = 9 * Cp
    x = torch.randn(N, H, W, Cp, device=dev)
    x[..., 3] = 0.0
    dy = torch.randn(P, Co, device=dev)
    out = torch.empty(Co, Ci, 3, 3, device=dev)
    default_S = F.wgrad_splits(Co, ncol, P)
    ref = None
    for S in sorted({default_S, 128, 256, 1024}):
        part = torch.empty((S, Co, ncol), dtype=torch.float32, device=dev)
        for tile in (-1, 0, 1, 3):
            def gemm():
                F.gemm(F.DENSE_OC, dy, Co, F.IM2COL_OC, x, 0, Co, ncol, P, part, geom=(Cp, H, W, 1), splits=S,
                       split_stride=Co * ncol, tile=tile)

            def both():
                gemm()
                F._call("ddpx_f32_conv_wgrad_reduce", part.data_ptr(), S, Co, Ci, Cp, out.data_ptr(), 0)
            tg = timed(gemm)
            tb = timed(both)
            if ref is None:
                ref = out.clone()
            rel = float((out - ref).norm() / ref.norm())
            print(json.dumps({"S": S, "default_S": S == default_S, "tile": tile, "gemm_us": round(tg, 1),
                              "gemm_reduce_us": round(tb, 1), "rel_vs_first": rel}), flush=True)


if __name__ == "__main__":
    main()
