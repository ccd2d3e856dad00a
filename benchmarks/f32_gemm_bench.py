"""Throughput of the exact-f32 MFMA GEMM core (``csrc/kernels/f32_train.hip``) per tile on the shapes of the
fp32 VGG / MLP steps, against torch fp32 (hipBLASLt / MIOpen) on the same shapes.

    python benchmarks/f32_gemm_bench.py [--reps 20]
"""
from __future__ import annotations

import argparse
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timed(fn, reps):
    import torch
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3  # us


def main():
    import torch
    import torch.nn.functional as F
    from ddpx.ops import f32
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    res = []
    # Linear (toy MLP fp32): fwd x[512,K] W[N,K]^T; wgrad dW[N,K] = dy^T x
    for (M, N, K) in [(512, 4096, 3072), (512, 4096, 4096)]:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        y = torch.empty(M, N, device=dev)
        dy = torch.randn(M, N, device=dev)
        dW = torch.empty(N, K, device=dev)
        fl = 2.0 * M * N * K
        for tile in (0, 1, 2):
            us = timed(lambda: f32.gemm(f32.DENSE_KC, x, K, f32.DENSE_KC, w, K, M, N, K, y, tile=tile), a.reps)
            res.append({"op": f"linear_fwd {M}x{N}x{K}", "tile": tile, "us": round(us, 1), "tf": round(fl / us / 1e6, 1)})
            us = timed(lambda: f32.gemm(f32.DENSE_OC, dy, N, f32.DENSE_OC, x, K, N, K, M, dW, tile=tile), a.reps)
            res.append({"op": f"linear_wgrad {N}x{K}x{M}", "tile": tile, "us": round(us, 1), "tf": round(fl / us / 1e6, 1)})
        us = timed(lambda: torch.mm(x, w.t()), a.reps)
        res.append({"op": f"linear_fwd {M}x{N}x{K}", "tile": "torch", "us": round(us, 1), "tf": round(fl / us / 1e6, 1)})
    # convolutions of the VGG at batch 512: forward implicit GEMM
    for (N, H, Ci, Co) in [(512, 32, 64, 128), (512, 16, 256, 256), (512, 8, 512, 512), (512, 4, 512, 512)]:
        x = torch.randn(N, H, H, Ci, device=dev)
        w = torch.randn(Co, Ci, 3, 3, device=dev)
        wf = torch.empty(9 * Ci * Co, device=dev)
        f32.conv_wprep(w, wf, None)
        P = N * H * H
        y = torch.empty(P, Co, device=dev)
        fl = 2.0 * P * Co * 9 * Ci
        for tile in (0, 1, 2):
            us = timed(lambda: f32.gemm(f32.IM2COL_KC, x, 0, f32.DENSE_OC, wf, Co, P, Co, 9 * Ci, y,
                                        geom=(Ci, H, H, 1), tile=tile), a.reps)
            res.append({"op": f"conv_fwd N{N} H{H} {Ci}->{Co}", "tile": tile, "us": round(us, 1),
                        "tf": round(fl / us / 1e6, 1)})
        xn = x.permute(0, 3, 1, 2).contiguous()
        us = timed(lambda: F.conv2d(xn, w, padding=1), a.reps)
        res.append({"op": f"conv_fwd N{N} H{H} {Ci}->{Co}", "tile": "torch", "us": round(us, 1),
                    "tf": round(fl / us / 1e6, 1)})
    for r in res:
        print(json.dumps(r))


if __name__ == "__main__":
    main()
