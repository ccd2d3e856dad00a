#!/usr/bin/env python3
"""fp32 VGG convolutions per layer: Winograd F(2,3) (csrc/kernels/f32_wino.hip) vs the exact implicit GEMM
(forward, data gradient, weight gradient).

    python benchmarks/wino_bench.py [--out FILE]        (DDPX_WINO_STAGES=2|3 selects the Winograd ring depth)

Each launch is timed as a HIP graph of back-to-back launches, median of rounds; TF/s counts the direct 3x3
product's FLOPs (2 N H W Co 9 Ci) for both, so the Winograd figure is the "effective" rate.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import f32  # noqa: E402

LAYERS = [(32, 64, 128), (16, 128, 256), (16, 256, 256), (8, 256, 512), (8, 512, 512), (4, 512, 512)]


def timed(fn, inner=5, rounds=5):
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
    ts = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000 / inner)
    return sorted(ts)[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--only", default="", help="wgrad: time only the weight gradients")
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    N = a.batch
    res = {}
    for H, Ci, Co in LAYERS:
        x = torch.randn(N, H, H, Ci, device=dev)
        w = torch.randn(Co, Ci, 3, 3, device=dev) / (9 * Ci) ** 0.5
        uf = torch.empty(16 * Ci * Co, device=dev)
        ud = torch.empty(16 * Co * Ci, device=dev)
        f32.wino_wprep(w, uf, ud)
        wf = torch.empty(9 * Ci * Co, device=dev)
        wd = torch.empty(9 * Ci * Co, device=dev)
        f32.conv_wprep(w, wf, wd)
        dy = torch.randn(N, H, H, Co, device=dev)
        flops = 2.0 * N * H * H * Co * 9 * Ci
        if a.only == "wgrad":
            gw = torch.empty(Co, Ci, 3, 3, device=dev)
            row = {"wino_wgrad": round(timed(lambda: f32.wino_wgrad(dy.view(-1, Co), x, Co, Ci, gw)), 1)}
            key = f"H{H}_C{Ci}_K{Co}"
            res[key] = row
            print(key, json.dumps(row), flush=True)
            continue
        row = {
            "wino_fwd": timed(lambda: f32.wino_conv(x, uf, Co, stats=True)),
            "direct_fwd": timed(lambda: f32.conv_fwd_stats(x, wf, Co)),
            "wino_dgrad": timed(lambda: f32.wino_conv(dy, ud, Ci)),
            "direct_dgrad": timed(lambda: f32.conv_dgrad(dy.view(-1, Co), wd, N, H, H, Ci, Co)),
            "wprep": timed(lambda: f32.wino_wprep(w, uf, ud)),
        }
        gw = torch.empty(Co, Ci, 3, 3, device=dev)
        dyf = dy.view(-1, Co)
        row["wino_wgrad"] = timed(lambda: f32.wino_wgrad(dyf, x, Co, Ci, gw))
        row["direct_wgrad"] = timed(lambda: f32.direct_wgrad(dyf, x, Co, Ci, gw))
        row = {k: round(v, 1) for k, v in row.items()}
        for k in ("wino_fwd", "direct_fwd", "wino_dgrad", "direct_dgrad", "wino_wgrad", "direct_wgrad"):
            row[k + "_tflops"] = round(flops / row[k] / 1e6, 1)
        key = f"H{H}_C{Ci}_K{Co}"
        res[key] = row
        print(key, json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
