#!/usr/bin/env python3
"""Time the native 3x3 conv fwd / dgrad / wgrad per VGG layer and tile config vs MIOpen (torch).

    python benchmarks/conv_sweep.py [--batch 512] [--out gpurun_out/conv_sweep.json]
"""
import argparse
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddpx.ops import conv as K  # noqa: E402

LAYERS = [(3, 64, 32), (64, 128, 32), (128, 256, 16), (256, 256, 16), (256, 512, 8), (512, 512, 8), (512, 512, 4),
          (512, 512, 4)]
# the reference's DeepNN (/root/reference/singlegpu.py:21-31): (Ci, Co, H)
DEEPNN_LAYERS = [(3, 128, 32), (128, 64, 32), (64, 64, 16), (64, 32, 16)]


def timeit(fn, iters=10, warm=3):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default=None)
    ap.add_argument("--net", default="vgg", choices=["vgg", "deepnn"])
    ap.add_argument("--cfgs", default="", help="comma list of tile configs (default 0-15)")
    ap.add_argument("--layers", default="", help="comma list of layer indices (default all)")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N = a.batch
    res = []
    cfgs = [int(c) for c in a.cfgs.split(",") if c] or list(range(16))
    layers = LAYERS if a.net == "vgg" else DEEPNN_LAYERS
    if a.layers:
        layers = [layers[int(i)] for i in a.layers.split(",")]
    for (Ci, Co, H) in layers:
        Cp = K.padded_channels(Ci)
        x = (torch.rand(N, H, H, Cp, device=dev) * 2 - 1).to(torch.bfloat16)
        w = torch.randn(Co, Ci, 3, 3, device=dev) * 0.05
        wf = torch.empty(Co * 9 * Cp, dtype=torch.bfloat16, device=dev)
        wd = torch.empty_like(wf)
        K.weight_prep(w, wf, wd)
        dy = (torch.rand(N * H * H, Co, device=dev) * 2 - 1).to(torch.bfloat16)
        dw = torch.empty(Co, Ci, 3, 3, device=dev)
        flop = 2.0 * N * H * H * Co * Ci * 9
        row = {"layer": f"{Ci}->{Co}@{H}", "gflop": round(flop / 1e9, 1)}
        xt = x[..., :Ci].permute(0, 3, 1, 2).contiguous(memory_format=torch.channels_last)
        wt = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        row["miopen_fwd"] = round(timeit(lambda: F.conv2d(xt, wt, padding=1)), 1)
        for cfg in cfgs:
            row[f"fwd{cfg}"] = round(timeit(lambda: K.conv_fwd(x, wf, Co, stats=True, tile=cfg)), 1)
            row[f"dgrad{cfg}"] = round(timeit(lambda: K.conv_dgrad(dy, wd, N, H, H, Cp, Co, tile=cfg)), 1)
            row[f"wgrad{cfg}"] = round(timeit(lambda: K.conv_wgrad(dy, x, Co, Ci, out=dw, tile=cfg)), 1)
        for kind in ("fwd", "dgrad", "wgrad"):
            best = min(cfgs, key=lambda c: row[f"{kind}{c}"])
            row[f"best_{kind}"] = best
            row[f"best_{kind}_tflops"] = round(flop / row[f"{kind}{best}"] / 1e6, 1)
        res.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
