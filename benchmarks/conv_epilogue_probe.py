#!/usr/bin/env python3
"""Cost of the BatchNorm-statistics epilogue of the conv forward GEMM (stats=True vs plain bf16 store).

    python benchmarks/conv_epilogue_probe.py [--out gpurun_out/conv_epilogue_probe.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from benchmarks.conv_sweep import timeit  # noqa: E402
from ddpx.ops import conv as K  # noqa: E402

LAYERS = [(64, 128, 32), (128, 256, 16), (256, 256, 16), (256, 512, 8), (512, 512, 8)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    N = a.batch
    res = []
    for (Ci, Co, H) in LAYERS:
        x = (torch.rand(N, H, H, Ci, device=dev) * 2 - 1).to(torch.bfloat16)
        w = torch.randn(Co, Ci, 3, 3, device=dev) * 0.05
        wf = torch.empty(Co * 9 * Ci, dtype=torch.bfloat16, device=dev)
        wd = torch.empty_like(wf)
        K.weight_prep(w, wf, wd)
        row = {"layer": f"{Ci}->{Co}@{H}"}
        for cfg in (8, 13):
            row[f"stats_t{cfg}"] = round(timeit(lambda: K.conv_fwd(x, wf, Co, stats=True, tile=cfg)), 1)
            row[f"plain_t{cfg}"] = round(timeit(lambda: K.conv_fwd(x, wf, Co, stats=False, tile=cfg)), 1)
        res.append(row)
        print(json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
