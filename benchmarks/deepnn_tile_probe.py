#!/usr/bin/env python3
"""DeepNN bf16 conv tiles with the fused epilogues (ops/conv.py conv_fwd_act / conv_dgrad_act), per layer and tile.

    python benchmarks/deepnn_tile_probe.py [--tiles 22,23,8,13,21,6,2,5]

Times (back-to-back launches) the data gradient of DeepNN's block 1 (64 -> 128 channels' input gradient at 32x32,
masked by block 0's ReLU, with the bias column sums) and the forward of block 0 / 1 (bias + ReLU epilogue) for
each tile config, so the per-layer picks can be re-made for the fused epilogues (profiles/r6_deepnn).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddpx.ops import conv as K  # noqa: E402


def timeit(fn, iters=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return round(a.elapsed_time(b) * 1000 / iters, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tiles", default="-1,22,23,8,13,21,6,2,5,3,7")
    a = ap.parse_args()
    dev = torch.device("cuda")
    bf = torch.bfloat16
    N = 512
    out = {}
    # block 1's data gradient: dy [N*32*32, 64], wd [9, 64, 128], mask = block 0's act [N*32*32, 128]
    dy = (torch.randn(N * 1024, 64, device=dev) * 0.1).to(bf)
    wd = (torch.randn(9 * 64 * 128, device=dev) * 0.05).to(bf)
    act0 = torch.relu(torch.randn(N * 1024, 128, device=dev)).to(bf)
    # forwards: block 0 (3 -> 128, Cp 8) and block 1 (128 -> 64) at 32x32
    x0 = torch.rand(N, 32, 32, 8, device=dev).to(bf)
    wf0 = (torch.randn(128 * 9 * 8, device=dev) * 0.1).to(bf)
    x1 = torch.relu(torch.randn(N, 32, 32, 128, device=dev)).to(bf)
    wf1 = (torch.randn(64 * 9 * 128, device=dev) * 0.05).to(bf)
    b128, b64 = torch.randn(128, device=dev), torch.randn(64, device=dev)
    for t in [int(v) for v in a.tiles.split(",")]:
        row = {}
        for name, fn in (("dgrad1_act", lambda: K.conv_dgrad_act(dy, wd, N, 32, 32, 128, 64, act0, tile=t)),
                         ("dgrad1_plain", lambda: K.conv_dgrad(dy, wd, N, 32, 32, 128, 64, tile=t)),
                         ("fwd0_act", lambda: K.conv_fwd_act(x0, wf0, 128, b128, tile=t)),
                         ("fwd1_act", lambda: K.conv_fwd_act(x1, wf1, 64, b64, tile=t))):
            try:
                row[name] = timeit(fn)
            except Exception as e:  # noqa: BLE001 - a config without a variant for this epilogue
                row[name] = f"{type(e).__name__}"
        out[t] = row
        print(t, json.dumps(row), flush=True)


if __name__ == "__main__":
    main()
