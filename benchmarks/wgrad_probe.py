#!/usr/bin/env python3
"""Weight-gradient GEMMs of the toy MLP (K = batch = 512): every pipe tile config with an fp32 output
and with the fused-SGD epilogue, against hipBLASLt (torch.mm) and the flat SGD stream alone.

    python benchmarks/wgrad_probe.py [--out gpurun_out/wgrad_probe.json]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import gemm as G  # noqa: E402
from ddpx.runtime import native  # noqa: E402


def timeit(fn, iters=40, warm=8):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return round(s.elapsed_time(e) / iters * 1e3, 2)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=512)
    ap.add_argument("--out", default=None)
    ap.add_argument("--cfgs", default="0,1,2,3,4,5,6,7,8,9,10,11,12,13")
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    B = a.batch
    cfgs = [int(c) for c in a.cfgs.split(",")]
    lib = native.kernels()
    res = {}
    for name, (H, I) in {"fc1": (4096, 4096), "fc0": (4096, 3072)}.items():
        dy = ((torch.rand(B, H, device=dev) * 2 - 1) * 1e-3).to(torch.bfloat16)
        x = (torch.rand(B, I, device=dev)).to(torch.bfloat16)
        dw = torch.empty(H, I, device=dev)
        p = torch.randn(H, I, device=dev) * 0.01
        buf = torch.zeros(H, I, device=dev)
        sh = p.to(torch.bfloat16)
        lr = torch.full((), 0.1, device=dev)
        sgd = (p, buf, sh, lr, 0.9, 5e-4)
        row = {"hipblaslt_bf16": timeit(lambda: dy.t() @ x)}
        row["sgd_flat_f32g"] = timeit(lambda: native.check(lib.ddpx_sgd_flat(
            p.data_ptr(), buf.data_ptr(), dw.data_ptr(), 0, sh.data_ptr(), p.numel(), lr.data_ptr(), 0.0, 0.9, 5e-4,
            1.0, 0, 0, None, None, native.stream_handle()), "sgd"))
        for c in cfgs:
            row[f"f32_t{c}"] = timeit(lambda: G.linear_wgrad(dy, x, dw, tile=c))
            row[f"sgd_t{c}"] = timeit(lambda: G.linear_wgrad(dy, x, None, tile=c, sgd=sgd))
        row["sgd_auto"] = timeit(lambda: G.linear_wgrad(dy, x, None, sgd=sgd))
        row["f32_auto"] = timeit(lambda: G.linear_wgrad(dy, x, dw))
        row["stream_MB"] = round(H * I * 18 / 1e6, 1)
        row["gflop"] = round(2 * B * H * I / 1e9, 2)
        res[name] = row
        print(name, json.dumps(row), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
