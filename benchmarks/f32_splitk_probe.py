#!/usr/bin/env python3
"""fp32 M = 512 GEMMs of the toy MLP: in-grid split-K (slab outputs) vs one pass, plus the slab reduce.

    python benchmarks/f32_splitk_probe.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import f32  # noqa: E402
from ddpx.runtime import native  # noqa: E402


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    dev = torch.device("cuda")
    res = {}
    for (M, N, K) in [(512, 4096, 3072), (512, 4096, 4096)]:
        x = torch.randn(M, K, device=dev)
        w = torch.randn(N, K, device=dev)
        for tile in (2, 1, 3, 0):
            for S in (1, 2, 4):
                part = torch.empty(S, M, N, device=dev)
                out = part[0]
                us = timed(lambda: f32.gemm(f32.DENSE_KC, x, K, f32.DENSE_KC, w, K, M, N, K, out if S == 1 else part,
                                            tile=tile, splits=S, split_stride=M * N))
                res[f"fwd_{M}x{N}x{K}_t{tile}_s{S}"] = round(us, 1)
        for S in (2, 4):
            part = torch.empty(S, M, N, device=dev)
            y = torch.empty(M, N, device=dev)
            us = timed(lambda: native.check(native.kernels().ddpx_f32_splitk_reduce(
                part.data_ptr(), S, M * N, y.data_ptr(), 0, native.stream_handle()), "reduce"))
            res[f"reduce_{M}x{N}_s{S}"] = round(us, 1)
    for k, v in res.items():
        print(k, v, flush=True)


if __name__ == "__main__":
    main()
