#!/usr/bin/env python3
"""Cost of the transposed MX-FP8 copy in the wgrad+SGD pair on the wide MLP's shapes (fc1 16384x16384, fc0
16384x3072, batch 512): back-to-back pair launches with the row copy only, + transposed codes, + transposed codes and
scales.

    python benchmarks/pair_fp8t.py
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import gemm as G  # noqa: E402
from ddpx.runtime import native  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    bf = torch.bfloat16
    B, D0, H = 512, 3072, 16384
    x0 = torch.rand(B, D0, device=dev).to(bf)
    h1 = torch.rand(B, H, device=dev).to(bf)
    d1 = (torch.randn(B, H, device=dev) * 0.01).to(bf)
    d2 = (torch.randn(B, H, device=dev) * 0.01).to(bf)
    lr = torch.full((), 0.01, device=dev)

    def state(m, n):
        return (torch.randn(m * n, device=dev) * 0.01, torch.zeros(m * n, device=dev),
                torch.empty(m * n, dtype=bf, device=dev),
                (torch.empty(m, n, dtype=torch.uint8, device=dev), torch.empty(m, n // 32, dtype=torch.uint8, device=dev)),
                (torch.empty(n, m, dtype=torch.uint8, device=dev), torch.empty(n, m // 32, dtype=torch.uint8, device=dev)))
    p1, m1, s1, r1, t1 = state(H, H)
    p0, m0, s0, r0, t0 = state(H, D0)
    sg1 = (p1, m1, s1, lr, 0.9, 5e-4)
    sg0 = (p0, m0, s0, lr, 0.9, 5e-4)
    lib = native.kernels()

    def raw(t_codes, t_scales):
        args = []
        for dy, x, sg, r, t, M, N in ((d2, h1, sg1, r1, t1, H, H), (d1, x0, sg0, r0, None, H, D0)):
            args += [dy.data_ptr(), x.data_ptr(), M, N, dy.stride(0), x.stride(0), N, sg[0].data_ptr(), sg[1].data_ptr(),
                     sg[2].data_ptr(), r[0].data_ptr(), r[1].data_ptr(),
                     t[0].data_ptr() if (t is not None and t_codes) else None,
                     t[1].data_ptr() if (t is not None and t_scales) else None]
        rc = lib.ddpx_wgrad_sgd_pair_t(*args, B, lr.data_ptr(), 0.9, 5e-4, native.stream_handle())
        native.check(rc, "pair_t")

    out = {}
    for name, tc, ts in (("rows_only", False, False), ("t_codes", True, False), ("t_codes_scales", True, True),
                         ("rows_only_2", False, False)):
        for _ in range(3):
            raw(tc, ts)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            raw(tc, ts)
        e1.record()
        torch.cuda.synchronize()
        out[name] = round(e0.elapsed_time(e1) * 100, 1)  # us per launch
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
