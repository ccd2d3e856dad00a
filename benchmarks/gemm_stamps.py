#!/usr/bin/env python3
"""Where a GEMM launch spends its time, per workgroup (in-kernel s_memrealtime stamps, 10 ns ticks).

    python benchmarks/gemm_stamps.py [--cases fwd1_t16s4,...]

For each case (toy-MLP M = 512 products, tile config, split-K): one warm launch, then one stamped launch.
Prints the launch span and, over workgroups, the median / max of: start skew (first start -> own start),
main loop, split-K slab store + ticket, combine (last arrivers), epilogue.  Stamps: ``ddpx_gemm_set_stamps``
(csrc/kernels/gemm_pipe.hip); the kernel writes [workgroup][8] int64 at fixed points (csrc/include/ddpx_pipe.h).
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import gemm as G  # noqa: E402
from ddpx.runtime import native  # noqa: E402


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    native.register_kernel_sig("ddpx_gemm_set_stamps", None, native.c_void_p)
    lib = native.kernels()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    bf = torch.bfloat16
    M, D0, H = 512, 3072, 4096
    x = torch.rand(M, D0, device=dev).to(bf)
    w0 = (torch.randn(H, D0, device=dev) * 0.02).to(bf)
    w1 = (torch.randn(H, H, device=dev) * 0.02).to(bf)
    b0, b1 = torch.randn(H, device=dev), torch.randn(H, device=dev)
    h1 = G.linear_fwd(x, w0, b0, relu=True)
    h2 = G.linear_fwd(h1, w1, b1, relu=True)
    d2 = (torch.randn(M, H, device=dev) * 0.01).to(bf)
    d1 = torch.empty_like(h1)
    cases = {}
    for tile, sp in ((12, None), (18, None), (14, 2)):
        tag = f"t{tile}" + (f"s{sp}" if sp else "")
        cases[f"fwd0_{tag}"] = lambda tile=tile, sp=sp: G.linear_fwd(x, w0, b0, relu=True, out=h1, tile=tile, splits=sp)
        cases[f"fwd1_{tag}"] = lambda tile=tile, sp=sp: G.linear_fwd(h1, w1, b1, relu=True, out=h2, tile=tile, splits=sp)
        cases[f"dgrad1_{tag}"] = lambda tile=tile, sp=sp: G.linear_dgrad(d2, w1, relu_mask_of=h1, out=d1, tile=tile,
                                                                          splits=sp)
    want = [c for c in a.cases.split(",") if c] or list(cases)
    st = torch.zeros((4096, 8), dtype=torch.int64, device=dev)
    res = {}
    for name in want:
        fn = cases[name]
        fn()
        torch.cuda.synchronize()
        st.zero_()
        lib.ddpx_gemm_set_stamps(st.data_ptr())
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        ev0.record()
        fn()
        ev1.record()
        torch.cuda.synchronize()
        lib.ddpx_gemm_set_stamps(None)
        s = st.cpu()
        rows = s[s[:, 0] != 0]
        t0 = int(rows[:, 0].min())
        us = lambda d: d / 100.0  # noqa: E731  (10 ns ticks -> us)
        loop = [us(int(r[1] - r[0])) for r in rows if r[1]]
        skew = [us(int(r[0]) - t0) for r in rows]
        tick = [us(int(r[2] - r[1])) for r in rows if r[2] and r[1]]
        comb = [us(int(r[3] - r[2])) for r in rows if r[3] and r[2]]
        epi = [us(int(r[4] - (r[3] if r[3] else r[1]))) for r in rows if r[4]]
        end = max(int(v) for v in rows[:, 1:5].flatten() if int(v))
        out = {"event_us": round(ev0.elapsed_time(ev1) * 1000, 2), "span_us": round(us(end - t0), 2),
               "wgs": int(rows.shape[0]), "start_skew_med_max": [round(med(skew), 2), round(max(skew), 2)],
               "loop_med_max": [round(med(loop), 2), round(max(loop), 2)],
               "ticket_med_max": [round(med(tick), 2), round(max(tick), 2)] if tick else None,
               "combine_med_max": [round(med(comb), 2), round(max(comb), 2)] if comb else None,
               "epilogue_med_max": [round(med(epi), 2), round(max(epi), 2)] if epi else None}
        res[name] = out
        print(name, json.dumps(out), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
