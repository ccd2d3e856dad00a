#!/usr/bin/env python3
"""Where the toy MLP's wgrad+SGD pair spends its time: per-role barrier arrival stamps.

    python benchmarks/pair_stamps.py [--out FILE.json] [--reps 5]

The pair (``csrc/include/ddpx_wgrad_sgd.h``) runs 4 MFMA ("math") waves and 4 optimizer-stream waves per CU in
lock-step: both roles pass the same s_barrier sequence (one per 64-deep K-step, one hand-off per tile).  With
``ddpx_gemm_set_stamps`` each role's lane 0 stamps its arrival at every barrier (s_memrealtime, 10 ns).  A
barrier is left when the later role arrives, so per barrier interval:

* ``math_wait`` = departure - math arrival: the math waves idle, waiting for the stream (stream-bound step);
* ``stream_wait`` = departure - stream arrival: the stream idle, waiting for the MFMA side (math-bound step).

Reported over CUs (median / max): span, the two roles' summed waits, and the interval split into math-bound /
stream-bound steps; plus the first-fill and drain iterations (the roles cannot overlap there).  Shapes: fc1
4096x4096 and fc0 4096x3072 weight gradients at batch 512 with the fused SGD, as in the training step.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import gemm as G  # noqa: E402
from ddpx.runtime import native  # noqa: E402

SLOTS = 256  # ddpx_wgrad_sgd.h kStampSlots


def med(v):
    v = sorted(v)
    return v[len(v) // 2] if v else float("nan")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--time_only", action="store_true")
    ap.add_argument("--xwg", action="store_true", help="two-workgroup pair: placement + per-role spans")
    a = ap.parse_args()
    native.register_kernel_sig("ddpx_gemm_set_stamps", None, native.c_void_p)
    lib = native.kernels()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    bf = torch.bfloat16
    B, D0, H = 512, 3072, 4096
    x0 = torch.rand(B, D0, device=dev).to(bf)
    h1 = torch.rand(B, H, device=dev).to(bf)
    d1 = (torch.randn(B, H, device=dev) * 0.01).to(bf)
    d2 = (torch.randn(B, H, device=dev) * 0.01).to(bf)
    lr = torch.full((), 0.01, device=dev)

    def state(n):
        return (torch.randn(n, device=dev) * 0.01, torch.zeros(n, device=dev), torch.empty(n, dtype=bf, device=dev))
    p1, m1, s1 = state(H * H)
    p0, m0, s0 = state(H * D0)
    sg1 = (p1, m1, s1, lr, 0.9, 5e-4)
    sg0 = (p0, m0, s0, lr, 0.9, 5e-4)

    def run():
        assert G.wgrad_sgd_pair(d2, h1, sg1, d1, x0, sg0)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    # plain timing: 20 back-to-back launches (every variant, stamped or not)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        run()
    e1.record()
    torch.cuda.synchronize()
    print(json.dumps({"pair_us_per_launch": round(e0.elapsed_time(e1) * 1000 / 20, 2),
                      "xwg_poll_timeouts": G.xwg_poll_timeouts(dev)}), flush=True)
    if a.time_only:
        return
    if a.xwg:
        # two-workgroup pair: per workgroup [HW_ID, XCC_ID, start, end] -> placement of the roles and their spans
        st = torch.zeros((1024, 4), dtype=torch.int64, device=dev)
        lib.ddpx_gemm_set_stamps(st.data_ptr())
        run()
        torch.cuda.synchronize()
        lib.ddpx_gemm_set_stamps(None)
        s = st.cpu().numpy()
        n = int((s[:, 2] != 0).sum())
        G2 = n // 2
        t0 = s[:n, 2].min()

        def cu_key(hw, xcc):  # (xcc, se, sh, cu) from HW_ID: cu [11:8], sh [12], se [15:13]
            return (int(xcc) & 0xf, (int(hw) >> 13) & 7, (int(hw) >> 12) & 1, (int(hw) >> 8) & 0xf)
        where = {}
        for b in range(n):
            where.setdefault(cu_key(s[b, 0], s[b, 1]), []).append("M" if b < G2 else "S")
        kinds = {}
        for v in where.values():
            k = "".join(sorted(v))
            kinds[k] = kinds.get(k, 0) + 1
        math_span = [(s[b, 3] - s[b, 2]) / 100.0 for b in range(G2)]
        strm_span = [(s[b, 3] - s[b, 2]) / 100.0 for b in range(G2, n)]
        end = (s[:n, 3].max() - t0) / 100.0
        print(json.dumps({"workgroups": n, "cus_used": len(where), "cu_role_mix": kinds,
                          "math_span_med": med(math_span), "math_span_max": max(math_span),
                          "stream_span_med": med(strm_span), "stream_span_max": max(strm_span),
                          "stream_start_med": med([(s[b, 2] - t0) / 100.0 for b in range(G2, n)]),
                          "kernel_span": end}), flush=True)
        return
    st = torch.zeros((256 * 2, SLOTS), dtype=torch.int64, device=dev)
    out = {"reps": []}
    for _ in range(a.reps):
        st.zero_()
        lib.ddpx_gemm_set_stamps(st.data_ptr())
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        lib.ddpx_gemm_set_stamps(None)
        s = st.view(-1, 2, SLOTS).cpu().numpy().astype("int64")
        rows = [i for i in range(s.shape[0]) if s[i, 0, 0] and s[i, 1, 0]]
        t0 = min(int(s[i, r, 0]) for i in rows for r in (0, 1))
        us = lambda d: d / 100.0  # noqa: E731
        per_cu = []
        for i in rows:
            m, q = s[i, 0], s[i, 1]
            nb = int(((m[1:SLOTS - 1] != 0)).sum())
            nbq = int(((q[1:SLOTS - 1] != 0)).sum())
            n = min(nb, nbq)
            mw = sw = mb = sb = 0.0
            fill = drain = 0.0
            prev = int(max(m[0], q[0]))
            per_iter = None
            for b in range(1, n + 1):
                am, aq = int(m[b]), int(q[b])
                dep = max(am, aq)
                mw += us(dep - am)
                sw += us(dep - aq)
                if aq >= am:
                    sb += us(dep - prev)
                else:
                    mb += us(dep - prev)
                prev = dep
            # barriers per iteration = nk + 1 (nk = 8 K-steps); iteration 0 = math fill, last = stream drain
            per_iter = 9
            if n >= 2 * per_iter:
                fill = us(int(max(m[per_iter], q[per_iter])) - int(max(m[0], q[0])))
                drain = us(int(max(m[n], q[n])) - int(max(m[n - per_iter], q[n - per_iter])))
            end = max(int(m[SLOTS - 1]), int(q[SLOTS - 1]))
            per_cu.append({"span": us(end - t0), "start_skew": us(int(min(m[0], q[0])) - t0), "barriers": n,
                           "math_wait": mw, "stream_wait": sw, "math_bound": mb, "stream_bound": sb,
                           "fill_iter": fill, "drain_iter": drain,
                           "tail": us(end - int(max(m[n], q[n])))})
        keys = list(per_cu[0])
        rep = {"event_us": round(e0.elapsed_time(e1) * 1000, 2), "cus": len(per_cu)}
        for k in keys:
            vals = [c[k] for c in per_cu]
            rep[k] = {"med": round(med(vals), 2), "max": round(max(vals), 2)}
        out["reps"].append(rep)
        print(json.dumps(rep), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
