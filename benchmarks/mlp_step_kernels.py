#!/usr/bin/env python3
"""Every kernel of the toy-MLP training step (batch 512, 3072-4096-4096-10), timed in ONE process with
interleaved rounds (cdna_hip_programming §5.4 rule 24), each variant captured as a HIP graph of
`inner` back-to-back launches so host launch cost does not leak into short kernels.

    python benchmarks/mlp_step_kernels.py [--out FILE] [--rounds 5]

Variants: the default launch plan (tile -1) against fixed tiles for the forward / data-gradient GEMMs,
the weight-gradient GEMMs (fp32 out), the head forward / backward and the flat SGD pass.  Prints and
writes {case: median µs}.
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from ddpx.ops import gemm as G  # noqa: E402
from ddpx.ops.elementwise import sgd_flat_  # noqa: E402
from ddpx.ops.head import head_backward, head_forward  # noqa: E402


def graph_of(fn, inner):
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
    torch.cuda.synchronize()
    return g


def time_graph(g, inner, reps=10):
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.replay()
        b.record()
        b.synchronize()
        ts.append(a.elapsed_time(b) * 1000 / inner)
    ts.sort()
    return ts[len(ts) // 2]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--inner", type=int, default=20)
    a = ap.parse_args()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M, D0, H, C = 512, 3072, 4096, 10
    bf = torch.bfloat16
    x = torch.rand(M, D0, device=dev).to(bf)
    w0 = (torch.randn(H, D0, device=dev) * 0.02).to(bf)
    w1 = (torch.randn(H, H, device=dev) * 0.02).to(bf)
    w2 = (torch.randn(C, H, device=dev) * 0.02).to(bf)
    b0, b1, b2 = (torch.randn(n, device=dev) * 0.1 for n in (H, H, C))
    h1 = G.linear_fwd(x, w0, b0, relu=True)
    h2 = G.linear_fwd(h1, w1, b1, relu=True)
    t = torch.randint(0, C, (M,), device=dev)
    loss, _, dl = head_forward(h2, w2, b2, t, want_logits=False)
    d2 = torch.empty_like(h2)
    dW2, db2, dbp = torch.empty(C, H, device=dev), torch.empty(C, device=dev), torch.empty(H, device=dev)
    go = torch.ones((), device=dev)
    head_backward(dl, go, h2, w2, dW2, db2, dH=d2, dbprev=dbp)
    dW1 = torch.empty(H, H, device=dev)
    dW0 = torch.empty(H, D0, device=dev)
    n = H * D0 + H * H + C * H + 2 * H + C
    p = torch.randn(n, device=dev) * 0.01
    mb = torch.zeros(n, device=dev)
    gg = torch.randn(n, device=dev) * 0.01
    sh = torch.empty(n, dtype=bf, device=dev)
    lr = torch.full((), 0.01, device=dev)
    d1 = torch.empty_like(h1)

    cases = {}
    for tile in (-1, 12, 18):
        cases[f"fwd0_t{tile}"] = lambda tile=tile: G.linear_fwd(x, w0, b0, relu=True, out=h1, tile=tile)
        cases[f"fwd1_t{tile}"] = lambda tile=tile: G.linear_fwd(h1, w1, b1, relu=True, out=h2, tile=tile)
        cases[f"dgrad1_t{tile}"] = lambda tile=tile: G.linear_dgrad(d2, w1, relu_mask_of=h1, out=d1, tile=tile)
    # warp-specialised split-K tiles (cfg 16: 256x128 8 math + 4 loader waves; 17: 128x128 4 + 4)
    for tile, sp in ((14, 2),):
        cases[f"fwd0_t{tile}s{sp}"] = lambda tile=tile, sp=sp: G.linear_fwd(x, w0, b0, relu=True, out=h1, tile=tile,
                                                                             splits=sp)
        cases[f"fwd1_t{tile}s{sp}"] = lambda tile=tile, sp=sp: G.linear_fwd(h1, w1, b1, relu=True, out=h2, tile=tile,
                                                                             splits=sp)
        cases[f"dgrad1_t{tile}s{sp}"] = lambda tile=tile, sp=sp: G.linear_dgrad(d2, w1, relu_mask_of=h1, out=d1,
                                                                                tile=tile, splits=sp)
    for tile in (-1, 13, 5, 1, 0):
        cases[f"wgrad1_t{tile}"] = lambda tile=tile: G.linear_wgrad(d2, h1, dW1, tile=tile)
        cases[f"wgrad0_t{tile}"] = lambda tile=tile: G.linear_wgrad(d1, x, dW0, tile=tile)
    mb1 = torch.zeros(H * H, device=dev)
    mb0 = torch.zeros(H * D0, device=dev)
    pw1 = torch.randn(H * H, device=dev) * 0.01
    pw0 = torch.randn(H * D0, device=dev) * 0.01
    sw1 = torch.empty(H * H, dtype=bf, device=dev)
    sw0 = torch.empty(H * D0, dtype=bf, device=dev)
    cases["wgrad1_sgd"] = lambda: G.linear_wgrad(d2, h1, None, sgd=(pw1, mb1, sw1, lr, 0.9, 5e-4))
    cases["wgrad0_sgd"] = lambda: G.linear_wgrad(d1, x, None, sgd=(pw0, mb0, sw0, lr, 0.9, 5e-4))
    cases["wgrad_pair_sgd"] = lambda: G.wgrad_sgd_pair(d2, h1, (pw1, mb1, sw1, lr, 0.9, 5e-4),
                                                       d1, x, (pw0, mb0, sw0, lr, 0.9, 5e-4))
    cases["head_fwd"] = lambda: head_forward(h2, w2, b2, t, want_logits=False)
    cases["head_bwd"] = lambda: head_backward(dl, go, h2, w2, dW2, db2, dH=d2, dbprev=dbp)
    cases["sgd_flat"] = lambda: sgd_flat_(p, mb, gg, sh, lr, 0.9, 5e-4)
    graphs = {k: graph_of(f, a.inner) for k, f in cases.items()}
    res = {k: [] for k in cases}
    for _ in range(a.rounds):
        for k, g in graphs.items():
            res[k].append(time_graph(g, a.inner))
    out = {k: round(sorted(v)[len(v) // 2], 2) for k, v in res.items()}
    for k, v in out.items():
        print(f"{k:16s} {v:8.2f} us", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
