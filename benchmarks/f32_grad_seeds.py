#!/usr/bin/env python3
"""fp32 VGG gradient error vs fp64 over several seeds: native Winograd, native direct, torch fp32 (MIOpen).

    python benchmarks/f32_grad_seeds.py [--seeds 6] [--out FILE]

Below a 2x2 max-pool a gradient moves by ~2e-3 per routing flip (two window candidates within fp32 round-off),
so one batch says little about a forward algorithm's precision; this runs the single-batch check of
tests/test_gpu_f32.py::test_native_fp32_gradients_match_torch_fp32 on several seeds and reports, per path, the
largest relative error over the parameters below the last pool.
"""
import argparse
import copy
import json
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / b.norm().clamp_min(1e-30)).item()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seeds", type=int, default=6)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import ddpx
    from ddpx.models import build_model
    from ddpx.ops import f32
    gpu = torch.device("cuda")
    rows = []
    for seed in range(a.seeds):
        torch.manual_seed(seed)
        base = build_model("vgg", dtype="fp32", device=gpu, kernels="native")
        x = torch.rand(64, 3, 32, 32, device=gpu)
        y = torch.randint(0, 10, (64,), device=gpu)
        r64 = copy.deepcopy(base).cpu().double()
        r64.use_native = False
        r64.compute_dtype = torch.float64
        F.cross_entropy(r64(x.cpu().double()), y.cpu()).backward()
        p64 = dict(r64.named_parameters())
        ref = copy.deepcopy(base).to(gpu)
        ref.use_native = False
        F.cross_entropy(ref(x), y).backward()
        errs = {"torch": {n: rel(p.grad.cpu(), p64[n].grad) for n, p in ref.named_parameters()}}
        for mode in ("wino", "direct"):
            f32._WINO = mode == "wino"
            m = copy.deepcopy(base)
            flat = ddpx.prepare_model(m, gpu)
            flat.zero_grad()
            loss, _ = m.forward_loss(x, y)
            loss.backward()
            errs[mode] = {n: rel(p.main_grad.cpu(), p64[n].grad) for n, p in m.named_parameters()}
        f32._WINO = True
        below = [n for n in errs["torch"] if not n.startswith(("classifier", "backbone.bn7"))]
        row = {"seed": seed, **{k: round(max(v[n] for n in below), 6) for k, v in errs.items()}}
        rows.append(row)
        print(json.dumps(row), flush=True)
    for k in ("torch", "wino", "direct"):
        v = sorted(r[k] for r in rows)
        print(f"{k:7s} max-below-pool error over seeds: median {v[len(v) // 2]:.2e}  max {v[-1]:.2e}", flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    main()
