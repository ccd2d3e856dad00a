"""Diagnose the scaled-MFMA operand/scale map: dumps probe results for several patterns."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ddpx.ops.fp8 import MX, _TORCH_FP8, probe  # noqa: E402

dev = torch.device("cuda")
out = {}
g = torch.Generator().manual_seed(0)


def codes(v, fmt=0):
    return v.float().to(_TORCH_FP8[fmt]).view(torch.uint8).to(dev)


def run(name, A, B, sa, sb, fa=0):
    C = probe(codes(A, fa), codes(B), sa.to(torch.uint8).to(dev), sb.to(torch.uint8).to(dev), fa).cpu()
    ref = MX(codes(A, fa).cpu(), sa.to(torch.uint8), fa).dequant() @ MX(codes(B).cpu(), sb.to(torch.uint8), 0).dequant().t()
    out[name] = {"maxerr": (C - ref).abs().max().item(), "C": C.tolist(), "ref": ref.tolist()}
    print(name, out[name]["maxerr"])


A = torch.randint(-6, 7, (16, 128), generator=g)
B = torch.randint(-6, 7, (16, 128), generator=g)
one = torch.full((16, 4), 127)
run("unit_scales", A, B, one, one)
# A row index in value, B ones: C[m][n] = sum_k A[m][k]
run("rowsum", A, torch.ones(16, 128), one, one)
# block structure: A ones; B one-hot in k-block
for kb in range(4):
    Bk = torch.zeros(16, 128)
    Bk[:, kb * 32:(kb + 1) * 32] = 1
    run(f"kblock{kb}_unitscale", torch.ones(16, 128), Bk, one, one)
sa = torch.randint(124, 130, (16, 4), generator=g)
run("scaleA_only", A, B, sa, one)
run("scaleB_only", A, B, one, sa)
with open("gpurun_out/mx_probe.json", "w") as f:
    json.dump(out, f)
