"""Per-step loss of the toy MLP: ddpx fp32 grads vs ddpx bf16 grads vs torch autocast (same init/data)."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(kind, steps=130):
    from ddpx.data.datasets import synthetic_cifar
    from ddpx.data.loader import DeviceLoader
    from ddpx.data.sampler import DistributedIndexSampler
    from ddpx.models import build_model
    from ddpx.optim.schedule import one_cycle, resolve_steps_per_epoch, OneCycleLambda
    from ddpx.optim.sgd import SGD
    from ddpx.runtime.setup import prepare_model
    dev = torch.device("cuda")
    ds = synthetic_cifar(50000, seed=0)
    sampler = DistributedIndexSampler(len(ds), 1, 0, shuffle=True, seed=0)
    layout = "flat_bf16" if kind != "torch" else "nchw_f32"
    loader = DeviceLoader(ds, 512, dev, sampler=sampler, train=True, layout=layout, seed=0)
    idx = loader._epoch_indices()
    torch.manual_seed(0)
    model = build_model("mlp", hidden=4096, layers=3, dtype="bf16", device=dev)
    losses = []
    if kind == "torch":
        import torch.nn as nn
        torch.manual_seed(0)
        ref = nn.Sequential(nn.Flatten(), nn.Linear(3072, 4096), nn.ReLU(), nn.Linear(4096, 4096), nn.ReLU(),
                            nn.Linear(4096, 10)).to(dev)
        opt = torch.optim.SGD(ref.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4)
        sched = torch.optim.lr_scheduler.LambdaLR(opt, OneCycleLambda(resolve_steps_per_epoch("compat", 0, False)))
        for k in range(steps):
            b = k % (idx.numel() // 512)
            x, y = loader.make_batch(idx[b * 512:(b + 1) * 512], k)
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                out = ref(x)
            loss = torch.nn.functional.cross_entropy(out.float(), y)
            loss.backward()
            opt.step()
            sched.step()
            losses.append(loss.item())
        return losses
    gd = torch.bfloat16 if kind == "bf16" else torch.float32
    prepare_model(model, dev, grad_dtype=gd)
    opt = SGD(model.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4, capturable=False,
              fused_backward=(kind == "fused"))
    sched = one_cycle(opt, resolve_steps_per_epoch("compat", 0, False))
    for k in range(steps):
        b = k % (idx.numel() // 512)
        x, y = loader.make_batch(idx[b * 512:(b + 1) * 512], k)
        opt.sync_lr()
        opt.zero_grad()
        loss, _ = model.forward_loss(x, y)
        loss.backward()
        opt.step()
        sched.step()
        losses.append(loss.item())
    return losses


if __name__ == "__main__":
    res = {k: run(k) for k in ("torch", "fp32", "bf16", "fused")}
    for k, v in res.items():
        print(k, [round(x, 3) for x in v[::10]])
    with open("gpurun_out/grad_dtype_drift.json", "w") as f:
        json.dump(res, f)
