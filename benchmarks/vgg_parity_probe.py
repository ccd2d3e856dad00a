#!/usr/bin/env python3
"""Spread of the bf16 VGG training trajectory (tests/test_gpu_parity.py's setup) across runs that differ only in
summation order: torch fp32 (twice), torch bf16 autocast (twice), and the native bf16 path under each BatchNorm
merge order (ddpx_bn_set_merge: legacy / split / bwd).  Prints one JSON line per run: last-20 mean loss and
test accuracy.  ``--seeds N``: repeat for initialisations / batch orders 0..N-1 (torch fp32 once per seed, no
autocast runs): the seed-to-seed spread the multi-seed parity test (tests/test_gpu_parity.py) is judged against.

    python benchmarks/vgg_parity_probe.py [--steps 100] [--batch 128] [--seeds 1]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--batch", type=int, default=128)
    ap.add_argument("--seeds", type=int, default=1)
    ap.add_argument("--noise", type=float, default=230.0)
    ap.add_argument("--merges", default="legacy,split,bwd", help="native BN merge orders to run")
    a = ap.parse_args()
    import ddpx
    from ddpx.data.datasets import synthetic_cifar
    from ddpx.data.loader import DeviceLoader
    from ddpx.models import VGG
    from ddpx.optim.schedule import OneCycleLambda
    from ddpx.optim.sgd import SGD
    from ddpx.runtime import native
    from test_gpu_parity import _accuracy, _train
    gpu = torch.device("cuda", 0)
    steps, B = a.steps, a.batch
    ref = VGG().to(gpu)
    train = synthetic_cifar(8192, seed=0, noise=a.noise)
    test = synthetic_cifar(2048, seed=0, noise=a.noise, split_seed_offset=7)
    lam = OneCycleLambda(steps_per_epoch=steps // 20, num_epochs=20)

    def torch_run(amp, init, seed):
        ref.load_state_dict(init)
        o = torch.optim.SGD(ref.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4)
        s = torch.optim.lr_scheduler.LambdaLR(o, lam)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            loss = _train(ref, DeviceLoader(train, B, gpu, layout="nchw_f32", seed=seed), o, s, steps, False)
        return loss, _accuracy(ref, DeviceLoader(test, B, gpu, train=False, layout="nchw_f32"))

    def native_run(merge, init, seed):
        if merge is not None:
            native.kernels().ddpx_bn_set_merge(merge)
        nat = VGG()
        nat.load_state_dict(init)
        nat.use_native = True
        ddpx.prepare_model(nat, gpu)
        o = SGD(nat.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4, fused_backward=True)
        s = torch.optim.lr_scheduler.LambdaLR(o, lam)
        loss = _train(nat, DeviceLoader(train, B, gpu, layout="nhwc8_bf16", seed=seed), o, s, steps, True)
        return loss, _accuracy(nat, DeviceLoader(test, B, gpu, train=False, layout="nhwc8_bf16"))

    for seed in range(a.seeds):
        torch.manual_seed(seed)
        init = {k: v.to(gpu) for k, v in VGG().state_dict().items()}
        if a.seeds == 1:
            runs = [("torch_fp32", lambda: torch_run(False, init, seed)), ("torch_fp32", lambda: torch_run(False, init, seed)),
                    ("torch_bf16_autocast", lambda: torch_run(True, init, seed)),
                    ("torch_bf16_autocast", lambda: torch_run(True, init, seed))]
        else:
            runs = [("torch_fp32", lambda: torch_run(False, init, seed))]
        for name, m in (("legacy", 1), ("split", 0), ("bwd", 2)):
            if name in a.merges.split(","):
                runs.append(("native_bf16_merge_" + name, lambda m=m: native_run(m, init, seed)))
        for name, fn in runs:
            loss, acc = fn()
            print(json.dumps({"run": name, "seed": seed, "batch": B, "noise": a.noise, "steps": steps, "tail20": round(loss[-20:].mean().item(), 4),
                              "head10": round(loss[:10].mean().item(), 4), "test_acc": round(acc, 2)}), flush=True)
        native.kernels().ddpx_bn_set_merge(-1)


if __name__ == "__main__":
    main()
