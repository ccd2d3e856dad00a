"""Training-outcome parity: the native bf16 VGG trained by ddpx vs stock PyTorch fp32 VGG.

The reference validates only the end-of-training accuracy (``/root/reference/singlegpu.py:248-249``,
VGG of ``singlegpu.py:60-82``, SGD lr 0.4 / momentum 0.9 / wd 5e-4 with the triangular one-cycle of
``singlegpu.py:136-149``).  Both models start from the same weights, see the same batches (the GPU
augment kernel is bitwise equal to its CPU twin, ``tests/test_gpu_kernels.py::test_augment_matches_cpu``)
and follow the same one-cycle compressed to the run length; the ddpx side runs its production path
(native NHWC bf16 kernels, flat fp32 master weights, fused SGD in the backward epilogues).

CIFAR-10 is not on the box, so the data are the learnable synthetic CIFAR-shaped set
(``ddpx.data.datasets.synthetic_cifar``): accuracy parity on CIFAR-10 itself stays unpinned.
"""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _train(model, loader, opt, sched, steps, native):
    idx = loader._epoch_indices()
    B = loader.batch_size
    nb = idx.numel() // B
    losses = []
    for k in range(steps):
        x, y = loader.make_batch(idx[(k % nb) * B:(k % nb + 1) * B], k)
        if hasattr(opt, "sync_lr"):
            opt.sync_lr()  # host LambdaLR value -> the device scalar the fused epilogues read
        opt.zero_grad()
        if native:
            loss, _ = model.forward_loss(x, y)
        else:
            loss = torch.nn.functional.cross_entropy(model(x), y)
        loss.backward()
        opt.step()
        sched.step()
        losses.append(loss.detach())
    return torch.stack(losses).float().cpu()


@torch.inference_mode()
def _accuracy(model, loader):
    model.eval()
    idx = loader._epoch_indices()
    B = loader.batch_size
    hit = n = 0
    for s in range(0, idx.numel() - B + 1, B):
        x, y = loader.make_batch(idx[s:s + B], s // B)
        hit += int((model(x).float().argmax(1) == y).sum())
        n += B
    model.train()
    return 100.0 * hit / n


SEEDS = tuple(range(8))


def test_vgg_native_bf16_trains_like_torch_fp32(gpu):
    """Outcome parity over an ensemble of initialisations / batch orders, not one trajectory.

    A single trajectory of this short, noisy run is chaotic: the native bf16 run from one init moved from 0.53
    to 0.71 last-20 loss with nothing but the summation order of the BatchNorm statistics, torch fp32 itself is
    not reproducible run to run, and at batch 128 some seeds of either engine fail to learn within the run
    (``profiles/r4_parity``).  So each seed trains both engines from the same weights on the same batches, at
    the reference's batch size (512, where the seeds learn), and the bar is on the ensemble: native bf16 must
    not end worse than torch fp32 — mean last-20 loss at most 25 % above fp32's, mean test accuracy at most 4
    points below, each margin widened by two standard errors of the mean paired difference (one pair's
    difference has a spread of ~0.25 in loss / ~9 points in accuracy) — and never beyond hard caps (loss within
    50 % either way, accuracy within 10 points)."""
    import math

    import ddpx
    from ddpx.data.datasets import synthetic_cifar
    from ddpx.data.loader import DeviceLoader
    from ddpx.models import VGG
    from ddpx.optim.schedule import OneCycleLambda
    from ddpx.optim.sgd import SGD

    steps, B = 100, 512
    # heavy pixel noise and a short run: the default set (noise 60) is separated perfectly within a few
    # epochs (loss 1e-4 after 300 steps), which would make any two trainers agree; this stops mid-way
    train = synthetic_cifar(8192, seed=0, noise=230.0)
    test = synthetic_cifar(2048, seed=0, noise=230.0, split_seed_offset=7)
    # one-cycle over the whole run: 20 "epochs" of steps/20 batches
    lam = OneCycleLambda(steps_per_epoch=steps // 20, num_epochs=20)

    rows = []
    fails_ref = fails_nat = 0
    for seed in SEEDS:
        torch.manual_seed(seed)
        ref = VGG().to(gpu)
        nat = VGG()
        nat.load_state_dict(ref.state_dict())
        nat.use_native = True
        ddpx.prepare_model(nat, gpu)
        assert nat.input_layout(gpu) == "nhwc8_bf16"

        o_ref = torch.optim.SGD(ref.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4)
        s_ref = torch.optim.lr_scheduler.LambdaLR(o_ref, lam)
        l_ref = _train(ref, DeviceLoader(train, B, gpu, layout="nchw_f32", seed=seed), o_ref, s_ref, steps, False)
        a_ref = _accuracy(ref, DeviceLoader(test, B, gpu, train=False, layout="nchw_f32"))

        o_nat = SGD(nat.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4, fused_backward=True)
        s_nat = torch.optim.lr_scheduler.LambdaLR(o_nat, lam)
        l_nat = _train(nat, DeviceLoader(train, B, gpu, layout="nhwc8_bf16", seed=seed), o_nat, s_nat, steps, True)
        a_nat = _accuracy(nat, DeviceLoader(test, B, gpu, train=False, layout="nhwc8_bf16"))
        torch.cuda.synchronize()

        assert torch.isfinite(l_nat).all() and torch.isfinite(l_ref).all()
        learned = lambda l, a: l[-20:].mean().item() < 0.8 * l[:10].mean().item() and a > 30.0  # noqa: E731
        fails_ref += not learned(l_ref, a_ref)
        fails_nat += not learned(l_nat, a_nat)
        rows.append((l_ref[-20:].mean().item(), l_nat[-20:].mean().item(), a_ref, a_nat))
        print(f"\nseed {seed}: loss last-20 fp32 {rows[-1][0]:.4f} native {rows[-1][1]:.4f}; "
              f"test accuracy fp32 {a_ref:.2f}% native {a_nat:.2f}%")

    n = len(rows)
    # both engines learn the task (a run that does not is a seed-level event at lr 0.4: allow one per engine)
    assert fails_ref <= 1 and fails_nat <= 1, (fails_ref, fails_nat, rows)

    def mean_sd(v):
        m = sum(v) / len(v)
        return m, math.sqrt(sum((x - m) ** 2 for x in v) / (len(v) - 1))

    tail_ref, _ = mean_sd([r[0] for r in rows])
    tail_nat, _ = mean_sd([r[1] for r in rows])
    acc_ref, _ = mean_sd([r[2] for r in rows])
    acc_nat, _ = mean_sd([r[3] for r in rows])
    _, sd_dt = mean_sd([r[1] - r[0] for r in rows])
    _, sd_da = mean_sd([r[3] - r[2] for r in rows])
    print(f"\nmean over {n} seeds: loss fp32 {tail_ref:.4f} native {tail_nat:.4f} (paired sd {sd_dt:.4f}); "
          f"accuracy fp32 {acc_ref:.2f}% native {acc_nat:.2f}% (paired sd {sd_da:.2f})")
    # the same outcome: bf16 compute vs fp32 changes each trajectory, not where the ensemble ends
    se_t, se_a = sd_dt / math.sqrt(n), sd_da / math.sqrt(n)
    assert tail_nat < tail_ref + max(0.05, 0.25 * tail_ref) + 2.0 * se_t, rows
    assert acc_nat > acc_ref - 4.0 - 2.0 * se_a, rows
    assert abs(tail_nat - tail_ref) < max(0.1, 0.5 * tail_ref), rows
    assert abs(acc_nat - acc_ref) < 10.0, rows
