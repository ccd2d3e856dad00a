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


def test_vgg_native_bf16_trains_like_torch_fp32(gpu):
    import ddpx
    from ddpx.data.datasets import synthetic_cifar
    from ddpx.data.loader import DeviceLoader
    from ddpx.models import VGG
    from ddpx.optim.schedule import OneCycleLambda
    from ddpx.optim.sgd import SGD

    steps, B = 100, 128
    torch.manual_seed(0)
    ref = VGG().to(gpu)
    nat = VGG()
    nat.load_state_dict(ref.state_dict())
    nat.use_native = True
    ddpx.prepare_model(nat, gpu)
    assert nat.input_layout(gpu) == "nhwc8_bf16"

    # heavy pixel noise and a short run: the default set (noise 60) is separated perfectly within a few
    # epochs (loss 1e-4 after 300 steps), which would make any two trainers agree; this stops mid-way
    train = synthetic_cifar(8192, seed=0, noise=230.0)
    test = synthetic_cifar(2048, seed=0, noise=230.0, split_seed_offset=7)
    # one-cycle over the whole run: 20 "epochs" of steps/20 batches
    lam = OneCycleLambda(steps_per_epoch=steps // 20, num_epochs=20)

    # the stock fp32 reference is not bitwise reproducible on the GPU (MIOpen / hipBLASLt algorithm choice and
    # reduction order): two runs from the same weights measured tail losses 0.47-0.56 and test accuracies
    # 86.5-90.1 % (profiles/r3_bn/NOTES.md).  The reference band below is widened by the spread of two runs.
    init = {k: v.clone() for k, v in ref.state_dict().items()}
    refs = []
    for _ in range(2):
        ref.load_state_dict(init)
        o_ref = torch.optim.SGD(ref.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4)
        s_ref = torch.optim.lr_scheduler.LambdaLR(o_ref, lam)
        l_ref = _train(ref, DeviceLoader(train, B, gpu, layout="nchw_f32", seed=0), o_ref, s_ref, steps, False)
        refs.append((l_ref, _accuracy(ref, DeviceLoader(test, B, gpu, train=False, layout="nchw_f32"))))

    o_nat = SGD(nat.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4, fused_backward=True)
    s_nat = torch.optim.lr_scheduler.LambdaLR(o_nat, lam)
    l_nat = _train(nat, DeviceLoader(train, B, gpu, layout="nhwc8_bf16", seed=0), o_nat, s_nat, steps, True)
    torch.cuda.synchronize()

    assert torch.isfinite(l_nat).all() and all(torch.isfinite(lr_).all() for lr_, _ in refs)
    tails = [lr_[-20:].mean().item() for lr_, _ in refs]
    accs = [a for _, a in refs]
    tail_ref, acc_ref = sum(tails) / 2, sum(accs) / 2
    tail_nat = l_nat[-20:].mean().item()
    acc_nat = _accuracy(nat, DeviceLoader(test, B, gpu, train=False, layout="nhwc8_bf16"))
    print(f"\nloss last-20 ref {tails[0]:.4f} / {tails[1]:.4f} native {tail_nat:.4f}; test accuracy ref "
          f"{accs[0]:.2f}% / {accs[1]:.2f}% native {acc_nat:.2f}%")
    # both learn the task ...
    for lr_, a in refs:
        assert lr_[-20:].mean().item() < 0.8 * lr_[:10].mean().item() and a > 30.0
    # ... and end in the same place: bf16 compute vs fp32 changes the trajectory, not the outcome
    assert abs(tail_nat - tail_ref) < max(0.05, 0.25 * tail_ref) + abs(tails[0] - tails[1]), (tail_nat, tails)
    assert abs(acc_nat - acc_ref) < 5.0 + abs(accs[0] - accs[1]), (acc_nat, accs)
