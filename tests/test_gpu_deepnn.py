"""Native DeepNN (conv+bias+ReLU(+pool) blocks, Linear, Philox dropout, fused head) vs PyTorch fp32."""
import copy

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


def _pair(gpu, seed=0, p=None):
    import ddpx
    from ddpx.models import DeepNN
    torch.manual_seed(seed)
    m = DeepNN()
    ref = DeepNN()
    ref.load_state_dict(m.state_dict())
    if p is not None:
        m.classifier[2].p = p
        ref.classifier[2].p = p
    m.use_native = True
    ddpx.prepare_model(m, gpu)
    ref.to(gpu)
    return m, ref


@pytest.mark.parametrize("pool", [False, True])
def test_bias_relu_pool_backward(gpu, pool):
    from ddpx.ops import conv as K
    from ddpx.ops.deepnn_native import bias_act_backward

    class _P:
        pass
    plan = _P()
    torch.manual_seed(4)
    N, H, C = 8, 8, 32
    plan.ones = torch.ones(C, device=gpu)
    plan.zeros = torch.zeros(C, device=gpu)
    y = _bf(torch.randn(N * H * H, C, device=gpu))
    bias = torch.randn(C, device=gpu) * 0.3
    out = K.bn_apply(y.to(torch.bfloat16).contiguous(), plan.ones, bias, N, H, H, C, relu=True, pool=pool)
    yn = y.view(N, H, H, C).permute(0, 3, 1, 2).clone().requires_grad_(True)
    br = bias.clone().requires_grad_(True)
    z = F.relu(yn + br.view(1, C, 1, 1))
    if pool:
        z = F.max_pool2d(z, 2)
    assert _rel(out.permute(0, 3, 1, 2), z) < 1e-2
    g = _bf(torch.randn_like(z))
    z.backward(g)
    db = torch.empty(C, device=gpu)
    dy = bias_act_backward(g.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous(), y.to(torch.bfloat16).contiguous(),
                           bias, N, H, H, C, pool, plan, db)
    assert _rel(db, br.grad) < 1e-2
    assert _rel(dy.view(N, H, H, C).permute(0, 3, 1, 2), yn.grad) < 1e-2


def test_dropout_kernel_statistics_and_graph(gpu):
    from ddpx.ops.deepnn_native import dropout_

    class _P:
        pass
    plan = _P()
    plan.rng = torch.tensor([1234, 0], dtype=torch.int64, device=gpu)
    plan.rng_done = torch.zeros(1, dtype=torch.int32, device=gpu)
    x = torch.ones(512, 4096, device=gpu, dtype=torch.bfloat16)
    a = dropout_(x, 0.1, plan)
    b = dropout_(x, 0.1, plan)
    torch.cuda.synchronize()
    assert int(plan.rng[1]) == 2 and int(plan.rng_done[0]) == 0
    keep = (a > 0).float().mean().item()
    assert abs(keep - 0.9) < 5e-3, keep
    kept = a[a > 0].float()
    assert torch.allclose(kept, torch.full_like(kept, 1 / 0.9), rtol=1e-2)
    assert not torch.equal(a, b)  # the offset advanced: a fresh mask
    # same (seed, offset) -> same mask (deterministic)
    plan.rng[1] = 0
    a2 = dropout_(x, 0.1, plan)
    assert torch.equal(a, a2)
    # captured in a graph, every replay draws a new mask
    out = torch.empty_like(x)
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        with torch.cuda.graph(g):
            dropout_(x, 0.1, plan, out=out)
    torch.cuda.current_stream().wait_stream(s)
    g.replay()
    m1 = out.clone()
    g.replay()
    torch.cuda.synchronize()
    assert not torch.equal(m1, out)
    # one kernel statistic per row: no row is systematically dropped
    rows = (out > 0).float().mean(1)
    assert rows.min().item() > 0.8 and rows.max().item() < 0.97


@pytest.mark.parametrize("shape", [(512, 8, 8, 32), (3, 5, 7, 24)])
def test_bf16_nchw_flatten_both_ways(gpu, shape):
    """The native classifier-input flatten: NHWC -> torch's (C, H, W) order and back, bit for bit."""
    from ddpx.ops.deepnn_native import _nchw_flatten
    N, H, W, C = shape
    x = torch.randn(N, H, W, C, device=gpu).to(torch.bfloat16)
    f = _nchw_flatten(x)
    assert torch.equal(f, x.permute(0, 3, 1, 2).reshape(N, C * H * W))
    assert torch.equal(_nchw_flatten(f, (N, H, W, C)), x)


def test_deepnn_native_matches_torch(gpu):
    """Whole native DeepNN (bf16) vs torch fp32 with dropout disabled (p = 0 on both), error budget set by
    torch's own bf16 autocast error on the same batch."""
    torch.manual_seed(5)
    m, ref = _pair(gpu, seed=5, p=0.0)
    amp = copy.deepcopy(ref)
    N = 64
    x = _bf(torch.rand(N, 3, 32, 32, device=gpu))
    t = torch.randint(0, 10, (N,), device=gpu)
    loss, _ = m.forward_loss(x, t)
    loss.backward()
    rl = F.cross_entropy(ref(x), t)
    rl.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        al = F.cross_entropy(amp(x).float(), t)
    al.backward()
    assert abs(loss.item() - rl.item()) < 2e-2 * max(1.0, rl.item())
    for (n, p), (_, q), (_, r) in zip(m.named_parameters(), ref.named_parameters(), amp.named_parameters()):
        ours, theirs = _rel(p.main_grad, q.grad), _rel(r.grad, q.grad)
        assert ours < 3 * theirs + 0.03, (n, ours, theirs)
    m.eval()
    ref.eval()
    with torch.no_grad():
        assert _rel(m(x), ref(x)) < 3e-2


def test_deepnn_dropout_training_semantics(gpu):
    """Dropout 0.1 active: the native backward must equal torch's backward for the SAME mask.  The mask is
    recovered from the native forward (kept = dropped activation > 0 where the ReLU output is > 0)."""
    from ddpx.ops import deepnn_native as D
    torch.manual_seed(6)
    m, ref = _pair(gpu, seed=6)
    amp = copy.deepcopy(ref)
    m.train()
    N = 64
    x = _bf(torch.rand(N, 3, 32, 32, device=gpu))
    t = torch.randint(0, 10, (N,), device=gpu)
    xi = D._prep_input(x)
    saved, last, loss, _, dl = D._forward(m, xi, t, False, True, True)
    _, feat, d0, scale = last
    assert abs(scale - 1 / 0.9) < 1e-6
    # torch replica with the mask the kernel drew
    f = ref.features(x).flatten(1)
    a0 = F.relu(ref.classifier[0](f))
    mask = (d0.float() > 0).float()
    live = (a0 > 0).float()
    frac = (mask.sum() / live.sum()).item()
    assert 0.85 < frac < 0.95, frac
    out = ref.classifier[3](a0 * mask * scale)
    rl = F.cross_entropy(out, t)
    assert abs(loss.item() - rl.item()) < 3e-2 * max(1.0, rl.item())
    rl.backward()
    # error budget: torch's own bf16 autocast run of the same masked network
    with torch.autocast("cuda", dtype=torch.bfloat16):
        fa = amp.features(x).flatten(1)
        aa = F.relu(amp.classifier[0](fa))
        al = F.cross_entropy(amp.classifier[3](aa * mask * scale).float(), t)
    al.backward()
    D._backward(m, saved, last, dl, torch.ones((), device=gpu))
    for (n, p), (_, q), (_, r) in zip(m.named_parameters(), ref.named_parameters(), amp.named_parameters()):
        ours, theirs = _rel(p.main_grad, q.grad), _rel(r.grad, q.grad)
        assert ours < 3 * theirs + 0.03, (n, ours, theirs)


def test_deepnn_fused_optimizer_bitwise(gpu):
    """Optimizer fused into the backward kernels == separate SGD step (same dropout masks: same seeds)."""
    from ddpx.optim.sgd import SGD
    a, _ = _pair(gpu, seed=7)
    b, _ = _pair(gpu, seed=7)
    b._ddpx_plan = None
    from ddpx.ops.deepnn_native import plan_of
    plan_of(a)
    plan_of(b).rng.copy_(a._ddpx_plan.rng)
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, fused_backward=True)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    for i in range(3):
        x = torch.rand(32, 3, 32, 32, device=gpu)
        t = torch.randint(0, 10, (32,), device=gpu)
        for m, o in ((a, oa), (b, ob)):
            o.sync_lr()
            o.zero_grad()
            loss, _ = m.forward_loss(x, t)
            loss.backward()
            o.step()
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p, q), n


def test_deepnn_trains_through_entrypoint(gpu, tmp_path):
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    r = subprocess.run([sys.executable, os.path.join(root, "singlegpu.py"), "2", "1", "--model", "deepnn", "--data",
                        "synthetic", "--train_size", "2048", "--test_size", "512", "--graph", "--dtype", "bf16"],
                       cwd=tmp_path, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "fp32 model has size=4.53 MiB" in r.stdout
    sd = torch.load(tmp_path / "checkpoint.pt", weights_only=True)
    from ddpx.models import DeepNN
    DeepNN().load_state_dict(sd, strict=True)
