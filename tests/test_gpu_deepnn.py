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
    """dz, dbias of out = [pool](act), act = relu(y + bias) stored bf16 (the conv epilogue's output): routing and
    ReLU mask from act alone, vs torch autograd through relu(y + bias) [+ max_pool2d]."""
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
    act = torch.relu(y + bias).to(torch.bfloat16).contiguous()
    out = K.bn_apply(act, plan.ones, plan.zeros, N, H, H, C, relu=False, pool=True) if pool else act
    yn = y.view(N, H, H, C).permute(0, 3, 1, 2).clone().requires_grad_(True)
    br = bias.clone().requires_grad_(True)
    zr = F.relu(yn + br.view(1, C, 1, 1))
    # the pool routes on the STORED bf16 activation (as torch's autocast pool does): straight-through rounding
    z = zr + (zr.to(torch.bfloat16).float() - zr).detach()
    if pool:
        z = F.max_pool2d(z, 2)
    assert _rel(out.view(N, *z.shape[2:], C).permute(0, 3, 1, 2), z) < 1e-2
    g = _bf(torch.randn_like(z))
    z.backward(g)
    db = torch.empty(C, device=gpu)
    dy = bias_act_backward(g.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous(), act, N, H, H, C, pool, plan, db)
    assert _rel(db, br.grad) < 1e-2
    assert _rel(dy.view(N, H, H, C).permute(0, 3, 1, 2), yn.grad) < 1e-2
    # the same sum applied as the bias's fused SGD update (no momentum history: p -= lr * (g + wd p))
    p0 = torch.randn(C, device=gpu)
    p1, buf = p0.clone(), torch.zeros(C, device=gpu)
    lr = torch.full((), 0.1, device=gpu)
    bias_act_backward(g.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous(), act, N, H, H, C, pool, plan,
                      sgd=(p1, buf, None, lr, 0.9, 5e-4))
    d = db + 5e-4 * p0
    assert torch.allclose(p1, p0 - 0.1 * d, atol=1e-6) and torch.allclose(buf, d, atol=1e-6)


@pytest.mark.parametrize("shape", [(8, 16, 16, 64, 32), (4, 32, 32, 8, 128), (2, 8, 8, 64, 64)])
def test_conv_bias_relu_epilogue_and_masked_dgrad(gpu, shape):
    """DeepNN's fused conv epilogues vs torch fp32: act = relu(conv(x) + b) (EPI_BIAS_RELU_BF16), and the data
    gradient masked by the ReLU of the block below with its bias-gradient column sums (EPI_RELUMASK_BF16 +
    per-tile partials finished in fixed order, stored or applied as SGD)."""
    from ddpx.ops import conv as K
    N, H, W, C, Co = shape
    torch.manual_seed(7)
    x = _bf(torch.randn(N, C, H, W, device=gpu))
    w = torch.randn(Co, C, 3, 3, device=gpu) * (1.0 / (9 * C) ** 0.5)
    b = torch.randn(Co, device=gpu) * 0.2
    wf = torch.empty(Co * 9 * C, dtype=torch.bfloat16, device=gpu)
    wd = torch.empty_like(wf)
    K.weight_prep(w.contiguous(), wf, wd)
    xh = x.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16)
    act = K.conv_fwd_act(xh, wf, Co, b)
    ref = torch.relu(F.conv2d(x, _bf(w), b, padding=1))
    assert _rel(act.view(N, H, W, Co).permute(0, 3, 1, 2), ref) < 1e-2
    # data gradient of this conv, masked by the ReLU of a block below whose activation is `below`
    below = torch.relu(_bf(torch.randn(N, H, W, C, device=gpu))).to(torch.bfloat16).contiguous()
    dy = _bf(torch.randn(N * H * W, Co, device=gpu)).to(torch.bfloat16)
    dz, (part, T) = K.conv_dgrad_act(dy, wd, N, H, W, C, Co, below.view(N * H * W, C))
    dyn = dy.float().view(N, H, W, Co).permute(0, 3, 1, 2)
    dx = torch.nn.grad.conv2d_input((N, C, H, W), _bf(w), dyn, padding=1)
    mask = (below.float().permute(0, 3, 1, 2) > 0).float()
    refz = dx * mask
    assert _rel(dz.view(N, H, W, C).permute(0, 3, 1, 2), refz) < 1e-2
    db = torch.empty(C, device=gpu)
    K.colsum_finish(part, T, C, out=db)
    assert _rel(db, dz.float().sum(0)) < 1e-5
    K.colsum_finish(part, T, C, out=db, accumulate=True)
    assert _rel(db, 2 * dz.float().sum(0)) < 1e-5


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
