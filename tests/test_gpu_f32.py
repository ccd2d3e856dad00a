"""The fp32 native path (``ddpx.ops.f32`` on ``csrc/kernels/f32_train.hip``) vs fp64 / fp32 torch references.

The reference trains VGG in fp32 (``/root/reference/singlegpu.py:134``); these kernels are exact-f32 MFMA
(f32 products, f32 accumulation), so they are held to fp32 round-off (relative 1e-5 .. 1e-4 against an
fp64 reference), not to bf16 tolerances.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    a, b = a.double(), b.double()
    return ((a - b).norm() / (b.norm() + 1e-30)).item()


@pytest.mark.parametrize("M,N,K", [(512, 4096, 3072), (100, 72, 36), (257, 132, 516)])
def test_linear_fwd_dgrad_wgrad(gpu, M, N, K):
    from ddpx.ops import f32
    torch.manual_seed(0)
    x = torch.randn(M, K, device=gpu)
    w = torch.randn(N, K, device=gpu) / K ** 0.5
    b = torch.randn(N, device=gpu)
    y = f32.linear_fwd(x, w, b, relu=True)
    ref = torch.relu(x.double() @ w.double().t() + b.double())
    assert _rel(y, ref) < 1e-5
    dy = torch.randn(M, N, device=gpu)
    mask = torch.randn(M, K, device=gpu)
    dx = f32.linear_dgrad(dy, w, mask=mask)
    refx = (dy.double() @ w.double()) * (mask > 0)
    assert _rel(dx, refx) < 1e-5
    dW = torch.empty(N, K, device=gpu)
    f32.linear_wgrad(dy, x, dW)
    refw = dy.double().t() @ x.double()
    assert _rel(dW, refw) < 1e-5
    f32.linear_wgrad(dy, x, dW, accumulate=True)
    assert _rel(dW, 2 * refw) < 1e-5
    db = torch.empty(N, device=gpu)
    f32.colsum(dy, db)
    assert _rel(db, dy.double().sum(0)) < 1e-5


@pytest.mark.parametrize("N,H,Ci,Co", [(4, 32, 3, 64), (8, 16, 64, 128), (16, 8, 128, 256), (32, 4, 256, 512),
                                       (64, 2, 512, 512), (2, 32, 64, 64)])
def test_conv_fwd_dgrad_wgrad(gpu, N, H, Ci, Co):
    from ddpx.ops import f32
    torch.manual_seed(0)
    Cp = f32.conv_channels(Ci)
    x = torch.randn(N, Ci, H, H, device=gpu)
    w = torch.randn(Co, Ci, 3, 3, device=gpu) / (Ci * 9) ** 0.5
    xn = F.pad(x.permute(0, 2, 3, 1), (0, Cp - Ci)).contiguous()
    wf = torch.empty(9 * Cp * Co, device=gpu)
    wd = torch.empty(9 * Co * Ci, device=gpu) if Ci % 4 == 0 else None
    f32.conv_wprep(w, wf, wd)
    y = f32.conv_fwd(xn, wf, Co)
    xd, wdd = x.double().cpu(), w.double().cpu()
    ref = F.conv2d(xd, wdd, padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    assert _rel(y.cpu(), ref) < 1e-5
    dy = torch.randn(N * H * H, Co, device=gpu)
    xr = xd.clone().requires_grad_(True)
    wr = wdd.clone().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(dy.double().cpu().view(N, H, H, Co).permute(0, 3, 1, 2))
    dw = torch.empty(Co, Ci, 3, 3, device=gpu)
    f32.conv_wgrad(dy, xn, Co, Ci, dw)
    assert _rel(dw.cpu(), wr.grad) < 1e-5
    if wd is not None:
        dx = f32.conv_dgrad(dy, wd, N, H, H, Ci, Co)
        assert _rel(dx.cpu().permute(0, 3, 1, 2), xr.grad) < 1e-5


@pytest.mark.parametrize("pool", [False, True])
@pytest.mark.parametrize("N,H,C", [(16, 8, 128), (8, 4, 512), (4, 32, 64),
                                   (256, 32, 64)])  # 1024 chunks of 64 channels: the split statistics merge
def test_bn_relu_pool_fwd_bwd(gpu, pool, N, H, C):
    from ddpx.ops import f32
    torch.manual_seed(1)
    y = torch.randn(N * H * H, C, device=gpu) * 2 + 0.5
    bn = torch.nn.BatchNorm2d(C).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.2, 0.2)
    ref_bn = torch.nn.BatchNorm2d(C).double()
    ref_bn.load_state_dict({k: v.double().cpu() if v.is_floating_point() else v.cpu()
                            for k, v in bn.state_dict().items()})
    out, a, b, mean, rstd = f32.bn_forward(y, N, H, H, C, bn, True, pool)
    yr = y.double().cpu().view(N, H, H, C).permute(0, 3, 1, 2).clone().requires_grad_(True)
    z = torch.relu(ref_bn(yr))
    if pool:
        z = F.max_pool2d(z, 2)
    assert _rel(out.cpu().permute(0, 3, 1, 2), z) < 1e-5
    assert _rel(bn.running_mean.cpu(), ref_bn.running_mean) < 1e-5
    assert _rel(bn.running_var.cpu(), ref_bn.running_var) < 1e-5
    assert int(bn.num_batches_tracked) == 1
    g = torch.randn_like(out)
    z.backward(g.double().cpu().permute(0, 3, 1, 2))
    dgam, dbet = torch.empty(C, device=gpu), torch.empty(C, device=gpu)
    dy = f32.bn_backward(g, y, a, b, mean, rstd, N, H, H, C, pool, dgam, dbet)
    assert _rel(dy.cpu().view(N, H, H, C).permute(0, 3, 1, 2), yr.grad) < 1e-4
    assert _rel(dgam.cpu(), ref_bn.weight.grad) < 1e-4
    assert _rel(dbet.cpu(), ref_bn.bias.grad) < 1e-4


def test_head_xent(gpu):
    from ddpx.ops import f32
    torch.manual_seed(2)
    M, K, NC = 300, 512, 10
    h = torch.randn(M, K, device=gpu).relu()
    w = torch.randn(NC, K, device=gpu) / K ** 0.5
    b = torch.randn(NC, device=gpu)
    t = torch.randint(0, NC, (M,), device=gpu)
    loss, logits, dl = f32.head_forward(h, w, b, t)
    hr, wr, br = (v.double().cpu().requires_grad_(True) for v in (h, w, b))
    lr = hr @ wr.t() + br
    ref = F.cross_entropy(lr, t.cpu())
    assert _rel(logits.cpu(), lr.detach()) < 1e-6
    assert abs(loss.item() - ref.item()) < 1e-5
    ref.backward(torch.tensor(0.5, dtype=torch.float64))
    dW, db = torch.empty(NC, K, device=gpu), torch.empty(NC, device=gpu)
    dh = f32.head_backward(dl, torch.tensor(0.5, device=gpu), h, w, dW, db, relu_mask=True)
    assert _rel(dW.cpu(), wr.grad) < 1e-5
    assert _rel(db.cpu(), br.grad) < 1e-5
    assert _rel(dh.cpu(), hr.grad * (hr.detach() > 0)) < 1e-5


def test_augment_nhwc4_f32_matches_cpu(gpu):
    from ddpx.data.loader import augment_cpu, augment_gpu
    torch.manual_seed(3)
    imgs = torch.randint(0, 256, (64, 3, 32, 32), dtype=torch.uint8)
    labels = torch.randint(0, 10, (64,))
    idx = torch.randperm(64)[:32]
    xc, yc = augment_cpu(imgs, labels, idx, 1234, True, 4, "nhwc4_f32")
    xg, yg = augment_gpu(imgs.to(gpu), labels.to(gpu), idx.to(gpu), 1234, True, 4, "nhwc4_f32")
    assert xg.shape == (32, 32, 32, 4)
    assert torch.equal(xg.cpu(), xc)
    assert torch.equal(yg.cpu(), yc)


def _train_pair(gpu, name, steps, lr=0.05, fp64=None):
    """(native fp32 losses, torch fp32 losses, native model, torch model) from one init; with ``fp64`` = a list,
    an fp64 torch copy trained on the same batches is appended to it (the arbiter for both fp32 runs)."""
    import copy

    import ddpx
    from ddpx.models import build_model
    from ddpx.optim.sgd import SGD
    torch.manual_seed(4)
    native = build_model(name, dtype="fp32", device=gpu, hidden=256 if name == "mlp" else None, kernels="native")
    ref = copy.deepcopy(native).to(gpu)
    ref.use_native = False
    ddpx.prepare_model(native, gpu)
    opt = SGD(native.parameters(), lr=lr, momentum=0.9, weight_decay=5e-4)
    ropt = torch.optim.SGD(ref.parameters(), lr=lr, momentum=0.9, weight_decay=5e-4)
    r64 = o64 = None
    if fp64 is not None:
        r64 = copy.deepcopy(ref).double()
        r64.compute_dtype = torch.float64
        o64 = torch.optim.SGD(r64.parameters(), lr=lr, momentum=0.9, weight_decay=5e-4)
        fp64.append(r64)
    gen = torch.Generator().manual_seed(5)
    ln, lt = [], []
    for _ in range(steps):
        x = torch.rand(64, 3, 32, 32, generator=gen).to(gpu)
        y = torch.randint(0, 10, (64,), generator=gen).to(gpu)
        opt.zero_grad()
        loss, logits = native.forward_loss(x, y)
        assert logits is None  # the native fp32 path ran
        loss.backward()
        opt.step()
        ln.append(loss.item())
        ropt.zero_grad()
        rl = F.cross_entropy(ref(x), y)
        rl.backward()
        ropt.step()
        lt.append(rl.item())
        if r64 is not None:
            o64.zero_grad()
            F.cross_entropy(r64(x.double()), y).backward()
            o64.step()
    return ln, lt, native, ref


@pytest.mark.parametrize("name", ["vgg", "mlp"])
def test_native_fp32_gradients_match_torch_fp32(gpu, name):
    """One backward from the same init and batch: every parameter gradient against fp64.

    Above every pooling decision (VGG's classifier; every MLP layer) the gradients are exact to 1e-5.
    Below a 2x2 max-pool a gradient moves by ~2e-3 whenever one of the 131K windows routes to another element
    because two candidates lie within fp32 round-off of each other, so a single batch says little: over 8 seeds
    (benchmarks/f32_grad_seeds.py, profiles/r5_wino) the largest below-pool error of torch's own fp32 run (MIOpen
    Winograd convolutions) has median 4.1e-3 and max 1.0e-2, the native Winograd path 2.8e-3 / 8.9e-3, the native
    direct GEMM 1.4e-3 / 4.1e-3.  The VGG bar is therefore torch's own distribution over 6 batches: the native
    median at most 1.5x torch's, and no batch beyond 1.5e-2."""
    import copy

    import ddpx
    from ddpx.models import build_model
    seeds = [7] if name == "mlp" else list(range(6))
    nat_below, tor_below = [], []
    for seed in seeds:
        torch.manual_seed(seed)
        native = build_model(name, dtype="fp32", device=gpu, hidden=256 if name == "mlp" else None, kernels="native")
        ref = copy.deepcopy(native).to(gpu)
        ref.use_native = False
        flat = ddpx.prepare_model(native, gpu)
        x = torch.rand(64, 3, 32, 32, device=gpu)
        y = torch.randint(0, 10, (64,), device=gpu)
        flat.zero_grad()
        loss, logits = native.forward_loss(x, y)
        assert logits is None
        loss.backward()
        rl = F.cross_entropy(ref(x), y)
        rl.backward()
        assert abs(loss.item() - rl.item()) < 1e-5
        # fp64 on the CPU is the arbiter: gradients that cancel over 65K pixels (conv0 after BatchNorm) differ
        # between any two fp32 summation orders by more than the usual 1e-5
        r64 = copy.deepcopy(ref).cpu().double()
        r64.compute_dtype = torch.float64
        r64.zero_grad()
        F.cross_entropy(r64(x.cpu().double()), y.cpu()).backward()
        rp, p64 = dict(ref.named_parameters()), dict(r64.named_parameters())
        bad, nb, tb = [], [0.0], [0.0]
        for n, p in native.named_parameters():
            e_native, e_torch = _rel(p.main_grad.cpu(), p64[n].grad), _rel(rp[n].grad.cpu(), p64[n].grad)
            print(f"seed {seed} {n}: native {e_native:.2e} torch-fp32 {e_torch:.2e}")
            # bn7 sits below pool3's routing (a flip moved its bias gradient by 3.4e-4 on one seed): only the
            # classifier is above every pooling decision
            top = name == "mlp" or n.startswith("classifier")
            if top:
                if not e_native < 1e-5:
                    bad.append((seed, n, e_native, e_torch))
            else:
                nb.append(e_native)
                tb.append(e_torch)
        assert not bad, bad
        nat_below.append(max(nb))
        tor_below.append(max(tb))
    if name == "vgg":
        med = lambda v: sorted(v)[len(v) // 2]  # noqa: E731
        print("below-pool max error per seed: native", nat_below, "torch", tor_below)
        assert med(nat_below) <= 1.5 * med(tor_below), (nat_below, tor_below)
        assert max(nat_below) < 1.5e-2, (nat_below, tor_below)


@pytest.mark.parametrize("name", ["vgg", "mlp"])
def test_native_fp32_training_tracks_torch_fp32(gpu, name):
    r64 = []
    ln, lt, native, ref = _train_pair(gpu, name, steps=5, lr=0.01, fp64=r64)
    r64 = r64[0]
    # fp32 kernels: the first loss agrees to round-off, later ones to fp32 trajectory drift
    assert abs(ln[0] - lt[0]) < 1e-4 * max(1.0, abs(lt[0])), (ln, lt)
    for a, b in zip(ln, lt):
        assert abs(a - b) < 2e-3 * max(1.0, abs(b)), (ln, lt)
    sd, rsd, sd64 = native.state_dict(), ref.state_dict(), r64.state_dict()
    assert sd.keys() == rsd.keys()
    bad = []
    for k in sd:
        if sd[k].is_floating_point():
            # matrices relative; BatchNorm / bias vectors start at 0 or 1 and move by ~lr*grad, so absolute.
            # Max-pool routing flips make any two fp32 trajectories drift apart; the bar is the fp64 run: the
            # native weights may be no further from it than twice torch fp32's own drift (or 5e-3 relative).
            scale = max(1.0, rsd[k].double().norm().item())
            e_nat = (sd[k].double() - sd64[k].double()).norm().item()
            e_tor = (rsd[k].double() - sd64[k].double()).norm().item()
            print(f"{k}: native-fp64 {e_nat / scale:.2e}  torch32-fp64 {e_tor / scale:.2e}")
            if not e_nat < max(5e-3 * scale, 2.0 * e_tor):
                bad.append((k, e_nat / scale, e_tor / scale))
    assert not bad, bad


def test_vgg_fp32_eval_logits(gpu):
    from ddpx.models import build_model
    import ddpx
    torch.manual_seed(6)
    m = build_model("vgg", dtype="fp32", device=gpu, kernels="native")
    ddpx.prepare_model(m, gpu)
    m.eval()
    x = torch.rand(32, 3, 32, 32, device=gpu)
    with torch.no_grad():
        got = m(x)
        m.use_native = False
        want = m(x)
    assert _rel(got, want) < 1e-4


def _err_vs_fp64(out, ref):
    out, ref = out.double(), ref.double()
    return {"rel_l2": ((out - ref).norm() / ref.norm()).item(), "max_abs": (out - ref).abs().max().item()}


@pytest.mark.parametrize("case", ["fc1", "conv7", "conv4", "conv7_wino", "conv4_wino", "conv1_wino"])
def test_error_no_worse_than_stock(gpu, case):
    """The accuracy bar of the native fp32 kernels is the stock fp32 libraries' own error against fp64
    (hipBLASLt for the MLP's fc1, MIOpen for VGG's conv7 / conv4), measured here on the same inputs: the
    native result may not be more than 1.5x further from fp64 than torch's fp32 result."""
    import json
    import os
    from ddpx.ops import f32
    torch.manual_seed(3)
    if case == "fc1":
        x = torch.randn(512, 4096, device=gpu)
        w = torch.randn(4096, 4096, device=gpu) / 64.0
        ref = x.double() @ w.double().t()
        stock = x @ w.t()
        ours = f32.linear_fwd(x, w)
    else:
        N, H, Ci, Co = {"conv7": (512, 4, 512, 512), "conv4": (512, 8, 256, 512),
                        "conv1": (128, 32, 64, 128)}[case.split("_")[0]]
        x = torch.relu(torch.randn(N, Ci, H, H, device=gpu))
        w = torch.randn(Co, Ci, 3, 3, device=gpu) / (Ci * 9) ** 0.5
        cols = F.unfold(x.double(), 3, padding=1)                      # [N, Ci*9, H*W]
        ref = (w.double().view(Co, -1) @ cols).view(N, Co, H, H)
        stock = F.conv2d(x, w, padding=1)
        Cp = f32.conv_channels(Ci)
        xn = F.pad(x.permute(0, 2, 3, 1), (0, Cp - Ci)).contiguous()
        if case.endswith("_wino"):  # the Winograd F(2,3) forward (MIOpen's algorithm for the stock fp32 recipe)
            uf = torch.empty(16 * Cp * Co, device=gpu)
            f32.wino_wprep(w, uf, None)
            ours = f32.wino_conv(xn, uf, Co).view(N, H, H, Co).permute(0, 3, 1, 2)
        else:
            wf = torch.empty(9 * Cp * Co, device=gpu)
            f32.conv_wprep(w, wf, None)
            ours = f32.conv_fwd(xn, wf, Co).view(N, H, H, Co).permute(0, 3, 1, 2)
        ref, stock = ref.permute(0, 2, 3, 1), stock.permute(0, 2, 3, 1)
        ours = ours.permute(0, 2, 3, 1)
    e_stock, e_ours = _err_vs_fp64(stock, ref), _err_vs_fp64(ours, ref)
    rec = {"case": case, "stock": e_stock, "native": e_ours, "sum": os.environ.get("DDPX_F32_SUM", "auto"),
           "staging": os.environ.get("DDPX_F32_STAGING", "reg"), "block": os.environ.get("DDPX_F32_BLOCK", "1")}
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/f32_error.jsonl", "a") as f:
        f.write(json.dumps(rec) + "\n")
    assert e_ours["rel_l2"] <= 1.5 * e_stock["rel_l2"] + 1e-9, rec


# ---------------------------------------------------------------------------------------------- DeepNN fp32
def _deepnn_pair(gpu, seed, p=0.1):
    import copy

    import ddpx
    from ddpx.models import build_model
    torch.manual_seed(seed)
    native = build_model("deepnn", dtype="fp32", device=gpu, kernels="native")
    native.classifier[2].p = p
    ref = copy.deepcopy(native).to(gpu)
    ref.use_native = False
    ddpx.prepare_model(native, gpu)
    assert native.input_layout(gpu) == "nhwc4_f32"
    return native, ref


def test_deepnn_fp32_gradients_match_fp64(gpu):
    """DeepNN at the reference's precision on the exact-f32 kernels (dropout off on both sides): every gradient
    against fp64, with torch's own fp32 error as the yardstick below the max-pools."""
    import copy
    native, ref = _deepnn_pair(gpu, seed=11, p=0.0)
    x = torch.rand(64, 3, 32, 32, device=gpu)
    y = torch.randint(0, 10, (64,), device=gpu)
    loss, logits = native.forward_loss(x, y)
    assert logits is None  # the native fp32 path ran
    loss.backward()
    rl = F.cross_entropy(ref(x), y)
    rl.backward()
    assert abs(loss.item() - rl.item()) < 1e-5
    r64 = copy.deepcopy(ref).cpu().double()
    r64.zero_grad()
    F.cross_entropy(r64(x.cpu().double()), y.cpu()).backward()
    rp, p64 = dict(ref.named_parameters()), dict(r64.named_parameters())
    bad = []
    for n, p in native.named_parameters():
        e_native, e_torch = _rel(p.main_grad.cpu(), p64[n].grad), _rel(rp[n].grad.cpu(), p64[n].grad)
        print(f"{n}: native {e_native:.2e} torch-fp32 {e_torch:.2e}")
        top = n.startswith("classifier")
        if not e_native < (1e-5 if top else max(5e-3, 3 * e_torch)):
            bad.append((n, e_native, e_torch))
    assert not bad, bad
    native.eval()
    ref.eval()
    with torch.no_grad():
        assert _rel(native(x), ref(x)) < 1e-5


def test_deepnn_fp32_dropout_semantics(gpu):
    """Dropout(0.1) active: the native backward equals torch fp32's for the mask the kernel drew (recovered from
    the dropped activation: kept = d0 > 0 where the ReLU output is > 0)."""
    from ddpx.ops import f32 as Fk
    native, ref = _deepnn_pair(gpu, seed=12)
    native.train()
    x = torch.rand(64, 3, 32, 32, device=gpu)
    t = torch.randint(0, 10, (64,), device=gpu)
    saved, last, loss, _, dl = Fk._deepnn_forward(native, Fk.prep_vgg_input(x), t, True)
    _, feat, d0, scale = last
    assert abs(scale - 1 / 0.9) < 1e-6
    a0 = F.relu(ref.classifier[0](ref.features(x).flatten(1)))
    mask = (d0 > 0).float()
    live = (a0 > 0).float()
    frac = (mask.sum() / live.sum()).item()
    assert 0.85 < frac < 0.95, frac
    k = d0 > 0  # kept elements carry a0 / (1 - p) (a0 from torch: fp32 round-off apart from the native one)
    assert torch.allclose(d0[k], a0[k].detach() * scale, rtol=1e-4, atol=1e-6)
    rl = F.cross_entropy(ref.classifier[3](a0 * mask * scale), t)
    assert abs(loss.item() - rl.item()) < 1e-5 * max(1.0, rl.item())
    rl.backward()
    Fk._deepnn_backward(native, saved, last, dl, torch.ones((), device=gpu))
    for (n, p), (_, q) in zip(native.named_parameters(), ref.named_parameters()):
        assert _rel(p.main_grad, q.grad) < (1e-5 if n.startswith("classifier") else 5e-3), n


def test_dropout_f32_kernel(gpu):
    from ddpx.ops.f32 import dropout_
    rng = torch.tensor([99, 0], dtype=torch.int64, device=gpu)
    done = torch.zeros(1, dtype=torch.int32, device=gpu)
    x = torch.ones(512, 512, device=gpu)
    a = dropout_(x, 0.1, rng, done)
    b = dropout_(x, 0.1, rng, done)
    torch.cuda.synchronize()
    assert int(rng[1]) == 2 and int(done[0]) == 0
    keep = (a > 0).float().mean().item()
    assert abs(keep - 0.9) < 5e-3, keep
    assert torch.equal(a[a > 0], torch.full_like(a[a > 0], 1.0 / (1.0 - 0.1)))
    assert not torch.equal(a, b)
    rng[1] = 0
    assert torch.equal(dropout_(x, 0.1, rng, done), a)  # same (seed, offset): same mask


def test_deepnn_fp32_trains_like_torch(gpu):
    """Five SGD steps with dropout off: the native fp32 DeepNN follows torch fp32's trajectory."""
    from ddpx.optim.sgd import SGD
    native, ref = _deepnn_pair(gpu, seed=13, p=0.0)
    opt = SGD(native.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
    ropt = torch.optim.SGD(ref.parameters(), lr=0.01, momentum=0.9, weight_decay=5e-4)
    gen = torch.Generator().manual_seed(3)
    for _ in range(5):
        x = torch.rand(64, 3, 32, 32, generator=gen).to(gpu)
        y = torch.randint(0, 10, (64,), generator=gen).to(gpu)
        opt.zero_grad()
        loss, logits = native.forward_loss(x, y)
        assert logits is None
        loss.backward()
        opt.step()
        ropt.zero_grad()
        rl = F.cross_entropy(ref(x), y)
        rl.backward()
        ropt.step()
        assert abs(loss.item() - rl.item()) < 2e-3 * max(1.0, rl.item())
    for (n, p), (_, q) in zip(native.named_parameters(), ref.named_parameters()):
        err = (p.detach().double() - q.detach().double()).norm().item()
        assert err < 5e-3 * max(1.0, q.detach().double().norm().item()), n


@pytest.mark.parametrize("case", ["fwd", "dgrad", "wgrad", "lin_fwd", "lin_dgrad", "lin_wgrad", "ragged"])
@pytest.mark.parametrize("tile", [0, 1, 2, 3])
def test_f32_dma_core_bitwise_equals_register_core(gpu, case, tile):
    """The LDS-DMA ring GEMM (default) runs the register-staged kernel's fragment / MFMA / summation sequence:
    results must be bitwise equal for every operand mode, tile and split."""
    from ddpx.ops import f32 as Fk
    torch.manual_seed(21)
    if case in ("fwd", "dgrad", "wgrad"):
        N, H, C, Co = 4, 8, 64, 128
        x = torch.randn(N, H, H, C, device=gpu)
        dy = torch.randn(N * H * H, Co, device=gpu)
        w = torch.randn(9 * C * Co, device=gpu)
        if case == "fwd":
            args = (Fk.IM2COL_KC, x, 0, Fk.DENSE_OC, w, Co, N * H * H, Co, 9 * C)
            kw = dict(geom=(C, H, H, 1))
            shape = (N * H * H, Co)
        elif case == "dgrad":
            args = (Fk.IM2COL_KC, dy, 0, Fk.DENSE_OC, w, C, N * H * H, C, 9 * Co)
            kw = dict(geom=(Co, H, H, -1))
            shape = (N * H * H, C)
        else:
            S = 3
            args = (Fk.DENSE_OC, dy, Co, Fk.IM2COL_OC, x, 0, Co, 9 * C, N * H * H)
            kw = dict(geom=(C, H, H, 1), splits=S, split_stride=Co * 9 * C)
            shape = (S, Co, 9 * C)
    else:
        M, Nn, K = (256, 192, 320) if case != "ragged" else (200, 132, 516)
        a = torch.randn(M, K, device=gpu)
        b = torch.randn(Nn, K, device=gpu)
        if case in ("lin_fwd", "ragged"):
            args = (Fk.DENSE_KC, a, K, Fk.DENSE_KC, b, K, M, Nn, K)
            shape = (M, Nn)
        elif case == "lin_dgrad":
            bt = torch.randn(K, Nn, device=gpu)
            args = (Fk.DENSE_KC, a, K, Fk.DENSE_OC, bt, Nn, M, Nn, K)
            shape = (M, Nn)
        else:
            at = torch.randn(K, M, device=gpu)
            bt = torch.randn(K, Nn, device=gpu)
            args = (Fk.DENSE_OC, at, M, Fk.DENSE_OC, bt, Nn, M, Nn, K)
            shape = (M, Nn)
        kw = {}
    outs = []
    prev, pblock = Fk.set_staging(True), Fk.set_block(1)
    try:
        for dma in (True, False):
            Fk.set_staging(dma)
            o = torch.full(shape, float("nan"), device=gpu)
            Fk.gemm(*args, o, tile=tile, **kw)
            outs.append(o)
    finally:
        Fk.set_staging(prev)
        Fk.set_block(pblock)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1]), (outs[0] - outs[1]).abs().max().item()


@pytest.mark.parametrize("N,H,C,Co", [(8, 32, 4, 64), (16, 8, 128, 256), (64, 4, 512, 512)])
def test_conv_fwd_stats_epilogue(gpu, N, H, C, Co):
    """BatchNorm tile statistics from the LDS-DMA conv GEMM's epilogue: y bitwise equal to the plain forward, and
    every tile's (mean, M2) equal to the statistics of its rows (fp64 arbiter)."""
    from ddpx.ops import f32 as Fk
    torch.manual_seed(9)
    x = torch.randn(N, H, H, C, device=gpu)
    wf = torch.randn(9 * C * Co, device=gpu) / (9 * C) ** 0.5
    prev = Fk.set_staging(True)
    try:
        y, st = Fk.conv_fwd_stats(x, wf, Co)
        y2 = Fk.conv_fwd(x, wf, Co)
    finally:
        Fk.set_staging(prev)
    assert st is not None
    part, T, R = st
    assert torch.equal(y, y2)
    P = N * H * H
    assert T == (P + R - 1) // R
    yd = y.double().cpu()
    for t in range(T):
        rows = yd[t * R:min(P, (t + 1) * R)]
        mu = rows.mean(0)
        m2 = ((rows - mu) ** 2).sum(0)
        assert _rel(part[t, 0].cpu(), mu) < 1e-5, t
        assert _rel(part[t, 1].cpu(), m2) < 1e-5, t
    prev = Fk.set_staging(False)
    try:
        y3, st3 = Fk.conv_fwd_stats(x, wf, Co)  # register-staged core: no fused statistics
        y4 = Fk.conv_fwd(x, wf, Co)
    finally:
        Fk.set_staging(prev)
    assert st3 is None and torch.equal(y3, y4)


class _MirrorComm:
    """A 2-rank communicator whose other rank holds exactly this rank's batch."""
    world_size = 2
    rank = 0

    def allgather(self, out, inp, stream=None):
        out.view(2, -1).copy_(inp.view(1, -1).expand(2, -1))

    def allreduce_(self, t, op="sum", stream=None, async_op=False):
        assert op == "sum"
        t.mul_(2.0)


def test_native_fp32_sync_batchnorm_matches_doubled_batch(gpu):
    """Native fp32 SyncBatchNorm (``--sync_bn`` at the reference's precision, /root/reference/multigpu.py:127):
    over a mirror communicator (the other rank holds the same batch) the statistics, running stats (unbiased with
    the GLOBAL count) and every gradient equal those of torch BatchNorm on the doubled batch [x, x] (fp64 arbiter)."""
    import copy

    import ddpx
    from ddpx.models import build_model
    from ddpx.ops import f32 as Fk
    torch.manual_seed(9)
    native = build_model("vgg", dtype="fp32", device=gpu, kernels="native")
    ref = copy.deepcopy(native).cpu().double()
    ref.use_native = False
    ref.compute_dtype = torch.float64
    flat = ddpx.prepare_model(native, gpu)
    native.sync_bn_comm = _MirrorComm()
    assert Fk._sync_comm(native, True) is not None
    x = torch.rand(32, 3, 32, 32, device=gpu)
    y = torch.randint(0, 10, (32,), device=gpu)
    flat.zero_grad()
    loss, logits = native.forward_loss(x, y)
    assert logits is None  # the native fp32 path ran
    loss.backward()
    x2, y2 = torch.cat([x, x]).cpu().double(), torch.cat([y, y]).cpu()
    rl = F.cross_entropy(ref(x2), y2)
    rl.backward()
    assert abs(loss.item() - rl.item()) < 1e-5, (loss.item(), rl.item())
    for (n, b), (_, rb) in zip(native.named_buffers(), ref.named_buffers()):
        if b.is_floating_point():
            assert torch.allclose(b.cpu().double(), rb, rtol=1e-5, atol=1e-6), n
        else:
            assert int(b) == int(rb), n
    rp = dict(ref.named_parameters())
    bad = []
    for n, p in native.named_parameters():
        e = _rel(p.main_grad.cpu(), rp[n].grad)
        top = n.startswith(("classifier", "backbone.bn7"))
        if not e < (1e-5 if top else 5e-3):  # pooling-decision flips below bn7 (test above)
            bad.append((n, e))
    assert not bad, bad


# ---------------------------------------------------------------------------------------------- Winograd F(2,3)
@pytest.mark.parametrize("shape", [(4, 32, 64, 128), (3, 8, 256, 64), (5, 4, 512, 32), (2, 2, 4, 32), (7, 16, 128, 96)])
def test_wino_conv_forward_dgrad_stats_match_fp64(gpu, shape):
    """Winograd F(2x2,3x3) forward (with the BatchNorm chunk statistics) and data gradient against fp64, on shapes
    with a partial last workgroup (P % 64 != 0) and output channels that are not a power of two."""
    from ddpx.ops import f32
    torch.manual_seed(5)
    N, H, Ci, Co = shape
    x = torch.randn(N, Ci, H, H, device=gpu)
    w = torch.randn(Co, Ci, 3, 3, device=gpu) / (Ci * 9) ** 0.5
    xn = x.permute(0, 2, 3, 1).contiguous()
    uf = torch.empty(16 * Ci * Co, device=gpu)
    ud = torch.empty(16 * Co * Ci, device=gpu)
    f32.wino_wprep(w, uf, ud)
    y, (st, T, R) = f32.wino_conv(xn, uf, Co, stats=True)
    ref = F.conv2d(x.double(), w.double(), padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    assert _err_vs_fp64(y, ref)["rel_l2"] < 1e-5
    # chunk statistics: R-row chunks of the pixels in (tile, 2x2) order; their Chan merge is the batch's
    assert R == 256 and T == (N * (H // 2) * (H // 2) + 63) // 64
    P = N * H * H
    cnt = torch.tensor([min(R, P - t * R) for t in range(T)], device=gpu, dtype=torch.float64)
    mean = (st[:, 0].double() * cnt[:, None]).sum(0) / P
    m2 = (st[:, 1].double() + cnt[:, None] * (st[:, 0].double() - mean) ** 2).sum(0)
    assert torch.allclose(mean, ref.mean(0), rtol=1e-4, atol=1e-5)
    assert torch.allclose(m2 / P, ref.var(0, unbiased=False), rtol=1e-4, atol=1e-6)
    if Co % 32 == 0 and Ci % 32 == 0 and Co >= 4:
        dy = torch.randn(N, H, H, Co, device=gpu)
        dx = f32.wino_conv(dy, ud, Ci).view(N, H, H, Ci)
        xr = x.double().requires_grad_(True)
        F.conv2d(xr, w.double(), padding=1).backward(dy.double().permute(0, 3, 1, 2))
        assert _err_vs_fp64(dx, xr.grad.permute(0, 2, 3, 1))["rel_l2"] < 1e-5


@pytest.mark.parametrize("shape", [(2, 8, 64, 64), (3, 6, 32, 128), (4, 16, 128, 64), (64, 4, 512, 512),
                                   (5, 2, 96, 192)])
def test_wino_wgrad_matches_fp64(gpu, shape):
    """Winograd F(2,3) weight gradient (dW = G^T sum_tiles (A dY A^T) (.) (B^T x B) G) against fp64 and against the
    direct split-K implicit GEMM's own error: partial last K-step (tiles % 8), several splits, accumulate."""
    from ddpx.ops import f32
    torch.manual_seed(6)
    N, H, Ci, Co = shape
    x = torch.randn(N, Ci, H, H, device=gpu)
    w = torch.randn(Co, Ci, 3, 3, device=gpu) / (Ci * 9) ** 0.5
    dy = torch.randn(N, H, H, Co, device=gpu)
    xn = x.permute(0, 2, 3, 1).contiguous()
    assert f32.wino_wgrad_applies(H, H, Ci, Co)
    xr = x.double()
    wr = w.double().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(dy.double().permute(0, 3, 1, 2))
    ref = wr.grad
    out = torch.full((Co, Ci, 3, 3), 0.25, device=gpu)
    f32.wino_wgrad(dy.reshape(-1, Co), xn, Co, Ci, out, accumulate=True)
    err = _err_vs_fp64(out - 0.25, ref)["rel_l2"]
    assert err < 1e-5, err
    f32.wino_wgrad(dy.reshape(-1, Co), xn, Co, Ci, out)
    assert _err_vs_fp64(out, ref)["rel_l2"] < 1e-5
    # no worse than 2x the direct implicit GEMM on the same operands (which needs power-of-two H, W, C)
    if H & (H - 1) or Ci & (Ci - 1):
        return
    direct = torch.empty_like(out)
    f32.direct_wgrad(dy.reshape(-1, Co), xn, Co, Ci, direct)
    e_direct = _err_vs_fp64(direct, ref)["rel_l2"]
    assert err < max(2 * e_direct, 2e-6), (err, e_direct)


@pytest.mark.parametrize("accumulate", [False, True])
def test_conv_wgrad_32_channels_padded_winograd(gpu, accumulate):
    """conv_wgrad of a 32-output-channel layer (DeepNN's 64 -> 32 at 16x16) runs the Winograd weight gradient over
    dy zero-padded to 64 channels: fp64 agreement, only the first 32 rows written, accumulate adds."""
    from ddpx.ops import f32
    torch.manual_seed(7)
    N, H, Ci, Co = 4, 16, 64, 32
    assert not f32.wino_wgrad_applies(H, H, Ci, Co) and f32.wino_wgrad_applies(H, H, Ci, 64)
    x = torch.randn(N, Ci, H, H, device=gpu)
    w = torch.randn(Co, Ci, 3, 3, device=gpu) / (Ci * 9) ** 0.5
    dy = torch.randn(N, H, H, Co, device=gpu)
    xn = x.permute(0, 2, 3, 1).contiguous()
    wr = w.double().requires_grad_(True)
    F.conv2d(x.double(), wr, padding=1).backward(dy.double().permute(0, 3, 1, 2))
    buf = torch.full((Co * Ci * 9 + 64,), 0.25, device=gpu)  # guard words after the gradient
    out = buf[:Co * Ci * 9].view(Co, Ci, 3, 3)
    f32.conv_wgrad(dy.reshape(-1, Co), xn, Co, Ci, out, accumulate=accumulate)
    got = out - 0.25 if accumulate else out
    assert _err_vs_fp64(got, wr.grad)["rel_l2"] < 1e-5
    assert torch.all(buf[Co * Ci * 9:] == 0.25)


def test_wino_conv_relu_mask_and_colsum_bias(gpu):
    """The Winograd data gradient with the ReLU mask of the block below in its epilogue equals the unmasked one
    times (mask > 0) bitwise; colsum_bias matches the fp64 column sums and accumulates."""
    from ddpx.ops import f32
    from ddpx.models import DeepNN
    torch.manual_seed(8)
    N, H, C, K = 8, 16, 64, 128
    x = torch.randn(N, H, H, C, device=gpu)
    w = torch.randn(K, C, 3, 3, device=gpu) / (C * 9) ** 0.5
    u = torch.empty(16 * C * K, device=gpu)
    f32.wino_wprep(w, u, None)
    mask = torch.relu(torch.randn(N * H * H, K, device=gpu))
    raw = f32.wino_conv(x, u, K)
    got = f32.wino_conv(x, u, K, mask=mask)
    assert torch.equal(got, torch.where(mask > 0, raw, torch.zeros_like(raw)))
    plan = f32._deepnn_plan(DeepNN().to(gpu))
    db = torch.full((K,), 0.5, device=gpu)
    f32.colsum_bias(got, N * H * H, K, plan, db, accumulate=True)
    ref = got.double().sum(0)
    assert _rel((db - 0.5).cpu(), ref.cpu()) < 1e-6
    f32.colsum_bias(got, N * H * H, K, plan, db)
    assert _rel(db.cpu(), ref.cpu()) < 1e-6


def test_vgg_fp32_runs_winograd_layers(gpu):
    """The fp32 VGG plan puts every layer with >= 64 input channels on Winograd (forward + data gradient)."""
    import ddpx
    from ddpx.models import build_model
    from ddpx.ops import f32
    m = build_model("vgg", dtype="fp32", device=gpu, kernels="native")
    ddpx.prepare_model(m, gpu)
    plan = f32._vgg_plan(m)
    assert plan.uf[0] is None and all(u is not None for u in plan.uf[1:])
    assert all(u is not None for u in plan.ud[1:])


def test_wino_conv_bias_relu_epilogue(gpu):
    """DeepNN's conv + bias + ReLU through the Winograd epilogue, against fp64."""
    from ddpx.ops import f32
    torch.manual_seed(6)
    N, H, Ci, Co = 6, 16, 128, 64
    x = torch.randn(N, Ci, H, H, device=gpu)
    w = torch.randn(Co, Ci, 3, 3, device=gpu) / (Ci * 9) ** 0.5
    b = torch.randn(Co, device=gpu)
    uf = torch.empty(16 * Ci * Co, device=gpu)
    f32.wino_wprep(w, uf, None)
    y = f32.wino_conv(x.permute(0, 2, 3, 1).contiguous(), uf, Co, bias=b, relu=True)
    ref = torch.relu(F.conv2d(x.double(), w.double(), b.double(), padding=1)).permute(0, 2, 3, 1).reshape(-1, Co)
    assert _err_vs_fp64(y, ref)["rel_l2"] < 1e-5


def test_deepnn_fp32_runs_winograd_layers(gpu):
    import ddpx
    from ddpx.models import build_model
    from ddpx.ops import f32
    m = build_model("deepnn", dtype="fp32", device=gpu, kernels="native")
    ddpx.prepare_model(m, gpu)
    plan = f32._deepnn_plan(m)
    assert plan.uf[0] is None and all(u is not None for u in plan.uf[1:]), [u is not None for u in plan.uf]


def test_mlp_fp32_fused_optimizer_bitwise(gpu):
    """SGD(fused_backward=True) on the fp32 MLP: the hidden layers' weight-gradient GEMMs apply the update in their
    epilogue (ddpx_f32_wgrad_sgd) - bitwise the unfused step (stored gradient + flat SGD), over 3 steps."""
    import ddpx
    from ddpx.models import build_model
    from ddpx.optim.sgd import SGD
    models = []
    for _ in range(2):
        torch.manual_seed(4)
        m = build_model("mlp", hidden=512, dtype="fp32", device=gpu, kernels="native")
        ddpx.prepare_model(m, gpu)
        models.append(m)
    a, b = models
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, fused_backward=True)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    flat = a.linears()[0].weight._ddpx_flat
    for _ in range(3):
        x = torch.rand(64, 3, 32, 32, device=gpu)
        t = torch.randint(0, 10, (64,), device=gpu)
        for m, o in ((a, oa), (b, ob)):
            o.sync_lr()
            o.zero_grad()
            loss, logits = m.forward_loss(x, t)
            assert logits is None  # the native fp32 path
            loss.backward()
            if m is a:
                assert flat.updated[flat.index[id(a.linears()[0].weight)]], "fused update did not run"
            o.step()
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p, q), n
