"""Numerics of every native HIP kernel vs a plain PyTorch fp32 reference of the same op."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _rand_bf16(*shape, dev):
    return (torch.randn(*shape, device=dev) * 0.5).to(torch.bfloat16)


@pytest.mark.parametrize("tile", list(range(-1, 14)) + [16, 17, 18, 19, 20, 21, 22, 23, 24, 25])
@pytest.mark.parametrize("layout", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("MNK", [(512, 4096, 3072), (336, 256, 512), (128, 128, 64), (106, 64, 200), (64, 192, 72),
                                 (200, 136, 1000), (2048, 4096, 512)])
def test_gemm_layouts(gpu, tile, layout, MNK):
    from ddpx.ops.gemm import matmul
    M, N, K = MNK
    ak, bk = layout
    if not ak and M % 8:
        pytest.skip("M-contig A requires M % 8 == 0")
    torch.manual_seed(0)
    A = _rand_bf16(M, K, dev=gpu)
    B = _rand_bf16(K, N, dev=gpu)  # logical [K,N]
    a_store = A if ak else A.t().contiguous()        # [M,K] or [K,M]
    b_store = B.t().contiguous() if bk else B         # [N,K] or [K,N]
    C = matmul(a_store, b_store, a_kcontig=ak, b_kcontig=bk, tile=tile)
    ref = A.float() @ B.float()
    assert _rel(C, ref) < 2e-3


def test_gemm_identity_asymmetric(gpu):
    """A = I with an asymmetric B catches a transposed C/D write (guide §3)."""
    from ddpx.ops.gemm import matmul
    n = 128
    A = torch.eye(n, device=gpu, dtype=torch.bfloat16)
    B = (torch.arange(n * n, device=gpu, dtype=torch.float32).view(n, n) % 97).to(torch.bfloat16)
    for ak in (True, False):
        for bk in (True, False):
            C = matmul(A if ak else A.t().contiguous(), B.t().contiguous() if bk else B, a_kcontig=ak, b_kcontig=bk)
            assert torch.equal(C, B.float()), (ak, bk)


def test_linear_fwd_dgrad_wgrad(gpu):
    from ddpx.ops import gemm as G
    torch.manual_seed(1)
    M, K, N = 512, 3072, 1024
    x = _rand_bf16(M, K, dev=gpu)
    w = _rand_bf16(N, K, dev=gpu)
    b = torch.randn(N, device=gpu)
    y = G.linear_fwd(x, w, b, relu=True)
    ref = torch.relu(x.float() @ w.float().t() + b)
    assert _rel(y, ref) < 5e-3
    dy = _rand_bf16(M, N, dev=gpu)
    dx = G.linear_dgrad(dy, w, relu_mask_of=x)
    refdx = (dy.float() @ w.float()) * (x.float() > 0)
    assert _rel(dx, refdx) < 5e-3
    dw = torch.empty(N, K, device=gpu)
    G.linear_wgrad(dy, x, dw)
    refdw = dy.float().t() @ x.float()
    assert _rel(dw, refdw) < 2e-3
    G.linear_wgrad(dy, x, dw, accumulate=True)
    assert _rel(dw, 2 * refdw) < 2e-3
    dwb = torch.empty(N, K, device=gpu, dtype=torch.bfloat16)
    G.linear_wgrad(dy, x, dwb)
    G.linear_wgrad(dy, x, dwb, accumulate=True)
    assert _rel(dwb, 2 * refdw) < 1e-2
    # ReLU backward with the fused bias gradient (per-tile column sums + fixed-order reduce)
    db = torch.empty(K, device=gpu)
    dx2 = G.linear_dgrad(dy, w, relu_mask_of=x, bias_grad=db)
    assert torch.equal(dx2, dx)
    assert _rel(db, dx2.float().sum(0)) < 1e-5
    G.linear_dgrad(dy, w, relu_mask_of=x, bias_grad=db, bias_grad_accumulate=True)
    assert _rel(db, 2 * dx2.float().sum(0)) < 1e-5


def test_linear_wide_default_tile(gpu):
    """The wide-layer default tile (pick -> 128x128, 2 stages, 4 waves, two workgroups per CU; profiles/r6_gemm
    sweep_wide.json): forward with bias + ReLU, ReLU-masked data gradient with the in-launch bias-gradient column sums,
    and the fused bias SGD, against fp32 references."""
    from ddpx.ops import gemm as G
    from ddpx.ops.elementwise import sgd_flat_
    torch.manual_seed(3)
    M, K, N = 512, 2048, 16384
    x = _rand_bf16(M, N, dev=gpu)
    w = _rand_bf16(K, N, dev=gpu) * 0.1
    b = torch.randn(K, device=gpu)
    y = G.linear_fwd(x, w.to(torch.bfloat16), b, relu=True)
    ref = torch.relu(x.float() @ w.float().t() + b)
    assert _rel(y, ref) < 5e-3
    dy = _rand_bf16(M, K, dev=gpu)
    db = torch.empty(N, device=gpu)
    dx = G.linear_dgrad(dy, w.to(torch.bfloat16), relu_mask_of=x, bias_grad=db)
    refdx = (dy.float() @ w.float()) * (x.float() > 0)
    assert _rel(dx, refdx) < 5e-3
    assert _rel(db, dx.float().sum(0)) < 1e-5
    p0 = torch.randn(N, device=gpu)
    buf0 = torch.randn(N, device=gpu) * 0.1
    lr = torch.full((), 0.05, device=gpu)
    pa, ba = p0.clone(), buf0.clone()
    G.linear_dgrad(dy, w.to(torch.bfloat16), relu_mask_of=x, bias_sgd=(pa, ba, None, lr, 0.9, 5e-4))
    pb, bb = p0.clone(), buf0.clone()
    sgd_flat_(pb, bb, db, None, lr, 0.9, 5e-4)
    assert torch.allclose(pa, pb, rtol=1e-6, atol=1e-6) and torch.allclose(ba, bb, rtol=1e-6, atol=1e-6)


def test_head_fwd_bwd(gpu):
    from ddpx.ops.head import head_backward, head_forward
    torch.manual_seed(2)
    M, K, C = 512, 4096, 10
    h = torch.relu(_rand_bf16(M, K, dev=gpu).float()).to(torch.bfloat16)
    w = _rand_bf16(C, K, dev=gpu)
    b = torch.randn(C, device=gpu)
    t = torch.randint(0, C, (M,), device=gpu)
    correct = torch.zeros((), dtype=torch.int32, device=gpu)
    loss, logits, dl = head_forward(h, w, b, t, correct=correct)
    hf = h.float().requires_grad_(True)
    wf = w.float().requires_grad_(True)
    bf = b.clone().requires_grad_(True)
    ref_logits = hf @ wf.t() + bf
    ref_loss = torch.nn.functional.cross_entropy(ref_logits, t)
    assert _rel(logits, ref_logits) < 1e-4
    assert abs(loss.item() - ref_loss.item()) < 1e-4 * max(1.0, abs(ref_loss.item()))
    assert correct.item() == (ref_logits.argmax(1) == t).sum().item()
    ref_loss.backward()
    dW = torch.empty(C, K, device=gpu)
    db = torch.empty(C, device=gpu)
    dH = torch.empty_like(h)
    dbp = torch.empty(K, device=gpu)
    go = torch.tensor(1.0, device=gpu)
    head_backward(dl, go, h, w, dW, db, dH=dH, dbprev=dbp, relu_mask=True)
    assert _rel(dW, wf.grad) < 1e-4
    assert _rel(db, bf.grad) < 1e-4
    ref_dh = hf.grad * (h.float() > 0)
    assert _rel(dH, ref_dh) < 5e-3
    assert _rel(dbp, dH.float().sum(0)) < 1e-4
    # bf16 gradient buffers + accumulate
    dWb = torch.zeros(C, K, device=gpu, dtype=torch.bfloat16)
    dbb = torch.zeros(C, device=gpu, dtype=torch.bfloat16)
    dbpb = torch.zeros(K, device=gpu, dtype=torch.bfloat16)
    head_backward(dl, go, h, w, dWb, dbb, dH=dH, dbprev=dbpb, relu_mask=True, accumulate=True)
    assert _rel(dWb, wf.grad) < 1e-2 and _rel(dbb, bf.grad) < 1e-2 and _rel(dbpb, dbp) < 1e-2
    # odd row counts (last batch of an epoch) and logits-only eval
    for Mo in (336, 106, 7):
        lo, lg, dlo = head_forward(h[:Mo], w, b, t[:Mo])
        rl = h[:Mo].float() @ w.float().t() + b
        assert _rel(lg, rl) < 1e-4
        assert abs(lo.item() - torch.nn.functional.cross_entropy(rl, t[:Mo]).item()) < 1e-3


def test_sgd_flat_matches_torch(gpu):
    from ddpx.ops.elementwise import sgd_flat_
    torch.manual_seed(3)
    n = 100003
    p = torch.randn(n, device=gpu)
    g = torch.randn(n, device=gpu)
    tp = p.clone().requires_grad_(False)
    opt = torch.optim.SGD([torch.nn.Parameter(tp)], lr=0.4, momentum=0.9, weight_decay=5e-4)
    buf = torch.zeros(n, device=gpu)
    sh = torch.empty(n, dtype=torch.bfloat16, device=gpu)
    lr_dev = torch.tensor(0.4, device=gpu)
    for step in range(3):
        opt.param_groups[0]["params"][0].grad = g.clone()
        opt.step()
        sgd_flat_(p, buf, g, sh, lr_dev if step % 2 else 0.4, 0.9, 5e-4)
    ref = opt.param_groups[0]["params"][0].detach()
    assert torch.allclose(p, ref, rtol=1e-5, atol=1e-6)
    assert torch.equal(sh, p.to(torch.bfloat16))


def test_colsum_and_cast(gpu):
    from ddpx.ops.elementwise import cast_bf16_, colsum_bf16
    x = _rand_bf16(517, 1000, dev=gpu)
    out = torch.empty(1000, device=gpu)
    colsum_bf16(x, out)
    assert _rel(out, x.float().sum(0)) < 1e-5
    f = torch.randn(12345, device=gpu)
    bb = torch.empty(12345, dtype=torch.bfloat16, device=gpu)
    cast_bf16_(f, bb)
    assert torch.equal(bb, f.to(torch.bfloat16))


@pytest.mark.parametrize("layout", ["nchw_f32", "nchw_bf16", "nhwc_bf16", "flat_bf16"])
def test_augment_matches_cpu(gpu, layout):
    from ddpx.data.datasets import synthetic_cifar
    from ddpx.data.loader import augment_cpu, augment_gpu
    ds = synthetic_cifar(300, seed=1)
    idx = torch.randperm(300)[:77]
    for train in (True, False):
        xc, yc = augment_cpu(ds.images, ds.labels, idx, seed=12345, train=train, layout=layout)
        xg, yg = augment_gpu(ds.images.to(gpu), ds.labels.to(gpu), idx.to(gpu), seed=12345, train=train,
                             layout=layout)
        assert torch.equal(yc, yg.cpu())
        assert torch.equal(xc, xg.cpu())


def _bf(t):
    return t.to(torch.bfloat16).float()


def _mlp_reference(x, t, W, b):
    """fp32 math with bf16 rounding exactly where the native path stores bf16 (activations, dpre)."""
    M = x.shape[0]
    h1 = _bf(torch.relu(x.float() @ W[0].t() + b[0]))
    h2 = _bf(torch.relu(h1 @ W[1].t() + b[1]))
    z = h2 @ W[2].t() + b[2]
    loss = torch.nn.functional.cross_entropy(z, t)
    dl = (torch.softmax(z, 1) - torch.nn.functional.one_hot(t, 10).float()) / M
    g = {}
    g["fc2.weight"], g["fc2.bias"] = dl.t() @ h2, dl.sum(0)
    d2 = _bf((dl @ W[2]) * (h2 > 0))
    g["fc1.weight"], g["fc1.bias"] = d2.t() @ h1, d2.sum(0)
    d1 = _bf((d2 @ W[1]) * (h1 > 0))
    g["fc0.weight"], g["fc0.bias"] = d1.t() @ x.float(), d1.sum(0)
    return loss, g


@pytest.mark.parametrize("grad_dtype", [torch.float32, torch.bfloat16])
def test_mlp_native_matches_reference(gpu, grad_dtype):
    """Native fused MLP (loss + every gradient) vs an fp32 reference with the same bf16 storage points."""
    import ddpx
    from ddpx.models import MLP
    torch.manual_seed(4)
    m = MLP(hidden=512, layers=3)
    ddpx.prepare_model(m, gpu, grad_dtype=grad_dtype)
    W = [_bf(getattr(m, f"fc{i}").weight.detach()) for i in range(3)]
    b = [getattr(m, f"fc{i}").bias.detach().clone() for i in range(3)]
    x = torch.rand(256, 3072, device=gpu).to(torch.bfloat16)
    t = torch.randint(0, 10, (256,), device=gpu)
    loss, _ = m.forward_loss(x, t)
    loss.backward()
    rl, rg = _mlp_reference(x, t, W, b)
    assert abs(loss.item() - rl.item()) < 1e-3
    tol = 2e-3 if grad_dtype == torch.float32 else 1e-2
    for n, p in m.named_parameters():
        assert _rel(p.main_grad, rg[n]) < tol, n


def test_mlp_graph_matches_eager_bf16_grads(gpu):
    """Captured step == eager step, bit for bit, with bf16 gradient buffers."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.optim.sgd import SGD
    from ddpx.runtime.graphs import CapturedStep
    torch.manual_seed(5)
    a, b = MLP(hidden=512), MLP(hidden=512)
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        ddpx.prepare_model(m, gpu, grad_dtype=torch.bfloat16)
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, capturable=True)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    xs = [torch.rand(256, 3072, device=gpu).to(torch.bfloat16) for _ in range(5)]
    ts = [torch.randint(0, 10, (256,), device=gpu) for _ in range(5)]

    def body(x, y):
        oa.zero_grad()
        loss, _ = a.forward_loss(x, y)
        loss.backward()
        oa.step()
        return loss

    oa.sync_lr()
    body(xs[0], ts[0])
    g = CapturedStep(body, xs[1], ts[1])
    la = [g(xs[i], ts[i]).item() for i in range(1, 5)]
    lb = []
    for i in range(5):
        ob.zero_grad()
        loss, _ = b.forward_loss(xs[i], ts[i])
        loss.backward()
        ob.step()
        lb.append(loss.item())
    assert la == lb[1:]
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)


@pytest.mark.parametrize("graph", [False, True])
def test_fused_backward_optimizer_bitwise(gpu, graph):
    """SGD applied inside the backward epilogues == materialised fp32 grads + flat SGD, bit for bit."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.optim.sgd import SGD
    from ddpx.runtime.graphs import CapturedStep
    torch.manual_seed(6)
    a, b = MLP(hidden=512), MLP(hidden=512)
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        ddpx.prepare_model(m, gpu)
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, capturable=True, fused_backward=True)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    assert oa.fused_active()
    xs = [torch.rand(256, 3072, device=gpu).to(torch.bfloat16) for _ in range(4)]
    ts = [torch.randint(0, 10, (256,), device=gpu) for _ in range(4)]

    def body(x, y):
        oa.zero_grad()
        loss, _ = a.forward_loss(x, y)
        loss.backward()
        oa.step()
        return loss

    oa.sync_lr()
    la = [body(xs[0], ts[0]).item()]
    if graph:
        g = CapturedStep(body, xs[1], ts[1])
        la += [g(xs[i], ts[i]).item() for i in range(1, 4)]
    else:
        la += [body(xs[i], ts[i]).item() for i in range(1, 4)]
    lb = []
    for i in range(4):
        ob.zero_grad()
        loss, _ = b.forward_loss(xs[i], ts[i])
        loss.backward()
        ob.step()
        lb.append(loss.item())
    assert la == lb
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
    assert torch.equal(oa.momentum_buffer, ob.momentum_buffer)


def test_native_libs_loaded(gpu):
    from ddpx.runtime import native
    libs = native.loaded_libraries()
    assert any("libddpx_kernels.so" in p for p in libs), libs


@pytest.mark.parametrize("tile,splits", [(-1, None), (12, None), (14, 2), (5, 2), (8, 4), (0, 3),
                                         (16, 4), (16, 2), (16, None), (17, 2), (17, None), (18, None),
                                         (19, None), (20, None)])
def test_linear_mlp_shapes_splitk(gpu, tile, splits):
    """The toy-MLP products at M=512: default plan, a fixed single-pass tile, and the in-launch split-K
    (K split over workgroups whose fp32 partials the last split of each tile combines in split order)."""
    from ddpx.ops import gemm as G
    torch.manual_seed(7)
    M, K, N = 512, 4096, 4096
    x = _rand_bf16(M, K, dev=gpu)
    w = (torch.randn(N, K, device=gpu) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=gpu)
    y = G.linear_fwd(x, w, b, relu=True, tile=tile, splits=splits)
    ref = torch.relu(x.float() @ w.float().t() + b)
    assert _rel(y, ref) < 5e-3
    for _ in range(3):  # fixed-order combine: identical bits whichever split arrives last
        assert torch.equal(y, G.linear_fwd(x, w, b, relu=True, tile=tile, splits=splits))
    dy = _rand_bf16(M, N, dev=gpu)
    db = torch.empty(K, device=gpu)
    dx = G.linear_dgrad(dy, w, relu_mask_of=x, bias_grad=db, tile=tile, splits=splits)
    refdx = (dy.float() @ w.float()) * (x.float() > 0)
    assert _rel(dx, refdx) < 5e-3
    assert _rel(db, dx.float().sum(0)) < 1e-4
    xs = x[:, :3072].contiguous()
    ws = w[:, :3072].contiguous()
    y3 = G.linear_fwd(xs, ws, b, relu=True, tile=tile, splits=splits)
    assert _rel(y3, torch.relu(xs.float() @ ws.float().t() + b)) < 5e-3
    # ragged shapes (row / column tails, uneven K split)
    for (m, n, k) in ((200, 392, 2048), (512, 136, 1088)):
        xa = _rand_bf16(m, k, dev=gpu)
        wa = (torch.randn(n, k, device=gpu) * 0.05).to(torch.bfloat16)
        ba = torch.randn(n, device=gpu)
        sp = None if splits is None else min(splits, k // 512)
        ya = G.linear_fwd(xa, wa, ba, relu=False, tile=tile, splits=sp)
        assert _rel(ya, xa.float() @ wa.float().t() + ba) < 5e-3, (m, n, k)


def test_splitk_graph_replays(gpu):
    """In-launch split-K inside a captured graph: tickets reset by every launch, replays reproduce eager."""
    from ddpx.ops import gemm as G
    torch.manual_seed(8)
    M, K, N = 512, 3072, 4096
    x = _rand_bf16(M, K, dev=gpu)
    w = (torch.randn(N, K, device=gpu) * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device=gpu)
    out = torch.empty(M, N, dtype=torch.bfloat16, device=gpu)
    G.linear_fwd(x, w, b, relu=True, out=out, tile=14, splits=2)
    eager = out.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            G.linear_fwd(x, w, b, relu=True, out=out, tile=14, splits=2)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(5):
        out.zero_()
        g.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, eager)


def test_device_lr_schedule_matches_lambdalr(gpu):
    """SGD.attach_device_schedule: the device table + counter reproduce torch LambdaLR step by step."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.optim.schedule import one_cycle
    from ddpx.optim.sgd import SGD
    m = MLP(hidden=256)
    ddpx.prepare_model(m, gpu)
    opt = SGD(m.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4, capturable=True)
    sched = one_cycle(opt, 7, num_epochs=3)
    for _ in range(3):  # start mid-schedule
        sched.step()
    assert opt.attach_device_schedule(sched)
    for _ in range(30):
        host = opt.param_groups[0]["lr"]
        opt.device_lr_step()
        assert abs(opt.lr_dev.item() - host) < 1e-7
        sched.step()


@pytest.mark.parametrize("M,N,K,mom", [(4096, 3072, 512, 0.9), (512, 384, 192, 0.9), (256, 128, 64, 0.0)])
def test_wgrad_sgd_warp_specialised_matches_unfused(gpu, M, N, K, mom):
    """dW = dY^T X applied as an SGD update by the warp-specialised kernel (MFMA waves + optimizer stream
    waves) == fp32 dW from the GEMM + the flat SGD pass, bit for bit (master, momentum, shadow)."""
    from ddpx.ops import gemm as G
    from ddpx.ops.elementwise import sgd_flat_
    torch.manual_seed(9)
    dy = _rand_bf16(K, M, dev=gpu)
    x = _rand_bf16(K, N, dev=gpu)
    p0 = torch.randn(M * N, device=gpu) * 0.02
    b0 = torch.randn(M * N, device=gpu) * 0.01
    lr = torch.full((), 0.05, device=gpu)
    pa, ba = p0.clone(), b0.clone()
    sa = torch.empty(M * N, dtype=torch.bfloat16, device=gpu)
    G.linear_wgrad(dy, x, None, sgd=(pa, ba if mom else None, sa, lr, mom, 5e-4))
    g = torch.empty(M, N, device=gpu)
    G.linear_wgrad(dy, x, g)
    pb, bb = p0.clone(), b0.clone()
    sb = torch.empty_like(sa)
    sgd_flat_(pb, bb if mom else pb, g.view(-1), sb, lr, mom, 5e-4)
    torch.cuda.synchronize()
    assert torch.equal(pa, pb)
    assert torch.equal(sa, sb)
    if mom:
        assert torch.equal(ba, bb)


@pytest.mark.parametrize("mom", [0.9, 0.0])
def test_wgrad_sgd_pair_matches_single_launches(gpu, mom):
    """Two fused weight-gradient + SGD updates in ONE warp-specialised launch (the toy MLP's fc1 + fc0)
    == the same two updates launched one by one, bit for bit (master, momentum, shadow)."""
    from ddpx.ops import gemm as G
    torch.manual_seed(10)
    K = 512
    shapes = [(256, 512), (128, 384)]  # (M_out, N_in) of the two layers
    dys = [_rand_bf16(K, m, dev=gpu) for m, _ in shapes]
    xs = [_rand_bf16(K, n, dev=gpu) for _, n in shapes]
    lr = torch.full((), 0.05, device=gpu)
    init = [(torch.randn(m * n, device=gpu) * 0.02, torch.randn(m * n, device=gpu) * 0.01) for m, n in shapes]

    def state():
        return [(p.clone(), b.clone(), torch.empty(p.numel(), dtype=torch.bfloat16, device=gpu)) for p, b in init]

    sa, sb = state(), state()
    specs = [(p, b if mom else None, s, lr, mom, 5e-4) for p, b, s in sa]
    assert G.wgrad_sgd_pair(dys[0], xs[0], specs[0], dys[1], xs[1], specs[1])
    for dy, x, (p, b, s) in zip(dys, xs, sb):
        G.linear_wgrad(dy, x, None, sgd=(p, b if mom else None, s, lr, mom, 5e-4))
    torch.cuda.synchronize()
    for (pa, ba, sha), (pb, bb, shb) in zip(sa, sb):
        assert torch.equal(pa, pb)
        assert torch.equal(sha, shb)
        if mom:
            assert torch.equal(ba, bb)


@pytest.mark.parametrize("mom", [0.9, 0.0])
def test_wgrad_sgd_dgrad_matches_dgrad_plus_pair(gpu, mom):
    """fc1's data gradient folded into the fc1 + fc0 weight-gradient + SGD launch (ddpx_wsgd_dgrad.h) == the
    standalone dgrad (ReLU mask, bf16 dX, fused fc0-bias SGD) + the pair launch, bit for bit: dX, both
    weights' master / momentum / bf16 copy, the bias' master / momentum.  Launched twice: the published-tile
    counter and the column tickets are re-zeroed by every launch."""
    from ddpx.ops import gemm as G
    torch.manual_seed(11)
    K, M1, N1, N0 = 512, 4096, 4096, 3072
    dy1 = (torch.randn(K, M1, device=gpu) * 0.05).to(torch.bfloat16)
    x1 = torch.relu(torch.randn(K, N1, device=gpu)).to(torch.bfloat16)  # H0 (half zeros: the mask matters)
    x0 = torch.rand(K, N0, device=gpu).to(torch.bfloat16)
    w1 = (torch.randn(M1, N1, device=gpu) * 0.02).to(torch.bfloat16)
    lr = torch.full((), 0.05, device=gpu)

    def state():
        g = torch.Generator(device=gpu).manual_seed(12)
        mk = lambda n: (torch.randn(n, device=gpu, generator=g) * 0.02,  # noqa: E731
                        torch.randn(n, device=gpu, generator=g) * 0.01,
                        torch.zeros(n, dtype=torch.bfloat16, device=gpu))
        return [mk(M1 * N1), mk(N1 * N0), mk(N1)]

    def spec(t):
        p, b, sh = t
        return (p, b if mom else None, sh, lr, mom, 5e-4)

    fa, ra = state(), state()
    for it in range(2):
        dx = G.wgrad_sgd_dgrad(dy1, x1, spec(fa[0]), w1, x1, x0, spec(fa[1]), spec(fa[2]))
        assert dx is not None, "toy-MLP shapes must be eligible"
        dxr = G.linear_dgrad(dy1, w1, relu_mask_of=x1, bias_sgd=spec(ra[2]))
        assert G.wgrad_sgd_pair(dy1, x1, spec(ra[0]), dxr, x0, spec(ra[1]))
        torch.cuda.synchronize()
        done, err = G.wgrad_sgd_dgrad_state(gpu, N1)
        assert err == 0 and done == (K // 64) * (N1 // 128), (done, err)
        assert torch.equal(dx, dxr), it
        for (pa, ba, sa), (pb, bb, sb) in zip(fa, ra):
            assert torch.equal(pa, pb), it
            assert torch.equal(sa, sb), it
            if mom:
                assert torch.equal(ba, bb), it


@pytest.mark.parametrize("graph", [False, True])
def test_toy_mlp_fused_dgrad_step_bitwise(gpu, graph):
    """The toy MLP (3072-4096-4096-10, batch 512) with fc1's data gradient inside the fused weight-gradient +
    SGD launch and fc1's bf16 copy ping-ponged between two buffers (eager, and as a 2-version captured cycle)
    == materialised fp32 gradients + the flat SGD pass, bit for bit over 5 steps."""
    import ddpx
    import ddpx.ops.mlp as mlp_ops
    from ddpx.models import MLP
    from ddpx.optim.sgd import SGD
    from ddpx.runtime.graphs import CapturedCycle, pingpong_signature_of
    old = mlp_ops._DGRAD_FUSE
    mlp_ops._DGRAD_FUSE = True  # opt-in path (DDPX_DGRAD_FUSE=1)
    try:
        _fused_dgrad_step(gpu, graph, ddpx, MLP, SGD, CapturedCycle, pingpong_signature_of)
    finally:
        mlp_ops._DGRAD_FUSE = old


def _fused_dgrad_step(gpu, graph, ddpx, MLP, SGD, CapturedCycle, pingpong_signature_of):
    torch.manual_seed(13)
    a, b = MLP(hidden=4096), MLP(hidden=4096)
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        ddpx.prepare_model(m, gpu)
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, capturable=True, fused_backward=True)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    xs = [torch.rand(512, 3072, device=gpu).to(torch.bfloat16) for _ in range(5)]
    ts = [torch.randint(0, 10, (512,), device=gpu) for _ in range(5)]

    def body(x, y):
        oa.zero_grad()
        loss, _ = a.forward_loss(x, y)
        loss.backward()
        oa.step()
        return loss

    oa.sync_lr()
    la = [body(xs[0], ts[0]).item()]
    assert getattr(a, "_dg_fuse_ok", None) is True, "the fused data-gradient launch must be eligible here"
    assert a.fc1.weight._ddpx_flat.has_pingpong(a.fc1.weight)
    if graph:
        g = CapturedCycle(body, xs[1], ts[1], signature=pingpong_signature_of(oa))
        assert g.period == 2
        # an ODD number of replays, then an eager step: the host's ping-pong parity must follow the replays
        # (the eager step reads the bf16 copy the last replay wrote)
        la += [g(xs[i], ts[i]).item() for i in range(1, 4)]
        la.append(body(xs[4], ts[4]).item())
    else:
        la += [body(xs[i], ts[i]).item() for i in range(1, 5)]
    lb = []
    for i in range(5):
        ob.zero_grad()
        loss, _ = b.forward_loss(xs[i], ts[i])
        loss.backward()
        ob.step()
        lb.append(loss.item())
    assert la == lb
    for (n, p), q in zip(a.named_parameters(), b.parameters()):
        assert torch.equal(p, q), n
    assert torch.equal(oa.momentum_buffer, ob.momentum_buffer)
    fa, fb = a.fc1.weight._ddpx_flat, b.fc1.weight._ddpx_flat
    for (n, p), q in zip(a.named_parameters(), b.parameters()):  # the CURRENT bf16 copies agree too
        assert torch.equal(fa.shadow_of(p), fb.shadow_of(q)), n
