"""MX-FP8 kernels (csrc/kernels/gemm_mx8.hip) vs plain PyTorch fp32 references."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _rand_codes(shape, fmt, dev, g):
    """fp8 codes of small integers (exact in both formats) as uint8."""
    from ddpx.ops.fp8 import _TORCH_FP8
    v = torch.randint(-6, 7, shape, generator=g).float()
    return v.to(_TORCH_FP8[fmt]).view(torch.uint8).to(dev)


@pytest.mark.parametrize("fa", [0, 1])
def test_mx_mfma_operand_map(gpu, fa):
    """One v_mfma_scale_f32_16x16x128_f8f6f4 with asymmetric data and per-(row, block) scales."""
    from ddpx.ops.fp8 import MX, probe
    g = torch.Generator().manual_seed(fa)
    A = _rand_codes((16, 128), fa, gpu, g)
    B = _rand_codes((16, 128), 0, gpu, g)
    sa = torch.randint(122, 132, (16, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(gpu)
    sb = torch.randint(122, 132, (16, 4), generator=g, dtype=torch.int32).to(torch.uint8).to(gpu)
    C = probe(A, B, sa, sb, fa)
    ref = MX(A, sa, fa).dequant() @ MX(B, sb, 0).dequant().t()
    assert torch.allclose(C, ref, rtol=1e-6, atol=0), (C - ref).abs().max().item()


@pytest.mark.parametrize("fmt", [0, 1])
@pytest.mark.parametrize("shape", [(64, 3072), (512, 160), (96, 64)])
def test_mx_quant_rows_and_cols(gpu, fmt, shape):
    from ddpx.ops.fp8 import quant, quant_reference
    torch.manual_seed(1)
    x = (torch.randn(*shape, device=gpu) * torch.logspace(-3, 2, shape[1], device=gpu)).to(torch.bfloat16)
    x[0, :32] = 0  # an all-zero block
    a, at = quant(x, fmt, rows=True, cols=True)
    r = quant_reference(x.cpu(), fmt)
    assert torch.equal(a.s.cpu(), r.s)
    agree = (a.q.cpu() == r.q).float().mean().item()
    assert agree > 0.999, agree
    assert _rel(a.dequant(), r.dequant().to(gpu)) < 1e-3
    rt = quant_reference(x.t().contiguous().cpu(), fmt)
    assert torch.equal(at.s.cpu(), rt.s)
    assert (at.q.cpu() == rt.q).float().mean().item() > 0.999
    # quantisation error of the format itself
    bound = 0.07 if fmt == 0 else 0.14
    assert _rel(a.dequant(), x.float()) < bound


@pytest.mark.parametrize("fa", [0, 1])
@pytest.mark.parametrize("MNK", [(512, 1024, 3072), (300, 200, 256), (128, 384, 128)])
def test_mx_gemm_matches_dequant_reference(gpu, fa, MNK):
    from ddpx.ops import fp8
    M, N, K = MNK
    torch.manual_seed(2)
    x = (torch.randn(M, K, device=gpu)).to(torch.bfloat16)
    w = (torch.randn(N, K, device=gpu) * 0.05).to(torch.bfloat16)
    a = fp8.quant(x, fa)
    b = fp8.quant(w, fp8.E4M3)
    ref = a.dequant() @ b.dequant().t()
    c32 = fp8.gemm(a, b, epi=fp8.EPI_F32)
    assert _rel(c32, ref) < 5e-5  # fp32 accumulation order differs from torch's
    bias = torch.randn(N, device=gpu)
    c16 = fp8.gemm(a, b, epi=fp8.EPI_BIAS_RELU_BF16, bias=bias)
    assert _rel(c16, torch.relu(ref + bias)) < 5e-3
    # against the unquantised bf16 product: the MX-fp8 error budget
    exact = x.float() @ w.float().t()
    assert _rel(c32, exact) < (0.06 if fa == 0 else 0.12)


def test_mx_gemm_sgd_epilogue(gpu):
    """fp8 wgrad with the fused SGD epilogue == fp32 wgrad + torch-style SGD on the same values."""
    from ddpx.ops import fp8
    torch.manual_seed(3)
    M, N, K = 256, 384, 512  # dW [M=out, N=in], reduction over K = batch
    dyT = (torch.randn(M, K, device=gpu) * 0.1).to(torch.bfloat16)
    xT = torch.randn(N, K, device=gpu).to(torch.bfloat16)
    a = fp8.quant(dyT, fp8.E5M2)
    b = fp8.quant(xT, fp8.E4M3)
    g = a.dequant() @ b.dequant().t()
    p = torch.randn(M * N, device=gpu) * 0.02
    buf = torch.randn(M * N, device=gpu) * 0.01
    sh = torch.empty(M * N, dtype=torch.bfloat16, device=gpu)
    lr = torch.full((), 0.1, device=gpu)
    p_ref, b_ref = p.clone(), buf.clone()
    fp8.gemm(a, b, epi=fp8.EPI_SGD, sgd=(p, buf, sh, lr, 0.9, 5e-4))
    d = g.reshape(-1) + 5e-4 * p_ref
    b_ref = 0.9 * b_ref + d
    p_ref = p_ref - 0.1 * b_ref
    assert _rel(buf, b_ref) < 1e-4 and _rel(p, p_ref) < 1e-4
    assert torch.equal(sh, p.to(torch.bfloat16))


@pytest.mark.parametrize("wgrad8", [False, True])
def test_mlp_fp8_step_tracks_bf16(gpu, wgrad8, monkeypatch):
    """A whole MX-FP8 MLP training step (fp8 forward; fp8 weight gradients too with DDPX_FP8_WGRAD) stays
    close to the bf16 step."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.ops import mlp as mlp_ops
    monkeypatch.setattr(mlp_ops, "_FP8_WGRAD", wgrad8)
    torch.manual_seed(4)
    a, b = MLP(hidden=1024), MLP(hidden=1024)
    b.load_state_dict(a.state_dict())
    a.fp8 = True
    for m in (a, b):
        ddpx.prepare_model(m, gpu)
    x = torch.rand(256, 3072, device=gpu).to(torch.bfloat16)
    t = torch.randint(0, 10, (256,), device=gpu)
    la, _ = a.forward_loss(x, t)
    lb, _ = b.forward_loss(x, t)
    la.backward()
    lb.backward()
    assert abs(la.item() - lb.item()) < 0.02 * abs(lb.item())
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        cos = torch.nn.functional.cosine_similarity(p.main_grad.flatten(), q.main_grad.flatten(), dim=0).item()
        assert cos > 0.97 and _rel(p.main_grad, q.main_grad) < 0.3, (n, cos)
    with torch.no_grad():
        assert _rel(a(x), b(x)) < 0.06


def test_sgd_flat_emits_mx8_copy(gpu):
    """The flat SGD's MX-FP8 output (codes + E8M0 scales of every 32-element run) == the separate quantiser
    applied to the bf16 copy it wrote, byte for byte."""
    from ddpx.ops import fp8 as F8
    from ddpx.ops.elementwise import sgd_flat_
    torch.manual_seed(12)
    n = 32 * 4099  # not a multiple of the grid stride: partial last iteration
    p = torch.randn(n, device=gpu) * 0.05
    p[:32] = 0.0  # an all-zero block (scale byte 0)
    buf = torch.randn(n, device=gpu) * 0.01
    g = torch.randn(n, device=gpu) * 0.1
    sh = torch.empty(n, dtype=torch.bfloat16, device=gpu)
    q = torch.empty(n, dtype=torch.uint8, device=gpu)
    s = torch.empty(n // 32, dtype=torch.uint8, device=gpu)
    lr = torch.full((), 0.05, device=gpu)
    sgd_flat_(p, buf, g, sh, lr, 0.9, 5e-4, mx8=(q, s))
    ref = F8.quant(sh.view(-1, 32), F8.E4M3)
    torch.cuda.synchronize()
    assert torch.equal(q.view(-1, 32), ref.q)
    assert torch.equal(s.view(-1, 1), ref.s)


@pytest.mark.parametrize("mom", [0.9, 0.0])
def test_wgrad_sgd_pair_emits_mx8_copy(gpu, mom):
    """The warp-specialised weight-gradient + SGD pair's stream waves write both weights' MX-FP8 copies:
    equal to the quantiser run on the bf16 copies, and master / momentum / bf16 unchanged by the extra output."""
    from ddpx.ops import fp8 as F8
    from ddpx.ops import gemm as G
    torch.manual_seed(13)
    K = 512
    shapes = [(256, 512), (128, 384)]
    dys = [((torch.rand(K, m, device=gpu) * 2 - 1) * 0.1).to(torch.bfloat16) for m, _ in shapes]
    xs = [((torch.rand(K, n, device=gpu) * 2 - 1)).to(torch.bfloat16) for _, n in shapes]
    lr = torch.full((), 0.05, device=gpu)
    init = [(torch.randn(m * n, device=gpu) * 0.02, torch.randn(m * n, device=gpu) * 0.01) for m, n in shapes]

    def state():
        return [(p.clone(), b.clone(), torch.empty(p.numel(), dtype=torch.bfloat16, device=gpu)) for p, b in init]

    sa, sb = state(), state()
    mxs = [(torch.empty(m, n, dtype=torch.uint8, device=gpu), torch.empty(m, n // 32, dtype=torch.uint8, device=gpu))
           for m, n in shapes]
    spec = lambda st: [(p, b if mom else None, s, lr, mom, 5e-4) for p, b, s in st]  # noqa: E731
    a, b = spec(sa), spec(sb)
    assert G.wgrad_sgd_pair(dys[0], xs[0], a[0], dys[1], xs[1], a[1], mxs[0], mxs[1])
    assert G.wgrad_sgd_pair(dys[0], xs[0], b[0], dys[1], xs[1], b[1])
    torch.cuda.synchronize()
    for (m, n), (pa, ba, sha), (pb, bb, shb), (q, s) in zip(shapes, sa, sb, mxs):
        assert torch.equal(pa, pb) and torch.equal(sha, shb)
        if mom:
            assert torch.equal(ba, bb)
        ref = F8.quant(sha.view(m, n), F8.E4M3)
        assert torch.equal(q, ref.q)
        assert torch.equal(s, ref.s)


@pytest.mark.parametrize("fused", [True, False])
@pytest.mark.parametrize("from_opt", [True, False])
def test_mlp_fp8_weight_copy_written_by_optimizer(gpu, fused, from_opt):
    """fp8 MLP training: the hidden weights' fp8 copy used by each forward equals the quantiser's output for
    the bf16 copy.  With the optimizer writing it (DDPX_FP8_COPY=1: the fused pair or the flat SGD) the forward
    never re-quantises after the first step; without (DDPX_FP8_COPY=0) it re-quantises both weights every step."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.ops import fp8 as F8
    from ddpx.optim.sgd import SGD
    torch.manual_seed(5)
    m = MLP(hidden=512)
    m.fp8 = True
    ddpx.prepare_model(m, gpu)
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, capturable=True, fused_backward=fused)
    x = torch.rand(512, 3072, device=gpu).to(torch.bfloat16)
    t = torch.randint(0, 10, (512,), device=gpu)
    flat = m.fc0.weight._ddpx_flat
    flat.fp8_from_optimizer = flat.fp8_from_flat_sgd = from_opt
    calls = []
    orig = F8.quant
    for step in range(3):
        opt.zero_grad()
        F8.quant = lambda *a, **k: (calls.append(k.get("out") is not None), orig(*a, **k))[1]
        try:
            loss, _ = m.forward_loss(x, t)
        finally:
            F8.quant = orig
        loss.backward()
        opt.step()
        # step 0 quantises the initial weights into the store; later forwards reuse the optimizer's copy
        assert sum(calls) == (2 if (step == 0 or not from_opt) else 0), (step, calls)
        calls.clear()
        for lin in m.linears()[:-1]:
            w = lin.weight
            assert flat.fp8_fresh[flat.index[id(w)]] == from_opt
            if from_opt:
                q, s = flat.mx8_views(w)
                ref = F8.quant(flat.shadow_of(w), F8.E4M3)
                torch.cuda.synchronize()
                assert torch.equal(q, ref.q) and torch.equal(s, ref.s), (step, lin)
    assert torch.isfinite(loss).item()


@pytest.mark.parametrize("fused", [True, False])
def test_mlp_fp8_dgrad_step_tracks_bf16(gpu, fused, monkeypatch):
    """DDPX_FP8_DGRAD=1: the hidden data gradients on MX-FP8 (W quantised transposed per step) - the step's
    gradients / updates stay close to the bf16 step's, with the fused optimizer and with stored gradients."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.ops import mlp as mlp_ops
    from ddpx.optim.sgd import SGD
    monkeypatch.setattr(mlp_ops, "_FP8_DGRAD", True)
    torch.manual_seed(5)
    a, b = MLP(hidden=1024), MLP(hidden=1024)
    b.load_state_dict(a.state_dict())
    a.fp8 = True
    for m in (a, b):
        ddpx.prepare_model(m, gpu)
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, fused_backward=fused)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, fused_backward=fused)
    w0 = [p.detach().clone() for p in b.parameters()]
    x = torch.rand(256, 3072, device=gpu).to(torch.bfloat16)
    t = torch.randint(0, 10, (256,), device=gpu)
    for m, o in ((a, oa), (b, ob)):
        o.sync_lr()
        o.zero_grad()
        loss, _ = m.forward_loss(x, t)
        loss.backward()
        o.step()
    for (n, p), q, p0 in zip(a.named_parameters(), b.parameters(), w0):
        du, dr = (p - p0).float().flatten(), (q - p0).float().flatten()
        cos = torch.nn.functional.cosine_similarity(du, dr, dim=0).item()
        assert cos > 0.97, (n, cos)


@pytest.mark.parametrize("both", [True, False])
def test_wgrad_sgd_pair_emits_transposed_mx8_copy(gpu, both):
    """The pair's stream waves also write Wᵀ as MX-FP8 with 32-blocks along W's rows (the fp8 data gradient's
    operand, 8 stream waves): equal to the quantiser's transposed output for the bf16 copy, and master / momentum /
    bf16 / row copy unchanged by the extra output (against a launch without it).  ``both=False``: only the first
    GEMM asks for it (the MLP's fc0 has no data gradient)."""
    from ddpx.ops import fp8 as F8
    from ddpx.ops import gemm as G
    torch.manual_seed(17)
    K = 512
    shapes = [(256, 512), (128, 384)]
    dys = [((torch.rand(K, m, device=gpu) * 2 - 1) * 0.1).to(torch.bfloat16) for m, _ in shapes]
    xs = [((torch.rand(K, n, device=gpu) * 2 - 1)).to(torch.bfloat16) for _, n in shapes]
    lr = torch.full((), 0.05, device=gpu)
    init = [(torch.randn(m * n, device=gpu) * 0.02, torch.randn(m * n, device=gpu) * 0.01) for m, n in shapes]

    def state():
        return [(p.clone(), b.clone(), torch.empty(p.numel(), dtype=torch.bfloat16, device=gpu)) for p, b in init]

    def mx_rows():
        return [(torch.empty(m, n, dtype=torch.uint8, device=gpu), torch.empty(m, n // 32, dtype=torch.uint8,
                                                                               device=gpu)) for m, n in shapes]
    sa, sb = state(), state()
    ra, rb = mx_rows(), mx_rows()
    mxt = [(torch.full((n, m), 0xAB, dtype=torch.uint8, device=gpu),
            torch.full((n, m // 32), 0xAB, dtype=torch.uint8, device=gpu)) for m, n in shapes]
    spec = lambda st: [(p, b, s, lr, 0.9, 5e-4) for p, b, s in st]  # noqa: E731
    a, b = spec(sa), spec(sb)
    assert G.wgrad_sgd_pair(dys[0], xs[0], a[0], dys[1], xs[1], a[1], ra[0], ra[1], mxt[0], mxt[1] if both else None)
    assert G.wgrad_sgd_pair(dys[0], xs[0], b[0], dys[1], xs[1], b[1], rb[0], rb[1])
    torch.cuda.synchronize()
    for i, ((m, n), (pa, ba, sha), (pb, bb, shb)) in enumerate(zip(shapes, sa, sb)):
        assert torch.equal(pa, pb) and torch.equal(ba, bb) and torch.equal(sha, shb)
        assert torch.equal(ra[i][0], rb[i][0]) and torch.equal(ra[i][1], rb[i][1])
        if i == 1 and not both:
            assert bool((mxt[1][0] == 0xAB).all()) and bool((mxt[1][1] == 0xAB).all())  # untouched
            continue
        ref = F8.quant(sha.view(m, n), F8.E4M3, rows=False, cols=True)
        assert torch.equal(mxt[i][0], ref.q), i
        assert torch.equal(mxt[i][1], ref.s), i


def test_mlp_fp8_dgrad_reads_pair_written_transposed_copy(gpu, monkeypatch):
    """DDPX_FP8_DGRAD=1 with the fused optimizer: after the first step the fc1 data gradient's transposed MX operand
    is the one the previous step's wgrad+SGD pair wrote (no per-step transposed quantisation), and it equals the
    quantiser's output for the bf16 copy."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.ops import fp8 as F8
    from ddpx.ops import mlp as mlp_ops
    from ddpx.optim.sgd import SGD
    monkeypatch.setattr(mlp_ops, "_FP8_DGRAD", True)
    torch.manual_seed(6)
    m = MLP(hidden=512)
    m.fp8 = True
    ddpx.prepare_model(m, gpu)
    opt = SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, capturable=True, fused_backward=True)
    x = torch.rand(512, 3072, device=gpu).to(torch.bfloat16)
    t = torch.randint(0, 10, (512,), device=gpu)
    flat = m.fc0.weight._ddpx_flat
    orig = F8.quant
    calls = []
    for step in range(3):
        opt.zero_grad()
        F8.quant = lambda *a, **k: (calls.append(k.get("out_t") is not None), orig(*a, **k))[1]
        try:
            loss, _ = m.forward_loss(x, t)
            loss.backward()
        finally:
            F8.quant = orig
        opt.step()
        assert sum(calls) == (1 if step == 0 else 0), (step, calls)
        calls.clear()
        w1 = m.linears()[1].weight
        assert flat.fp8t_fresh[flat.index[id(w1)]]
        q, s = flat.mx8t_views(w1)
        ref = F8.quant(flat.shadow_of(w1), F8.E4M3, rows=False, cols=True)
        torch.cuda.synchronize()
        assert torch.equal(q, ref.q) and torch.equal(s, ref.s), step
    assert torch.isfinite(loss).item()
