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
