"""Native conv / BatchNorm / pool kernels and the native VGG vs PyTorch fp32 references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _rel(a, b):
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _bf(t):
    return t.to(torch.bfloat16).float()


@pytest.mark.parametrize("N,H,Ci,Co", [(4, 32, 3, 64), (8, 16, 64, 128), (16, 8, 128, 256), (32, 4, 256, 512),
                                       (64, 2, 512, 512), (6, 32, 64, 64),
                                       # non-power-of-two H, W and channel counts: the im2col addressing
                                       # divides by them with multiply-high fast division
                                       (3, 12, 24, 40), (5, 6, 3, 24), (2, 10, 40, 48), (7, 5, 16, 8)])
def test_conv_fwd_dgrad_wgrad(gpu, N, H, Ci, Co):
    from ddpx.ops import conv as K
    torch.manual_seed(0)
    Cp = K.padded_channels(Ci)
    x = _bf(torch.randn(N, Ci, H, H, device=gpu))
    w = torch.randn(Co, Ci, 3, 3, device=gpu) * (1.0 / (Ci * 9) ** 0.5)
    xn = F.pad(x.permute(0, 2, 3, 1), (0, Cp - Ci)).to(torch.bfloat16).contiguous()
    wf = torch.empty(Co * 9 * Cp, dtype=torch.bfloat16, device=gpu)
    wd = torch.empty_like(wf)
    K.weight_prep(w, wf, wd)
    y, st, T, BM = K.conv_fwd(xn, wf, Co)
    ref = F.conv2d(x, _bf(w), padding=1)  # [N,Co,H,W]
    refn = ref.permute(0, 2, 3, 1).reshape(-1, Co)
    assert _rel(y, refn) < 1e-2
    # per-tile BN statistics of the stored bf16 values
    yf = y.float()
    for t in (0, T - 1):
        rows = yf[t * BM:min((t + 1) * BM, yf.shape[0])]
        assert torch.allclose(st[t, 0], rows.mean(0), rtol=1e-3, atol=1e-3)
        assert torch.allclose(st[t, 1], ((rows - rows.mean(0)) ** 2).sum(0), rtol=2e-3, atol=1e-2)
    # backward
    dy = _bf(torch.randn(N * H * H, Co, device=gpu))
    dyn = dy.view(N, H, H, Co).permute(0, 3, 1, 2)
    xr = x.clone().requires_grad_(True)
    wr = _bf(w).clone().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(dyn)
    dx = K.conv_dgrad(dy.to(torch.bfloat16), wd, N, H, H, Cp, Co)
    assert _rel(dx[..., :Ci].permute(0, 3, 1, 2), xr.grad) < 1e-2
    if Cp > Ci:
        assert torch.all(dx[..., Ci:] == 0)  # zero-padded weight channels give exactly zero gradient
    dw = torch.empty(Co, Ci, 3, 3, device=gpu)
    K.conv_wgrad(dy.to(torch.bfloat16), xn, Co, Ci, out=dw)
    assert _rel(dw, wr.grad) < 5e-3


@pytest.mark.parametrize("tile", [21, 22, 23])
@pytest.mark.parametrize("N,H,Ci,Co", [(8, 32, 64, 128), (3, 12, 24, 40), (16, 8, 256, 256)])
def test_conv_two_deep_128_tiles(gpu, tile, N, H, Ci, Co):
    """The 2-deep ring configs (two workgroups per CU): 128x128 (statistics per 64-row epilogue half), 256x64."""
    from ddpx.ops import conv as K
    torch.manual_seed(3)
    Cp = K.padded_channels(Ci)
    x = _bf(torch.randn(N, Ci, H, H, device=gpu))
    w = torch.randn(Co, Ci, 3, 3, device=gpu) * (1.0 / (Ci * 9) ** 0.5)
    xn = F.pad(x.permute(0, 2, 3, 1), (0, Cp - Ci)).to(torch.bfloat16).contiguous()
    wf = torch.empty(Co * 9 * Cp, dtype=torch.bfloat16, device=gpu)
    wd = torch.empty_like(wf)
    K.weight_prep(w, wf, wd)
    y, st, T, BM = K.conv_fwd(xn, wf, Co, tile=tile)
    assert BM == (256 if tile == 23 else 128)  # one statistics row per tile (row parts merged in the epilogue)
    refn = F.conv2d(x, _bf(w), padding=1).permute(0, 2, 3, 1).reshape(-1, Co)
    assert _rel(y, refn) < 1e-2
    yf = y.float()
    for t in (0, T // 2, T - 1):
        rows = yf[t * BM:min((t + 1) * BM, yf.shape[0])]
        if rows.shape[0] == 0:  # a trailing epilogue half wholly past P: zero statistics, weight 0 in the merge
            assert torch.all(st[t] == 0)
            continue
        assert torch.allclose(st[t, 0], rows.mean(0), rtol=1e-3, atol=1e-3)
        assert torch.allclose(st[t, 1], ((rows - rows.mean(0)) ** 2).sum(0), rtol=2e-3, atol=1e-2)
    dy = _bf(torch.randn(N * H * H, Co, device=gpu))
    xr = x.clone().requires_grad_(True)
    wr = _bf(w).clone().requires_grad_(True)
    F.conv2d(xr, wr, padding=1).backward(dy.view(N, H, H, Co).permute(0, 3, 1, 2))
    dx = K.conv_dgrad(dy.to(torch.bfloat16), wd, N, H, H, Cp, Co, tile=tile)
    assert _rel(dx[..., :Ci].permute(0, 3, 1, 2), xr.grad) < 1e-2
    dw = torch.empty(Co, Ci, 3, 3, device=gpu)
    K.conv_wgrad(dy.to(torch.bfloat16), xn, Co, Ci, out=dw, tile=tile)
    assert _rel(dw, wr.grad) < 5e-3


@pytest.mark.parametrize("pool", [False, True])
def test_bn_relu_pool_fwd_bwd(gpu, pool):
    from ddpx.ops import conv as K
    torch.manual_seed(1)
    N, H, C = 8, 8, 64
    y = _bf(torch.randn(N * H * H, C, device=gpu) * 2 + 0.5)
    bn = torch.nn.BatchNorm2d(C).to(gpu)
    with torch.no_grad():
        bn.weight.uniform_(0.5, 1.5)
        bn.bias.uniform_(-0.5, 0.5)
    bn_ref = torch.nn.BatchNorm2d(C).to(gpu)
    bn_ref.load_state_dict(bn.state_dict())
    # statistics as the conv epilogue would produce them (tiles of 64 rows)
    BM = 64
    T = y.shape[0] // BM
    st = torch.stack([torch.stack([y[t * BM:(t + 1) * BM].mean(0),
                                   ((y[t * BM:(t + 1) * BM] - y[t * BM:(t + 1) * BM].mean(0)) ** 2).sum(0)])
                      for t in range(T)])
    a, b, mean, rstd = (torch.empty(C, device=gpu) for _ in range(4))
    K.bn_finalize(st.contiguous(), T, BM, N * H * H, bn, True, a, b, mean, rstd)
    out = K.bn_apply(y.to(torch.bfloat16).contiguous(), a, b, N, H, H, C, relu=True, pool=pool)
    yn = y.view(N, H, H, C).permute(0, 3, 1, 2).clone().requires_grad_(True)
    z = F.relu(bn_ref(yn))
    if pool:
        z = F.max_pool2d(z, 2)
    assert _rel(out.permute(0, 3, 1, 2), z) < 1e-2
    assert torch.allclose(bn.running_mean, bn_ref.running_mean, rtol=1e-4, atol=1e-5)
    assert torch.allclose(bn.running_var, bn_ref.running_var, rtol=1e-4, atol=1e-5)
    assert int(bn.num_batches_tracked) == 1
    g = _bf(torch.randn_like(z))
    z.backward(g)
    dg = torch.empty(C, device=gpu)
    db = torch.empty(C, device=gpu)
    dy = K.bn_backward(g.permute(0, 2, 3, 1).to(torch.bfloat16).contiguous(), y.to(torch.bfloat16).contiguous(),
                       a, b, mean, rstd, N, H, H, C, pool, dgamma=dg, dbeta=db)
    assert _rel(dg, bn_ref.weight.grad) < 1e-2
    assert _rel(db, bn_ref.bias.grad) < 1e-2
    assert _rel(dy.view(N, H, H, C).permute(0, 3, 1, 2), yn.grad) < 2e-2


def _vgg_pair(gpu, seed=0):
    import ddpx
    from ddpx.models import VGG
    torch.manual_seed(seed)
    m = VGG()
    ref = VGG()
    ref.load_state_dict(m.state_dict())
    m.use_native = True
    ddpx.prepare_model(m, gpu)
    ref.to(gpu)
    return m, ref


def test_vgg_native_matches_torch(gpu):
    """Whole native VGG (bf16 NHWC) vs torch fp32; the error budget is set by torch's own bf16 autocast
    error on the same batch (same precision class), since bf16 rounding compounds through 8 BN layers."""
    import copy
    torch.manual_seed(2)
    m, ref = _vgg_pair(gpu)
    amp = copy.deepcopy(ref)
    N = 32
    x = _bf(torch.rand(N, 3, 32, 32, device=gpu))
    t = torch.randint(0, 10, (N,), device=gpu)
    loss, _ = m.forward_loss(x, t)
    loss.backward()
    rl = F.cross_entropy(ref(x), t)
    rl.backward()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        al = F.cross_entropy(amp(x).float(), t)
    al.backward()
    assert abs(loss.item() - rl.item()) < 3e-2 * max(1.0, rl.item())
    for (n, p), (_, q), (_, r) in zip(m.named_parameters(), ref.named_parameters(), amp.named_parameters()):
        ours, theirs = _rel(p.main_grad, q.grad), _rel(r.grad, q.grad)
        assert ours < 3 * theirs + 0.03, (n, ours, theirs)
    for (n, bb), (_, cc) in zip(m.named_buffers(), ref.named_buffers()):
        if bb.dtype == torch.int64:
            assert int(bb) == int(cc), n
        else:
            assert _rel(bb, cc) < 2e-2, n
    # eval (running statistics)
    m.eval()
    ref.eval()
    with torch.no_grad():
        lg = m(x)
        rlg = ref(x)
    assert _rel(lg, rlg) < 5e-2


def test_vgg_fused_optimizer_bitwise(gpu):
    from ddpx.optim.sgd import SGD
    torch.manual_seed(3)
    a, _ = _vgg_pair(gpu, seed=3)
    b, _ = _vgg_pair(gpu, seed=3)
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, fused_backward=True)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    for i in range(3):
        x = torch.rand(16, 3, 32, 32, device=gpu)
        t = torch.randint(0, 10, (16,), device=gpu)
        for m, o in ((a, oa), (b, ob)):
            o.sync_lr()
            o.zero_grad()
            loss, _ = m.forward_loss(x, t)
            loss.backward()
            o.step()
    for (n, p), (_, q) in zip(a.named_parameters(), b.named_parameters()):
        assert torch.equal(p, q), n


class _MirrorComm:
    """A 2-rank communicator whose other rank holds exactly this rank's data: SyncBatchNorm over it must
    reproduce plain BatchNorm on the local batch (global statistics == local ones)."""
    world_size = 2
    rank = 0

    def allgather(self, out, inp, stream=None):
        out.view(2, -1).copy_(inp.view(1, -1).expand(2, -1))

    def allreduce_(self, t, op="sum", stream=None, async_op=False):
        assert op == "sum"
        t.mul_(2.0)


def test_native_sync_batchnorm_kernels_match_local_bn(gpu):
    """Native SyncBN forward (local stats -> all-gather -> rank-ordered merge) and backward (sums ->
    all-reduce -> apply) against the plain native BN on the same batch, through a mirror communicator."""
    import ddpx
    from ddpx.models import VGG
    torch.manual_seed(3)
    a, b = VGG(), VGG()
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        m.use_native = True
        ddpx.prepare_model(m, gpu)
    b.sync_bn_comm = _MirrorComm()
    x = torch.rand(24, 32, 32, 8, device=gpu)
    x[..., 3:] = 0
    x = x.to(torch.bfloat16)
    t = torch.randint(0, 10, (24,), device=gpu)
    la, _ = a.forward_loss(x, t)
    lb, _ = b.forward_loss(x, t)
    assert abs(la.item() - lb.item()) < 1e-4 * max(1.0, abs(la.item()))
    for (n, ba), bb in zip(a.named_buffers(), b.buffers()):
        if ba.is_floating_point():
            assert torch.allclose(ba, bb, rtol=1e-4, atol=1e-6), n
    la.backward()
    lb.backward()
    # the sync path divides (2 x local sums) by 2M instead of local sums by M: the same values up to
    # fp32 rounding, which can flip bf16 roundings of dy; 8 layers deep that stays under 2 %
    bad = [(n, _rel(q.main_grad, p.main_grad)) for (n, p), q in zip(a.named_parameters(), b.parameters())
           if _rel(q.main_grad, p.main_grad) > 2e-2]
    assert not bad, bad


@pytest.mark.parametrize("N,H,Ci,Co", [(512, 32, 8, 64), (512, 8, 256, 256), (64, 4, 512, 512), (5, 6, 16, 24)])
def test_bn_merges_match_fp64(gpu, N, H, Ci, Co):
    """BatchNorm statistics from the conv epilogue's tile partials: the two-level channel-coalesced merges
    (mode 0, DDPX_BN_MERGE=split) and the per-channel ones (mode 1) both match an fp64 reduction of the stored
    bf16 outputs (batch mean / biased variance / running stats), and so do the backward sums (c1, c2, dgamma,
    dbeta); the default (mode 2) pairs the per-channel forward merge with the split backward one."""
    from ddpx.ops import conv as K
    from ddpx.runtime import native
    torch.manual_seed(3)
    lib = native.kernels()
    xn = torch.randn(N, H, H, Ci, device=gpu).to(torch.bfloat16).contiguous()
    wf = (torch.randn(Co * 9 * Ci, device=gpu) * (1.0 / (Ci * 9) ** 0.5)).to(torch.bfloat16)
    y, st, T, BM = K.conv_fwd(xn, wf, Co)
    P = N * H * H
    y64 = y.double()
    mean64 = y64.mean(0)
    var64 = y64.var(0, unbiased=False)
    g = torch.randn(P, Co, device=gpu).to(torch.bfloat16).contiguous()
    outs = {}
    try:
        for legacy in (0, 1):
            lib.ddpx_bn_set_merge(1 if legacy else 0)
            bn = torch.nn.BatchNorm2d(Co).to(gpu)
            a, b, mean, rstd = (torch.empty(Co, device=gpu) for _ in range(4))
            K.bn_finalize(st, T, BM, P, bn, True, a, b, mean, rstd)
            dgam, dbet = torch.zeros(Co, device=gpu), torch.zeros(Co, device=gpu)
            dy = K.bn_backward(g, y, a, b, mean, rstd, N, H, H, Co, False, dgamma=dgam, dbeta=dbet)
            torch.cuda.synchronize()
            outs[legacy] = (mean.clone(), rstd.clone(), bn.running_var.clone(), dgam, dbet, dy.float())
    finally:
        lib.ddpx_bn_set_merge(-1)
    rstd64 = (var64 + 1e-5).rsqrt()
    xhat64 = (y64 - mean64) * rstd64
    gz64 = xhat64.gt(0).double() * g.double()  # gamma 1, beta 0: ReLU mask of xhat (a rare fp32 flip at 0 is
    # one |g| ~ 1 term of a sum over P elements: atol 4)
    for legacy, (mean, rstd, rvar, dgam, dbet, dy) in outs.items():
        assert torch.allclose(mean.double(), mean64, rtol=1e-5, atol=1e-5), legacy
        assert torch.allclose(rstd.double(), rstd64, rtol=1e-4, atol=1e-5), legacy
        assert torch.allclose(rvar.double(), 0.9 + 0.1 * y64.var(0, unbiased=True), rtol=1e-4, atol=1e-5), legacy
        assert torch.allclose(dbet.double(), gz64.sum(0), rtol=1e-3, atol=4.0), legacy
        assert torch.allclose(dgam.double(), (gz64 * xhat64).sum(0), rtol=1e-3, atol=4.0), legacy
    # the two merges differ only by fp32 rounding of the merge order
    assert _rel(outs[0][0], outs[1][0]) < 1e-5 and _rel(outs[0][1], outs[1][1]) < 1e-5
    assert _rel(outs[0][5], outs[1][5]) < 1e-2


@pytest.mark.parametrize("N,H,C,Co,tile", [(8, 32, 64, 128, -1), (4, 32, 64, 128, 7), (3, 16, 128, 256, -1),
                                            (2, 8, 256, 512, -1), (5, 4, 512, 512, -1), (3, 6, 64, 64, 5),
                                            (2, 32, 8, 64, -1)])
def test_im2col_row_cache_bitwise(gpu, N, H, C, Co, tile):
    """The cached im2col addressing (ImRows for the forward / data-gradient A operand when C % 64 == 0,
    ColRows for the weight-gradient B operand when W divides 64; csrc/include/ddpx_pipe.h) loads exactly the
    bytes the per-chunk path does: forward output, its BatchNorm tile statistics, the data gradient and the
    weight gradient are bitwise equal with ddpx_conv_set_rowcache(0) (ragged tiles, W = 6 and the C = 8
    fallbacks included)."""
    from ddpx.ops import conv as K
    from ddpx.runtime import native
    lib = native.kernels()
    torch.manual_seed(5)
    xn = torch.randn(N, H, H, C, device=gpu).to(torch.bfloat16).contiguous()
    w = torch.randn(Co, C, 3, 3, device=gpu) * (1.0 / (C * 9) ** 0.5)
    wf = torch.empty(Co * 9 * C, dtype=torch.bfloat16, device=gpu)
    wd = torch.empty_like(wf)
    K.weight_prep(w, wf, wd)
    dy = torch.randn(N * H * H, Co, device=gpu).to(torch.bfloat16).contiguous()
    outs = []
    try:
        for on in (1, 0):
            lib.ddpx_conv_set_rowcache(on)
            y, st, T, BM = K.conv_fwd(xn, wf, Co, tile=tile)
            dx = K.conv_dgrad(dy, wd, N, H, H, C, Co, tile=tile)
            dw = torch.empty(Co, C, 3, 3, device=gpu)
            K.conv_wgrad(dy, xn, Co, C, out=dw, tile=tile)
            torch.cuda.synchronize()
            outs.append((y, st, dx, dw))
    finally:
        lib.ddpx_conv_set_rowcache(-1)
    (y1, s1, d1, w1), (y0, s0, d0, w0) = outs
    assert torch.equal(y1, y0) and torch.equal(s1, s0) and torch.equal(d1, d0) and torch.equal(w1, w0)


@pytest.mark.parametrize("N,H,C,Co", [(4, 8, 256, 512), (2, 16, 64, 128), (3, 4, 512, 512), (2, 32, 8, 64)])
def test_wgrad_fused_sgd_writes_prepared_layouts(gpu, N, H, C, Co):
    """conv_wgrad(sgd=..., prepared=(wf, wd)): the fused update's reduce also writes the bf16 forward / dgrad
    GEMM layouts of the UPDATED weight; they equal weight_prep of the new master bitwise (the forward after a
    fused step skips weight_prep), and the master / momentum equal an unfused step."""
    from ddpx.ops import conv as K
    torch.manual_seed(11)
    Cr = 3 if C == 8 else C
    x = torch.randn(N, H, H, C, device=gpu)
    if Cr < C:
        x[..., Cr:] = 0
    xn = x.to(torch.bfloat16).contiguous()
    dy = torch.randn(N * H * H, Co, device=gpu).to(torch.bfloat16).contiguous()
    w0 = torch.randn(Co, Cr, 3, 3, device=gpu) * 0.05
    buf0 = torch.randn_like(w0) * 0.01
    lr = torch.tensor(0.1, device=gpu)
    p, buf = w0.clone(), buf0.clone()
    wf = torch.zeros(Co * 9 * C, dtype=torch.bfloat16, device=gpu)
    wd = torch.zeros_like(wf)
    K.weight_prep(w0, wf, wd)  # the padded channels' zeros the update must keep
    K.conv_wgrad(dy, xn, Co, Cr, sgd=(p, buf, None, lr, 0.9, 5e-4), prepared=(wf, wd))
    g = torch.empty_like(w0)
    K.conv_wgrad(dy, xn, Co, Cr, out=g)
    buf_ref = buf0 * 0.9 + (g + 5e-4 * w0)
    p_ref = w0 - 0.1 * buf_ref
    wf_ref, wd_ref = torch.zeros_like(wf), torch.zeros_like(wd)
    K.weight_prep(p, wf_ref, wd_ref)
    torch.cuda.synchronize()
    assert torch.equal(wf, wf_ref) and torch.equal(wd, wd_ref)
    assert torch.allclose(p, p_ref, rtol=1e-6, atol=1e-6) and torch.allclose(buf, buf_ref, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("N,H,C,Co,pool", [(8, 16, 64, 128, True), (2, 8, 256, 256, False), (64, 16, 128, 256, True),
                                           (64, 16, 256, 256, False), (16, 4, 512, 512, True), (256, 8, 256, 512, False),
                                           (512, 32, 64, 128, False)])  # VGG conv1's dx: 256x64 tile (cfg 23), unfused
def test_dgrad_bn_epilogue_matches_separate_reduce(gpu, N, H, C, Co, pool):
    """The conv data gradient with the BatchNorm backward sums of the block below in its epilogue
    (EPI_BNBWD_BF16 on tile configs 8, 15 and 22; the other picks fall back to the plain data gradient) = the plain
    data gradient + bn_backward's own reduce: g bitwise, the sums / dgamma / dbeta / dy to fp32 summation order."""
    from ddpx.ops import conv as K
    from ddpx.runtime import native
    torch.manual_seed(3)
    Hy = 2 * H if pool else H
    y = (torch.randn(N, Hy, Hy, C, device=gpu) * 1.5 + 0.3).to(torch.bfloat16).contiguous()
    a = torch.rand(C, device=gpu) + 0.5
    mean = y.float().mean((0, 1, 2))
    rstd = torch.rsqrt(y.float().var((0, 1, 2), unbiased=False) + 1e-5)
    b = torch.randn(C, device=gpu) * 0.3 - mean * a
    w = torch.randn(Co, C, 3, 3, device=gpu) / (9 * C) ** 0.5
    wf = torch.empty(Co * 9 * C, dtype=torch.bfloat16, device=gpu)
    wd = torch.empty_like(wf)
    K.weight_prep(w, wf, wd)
    dy = (torch.randn(N * H * H, Co, device=gpu) * 0.1).to(torch.bfloat16)
    g_f, part = K.conv_dgrad_bn(dy, wd, N, H, H, C, Co, y, a, b, mean, rstd, pool)
    fused = native.kernels().ddpx_conv_dgrad_parts(N, H, H, C, Co, -1) > 0
    assert (part is not None) == fused
    g_u = K.conv_dgrad(dy, wd, N, H, H, C, Co)
    assert torch.equal(g_f, g_u)
    dg_f, db_f, dg_u, db_u = (torch.empty(C, device=gpu) for _ in range(4))
    dz_f = K.bn_backward(g_f, y, a, b, mean, rstd, N, Hy, Hy, C, pool, dgamma=dg_f, dbeta=db_f, part=part)
    dz_u = K.bn_backward(g_u, y, a, b, mean, rstd, N, Hy, Hy, C, pool, dgamma=dg_u, dbeta=db_u)
    assert torch.allclose(db_f, db_u, rtol=1e-4, atol=1e-4 * db_u.abs().max().item())
    assert torch.allclose(dg_f, dg_u, rtol=1e-4, atol=1e-4 * dg_u.abs().max().item())
    assert _rel(dz_f, dz_u) < 1e-3
