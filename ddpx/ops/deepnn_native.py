"""The reference's DeepNN as one autograd node on ddpx's MI355X kernels (NHWC, bf16 compute).

``/root/reference/singlegpu.py:18-44`` (defined there, never instantiated):

    features   : [conv3x3+bias → ReLU] x2 → MaxPool2 → [conv3x3+bias → ReLU] x2 → MaxPool2
    classifier : flatten(C,H,W) → Linear(2048→512) → ReLU → Dropout(0.1) → Linear(512→10)

Schedule:

    forward : act = relu(conv3x3(x, W) + bias)    implicit-GEMM MFMA, bias + ReLU in its epilogue
              x'  = maxpool2(act) (pooled blocks) one pass; un-pooled blocks feed act on as is
              f  = flatten in torch's (C,H,W) order (NHWC → NCHW view of 2048 features)
              a0 = relu(f W0ᵀ + b0)               MFMA GEMM, bias+ReLU epilogue
              d0 = dropout(a0)                    Philox kernel, device-resident (seed, offset)
              loss, dlogits = head(d0, W1, b1)    fused Linear(512→10) + softmax cross-entropy
    backward: dd0, dW1, db1, db0 = head_bwd(...)  dropout+ReLU backward folded in: mask = d0 > 0,
                                                  scale 1/(1-p); db0 = Σ dd0 from the same kernel
              dW0 = dd0ᵀ f,  df = dd0 W0          MFMA GEMMs
              per conv block (reverse):
                pooled: dz, dbias = bias_act_bwd(g, act)   (pool routing + ReLU mask from act)
                un-pooled: dz = dgrad(dz', W') * (act > 0) and its bias-gradient column sums, both in the
                           epilogue of the block above's data-gradient GEMM (EPI_RELUMASK_BF16), finished
                           in fixed order (or applied as the bias's fused SGD)
                dW = wgrad(dz, x) (split-K MFMA); the fused update rewrites the bf16 GEMM layouts of W, so
                the next forward runs no weight_prep pass

Gradients land in the flat store (DDP buckets) in grad-ready order, or — single process with
``SGD(fused_backward=True)`` — weights are updated inside the kernels that produce their
gradients (conv weights and the un-pooled blocks' biases, Linear weights, classifier); the pooled blocks'
conv biases are stepped by the optimizer.
"""
from __future__ import annotations

import torch
from torch import nn

from . import conv as K
from . import gemm as G
from ..optim.sgd import take_lr_advance
from .head import head_backward, head_forward
from .vgg_native import _prep_input
from ..runtime import native


class _Plan:
    def __init__(self, model):
        mods = list(model.features.children())
        self.blocks = []  # (conv, pool)
        i = 0
        while i < len(mods):
            conv = mods[i]
            assert isinstance(conv, nn.Conv2d) and conv.bias is not None and isinstance(mods[i + 1], nn.ReLU)
            i += 2
            pool = i < len(mods) and isinstance(mods[i], nn.MaxPool2d)
            if pool:
                i += 1
            self.blocks.append((conv, pool))
        cls = list(model.classifier.children())
        self.lin0, self.drop, self.lin1 = cls[0], cls[2], cls[3]
        assert isinstance(self.lin0, nn.Linear) and isinstance(self.drop, nn.Dropout) and isinstance(self.lin1,
                                                                                                  nn.Linear)
        dev = self.lin0.weight.device
        self.wf, self.wd = [], []
        for conv, _ in self.blocks:
            Co, Ci = conv.weight.shape[:2]
            n = Co * 9 * K.padded_channels(Ci)
            self.wf.append(torch.empty(n, dtype=torch.bfloat16, device=dev))
            self.wd.append(torch.empty(n, dtype=torch.bfloat16, device=dev))
        # FlatParams version each block's prepared layouts were made from (vgg_native's scheme): the fused update
        # rewrites them, any other update makes them stale
        self.wver = [None] * len(self.blocks)
        cmax = max(c.weight.shape[0] for c, _ in self.blocks)
        self.ones = torch.ones(cmax, dtype=torch.float32, device=dev)
        self.zeros = torch.zeros(cmax, dtype=torch.float32, device=dev)
        # dropout generator state on the device: [seed, offset] (+ workgroup completion counter)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item())
        self.rng = torch.tensor([seed, 0], dtype=torch.int64, device=dev)
        self.rng_done = torch.zeros(1, dtype=torch.int32, device=dev)


def plan_of(model):
    p = getattr(model, "_ddpx_plan", None)
    if p is None:
        p = _Plan(model)
        model._ddpx_plan = p
    return p


def dropout_(x, p, plan, out=None):
    """Inverted dropout of a bf16 tensor with the plan's device-resident Philox state."""
    _req = K._req
    _req(x.is_cuda and x.dtype == torch.bfloat16 and x.is_contiguous() and x.numel() % 8 == 0,
         "dropout: x must be contiguous bf16 with numel % 8 == 0")
    out = torch.empty_like(x) if out is None else out
    native.check(native.kernels().ddpx_dropout_fwd(x.data_ptr(), out.data_ptr(), x.numel(), float(p),
                                                   plan.rng.data_ptr(), plan.rng_done.data_ptr(),
                                                   native.stream_handle()), "ddpx_dropout_fwd")
    return out


# (gout, y, bias, ones, zeros, N, H, W, C, pool, relu, part, c1, c2, dbias, out_bf16, accumulate, dy,
#  sgd p, buf, shadow, lr, mom, wd, stream)
native.register_kernel_sig("ddpx_bias_act_bwd_sgd", native.c_int, *([native.c_void_p] * 5 + [native.c_int] * 6
                                                                     + [native.c_void_p] * 4 + [native.c_int] * 2
                                                                     + [native.c_void_p] * 5 + [native.c_float] * 2
                                                                     + [native.c_void_p]))


def bias_act_backward(gout, act, N, H, W, C, pool, plan, dbias=None, accumulate=False, sgd=None):
    """dz [N*H*W, C] bf16 and dbias (=|+=) Σ dz — or, with ``sgd``, that sum applied as the bias's fused SGD
    update — for out = [pool](act), act = relu(conv + bias): the pool routing (first maximum) and the ReLU mask
    recomputed from act (bn_pool.hip's backward with a = 1, b = 0)."""
    K._nhwc(gout, "gout", C)
    K._nhwc(act, "act", C)
    lib = native.kernels()
    B = lib.ddpx_bn_bwd_blocks(N, H, W, C)
    dev = act.device
    part = torch.empty((B, 2, C), dtype=torch.float32, device=dev)
    c1 = torch.empty(C, dtype=torch.float32, device=dev)
    c2 = torch.empty(C, dtype=torch.float32, device=dev)
    dy = torch.empty((N * H * W, C), dtype=torch.bfloat16, device=dev)
    native.check(lib.ddpx_bias_act_bwd_sgd(gout.data_ptr(), act.data_ptr(), plan.zeros.data_ptr(),
                                           plan.ones.data_ptr(), plan.zeros.data_ptr(), N, H, W, C, int(pool), 1,
                                           part.data_ptr(), c1.data_ptr(), c2.data_ptr(), native.ptr(dbias),
                                           int(dbias is not None and dbias.dtype == torch.bfloat16), int(accumulate),
                                           dy.data_ptr(), *native.sgd_args(sgd), native.stream_handle()),
                 "ddpx_bias_act_bwd_sgd")
    return dy


def _nchw_flatten(x, nhwc=None):
    """NHWC [N,H,W,C] -> [N, C*H*W] in torch's (C, H, W) flatten order; with ``nhwc`` = (N, H, W, C) the inverse
    (the gradient of [N, C*H*W] back to NHWC).  One native launch (csrc/kernels/f32_train.hip)."""
    lib = native.kernels()
    if nhwc is None:
        N, H, W, C = x.shape
        out = torch.empty((N, C * H * W), dtype=x.dtype, device=x.device)
        back = 0
    else:
        N, H, W, C = nhwc
        out = torch.empty((N, H, W, C), dtype=x.dtype, device=x.device)
        back = 1
    K._req(x.dtype == torch.bfloat16 and x.is_contiguous(), "flatten: contiguous bf16 expected")
    native.check(lib.ddpx_bf16_nchw_flatten(x.data_ptr(), N, H * W, C, back, out.data_ptr(), native.stream_handle()),
                 "ddpx_bf16_nchw_flatten")
    return out


def _forward(model, x, targets, want_logits, want_grad, training):
    plan = plan_of(model)
    flat = plan.lin0.weight._ddpx_flat
    N, H, W, C = x.shape
    saved = []
    for bi, (conv, pool) in enumerate(plan.blocks):
        Co = conv.weight.shape[0]
        ver = flat.version_of(conv.weight)
        if plan.wver[bi] != ver:
            K.weight_prep(conv.weight, plan.wf[bi], plan.wd[bi])
            plan.wver[bi] = ver
        act = K.conv_fwd_act(x, plan.wf[bi], Co, conv.bias)
        if pool:
            xn = K.bn_apply(act, plan.ones, plan.zeros, N, H, W, Co, relu=False, pool=True)
        else:
            xn = act.view(N, H, W, Co)
        saved.append((x, act, (N, H, W, C, Co), pool))
        x = xn
        H, W, C = xn.shape[1], xn.shape[2], Co
    # torch.flatten(x, 1) of the NCHW tensor: features in (C, H, W) order
    feat = _nchw_flatten(x)
    a0 = G.linear_fwd(feat, flat.shadow_of(plan.lin0.weight), plan.lin0.bias, relu=True)
    p = float(plan.drop.p)
    drop = training and p > 0.0
    d0 = dropout_(a0, p, plan) if drop else a0
    loss, logits, dl = head_forward(d0, flat.shadow_of(plan.lin1.weight), plan.lin1.bias, targets,
                                    want_logits=want_logits, want_grad=want_grad,
                                    lr_advance=take_lr_advance(flat) if want_grad else None)
    scale = 1.0 / (1.0 - p) if drop else 1.0
    return saved, (x.shape, feat, d0, scale), loss, logits, dl


def _backward(model, saved, last, dl, grad_out):
    plan = plan_of(model)
    flat = plan.lin0.weight._ddpx_flat
    xshape, feat, d0, scale = last
    l0, l1 = plan.lin0, plan.lin1
    dd0 = torch.empty_like(d0)
    sw, sb, sp = flat.fused_spec(l1.weight), flat.fused_spec(l1.bias), flat.fused_spec(l0.bias)
    if sw is not None and sb is not None and sp is not None:
        head_backward(dl, grad_out, d0, flat.shadow_of(l1.weight), None, None, dH=dd0, relu_mask=True,
                      sgd_w=sw, sgd_b=sb, sgd_prev=sp, dh_scale=scale)
        for q in (l1.weight, l1.bias, l0.bias):
            flat.mark_updated(q)
    else:
        dW1, acc = flat.grad_target(l1.weight)
        db1, acc1 = flat.grad_target(l1.bias)
        db0, acc0 = flat.grad_target(l0.bias)
        if not (acc == acc1 == acc0):
            raise NotImplementedError("mixed gradient-accumulation state inside the DeepNN classifier")
        head_backward(dl, grad_out, d0, flat.shadow_of(l1.weight), dW1, db1, dH=dd0, dbprev=db0, relu_mask=True,
                      accumulate=acc, dh_scale=scale)
        for q in (l1.weight, l1.bias, l0.bias):
            flat.grad_done(q)
    # data gradient first: it reads W0's shadow before a fused update rewrites it
    dfeat = G.linear_dgrad(dd0, flat.shadow_of(l0.weight))
    s0 = flat.fused_spec(l0.weight)
    if s0 is not None:
        G.linear_wgrad(dd0, feat, None, sgd=s0)
        flat.mark_updated(l0.weight)
    else:
        dW0, acc = flat.grad_target(l0.weight)
        G.linear_wgrad(dd0, feat, dW0, accumulate=acc)
        flat.grad_done(l0.weight)
    N, Hf, Wf, Cf = xshape
    g = _nchw_flatten(dfeat, (N, Hf, Wf, Cf))
    dz_next = None  # (dz, (part, T)) of the current block, made by the data gradient of the block above
    for bi in range(len(plan.blocks) - 1, -1, -1):
        conv, pool = plan.blocks[bi]
        x, act, (N, H, W, C, Co), _ = saved[bi]
        if dz_next is None:
            # pooled block (or the last one): routing + ReLU mask + bias gradient (or its fused SGD) from g and act
            sb = flat.fused_spec(conv.bias)
            if sb is not None:
                dy = bias_act_backward(g, act, N, H, W, Co, pool, plan, sgd=sb)
                flat.mark_updated(conv.bias)
            else:
                dbias, accb = flat.grad_target(conv.bias)
                dy = bias_act_backward(g, act, N, H, W, Co, pool, plan, dbias, accumulate=accb)
                flat.grad_done(conv.bias)
        else:
            dy, (part, T) = dz_next
            sb = flat.fused_spec(conv.bias)
            if sb is not None:
                K.colsum_finish(part, T, Co, sgd=sb)
                flat.mark_updated(conv.bias)
            else:
                dbias, accb = flat.grad_target(conv.bias)
                K.colsum_finish(part, T, Co, out=dbias, accumulate=accb)
                flat.grad_done(conv.bias)
        dz_next = None
        below_pooled = bi > 0 and plan.blocks[bi - 1][1]

        def dgrad():
            """the gradient for the block below: its pre-activation gradient (+ bias sums) straight from the GEMM
            epilogue when no pool sits between, else the gradient of its pooled output"""
            nonlocal g, dz_next
            if below_pooled:
                g = K.conv_dgrad(dy, plan.wd[bi], N, H, W, C, Co)
            else:
                dz_next = K.conv_dgrad_act(dy, plan.wd[bi], N, H, W, C, Co, saved[bi - 1][1])
        Cr = conv.weight.shape[1]
        sc = flat.fused_spec(conv.weight)
        if sc is not None:
            # layouts current before this update (the forward made or kept them): the reduce rewrites them with the
            # updated weight, after this block's data gradient below has read wd (stream order)
            prep = plan.wver[bi] == flat.version_of(conv.weight)
            if bi > 0:
                dgrad()
            K.conv_wgrad(dy, x, Co, Cr, sgd=sc, prepared=(plan.wf[bi], plan.wd[bi]) if prep else None)
            flat.mark_updated(conv.weight)
            if prep:
                plan.wver[bi] = flat.version_of(conv.weight)
            continue
        dw, accw = flat.grad_target(conv.weight)
        K.conv_wgrad(dy, x, Co, Cr, out=dw, accumulate=accw)
        flat.grad_done(conv.weight)
        if bi > 0:
            dgrad()


class _DeepNNLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, targets, model, *params):
        saved, last, loss, _, dl = _forward(model, x, targets, False, True, model.training)
        ctx.model, ctx.saved, ctx.last, ctx.dl, ctx.n = model, saved, last, dl, len(params)
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        _backward(ctx.model, ctx.saved, ctx.last, ctx.dl, grad_loss)
        ctx.saved = ctx.last = ctx.dl = None
        return (None, None, None) + (None,) * ctx.n


class _DeepNNLogits(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, *params):
        saved, last, _, logits, _ = _forward(model, x, None, True, False, model.training)
        ctx.model, ctx.saved, ctx.last, ctx.n = model, saved, last, len(params)
        return logits

    @staticmethod
    def backward(ctx, grad_logits):
        _backward(ctx.model, ctx.saved, ctx.last, grad_logits.float().contiguous(), None)
        ctx.saved = ctx.last = None
        return (None, None) + (None,) * ctx.n


def deepnn_loss(model, x, targets):
    return _DeepNNLoss.apply(_prep_input(x), targets, model, *model.parameters())


def deepnn_forward(model, x):
    x = _prep_input(x)
    if not torch.is_grad_enabled():
        _, _, _, logits, _ = _forward(model, x, None, True, False, model.training)
        return logits
    return _DeepNNLogits.apply(x, model, *model.parameters())
