"""The reference VGG as one autograd node on ddpx's MI355X kernels (NHWC, bf16 compute).

Per conv block (``/root/reference/singlegpu.py:60-70``):

    forward : y   = conv3x3(x, W)                implicit-GEMM MFMA, epilogue emits BN tile statistics
              a,b = bn_finalize(stats)           Chan merge, running-stat update (momentum 0.1, unbiased var)
              x'  = [maxpool2](relu(a*y + b))    one fused elementwise pass
    backward: dy  = bn_backward(g, y)            pool routing + ReLU mask recomputed from y; dγ, dβ
              dW  = wgrad(dy, x)                 split-K MFMA, fixed-order reduce, torch weight layout
              g   = dgrad(dy, W)                 (skipped for the first block)

then ``x.mean([2,3])`` (global average pool) and the classifier + cross-entropy on the fused head.
``model.sync_bn_comm`` (native SyncBatchNorm, ``--sync_bn``; reference: the commented-out
``convert_sync_batchnorm`` at ``/root/reference/multigpu.py:127``) merges the BatchNorm statistics across
ranks: an all-gather of each rank's [2][C] (mean, M2) in the forward, an all-reduce of (Σdy, Σdy·x̂) in the
backward, both on the compute stream between the same native kernels.
Weight gradients land straight in the DDP bucket storage (grad-ready order: classifier, bn7, conv7,
..., as torch DDP's rebuilt buckets) or — single process with ``SGD(fused_backward=True)`` — are
applied in the reduce kernels without ever being stored.  The forward reads bf16 copies of the conv
weights permuted for the GEMMs (``Wf``: [Co][3][3][Ci], ``Wd``: [3][3][Co][Ci]) that are refreshed from
the fp32 masters once per forward; dgrad reads them, so the fused update of W never races dgrad.
"""
from __future__ import annotations

import os

import torch
from torch import nn

from . import conv as K
from ..optim.sgd import take_lr_advance
from .head import head_backward, head_forward


# DDPX_CONV_PREP_FROM_UPDATE=0: re-derive the bf16 conv layouts every forward (weight_prep) even when the fused
# update already wrote them (A/B checks)
_PREP_FROM_UPDATE = os.environ.get("DDPX_CONV_PREP_FROM_UPDATE", "1") != "0"
# DDPX_BN_BWD_FUSE=0: the BatchNorm backward sums by their own reduce pass over g and y, instead of in the epilogue
# of the conv data gradient that produces g (csrc/include/ddpx_pipe.h EPI_BNBWD_BF16)
_BN_BWD_FUSE = os.environ.get("DDPX_BN_BWD_FUSE", "1") != "0"


class _Plan:
    """Static description of the network + persistent prepared-weight buffers."""

    def __init__(self, model):
        self.blocks = []  # (conv, bn, pool)
        mods = list(model.backbone.children())
        i = 0
        while i < len(mods):
            conv, bn = mods[i], mods[i + 1]
            assert isinstance(conv, nn.Conv2d) and isinstance(bn, nn.BatchNorm2d)
            i += 3  # conv, bn, relu
            pool = i < len(mods) and isinstance(mods[i], nn.MaxPool2d)
            if pool:
                i += 1
            self.blocks.append((conv, bn, pool))
        dev = model.classifier.weight.device
        self.wf, self.wd = [], []
        # FlatParams version of each conv weight the prepared layouts were made from (None: never): the fused
        # single-process update rewrites them in its reduce kernel, any other update makes them stale
        self.wver = [None] * 0
        for conv, _, _ in self.blocks:
            Co, Ci = conv.weight.shape[:2]
            n = Co * 9 * K.padded_channels(Ci)
            self.wf.append(torch.empty(n, dtype=torch.bfloat16, device=dev))
            self.wd.append(torch.empty(n, dtype=torch.bfloat16, device=dev))
        self.wver = [None] * len(self.blocks)


def _sync_comm(model, training):
    """The communicator of native SyncBatchNorm (``--sync_bn`` under DDP), or None: batch statistics are
    then merged across ranks inside the forward and the backward (``ops/conv.py`` bn_*_sync)."""
    comm = getattr(model, "sync_bn_comm", None)
    if training and comm is not None and comm.world_size > 1:
        return comm
    return None


def plan_of(model):
    p = getattr(model, "_ddpx_plan", None)
    if p is None:
        p = _Plan(model)
        model._ddpx_plan = p
    return p


def _forward(model, x, targets, want_logits, want_grad, training):
    plan = plan_of(model)
    flat = model.classifier.weight._ddpx_flat
    N, H, W, C = x.shape
    saved = []
    for bi, (conv, bn, pool) in enumerate(plan.blocks):
        Co = conv.weight.shape[0]
        ver = flat.version_of(conv.weight)
        if plan.wver[bi] != ver:
            K.weight_prep(conv.weight, plan.wf[bi], plan.wd[bi])
            plan.wver[bi] = ver
        y, st, T, BM = K.conv_fwd(x, plan.wf[bi], Co, stats=training)
        dev = x.device
        a = torch.empty(Co, dtype=torch.float32, device=dev)
        b = torch.empty_like(a)
        mean = torch.empty_like(a)
        rstd = torch.empty_like(a)
        comm = _sync_comm(model, training)
        if comm is not None:
            K.bn_finalize_sync(st, T, BM, N * H * W, bn, a, b, mean, rstd, comm)
        else:
            K.bn_finalize(st, T, BM, N * H * W, bn, training, a, b, mean, rstd)
        xn = K.bn_apply(y, a, b, N, H, W, Co, relu=True, pool=pool)
        saved.append((x, y, a, b, mean, rstd, (N, H, W, C, Co), pool))
        x = xn
        H, W, C = xn.shape[1], xn.shape[2], Co
    feat = K.avgpool(x)  # [N, 512] bf16
    cls = model.classifier
    loss, logits, dl = head_forward(feat, flat.shadow_of(cls.weight), cls.bias, targets, want_logits=want_logits,
                                    want_grad=want_grad, lr_advance=take_lr_advance(flat) if want_grad else None)
    return saved, (x.shape, feat), loss, logits, dl


def _backward(model, saved, last, dl, grad_out):
    plan = plan_of(model)
    flat = model.classifier.weight._ddpx_flat
    cls = model.classifier
    xshape, feat = last
    dfeat = torch.empty_like(feat)
    sw, sb = flat.fused_spec(cls.weight), flat.fused_spec(cls.bias)
    if sw is not None:
        head_backward(dl, grad_out, feat, flat.shadow_of(cls.weight), None, None, dH=dfeat, relu_mask=False,
                      sgd_w=sw, sgd_b=sb)
        flat.mark_updated(cls.weight)
        flat.mark_updated(cls.bias)
    else:
        dW, acc = flat.grad_target(cls.weight)
        db, _ = flat.grad_target(cls.bias)
        head_backward(dl, grad_out, feat, flat.shadow_of(cls.weight), dW, db, dH=dfeat, relu_mask=False,
                      accumulate=acc)
        flat.grad_done(cls.weight)
        flat.grad_done(cls.bias)
    g = K.avgpool_backward(dfeat, *xshape)
    comm = _sync_comm(model, True)
    gpart = None  # BatchNorm pass-1 sums of g, when the data gradient that made g produced them

    def dgrad(dy, wd, bi, N, H, W, C, Co):
        """g of the block below, with its BatchNorm backward sums from the GEMM epilogue when possible."""
        if _BN_BWD_FUSE:
            _, yp, ap, bp, mp, rp, _, poolp = saved[bi - 1]
            return K.conv_dgrad_bn(dy, wd, N, H, W, C, Co, yp, ap, bp, mp, rp, poolp)
        return K.conv_dgrad(dy, wd, N, H, W, C, Co), None

    for bi in range(len(plan.blocks) - 1, -1, -1):
        conv, bn, pool = plan.blocks[bi]
        x, y, a, b, mean, rstd, (N, H, W, C, Co), _ = saved[bi]
        sg, sbeta = flat.fused_spec(bn.weight), flat.fused_spec(bn.bias)
        if comm is not None:
            if sg is not None:
                raise RuntimeError("SyncBatchNorm runs under DDP; the fused single-process optimizer does not apply")
            dgam, accg = flat.grad_target(bn.weight)
            dbet, _ = flat.grad_target(bn.bias)
            dy = K.bn_backward_sync(g, y, a, b, mean, rstd, N, H, W, Co, pool, comm, dgamma=dgam, dbeta=dbet,
                                    accumulate=accg, part=gpart)
            flat.grad_done(bn.weight)
            flat.grad_done(bn.bias)
        elif sg is not None:
            dy = K.bn_backward(g, y, a, b, mean, rstd, N, H, W, Co, pool, sgd_gamma=sg, sgd_beta=sbeta, part=gpart)
            flat.mark_updated(bn.weight)
            flat.mark_updated(bn.bias)
        else:
            dgam, accg = flat.grad_target(bn.weight)
            dbet, _ = flat.grad_target(bn.bias)
            dy = K.bn_backward(g, y, a, b, mean, rstd, N, H, W, Co, pool, dgamma=dgam, dbeta=dbet, accumulate=accg,
                               part=gpart)
            flat.grad_done(bn.weight)
            flat.grad_done(bn.bias)
        Cr = conv.weight.shape[1]
        sw = flat.fused_spec(conv.weight)
        if sw is not None:
            # prepared layouts current before this update (the forward made or kept them): the reduce rewrites
            # them with the updated weight, after this block's dgrad below has read wd (stream order)
            prep = _PREP_FROM_UPDATE and plan.wver[bi] == flat.version_of(conv.weight)
            if prep and bi > 0:
                g, gpart = dgrad(dy, plan.wd[bi], bi, N, H, W, C, Co)
            K.conv_wgrad(dy, x, Co, Cr, sgd=sw, prepared=(plan.wf[bi], plan.wd[bi]) if prep else None)
            flat.mark_updated(conv.weight)
            if prep:
                plan.wver[bi] = flat.version_of(conv.weight)
                continue
        else:
            dw, accw = flat.grad_target(conv.weight)
            K.conv_wgrad(dy, x, Co, Cr, out=dw, accumulate=accw)
            flat.grad_done(conv.weight)
        if bi > 0:
            g, gpart = dgrad(dy, plan.wd[bi], bi, N, H, W, C, Co)


class _VGGLoss(torch.autograd.Function):
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


class _VGGLogits(torch.autograd.Function):
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


def _prep_input(x):
    if x.dim() == 4 and x.shape[-1] == 8 and x.dtype == torch.bfloat16:
        return x.contiguous()
    if x.dim() == 4 and x.shape[1] == 3:  # NCHW fp32 from a reference-style loader
        x = x.permute(0, 2, 3, 1)
        x = torch.nn.functional.pad(x, (0, 8 - x.shape[-1]))
        return x.to(torch.bfloat16).contiguous()
    raise ValueError(f"unsupported VGG input {tuple(x.shape)} {x.dtype}")


def vgg_loss(model, x, targets):
    return _VGGLoss.apply(_prep_input(x), targets, model, *model.parameters())


def vgg_forward(model, x):
    x = _prep_input(x)
    if not torch.is_grad_enabled():
        _, _, _, logits, _ = _forward(model, x, None, True, False, model.training)
        return logits
    return _VGGLogits.apply(x, model, *model.parameters())
