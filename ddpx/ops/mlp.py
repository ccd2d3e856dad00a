"""The MLP as a single autograd node with an explicit MI355X schedule.

Forward  (per hidden layer)  h_{l+1} = relu(h_l W_lᵀ + b_l)   → bf16 MFMA GEMM, bias+ReLU epilogue
         (head)              loss    = CE(h_L W_Lᵀ + b_L, t)   → fused head kernel (logits, NLL, dlogits)
Backward (grad-ready order, each weight gradient written fp32 straight into
its DDP bucket slice, then announced to the reducer):
   head_bwd : dW_L, db_L, dpre_{L-1} = (dlogits W_L) ⊙ (h_L > 0), db_{L-1}
   for l = L-1 .. 0:
      wgrad  : dW_l = dpre_lᵀ h_l                          (announce W_l → bucket may fire)
      dgrad  : dpre_{l-1} = (dpre_l W_l) ⊙ (h_l > 0)        (skipped for l = 0)
      (db_{l-1} = Σ_m dpre_{l-1} from the dgrad epilogue's per-tile column sums)
The weight gradient of a layer is issued BEFORE its data gradient so the
bucket holding it starts its all-reduce while the next GEMMs run.
"""
from __future__ import annotations

import torch

from . import gemm as G
from .head import head_backward, head_forward


def _to_bf16_2d(x):
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if not x.is_contiguous():
        x = x.contiguous()
    return x


def _params(model):
    lins = model.linears()
    return [(lin.weight, lin.bias) for lin in lins]


def _forward(model, x, targets, want_logits, want_grad):
    flat = model.fc0.weight._ddpx_flat
    ps = _params(model)
    hs = [x]
    for (w, b) in ps[:-1]:
        hs.append(G.linear_fwd(hs[-1], flat.shadow_of(w), b, relu=True))
    wl, bl = ps[-1]
    loss, logits, dl = head_forward(hs[-1], flat.shadow_of(wl), bl, targets, want_logits=want_logits,
                                    want_grad=want_grad)
    return hs, loss, logits, dl


def _backward(model, hs, dl, grad_out):
    flat = model.fc0.weight._ddpx_flat
    ps = _params(model)
    L = len(ps) - 1  # number of hidden layers
    wl, bl = ps[-1]
    bprev = ps[L - 1][1]
    fused = flat.fused_spec(wl) is not None
    dpre = torch.empty_like(hs[L])
    if fused:
        # optimizer fused into backward: each kernel that produces a gradient applies the SGD
        # update in its epilogue.  W_L is read (for dH) before the finalize kernel updates it.
        head_backward(dl, grad_out, hs[L], flat.shadow_of(wl), None, None, dH=dpre, relu_mask=True,
                      sgd_w=flat.fused_spec(wl), sgd_b=flat.fused_spec(bl), sgd_prev=flat.fused_spec(bprev))
        for p in (wl, bl, bprev):
            flat.mark_updated(p)
        for l in range(L - 1, -1, -1):
            w, _ = ps[l]
            dnext = None
            if l > 0:  # data gradient first: it must read W_l before the fused update rewrites it
                bp = ps[l - 1][1]
                dnext = G.linear_dgrad(dpre, flat.shadow_of(w), relu_mask_of=hs[l], bias_sgd=flat.fused_spec(bp))
                flat.mark_updated(bp)
            G.linear_wgrad(dpre, hs[l], None, sgd=flat.fused_spec(w))
            flat.mark_updated(w)
            dpre = dnext
        return
    dW, acc = flat.grad_target(wl)
    db, accb = flat.grad_target(bl)
    dbp, accp = flat.grad_target(bprev)
    if not (acc == accb == accp):
        raise NotImplementedError("mixed gradient-accumulation state inside the MLP head")
    head_backward(dl, grad_out, hs[L], flat.shadow_of(wl), dW, db, dH=dpre, dbprev=dbp, relu_mask=True,
                  accumulate=acc)
    flat.grad_done(wl)
    flat.grad_done(bl)
    flat.grad_done(bprev)
    for l in range(L - 1, -1, -1):
        w, _ = ps[l]
        dWl, accw = flat.grad_target(w)
        G.linear_wgrad(dpre, hs[l], dWl, accumulate=accw)
        flat.grad_done(w)
        if l > 0:
            bp = ps[l - 1][1]
            dbl, accl = flat.grad_target(bp)
            # ReLU backward + bias gradient of layer l-1 fused into the dgrad epilogue
            dnext = G.linear_dgrad(dpre, flat.shadow_of(w), relu_mask_of=hs[l], bias_grad=dbl,
                                   bias_grad_accumulate=accl)
            flat.grad_done(bp)
            dpre = dnext


class _MLPLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, targets, model, *weights):
        hs, loss, _, dl = _forward(model, x, targets, want_logits=False, want_grad=True)
        ctx.model = model
        ctx.hs = hs
        ctx.dl = dl
        ctx.n_in = len(weights)
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        _backward(ctx.model, ctx.hs, ctx.dl, grad_loss)
        ctx.hs = ctx.dl = None
        return (None, None, None) + (None,) * ctx.n_in


class _MLPLogits(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, *weights):
        hs, _, logits, _ = _forward(model, x, None, want_logits=True, want_grad=False)
        ctx.model = model
        ctx.hs = hs
        ctx.n_in = len(weights)
        return logits

    @staticmethod
    def backward(ctx, grad_logits):
        _backward(ctx.model, ctx.hs, grad_logits.float().contiguous(), None)
        ctx.hs = None
        return (None, None) + (None,) * ctx.n_in


def _weights(model):
    out = []
    for w, b in _params(model):
        out += [w, b]
    return out


def mlp_loss(model, x, targets):
    return _MLPLoss.apply(_to_bf16_2d(x), targets, model, *_weights(model))


def mlp_logits(model, x):
    x = _to_bf16_2d(x)
    if not torch.is_grad_enabled():
        _, _, logits, _ = _forward(model, x, None, want_logits=True, want_grad=False)
        return logits
    return _MLPLogits.apply(x, model, *_weights(model))
