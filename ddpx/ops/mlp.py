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

``model.fp8`` (the wide-MLP config, BASELINE.json configs[4]): the hidden layers' forward (and, with
``DDPX_FP8_WGRAD=1``, weight-gradient) GEMMs run on MX-FP8 (``ddpx.ops.fp8``: e4m3 activations, weights and output
gradients, E8M0 block-32 scales applied inside ``v_mfma_scale_f32_16x16x128_f8f6f4``); the
forward quantises each input both row-wise (its GEMM) and transposed (the later wgrad's B operand).
The data-gradient GEMM stays bf16.  Master weights, gradients and SGD are unchanged (fp32).
"""
from __future__ import annotations

import os

import torch

from . import gemm as G
from ..optim.sgd import take_lr_advance
from .head import head_backward, head_forward

# DDPX_WGRAD_PAIR=0: launch the last two layers' fused weight-gradient + SGD kernels one by one
_PAIR_WGRAD = os.environ.get("DDPX_WGRAD_PAIR", "1") != "0"
# DDPX_FP8_WGRAD=1: MX-FP8 weight-gradient GEMMs too (default: MX-FP8 forward GEMMs, bf16 backward)
_FP8_WGRAD = os.environ.get("DDPX_FP8_WGRAD", "0") == "1"
# DDPX_FP8_DGRAD=1 (fp8 models): the hidden layers' data gradients on MX-FP8 too - dY row-quantised, W_l quantised
# transposed (32-blocks along its output dimension, the data gradient's K) every step, the ReLU mask in the MX
# GEMM's epilogue.  Opt-in: at N = 1 the per-step transposed quantisation of W costs about what the 1.8x faster
# GEMM saves (profiles/r5_fp8/NOTES.md)
_FP8_DGRAD = os.environ.get("DDPX_FP8_DGRAD", "0") == "1"


def _dgrad_mx8(dpre, wq, h, bias_grad=None, bias_acc=False, bias_sgd=None):
    """dX = (dpre W) * (h > 0) on MX-FP8, plus the bias gradient of the layer below (stored / accumulated into
    ``bias_grad`` or applied through ``bias_sgd``), as G.linear_dgrad's epilogue does on the bf16 pipe.
    ``wq``: Wᵀ [in][out] as MX-FP8 with blocks along out (FlatParams.mx8t_weight: the copy the previous step's
    wgrad+SGD pair wrote, or the bf16 copy quantised now)."""
    from . import fp8 as F8
    from .elementwise import colsum_bf16, sgd_flat_
    dq = F8.quant(dpre, F8.E4M3)                            # dpre [batch][out], blocks along out
    dx = F8.gemm(dq, wq, epi=G.EPI_RELUMASK_BF16, aux=h)
    if bias_sgd is not None:
        p, buf, sh, lr, mom, wd = bias_sgd
        g = torch.empty(p.numel(), dtype=torch.float32, device=dx.device)
        colsum_bf16(dx, g)
        sgd_flat_(p, buf if buf is not None else torch.zeros_like(p), g, sh, lr, mom, wd)
    elif bias_grad is not None:
        if bias_grad.dtype == torch.float32:
            colsum_bf16(dx, bias_grad, accumulate=bias_acc)
        else:
            g = torch.empty(bias_grad.numel(), dtype=torch.float32, device=dx.device)
            colsum_bf16(dx, g)
            bias_grad.copy_(g + bias_grad.float() if bias_acc else g)
    return dx
# DDPX_DGRAD_FUSE=1: fc1's data gradient inside the pair's launch (csrc/include/ddpx_wsgd_dgrad.h, fc1's bf16
# weight copy ping-ponged between two buffers).  Opt-in: measured slower than the two launches on MI355X
# (toy step 0.2905 vs 0.2379-0.2391 ms, one box, profiles/r4_dgfuse): the pair's math waves are bound by their
# L2 -> LDS operand DMA, not idle behind the optimizer stream, so the data gradient's operand stream adds its
# full cost, and the LDS left for two rings allows only 2 stages each.
_DGRAD_FUSE = os.environ.get("DDPX_DGRAD_FUSE", "0") == "1"


def _to_bf16_2d(x):
    if x.dtype != torch.bfloat16:
        x = x.to(torch.bfloat16)
    if not x.is_contiguous():
        x = x.contiguous()
    return x


def _params(model):
    lins = model.linears()
    return [(lin.weight, lin.bias) for lin in lins]


def _fp8_ok(model, x):
    if not getattr(model, "fp8", False):
        return False
    B = x.shape[0]
    return B % 128 == 0 and all(w.shape[1] % 128 == 0 for w, _ in _params(model)[:-1])


def _forward(model, x, targets, want_logits, want_grad, for_backward=None):
    flat = model.fc0.weight._ddpx_flat
    ps = _params(model)
    hs = [x]
    fp8 = _fp8_ok(model, x)
    if for_backward is None:
        for_backward = want_grad
    # the backward's weight-gradient GEMMs stay bf16 unless DDPX_FP8_WGRAD=1: single-process, the fused
    # bf16 weight-gradient + SGD pair hides those GEMMs under the optimizer's HBM stream, which the fp8
    # GEMM's per-tile SGD epilogue cannot (profiles/r2_fp8)
    saved8 = [] if (fp8 and for_backward and _FP8_WGRAD) else None
    for (w, b) in ps[:-1]:
        rc = None if fp8 else flat.chunks_of(w)
        if rc is not None:
            # row-chunked weight (DDP chunk buckets, deferred ZeRO gathers): each chunk's output columns
            # are computed as soon as that chunk's all-gather has landed
            h = torch.empty((hs[-1].shape[0], w.shape[0]), dtype=torch.bfloat16, device=hs[-1].device)
            sw = flat.shadow_of(w)
            for c, (r0, r1) in enumerate(rc):
                flat.before_read(w, c)
                G.linear_fwd(hs[-1], sw[r0:r1], b[r0:r1], relu=True, out=h[:, r0:r1])
            hs.append(h)
            continue
        flat.before_read(w)
        if fp8:
            from . import fp8 as F8
            if saved8 is not None:
                hq, hqt = F8.quant(hs[-1], F8.E4M3, rows=True, cols=True)
                saved8.append(hqt)
            else:
                hq = F8.quant(hs[-1], F8.E4M3)
            if flat.shadow8 is None:
                flat.enable_fp8_shadow()
            # the e4m3 weight copy in the store: the fused wgrad+SGD pair writes it (default), anything else that
            # updated the weight leaves it stale and it is re-quantised from the bf16 copy here
            wq = flat.mx8_weight(w)
            hs.append(F8.gemm(hq, wq, epi=G.EPI_BIAS_RELU_BF16, bias=b))
        else:
            hs.append(G.linear_fwd(hs[-1], flat.shadow_of(w), b, relu=True))
    wl, bl = ps[-1]
    flat.before_read(wl)
    loss, logits, dl = head_forward(hs[-1], flat.shadow_of(wl), bl, targets, want_logits=want_logits,
                                    want_grad=want_grad, lr_advance=take_lr_advance(flat) if want_grad else None)
    return hs, loss, logits, dl, saved8


def _wgrad(saved, l, dpre, h, out, accumulate=False, sgd=None):
    """dW_l = dpreᵀ h — MX-FP8 when the forward saved hᵀ in fp8, else the bf16 pipe."""
    if saved:
        from . import fp8 as F8
        # output gradients in e4m3 too: with per-32-element E8M0 block scales the range is covered
        # by the scale, and e4m3's extra mantissa bit halves the wgrad error vs e5m2
        dq = F8.quant(dpre, F8.E4M3, rows=False, cols=True)  # dpreᵀ [out][batch]
        if sgd is not None:
            return F8.gemm(dq, saved[l], epi=G.EPI_SGD, sgd=sgd)
        epi = G.EPI_F32 if out.dtype == torch.float32 else G.EPI_BF16
        return F8.gemm(dq, saved[l], out=out, epi=epi, accumulate=accumulate)
    if sgd is not None:
        return G.linear_wgrad(dpre, h, None, sgd=sgd)
    return G.linear_wgrad(dpre, h, out, accumulate=accumulate)


def _backward(model, hs, dl, grad_out, saved8=None):
    flat = model.fc0.weight._ddpx_flat
    ps = _params(model)
    L = len(ps) - 1  # number of hidden layers
    wl, bl = ps[-1]
    bprev = ps[L - 1][1]
    fused = flat.fused_spec(wl) is not None
    fp8_dgrad = _FP8_DGRAD and bool(getattr(model, "fp8", False)) and hs[L].is_cuda
    if fp8_dgrad and flat.shadow8t is None and not torch.cuda.is_current_stream_capturing():
        flat.enable_fp8_transposed()
    dpre = torch.empty_like(hs[L])
    if fused:
        # optimizer fused into backward: each kernel that produces a gradient applies the SGD
        # update in its epilogue.  W_L is read (for dH) before the finalize kernel updates it.
        head_backward(dl, grad_out, hs[L], flat.shadow_of(wl), None, None, dH=dpre, relu_mask=True,
                      sgd_w=flat.fused_spec(wl), sgd_b=flat.fused_spec(bl), sgd_prev=flat.fused_spec(bprev))
        for p in (wl, bl, bprev):
            flat.mark_updated(p)
        if L == 2 and not saved8 and not fp8_dgrad and _PAIR_WGRAD and _DGRAD_FUSE and \
                _fused_dgrad(model, flat, ps, hs, dpre):
            return
        deferred = None  # layer 1's update, launched together with layer 0's (one warp-specialised launch)
        for l in range(L - 1, -1, -1):
            w, _ = ps[l]
            dnext = None
            if l > 0:  # data gradient first: it must read W_l before the fused update rewrites it
                bp = ps[l - 1][1]
                flat.normalize_pingpong()  # (the unfused update writes the main bf16 copy)
                if fp8_dgrad:
                    dnext = _dgrad_mx8(dpre, flat.mx8t_weight(w), hs[l], bias_sgd=flat.fused_spec(bp))
                else:
                    dnext = G.linear_dgrad(dpre, flat.shadow_of(w), relu_mask_of=hs[l], bias_sgd=flat.fused_spec(bp))
                flat.mark_updated(bp)
            if l == 1 and not saved8 and _PAIR_WGRAD:
                deferred = (dpre, hs[1], flat.fused_spec(w), w)
            elif l == 0 and deferred is not None:
                d1, h1, s1, w1 = deferred
                s0 = flat.fused_spec(w)
                # fp8 model (DDPX_FP8_COPY=pair|1, default pair): the stream waves also emit both weights' MX-FP8 copies
                emit = flat.shadow8 is not None and flat.fp8_from_optimizer
                mx1, mx0 = (flat.mx8_views(w1), flat.mx8_views(w)) if emit else (None, None)
                if mx1 is None or mx0 is None:  # both copies or neither (a store without 128-aligned offsets)
                    mx1 = mx0 = None
                # fp8 data gradients: W1's transposed copy for the next step's fc1 dgrad (fc0 has none)
                mxt1 = flat.mx8t_views(w1) if (fp8_dgrad and mx1 is not None) else None
                paired = G.wgrad_sgd_pair(d1, h1, s1, dpre, hs[0], s0, mx1, mx0, mxt1, None)
                if not paired:
                    G.linear_wgrad(d1, h1, None, sgd=s1)
                    _wgrad(saved8, 0, dpre, hs[0], None, sgd=s0)
                flat.mark_updated(w1, fp8_written=paired and mx1 is not None,
                                  fp8t_written=paired and mxt1 is not None)
                flat.mark_updated(w, fp8_written=paired and mx0 is not None)
                dpre = dnext
                continue
            else:
                _wgrad(saved8, l, dpre, hs[l], None, sgd=flat.fused_spec(w))
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
        rc = None if saved8 else flat.chunks_of(w)
        if rc is None:
            _wgrad(saved8, l, dpre, hs[l], dWl, accumulate=accw)
            flat.grad_done(w)
        else:
            # one weight-gradient GEMM per row chunk, each announced at once: that chunk's bucket
            # collective (reduce-scatter / all-reduce) overlaps the remaining chunks and the dgrad
            for c, (r0, r1) in enumerate(rc):
                G.linear_wgrad(dpre[:, r0:r1], hs[l], dWl[r0:r1], accumulate=accw)
                flat.grad_done(w, chunk=c)
        if l > 0:
            bp = ps[l - 1][1]
            dbl, accl = flat.grad_target(bp)
            # ReLU backward + bias gradient of layer l-1 fused into the dgrad epilogue
            if fp8_dgrad:
                dnext = _dgrad_mx8(dpre, flat.mx8t_weight(w), hs[l], bias_grad=dbl, bias_acc=accl)
            else:
                dnext = G.linear_dgrad(dpre, flat.shadow_of(w), relu_mask_of=hs[l], bias_grad=dbl,
                                       bias_grad_accumulate=accl)
            flat.release(w)  # W_l's last read: a side-stream update of its bucket may start now
            flat.grad_done(bp)
            dpre = dnext


def _fused_dgrad(model, flat, ps, hs, dpre) -> bool:
    """Two hidden layers, optimizer fused into backward: fc1's data gradient, fc1's and fc0's weight gradients
    and all three SGD updates (W1, W0, b0) in ONE launch (G.wgrad_sgd_dgrad).  fc1's new bf16 copy goes to the
    other buffer of its ping-pong pair (the launch's data gradient reads the current one).  False (nothing
    launched) when the shapes are not eligible."""
    (w0, b0), (w1, _) = ps[0], ps[1]
    K, M1 = dpre.shape
    N1, N0 = hs[1].shape[1], hs[0].shape[1]
    if getattr(model, "_dg_fuse_ok", None) is False or not G.wgrad_sgd_dgrad_eligible(K, M1, N1, N0, dpre.device):
        model._dg_fuse_ok = False
        return False
    if not flat.has_pingpong(w1):
        if torch.cuda.is_current_stream_capturing():
            return False  # first use must allocate the second buffer outside a capture
        flat.enable_pingpong(w1)
    s1, s0, sb = flat.fused_spec(w1), flat.fused_spec(w0), flat.fused_spec(b0)
    if s1 is None or s0 is None or sb is None:
        return False
    s1 = (s1[0], s1[1], flat.shadow_next(w1), s1[3], s1[4], s1[5])
    emit = flat.shadow8 is not None and flat.fp8_from_optimizer
    mx1, mx0 = (flat.mx8_views(w1), flat.mx8_views(w0)) if emit else (None, None)
    if mx1 is None or mx0 is None:
        mx1 = mx0 = None
    dx = G.wgrad_sgd_dgrad(dpre, hs[1], s1, flat.shadow_of(w1), hs[1], hs[0], s0, sb, mx1=mx1, mx0=mx0)
    if dx is None:
        model._dg_fuse_ok = False
        return False
    model._dg_fuse_ok = True
    flat.flip_pingpong(w1)
    flat.mark_updated(w1, fp8_written=mx1 is not None)
    flat.mark_updated(w0, fp8_written=mx0 is not None)
    flat.mark_updated(b0)
    return True


class _MLPLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, targets, model, *weights):
        hs, loss, _, dl, saved8 = _forward(model, x, targets, want_logits=False, want_grad=True)
        ctx.model = model
        ctx.hs = hs
        ctx.dl = dl
        ctx.saved8 = saved8
        ctx.n_in = len(weights)
        return loss

    @staticmethod
    def backward(ctx, grad_loss):
        _backward(ctx.model, ctx.hs, ctx.dl, grad_loss, ctx.saved8)
        ctx.hs = ctx.dl = ctx.saved8 = None
        return (None, None, None) + (None,) * ctx.n_in


class _MLPLogits(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, *weights):
        hs, _, logits, _, saved8 = _forward(model, x, None, want_logits=True, want_grad=False, for_backward=True)
        ctx.model = model
        ctx.hs = hs
        ctx.saved8 = saved8
        ctx.n_in = len(weights)
        return logits

    @staticmethod
    def backward(ctx, grad_logits):
        _backward(ctx.model, ctx.hs, grad_logits.float().contiguous(), None, ctx.saved8)
        ctx.hs = ctx.saved8 = None
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
        _, _, logits, _, _ = _forward(model, x, None, want_logits=True, want_grad=False)
        return logits
    return _MLPLogits.apply(x, model, *_weights(model))
