"""Fused classifier head: Linear(K→10) + softmax cross-entropy (+ argmax count).

Native on GPU (``csrc/kernels/head_xent.hip``); torch reference math on CPU.
Reference: ``/root/reference/singlegpu.py:73,105,200-206``.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F

from ..runtime import native


def _check(h, w, b, targets):
    if h.dim() != 2 or w.dim() != 2 or h.shape[1] != w.shape[1]:
        raise ValueError(f"head: h {tuple(h.shape)} incompatible with w {tuple(w.shape)}")
    if w.shape[0] != 10:
        raise ValueError("head: native head is specialised for 10 classes")
    if h.dtype != torch.bfloat16 or w.dtype != torch.bfloat16:
        raise ValueError("head: h and w must be bf16 on GPU")
    if b is not None and (b.dtype != torch.float32 or b.numel() != w.shape[0]):
        raise ValueError("head: bias must be fp32 [C]")
    if h.stride(1) != 1 or h.stride(0) % 8 or not w.is_contiguous():
        raise ValueError("head: h must be row-contiguous with ld % 8 == 0, w contiguous")
    if targets is not None and (targets.dtype != torch.int64 or targets.numel() != h.shape[0]):
        raise ValueError("head: targets must be int64 [M]")


def head_forward(h, w, b, targets=None, want_logits=True, want_grad=True, correct=None, lr_advance=None):
    """Returns (loss 0-d fp32 | None, logits [M,C] fp32 | None, dlogits [M,C] fp32 | None).

    ``lr_advance`` ((table, counter, lr) device tensors, from ``ddpx.optim.sgd.take_lr_advance``): the
    same launch also advances the training step's device LR schedule (lr = table[step]; step += 1)."""
    M, K = h.shape
    C = w.shape[0]
    if not h.is_cuda:
        logits = F.linear(h.float(), w.float(), b)
        loss = F.cross_entropy(logits, targets) if targets is not None else None
        dl = None
        if want_grad and targets is not None:
            dl = (torch.softmax(logits, 1) - F.one_hot(targets, C).float()) / M
        if correct is not None and targets is not None:
            correct += (logits.argmax(1) == targets).sum().to(correct.dtype)
        return loss, logits, dl
    _check(h, w, b, targets)
    dev = h.device
    logits = torch.empty((M, C), dtype=torch.float32, device=dev) if want_logits else None
    have_t = targets is not None
    dl = torch.empty((M, C), dtype=torch.float32, device=dev) if (want_grad and have_t) else None
    loss = torch.empty((), dtype=torch.float32, device=dev) if have_t else None
    lib = native.kernels()
    # slice partials of the logits + row losses of the batch mean (combined in-launch by last arrivers)
    scratch = torch.empty((int(lib.ddpx_head_fwd_scratch(M, K)),), dtype=torch.float32, device=dev)
    tab, cnt, lrd = lr_advance if (lr_advance is not None and have_t) else (None, None, None)
    rc = lib.ddpx_head_fwd(h.data_ptr(), w.data_ptr(), b.data_ptr(), native.ptr(targets), M, K, C, h.stride(0),
                           1.0 / M, native.ptr(logits), native.ptr(dl), native.ptr(correct), scratch.data_ptr(),
                           _tickets(dev, int(lib.ddpx_head_fwd_tickets(M))).data_ptr(), native.ptr(loss),
                           native.ptr(tab), int(tab.numel()) if tab is not None else 0, native.ptr(cnt),
                           native.ptr(lrd), native.stream_handle())
    native.check(rc, "ddpx_head_fwd")
    return loss, logits, dl


_TICKETS: dict = {}
_RETIRED: list = []


def _tickets(dev, n):
    """Per-device arrival counters of the forward's in-launch reductions: zero between launches (each last
    arriver resets its counter).  Head forwards on one device are ordered on its compute stream."""
    t = _TICKETS.get(dev)
    if t is None or t.numel() < n:
        if torch.cuda.is_current_stream_capturing():
            raise RuntimeError("head_forward: first call for this batch size must happen outside graph capture")
        if t is not None:
            _RETIRED.append(t)  # a captured graph may still take tickets at the old address: keep it
        t = _TICKETS[dev] = torch.zeros((max(n, 1025),), dtype=torch.int32, device=dev)
    return t


def head_backward(dlogits, grad_out, h, w, dW, db, dH=None, dbprev=None, relu_mask=True, accumulate=False,
                  sgd_w=None, sgd_b=None, sgd_prev=None, dh_scale=1.0):
    """Backward of the fused head.

    dW [C,K] fp32, db [C] fp32 (=|+=); dH [M,K] bf16 = (grad · W) ⊙ (h>0 if relu_mask);
    dbprev [K] fp32 = Σ_m dH (bias gradient of the layer that produced h).
    dh_scale: multiplies dH — 1/(1-p) when h is an inverted-Dropout(p) output of a ReLU (DeepNN's
    classifier, ``/root/reference/singlegpu.py:33-38``): h > 0 is then the keep-and-positive mask.
    sgd_w / sgd_b / sgd_prev: fused optimizer targets (master, momentum, shadow, lr, mom, wd) that
    replace dW / db / dbprev (the gradients are applied instead of stored).
    """
    M, K = h.shape
    C = w.shape[0]
    if not h.is_cuda:
        g = dlogits * grad_out
        gw = g.t() @ h.float()
        gb = g.sum(0)
        if accumulate:
            dW.add_(gw)
            db.add_(gb)
        else:
            dW.copy_(gw)
            db.copy_(gb)
        if dH is not None:
            gh = g @ w.float()
            if relu_mask:
                gh = gh * (h > 0)
            gh = gh * dh_scale
            dH.copy_(gh)
            if dbprev is not None:
                s = dH.float().sum(0)
                dbprev.add_(s) if accumulate else dbprev.copy_(s)
        return dH
    _check(h, w, None, None)
    if K % 32:
        raise ValueError("head_backward: K must be a multiple of 32")
    if dH is not None and (dH.shape != h.shape or dH.dtype != torch.bfloat16 or dH.stride(0) != h.stride(0)):
        raise ValueError("head_backward: dH must match h")
    if dlogits.dtype != torch.float32 or not dlogits.is_contiguous() or tuple(dlogits.shape) != (M, C):
        raise ValueError("head_backward: dlogits must be contiguous fp32 [M, C]")
    fused = sgd_w is not None
    if fused:
        if sgd_b is None or (dbprev is not None) or sgd_w[0].numel() != C * K or sgd_b[0].numel() != C:
            raise ValueError("head_backward: fused optimizer needs sgd_w, sgd_b (and sgd_prev instead of dbprev)")
        gdt = torch.float32
    else:
        gdt = dW.dtype
        if tuple(dW.shape) != (C, K) or gdt not in (torch.float32, torch.bfloat16) or not dW.is_contiguous():
            raise ValueError("head_backward: dW must be contiguous [C,K] fp32/bf16")
        if db.dtype != gdt or (dbprev is not None and dbprev.dtype != gdt):
            raise ValueError("head_backward: dW, db, dbprev must share one dtype")
    lib = native.kernels()
    go = grad_out if torch.is_tensor(grad_out) else None
    if go is not None:
        go = go.to(torch.float32).contiguous()
    sw, sb, sp = (native.sgd_args(x) for x in (sgd_w, sgd_b, sgd_prev))
    lr_ptr = sw[3] if fused else None
    mom, wd = (sw[4], sw[5]) if fused else (0.0, 0.0)
    rc = lib.ddpx_head_bwd(dlogits.data_ptr(), native.ptr(go), h.data_ptr(), w.data_ptr(), M, K, C, h.stride(0),
                           native.ptr(dH), int(relu_mask), float(dh_scale), native.ptr(dW), native.ptr(db),
                           native.ptr(dbprev), int(gdt == torch.bfloat16), int(accumulate), *sw[:3], *sb[:3], *sp[:3],
                           lr_ptr, mom, wd, native.stream_handle())
    native.check(rc, "ddpx_head_bwd")
    return dH


def accuracy_count(logits, targets, correct):
    """correct (int32 0-d device tensor) += #(argmax(logits) == targets)."""
    if not logits.is_cuda:
        correct += (logits.argmax(1) == targets).sum().to(correct.dtype)
        return correct
    M, C = logits.shape
    lg = logits.float().contiguous()
    lib = native.kernels()
    native.check(lib.ddpx_accuracy(lg.data_ptr(), targets.data_ptr(), M, C, correct.data_ptr(),
                                   native.stream_handle()), "ddpx_accuracy")
    return correct
