"""The MLP's hidden stack as one autograd node on the CPU (BASELINE config 1), writing weight gradients
straight into the flat DDP-bucket storage.

torch's autograd gives every Linear a freshly allocated ``.grad`` that ``FlatParams`` then copies into its
flat gradient buffer (``flat_params.py`` ``_on_accumulated``): a 118 MB allocation plus a 118 MB copy per
step on the toy MLP.  Here the backward computes dW = dyᵀ·x with ``torch.mm(..., out=main_grad)`` (or
``addmm_`` when gradients accumulate across backwards) and announces each parameter with
``FlatParams.grad_done`` in gradient-ready order (classifier first), exactly like the native GPU path
(``ddpx/ops/mlp.py``), so DDP's bucket all-reduces still overlap the rest of the backward.  The loss stays
torch's ``F.cross_entropy`` on the returned logits.  Reference recipe: ``/root/reference/singlegpu.py:102-108``
(one ``_run_batch``: forward, cross-entropy, backward, SGD step).
"""
from __future__ import annotations

import torch


def eligible(model, x) -> bool:
    w = model.fc0.weight
    flat = getattr(w, "_ddpx_flat", None)
    # the backward writes fp32 GEMM results straight into the flat gradient buffer (``out=``): a bf16 gradient
    # buffer (--grad_dtype bf16) takes the generic autograd path, which casts on accumulation
    return (not x.is_cuda and torch.is_grad_enabled() and not x.requires_grad and w.dtype == torch.float32
            and flat is not None and flat.grad is not None and flat.grad.dtype == torch.float32)


class _MLPCPU(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, model, *params):
        lins = model.linears()
        hs = [x]
        h = x
        for lin in lins[:-1]:
            h = torch.addmm(lin.bias, h, lin.weight.t()).relu_()
            hs.append(h)
        ctx.model, ctx.hs, ctx.n = model, hs, len(params)
        return torch.addmm(lins[-1].bias, h, lins[-1].weight.t())

    @staticmethod
    def backward(ctx, d):
        model, hs = ctx.model, ctx.hs
        lins = model.linears()
        flat = lins[0].weight._ddpx_flat
        d = d.contiguous()
        for i in range(len(lins) - 1, -1, -1):
            lin = lins[i]
            dw, acc = flat.grad_target(lin.weight)
            if acc:
                dw.addmm_(d.t(), hs[i])
            else:
                torch.mm(d.t(), hs[i], out=dw)
            db, acc_b = flat.grad_target(lin.bias)
            if acc_b:
                db.add_(d.sum(0))
            else:
                torch.sum(d, 0, out=db)
            if i > 0:
                # ReLU backward from the stored output (threshold_backward's rule: gradient where output > 0)
                d = torch.mm(d, lin.weight).mul_(hs[i] > 0)
            flat.grad_done(lin.weight)
            flat.grad_done(lin.bias)
        ctx.hs = None
        return (None, None) + (None,) * ctx.n


def mlp_logits(model, x):
    """Logits of ``model`` (an ``ddpx.models.MLP`` on a FlatParams store) for flattened fp32 ``x``."""
    return _MLPCPU.apply(x, model, *model.parameters())
