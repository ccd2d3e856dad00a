"""SyncBatchNorm over a ddpx ``Comm`` (the reference's commented-out option).

Reference: ``#model = torch.nn.SyncBatchNorm.convert_sync_batchnorm(model)`` at
``/root/reference/multigpu.py:127`` ("considered, disabled"; exposed here as
``--sync_bn``, default off).

Batch statistics are computed over the GLOBAL batch: each rank computes its local per-channel
(count, mean, M2) and one all-gather + Chan merge makes them global; the backward all-reduces
(sum dy, sum dy*xhat).  Unlike torch's SyncBatchNorm this works on any ddpx comm — RCCL for GPU
tensors, gloo on the CPU test path — and keeps the module's state_dict keys identical to
``nn.BatchNorm2d`` so checkpoints stay in the reference format.
"""
from __future__ import annotations

import torch
from torch import nn


class _SyncBNFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, running_mean, running_var, num_batches_tracked, eps, momentum, comm, training):
        C = x.shape[1]
        if training:
            # local two-pass (mean, M2), then ONE all-gather of [n, mean, M2] per rank and a Chan merge
            # in fp64 — no E[x^2]-E[x]^2 cancellation, and the merge order is the same on every rank.
            xf = x.float()
            n_local = x.numel() // C
            lmean = xf.mean(dim=(0, 2, 3))
            lm2 = ((xf - lmean[None, :, None, None]) ** 2).sum(dim=(0, 2, 3))
            packed = torch.cat([torch.full((1,), float(n_local), device=x.device), lmean, lm2])
            ws = comm.world_size if comm is not None else 1
            if ws > 1:
                allp = torch.empty(ws * packed.numel(), dtype=packed.dtype, device=x.device)
                comm.allgather(allp, packed)
                allp = allp.view(ws, -1).double()
            else:
                allp = packed.view(1, -1).double()
            ns, means, m2s = allp[:, :1], allp[:, 1:C + 1], allp[:, C + 1:]
            n = ns.sum()
            mean64 = (ns * means).sum(0) / n
            m2 = m2s.sum(0) + (ns * (means - mean64) ** 2).sum(0)
            mean = mean64.float()
            var = (m2 / n).float()
            n = n.float()
            with torch.no_grad():
                unbiased = (m2 / (n.double() - 1).clamp_min(1)).float()
                running_mean.mul_(1 - momentum).add_(momentum * mean)
                running_var.mul_(1 - momentum).add_(momentum * unbiased)
                if num_batches_tracked is not None:
                    num_batches_tracked.add_(1)
        else:
            mean, var, n = running_mean, running_var, None
        rstd = torch.rsqrt(var + eps)
        xhat = (x.float() - mean[None, :, None, None]) * rstd[None, :, None, None]
        y = xhat * weight[None, :, None, None] + bias[None, :, None, None]
        ctx.save_for_backward(xhat, weight, rstd)
        ctx.comm, ctx.n = comm, n
        return y.to(x.dtype)

    @staticmethod
    def backward(ctx, gy):
        xhat, weight, rstd = ctx.saved_tensors
        g = gy.float()
        C = g.shape[1]
        dbeta = g.sum(dim=(0, 2, 3))
        dgamma = (g * xhat).sum(dim=(0, 2, 3))
        packed = torch.cat([dbeta, dgamma])
        if ctx.comm is not None and ctx.comm.world_size > 1:
            glob = packed.clone()
            ctx.comm.allreduce_(glob, op="sum")
        else:
            glob = packed
        n = ctx.n
        c1 = glob[:C] / n
        c2 = glob[C:] / n
        dx = (weight * rstd)[None, :, None, None] * (g - c1[None, :, None, None] - xhat * c2[None, :, None, None])
        # parameter gradients are local (DDP averages them across ranks), as in torch's SyncBatchNorm
        return dx.to(gy.dtype), dgamma, dbeta, None, None, None, None, None, None, None


class SyncBatchNorm2d(nn.BatchNorm2d):
    """Drop-in BatchNorm2d whose batch statistics are global across the comm's ranks."""

    comm = None

    def forward(self, x):
        if not self.training and self.track_running_stats:
            return super().forward(x)
        return _SyncBNFn.apply(x, self.weight, self.bias, self.running_mean, self.running_var,
                               self.num_batches_tracked, self.eps, self.momentum, self.comm, self.training)


def convert_sync_batchnorm(module: nn.Module, comm) -> nn.Module:
    """Replace every BatchNorm2d (keeping parameters, buffers and state_dict keys)."""
    out = module
    if isinstance(module, nn.BatchNorm2d) and not isinstance(module, SyncBatchNorm2d):
        out = SyncBatchNorm2d(module.num_features, module.eps, module.momentum, module.affine,
                              module.track_running_stats).to(module.weight.device)
        with torch.no_grad():
            out.weight.copy_(module.weight)
            out.bias.copy_(module.bias)
            out.running_mean.copy_(module.running_mean)
            out.running_var.copy_(module.running_var)
            out.num_batches_tracked.copy_(module.num_batches_tracked)
        out.train(module.training)
    if isinstance(out, SyncBatchNorm2d):
        out.comm = comm
    for name, child in module.named_children():
        out.add_module(name, convert_sync_batchnorm(child, comm))
    return out
