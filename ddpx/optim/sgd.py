"""Fused flat-buffer SGD (momentum, weight decay) — drop-in for torch.optim.SGD.

Reference: ``torch.optim.SGD(model.parameters(), lr=0.4, momentum=0.9,
weight_decay=5e-4)`` at ``/root/reference/singlegpu.py:136-141`` (default
foreach path, ``torch/optim/sgd.py:383-478``: 4 multi-tensor passes / step).

Here all parameters are views of one flat fp32 buffer (``FlatParams``), so a
step is ONE kernel launch (``ddpx_sgd_flat``) that reads p, g, momentum once
and writes p, momentum and the bf16 compute shadow once — or one launch per
DDP bucket when the optimizer is overlapped with the gradient all-reduce
(each slice starts as soon as its bucket's collective lands).

The class subclasses ``torch.optim.Optimizer`` so torch LR schedulers
(``LambdaLR``) drive it unchanged.  ``capturable=True`` reads the learning rate
from a device scalar, which makes ``step()`` safe inside a HIP graph.
"""
from __future__ import annotations

import os

import torch
from torch.optim import Optimizer

from ..ops.elementwise import sgd_flat_
from ..runtime.flat_params import FlatParams, flat_of


# Device LR-schedule advance waiting for a kernel to carry it (SGD.device_lr_step): the classifier head's
# forward launch takes it (take_lr_advance), which saves the training step a separate 1-thread kernel;
# anything that reads lr before a head forward took it launches it on its own first (SGD._flush_lr).
# The pending advance is a field of the parameter store the optimizer owns (``FlatParams.pending_lr``),
# so optimizers of different models in one process never hand their advances to each other.
# DDPX_LR_IN_HEAD=0 always launches the separate kernel.
_LR_IN_HEAD = os.environ.get("DDPX_LR_IN_HEAD", "1") != "0"


def take_lr_advance(flat):
    """(table, counter, lr) if the optimizer of ``flat`` has an LR advance pending (it is then the caller's
    launch that performs it), else None."""
    p = getattr(flat, "pending_lr", None)
    if p is None:
        return None
    flat.pending_lr = None
    return p


class SGD(Optimizer):
    def __init__(self, params, lr: float = 1e-3, momentum: float = 0.0, dampening: float = 0.0,
                 weight_decay: float = 0.0, nesterov: bool = False, capturable: bool = False,
                 fused_backward: bool = False):
        if dampening != 0.0:
            raise ValueError("ddpx.optim.SGD implements dampening=0 (the reference's setting)")
        if nesterov and momentum <= 0:
            raise ValueError("Nesterov momentum requires a momentum")
        params = list(params)
        super().__init__(params, dict(lr=lr, momentum=momentum, dampening=dampening, weight_decay=weight_decay,
                                      nesterov=nesterov))
        if len(self.param_groups) != 1:
            raise ValueError("ddpx.optim.SGD supports a single parameter group")
        flat = flat_of(params)
        if flat is None:
            raise ValueError("parameters are not flattened: wrap the model with ddpx.prepare_model() first")
        ids = {id(p) for p in params}
        if ids != {id(p) for p in flat.params}:
            raise ValueError("SGD must own exactly the parameters of one FlatParams store")
        self.flat: FlatParams = flat
        if momentum:
            # registered with the store so a re-layout (sharded DDP) carries it along
            flat.state_tensors["momentum"] = torch.zeros_like(flat.master)
        self.capturable = capturable
        # fused_backward: single-process training applies each parameter's update inside the kernel
        # that produces its gradient (no gradient round trip through HBM, no separate SGD pass).
        self.fused_backward = bool(fused_backward and flat.master.is_cuda and not nesterov)
        need_dev_lr = capturable or self.fused_backward
        self._lr_dev = torch.full((), float(lr), dtype=torch.float32, device=flat.device) if need_dev_lr else None
        if self.fused_backward:
            flat.fused_opt = self
        self._lr_table = None  # device-side LR schedule (attach_device_schedule)
        self._lr_counter = None
        self.bucket_source = None  # set by DDP when the optimizer overlaps the all-reduce or is sharded
        flat.optimizer = self
        if getattr(flat.sink, "sharded", False):
            flat.sink.attach_optimizer(self)
        self.step_count = 0

    @property
    def lr_dev(self):
        """Device learning-rate scalar (None without one); current once any pending advance has run."""
        self._flush_lr()
        return self._lr_dev

    @property
    def momentum_buffer(self):
        return self.flat.state_tensors.get("momentum")

    # ------------------------------------------------------------------ API
    def zero_grad(self, set_to_none: bool = True):  # noqa: D401 - torch signature
        self.flat.zero_grad()

    def fused_active(self) -> bool:
        return self.fused_backward

    def disable_fused(self):
        self.fused_backward = False
        if self.flat.fused_opt is self:
            self.flat.fused_opt = None

    def sync_lr(self):
        """Copy the host learning rate into the device scalar (outside graph capture).

        No-op while a device-side schedule is attached (the step kernel sequence advances it)."""
        if self._lr_dev is not None and self._lr_table is None:
            self._lr_dev.fill_(float(self.param_groups[0]["lr"]))

    def attach_device_schedule(self, scheduler, horizon: int | None = None):
        """Tabulate a LambdaLR-style schedule on the device (lr[k] = base_lr * lambda(k)).

        After this, :meth:`device_lr_step` — called at the start of every training step, inside the
        captured graph — sets ``lr_dev`` from the table and advances a device step counter, so graph
        replays need no host-to-device write.  The host scheduler keeps stepping for bookkeeping
        (state_dict, logging).  ``horizon``: table length (default: the one-cycle's end + 1).
        """
        if self._lr_dev is None or not self._lr_dev.is_cuda:
            return False
        lam = scheduler.lr_lambdas[0]
        base = scheduler.base_lrs[0]
        if horizon is None:
            spe, ne = getattr(lam, "steps_per_epoch", None), getattr(lam, "num_epochs", None)
            horizon = spe * ne + 1 if spe and ne else 100_000
        table = torch.tensor([base * lam(k) for k in range(horizon)], dtype=torch.float32)
        self._lr_table = table.to(self._lr_dev.device)
        self._lr_counter = torch.tensor([scheduler.last_epoch], dtype=torch.int32, device=self._lr_dev.device)
        return True

    def step_counter(self):
        """The device step counter the LR-table kernel advances once per ``device_lr_step`` (int32 [1]), or
        None without a device schedule; other per-step device work (the data cursor) may read it."""
        return getattr(self, "_lr_counter", None) if self._lr_table is not None else None

    def device_lr_step(self):
        if self._lr_table is None:
            return
        self._flush_lr()
        if _LR_IN_HEAD:
            self.flat.pending_lr = (self._lr_table, self._lr_counter, self._lr_dev)
            return
        self._launch_lr_advance()

    def _flush_lr(self):
        """Launch this optimizer's pending LR advance if no kernel took it (before anything reads lr)."""
        if getattr(self.flat, "pending_lr", None) is not None:
            self.flat.pending_lr = None
            self._launch_lr_advance()

    def _launch_lr_advance(self):
        from ..runtime import native
        native.check(native.kernels().ddpx_lr_advance(self._lr_table.data_ptr(), self._lr_table.numel(),
                                                      self._lr_counter.data_ptr(), self._lr_dev.data_ptr(),
                                                      native.stream_handle()), "ddpx_lr_advance")

    def _lr_arg(self):
        self._flush_lr()
        return self._lr_dev if self._lr_dev is not None else float(self.param_groups[0]["lr"])

    def _update(self, start, end, g, fp8=True):
        f = self.flat
        if f.pp_parity:
            f.normalize_pingpong(start, end)  # the flat pass writes the main bf16 copy
        buf = self.momentum_buffer[start:end] if self.momentum_buffer is not None else f.master[start:end]
        sh = f.shadow[start:end] if f.shadow is not None else None
        # a store that keeps an MX-FP8 weight copy gets it written in the same pass (fp8 forward GEMMs)
        mx8 = f.mx8_range(start, end) if (fp8 and f.master.is_cuda) else None
        sgd_flat_(f.master[start:end], buf, f.grad[start:end], sh, self._lr_arg(), g["momentum"],
                  g["weight_decay"], nesterov=g["nesterov"], mx8=mx8)
        f.fp8_mark(start, end, mx8 is not None)

    def _stepped(self, ranges):
        """``ranges`` (flat [start, end) pairs) minus the spans of parameters already stepped or skipped this
        iteration (``FlatParams.updated``): what the optimizer still has to update."""
        f = self.flat
        if not any(f.updated):
            return list(ranges)
        holes = [f.span(i, i) for i, u in enumerate(f.updated) if u]
        out = []
        for (s, e) in ranges:
            cur = s
            for (hs, he) in sorted(holes):
                if he <= cur or hs >= e:
                    continue
                if hs > cur:
                    out.append((cur, hs))
                cur = max(cur, he)
            if cur < e:
                out.append((cur, e))
        return out

    @torch.no_grad()
    def step(self, closure=None):
        loss = None
        if closure is not None:
            with torch.enable_grad():
                loss = closure()
        g = self.param_groups[0]
        if not (self.flat.master.is_cuda and torch.cuda.is_current_stream_capturing()):
            # torch.optim.SGD skips a parameter whose .grad is None (no weight decay, no momentum step):
            # a parameter nobody produced a gradient for this step is marked as already stepped, so every
            # branch below leaves it alone (DDP's find_unused_parameters path marks the globally unused ones)
            for i in self.flat.fix_unwritten():
                self.flat.updated[i] = True
        src = self.bucket_source
        if src is not None and getattr(src, "sharded", False):
            # ZeRO-1: each rank updates only its shard of every sharded bucket (gradients were
            # reduce-scattered), then the bucket's parameter copy is all-gathered in place
            side = src.optimizer_stream() if hasattr(src, "optimizer_stream") else None
            if side is None:
                for b in src.bucket_order():
                    src.wait_bucket(b)
                    for (start, end) in self._stepped(src.update_ranges(b)):
                        self._update(start, end, g, fp8=False)
                    src.gather_bucket(b)
            else:
                # shard updates on the communicator stream, in stream order behind each bucket's
                # reduce-scatter: one compute -> comm edge (end of backward: nothing still reads the
                # weights) and one comm -> compute join at the end instead of a join per bucket
                cur = torch.cuda.current_stream()
                ev = torch.cuda.Event()
                ev.record(cur)
                side.wait_event(ev)
                with torch.cuda.stream(side):
                    for b in src.bucket_order():
                        src.claim_bucket_on_comm_stream(b)
                        for (start, end) in self._stepped(src.update_ranges(b)):
                            self._update(start, end, g, fp8=False)
                        src.gather_bucket(b)
                done = torch.cuda.Event()
                done.record(side)
                cur.wait_event(done)
            src.optimizer_done()
            # the all-gathers refreshed master / bf16 copies of every shard, not the fp8 copy
            self.flat.fp8_mark(0, self.flat.total, False)
        elif any(self.flat.updated):
            # fused-backward parameters are already stepped; update the rest range by range
            f = self.flat
            i, n = 0, len(f.params)
            while i < n:
                if f.updated[i]:
                    i += 1
                    continue
                j = i
                while j + 1 < n and not f.updated[j + 1]:
                    j += 1
                self._update(*f.span(i, j), g)
                i = j + 1
        elif src is not None and src.overlap_active():
            side = src.update_side_stream() if hasattr(src, "update_side_stream") else None
            if side is None:
                for (start, end) in src.bucket_ranges_in_completion_order():
                    src.wait_range(start, end)
                    self._update(start, end, g)
            else:
                # each bucket's update on the side stream behind its all-reduce and its weights' release, in
                # completion order (no wait for the end of backward); one join into the compute stream.  A pending
                # LR advance (none when the head kernel took it) is launched on the side stream before the first
                # update reads the LR.
                cur = torch.cuda.current_stream()
                for (start, end) in src.bucket_ranges_in_completion_order():
                    b = src.bucket_ranges.index((start, end))
                    src.side_wait_bucket(b, side)
                    with torch.cuda.stream(side):
                        self._update(start, end, g)
                done = torch.cuda.Event()
                done.record(side)
                cur.wait_event(done)
            src.optimizer_done()
        else:
            self._update(0, self.flat.total, g)
        self.step_count += 1
        return loss

    # ------------------------------------------------------- (de)serialise
    def state_dict(self):
        sd = super().state_dict()
        state = {}
        if self.momentum_buffer is not None and self.step_count > 0:
            for i, p in enumerate(self.param_groups[0]["params"]):
                j = self.flat.index[id(p)]
                state[i] = {"momentum_buffer": self.momentum_buffer[self.flat.slice(j)].view(p.shape).clone()}
        sd["state"] = state
        sd["ddpx_step_count"] = self.step_count
        return sd

    def load_state_dict(self, state_dict):
        state_dict = dict(state_dict)
        st = state_dict.pop("state", {})
        self.step_count = int(state_dict.pop("ddpx_step_count", 0))
        groups = state_dict["param_groups"]
        for k, v in groups[0].items():
            if k != "params":
                self.param_groups[0][k] = v
        if self.momentum_buffer is not None:
            for i, p in enumerate(self.param_groups[0]["params"]):
                s = st.get(i, st.get(str(i)))
                if s is not None and s.get("momentum_buffer") is not None:
                    j = self.flat.index[id(p)]
                    self.momentum_buffer[self.flat.slice(j)].copy_(s["momentum_buffer"].reshape(-1))
        self._lr_table = None  # a resumed schedule position: re-attach the device schedule
        self.sync_lr()
