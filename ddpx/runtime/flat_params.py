"""Flat parameter / gradient / shadow storage for a module.

MI355X-first memory layout:

* every trainable parameter becomes a view into ONE contiguous fp32 ``master``
  buffer, laid out in *gradient-ready order* (reverse registration order, the
  order backward produces gradients — the same order torch DDP's reducer
  rebuilds its buckets into, ``torch/nn/parallel/distributed.py:1551``);
* gradients live in a parallel flat buffer; ``p.main_grad`` is the view.  DDP
  buckets are contiguous slices of it, so an all-reduce never packs/unpacks;
* an optional parallel bf16 ``shadow`` holds the compute copy of the weights
  the MFMA GEMMs read; the fused SGD kernel refreshes it in the same pass that
  updates ``master`` (no separate cast kernel per step);
* each parameter offset is 64-element aligned so every slice is 256-B aligned
  for the 16-B vector loads of the kernels.

Gradients arrive in two ways:

1. native ops (``ddpx.ops``) write straight into ``main_grad`` with the GEMM
   epilogue and call :meth:`grad_done`;
2. parameters used by stock torch ops get a post-accumulate-grad hook that
   moves ``p.grad`` into ``main_grad`` and then calls :meth:`grad_done`.

``zero_grad`` is O(#params) host work: it only resets the "written" flags; the
first writer of an iteration overwrites instead of accumulating
(``set_to_none=True`` semantics of ``/root/reference/singlegpu.py:103``).
"""
from __future__ import annotations

import os
import warnings

import torch

ALIGN = 64


def _round_up(x, a):
    return (x + a - 1) // a * a


class FlatParams:
    def __init__(self, module: torch.nn.Module, grad_dtype=torch.float32, shadow_dtype=None,
                 native_params=(), align: int = ALIGN):
        params = [p for p in module.parameters() if p.requires_grad]
        if not params:
            raise ValueError("module has no trainable parameters")
        device = params[0].device
        for p in params:
            if p.device != device:
                raise ValueError("all parameters must be on one device")
            if p.dtype != torch.float32:
                raise ValueError("FlatParams expects fp32 master parameters")
        self.device = device
        self.align = max(ALIGN, int(align))  # element alignment of every parameter offset (and of relayout groups)
        self.params = list(reversed(params))  # gradient-ready order
        self.names = {}
        for name, p in module.named_parameters():
            self.names[id(p)] = name
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.offsets, self.numels = [], []
        off = 0
        for p in self.params:
            self.offsets.append(off)
            self.numels.append(p.numel())
            off = _round_up(off + p.numel(), align)
        self.total = off
        # per-parameter update counter: consumers that keep a derived copy of a weight (the VGG path's permuted
        # bf16 conv layouts) re-derive it when the counter moved since they last did
        self.version = [0] * len(self.params)
        # ping-pong bf16 copies (enable_pingpong): param index -> the alternate buffer's view; pp_parity[i] = 1
        # while the param's current copy (p._ddpx_shadow, what readers read) is the alternate buffer
        self.pp_alt = {}
        self.pp_parity = {}
        self.master = torch.zeros(self.total, dtype=torch.float32, device=device)
        self.grad = torch.zeros(self.total, dtype=grad_dtype, device=device)
        self.shadow = torch.zeros(self.total, dtype=shadow_dtype, device=device) if shadow_dtype else None
        with torch.no_grad():
            for p, o, n in zip(self.params, self.offsets, self.numels):
                view = self.master[o:o + n].view_as(p)
                view.copy_(p.data)
                p.data = view
                p.main_grad = self.grad[o:o + n].view(p.shape)
                if self.shadow is not None:
                    p._ddpx_shadow = self.shadow[o:o + n].view(p.shape)
                p._ddpx_flat = self
        self.refresh_shadow()
        self.native = {id(p) for p in native_params}
        self.written = [False] * len(self.params)
        self.updated = [False] * len(self.params)  # parameter already stepped by a fused-optimizer epilogue
        self.fused_opt = None  # set by ddpx.optim.SGD(fused_backward=True)
        self.sink = None
        # parameters the model reads in backward AFTER producing their gradient (announced through release()):
        # a side-stream optimizer must not rewrite them before that read (ddpx.parallel.ddp)
        self.late_read = None
        self.optimizer = None  # the ddpx SGD that owns this store (set by SGD)
        # device LR-schedule advance of that optimizer not launched yet: (table, counter, lr) until a kernel
        # (the classifier head's forward) carries it or the optimizer launches it itself (ddpx.optim.sgd)
        self.pending_lr = None
        # params whose forward/backward read ONLY the bf16 shadow (never the fp32 master) —
        # a sharded optimizer may then all-gather just the shadow for them
        self.shadow_only = set()
        # per-parameter optimizer state laid out like master (e.g. momentum), remapped by relayout()
        self.state_tensors = {}
        self.layout_version = 0
        self.group_spans = None
        # row-chunked parameters (DDP splits big weights into per-chunk buckets): index -> [(r0, r1)]
        self.chunk_rows = {}
        self._chunks_done = {}
        self._warned_unused = False
        # optional MX-FP8 (e4m3) copy of every parameter (enable_fp8_shadow): codes [total] + E8M0 scales of
        # each 32-element run [total / 32] (offsets are 64-aligned, so every parameter starts a block);
        # fp8_fresh[i]: the copy of parameter i matches its master (an optimizer stream wrote it)
        self.shadow8 = None
        self.scale8 = None
        self.fp8_fresh = [False] * len(self.params)
        # optional transposed MX-FP8 copy (enable_fp8_transposed): parameter [M, N] stored as its transpose [N, M]
        # with 32-blocks along M (the data gradient's operand), written by the fused wgrad+SGD pair
        self.shadow8t = None
        self.scale8t = None
        self.fp8t_fresh = [False] * len(self.params)
        # which optimizer kernels write the fp8 copy next to the bf16 one (DDPX_FP8_COPY): "pair" (default) the
        # fused wgrad+SGD stream (+53-126 us on the wide MLP's pair vs 175 us for quantising both weights
        # separately, profiles/r3_fp8), "1" also the flat SGD (DDP path; not measured faster), "0" none (every
        # fp8 forward re-quantises the bf16 copy)
        mode = os.environ.get("DDPX_FP8_COPY", "pair")
        self.fp8_from_optimizer = mode in ("1", "pair")
        self.fp8_from_flat_sgd = mode == "1"
        self._hooks = []
        for p in self.params:
            if id(p) not in self.native:
                self._hooks.append(p.register_post_accumulate_grad_hook(self._on_accumulated))

    # -- views --------------------------------------------------------------
    def slice(self, i):
        o, n = self.offsets[i], self.numels[i]
        return slice(o, o + n)

    def span(self, first: int, last: int):
        """Flat element range [start, end) covering params first..last (inclusive, aligned end)."""
        start = self.offsets[first]
        end = self.offsets[last + 1] if last + 1 < len(self.params) else self.total
        return start, end

    def shadow_of(self, p):
        return getattr(p, "_ddpx_shadow", None)

    # -- ping-pong bf16 copies ---------------------------------------------------
    # A kernel that READS a weight's bf16 copy while an optimizer stream in the same launch rewrites that weight
    # (the toy MLP's fc1 data gradient inside the fused weight-gradient + SGD launch, ops/mlp.py) writes the new
    # copy into a second buffer instead; the copies then alternate every step, so a captured step exists in
    # two versions (ddpx.runtime.graphs.CapturedCycle).  Generic writers of ``shadow`` (flat SGD, DDP gathers,
    # refresh) see the main buffer: normalize_pingpong() moves a parameter back to it first.
    def enable_pingpong(self, p):
        i = self.index[id(p)]
        if i in self.pp_alt:
            return
        if self.shadow is None:
            raise RuntimeError("ping-pong copies need a bf16 shadow")
        if torch.cuda.is_available() and self.master.is_cuda and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("enable_pingpong must run outside graph capture")
        main = self.shadow[self.slice(i)].view(p.shape)
        self.pp_alt[i] = main.clone()
        self.pp_parity[i] = 0
        p._ddpx_shadow = main

    def has_pingpong(self, p) -> bool:
        return self.index[id(p)] in self.pp_alt

    def shadow_next(self, p):
        """The buffer an update of p that must not overwrite its current copy writes the new copy to."""
        i = self.index[id(p)]
        main = self.shadow[self.slice(i)].view(p.shape)
        return main if self.pp_parity[i] else self.pp_alt[i]

    def flip_pingpong(self, p):
        """p's new copy (written to shadow_next) becomes the current one."""
        i = self.index[id(p)]
        p._ddpx_shadow = self.shadow_next(p)
        self.pp_parity[i] ^= 1

    def pingpong_signature(self):
        return tuple(sorted(self.pp_parity.items()))

    def set_pingpong_signature(self, sig):
        """Restore parities taken by pingpong_signature() (host bookkeeping of an aborted capture)."""
        for i, par in sig:
            if self.pp_parity.get(i) != par:
                p = self.params[i]
                p._ddpx_shadow = self.shadow_next(p)
                self.pp_parity[i] = par

    def normalize_pingpong(self, start=None, end=None):
        """Parameters (overlapping [start, end)) whose current copy is the alternate buffer: copy it back into the
        main shadow and make that current (before a generic writer updates the main buffer)."""
        for i, par in list(self.pp_parity.items()):
            if not par:
                continue
            o, n = self.offsets[i], self.numels[i]
            if start is not None and (o >= end or o + n <= start):
                continue
            p = self.params[i]
            main = self.shadow[self.slice(i)].view(p.shape)
            main.copy_(self.pp_alt[i])
            p._ddpx_shadow = main
            self.pp_parity[i] = 0

    def enable_fp8_shadow(self):
        """Keep an MX-FP8 copy of the parameters for fp8 forward GEMMs: the optimizer kernels that can write it
        next to the bf16 copy do (flat SGD, fused weight-gradient + SGD pair), anything else marks it stale and
        the next reader re-quantises (``mx8_weight``)."""
        if self.shadow8 is None:
            self.shadow8 = torch.zeros(self.total, dtype=torch.uint8, device=self.device)
            self.scale8 = torch.zeros(self.total // 32, dtype=torch.uint8, device=self.device)
        self.fp8_fresh = [False] * len(self.params)

    def mx8_views(self, p):
        """(codes [rows, cols], scales [rows, cols / 32]) views of p's fp8 copy, or None without one."""
        if self.shadow8 is None or p.dim() != 2 or p.shape[1] % 32:
            return None
        i = self.index[id(p)]
        o, n = self.offsets[i], self.numels[i]
        if o % 128:
            return None  # the MX GEMM needs 16-B code / 4-B scale alignment (a 128-aligned store: align=128)
        return (self.shadow8[o:o + n].view(p.shape),
                self.scale8[o // 32:(o + n) // 32].view(p.shape[0], p.shape[1] // 32))

    def enable_fp8_transposed(self):
        """Keep the transposed MX-FP8 copy too (fp8 data gradients); stale until an optimizer writes it."""
        if self.shadow8t is None:
            self.shadow8t = torch.zeros(self.total, dtype=torch.uint8, device=self.device)
            self.scale8t = torch.zeros(self.total // 32, dtype=torch.uint8, device=self.device)
        self.fp8t_fresh = [False] * len(self.params)

    def mx8t_views(self, p):
        """(codes [cols, rows], scales [cols, rows / 32]) views of p's transposed fp8 copy, or None."""
        if self.shadow8t is None or p.dim() != 2 or p.shape[0] % 64:
            return None
        i = self.index[id(p)]
        o, n = self.offsets[i], self.numels[i]
        if o % 128:
            return None
        return (self.shadow8t[o:o + n].view(p.shape[1], p.shape[0]),
                self.scale8t[o // 32:(o + n) // 32].view(p.shape[1], p.shape[0] // 32))

    def mx8t_weight(self, p):
        """pᵀ as an MX-FP8 operand with blocks along p's rows: the optimizer-written copy when current, else the
        bf16 copy quantised transposed now (into the store when it keeps one)."""
        from ..ops import fp8 as F8
        v = self.mx8t_views(p)
        if v is None:
            return F8.quant(self.shadow_of(p), F8.E4M3, rows=False, cols=True)
        i = self.index[id(p)]
        if not self.fp8t_fresh[i]:
            F8.quant(self.shadow_of(p), F8.E4M3, rows=False, cols=True, out_t=v)
            self.fp8t_fresh[i] = True
        return F8.MX(v[0], v[1], F8.E4M3)

    def mx8_weight(self, p):
        """p's MX-FP8 operand (ddpx.ops.fp8.MX): the optimizer-written copy when current, else the bf16 copy
        quantised now (into the store when it keeps one, so later readers of this step reuse it)."""
        from ..ops import fp8 as F8
        v = self.mx8_views(p)
        if v is None:
            return F8.quant(self.shadow_of(p), F8.E4M3)
        i = self.index[id(p)]
        if not self.fp8_fresh[i]:
            F8.quant(self.shadow_of(p), F8.E4M3, out=v)
            self.fp8_fresh[i] = True
        return F8.MX(v[0], v[1], F8.E4M3)

    def fp8_mark(self, start, end, written):
        """Parameters overlapping the flat range [start, end) were updated; ``written``: the update also wrote
        the fp8 copy of the range (only parameters entirely inside it count as current)."""
        for i, (o, n) in enumerate(zip(self.offsets, self.numels)):
            if o < end and o + n > start:
                self.version[i] += 1
                if self.shadow8 is not None:
                    self.fp8_fresh[i] = bool(written and o >= start and o + n <= end)
                self.fp8t_fresh[i] = False  # (no flat optimizer writes the transposed copy)

    def mx8_range(self, start, end):
        """(codes, scales) slices of the fp8 copy for a flat update of [start, end), or None."""
        if self.shadow8 is None or not self.fp8_from_flat_sgd or start % 32 or (end - start) % 32:
            return None
        return self.shadow8[start:end], self.scale8[start // 32:end // 32]

    def invalidate_derived(self):
        """Treat every derived copy of the weights as stale: the MX-FP8 copy and any consumer-held layout keyed
        by :meth:`version_of` (the VGG path's bf16 conv layouts) are re-derived by their next reader.

        For host bookkeeping that ran without its device work, e.g. a HIP-graph capture that aborted after the
        forward had recorded a weight re-layout or quantisation (and marked it current) that never executed."""
        self.fp8_fresh = [False] * len(self.params)
        self.fp8t_fresh = [False] * len(self.params)
        # every parameter moves past any version a consumer may hold
        self.version = [max(self.version, default=0) + 1] * len(self.params)

    def refresh_shadow(self):
        self.invalidate_derived()  # (also across a relayout's re-indexing)
        for i in list(self.pp_parity):  # every copy back on the main buffer (rewritten just below)
            p = self.params[i]
            p._ddpx_shadow = self.shadow[self.slice(i)].view(p.shape)
            self.pp_parity[i] = 0
        if self.shadow is None:
            return
        from ..ops.elementwise import cast_bf16_
        cast_bf16_(self.master, self.shadow)

    def relayout(self, groups, pad_to: int = ALIGN):
        """Re-pack the store as ``groups`` (lists of current param indices) in the given order.

        Each group starts 64-element aligned and its length is padded to a multiple of ``pad_to``
        (a sharded optimizer needs every bucket divisible into equal, aligned shards).  Values of
        master, shadow and registered state tensors move with their parameters; gradients reset.
        Returns the new [start, end) span of every group.
        """
        order = [i for g in groups for i in g]
        if sorted(order) != list(range(len(self.params))):
            raise ValueError("relayout groups must cover every parameter exactly once")
        self.normalize_pingpong()
        self.pp_alt, self.pp_parity = {}, {}  # (indices change; re-enabled by their user)
        if pad_to % ALIGN:
            raise ValueError("pad_to must be a multiple of the alignment")
        new_params = [self.params[i] for i in order]
        old_params = list(self.params)
        offsets, spans, off, k = [], [], 0, 0
        for g in groups:
            start = off = _round_up(off, self.align)
            for _ in g:
                p = new_params[k]
                offsets.append(off)
                off = _round_up(off + p.numel(), self.align)
                k += 1
            off = start + _round_up(max(off - start, pad_to), pad_to)
            spans.append((start, off))
        off = _round_up(off, self.align)
        total = off
        dev = self.device
        master = torch.zeros(total, dtype=torch.float32, device=dev)
        grad = torch.zeros(total, dtype=self.grad.dtype, device=dev)
        shadow = torch.zeros(total, dtype=self.shadow.dtype, device=dev) if self.shadow is not None else None
        states = {k_: torch.zeros(total, dtype=t.dtype, device=dev) for k_, t in self.state_tensors.items()}
        with torch.no_grad():
            for p, o in zip(new_params, offsets):
                i_old = self.index[id(p)]
                so, n = self.offsets[i_old], self.numels[i_old]
                master[o:o + n].copy_(self.master[so:so + n])
                for k_, t in self.state_tensors.items():
                    states[k_][o:o + n].copy_(t[so:so + n])
                view = master[o:o + n].view_as(p)
                p.data = view
                p.main_grad = grad[o:o + n].view(p.shape)
                if shadow is not None:
                    p._ddpx_shadow = shadow[o:o + n].view(p.shape)
        self.params = new_params
        self.index = {id(p): i for i, p in enumerate(self.params)}
        self.offsets = offsets
        self.numels = [p.numel() for p in self.params]
        self.total = total
        self.master, self.grad, self.shadow = master, grad, shadow
        if self.shadow8 is not None:
            self.shadow8 = torch.zeros(total, dtype=torch.uint8, device=dev)
            self.scale8 = torch.zeros(total // 32, dtype=torch.uint8, device=dev)
        if self.shadow8t is not None:
            self.shadow8t = torch.zeros(total, dtype=torch.uint8, device=dev)
            self.scale8t = torch.zeros(total // 32, dtype=torch.uint8, device=dev)
        self.state_tensors = states
        self.refresh_shadow()
        self.written = [False] * len(self.params)
        self.updated = [False] * len(self.params)
        self.chunk_rows = {self.index[id(p)]: r for p, r in ((old_params[i], r) for i, r in self.chunk_rows.items())}
        self._chunks_done = {}
        self.group_spans = spans
        self.layout_version += 1
        return spans

    # -- row chunks --------------------------------------------------------------
    def set_chunks(self, p, ranges):
        """Declare p's gradient/parameter as row chunks [(r0, r1), ...] (dim 0), each its own DDP bucket.

        Producers that know about chunks announce them one by one (``grad_done(p, chunk=c)``) so each
        chunk's collective starts while the rest of the gradient is still being computed; producers that
        do not simply call ``grad_done(p)``, which completes every chunk."""
        i = self.index[id(p)]
        if ranges:
            self.chunk_rows[i] = list(ranges)
        else:
            self.chunk_rows.pop(i, None)

    def chunks_of(self, p):
        return self.chunk_rows.get(self.index[id(p)])

    def release(self, p):
        """The model's last read of p in this backward has been issued (p in ``late_read``)."""
        if self.sink is not None and hasattr(self.sink, "param_released"):
            self.sink.param_released(self.index[id(p)])

    def before_read(self, p, chunk=None):
        """Called by native ops right before they read p (or its row chunk) in a forward: a sharded
        optimizer with deferred all-gathers makes the current stream wait for that data here."""
        if self.sink is not None and hasattr(self.sink, "before_read"):
            self.sink.before_read(self.index[id(p)], chunk)

    # -- gradient protocol -----------------------------------------------------
    def grad_target(self, p):
        """(main_grad view, accumulate?) for a native op about to write p's gradient."""
        i = self.index[id(p)]
        return p.main_grad, self.written[i]

    def fused_spec(self, p):
        """(master, momentum, shadow, lr, mom, wd) if p's update should be fused into its backward kernel."""
        o = self.fused_opt
        if o is None or not o.fused_active():
            return None
        i = self.index[id(p)]
        if self.written[i] or self.updated[i]:
            return None  # gradient accumulation across backwards: fall back to materialised grads
        sl = self.slice(i)
        g = o.param_groups[0]
        buf = o.momentum_buffer[sl] if o.momentum_buffer is not None else None
        sh = self.shadow[sl] if self.shadow is not None else None
        o._flush_lr()  # an LR advance no head forward took must land before this epilogue reads lr
        return (self.master[sl], buf, sh, o.lr_dev, g["momentum"], g["weight_decay"])

    def version_of(self, p) -> int:
        return self.version[self.index[id(p)]]

    def mark_updated(self, p, fp8_written: bool = False, fp8t_written: bool = False):
        i = self.index[id(p)]
        self.updated[i] = True
        self.written[i] = True
        self.version[i] += 1
        self.fp8_fresh[i] = bool(fp8_written and self.shadow8 is not None)
        self.fp8t_fresh[i] = bool(fp8t_written and self.shadow8t is not None)

    def grad_done(self, p, chunk=None):
        i = self.index[id(p)]
        if chunk is not None and i in self.chunk_rows:
            done = self._chunks_done.setdefault(i, set())
            if chunk in done:
                raise RuntimeError(f"chunk {chunk} of {self.names.get(id(p), i)} announced twice")
            done.add(chunk)
            if len(done) == len(self.chunk_rows[i]):
                self.written[i] = True
                del self._chunks_done[i]
            if self.sink is not None:
                self.sink.grad_ready(i, chunk)
            return
        if i in self._chunks_done:  # remaining chunks of a partially announced parameter
            rest = [c for c in range(len(self.chunk_rows[i])) if c not in self._chunks_done.pop(i)]
        else:
            rest = None
        self.written[i] = True
        if self.sink is not None:
            if rest is None:
                self.sink.grad_ready(i)
            else:
                for c in rest:
                    self.sink.grad_ready(i, c)

    def _on_accumulated(self, p):
        i = self.index[id(p)]
        g = p.grad
        if g is None:
            return
        if self.written[i]:
            p.main_grad.add_(g)
        else:
            p.main_grad.copy_(g)
        p.grad = None
        self.written[i] = True
        if self.sink is not None:
            self.sink.grad_ready(i)

    def zero_grad(self):
        self._chunks_done = {}
        self.written = [False] * len(self.params)
        self.updated = [False] * len(self.params)
        for p in self.params:
            p.grad = None

    def fix_unwritten(self, mark_written: bool = False):
        """Zero gradients nobody produced this iteration (stale values would otherwise be applied).

        ``mark_written``: the zeros are this iteration's gradient (DDP reduces them next), so later
        callers (``SGD.step``) must not zero the reduced result again."""
        missing = [i for i, w in enumerate(self.written) if not w and not self.updated[i]]
        if missing:
            if not self._warned_unused:
                names = [self.names.get(id(self.params[i]), str(i)) for i in missing]
                warnings.warn(f"ddpx: parameters without gradient this step (gradient zeroed; the optimizer "
                              f"does not step them, as torch.optim.SGD skips grad=None): {names}")
                self._warned_unused = True
            for i in missing:
                self.grad[self.slice(i)].zero_()
                if mark_written:
                    self.written[i] = True
        return missing

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []


def flat_of(module_or_params):
    """Find the FlatParams that owns a module's (or a param list's) parameters."""
    if isinstance(module_or_params, torch.nn.Module):
        ps = list(module_or_params.parameters())
    else:
        ps = list(module_or_params)
    for p in ps:
        f = getattr(p, "_ddpx_flat", None)
        if f is not None:
            return f
    return None
