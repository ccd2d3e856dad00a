"""DistributedDataParallel for one process per MI355X.

Behaviour parity with ``DDP(model, device_ids=[gpu_id])`` as the reference
uses it (``/root/reference/multigpu.py:89``):

* construction: verify parameter shapes across ranks (C1), broadcast all
  parameters and buffers from rank 0 (C2) — the reference never seeds, so
  this is what makes the replicas identical;
* every forward: broadcast the module buffers (BN running stats) from rank 0
  (C3, ``broadcast_buffers=True``);
* backward: gradients are averaged across ranks bucket by bucket while
  backward is still running (C6); bucket k's all-reduce is issued the moment
  its last gradient is produced.

MI355X-specific design:

* Buckets are contiguous slices of the flat gradient buffer (``FlatParams``),
  assigned by torch's size rule (``_compute_bucket_assignment_by_size``) on the
  grad-ready order from the first iteration on — no pack/unpack, no rebuild
  step (C4/C5 become unnecessary).
* Bucket caps default to 1 MiB first / 25 MiB after, overridable
  (``bucket_cap_mb``, ``first_bucket_mb``) to tune for point-to-point xGMI
  rings.
* With :class:`~ddpx.parallel.comm.RcclComm` the reducer is native C++
  (events + RCCL on a dedicated high-priority stream, ``ncclAvg``).  With a
  ``TorchComm`` (gloo, CPU tests) an equivalent Python reducer is used.
* ``overlap_optimizer=True`` leaves the buckets un-joined at the end of
  backward; ``ddpx.optim.SGD`` then updates each bucket's slice as soon as its
  collective lands, overlapping the optimizer with the remaining traffic.
* ``shard_optimizer=True`` (ZeRO-1, not in the reference — SURVEY §2.5 lists it as absent):
  the flat store is re-packed so every bucket splits into ``world_size`` equal 256-B-aligned
  shards; backward reduce-scatters each bucket in place (same bytes on the wire as the
  all-reduce's first half), every rank runs SGD on its own shard only (1/N of the optimizer's
  HBM traffic), and the updated parameters are all-gathered in place.  For models whose
  kernels read weights only through the bf16 compute shadow (the native MLP) just the shadow
  is gathered — half the bytes of an fp32 all-gather — and the few fp32-read parameters
  (biases) stay replicated in one all-reduced bucket.  ``consolidate()`` gathers fp32 master
  weights and momentum on every rank before a checkpoint.
"""
from __future__ import annotations

import contextlib
import os

import torch
import torch.distributed as dist
from torch import nn

from ..runtime import native
from ..runtime.flat_params import ALIGN, FlatParams, flat_of
from .comm import NCCL_DTYPE, NCCL_OP, Comm, RcclComm, TorchComm

DEFAULT_FIRST_BUCKET_MB = 1.0   # dist._DEFAULT_FIRST_BUCKET_BYTES
DEFAULT_BUCKET_CAP_MB = 25.0    # DDP bucket_cap_mb default


def compute_bucket_assignment(sizes_bytes, limits_bytes):
    """torch's greedy rule: close a bucket once it reaches the current limit."""
    buckets, cur, cur_size, li = [], [], 0, 0
    for i, s in enumerate(sizes_bytes):
        cur.append(i)
        cur_size += s
        if cur_size >= limits_bytes[min(li, len(limits_bytes) - 1)]:
            buckets.append(cur)
            cur, cur_size = [], 0
            li += 1
    if cur:
        buckets.append(cur)
    return buckets


def plan_buckets(order, sizes_bytes, limits_bytes, chunked=()):
    """torch's greedy rule over ``order``; a parameter in ``chunked`` closes the open bucket and becomes
    its own entry ("c", i) (expanded into one bucket per row chunk); others group as ("p", [i, ...])."""
    out, cur, cur_size, li = [], [], 0, 0
    for i in order:
        if i in chunked:
            if cur:
                out.append(("p", cur))
                cur, cur_size = [], 0
                li += 1
            out.append(("c", i))
            li += 1
            continue
        cur.append(i)
        cur_size += sizes_bytes[i]
        if cur_size >= limits_bytes[min(li, len(limits_bytes) - 1)]:
            out.append(("p", cur))
            cur, cur_size = [], 0
            li += 1
    if cur:
        out.append(("p", cur))
    return out


def row_chunks(shape, elem_bytes, chunk_bytes, pad):
    """Row ranges of ~chunk_bytes for a parameter of ``shape``; every chunk boundary is a multiple of
    ``pad`` elements (equal aligned shards per chunk) and of 64 rows' worth of 16-B column offsets."""
    import math
    rows = shape[0]
    cols = 1
    for d in shape[1:]:
        cols *= d
    g = pad // math.gcd(cols, pad)
    g = g * 64 // math.gcd(g, 64)  # also a multiple of 64 rows (aligned column slices of dY)
    n = max(1, round(rows * cols * elem_bytes / max(1, chunk_bytes)))
    per = -(-(-(-rows // n)) // g) * g  # ceil(rows / n), rounded up to the granule: near-equal chunks
    if per >= rows:
        return None
    return [(r, min(rows, r + per)) for r in range(0, rows, per)]


class FlatBuffers:
    """Module buffers rebound as views of one flat tensor per dtype (broadcast in one call each)."""

    def __init__(self, module: nn.Module):
        entries = [(m, n, b) for m in module.modules() for n, b in m._buffers.items() if b is not None]
        self.flats = {}
        by_dtype = {}
        for m, n, b in entries:
            by_dtype.setdefault(b.dtype, []).append((m, n, b))
        for dt, items in by_dtype.items():
            total = sum(b.numel() for _, _, b in items)
            flat = torch.empty(total, dtype=dt, device=items[0][2].device)
            off = 0
            for m, n, b in items:
                view = flat[off:off + b.numel()].view(b.shape)
                view.copy_(b)
                m._buffers[n] = view
                off += b.numel()
            self.flats[dt] = flat

    def tensors(self):
        return list(self.flats.values())


class _PyReducer:
    """Bucket state machine over torch.distributed async collectives (CPU / gloo)."""

    def __init__(self, comm: TorchComm, ranges, modes=None):
        self.comm = comm
        self.ranges = ranges
        self.modes = modes or [0] * len(ranges)
        self.tensors = None
        self.expected = None
        self.pending = None
        self.works = None
        self.gather_targets = [None] * len(ranges)

    def set_gather(self, b, t):
        self.gather_targets[b] = t

    def gather(self, b):
        """In-place all-gather of bucket b's parameter copy (synchronous on gloo)."""
        t = self.gather_targets[b]
        self.comm.allgather(t, t.chunk(self.comm.world_size)[self.comm.rank])

    def wait_gather(self, b, stream=None):
        pass

    def setup(self, grad_flat, expected):
        self.tensors = [grad_flat[s:e] for s, e in self.ranges]
        self.expected = list(expected)
        self.prepare()

    def prepare(self):
        self.pending = list(self.expected)
        self.works = [None] * len(self.ranges)
        self.launched = [False] * len(self.ranges)

    def _launch(self, b):
        # gloo has no reduce-scatter: a sharded bucket is all-reduced (its own shard is what the
        # optimizer reads, exactly as after an in-place reduce-scatter)
        self.works[b] = self.comm.allreduce_(self.tensors[b], op="avg", async_op=True)
        self.launched[b] = True

    def mark_ready(self, b, n=1):
        if self.launched[b]:
            raise RuntimeError(f"bucket {b} marked ready twice in one backward")
        self.pending[b] -= n
        if self.pending[b] == 0:
            self._launch(b)

    def wait_bucket(self, b, stream=None):
        w = self.works[b]
        if w is not None:
            w.wait()
            self.works[b] = None

    def finalize(self, join=True):
        forced = 0
        for b in range(len(self.ranges)):
            if not self.launched[b]:
                self._launch(b)
                forced += 1
        if join:
            for b in range(len(self.ranges)):
                self.wait_bucket(b)
        return forced


class _NativeReducer:
    """ctypes front-end of the C++ reducer (csrc/runtime/rccl_comm.cpp)."""

    def __init__(self, comm: RcclComm, ranges, modes=None):
        self.comm = comm
        self.ranges = ranges
        self.modes = modes or [0] * len(ranges)
        self.rt = native.runtime()
        self.h = self.rt.ddpx_reducer_create(comm.handle, len(ranges), NCCL_OP["avg"])
        self._gkeep = {}

    def setup(self, grad_flat, expected):
        dt = NCCL_DTYPE[grad_flat.dtype]
        self._keep = grad_flat
        for b, (s, e) in enumerate(self.ranges):
            t = grad_flat[s:e]
            native.check(self.rt.ddpx_reducer_set_bucket(self.h, b, t.data_ptr(), t.numel(), dt, expected[b],
                                                         self.modes[b]), "reducer_set_bucket")

    def set_gather(self, b, t):
        self._gkeep[b] = t
        native.check(self.rt.ddpx_reducer_set_gather(self.h, b, t.data_ptr(), t.numel(), NCCL_DTYPE[t.dtype]),
                     "reducer_set_gather")

    def gather(self, b):
        native.check(self.rt.ddpx_reducer_gather(self.h, b, native.stream_handle()), "reducer_gather")

    def wait_gather(self, b, stream=None):
        native.check(self.rt.ddpx_reducer_wait_gather(self.h, b, native.stream_handle(stream)),
                     "reducer_wait_gather")

    def prepare(self):
        self.rt.ddpx_reducer_prepare(self.h)

    def mark_ready(self, b, n=1):
        rc = self.rt.ddpx_reducer_mark_ready(self.h, b, n, native.stream_handle())
        if rc not in (0, 1):
            raise RuntimeError(f"reducer mark_ready(bucket={b}) failed: {rc}")

    def wait_bucket(self, b, stream=None):
        rc = self.rt.ddpx_reducer_wait_bucket(self.h, b, native.stream_handle(stream))
        if rc != 0:
            raise RuntimeError(f"reducer wait_bucket({b}) failed: {rc}")

    def finalize(self, join=True):
        if join:
            rc = self.rt.ddpx_reducer_finalize(self.h, native.stream_handle())
            if rc < 0:
                raise RuntimeError(f"reducer finalize failed: {rc}")
            return rc
        self.rt.ddpx_reducer_mark_backward_end(self.h, native.stream_handle())
        return 0

    def comm_stats(self):
        c, e = native.ctypes.c_float(0), native.ctypes.c_float(0)
        if self.rt.ddpx_reducer_comm_stats(self.h, native.ctypes.byref(c), native.ctypes.byref(e)) != 0:
            return None
        return {"comm_ms": c.value, "comm_exposed_ms": e.value,
                "comm_overlap": (1.0 - e.value / c.value) if c.value > 0 else None}

    def close(self):
        if self.h:
            self.rt.ddpx_reducer_destroy(self.h)
            self.h = None


class DistributedDataParallel(nn.Module):
    _side_seq = 0  # names of registered optimizer side streams

    def __init__(self, module: nn.Module, device_ids=None, comm: Comm | None = None,
                 bucket_cap_mb: float = DEFAULT_BUCKET_CAP_MB, first_bucket_mb: float = DEFAULT_FIRST_BUCKET_MB,
                 broadcast_buffers: bool = True, overlap_optimizer: bool = False, verify: bool = True,
                 reduce_single: bool = False, shard_optimizer: bool = False, chunk_mb: float | None = None,
                 defer_gather: bool = False, comm_side_optimizer: bool = False,
                 find_unused_parameters: bool = False, side_stream_optimizer: bool = False):
        super().__init__()
        # torch DDP semantics: False (default) -> a parameter without gradient on some rank is an error at
        # world size > 1 (its bucket would otherwise be issued in a different order on different ranks);
        # True -> buckets are issued at the end of backward in bucket order, unused gradients as zeros
        self.find_unused_parameters = bool(find_unused_parameters)
        self.comm_side_optimizer = comm_side_optimizer
        self.module = module
        dev = next(module.parameters()).device
        self.device = dev
        self.flat: FlatParams = flat_of(module) or FlatParams(module)
        if self.flat.fused_opt is not None:
            # gradients must be all-reduced before the update: no optimizer-in-backward fusion
            self.flat.fused_opt.disable_fused()
        if comm is None:
            from .comm import default_comm
            comm = default_comm(dev)
        self.comm = comm
        self.world_size = comm.world_size
        self.rank = comm.rank
        self.broadcast_buffers = broadcast_buffers
        self.overlap_optimizer = overlap_optimizer
        self._sync_enabled = True
        self._queued = False
        self._overlap_pending = False

        # C1: parameter metadata must agree across ranks.
        if verify and self.world_size > 1:
            meta = [(tuple(p.shape), str(p.dtype)) for p in self.flat.params]
            allm = comm.all_gather_object(meta)
            for r, m in enumerate(allm):
                if m != meta:
                    raise RuntimeError(f"DDP: parameter shapes differ between rank {self.rank} and rank {r}")

        # Buffers as flat per-dtype tensors (one broadcast each).
        self.buffers_flat = FlatBuffers(module) if any(True for _ in module.buffers()) else None

        # C2: make replicas identical.
        self._broadcast_state()

        # Buckets: contiguous flat ranges over grad-ready order.
        active = self.world_size > 1 or reduce_single  # reduce_single: exercise the reducer at ws=1 (tests)
        self.sharded = bool(shard_optimizer and active)
        esz = self.flat.grad.element_size()
        limits = [int(first_bucket_mb * 1024 * 1024), int(bucket_cap_mb * 1024 * 1024)]
        # big weights split into row chunks, each its own bucket (its collective starts as soon as that
        # chunk's gradient is written; producers that do not announce chunks complete them all at once)
        pad = self.world_size * ALIGN if self.sharded else ALIGN
        chunk_plan = {}
        if chunk_mb and active:
            for i, p in enumerate(self.flat.params):
                if p.dim() >= 2 and p.numel() * esz > chunk_mb * 1024 * 1024:
                    rc = row_chunks(tuple(p.shape), esz, int(chunk_mb * 1024 * 1024), pad)
                    if rc:
                        chunk_plan[id(p)] = rc
        if self.sharded:
            plan, modes = self._shard_layout(limits, esz, chunk_plan)
        else:
            sizes = [n * esz for n in self.flat.numels]
            chunked = {i for i, p in enumerate(self.flat.params) if id(p) in chunk_plan}
            plan = plan_buckets(range(len(self.flat.params)), sizes, limits, chunked)
            modes = None
        for p in self.flat.params:
            self.flat.set_chunks(p, chunk_plan.get(id(p)))
        # expand the plan into buckets: (param list, chunk index or None, flat range)
        f = self.flat
        assign, ranges, expected, chunk_ids, bmodes = [], [], [], [], []
        self.bucket_of = [0] * len(f.params)
        self.chunk_bucket = {}
        for k, entry in enumerate(plan):
            mode = modes[k] if modes is not None else 0
            if entry[0] == "p":
                idxs = entry[1]
                for i in idxs:
                    self.bucket_of[i] = len(assign)
                assign.append(list(idxs))
                ranges.append(f.span(idxs[0], idxs[-1]))
                expected.append(len(idxs))
                chunk_ids.append(None)
                bmodes.append(mode)
            else:
                i = entry[1]
                rc = f.chunk_rows[i]
                cols = f.numels[i] // f.params[i].shape[0]
                s0, e0 = f.span(i, i)
                if self.sharded:
                    e0 = f.group_spans[k][1]
                self.chunk_bucket[i] = []
                for c, (r0, r1) in enumerate(rc):
                    self.chunk_bucket[i].append(len(assign))
                    self.bucket_of[i] = len(assign)
                    assign.append([i])
                    ranges.append((s0 + r0 * cols, e0 if c == len(rc) - 1 else s0 + r1 * cols))
                    expected.append(1)
                    chunk_ids.append(c)
                    bmodes.append(mode)
        modes = bmodes
        self.bucket_params = assign
        self.bucket_modes = modes
        self.bucket_chunk = chunk_ids
        self.bucket_expected = expected
        self.bucket_ranges = ranges
        if active:
            cls = _NativeReducer if isinstance(comm, RcclComm) else _PyReducer
            self.reducer = cls(comm, ranges, modes)
            self.reducer.setup(self.flat.grad, expected)
            if self.sharded:
                for b, (s0, e0) in enumerate(ranges):
                    if modes[b] == 1:
                        self.reducer.set_gather(b, self._gather_src[s0:e0])
        else:
            self.reducer = None
        opt = getattr(self.flat, "optimizer", None)
        if self.sharded and opt is not None:
            self.attach_optimizer(opt)
        # every rank must agree on the bucket layout (a mismatch would pair wrong slices in RCCL)
        if verify and self.world_size > 1:
            layout = [tuple(r) for r in self.bucket_ranges], list(self.bucket_modes)
            for r, other in enumerate(comm.all_gather_object(layout)):
                if other != layout:
                    raise RuntimeError(f"DDP: bucket layout differs between rank {self.rank} and rank {r}")
        self.debug = os.environ.get("DDPX_DEBUG", "0") == "1"
        self.flat.sink = self
        # replicated plan, optimizer overlap: every bucket's SGD update runs on a side stream as soon as (a) its
        # all-reduce has landed and (b) nothing later in this backward reads its weights — the bucket's ready
        # point, or for a parameter the model declares read after its gradient (flat.late_read: the MLP's data
        # gradient reads W_l after W_l's gradient was produced) the model's release (flat.release, recorded on
        # the compute stream right after that last read), or the end of backward if the release never came.
        # One join of the side stream per step instead of one wait per bucket on the compute stream, and the
        # updates overlap the rest of backward (at N > 1: the later buckets' collectives)
        self._opt_stream = None
        if (side_stream_optimizer and active and not self.sharded and overlap_optimizer
                and isinstance(comm, RcclComm) and dev.type == "cuda"):
            self._opt_stream = torch.cuda.Stream(dev)
            from ..runtime.graphs import register_side_stream
            DistributedDataParallel._side_seq += 1
            self._side_name = f"DDP optimizer stream #{DistributedDataParallel._side_seq}"
            # by (owner, attribute), held weakly: a dropped wrapper leaves no stale stream in the registry
            register_side_stream(self, self._side_name, attr="_opt_stream")
        late = getattr(self.flat, "late_read", None)
        # late-read parameters per bucket; unknown read pattern (late = None): every bucket waits for backward's end
        self._late = [(sum(1 for i in self.bucket_params[b] if id(self.flat.params[i]) in late) if late is not None
                       else 1 << 30) for b in range(len(self.bucket_ranges))]
        self._released = [0] * len(self.bucket_ranges)
        self._rel_ev = [None] * len(self.bucket_ranges)
        self._bwd_end_ev = None
        self._completion_order = []
        self._marks = [0] * len(self.bucket_ranges)
        # deferred all-gather (ZeRO-1 shadow gathers): the optimizer leaves the gathers of the updated
        # shards to the NEXT forward, which issues them first thing, in forward order, and waits per
        # bucket right before the first read, so the traffic overlaps the forward GEMMs (and, captured
        # in one HIP graph per step, still overlaps: issue and waits live in the same replay)
        self.defer_gather = bool(defer_gather and self.sharded and self.gather_what == "shadow")
        self._gather_todo = []
        self._gather_wait = set()
        if self.sharded:
            def fwd_key(b):
                return (-max(self.bucket_params[b]), self.bucket_chunk[b] or 0)
            self._gather_order = sorted([b for b, m in enumerate(self.bucket_modes) if m == 1], key=fwd_key)

    def _shard_layout(self, limits, esz, chunk_plan):
        """Re-pack the flat store for ZeRO-1 (see module docstring); returns (bucket plan, modes) in the
        new parameter indices (a chunked parameter is one group, expanded into chunk buckets later)."""
        f = self.flat
        if f.shadow is not None and f.shadow_only:
            S = [i for i, p in enumerate(f.params) if id(p) in f.shadow_only]
            self.gather_what = "shadow"
        else:
            S = list(range(len(f.params)))
            self.gather_what = "master"
        R = [i for i in range(len(f.params)) if i not in set(S)]
        chunked = {i for i in S if id(f.params[i]) in chunk_plan}
        sizes = {i: f.numels[i] * esz for i in S}
        plan = plan_buckets(S, sizes, limits, chunked)
        groups = [e[1] if e[0] == "p" else [e[1]] for e in plan]
        kinds = [e[0] for e in plan]
        modes = [1] * len(groups)
        if R:
            groups.append(R)  # fp32-read params: one replicated (all-reduced) bucket, produced last
            kinds.append("p")
            modes.append(0)
        f.relayout(groups, pad_to=self.world_size * ALIGN)
        self._gather_src = f.shadow if self.gather_what == "shadow" else f.master
        out, k = [], 0
        for g, kind in zip(groups, kinds):
            idxs = list(range(k, k + len(g)))
            out.append(("p", idxs) if kind == "p" else ("c", idxs[0]))
            k += len(g)
        return out, modes

    # ------------------------------------------------------- sharded optimizer
    def bucket_order(self):
        if self._overlap_pending:
            order = list(self._completion_order)
            return order + [b for b in range(len(self.bucket_ranges)) if b not in order]
        return list(range(len(self.bucket_ranges)))

    def wait_bucket(self, b):
        self.reducer.wait_bucket(b)
        if b in self._gather_wait:  # the shard about to be updated must not race its pending gather
            self.reducer.wait_gather(b)
            self._gather_wait.discard(b)

    def claim_bucket_on_comm_stream(self, b):
        """wait_bucket() for an update issued ON the communicator stream: the reduce-scatter and any
        pending gather of ``b`` precede it in stream order, so only the bookkeeping remains (a HIP graph
        capture must not see an event waited on by the stream that recorded it)."""
        self._gather_wait.discard(b)

    def update_ranges(self, b):
        s, e = self.bucket_ranges[b]
        if self.bucket_modes[b] == 1:
            c = (e - s) // self.world_size
            return [(s + self.rank * c, s + (self.rank + 1) * c)]
        return [(s, e)]

    def gather_bucket(self, b):
        if self.bucket_modes[b] == 1:
            if self.defer_gather:
                self._gather_todo.append(b)
            else:
                self.reducer.gather(b)

    def _issue_gathers(self):
        todo = set(self._gather_todo)
        self._gather_todo = []
        for b in self._gather_order:
            if b in todo:
                self.reducer.gather(b)
                self._gather_wait.add(b)

    def _wait_gathers(self, buckets=None):
        for b in (sorted(self._gather_wait) if buckets is None else buckets):
            if b in self._gather_wait:
                self.reducer.wait_gather(b)
                self._gather_wait.discard(b)

    def flush_gathers(self):
        """Complete every deferred all-gather (before eval, checkpoints, or handing weights out)."""
        if self._gather_todo:
            self._issue_gathers()
        self._wait_gathers()

    def before_read(self, i, chunk=None):
        if not self._gather_wait:
            return
        if i in self.chunk_bucket:
            bs = self.chunk_bucket[i] if chunk is None else [self.chunk_bucket[i][chunk]]
        else:
            bs = [self.bucket_of[i]]
        self._wait_gathers(bs)

    def _join_gathers(self):
        if self.defer_gather:
            return
        for b, m in enumerate(self.bucket_modes):
            if m == 1:
                self.reducer.wait_gather(b)
                if self.gather_what == "master" and self.flat.shadow is not None:
                    from ..ops.elementwise import cast_bf16_
                    s, e = self.bucket_ranges[b]
                    cast_bf16_(self.flat.master[s:e], self.flat.shadow[s:e])

    @torch.no_grad()
    def consolidate(self):
        """Collective: make fp32 master weights and optimizer state complete on every rank.

        Needed before ``state_dict()`` / checkpointing when the optimizer is sharded (each rank
        only keeps its own shards of master/momentum current).  No-op otherwise.
        """
        if not self.sharded:
            return
        self.flush_gathers()
        tensors = [self.flat.master] + list(self.flat.state_tensors.values())
        for b, (s, e) in enumerate(self.bucket_ranges):
            if self.bucket_modes[b] != 1:
                continue
            for t in tensors:
                full = t[s:e]
                self.comm.allgather(full, full.chunk(self.world_size)[self.rank])
        if self.flat.master.is_cuda:
            torch.cuda.current_stream().synchronize()

    # ------------------------------------------------------------- state sync
    @torch.no_grad()
    def _broadcast_state(self):
        if self.world_size == 1:
            return
        self.comm.broadcast_(self.flat.master, 0)
        if self.buffers_flat is not None:
            for t in self.buffers_flat.tensors():
                self.comm.broadcast_(t, 0)
        self.flat.refresh_shadow()

    @torch.no_grad()
    def _sync_buffers(self):
        if self.world_size > 1 and self.broadcast_buffers and self.buffers_flat is not None:
            for t in self.buffers_flat.tensors():
                self.comm.broadcast_(t, 0)

    # ---------------------------------------------------------------- forward
    def _pre_forward(self):
        self.comm.check()
        if self._gather_todo:
            self._issue_gathers()
            if not getattr(self.module, "ddpx_lazy_gather", False):
                self._wait_gathers()  # the model's ops do not announce reads: wait for everything now
        if torch.is_grad_enabled() and self.reducer is not None and self._sync_enabled:
            if self._overlap_pending:
                raise RuntimeError("DDP: optimizer.step() did not consume the previous iteration's buckets")
            self.reducer.prepare()
            self._completion_order = []
            self._marks = [0] * len(self.bucket_ranges)
            self._released = [0] * len(self.bucket_ranges)
            self._rel_ev = [None] * len(self.bucket_ranges)
            self._bwd_end_ev = None
        self._queued = False
        if self.module.training:
            self._sync_buffers()

    def forward(self, *args, **kwargs):
        self._pre_forward()
        return self.module(*args, **kwargs)

    def forward_loss(self, *args, **kwargs):
        self._pre_forward()
        return self.module.forward_loss(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        old = self._sync_enabled
        self._sync_enabled = False
        try:
            yield
        finally:
            self._sync_enabled = old

    # ------------------------------------------------------ gradient protocol
    def grad_ready(self, i: int, chunk=None):
        if self.reducer is None or not self._sync_enabled:
            return
        if not self._queued:
            self._queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finalize)
        if i in self.chunk_bucket:
            bs = self.chunk_bucket[i] if chunk is None else [self.chunk_bucket[i][chunk]]
        else:
            bs = [self.bucket_of[i]]
        for b in bs:
            self._marks[b] += 1
            if not self.find_unused_parameters:
                self.reducer.mark_ready(b, 1)
            if self._marks[b] == self.bucket_expected[b]:
                self._completion_order.append(b)

    def param_released(self, i: int):
        """The model's last read of parameter i in this backward has been issued (flat.release): once every
        late-read parameter of its bucket is released, the side-stream update of that bucket may start."""
        if self._opt_stream is None or not self._sync_enabled:
            return
        bs = self.chunk_bucket[i] if i in self.chunk_bucket else [self.bucket_of[i]]
        for b in bs:
            self._released[b] += 1
            if self._released[b] == self._late[b]:
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream())
                self._rel_ev[b] = ev

    def reducer_launched(self, b):
        return self._marks_complete(b)

    def _marks_complete(self, b):
        return self._marks[b] == self.bucket_expected[b]

    def _unused_names(self):
        f = self.flat
        return [f.names.get(id(f.params[i]), str(i)) for i, w in enumerate(f.written) if not w and not f.updated[i]]

    def _finalize(self):
        if self.reducer is None:
            return
        skip = []
        if self.find_unused_parameters:
            # every bucket is issued here, in bucket order (identical on every rank); gradients of
            # parameters this rank did not use are zeros
            f = self.flat
            local_used = [1 if (w or u) else 0 for w, u in zip(f.written, f.updated)]
            f.fix_unwritten(mark_written=True)
            for b in range(len(self.bucket_ranges)):
                self.reducer.mark_ready(b, self.bucket_expected[b])
            self._completion_order = list(range(len(self.bucket_ranges)))
            # torch's local_used_map: a parameter NO rank used this iteration has no gradient (None in torch),
            # so the optimizer must not apply weight decay / momentum to it (one small MAX all-reduce + a host
            # read: this opt-in path is not graph-capturable, as in torch)
            used = torch.tensor(local_used, dtype=torch.int32, device=f.master.device)
            if self.world_size > 1:
                self.comm.allreduce_(used, op="max")
            skip = [i for i, v in enumerate(used.tolist()) if v == 0]
        elif len(self._completion_order) < len(self.bucket_ranges):
            unused = self._unused_names()
            if self.world_size > 1:
                raise RuntimeError(
                    f"DDP (rank {self.rank}): parameters {unused} received no gradient in this backward; their "
                    "buckets cannot be reduced in the same order on every rank.  Pass find_unused_parameters=True "
                    "(torch DDP's flag) if the model skips parameters.")
            # world size 1 (reduce_single): no ordering hazard; stale gradients must not be reduced
            self.flat.fix_unwritten(mark_written=True)
        if self.debug and self.world_size > 1:
            # TORCH_DISTRIBUTED_DEBUG=DETAIL-style check: identical bucket completion order on every rank
            order = list(self._completion_order)
            for r, other in enumerate(self.comm.all_gather_object(order)):
                if other != order:
                    raise RuntimeError(f"DDP debug: bucket completion order {order} on rank {self.rank} "
                                       f"!= {other} on rank {r}")
        if skip:
            # the optimizer steps parameter ranges around the skipped ones: every bucket must be joined first
            self.reducer.finalize(join=True)
            for i in skip:
                self.flat.updated[i] = True
            return
        if self._opt_stream is not None:
            ev = torch.cuda.Event()
            ev.record(torch.cuda.current_stream())
            self._bwd_end_ev = ev  # release point of buckets whose model never released their late reads
        if self.overlap_optimizer:
            self._overlap_pending = True
            # launch stragglers but do not join: the optimizer waits per bucket
            if isinstance(self.reducer, _PyReducer):
                self.reducer.finalize(join=False)
            else:
                missing = [b for b in range(len(self.bucket_ranges)) if b not in self._completion_order]
                if missing:
                    self.reducer.finalize(join=True)
                    self._overlap_pending = False
                else:
                    self.reducer.finalize(join=False)  # timing marker for comm_stats()
        else:
            self.reducer.finalize(join=True)

    # ----------------------------------------- optimizer overlap (SGD hooks)
    def overlap_active(self):
        return self.overlap_optimizer and self._overlap_pending

    def bucket_ranges_in_completion_order(self):
        order = list(self._completion_order)
        order += [b for b in range(len(self.bucket_ranges)) if b not in order]
        self._iter_order = order
        return [self.bucket_ranges[b] for b in order]

    def wait_range(self, start, end):
        b = self.bucket_ranges.index((start, end))
        self.reducer.wait_bucket(b)

    def update_side_stream(self):
        """Replicated plan: the stream the per-bucket SGD updates run on (side_stream_optimizer), else None."""
        return self._opt_stream if self.overlap_active() else None

    def side_wait_bucket(self, b, stream):
        """Make ``stream`` wait for bucket b's all-reduce and for the release of its weights."""
        self.reducer.wait_bucket(b, stream)
        if self._late[b]:
            ev = self._rel_ev[b] if self._released[b] >= self._late[b] else self._bwd_end_ev
            if ev is not None:
                stream.wait_event(ev)

    def optimizer_stream(self):
        """The stream the ZeRO-1 shard updates run on when ``comm_side_optimizer`` is set (the native
        RCCL stream, right behind each bucket's reduce-scatter: no per-bucket join back into the compute
        stream), else None."""
        if (self.comm_side_optimizer and self.sharded and isinstance(self.reducer, _NativeReducer)
                and getattr(self.comm, "stream", None) is not None):
            return self.comm.stream
        return None

    def optimizer_done(self):
        if self.sharded:
            self._join_gathers()
        self._overlap_pending = False

    def attach_optimizer(self, opt):
        opt.bucket_source = self

    def sync_grads(self):
        """Join all outstanding bucket collectives (overlap mode) into the current stream."""
        if self._overlap_pending:
            for b in range(len(self.bucket_ranges)):
                self.reducer.wait_bucket(b)
            self._overlap_pending = False

    def comm_stats(self):
        """{'comm_ms', 'comm_exposed_ms', 'comm_overlap'} of the last iteration (native RCCL reducer)."""
        if self.reducer is None or not hasattr(self.reducer, "comm_stats"):
            return None
        return self.reducer.comm_stats()

    # ------------------------------------------------- aborted-iteration recovery
    def iteration_state(self):
        """Host-side bucket bookkeeping between iterations (see :meth:`restore_iteration_state`)."""
        return {"gather_todo": list(self._gather_todo), "gather_wait": set(self._gather_wait)}

    def restore_iteration_state(self, st):
        """Forget an iteration that never ran on the device (a HIP-graph capture that failed part-way): the
        bucket state goes back to ``st`` (taken by :meth:`iteration_state` before it), no collective is
        waited for, and deferred ZeRO-1 all-gathers the aborted capture consumed are owed again."""
        self._overlap_pending = False
        self._queued = False
        self._completion_order = []
        self._marks = [0] * len(self.bucket_ranges)
        self._gather_todo = list(st["gather_todo"])
        self._gather_wait = set(st["gather_wait"])
        if self.reducer is not None:
            self.reducer.prepare()

    # ----------------------------------------------------------------- misc
    def state_dict(self, *args, **kwargs):
        return super().state_dict(*args, **kwargs)

    def close(self):
        if self._opt_stream is not None:
            from ..runtime.graphs import unregister_side_stream
            unregister_side_stream(self._side_name)
            self._opt_stream = None
        if self.reducer is not None and hasattr(self.reducer, "close"):
            self.reducer.close()
