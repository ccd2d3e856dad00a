"""Whole-training-step HIP graph capture.

At the reference's batch size the MLP step is ~0.2 ms of GPU work spread over
~20 kernels plus the collectives: launch- and host-bound in eager mode.  The
step (zero_grad → forward → backward with bucketed all-reduces on the comm
stream → fused SGD) is captured once into a hipGraph and replayed, so the host
cost per step is one graph launch plus the learning-rate scalar update.

Rules this relies on (all ddpx ops follow them):
* no host synchronisation inside the step (loss stays on device, lr is read
  from a device scalar: ``SGD(capturable=True)``);
* inputs are copied into static buffers before each replay;
* every side stream (RCCL comm stream) forks from and joins back into the
  capturing stream through events.
"""
from __future__ import annotations

import torch


_UPLOAD_SIG = False


def _upload(graph):
    """Upload the instantiated executable now (csrc/kernels/graph_util.hip), not on its first replay: a graph
    first launched inside a timed region would otherwise pay the upload there.  Best effort."""
    global _UPLOAD_SIG
    import os
    if os.environ.get("DDPX_GRAPH_UPLOAD", "1") == "0":
        return
    try:
        from . import native
        if not _UPLOAD_SIG:
            native.register_kernel_sig("ddpx_graph_upload", native.c_int, native.c_void_p, native.c_void_p)
            _UPLOAD_SIG = True
        exec_ptr = graph.raw_cuda_graph_exec()
        if exec_ptr:
            native.kernels().ddpx_graph_upload(exec_ptr, native.stream_handle())
    except Exception:  # noqa: BLE001 - an older torch without raw_cuda_graph_exec(): upload on first launch
        pass


class CapturedStep:
    """Capture ``fn(x, y) -> loss`` into a graph; ``__call__`` replays it."""

    def __init__(self, fn, example_x: torch.Tensor, example_y: torch.Tensor, warmup: int = 0, pre_replay=None,
                 use_inputs_as_static: bool = False, comm=None):
        """``warmup`` extra eager calls run on a side stream first (they execute ``fn`` for real:
        in training they are real optimizer steps, so callers normally warm up with their own
        eager steps and pass 0).  Capture itself records without executing: call the object
        to run the captured step for the example batch."""
        self.fn = fn
        # communicator whose collectives the graph contains: its watchdog tracks every replay (a
        # collective captured in the graph is not seen by per-collective tracking) and its error state
        # is checked before each replay, so a timed-out step fails on the owning thread
        self.comm = comm
        # use_inputs_as_static: the caller writes every batch straight into these buffers
        self.static_x = example_x if use_inputs_as_static else example_x.clone()
        self.static_y = example_y if use_inputs_as_static else example_y.clone()
        self.pre_replay = pre_replay
        if warmup:
            s = torch.cuda.Stream()
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s):
                for _ in range(warmup):
                    if pre_replay is not None:
                        pre_replay()
                    self.fn(self.static_x, self.static_y)
            torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        if pre_replay is not None:
            pre_replay()
        with torch.cuda.graph(self.graph, capture_error_mode="thread_local"):
            self.static_loss = self.fn(self.static_x, self.static_y)
        _upload(self.graph)
        torch.cuda.synchronize()

    def load(self, x: torch.Tensor, y: torch.Tensor):
        if x.data_ptr() != self.static_x.data_ptr():
            self.static_x.copy_(x, non_blocking=True)
        if y.data_ptr() != self.static_y.data_ptr():
            self.static_y.copy_(y, non_blocking=True)

    def __call__(self, x: torch.Tensor | None = None, y: torch.Tensor | None = None):
        if x is not None:
            self.load(x, y)
        if self.pre_replay is not None:
            self.pre_replay()
        if self.comm is not None:
            self.comm.check()
        self.graph.replay()
        if self.comm is not None:
            self.comm.track(what="graph replay")
        return self.static_loss


class CapturedCycle:
    """A training step whose host-visible state alternates (a weight's bf16 copy ping-pongs between two buffers,
    ``FlatParams.enable_pingpong``): captured once per state, ``signature()`` telling them apart, until the state
    returns to the first one; replays cycle through the versions in capture order (period 1 for every other
    step).  All versions share the first one's static input buffers."""

    def __init__(self, fn, example_x, example_y, signature=None, max_period: int = 2, use_inputs_as_static=False,
                 comm=None):
        sig0 = signature() if signature is not None else None
        first = CapturedStep(fn, example_x, example_y, use_inputs_as_static=use_inputs_as_static, comm=comm)
        self.graphs = [first]
        while signature is not None and signature() != sig0:
            if len(self.graphs) >= max_period:
                raise RuntimeError(f"training-step state does not return to its start within {max_period} steps")
            self.graphs.append(CapturedStep(fn, first.static_x, first.static_y, use_inputs_as_static=True, comm=comm))
        self.static_x, self.static_y = first.static_x, first.static_y
        self.k = 0

    @property
    def period(self):
        return len(self.graphs)

    def load(self, x, y):
        self.graphs[0].load(x, y)

    def __call__(self, x=None, y=None):
        if x is not None:
            self.load(x, y)
        g = self.graphs[self.k % len(self.graphs)]
        self.k += 1
        return g()


def pingpong_signature_of(opt):
    flat = getattr(opt, "flat", None)
    return flat.pingpong_signature if flat is not None else None


def agree_all_ranks(ok: bool) -> bool:
    """True iff ``ok`` on every rank of the default c10d group (CPU tensors: the gloo group that carries the
    native communicator's bootstrap), or the local value without one."""
    import torch.distributed as dist
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return ok
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def step_state_snapshot(net, opt):
    """Host-side step bookkeeping a HIP-graph capture changes without running anything on the device."""
    flat = getattr(opt, "flat", None)
    return {"ddp": net.iteration_state() if hasattr(net, "iteration_state") else None,
            "step_count": getattr(opt, "step_count", None),
            "pingpong": flat.pingpong_signature() if flat is not None else None}


def restore_after_failed_capture(net, opt, snap):
    """Put the host bookkeeping back to where the last eager step left it after an aborted capture (nothing
    of it ran on the device): DDP bucket state, optimizer step count, a pending device-LR advance, and every
    derived weight copy the capture recorded (and marked current) but never produced."""
    torch.cuda.synchronize()
    if snap.get("ddp") is not None:
        net.restore_iteration_state(snap["ddp"])
    flat = getattr(opt, "flat", None)
    if flat is not None:
        flat.pending_lr = None
        flat.invalidate_derived()
        if snap.get("pingpong") is not None:
            flat.set_pingpong_signature(snap["pingpong"])  # (the aborted capture flipped copies it never wrote)
    if snap.get("step_count") is not None:
        opt.step_count = snap["step_count"]


def try_capture(fn, x, y, net, opt, comm=None, agree=agree_all_ranks):
    """``CapturedCycle(fn, x, y)`` if capture succeeds on EVERY rank, else None with the host state restored
    (every rank then steps eagerly: a graph replay on one rank and eager collectives on another would pair
    different collectives).  Returns (graph or None, error text or None)."""
    snap = step_state_snapshot(net, opt)
    g, err = None, None
    try:
        g = CapturedCycle(fn, x, y, signature=pingpong_signature_of(opt), comm=comm)
    except Exception as e:  # noqa: BLE001 - any capture failure falls back to eager steps
        err = f"{type(e).__name__}: {e}"
    if agree(g is not None):
        return g, None
    restore_after_failed_capture(net, opt, snap)
    return None, err or "graph capture failed on another rank"


class GraphedSteps:
    """Training steps: eager for the first ``eager_first`` (allocator / lazy-init warm-up), then replays of
    captured graphs — or, if capture fails on ANY rank, eager steps on every rank in the same process.

    ``eager_step()`` runs one step and returns its loss; ``make_graphs()`` captures and returns
    ``{steps_per_graph: callable}`` (each call replays that many steps and returns the last loss).  A
    failed capture is never retried and never restarts anything: the exception text is kept in
    ``graph_error``, ``on_fallback()`` (if given) resets whatever step state the aborted capture left
    half-done, and the loop continues eagerly.  ``agree(ok) -> bool`` turns one rank's capture outcome into
    the job's (all ranks must take the same path: a graph replay on one rank and eager collectives on
    another would pair different collectives); default: the local outcome.  ``after(m)`` is called after
    every ``m`` executed steps (host bookkeeping such as ``scheduler.step()``).
    """

    def __init__(self, eager_step, make_graphs, steps_per_graph: int = 1, use_graph: bool = True, eager_first: int = 2,
                 agree=None, on_fallback=None, after=None):
        self.eager_step = eager_step
        self.make_graphs = make_graphs
        self.S = max(1, int(steps_per_graph))
        self.use_graph = bool(use_graph)
        self.eager_first = eager_first
        self.agree = agree
        self.on_fallback = on_fallback
        self.after = after
        self.graphs = None
        self.graph_error = None

    def _capture(self):
        ok, err, graphs = True, None, None
        try:
            graphs = self.make_graphs()
        except Exception as e:  # noqa: BLE001 - any capture failure falls back to eager steps
            ok, err = False, f"{type(e).__name__}: {e}"
            import os
            if os.environ.get("DDPX_DEBUG_CAPTURE") == "1":
                import sys
                import traceback
                print(f"[ddpx] graph capture failed: {err}", file=sys.stderr, flush=True)
                traceback.print_exc()
        all_ok = self.agree(ok) if self.agree is not None else ok
        if all_ok:
            self.graphs = graphs
            return
        self.graphs = None
        self.use_graph = False
        self.graph_error = err or "graph capture failed on another rank"
        if self.on_fallback is not None:
            self.on_fallback()

    def run(self, k: int, n: int):
        """Steps k .. k+n-1; returns the last step's loss."""
        loss = None
        while n > 0:
            if self.use_graph and k >= self.eager_first and self.graphs is None:
                self._capture()
            if not self.use_graph or k < self.eager_first:
                loss = self.eager_step()
                m = 1
            else:
                m = self.S if (n >= self.S and self.S in self.graphs) else 1
                loss = self.graphs[m]()
            if self.after is not None:
                self.after(m)
            k += m
            n -= m
        return loss
