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

import os
import weakref

import torch


_UPLOAD_SIG = False
_CAPTURE_SIG = False


class CaptureLeak(RuntimeError):
    """A stream is still capturing (or stuck "invalidated") after a capture ended: any later synchronous copy
    on it would fail with hipErrorStreamCaptureUnsupported, and kernels issued on it would be recorded instead
    of executed.  Raised instead of continuing silently (profiles/r5_capture/NOTES.md)."""


# ---------------------------------------------------------------- capture status of arbitrary streams
_STATUS = {0: "none", 1: "active", 2: "invalidated"}


def _capture_native():
    global _CAPTURE_SIG
    from . import native
    if not _CAPTURE_SIG:
        native.register_kernel_sig("ddpx_stream_capture_info", native.c_int, native.c_void_p,
                                   native.ctypes.POINTER(native.c_int), native.ctypes.POINTER(native.c_uint64))
        native.register_kernel_sig("ddpx_stream_end_capture_discard", native.c_int, native.c_void_p)
        native.register_kernel_sig("ddpx_stream_force_reset", native.c_int, native.c_void_p)
        _CAPTURE_SIG = True
    return native


def stream_capture_info(stream) -> tuple[str, int]:
    """(status, capture id) of ``stream`` (a torch stream): status none / active / invalidated."""
    native = _capture_native()
    st, cid = native.c_int(0), native.c_uint64(0)
    rc = native.kernels().ddpx_stream_capture_info(stream.cuda_stream, native.ctypes.byref(st),
                                                    native.ctypes.byref(cid))
    if rc != 0:
        raise RuntimeError(f"hipStreamGetCaptureInfo failed with code {rc}")
    return _STATUS.get(st.value, str(st.value)), int(cid.value)


def stream_capture_status(stream) -> str:
    return stream_capture_info(stream)[0]


# Side streams a captured step may fork onto (the RCCL communicator's stream, a prefetch stream): the capture
# joins them back if a failure left them forked, and the leak check covers them.  name -> (getter, renew):
# getter() returns the stream now (None once its owner is gone); renew() replaces a stream that a failed capture
# left unusable, or is None.
_SIDE: dict = {}


def register_side_stream(stream_or_owner, name: str, renew=None, attr: str | None = None):
    """Register a side stream by object, or by (owner, attribute) so a renewed stream is followed; the owner
    is held weakly."""
    if attr is None:
        s = stream_or_owner
        _SIDE[name] = (lambda: s, renew)
    else:
        ref = weakref.ref(stream_or_owner)

        def get():
            o = ref()
            return getattr(o, attr, None) if o is not None else None

        def ren():
            o = ref()
            if o is not None and renew is not None:
                renew(o)
        _SIDE[name] = (get, ren if renew is not None else None)


def unregister_side_stream(name: str):
    _SIDE.pop(name, None)


def _side_streams():
    out = []
    for name, (get, renew) in list(_SIDE.items()):
        s = get()
        if s is None:
            _SIDE.pop(name, None)
            continue
        out.append((name, s, renew))
    return out


_CAP_STREAM = None


def _capture_stream():
    global _CAP_STREAM
    if _CAP_STREAM is None:
        _CAP_STREAM = torch.cuda.Stream()
    return _CAP_STREAM


def _join_into(cap, cid):
    """Join every registered side stream that is part of capture ``cid`` back into ``cap`` (what the body did
    not get to, e.g. because it raised between a fork and its join)."""
    joined = []
    for name, s, _ in _side_streams():
        if s == cap:
            continue
        st, sid = stream_capture_info(s)
        if st == "active" and sid == cid:
            ev = torch.cuda.Event()
            ev.record(s)
            cap.wait_event(ev)
            joined.append(name)
    return joined


def _abort_capture(graph, cap):
    """End a capture whose body or end failed, leaving no stream capturing; retire streams it left unusable."""
    global _CAP_STREAM
    native = _capture_native()
    st, cid = stream_capture_info(cap)
    ended = False
    if st == "active":
        _join_into(cap, cid)
        try:
            graph.capture_end()  # also ends torch's allocation routing into the graph's private pool
            ended = True
        except Exception:  # noqa: BLE001 - invalidated: ended below
            pass
    if not ended:
        try:  # capture_end raised before it stopped routing this stream's allocations into the graph's pool
            torch._C._cuda_endAllocateToPool(cap.device.index, graph.pool())
        except Exception:  # noqa: BLE001
            pass
        if stream_capture_status(cap) != "none":
            native.kernels().ddpx_stream_end_capture_discard(cap.cuda_stream)
    try:
        graph.reset()
    except Exception:  # noqa: BLE001
        pass
    if stream_capture_status(cap) != "none":
        native.kernels().ddpx_stream_force_reset(cap.cuda_stream)
        if stream_capture_status(cap) != "none":
            _CAP_STREAM = None  # never capture on it again: the next capture gets a fresh stream
    for name, s, renew in _side_streams():
        # a side stream of an invalidated capture stays "active" after the origin's end; one of an aborted
        # capture may read "invalidated": both are brought back to "none", or the stream is replaced
        if stream_capture_status(s) != "none":
            native.kernels().ddpx_stream_force_reset(s.cuda_stream)
        if stream_capture_status(s) != "none" and renew is not None:
            torch.cuda.synchronize()
            renew()


def capture_step(graph, fn):
    """Capture ``fn()`` into ``graph`` (thread-local mode) and return its result; the replacement of
    ``with torch.cuda.graph(graph)`` for every captured training step.

    torch's context manager does not end a capture cleanly on failure: when ``capture_end`` raises (an unjoined
    side stream, an invalidated capture) it skips restoring the current stream, so the thread keeps issuing work
    to a stream that is still capturing (ROCm 7 leaves an unjoined capture active on both streams), and an
    "eager" fallback step is silently recorded instead of run, until the next synchronous copy fails with
    hipErrorStreamCaptureUnsupported (profiles/r4_flaky, profiles/r5_capture/NOTES.md).  Here, on any
    failure: forked side streams are joined back, the capture is ended and discarded, streams left unusable are
    retired / renewed, the current stream is always restored, and the failure is re-raised."""
    cap = _capture_stream()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    with torch.cuda.stream(cap):
        graph.capture_begin(capture_error_mode="thread_local")
        try:
            out = fn()
        except BaseException:
            _abort_capture(graph, cap)
            raise
        try:
            # a side stream the body forked and never joined back would make the end fail AND leave both
            # streams capturing for good (ROCm 7: a second end is refused, WrongThread): join every side stream
            # that took part first.  HIP reports a side stream as part of the capture whether or not its last
            # nodes were already joined, so this cannot tell a missing join from a done one (an extra edge to
            # already-joined nodes is free); DDPX_CAPTURE_DEBUG=1 names the streams.
            late = _join_into(cap, stream_capture_info(cap)[1])
            if late and os.environ.get("DDPX_CAPTURE_DEBUG", "0") == "1":
                _warn_once(f"capture_step: joined side stream(s) that took part in the capture: {late}")
            graph.capture_end()
        except BaseException:
            _abort_capture(graph, cap)
            raise
    return out


_WARNED = set()


def _warn_once(msg):
    if msg not in _WARNED:
        _WARNED.add(msg)
        import warnings
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def assert_no_capture(where: str, extra=()):
    """Raise :class:`CaptureLeak` if the current stream, the capture stream or any registered side stream is
    not in the capture status "none" (call between calibration trials, before building a timed engine, and
    after a capture fallback)."""
    if not torch.cuda.is_available() or not torch.cuda.is_initialized():
        return
    streams = [("current stream", torch.cuda.current_stream(), None)]
    if _CAP_STREAM is not None:
        streams.append(("capture stream", _CAP_STREAM, None))
    streams += _side_streams()
    streams += [(n, s, None) for n, s in extra]
    bad = []
    for name, s, _ in streams:
        st = stream_capture_status(s)
        if st != "none":
            bad.append(f"{name} (0x{s.cuda_stream:x}) is {st}")
    if bad:
        raise CaptureLeak(f"{where}: " + "; ".join(bad))


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
        self.static_loss = capture_step(self.graph, lambda: self.fn(self.static_x, self.static_y))
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
        # host-visible state after each version (its capture advanced the host bookkeeping exactly as a replay
        # advances the device): every replay puts the host back in step with the device, so an eager step after
        # an odd number of replays reads the bf16 copy the last replay wrote
        self.post = [signature() if signature is not None else None]
        while signature is not None and signature() != sig0:
            if len(self.graphs) >= max_period:
                raise RuntimeError(f"training-step state does not return to its start within {max_period} steps")
            self.graphs.append(CapturedStep(fn, first.static_x, first.static_y, use_inputs_as_static=True, comm=comm))
            self.post.append(signature())
        owner = getattr(signature, "__self__", None)
        self._set_sig = getattr(owner, "set_pingpong_signature", None) if len(self.graphs) > 1 else None
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
        i = self.k % len(self.graphs)
        self.k += 1
        out = self.graphs[i]()
        if self._set_sig is not None:
            self._set_sig(self.post[i])
        return out


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
    assert_no_capture("after a failed step capture")
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
        self.warm = set()  # graph sizes replayed at least once
        self._fresh = False
        import os
        # windows this long may replay a graph for the first time (DDPX_GRAPH_COLD_OK=1: any window, as before r5)
        self.cold_ok = int(os.environ.get("DDPX_GRAPH_COLD_OK", "100"))

    def capture_now(self):
        """Capture at once (after the eager steps; normally done lazily by run()): lets a caller put unrelated GPU
        work between the capture and the replays that follow it."""
        if self.use_graph and self.graphs is None:
            self._capture()

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
            self._fresh = True  # the next run() warms the largest graph that fits it
            return
        self.graphs = None
        self.use_graph = False
        self.graph_error = err or "graph capture failed on another rank"
        if self.on_fallback is not None:
            self.on_fallback()
        # the eager steps that follow must run, not be recorded into a capture the failure left open
        assert_no_capture("after a failed step capture")

    def schedule(self, n: int, capture_run: bool = False):
        """Graph sizes replayed for n consecutive steps (largest first).

        The first replay of a freshly captured graph runs slower on the GPU than every later one (the 20-step
        graph's first replay cost ~0.4 ms more: the driver's 20-step window ran at 0.2546 ms/step against 0.2347 with
        warm graphs in one process, profiles/r5_window).  So a short window replays only graphs that have already
        run once (the run that captured warms the largest graph fitting its remaining steps), and cold graphs are
        used only in windows of ``cold_ok`` steps or more, where that one-off cost is amortised."""
        sizes = sorted(self.graphs) if self.graphs else [1]
        if capture_run or n >= self.cold_ok:
            pool = sizes
        else:
            pool = sorted({1} | {s for s in sizes if s in self.warm})
        out = []
        while n > 0:
            m = max(s for s in pool if s <= n)
            out.append(m)
            n -= m
        return out

    def run(self, k: int, n: int):
        """Steps k .. k+n-1; returns the last step's loss."""
        loss = None
        plan = None
        while n > 0:
            if self.use_graph and k >= self.eager_first and self.graphs is None:
                self._capture()
            if not self.use_graph or k < self.eager_first:
                loss = self.eager_step()
                m = 1
            else:
                if plan is None:
                    plan = self.schedule(n, capture_run=self._fresh)
                    self._fresh = False
                m = plan.pop(0) if plan else 1
                loss = self.graphs[m]()
                self.warm.add(m)
            if self.after is not None:
                self.after(m)
            k += m
            n -= m
        return loss
