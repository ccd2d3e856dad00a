"""Communication backends behind one small interface.

* :class:`RcclComm` — the MI355X path: a native RCCL communicator
  (``csrc/runtime/rccl_comm.cpp``) bootstrapped through the c10d TCPStore,
  with its own high-priority HIP stream and a timeout watchdog.  Collectives
  are issued on explicit streams, so they overlap compute and are captured
  by HIP graphs.
* :class:`TorchComm` — ``torch.distributed`` (gloo on CPU, used by the CPU
  test-suite; or stock ProcessGroupNCCL for A/B runs).

Reference equivalent: ``init_process_group(backend="nccl")`` at
``/root/reference/multigpu.py:32`` and the collectives DDP issues implicitly
(SURVEY §2.4 C0–C7).
"""
from __future__ import annotations

import itertools
import os

import torch
import torch.distributed as dist

from ..runtime import native

# RCCL enums (rccl.h)
NCCL_DTYPE = {
    torch.int64: 4,
    torch.float16: 6,
    torch.float32: 7,
    torch.float64: 8,
    torch.bfloat16: 9,
    torch.uint8: 1,
    torch.int32: 2,
}
NCCL_OP = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}

_uid_counter = itertools.count()


class CommError(RuntimeError):
    """A collective failed or timed out (watchdog), reported on the owning thread."""


class Comm:
    rank: int = 0
    world_size: int = 1
    native: bool = False
    supports_avg: bool = True

    def allreduce_(self, t: torch.Tensor, op: str = "avg", stream=None, async_op=False):
        raise NotImplementedError

    def broadcast_(self, t: torch.Tensor, src: int = 0, stream=None):
        raise NotImplementedError

    def reduce_scatter(self, out: torch.Tensor, inp: torch.Tensor, op: str = "avg", stream=None):
        raise NotImplementedError

    def allgather(self, out: torch.Tensor, inp: torch.Tensor, stream=None):
        raise NotImplementedError

    def barrier(self):
        if dist.is_initialized() and dist.get_world_size() > 1:
            dist.barrier()

    def all_gather_object(self, obj):
        if not dist.is_initialized() or dist.get_world_size() == 1:
            return [obj]
        out = [None] * dist.get_world_size()
        dist.all_gather_object(out, obj)
        return out

    def check(self):
        pass

    def track(self, stream=None, what: str = "graph replay"):
        pass

    def close(self, abort=False):
        pass


class TorchComm(Comm):
    """torch.distributed-backed collectives (gloo for CPU tensors, nccl for GPU)."""

    def __init__(self, group=None):
        if not dist.is_initialized():
            raise RuntimeError("TorchComm requires torch.distributed to be initialised")
        self.group = group
        self.rank = dist.get_rank(group)
        self.world_size = dist.get_world_size(group)
        self.native = False

    def _avg_ok(self, t):
        return t.is_cuda and dist.get_backend(self.group) in ("nccl", "cpu:gloo,cuda:nccl")

    def allreduce_(self, t, op="avg", stream=None, async_op=False):
        if self.world_size == 1:
            return None
        if op == "avg" and not self._avg_ok(t):
            work = dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group, async_op=async_op)
            if async_op:
                return _ScaleOnWait(work, t, 1.0 / self.world_size)
            t.div_(self.world_size)
            return None
        rop = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.AVG, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN}[op]
        return dist.all_reduce(t, op=rop, group=self.group, async_op=async_op)

    def broadcast_(self, t, src=0, stream=None):
        if self.world_size > 1:
            dist.broadcast(t, src=src, group=self.group)

    def reduce_scatter(self, out, inp, op="avg", stream=None):
        if self.world_size == 1:
            out.copy_(inp)
            return
        chunks = list(inp.chunk(self.world_size))
        if inp.is_cuda:
            dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=self.group)
        else:  # gloo has no reduce_scatter: all-reduce then slice
            tmp = inp.clone()
            dist.all_reduce(tmp, group=self.group)
            out.copy_(tmp.chunk(self.world_size)[self.rank])
        del chunks
        if op == "avg":
            out.div_(self.world_size)

    def allgather(self, out, inp, stream=None):
        if self.world_size == 1:
            out.copy_(inp)
            return
        if inp.is_cuda:
            dist.all_gather_into_tensor(out, inp, group=self.group)
        else:  # inp may alias its own chunk of out (in-place gather): send a copy
            dist.all_gather(list(out.chunk(self.world_size)), inp.clone(), group=self.group)


class HostStagedComm(TorchComm):
    """GPU tensors reduced through a CPU gloo group (synchronous, staged in fp32 host copies).

    Not a production path: RCCL refuses two ranks on one device, so this is how several ranks
    sharing ONE MI355X exercise the multi-rank DDP / ZeRO-1 logic together with the native
    kernels (``tests/test_gpu_multirank.py``, ``bench.py --comm host``).  Not graph-capturable.
    """

    def __init__(self, group=None):
        super().__init__(group)

    def _host(self, t):
        return t.detach().to("cpu", torch.float32 if t.is_floating_point() else t.dtype, copy=True)

    def allreduce_(self, t, op="avg", stream=None, async_op=False):
        if self.world_size == 1:
            return None
        h = self._host(t)
        rop = {"sum": dist.ReduceOp.SUM, "avg": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX,
               "min": dist.ReduceOp.MIN}[op]
        dist.all_reduce(h, op=rop, group=self.group)
        if op == "avg":
            h.div_(self.world_size)
        t.copy_(h)
        return None

    def broadcast_(self, t, src=0, stream=None):
        if self.world_size > 1:
            h = self._host(t)
            dist.broadcast(h, src=src, group=self.group)
            t.copy_(h)

    def reduce_scatter(self, out, inp, op="avg", stream=None):
        h = self._host(inp)
        if self.world_size > 1:
            dist.all_reduce(h, group=self.group)
        r = h.chunk(self.world_size)[self.rank]
        if op == "avg":
            r = r / self.world_size
        out.copy_(r)

    def allgather(self, out, inp, stream=None):
        h = self._host(inp)
        parts = [torch.empty_like(h) for _ in range(self.world_size)]
        dist.all_gather(parts, h, group=self.group)
        out.copy_(torch.cat(parts))


class _ScaleOnWait:
    def __init__(self, work, t, s):
        self.work, self.t, self.s = work, t, s

    def wait(self):
        self.work.wait()
        self.t.mul_(self.s)


def parse_channels(spec):
    """None / "" / 0 -> None; N or "N" -> (N, N); (a, b) or "a:b" -> (a, b) (0 = RCCL's bound)."""
    if spec is None or spec == "" or spec == 0:
        return None
    if isinstance(spec, str):
        parts = [int(v) for v in spec.split(":")]
        spec = parts[0] if len(parts) == 1 else tuple(parts)
    if isinstance(spec, int):
        spec = (spec, spec)
    lo, hi = (int(spec[0]), int(spec[1]))
    if lo < 0 or hi < 0 or (hi and lo > hi):
        raise ValueError(f"bad RCCL channel bounds {spec!r}")
    return (lo, hi) if (lo or hi) else None


def set_rccl_protocol(proto):
    """RCCL reads ``NCCL_PROTO`` once per process (Simple | LL | LL128, or a comma list): set it before the first
    communicator.  None leaves RCCL's own per-size choice."""
    if proto:
        os.environ["NCCL_PROTO"] = str(proto)


class RcclComm(Comm):
    """Native RCCL communicator for one process per MI355X."""

    def __init__(self, device: torch.device, timeout_s: float | None = None, high_priority: bool = True,
                 channels=None, sim_world: int | None = None):
        """``channels``: None (RCCL's choice), N, or (min, max) channel / CTA bounds for THIS communicator
        (``ncclConfig_t.minCTAs/maxCTAs``); default from ``DDPX_RCCL_CHANNELS`` ("N" or "MIN:MAX").  The
        protocol is process-wide in RCCL: set ``NCCL_PROTO`` (``--rccl_proto``) before the first communicator.

        ``sim_world`` (diagnostics, ``bench.py --ddp_single --sim_world N``): a one-process job that PRESENTS world
        size N, rank 0, to DDP — the N-rank bucket plan, ZeRO-1 shards of 1/N, the deferred gathers and this rank's
        1/N optimizer stream are built and run exactly as on rank 0 of N ranks — while the communicator itself has
        one rank: every collective DDP issues is then the in-place identity and is skipped
        (``DDPX_COMM_SKIP_IDENTITY=1``), so a step times the per-rank compute of an N-GPU job without its wire
        time.  Not a training mode: the gradients are this rank's own, not averages."""
        if not dist.is_initialized():
            raise RuntimeError("RcclComm bootstraps through the default c10d store: init_process_group first")
        self.channels = parse_channels(os.environ.get("DDPX_RCCL_CHANNELS") if channels is None else channels)
        rt = native.runtime()
        self.rank = dist.get_rank()
        self.world_size = dist.get_world_size()
        nranks = self.world_size
        self.sim_world = None
        if sim_world is not None and int(sim_world) > 1:
            if self.world_size != 1:
                raise ValueError("sim_world needs a one-process job")
            if os.environ.get("DDPX_COMM_SKIP_IDENTITY") != "1":
                raise ValueError("sim_world needs DDPX_COMM_SKIP_IDENTITY=1 (collectives must not run)")
            self.sim_world = int(sim_world)
            self.world_size = self.sim_world
        self.device = torch.device(device)
        self.native = True
        store = dist.distributed_c10d._get_default_store()
        key = f"ddpx/rccl_uid/{next(_uid_counter)}"
        if self.rank == 0:
            uid = (native.ctypes.c_char * 128)()
            native.check(rt.ddpx_comm_unique_id(uid, 128), "ncclGetUniqueId")
            store.set(key, bytes(uid))
        uid = store.get(key)
        if timeout_s is None:
            timeout_s = float(os.environ.get("DDPX_COMM_TIMEOUT", "600"))
        err = native.ctypes.c_int(0)
        torch.cuda.set_device(self.device)
        lo, hi = self.channels or (0, 0)
        self.handle = rt.ddpx_comm_create2(uid, nranks, self.rank, self.device.index or 0,
                                           int(high_priority), float(timeout_s), lo, hi, native.ctypes.byref(err))
        if not self.handle:
            raise RuntimeError(f"ncclCommInitRank failed (code {err.value})")
        self._rt = rt
        self.stream = torch.cuda.ExternalStream(rt.ddpx_comm_stream(self.handle), device=self.device)
        # captured steps fork onto this stream: a failed capture joins it back / renews it, and the capture-leak
        # check covers it (ddpx.runtime.graphs)
        from ..runtime.graphs import register_side_stream
        self._side_name = f"RCCL comm stream #{id(self)}"
        register_side_stream(self, self._side_name, renew=RcclComm.renew_stream, attr="stream")

    def renew_stream(self):
        """Swap in a fresh communicator stream (the old one was left unusable by a failed capture)."""
        native.check(self._rt.ddpx_comm_renew_stream(self.handle), "ddpx_comm_renew_stream")
        self.stream = torch.cuda.ExternalStream(self._rt.ddpx_comm_stream(self.handle), device=self.device)

    def _s(self, stream):
        return native.stream_handle(stream) if stream is not None else native.stream_handle()

    def _dt(self, t):
        try:
            return NCCL_DTYPE[t.dtype]
        except KeyError:
            raise TypeError(f"RCCL: unsupported dtype {t.dtype}") from None

    def allreduce_(self, t, op="avg", stream=None, async_op=False):
        if not t.is_contiguous():
            raise ValueError("allreduce_: tensor must be contiguous")
        rc = self._rt.ddpx_comm_allreduce(self.handle, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t),
                                          NCCL_OP[op], self._s(stream))
        native.check(rc, "ncclAllReduce")
        return None

    def broadcast_(self, t, src=0, stream=None):
        if not t.is_contiguous():
            raise ValueError("broadcast_: tensor must be contiguous")
        rc = self._rt.ddpx_comm_broadcast(self.handle, t.data_ptr(), t.data_ptr(), t.numel(), self._dt(t), src,
                                          self._s(stream))
        native.check(rc, "ncclBroadcast")

    def reduce_scatter(self, out, inp, op="avg", stream=None):
        rc = self._rt.ddpx_comm_reduce_scatter(self.handle, inp.data_ptr(), out.data_ptr(), out.numel(),
                                               self._dt(inp), NCCL_OP[op], self._s(stream))
        native.check(rc, "ncclReduceScatter")

    def allgather(self, out, inp, stream=None):
        rc = self._rt.ddpx_comm_allgather(self.handle, inp.data_ptr(), out.data_ptr(), inp.numel(), self._dt(inp),
                                          self._s(stream))
        native.check(rc, "ncclAllGather")

    TIMEOUT_ACTIONS = {"raise": 0, "abort": 1, "exit": 2}

    def check(self):
        e = self._rt.ddpx_comm_error(self.handle)
        if e:
            raise CommError(f"[rank {self.rank}] " + {1: "RCCL asynchronous error", 2: "RCCL collective timed out",
                                                      3: "RCCL communicator aborted",
                                                      4: "RCCL abort escalated: a collective call is stuck inside "
                                                         "RCCL, the process exits with code 3"
                                                      }.get(e, f"RCCL error {e}"))

    def track(self, stream=None, what: str = "graph replay"):
        """Register everything enqueued on ``stream`` so far with the watchdog (call after each graph
        replay: collectives captured in a graph are invisible to per-collective tracking)."""
        rc = self._rt.ddpx_comm_track(self.handle, self._s(stream), what.encode())
        if rc:
            self.check()

    def tracked(self) -> int:
        return int(self._rt.ddpx_comm_tracked(self.handle))

    def set_timeout(self, timeout_s: float, action: str | None = None):
        self._rt.ddpx_comm_set_timeout(self.handle, float(timeout_s),
                                       -1 if action is None else self.TIMEOUT_ACTIONS[action])

    def close(self, abort=False):
        if getattr(self, "handle", None):
            from ..runtime.graphs import unregister_side_stream
            unregister_side_stream(self._side_name)
            self._rt.ddpx_comm_destroy(self.handle, int(abort))
            self.handle = None


def default_comm(device: torch.device | None = None) -> Comm:
    """RcclComm for GPU tensors (DDPX_COMM=torch: torch.distributed; DDPX_COMM=host: gloo-staged), TorchComm
    otherwise."""
    kind = os.environ.get("DDPX_COMM", "rccl")
    if device is not None and torch.device(device).type == "cuda":
        if kind == "rccl":
            return RcclComm(device)
        if kind == "host":
            return HostStagedComm()
    return TorchComm()
