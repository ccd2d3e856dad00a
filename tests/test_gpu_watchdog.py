"""RCCL watchdog on graph-replayed collectives (ProcessGroupNCCL's watchdog, implied by
``init_process_group(backend="nccl")`` at /root/reference/multigpu.py:32).

A HIP graph is captured whose RCCL stream first runs a kernel that waits on a host-mapped flag (standing
in for a peer that never arrives), then an all-reduce.  Nothing of the replay can complete, so the
watchdog must report the timeout from the event it tracks per replay — collectives inside a graph are
invisible to per-collective tracking.  The waiting kernel is bounded (``ddpx_debug_spin_wait`` gives up
after 60 s) and every test releases the flag before it ends, so the GPU is idle afterwards.
"""
import os
import subprocess
import sys
import textwrap
import time

import pytest
import torch

from tests._dist_util import free_port

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


class HostFlag:
    def __init__(self):
        from ddpx.runtime import native
        self.rt = native.runtime()
        h, d = native.ctypes.c_void_p(), native.ctypes.c_void_p()
        native.check(self.rt.ddpx_hostflag_create(native.ctypes.byref(h), native.ctypes.byref(d)), "hostflag")
        self.host, self.dev = h.value, d.value

    def set(self, v=1):
        self.rt.ddpx_hostflag_set(self.host, v)

    def close(self):
        self.rt.ddpx_hostflag_destroy(self.host)


def _stalled_step(comm, flag, status, x):
    """Step body: fork the RCCL stream, wait on the flag there, all-reduce, join."""
    from ddpx.runtime import native

    def body(_x, _y):
        cur = torch.cuda.current_stream()
        ev = torch.cuda.Event()
        ev.record(cur)
        comm.stream.wait_event(ev)
        native.check(native.kernels().ddpx_debug_spin_wait(flag.dev, 1, 60.0, status.data_ptr(),
                                                           comm.stream.cuda_stream), "spin_wait")
        comm.allreduce_(x, "sum", stream=comm.stream)
        done = torch.cuda.Event()
        done.record(comm.stream)
        cur.wait_event(done)
        return x.sum()
    return body


def _timeout_case():
    from ddpx.parallel.comm import CommError, RcclComm
    from ddpx.runtime.graphs import CapturedStep
    gpu = torch.device("cuda", 0)
    comm = RcclComm(gpu, timeout_s=2.0)
    comm.set_timeout(2.0, "raise")
    flag = HostFlag()
    status = torch.zeros(1, dtype=torch.int32, device=gpu)
    x = torch.ones(4096, device=gpu)
    dummy = torch.zeros(1, device=gpu)
    try:
        flag.set(1)  # capture records without executing; the flag only matters at replay
        g = CapturedStep(_stalled_step(comm, flag, status, x), dummy, dummy, use_inputs_as_static=True, comm=comm)
        flag.set(0)
        n0 = comm.tracked()
        g()  # the replay is enqueued and tracked; it cannot finish while the flag is 0
        assert comm.tracked() == n0 + 1
        t0 = time.time()
        with pytest.raises(CommError, match="timed out"):
            while time.time() - t0 < 20.0:
                comm.check()
                time.sleep(0.05)
        waited = time.time() - t0
        assert 1.5 < waited < 10.0, waited
        with pytest.raises(CommError):  # a failed communicator refuses further replays
            g()
    finally:
        flag.set(1)  # release the stalled stream: the spin kernel exits, the all-reduce runs
        torch.cuda.synchronize()
        flag.close()
    assert status.item() == 1  # the kernel saw the flag (did not give up on its own bound)
    assert torch.equal(x, torch.ones_like(x))  # ws=1 sum is the identity
    comm.close()


def _healthy_case():
    from ddpx.parallel.comm import RcclComm
    from ddpx.runtime.graphs import CapturedStep
    gpu = torch.device("cuda", 0)
    comm = RcclComm(gpu, timeout_s=2.0)
    comm.set_timeout(2.0, "raise")
    flag = HostFlag()
    flag.set(1)
    status = torch.zeros(1, dtype=torch.int32, device=gpu)
    x = torch.ones(4096, device=gpu)
    dummy = torch.zeros(1, device=gpu)
    g = CapturedStep(_stalled_step(comm, flag, status, x), dummy, dummy, use_inputs_as_static=True, comm=comm)
    for _ in range(20):
        g()
    torch.cuda.synchronize()
    time.sleep(2.5)  # past the timeout: completed replays must not be reported
    comm.check()
    flag.close()
    comm.close()


_CASE_SCRIPT = textwrap.dedent("""
    import os, sys
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=0, world_size=1)
    import tests.test_gpu_watchdog as t
    getattr(t, {case!r})()
    dist.destroy_process_group()
    print("CASE OK", flush=True)
""")


def _run_case(case):
    """Each case in a process of its own: they drive RCCL communicators into timeouts / aborts, which must
    not share a process with the rest of the suite (an aborted communicator's leftovers broke a later
    one only when ~660 tests had run before it in the same process)."""
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), PYTHONPATH=ROOT)
    r = subprocess.run([sys.executable, "-c", _CASE_SCRIPT.format(root=ROOT, case=case)], env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, errors="replace", timeout=90)
    assert r.returncode == 0 and "CASE OK" in r.stdout, (r.returncode, r.stdout[-2000:], r.stderr[-3000:])


def test_watchdog_reports_timeout_of_graph_replayed_collective(gpu):
    _run_case("_timeout_case")


def test_healthy_replays_do_not_time_out(gpu):
    _run_case("_healthy_case")


_EXIT_SCRIPT = textwrap.dedent("""
    import os, sys, threading, time
    sys.path.insert(0, {root!r})
    import torch, torch.distributed as dist
    from tests.test_gpu_watchdog import HostFlag, _stalled_step
    from ddpx.parallel.comm import RcclComm
    from ddpx.runtime.graphs import CapturedStep
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=0, world_size=1)
    comm = RcclComm(dev)  # DDPX_COMM_TIMEOUT / _ACTION / _EXIT_GRACE_S from the environment
    flag = HostFlag(); flag.set(1)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    x = torch.ones(1024, device=dev); dummy = torch.zeros(1, device=dev)
    g = CapturedStep(_stalled_step(comm, flag, status, x), dummy, dummy, use_inputs_as_static=True, comm=comm)
    flag.set(0)
    g()
    def release():  # keep the GPU clean: free the stalled stream once the watchdog has fired
        while comm._rt.ddpx_comm_error(comm.handle) == 0:
            time.sleep(0.05)
        flag.set(1)
    threading.Thread(target=release, daemon=True).start()
    print("replayed", flush=True)
    time.sleep(60)  # the owning thread is busy elsewhere: the watchdog must end the process
    print("still alive", flush=True)
""")


def test_watchdog_terminates_process_on_timeout(gpu):
    env = dict(os.environ, DDPX_COMM_TIMEOUT="2", DDPX_COMM_TIMEOUT_ACTION="exit", DDPX_COMM_EXIT_GRACE_S="2",
               MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), PYTHONPATH=ROOT)
    t0 = time.time()
    r = subprocess.run([sys.executable, "-c", _EXIT_SCRIPT.format(root=ROOT)], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.PIPE, text=True, errors="replace", timeout=90)
    dt = time.time() - t0
    assert r.returncode == 3, (r.returncode, r.stdout[-2000:], r.stderr[-2000:])
    assert "replayed" in r.stdout and "still alive" not in r.stdout
    assert "[ddpx rank 0] collective 'graph replay' timed out" in r.stderr, r.stderr[-2000:]
    assert "terminating (exit code 3)" in r.stderr
    assert dt < 60, dt
