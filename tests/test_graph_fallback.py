"""bench.py's step loop must survive a failed HIP-graph capture (e.g. RCCL with real peers refusing
capture on the driver's 8-GPU node): every rank falls back to eager steps in the same process, agreed over
the CPU group, and the failure is reported instead of aborting the run (``ddpx.runtime.graphs.GraphedSteps``).
"""
import os
import sys

import torch
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from ddpx.runtime.graphs import GraphedSteps  # noqa: E402


def test_capture_failure_falls_back_to_eager():
    calls = {"eager": 0, "graph": 0, "reset": 0, "after": 0}

    def eager():
        calls["eager"] += 1
        return calls["eager"]

    def make_graphs():
        raise RuntimeError("hipErrorStreamCaptureUnsupported: operation not permitted when stream is capturing")

    def reset():
        calls["reset"] += 1

    def after(m):
        calls["after"] += m

    r = GraphedSteps(eager, make_graphs, steps_per_graph=4, on_fallback=reset, after=after)
    r.run(0, 3)
    r.run(3, 7)
    assert calls["eager"] == 10 and calls["after"] == 10 and calls["reset"] == 1
    assert not r.use_graph and "StreamCaptureUnsupported" in r.graph_error


def test_capture_success_replays_multi_step_graphs():
    seen = []

    def eager():
        seen.append("e")

    def make_graphs():
        return {1: lambda: seen.append("g1"), 4: lambda: seen.append("g4")}

    steps = []
    r = GraphedSteps(eager, make_graphs, steps_per_graph=4, after=steps.append)
    r.run(0, 11)
    # the run that captured replays the largest graph that fits (warming it), then greedily
    assert seen == ["e", "e", "g4", "g4", "g1"] and sum(steps) == 11 and r.graph_error is None
    assert r.warm == {1, 4}


def test_replay_schedule_short_windows_use_warm_graphs_only():
    r = GraphedSteps(lambda: None, lambda: {}, steps_per_graph=20)
    r.graphs = {1: None, 3: None, 20: None}
    assert r.schedule(3, capture_run=True) == [3]
    r.warm = {3}
    assert r.schedule(20) == [3] * 6 + [1] * 2  # the cold 20-step graph is not replayed in a short window
    assert r.schedule(200) == [20] * 10  # long window: the one-off first-replay cost is amortised
    r.warm = {3, 20}
    assert r.schedule(20) == [20]
    for n in range(1, 130):
        assert sum(r.schedule(n)) == n


def _rank(rank, world, port, q):
    import torch.distributed as dist
    from tests._dist_util import init_gloo
    init_gloo(rank, world, port)
    n_eager = [0]

    def eager():
        n_eager[0] += 1
        # a collective every step: ranks on different paths would pair it with a graph replay and hang
        t = torch.ones(1)
        dist.all_reduce(t)
        return float(t.item())

    def make_graphs():
        if rank == 1:
            raise RuntimeError("capture failed on rank 1 only")
        return {1: lambda: 0.0}

    def agree(ok):
        t = torch.tensor([1 if ok else 0])
        dist.all_reduce(t, op=dist.ReduceOp.MIN)
        return bool(t.item())

    r = GraphedSteps(eager, make_graphs, agree=agree)
    last = r.run(0, 6)
    q.put((rank, n_eager[0], last, r.use_graph, r.graph_error))
    dist.destroy_process_group()


def test_capture_failure_on_one_rank_moves_every_rank_to_eager():
    from tests._dist_util import free_port
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in ps)
    for rank, n_eager, last, use_graph, err in out:
        assert n_eager == 6 and last == float(world) and not use_graph, out
    assert "rank 1 only" in out[1][4] and "another rank" in out[0][4]
