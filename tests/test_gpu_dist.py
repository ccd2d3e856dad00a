"""Native RCCL communicator + C++ reducer on one MI355X (world size 1), incl. HIP-graph capture.

Multi-rank RCCL needs distinct GPUs; the multi-rank reducer logic is covered on CPU/gloo
(test_ddp_cpu.py) — here the native pieces (uid exchange through the store, RCCL calls on the
comm stream, event fork/join, capture of collectives) run for real.
"""
import os

import pytest
import torch
import torch.distributed as dist

from tests._dist_util import free_port

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def pg(gpu):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(free_port())
    dist.init_process_group("gloo", rank=0, world_size=1)
    yield
    dist.destroy_process_group()


@pytest.mark.parametrize("channels", [None, "2:8", 16])
def test_rccl_collectives(gpu, pg, channels):
    from ddpx.parallel.comm import RcclComm
    c = RcclComm(gpu, channels=channels)  # explicit bounds: ncclCommInitRankConfig (minCTAs / maxCTAs)
    x = torch.randn(1000, device=gpu)
    y = x.clone()
    c.allreduce_(y, "avg")
    c.allreduce_(y, "sum")
    c.broadcast_(y, 0)
    torch.cuda.synchronize()
    assert torch.equal(x, y)
    out = torch.empty_like(x)
    c.reduce_scatter(out, x, "sum")
    c.allgather(y, out)
    torch.cuda.synchronize()
    assert torch.equal(y, x)
    b = torch.randn(77, device=gpu).to(torch.bfloat16)
    b2 = b.clone()
    c.allreduce_(b2, "avg")
    torch.cuda.synchronize()
    assert torch.equal(b, b2)
    c.check()
    c.close()


@pytest.mark.parametrize("overlap,shard,side", [(False, False, False), (True, False, False), (False, True, False),
                                               (True, True, False), (True, True, True)])
def test_native_reducer_ddp_matches_plain(gpu, pg, overlap, shard, side):
    import ddpx
    from ddpx.models import MLP
    from ddpx.optim.sgd import SGD
    from ddpx.parallel.comm import RcclComm
    from ddpx.parallel.ddp import DistributedDataParallel
    torch.manual_seed(0)
    a, b = MLP(hidden=512), MLP(hidden=512)
    b.load_state_dict(a.state_dict())
    ddpx.prepare_model(a, gpu)
    ddpx.prepare_model(b, gpu)
    comm = RcclComm(gpu)
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    da = DistributedDataParallel(a, comm=comm, bucket_cap_mb=1.0, first_bucket_mb=0.25, reduce_single=True,
                                 overlap_optimizer=overlap, shard_optimizer=shard, comm_side_optimizer=side)
    assert len(da.bucket_ranges) >= 2
    if shard:  # native MLP weights are shadow-only: reduce-scatter + bf16 shadow gather, biases replicated
        assert da.sharded and da.gather_what == "shadow" and da.bucket_modes[-1] == 0
        assert oa.bucket_source is da
    if overlap:
        da.attach_optimizer(oa)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    x = torch.rand(256, 3072, device=gpu).to(torch.bfloat16)
    t = torch.randint(0, 10, (256,), device=gpu)
    for _ in range(3):
        for net, opt in ((da, oa), (b, ob)):
            opt.zero_grad()
            loss, _ = net.forward_loss(x, t)
            loss.backward()
            opt.step()
    torch.cuda.synchronize()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
    da.close()
    comm.close()


@pytest.mark.parametrize("shard,chunk_mb,defer,side", [(False, None, False, False), (True, None, False, False),
                                                       (True, 0.25, True, False), (False, 0.25, False, False),
                                                       (True, None, True, True), (True, None, False, True)])
def test_graph_capture_with_rccl(gpu, pg, shard, chunk_mb, defer, side):
    """Whole step (fwd, bwd with bucketed all-reduce on the comm stream, SGD) in one HIP graph."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.optim.sgd import SGD
    from ddpx.parallel.comm import RcclComm
    from ddpx.parallel.ddp import DistributedDataParallel
    from ddpx.runtime.graphs import CapturedStep
    torch.manual_seed(1)
    a, b = MLP(hidden=512), MLP(hidden=512)
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        ddpx.prepare_model(m, gpu)
    comm = RcclComm(gpu)
    da = DistributedDataParallel(a, comm=comm, bucket_cap_mb=1.0, first_bucket_mb=0.25, reduce_single=True,
                                 shard_optimizer=shard, chunk_mb=chunk_mb, defer_gather=defer,
                                 comm_side_optimizer=side)
    assert (da.optimizer_stream() is not None) == side
    if chunk_mb:
        assert da.chunk_bucket
    assert da.defer_gather == defer
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, capturable=True)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    xs = [torch.rand(128, 3072, device=gpu).to(torch.bfloat16) for _ in range(4)]
    ts = [torch.randint(0, 10, (128,), device=gpu) for _ in range(4)]

    def body(x, y):
        oa.zero_grad()
        loss, _ = da.forward_loss(x, y)
        loss.backward()
        oa.step()
        return loss

    oa.sync_lr()
    body(xs[0], ts[0])  # eager warm-up step
    g = CapturedStep(body, xs[1], ts[1])
    losses = []
    for i in range(1, 4):
        g.load(xs[i], ts[i])
        losses.append(g().item())
    for i in range(4):
        ob.zero_grad()
        loss, _ = b.forward_loss(xs[i], ts[i])
        loss.backward()
        ob.step()
        if i:
            assert abs(loss.item() - losses[i - 1]) < 1e-6
    da.consolidate()  # deferred gathers: complete the last step's all-gathers
    torch.cuda.synchronize()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
    if defer:  # the bf16 compute copies must agree too (they are what the deferred gather moves)
        assert torch.equal(a.fc0.weight._ddpx_shadow, b.fc0.weight._ddpx_shadow)
    da.close()
    comm.close()


@pytest.mark.parametrize("shard", [False, True])
def test_capture_aborted_after_rccl_collectives_then_eager(gpu, pg, shard):
    """A capture that dies AFTER the backward's bucket collectives were recorded on the real RCCL communicator
    (what an N > 1 rank sees when a peer's capture fails): the graph is dropped, the host step state restored
    (ddpx.runtime.graphs.try_capture), and the following eager steps on the same communicator must match a
    run that never tried to capture, bitwise."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.optim.sgd import SGD
    from ddpx.parallel.comm import RcclComm
    from ddpx.parallel.ddp import DistributedDataParallel
    from ddpx.runtime.graphs import try_capture
    torch.manual_seed(2)
    a, b = MLP(hidden=512), MLP(hidden=512)
    b.load_state_dict(a.state_dict())
    for m in (a, b):
        ddpx.prepare_model(m, gpu)
    comm = RcclComm(gpu)
    da = DistributedDataParallel(a, comm=comm, bucket_cap_mb=1.0, first_bucket_mb=0.25, reduce_single=True,
                                 shard_optimizer=shard)
    oa = SGD(a.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, capturable=True)
    ob = SGD(b.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4)
    xs = [torch.rand(128, 3072, device=gpu).to(torch.bfloat16) for _ in range(4)]
    ts = [torch.randint(0, 10, (128,), device=gpu) for _ in range(4)]
    inject = {"on": False, "hit": 0}

    def body(x, y):
        oa.zero_grad()
        loss, _ = da.forward_loss(x, y)
        loss.backward()
        if inject["on"]:
            inject["hit"] += 1
            raise RuntimeError("injected capture failure after the backward's collectives")
        oa.step()
        return loss

    oa.sync_lr()
    losses = [body(xs[0], ts[0]).item()]
    inject["on"] = True
    g, err = try_capture(body, xs[1], ts[1], da, oa, comm=comm)
    assert g is None and "injected" in err and inject["hit"] == 1
    inject["on"] = False
    for i in range(1, 4):
        oa.sync_lr()
        losses.append(body(xs[i], ts[i]).item())
    for i in range(4):
        ob.zero_grad()
        loss, _ = b.forward_loss(xs[i], ts[i])
        loss.backward()
        ob.step()
        assert loss.item() == losses[i], (i, loss.item(), losses[i])
    da.consolidate()
    torch.cuda.synchronize()
    for p, q in zip(a.parameters(), b.parameters()):
        assert torch.equal(p, q)
    da.close()
    comm.close()


@pytest.mark.parametrize("kind", ["mlp_bf16", "mlp_fp32", "deepnn_bf16"])
def test_side_stream_optimizer_matches_in_stream(gpu, pg, kind):
    """Replicated plan with per-bucket optimizer overlap: each bucket's SGD on a side stream behind its
    all-reduce and the release of its weights (``side_stream_optimizer``) vs on the compute stream.  The side
    update may rewrite W_l (and its bf16 compute copy) while backward is still running, so a missed release
    (``flat.release`` / ``late_read_params``) or end-of-backward fallback would corrupt the data gradients that
    read W_l.  Master weights + momentum must be bitwise equal after eager AND graph-captured steps, for the bf16
    MLP (declares late reads), the fp32 MLP, and DeepNN (no late-read declaration: every bucket waits for the
    end of backward)."""
    import ddpx
    from ddpx.models import build_model
    from ddpx.optim.sgd import SGD
    from ddpx.parallel.comm import RcclComm
    from ddpx.parallel.ddp import DistributedDataParallel
    from ddpx.runtime.flat_params import flat_of
    from ddpx.runtime.graphs import CapturedStep
    name, dt = kind.split("_")
    comm = RcclComm(gpu)
    runs = []
    for side in (False, True):
        torch.manual_seed(3)
        m = build_model(name, hidden=512, layers=3, dtype=dt, device=gpu)
        ddpx.prepare_model(m, gpu)
        d = DistributedDataParallel(m, comm=comm, bucket_cap_mb=0.5, first_bucket_mb=0.125, reduce_single=True,
                                    overlap_optimizer=True, side_stream_optimizer=side)
        assert len(d.bucket_ranges) >= 2
        o = SGD(m.parameters(), lr=0.05, momentum=0.9, weight_decay=5e-4, capturable=True)
        d.attach_optimizer(o)
        assert (d._opt_stream is not None) == side  # (update_side_stream() answers only inside a step)
        g = torch.Generator(device="cpu").manual_seed(4)
        if name == "mlp":
            xs = [torch.rand(128, 3072, generator=g).to(gpu) for _ in range(6)]
            xs = [x.to(torch.bfloat16) if dt == "bf16" else x for x in xs]
        else:
            lay = m.input_layout(gpu) if hasattr(m, "input_layout") else "nchw_f32"
            assert lay.startswith("nhwc8") or lay.startswith("nchw"), lay
            xs = [torch.rand(64, 3, 32, 32, generator=g) for _ in range(6)]
            if lay.startswith("nhwc8"):
                xs = [torch.nn.functional.pad(x.permute(0, 2, 3, 1), (0, 5)).contiguous().to(torch.bfloat16)
                      for x in xs]
            xs = [x.to(gpu) for x in xs]
        ts = [torch.randint(0, 10, (xs[0].shape[0],), generator=g).to(gpu) for _ in range(6)]

        def body(x, y):
            o.zero_grad()
            loss, _ = d.forward_loss(x, y) if hasattr(m, "forward_loss") else (
                torch.nn.functional.cross_entropy(d(x), y), None)
            loss.backward()
            o.step()
            return loss

        o.sync_lr()
        losses = [body(xs[i], ts[i]).item() for i in range(3)]  # eager
        cap = CapturedStep(body, xs[3], ts[3])
        for i in range(3, 6):
            cap.load(xs[i], ts[i])
            losses.append(cap().item())
        d.consolidate()
        torch.cuda.synchronize()
        f = flat_of(m)
        runs.append((losses, f.master.detach().clone(),
                     {k: v.detach().clone() for k, v in f.state_tensors.items()}))
        cap = None
        d.close()
    (la, ma, sa), (lb, mb, sb) = runs
    assert la == lb, (la, lb)
    assert torch.equal(ma, mb)
    assert sa.keys() == sb.keys() and all(torch.equal(sa[k], sb[k]) for k in sa)
    comm.close()
