"""Unused parameters and ZeRO-1 shard geometry (CPU, gloo).

torch DDP semantics (``torch/nn/parallel/distributed.py``, ``find_unused_parameters``): with the flag a
rank that skips a parameter contributes a zero gradient and buckets are reduced in one order on every
rank; without it a skipped parameter is an error at world size > 1.  Regression test for the advisor
finding where a rank that skipped a layer force-launched its bucket with stale gradients and the
replicas drifted apart.
"""
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F
from torch import nn

from tests._dist_util import free_port, init_gloo


class TwoBranch(nn.Module):
    def __init__(self):
        super().__init__()
        self.a = nn.Linear(16, 8)
        self.b = nn.Linear(16, 8)
        self.head = nn.Linear(8, 4)

    def forward(self, x, use_b=True):
        h = self.a(x)
        if use_b:
            h = h + self.b(x)
        return self.head(torch.relu(h))


def _unused_worker(rank, ws, port, find_unused):
    import ddpx
    from ddpx.optim.sgd import SGD
    from ddpx.parallel.comm import TorchComm
    from ddpx.parallel.ddp import DistributedDataParallel
    from torch.nn.parallel import DistributedDataParallel as TorchDDP
    init_gloo(rank, ws, port)
    try:
        torch.manual_seed(0)
        ours, ref = TwoBranch(), TwoBranch()
        ref.load_state_dict(ours.state_dict())
        ddpx.prepare_model(ours, "cpu")
        d_ours = DistributedDataParallel(ours, comm=TorchComm(), bucket_cap_mb=1e-4, first_bucket_mb=1e-4,
                                         find_unused_parameters=find_unused)
        assert len(d_ours.bucket_ranges) >= 3  # one bucket per parameter group: ordering matters
        d_ref = TorchDDP(ref, find_unused_parameters=True)
        o_ours = SGD(ours.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
        o_ref = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-4)
        g = torch.Generator().manual_seed(rank)
        for step in range(3):
            x = torch.rand((4, 16), generator=g)
            t = torch.randint(0, 4, (4,), generator=g)
            use_b = not (rank == 1 and step == 1)  # rank 1 skips branch b once
            if not find_unused and not use_b:
                with pytest.raises(RuntimeError, match="find_unused_parameters"):
                    o_ours.zero_grad()
                    F.cross_entropy(d_ours(x, use_b), t).backward()
                return
            for net, opt in ((d_ours, o_ours), (d_ref, o_ref)):
                opt.zero_grad()
                F.cross_entropy(net(x, use_b), t).backward()
                opt.step()
        for (n, p), (_, q) in zip(ours.named_parameters(), ref.named_parameters()):
            assert torch.allclose(p, q, atol=1e-6, rtol=1e-5), (rank, n, (p - q).abs().max().item())
        flat = d_ours.flat.master.clone()
        lst = [torch.empty_like(flat) for _ in range(ws)]
        dist.all_gather(lst, flat)
        assert all(torch.equal(o, lst[0]) for o in lst), "replicas drifted apart"
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_find_unused_parameters_matches_torch_ddp():
    mp.spawn(_unused_worker, args=(2, free_port(), True), nprocs=2, join=True)


def _all_skip_worker(rank, ws, port, overlap, shard=False):
    """Both ranks skip branch b at step 1, weight decay and momentum on: torch leaves b's gradient None and its
    SGD does not touch b (no decay, no momentum step); ours must do the same, replicas bit-identical."""
    import ddpx
    from ddpx.optim.sgd import SGD
    from ddpx.parallel.comm import TorchComm
    from ddpx.parallel.ddp import DistributedDataParallel
    from torch.nn.parallel import DistributedDataParallel as TorchDDP
    init_gloo(rank, ws, port)
    try:
        torch.manual_seed(0)
        ours, ref = TwoBranch(), TwoBranch()
        ref.load_state_dict(ours.state_dict())
        ddpx.prepare_model(ours, "cpu")
        d_ours = DistributedDataParallel(ours, comm=TorchComm(), bucket_cap_mb=1e-4, first_bucket_mb=1e-4,
                                         find_unused_parameters=True, overlap_optimizer=overlap,
                                         shard_optimizer=shard)
        assert d_ours.sharded == shard
        d_ref = TorchDDP(ref, find_unused_parameters=True)
        o_ours = SGD(ours.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-2)
        if overlap or shard:
            d_ours.attach_optimizer(o_ours)
        o_ref = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-2)
        g = torch.Generator().manual_seed(rank)
        b_before = None
        for step in range(3):
            x = torch.rand((4, 16), generator=g)
            t = torch.randint(0, 4, (4,), generator=g)
            use_b = step != 1
            if step == 1:
                b_before = ours.b.weight.detach().clone()
            for net, opt in ((d_ours, o_ours), (d_ref, o_ref)):
                opt.zero_grad()
                F.cross_entropy(net(x, use_b), t).backward()
                opt.step()
            if shard:
                d_ours.consolidate()
            if step == 1:
                assert torch.equal(ours.b.weight, b_before), "a parameter no rank used was stepped"
        for (n, p), (_, q) in zip(ours.named_parameters(), ref.named_parameters()):
            assert torch.allclose(p, q, atol=1e-6, rtol=1e-5), (rank, n, (p - q).abs().max().item())
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [False, True])
def test_parameter_unused_on_every_rank_is_not_stepped(overlap):
    mp.spawn(_all_skip_worker, args=(2, free_port(), overlap), nprocs=2, join=True)


def test_parameter_unused_on_every_rank_is_not_stepped_zero1():
    """ZeRO-1 (shard_optimizer) + find_unused_parameters: the shard update skips the unused parameter's span
    (advisor r3 finding: the sharded branch ignored it and applied weight decay / momentum)."""
    mp.spawn(_all_skip_worker, args=(2, free_port(), False, True), nprocs=2, join=True)


def test_single_process_sgd_skips_parameters_without_gradient():
    """torch.optim.SGD skips grad=None parameters (no weight decay, no momentum step); ddpx's flat SGD too."""
    import ddpx
    from ddpx.optim.sgd import SGD
    torch.manual_seed(0)
    ours, ref = TwoBranch(), TwoBranch()
    ref.load_state_dict(ours.state_dict())
    ddpx.prepare_model(ours, "cpu")
    o_ours = SGD(ours.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-2)
    o_ref = torch.optim.SGD(ref.parameters(), lr=0.1, momentum=0.9, weight_decay=5e-2)
    g = torch.Generator().manual_seed(0)
    for step in range(4):
        x = torch.rand((4, 16), generator=g)
        t = torch.randint(0, 4, (4,), generator=g)
        use_b = step not in (1, 2)
        b_before = ours.b.weight.detach().clone()
        for net, opt in ((ours, o_ours), (ref, o_ref)):
            opt.zero_grad()
            F.cross_entropy(net(x, use_b), t).backward()
            opt.step()
        if not use_b:
            assert torch.equal(ours.b.weight, b_before), "a parameter without gradient was stepped"
    for (n, p), (_, q) in zip(ours.named_parameters(), ref.named_parameters()):
        assert torch.allclose(p, q, atol=1e-6, rtol=1e-5), (n, (p - q).abs().max().item())


def _both_skip_worker(rank, ws, port):
    import ddpx
    from ddpx.optim.sgd import SGD
    from ddpx.parallel.comm import TorchComm
    from ddpx.parallel.ddp import DistributedDataParallel
    init_gloo(rank, ws, port)
    try:
        torch.manual_seed(0)
        m = TwoBranch()
        ddpx.prepare_model(m, "cpu")
        d = DistributedDataParallel(m, comm=TorchComm(), bucket_cap_mb=1e-4, first_bucket_mb=1e-4)
        opt = SGD(m.parameters(), lr=0.1)
        opt.zero_grad()
        with pytest.raises(RuntimeError, match=r"b\.weight.*find_unused_parameters"):
            F.cross_entropy(d(torch.rand(4, 16), use_b=False), torch.zeros(4, dtype=torch.long)).backward()
    finally:
        dist.destroy_process_group()


def test_unused_parameter_without_flag_raises():
    """Default (torch's find_unused_parameters=False): a skipped parameter is reported, not reduced stale."""
    mp.spawn(_both_skip_worker, args=(2, free_port()), nprocs=2, join=True)


class _FakeComm:
    """Comm stand-in for rank r of ws ranks (layout only: no collective is issued)."""

    def __init__(self, rank, ws):
        self.rank, self.world_size, self.native = rank, ws, False

    def all_gather_object(self, obj):
        return [obj] * self.world_size

    def broadcast_(self, t, src=0, stream=None):
        pass

    def allreduce_(self, t, op="avg", stream=None, async_op=False):
        raise AssertionError("no collective expected")

    def check(self):
        pass


@pytest.mark.parametrize("ws", [2, 4, 8])
def test_zero1_shard_offsets_for_every_rank(ws):
    """update_ranges(b) of rank r is exactly the [r*c, (r+1)*c) shard the in-place reduce-scatter writes
    (rccl_comm.cpp issue_bucket: recv = ptr + rank*shard), aligned, disjoint, covering the bucket."""
    import ddpx
    from ddpx.models import MLP
    from ddpx.parallel.ddp import DistributedDataParallel
    from ddpx.runtime.flat_params import ALIGN
    layouts = []
    for r in range(ws):
        torch.manual_seed(0)
        m = MLP(hidden=192, layers=3)
        ddpx.prepare_model(m, "cpu")
        d = DistributedDataParallel(m, comm=_FakeComm(r, ws), shard_optimizer=True, reduce_single=True,
                                    bucket_cap_mb=0.5, first_bucket_mb=0.1, verify=False)
        assert d.sharded
        layouts.append(d)
    ref = layouts[0]
    for b, (s, e) in enumerate(ref.bucket_ranges):
        if ref.bucket_modes[b] != 1:
            for d in layouts:
                assert d.update_ranges(b) == [(s, e)]
            continue
        assert (e - s) % (ws * ALIGN) == 0
        c = (e - s) // ws
        shards = [layouts[r].update_ranges(b) for r in range(ws)]
        for r, sh in enumerate(shards):
            assert layouts[r].bucket_ranges == ref.bucket_ranges
            assert sh == [(s + r * c, s + (r + 1) * c)]
            assert sh[0][0] % ALIGN == 0
        covered = sorted(x for sh in shards for x in sh)
        assert covered[0][0] == s and covered[-1][1] == e
        assert all(a[1] == b_[0] for a, b_ in zip(covered, covered[1:]))
