"""Host-logic parity with the torch components the reference relies on."""
import math

import numpy as np
import pytest
import torch
import torch.distributed as dist
from torch.optim.lr_scheduler import LambdaLR
from torch.utils.data.distributed import DistributedSampler

from ddpx.data.sampler import DistributedIndexSampler
from ddpx.optim.schedule import OneCycleLambda, resolve_steps_per_epoch
from ddpx.parallel.ddp import compute_bucket_assignment


class _Len:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n", [50000, 10000, 1, 3, 7, 100])
@pytest.mark.parametrize("ws", [1, 2, 4, 8])
def test_sampler_bit_identical(n, ws):
    for epoch in range(3):
        for rank in range(ws):
            ref = DistributedSampler(_Len(n), num_replicas=ws, rank=rank, shuffle=True, seed=0)
            ref.set_epoch(epoch)
            ours = DistributedIndexSampler(n, ws, rank, shuffle=True, seed=0)
            ours.set_epoch(epoch)
            assert list(ref) == ours.indices().tolist()
            assert len(ref) == len(ours)


@pytest.mark.parametrize("drop_last", [True, False])
def test_sampler_no_shuffle_drop_last(drop_last):
    for ws in (2, 3):
        for rank in range(ws):
            ref = DistributedSampler(_Len(101), num_replicas=ws, rank=rank, shuffle=False, drop_last=drop_last)
            ours = DistributedIndexSampler(101, ws, rank, shuffle=False, drop_last=drop_last)
            assert list(ref) == ours.indices().tolist()


def test_steps_per_epoch_match_reference():
    # 98 @1, 49 @2, 25 @4, 13 @8 (SURVEY §2.3 / BASELINE.md)
    for ws, steps in [(1, 98), (2, 49), (4, 25), (8, 13)]:
        s = DistributedIndexSampler(50000, ws, 0)
        assert math.ceil(len(s) / 512) == steps


def test_one_cycle_matches_reference_lambda():
    for spe in (98, 49):
        ref = lambda step: np.interp([step / spe], [0, 20 * 0.3, 20], [0, 1, 0])[0]  # noqa: E731
        ours = OneCycleLambda(spe)
        for step in [0, 1, 2, 97, 98, 293, 294, 588, 589, 1000, 1959, 1960, 1961, 5000]:
            assert ours(step) == pytest.approx(ref(step), abs=0, rel=0)
        assert ours(0) == 0.0


def test_lambdalr_drives_ddpx_sgd():
    import ddpx
    from ddpx.models import MLP
    from ddpx.optim.sgd import SGD
    m = MLP(in_features=12, hidden=8, layers=2)
    ddpx.prepare_model(m, "cpu")
    opt = SGD(m.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4)
    sch = LambdaLR(opt, OneCycleLambda(98))
    lrs = []
    for _ in range(5):
        lrs.append(opt.param_groups[0]["lr"])
        opt.step()
        sch.step()
    assert lrs[0] == 0.0
    assert lrs[1] == pytest.approx(0.4 * (1 / 98) / 6)


def test_resolve_steps_per_epoch():
    assert resolve_steps_per_epoch("compat", 25, True) == 49
    assert resolve_steps_per_epoch("compat", 25, False) == 98
    assert resolve_steps_per_epoch("auto", 25, True) == 25
    assert resolve_steps_per_epoch("7", 25, True) == 7


def test_bucket_assignment_matches_torch():
    torch.manual_seed(0)
    sizes = [40, 4 * 5120, 2048, 9437184, 2048, 2048, 9437184, 4096, 123, 4 * 2359296, 8, 4 * 36864]
    tensors = [torch.empty(s // 4 if s >= 4 else 1) for s in sizes]
    sizes_b = [t.numel() * 4 for t in tensors]
    limits = [1024 * 1024, 25 * 1024 * 1024]
    ref, _ = dist._compute_bucket_assignment_by_size(tensors, limits, [False] * len(tensors))
    ours = compute_bucket_assignment(sizes_b, limits)
    assert [sorted(b) for b in ref] == ours


def test_vgg_buckets_match_survey():
    """3 buckets of 9,461,800 / 27,148,288 / 303,360 bytes in grad-ready order."""
    from ddpx.models import VGG
    m = VGG()
    ps = list(reversed([p for p in m.parameters()]))
    sizes = [p.numel() * 4 for p in ps]
    buckets = compute_bucket_assignment(sizes, [1024 * 1024, 25 * 1024 * 1024])
    got = [sum(sizes[i] for i in b) for b in buckets]
    assert got == [9461800, 27148288, 303360]
