"""bench.py flag resolution (CPU): the defaults the driver's 1/2/4/8-GPU runs get.

N = 1 toy MLP: fp32 gradients + flat SGD pass (profiles/r1_n1alt); N > 1: bf16 gradient buckets,
ZeRO-1 with comm-stream shard updates and deferred gathers; other models keep their own defaults.
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _args(argv):
    import bench
    old = sys.argv
    sys.argv = ["bench.py", *argv]
    try:
        return bench.parse()
    finally:
        sys.argv = old


def _resolved(argv, world):
    import bench
    a = _args(argv)
    bench.resolve_defaults(a, world)
    return a


def test_single_gpu_toy_mlp_defaults():
    a = _resolved([], 1)
    assert a.model == "mlp" and a.hidden == 4096 and a.batch_size == 512
    assert a.grad_dtype == "fp32" and a.fused_optimizer == 0
    assert not a.shard_optimizer and not a.overlap_optimizer and not a.comm_side_optimizer


@pytest.mark.parametrize("world", [2, 4, 8])
def test_multi_gpu_toy_mlp_defaults(world):
    a = _resolved(["--gpus", str(world)], world)
    assert a.grad_dtype == "bf16"
    assert a.shard_optimizer == 1 and a.overlap_optimizer == 1
    assert a.comm_side_optimizer == 1 and a.defer_gather == 1 and a.chunk_mb == 0.0


def test_other_models_keep_fused_optimizer():
    for m in ("mlp_wide", "vgg", "deepnn"):
        a = _resolved(["--model", m], 1)
        assert a.fused_optimizer == 1, m
    assert _resolved(["--model", "mlp_wide"], 1).hidden == 16384
    v = _resolved(["--model", "vgg"], 8)
    assert v.shard_optimizer == 0 and v.comm_side_optimizer == 0 and v.defer_gather == 0


def test_explicit_flags_win():
    a = _resolved(["--fused_optimizer", "1", "--grad_dtype", "bf16"], 1)
    assert a.fused_optimizer == 1 and a.grad_dtype == "bf16"
    assert _resolved(["--model", "vgg", "--no_fused_optimizer"], 1).fused_optimizer == 0
    b = _resolved(["--gpus", "8", "--comm_side_optimizer", "0", "--shard_optimizer", "0"], 8)
    assert b.comm_side_optimizer == 0 and b.shard_optimizer == 0 and b.defer_gather == 0
