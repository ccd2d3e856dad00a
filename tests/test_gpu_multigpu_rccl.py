"""Real multi-GPU runs of the DDP path over RCCL / xGMI (the C++ reducer's in-place reduce-scatter /
all-gather offsets and the comm-stream optimizer had only run at world size 1).

Skipped unless at least two GPUs are visible (the 1-GPU development boxes); on an 8 x MI355X node they run
``bench.py --gpus 2`` exactly as the driver's scaling run does (self-launched ranks, native RCCL
communicator, HIP-graph-captured step) and require every replica to end bitwise identical — for the default
replicated fp32 all-reduce and for ZeRO-1 (reduce-scatter + shard SGD + all-gather).
"""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(extra):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "10", "--warmup", "3",
           "--stock_ref", "0", *extra]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-4000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    return json.loads(line)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs >= 2 GPUs")
@pytest.mark.parametrize("extra", [[], ["--shard_optimizer", "1"]], ids=["allreduce_fp32", "zero1"])
def test_two_gpu_ddp_over_rccl_keeps_replicas_identical(extra):
    d = _bench(extra)
    c = d["config"]
    assert d["n_gpus"] == 2 and c["parallelism"] == "dp2" and c["comm"] in (None, "rccl")
    assert c["grad_dtype"] == "fp32"
    assert c["replicas_consistent"] is True
    assert d["value"] > 0 and c["final_loss"] == c["final_loss"]
