"""bench.py flag resolution (CPU): the defaults the driver's 1/2/4/8-GPU runs get.

N = 1 toy MLP: fp32 gradients + flat SGD pass (profiles/r1_n1alt); N > 1: the stock DDP algorithm
(fp32 gradients, fp32 all-reduce, replicated optimizer overlapped per bucket); bf16 gradient comm and
ZeRO-1 are opt-in.  Also: the self-launch and CPU modes end to end (BASELINE config 1).
"""
import json
import subprocess
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


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
    # single process: SGD fused into the backward kernels (fp32 master / momentum, same arithmetic)
    assert a.grad_dtype == "fp32" and a.fused_optimizer == 1
    assert not a.shard_optimizer and not a.overlap_optimizer and not a.comm_side_optimizer


@pytest.mark.parametrize("world", [2, 4, 8])
def test_multi_gpu_toy_mlp_defaults(world):
    a = _resolved(["--gpus", str(world)], world)
    assert a.grad_dtype == "fp32" and a.overlap_optimizer == 1 and a.chunk_mb == 0.0
    # bucket caps and replicated-vs-ZeRO-1 are left to the start-up calibration on the node
    assert a.calibrate and a.shard_optimizer is None and a.bucket_cap_mb is None and a.first_bucket_mb is None
    assert a.stock_ref == 1 and a.fp8 == 0
    # the calibration's ZeRO-1 choice brings its companions
    import bench
    a.shard_optimizer = 1
    bench.resolve_zero_defaults(a)
    assert a.comm_side_optimizer == 1 and a.defer_gather == 1


@pytest.mark.parametrize("world", [2, 8])
def test_multi_gpu_uncalibrated_defaults(world):
    a = _resolved(["--gpus", str(world), "--bucket_plan", "default"], world)
    assert not a.calibrate and a.shard_optimizer == 0 and a.bucket_cap_mb == 25.0 and a.first_bucket_mb == 1.0
    assert a.comm_side_optimizer == 0 and a.defer_gather == 0


def test_zero1_opt_in():
    a = _resolved(["--gpus", "8", "--shard_optimizer", "1"], 8)
    assert a.shard_optimizer == 1 and a.comm_side_optimizer == 1 and a.defer_gather == 1
    b = _resolved(["--gpus", "8", "--shard_optimizer", "1", "--bucket_cap_mb", "25", "--first_bucket_mb", "1"], 8)
    assert not b.calibrate


def test_every_model_fuses_the_single_gpu_optimizer():
    for m in ("mlp", "mlp_wide", "vgg", "deepnn"):
        a = _resolved(["--model", m], 1)
        assert a.fused_optimizer == 1, m
    assert _resolved(["--model", "mlp_wide"], 1).hidden == 16384
    v = _resolved(["--model", "vgg", "--bucket_plan", "default"], 8)
    assert v.shard_optimizer == 0 and v.comm_side_optimizer == 0 and v.defer_gather == 0


def test_explicit_flags_win():
    a = _resolved(["--fused_optimizer", "1", "--grad_dtype", "bf16"], 1)
    assert a.fused_optimizer == 1 and a.grad_dtype == "bf16"
    assert _resolved(["--model", "vgg", "--no_fused_optimizer"], 1).fused_optimizer == 0
    b = _resolved(["--gpus", "8", "--comm_side_optimizer", "0", "--shard_optimizer", "0"], 8)
    assert b.comm_side_optimizer == 0 and b.shard_optimizer == 0 and b.defer_gather == 0


def test_self_launch_command_needs_no_launcher():
    import bench
    a = _args(["--gpus", "4", "--steps", "5"])
    assert bench.needs_self_launch(a, env={})
    assert not bench.needs_self_launch(a, env={"WORLD_SIZE": "4", "RANK": "0"})
    assert not bench.needs_self_launch(_args([]), env={})
    cmd = bench.self_launch_cmd(a, ["--gpus", "4", "--steps", "5"], 12345)
    assert cmd[1:3] == ["-m", "torch.distributed.run"] and "--nproc-per-node=4" in cmd
    assert "--master-addr=127.0.0.1" in cmd and cmd[-4:] == ["--gpus", "4", "--steps", "5"]


def _bench(argv, timeout=600, env_extra=None, stock_tail=False):
    env = dict(os.environ, OMP_NUM_THREADS="2", **(env_extra or {}))
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], cwd=ROOT, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    assert r.returncode == 0, (r.stdout + r.stderr)[-3000:]
    # the driver contract: exactly ONE JSON line on stdout
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith('{"metric"')]
    assert len(lines) == 1, r.stdout[-3000:]
    rec = json.loads(lines[0])
    if not stock_tail:
        return rec
    tails = [ln[len("STOCK "):] for ln in r.stderr.splitlines() if ln.startswith("STOCK ")]
    assert len(tails) == 1, r.stderr[-3000:]
    # the headline line is printed before the stock comparison starts
    return rec, json.loads(tails[0])


SMALL = ["--steps", "3", "--warmup", "1", "--batch_size", "64", "--hidden", "256", "--train_size", "1024"]


def test_bench_cpu_single_process():
    rec = _bench(["--device", "cpu", *SMALL])
    assert rec["n_gpus"] == 1 and rec["dtype"] == "fp32" and rec["value"] > 0
    assert rec["config"]["device"] == "cpu" and rec["config"]["ddp"] is False


def test_bench_cpu_two_ranks_self_launched():
    """``bench.py --gpus 2 --device cpu`` with no launcher: N ranks are started by bench.py itself."""
    rec = _bench(["--gpus", "2", "--device", "cpu", *SMALL])
    c = rec["config"]
    assert rec["n_gpus"] == 2 and c["global_batch"] == 128 and c["parallelism"] == "dp2"
    assert c["launcher"] == "self:torch.distributed.run"
    assert c["grad_dtype"] == "fp32" and c["grad_comm"].startswith("fp32 all-reduce")
    assert c["replicas_consistent"] is True and c["sharded_optimizer"] is False
    assert c["buckets_mb"] and rec["value"] > 0
    # bucket plans judged by timed training steps on this node (no ZeRO-1 candidate on the CPU: no bf16 shadow)
    assert c["bucket_plan"] == "calibrated" and c["calibration"]["chosen"].startswith("allreduce")
    assert all(v > 0 for v in c["calibration"]["step_ms"].values()) and len(c["calibration"]["step_ms"]) >= 1
    assert "step" in c["calibration"]["objective"]
    assert c["graph"] is False and c["graph_error"] is None


def test_bench_cpu_two_ranks_stock_after_the_line():
    """N > 1: the stock recipe (torch DDP over gloo here, over a second RCCL communicator on the GPU) runs only
    after the ddpx line is printed; its result is a ``STOCK`` line on stderr."""
    rec, tail = _bench(["--gpus", "2", "--device", "cpu", *SMALL], stock_tail=True)
    assert rec["config"]["stock_same_run"]["placement"].startswith("after this line")
    assert rec["config"]["vs_stock_same_run"] is None
    st = tail["stock_same_run"]
    assert st["ms_per_step"] > 0 and "torch DDP" in st["recipe"] and tail["vs_stock_same_run"] > 0
    assert tail["n_gpus"] == 2


def test_bench_cpu_two_ranks_survives_optional_failures():
    """a calibration candidate that fails is dropped on every rank, and a stock recipe failing
    on ONE rank becomes an agreed ``error`` — the job still exits 0 with its one ddpx line.  (The candidate fails
    on every rank, in its first training step: a failure on one rank only, after its peers issued that step's
    collectives, cannot be met by an agreement point — the communicator watchdog owns that case.)"""
    argv = ["--gpus", "2", "--device", "cpu", "--steps", "3", "--warmup", "1", "--batch_size", "64", "--hidden",
            "1024", "--train_size", "1024"]
    rec, tail = _bench(argv, stock_tail=True,
                       env_extra={"DDPX_BENCH_INJECT": "calib:allreduce:1/25MB,stock@rank1"})
    cal = rec["config"]["calibration"]
    assert cal["dropped"] == ["allreduce:1/25MB"], cal
    assert "InjectedFault" in cal["step_ms"]["allreduce:1/25MB"]["error"] or \
        "another rank" in cal["step_ms"]["allreduce:1/25MB"]["error"]
    assert cal["chosen"] != "allreduce:1/25MB" and cal["step_ms"][cal["chosen"]] > 0
    assert rec["config"]["replicas_consistent"] is True and rec["value"] > 0
    assert "error" in tail["stock_same_run"] and tail["vs_stock_same_run"] is None


def test_bench_cpu_every_candidate_failing_falls_back_to_torch_caps():
    rec = _bench(["--gpus", "2", "--device", "cpu", *SMALL, "--stock_ref", "0"],
                 env_extra={"DDPX_BENCH_INJECT": "calib"})
    c = rec["config"]
    assert c["calibration"]["chosen"] is None and "every candidate failed" in c["calibration"]["error"]
    assert c["bucket_cap_mb"] == 25.0 and c["first_bucket_mb"] == 1.0 and c["sharded_optimizer"] is False
    assert c["replicas_consistent"] is True and rec["value"] > 0
