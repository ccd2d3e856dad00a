"""singlegpu.py / multigpu.py as the reference's users run them (CPU, gloo)."""
import os
import re
import subprocess
import sys

import torch

from tests._dist_util import free_port
from tests.test_models import VanillaVGG

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, cwd, extra_env=None, timeout=600):
    env = dict(os.environ)
    env["PYTHONPATH"] = ROOT
    env["OMP_NUM_THREADS"] = "2"
    if extra_env:
        env.update(extra_env)
    r = subprocess.run([sys.executable, *args], cwd=cwd, env=env, stdout=subprocess.PIPE, stderr=subprocess.STDOUT,
                       text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-4000:]
    return r.stdout


def test_singlegpu_cpu_vgg_prints_and_checkpoint(tmp_path):
    out = _run([os.path.join(ROOT, "singlegpu.py"), "2", "1", "--batch_size", "64", "--device", "cpu",
                "--data", "synthetic", "--train_size", "256", "--test_size", "128"], tmp_path)
    lines = out.splitlines()
    assert "[GPU0] Epoch 0 | Batchsize: 64 | Steps: 4" in lines
    assert "Epoch 0 | Training checkpoint saved at checkpoint.pt" in lines
    assert "Epoch 1 | Training checkpoint saved at checkpoint.pt" in lines
    assert any(re.fullmatch(r"Total training time: \d+\.\d\d seconds", ln) for ln in lines)
    assert "fp32 model has size=35.20 MiB" in lines
    assert any(re.search(r"fp32 model has accuracy=\d+\.\d\d%", ln) for ln in lines)
    sd = torch.load(tmp_path / "checkpoint.pt", weights_only=True)
    assert len(sd) == 50 and "backbone.conv0.weight" in sd and not any(k.startswith("module.") for k in sd)
    VanillaVGG().load_state_dict(sd, strict=True)


def test_singlegpu_cpu_mlp_learns(tmp_path):
    out = _run([os.path.join(ROOT, "singlegpu.py"), "3", "5", "--model", "mlp", "--hidden", "128",
                "--batch_size", "128", "--device", "cpu", "--data", "synthetic", "--train_size", "2048",
                "--test_size", "512", "--steps_per_epoch", "auto", "--metrics", "m.jsonl", "--lr", "0.02",
                "--seed", "0"], tmp_path)
    acc = float(re.search(r"accuracy=(\d+\.\d\d)%", out).group(1))
    assert acc > 30.0, out  # learnable synthetic data: well above chance (10%)
    assert (tmp_path / "m.jsonl").exists()


def test_multigpu_cpu_spawn(tmp_path):
    out = _run([os.path.join(ROOT, "multigpu.py"), "1", "1", "--batch_size", "32", "--device", "cpu",
                "--nprocs", "2", "--model", "deepnn", "--data", "synthetic", "--train_size", "256",
                "--test_size", "64"], tmp_path, extra_env={"MASTER_PORT": str(free_port())})
    # two processes share the pipe: lines may interleave, so check substrings
    assert "[GPU0] Epoch 0 | Batchsize: 32 | Steps: 4" in out
    assert "[GPU1] Epoch 0 | Batchsize: 32 | Steps: 4" in out
    assert out.count("Epoch 0 | Training checkpoint saved at checkpoint.pt") == 1  # rank 0 only
    assert out.count("Total training time:") == 2  # every rank
    sd = torch.load(tmp_path / "checkpoint.pt", weights_only=True)
    assert not any(k.startswith("module.") for k in sd)


def test_multigpu_sharded_optimizer(tmp_path):
    out = _run([os.path.join(ROOT, "multigpu.py"), "2", "1", "--batch_size", "32", "--device", "cpu",
                "--nprocs", "2", "--model", "mlp", "--hidden", "64", "--data", "synthetic", "--train_size", "256",
                "--test_size", "64", "--shard_optimizer", "--full_checkpoint", "--lr", "0.02"], tmp_path,
               extra_env={"MASTER_PORT": str(free_port())})
    assert "[GPU1] Epoch 1 | Batchsize: 32 | Steps: 4" in out
    sd = torch.load(tmp_path / "checkpoint.pt", weights_only=True)
    full = torch.load(tmp_path / "checkpoint_full.pt", weights_only=True)
    for k, v in sd.items():
        assert torch.isfinite(v.float()).all(), k
    assert len(full["optimizer"]["state"]) == len(sd)


def test_multigpu_torchrun(tmp_path):
    out = _run(["-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr", "127.0.0.1",
                "--master-port", str(free_port()), os.path.join(ROOT, "multigpu.py"), "1", "1", "--batch_size", "64",
                "--device", "cpu", "--model", "mlp", "--hidden", "64", "--data", "synthetic", "--train_size", "512",
                "--test_size", "64", "--no_eval"], tmp_path)
    assert "[GPU0] Epoch 0 | Batchsize: 64 | Steps: 4" in out
    assert "[GPU1] Epoch 0 | Batchsize: 64 | Steps: 4" in out


def test_multigpu_runs_the_calibrated_plan_by_default(tmp_path):
    """The reference entry point runs the tuned path by default: the bucket plan is
    calibrated on the node by timed training steps, once, on rank 0's print; explicit caps skip it."""
    common = [os.path.join(ROOT, "multigpu.py"), "1", "1", "--batch_size", "64", "--device", "cpu", "--nprocs", "2",
              "--model", "mlp", "--hidden", "1536", "--data", "synthetic", "--train_size", "256", "--test_size",
              "64", "--no_eval"]
    out = _run(common, tmp_path, extra_env={"MASTER_PORT": str(free_port())})
    m = re.findall(r"bucket plan: calibrated (\S+) \(first [\d.]+ MB, cap [\d.]+ MB; training step ms per "
                   r"candidate: (\{.*\})\)", out)
    assert len(m) == 1, out
    table = eval(m[0][1])  # noqa: S307 - our own dict repr
    assert m[0][0] in table and len(table) >= 2 and all(v > 0 for v in table.values())
    out = _run(common + ["--bucket_cap_mb", "25", "--first_bucket_mb", "1"], tmp_path,
               extra_env={"MASTER_PORT": str(free_port())})
    assert "bucket plan" not in out


def test_reference_cli_defaults_to_reference_precision():
    """``python singlegpu.py E S`` trains fp32 like the reference (no autocast, /root/reference/singlegpu.py:134-141);
    bf16 is opt-in."""
    from ddpx.train.app import build_parser
    a = build_parser("x").parse_args(["20", "5"])
    assert a.dtype == "fp32" and a.model == "vgg" and a.batch_size == 512
    assert build_parser("x").parse_args(["1", "1", "--dtype", "bf16"]).dtype == "bf16"


def test_resume_full_checkpoint(tmp_path):
    common = [os.path.join(ROOT, "singlegpu.py"), "--model", "mlp", "--hidden", "64", "--batch_size", "64",
              "--device", "cpu", "--data", "synthetic", "--train_size", "256", "--test_size", "64", "--no_eval",
              "--full_checkpoint", "--seed", "0"]
    _run([common[0], "2", "1", *common[1:]], tmp_path)
    out = _run([common[0], "3", "1", *common[1:], "--resume"], tmp_path)
    assert "[GPU0] Epoch 0" not in out and "[GPU0] Epoch 2 | Batchsize: 64 | Steps: 4" in out
    st = torch.load(tmp_path / "checkpoint_full.pt", weights_only=True)
    assert st["epoch"] == 2 and st["optimizer"]["state"]


def test_fault_injection_all_ranks_exit_nonzero(tmp_path):
    """a rank failing mid-training takes the whole job down with a non-zero exit."""
    import subprocess
    import sys
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), PYTHONPATH=ROOT)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "multigpu.py"), "2", "1", "--batch_size", "32",
                        "--device", "cpu", "--nprocs", "2", "--model", "mlp", "--hidden", "64", "--data",
                        "synthetic", "--train_size", "256", "--test_size", "64", "--fault_step", "5",
                        "--fault_rank", "1"], cwd=tmp_path, env=env, capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert "injected fault at step 5" in (p.stdout + p.stderr)


def test_ddpx_launch_wrapper(tmp_path):
    """python -m ddpx.launch == torchrun with single-node 127.0.0.1 defaults."""
    out = _run(["-m", "ddpx.launch", "--nproc-per-node", "2", os.path.join(ROOT, "multigpu.py"), "1", "1",
                "--batch_size", "64", "--device", "cpu", "--model", "mlp", "--hidden", "64", "--data", "synthetic",
                "--train_size", "256", "--test_size", "64", "--no_eval"], tmp_path)
    assert "[GPU1] Epoch 0 | Batchsize: 64 | Steps: 2" in out


def test_port_in_use_gives_clear_error(tmp_path):
    """SURVEY §4 'Fault': a taken MASTER_PORT fails fast with an address-in-use error, not a hang."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        s.listen(1)
        port = s.getsockname()[1]
        env = dict(os.environ, PYTHONPATH=ROOT, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                   TORCH_DIST_INIT_BARRIER="0")
        p = subprocess.run([sys.executable, os.path.join(ROOT, "multigpu.py"), "1", "1", "--device", "cpu",
                            "--nprocs", "2", "--model", "mlp", "--hidden", "64", "--data", "synthetic",
                            "--train_size", "128", "--test_size", "64", "--no_eval"], cwd=tmp_path, env=env,
                           capture_output=True, text=True, timeout=300)
    assert p.returncode != 0
    assert re.search(r"address already in use|EADDRINUSE|Address already in use", p.stdout + p.stderr, re.I)
