#!/usr/bin/env python3
"""Headline benchmark: samples/s (whole node) of the toy 3-layer MLP, bf16, DDP.

BASELINE.json metric: "samples/sec (whole node) + DDP scaling efficiency, toy MLP
at 1/2/4/8 MI355X".  Config: MLP 3072→4096→4096→10 on CIFAR-shaped
synthetic data (uint8 images resident on the GPU, RandomCrop+Flip augmentation
each step as in the reference), batch 512 per GPU (the reference's default
``--batch_size``), SGD lr 0.4 / momentum 0.9 / wd 5e-4 with the reference's
one-cycle schedule, fp32 master weights, fp32 gradients, bf16 MFMA compute.
Weak scaling: per-GPU batch fixed as N grows.

    python bench.py --gpus 1 --steps 200 --warmup 30
    python bench.py --gpus 8                     # self-launches 8 ranks (torch.distributed.run child)
    torchrun --nproc-per-node 8 bench.py --gpus 8  # or under an external launcher
    python bench.py --gpus 2 --comm host         # 2 ranks sharing ONE GPU (logic rehearsal, not perf)
    python bench.py --device cpu [--gpus 2]      # BASELINE config 1 (CPU, gloo for N > 1)

N > 1 averages fp32 gradients across ranks bucket by bucket while backward runs (reference
``multigpu.py:89``).  Before the first step the gradient-communication plan is calibrated on the node
(``ddpx.parallel.calibrate``; ``--bucket_plan default`` skips it): every candidate — fp32 all-reduce per
bucket with torch's greedy size rule at several caps (replicated optimizer, stock DDP), or fp32
reduce-scatter + bf16 shadow all-gather per bucket (ZeRO-1: same fp32 gradients and update, 0.75x the
bytes, 1/N of the optimizer stream per rank) — is built for real and a few graph-captured TRAINING STEPS of
it are timed (the max over ranks), so the choice accounts for overlap with backward and for the optimizer;
the line reports the plan and every timing (``bucket_plan``, ``calibration``).  bf16 gradient communication
(``--grad_dtype bf16``) is opt-in only.  ``--ddp_single`` runs the same machinery (calibration, RCCL reducer,
digest; ``--stock_ddp 1``: the stock torch-DDP baseline) at world size 1.

Every timed step does the whole job: batch gather+augment, forward, loss, backward, bucketed gradient
communication (N > 1), optimizer step and LR update.  The step is captured in a HIP graph; if capture fails
on any rank (agreed over the CPU group) every rank continues eagerly in the same process and the line says
so (``graph``: false, ``graph_error``).  After the timed region the replicas' fp32 master weights and
optimizer state are compared byte for byte (SHA-256 digests, ``replicas_consistent``), and the stock
PyTorch-ROCm recipe (nn.Linear + autocast + foreach SGD, torch DDP over its own RCCL group at N > 1) is
timed in the same job on the same data (``stock_same_run``, ``vs_stock_same_run``).  ``--impl torch`` runs
only the stock recipe.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

_PF_SEQ = __import__("itertools").count()
BASELINE_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "BASELINE.json")
LAUNCHER_ENV = "DDPX_BENCH_LAUNCHER"


def parse(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1, help="ranks (GPUs; CPU processes with --device cpu)")
    p.add_argument("--steps", type=int, default=100)
    p.add_argument("--warmup", type=int, default=20)
    p.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                   help="cpu: BASELINE config 1 (torch CPU kernels under the ddpx engine, gloo for N > 1)")
    p.add_argument("--batch_size", type=int, default=512, help="per-rank batch")
    p.add_argument("--hidden", type=int, default=None, help="MLP hidden width (default 4096 toy, 16384 wide)")
    p.add_argument("--layers", type=int, default=3)
    p.add_argument("--model", default="mlp", choices=["mlp", "mlp_wide", "vgg", "deepnn"])
    p.add_argument("--impl", default="ddpx", choices=["ddpx", "torch"])
    p.add_argument("--fp8", type=int, default=None,
                   help="1: MX-FP8 hidden-layer forward / weight-gradient GEMMs (MLP models; default 0)")
    p.add_argument("--torch_amp", action="store_true", help="--impl torch: bf16 autocast (+channels_last for VGG)")
    p.add_argument("--dtype", default="auto", choices=["auto", "bf16", "fp32"],
                   help="compute precision of the ddpx engine on the GPU: bf16 (default here: BASELINE.json's headline "
                        "config is the bf16 toy MLP) or fp32, the reference's recipe on the exact-f32 MFMA kernels (the "
                        "stock reference then runs without autocast; singlegpu.py / multigpu.py default to fp32 like "
                        "the reference)")
    p.add_argument("--kernels", default="auto", choices=["auto", "native", "torch"],
                   help="ddpx engine ops: auto / native = the hand-written HIP kernels for every model and precision; "
                        "torch = torch ops (MIOpen / hipBLASLt) under the ddpx engine")
    p.add_argument("--no_graph", action="store_true")
    p.add_argument("--prefetch_batch", type=int, default=0,
                   help="1 (N = 1, graphs): step k's kernels read a batch augmented during step k-1 on a side stream "
                        "(double-buffered input), so the augment kernel overlaps the previous step instead of "
                        "opening each step; same batches, same seeds, one augment per step.  Default 0: the "
                        "side-stream fork/join inside the graph costs more than the 8 us augment "
                        "(0.2753-0.2782 vs 0.2521-0.2531 ms/step, profiles/r3_val/NOTES.md)")
    p.add_argument("--graph_steps", type=int, default=None,
                   help="training steps per captured HIP graph (the launch gap between replays is paid once "
                        "per graph); the timed region still runs exactly --steps steps, every one of them a full "
                        "step (batch gather + augment, LR advance, forward, backward, optimizer).  Default: "
                        "min(20, --steps) (toy MLP, 20-step window: 0.2471-0.2542 ms vs 0.2566-0.2610 for one "
                        "step per graph; 200 steps in graphs of 5: 0.2339 vs 0.2368 ms, profiles/r4_graphsteps)")
    p.add_argument("--overlap_optimizer", type=int, default=None,
                   help="1: per-bucket optimizer as each collective lands (default 1 for N>1)")
    p.add_argument("--shard_optimizer", type=int, default=None,
                   help="1: ZeRO-1 reduce-scatter / shard update / all-gather; default: chosen by the start-up "
                        "calibration at N > 1 (--bucket_plan calibrated), else 0")
    p.add_argument("--no_fused_optimizer", action="store_true", help="N=1: separate SGD pass instead of fused")
    p.add_argument("--fused_optimizer", type=int, default=None,
                   help="N=1: 1 = SGD inside the backward kernels (default), 0 = fp32 gradients then one "
                        "non-temporal flat SGD pass")
    p.add_argument("--grad_dtype", default="auto", choices=["auto", "fp32", "bf16"],
                   help="gradient buffer / all-reduce dtype; auto = fp32 at every N (stock DDP precision)")
    p.add_argument("--bucket_cap_mb", type=float, default=None,
                   help="DDP bucket cap (default: calibrated on this node at N > 1, else torch's 25)")
    p.add_argument("--bucket_plan", default="calibrated", choices=["calibrated", "default"],
                   help="N > 1: time every candidate gradient-communication plan (bucket caps; replicated "
                        "all-reduce vs ZeRO-1 reduce-scatter + all-gather) on this node's links before the first "
                        "step and use the fastest (ddpx.parallel.calibrate); default = torch's 25 / 1 MiB caps")
    p.add_argument("--chunk_mb", type=float, default=None,
                   help="split weights larger than this into row-chunk buckets, each reduced as soon as its "
                        "slice of the weight gradient is written (opt-in; default off)")
    p.add_argument("--defer_gather", type=int, default=None,
                   help="ZeRO-1 only: all-gathers issued at the start of the next step, waited per chunk")
    p.add_argument("--side_optimizer", type=int, default=None,
                   help="replicated plan with optimizer overlap: each bucket's SGD update on a side stream behind its "
                        "all-reduce and its weights' last read in backward, one join per step (default 0: measured "
                        "slower at world size 1, profiles/r5_ddp1; DDPX_SIDE_OPTIMIZER=1 flips it)")
    p.add_argument("--comm_side_optimizer", type=int, default=None,
                   help="ZeRO-1 only: shard updates on the RCCL stream behind each reduce-scatter")
    p.add_argument("--first_bucket_mb", type=float, default=None)
    p.add_argument("--train_size", type=int, default=50000)
    p.add_argument("--json_out", default=None)
    p.add_argument("--ddp_single", action="store_true",
                   help="N=1: still run the DDP machinery (RCCL reducer at world size 1) to measure its overhead")
    p.add_argument("--sim_world", type=int, default=None,
                   help="diagnostics, with --ddp_single: present world size N to DDP (the N-rank bucket plan, ZeRO-1 "
                        "shards of 1/N, this rank's 1/N optimizer stream) on a one-rank communicator whose collectives "
                        "are skipped: the per-rank compute of an N-GPU step without its wire time (docs/SCALING.md)")
    p.add_argument("--comm", default="rccl", choices=["rccl", "host"],
                   help="host: gloo-staged collectives so several ranks can share one GPU (logic rehearsal on a "
                        "1-GPU box; not graph-capturable, not a performance path)")
    p.add_argument("--rccl_channels", default=None,
                   help="RCCL channel (CTA) bounds of the gradient communicator: N or MIN:MAX (default: RCCL's "
                        "choice, or DDPX_RCCL_CHANNELS); benchmarks/rccl_sweep.py measures the options")
    p.add_argument("--rccl_proto", default=None, help="NCCL_PROTO for this job (Simple, LL, LL128; default RCCL's)")
    p.add_argument("--stock_ref", type=int, default=None,
                   help="1: also time the stock PyTorch recipe (torch.nn + torch DDP over RCCL at N > 1) in this "
                        "job, after the ddpx timing, on the same data (default 1)")
    p.add_argument("--stock_steps", type=int, default=30)
    p.add_argument("--stock_ddp", type=int, default=0,
                   help="1: wrap the stock recipe in torch DDP over its own RCCL group even at world size 1 "
                        "(a rehearsal of the N > 1 baseline path; with --ddp_single)")
    p.add_argument("--digest", type=int, default=0,
                   help="1: report a SHA-256 of this rank's fp32 master weights + optimizer state after the timed "
                        "steps (``master_digest``; tests compare schedules for bitwise-identical training)")
    p.add_argument("--stock_first", type=int, default=None,
                   help="1: time the stock recipe BEFORE the ddpx warm-up instead of after the ddpx timing "
                        "(default 0)")
    p.add_argument("--stock_between", type=int, default=None,
                   help="1: time the stock recipe after the ddpx graph capture, before the last ddpx warm-up steps "
                        "(the timed window then starts on a GPU at sustained-load clocks; default for one process); "
                        "0: after the timed steps (default with DDP: N > 1 or --ddp_single).  With DDP and 0 the ddpx "
                        "JSON line is printed BEFORE the stock recipe starts (its result goes to stderr and "
                        "--json_out), so nothing in the optional comparison can cost the job its headline line")
    p.add_argument("--seed", type=int, default=0, help="model init seed (identical replicas are also enforced by DDP)")
    return p.parse_args(argv)


# ----------------------------------------------------------------------------------------- launcher
def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def needs_self_launch(args, env=None) -> bool:
    env = os.environ if env is None else env
    return args.gpus > 1 and "WORLD_SIZE" not in env and "RANK" not in env


def self_launch_cmd(args, argv, port: int):
    """torch.distributed.run child command for ``--gpus N`` without an external launcher."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
            "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__), *argv]


def self_launch(args, argv) -> int:
    """Run N ranks as a torch.distributed.run child (reference: ``mp.spawn`` at multigpu.py:262-263).

    This process never initialises HIP (no torch.cuda call), so starting the ranks is safe.  Their output is
    forwarded line by line; rank 0 prints the one JSON line (with ``config.launcher`` set)."""
    env = dict(os.environ)
    env[LAUNCHER_ENV] = "self:torch.distributed.run"
    env.setdefault("MASTER_ADDR", "127.0.0.1")
    env.setdefault("OMP_NUM_THREADS", "4")
    proc = subprocess.Popen(self_launch_cmd(args, argv, _free_port()), env=env, stdout=subprocess.PIPE, text=True,
                            bufsize=1)
    for line in proc.stdout:
        sys.stdout.write(line)
        sys.stdout.flush()
    return proc.wait()


def baseline_value(metric_key: str):
    try:
        with open(BASELINE_FILE) as f:
            b = json.load(f)
        v = b.get("published", {}).get(metric_key)
        return float(v) if v else None
    except Exception:
        return None


# ------------------------------------------------------------------------------------------ setup
def setup_dist(args):
    import torch
    import torch.distributed as dist
    n, impl = args.gpus, args.impl
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != n:
        print(f"bench.py: --gpus {n} but WORLD_SIZE={world}", file=sys.stderr)
        sys.exit(2)
    cpu = args.device == "cpu"
    if not cpu:
        ndev = torch.cuda.device_count()
        if args.comm == "host" or (ndev and local >= ndev):
            local = local % ndev  # ranks may share a device (host-staged comm, or the tests' one-GPU rehearsals)
        torch.cuda.set_device(local)
    # a hung collective is reported per rank after this long (RcclComm watchdog, eager steps and graph replays)
    os.environ.setdefault("DDPX_COMM_TIMEOUT", "300")
    if n == 1 and args.ddp_single and world == 1:
        # time the DDP machinery, not RCCL's one-rank in-place copy kernels (identity at world size 1)
        os.environ.setdefault("DDPX_COMM_SKIP_IDENTITY", "1")
    if world > 1 or (n == 1 and args.ddp_single):
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if world == 1 and "MASTER_PORT" not in os.environ:
            os.environ["MASTER_PORT"] = str(_free_port())
        # ddpx: GPU collectives go through its own RCCL communicator; the c10d group only
        # bootstraps it (TCPStore) and carries CPU barriers/timing -> gloo.  torch: stock RCCL PG.
        backend = "gloo" if (impl == "ddpx" or cpu) else "nccl"
        dist.init_process_group(backend=backend, rank=rank, world_size=world)
    return rank, world, local


def make_data(args, device, rank, world, layout=None):
    from ddpx.data.datasets import synthetic_cifar
    from ddpx.data.loader import DeviceLoader
    from ddpx.data.sampler import DistributedIndexSampler
    ds = synthetic_cifar(args.train_size, seed=0)
    sampler = DistributedIndexSampler(len(ds), world, rank, shuffle=True, seed=0)
    if layout is None:
        from ddpx.models import native_kernels_for
        fp32 = getattr(args, "dtype", "auto") == "fp32"
        native = args.impl == "ddpx" and native_kernels_for(args.model, "fp32" if fp32 else "bf16",
                                                            getattr(args, "kernels", "auto"))
        layout = "flat_bf16" if (native and args.model.startswith("mlp")) else "nchw_f32"
        if native and args.model in ("vgg", "deepnn"):
            layout = "nhwc8_bf16"
        if native and fp32:
            layout = {"vgg": "nhwc4_f32", "deepnn": "nhwc4_f32"}.get(args.model, "flat_f32")
        if device.type == "cpu":
            layout = "nchw_f32"
    return DeviceLoader(ds, args.batch_size, device, sampler=sampler, train=True, layout=layout, seed=rank)


def resolve_defaults(args, world):
    if args.graph_steps is None:
        # (--prefetch_batch alternates two single-step graphs)
        args.graph_steps = 1 if args.prefetch_batch else max(1, min(20, args.steps))
    if args.hidden is None:
        args.hidden = 16384 if args.model == "mlp_wide" else 4096
    multi = world > 1 or args.ddp_single
    if args.fp8 is None:
        args.fp8 = 0
    if args.grad_dtype == "auto":
        # stock DDP precision at every N: fp32 gradients, fp32 all-reduce (bf16 is opt-in)
        args.grad_dtype = "fp32"
    if args.overlap_optimizer is None:
        args.overlap_optimizer = int(multi)
    # N > 1 ddpx: bucket caps and replicated-vs-ZeRO-1 come from the start-up calibration unless given
    # (--ddp_single: the same calibration at world size 1 on the real communicator, a rehearsal of the N > 1 path)
    args.calibrate = bool((world > 1 or args.ddp_single) and args.impl == "ddpx" and args.bucket_plan == "calibrated"
                          and (args.shard_optimizer is None or args.bucket_cap_mb is None
                               or args.first_bucket_mb is None))
    if args.shard_optimizer is None and not args.calibrate:
        args.shard_optimizer = 0  # the replicated (stock DDP) optimizer
    if args.bucket_cap_mb is None and not args.calibrate:
        args.bucket_cap_mb = 25.0
    if args.first_bucket_mb is None and not args.calibrate:
        args.first_bucket_mb = 1.0
    args.chunk_explicit = args.chunk_mb is not None
    if args.chunk_mb is None:
        args.chunk_mb = 0.0
    if args.fused_optimizer is None:
        # single process: SGD inside the backward kernels (toy MLP: the warp-specialised weight-gradient +
        # optimizer kernel, profiles/r2_wsgd: 0.257 vs 0.275 ms/step for fp32 gradients + a flat SGD pass)
        args.fused_optimizer = 1
    if args.no_fused_optimizer:
        args.fused_optimizer = 0
    resolve_zero_defaults(args)
    if args.stock_ref is None:
        args.stock_ref = int(args.impl == "ddpx" and (not args.ddp_single or bool(args.stock_ddp))
                             and args.comm == "rccl")
    if args.stock_between is None:
        # N > 1: the stock torch-DDP run opens a second NCCL communicator next to ddpx's own; it runs only after the
        # ddpx line is out
        args.stock_between = int(not multi)
    if args.stock_first is None:
        # measured (profiles/r3_val): stock-first gives the stock recipe a cold GPU (0.88-0.90 vs 0.62-0.73 ms) and
        # ddpx no clear gain, so the baseline runs last unless asked
        args.stock_first = 0


def resolve_zero_defaults(args):
    """ZeRO-1 companions (known once shard_optimizer is: after the calibration at N > 1)."""
    if args.shard_optimizer is None:
        return
    if args.comm_side_optimizer is None:
        args.comm_side_optimizer = int(bool(args.shard_optimizer))
    if getattr(args, "side_optimizer", None) is None:
        args.side_optimizer = int(os.environ.get("DDPX_SIDE_OPTIMIZER", "0") == "1")
    if args.defer_gather is None:
        args.defer_gather = int(bool(args.shard_optimizer) and args.model.startswith("mlp"))


def make_comm(args, device, world):
    """The gradient communicator of the ddpx engine (None for a single process without ``--ddp_single``): one per
    job, shared by the calibration trials and the timed run."""
    if not (world > 1 or args.ddp_single) or args.impl != "ddpx":
        return None
    from ddpx.parallel.comm import HostStagedComm, RcclComm, TorchComm, set_rccl_protocol
    if device.type == "cpu":
        return TorchComm()
    if args.comm == "host":
        return HostStagedComm()
    set_rccl_protocol(args.rccl_proto)
    sim = args.sim_world if (args.ddp_single and args.sim_world) else None
    if world <= 1:
        return RcclComm(device, channels=args.rccl_channels, sim_world=sim)
    # N > 1: the native RCCL communicator is created on every rank, and every rank learns (over the gloo group)
    # whether all of them got one.  If any rank failed, all fall back to the gloo-staged communicator, which is slow
    # but correct and still yields the job's line (recorded as config.comm "host" + comm_fallback), instead of a
    # job that dies, or ranks that disagree on the collective they run.
    import torch.distributed as dist
    from ddpx.parallel.calibrate import _all_ok
    from ddpx.utils.faults import maybe_inject
    comm, err = None, None
    try:
        maybe_inject("rccl", "", dist.get_rank())  # tests: a communicator that cannot be created (every rank)
        comm = RcclComm(device, channels=args.rccl_channels, sim_world=sim)
    except Exception as e:  # noqa: BLE001 - any failure of the native communicator
        err = f"{type(e).__name__}: {e}"[:400]
    if _all_ok(err is None):
        return comm
    if comm is not None:
        try:
            comm.close(abort=True)
        except Exception:  # noqa: BLE001
            pass
    args.comm = "host"
    args.comm_fallback = err or "RCCL communicator failed on another rank"
    print(f"[bench] native RCCL communicator unavailable ({args.comm_fallback}); gloo-staged fallback",
          file=sys.stderr, flush=True)
    return HostStagedComm()


def build_ddpx(args, device, world, comm=None):
    import torch
    from ddpx.models import build_model
    from ddpx.optim.schedule import one_cycle, resolve_steps_per_epoch
    from ddpx.optim.sgd import SGD
    from ddpx.parallel.ddp import DistributedDataParallel
    from ddpx.runtime.setup import prepare_model
    torch.manual_seed(args.seed)
    cpu = device.type == "cpu"
    fp32 = cpu or args.dtype == "fp32"
    model = build_model(args.model, hidden=args.hidden, layers=args.layers, dtype="fp32" if fp32 else "bf16",
                        device=device, fp8=bool(args.fp8), kernels=args.kernels)
    prepare_model(model, device, grad_dtype=torch.bfloat16 if args.grad_dtype == "bf16" else torch.float32)
    # single process: the SGD update may be fused into the kernels that produce each gradient
    opt = SGD(model.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4,
              capturable=not (args.no_graph or cpu),
              fused_backward=(world == 1 and not args.ddp_single and bool(args.fused_optimizer) and not cpu))
    net = model
    if comm is not None:
        net = DistributedDataParallel(model, comm=comm, bucket_cap_mb=args.bucket_cap_mb,
                                      reduce_single=args.ddp_single,
                                      first_bucket_mb=args.first_bucket_mb,
                                      overlap_optimizer=bool(args.overlap_optimizer),
                                      shard_optimizer=bool(args.shard_optimizer), chunk_mb=args.chunk_mb or None,
                                      defer_gather=bool(args.defer_gather),
                                      comm_side_optimizer=bool(args.comm_side_optimizer),
                                      side_stream_optimizer=bool(getattr(args, "side_optimizer", 0)))
        if args.overlap_optimizer or args.shard_optimizer:
            net.attach_optimizer(opt)
    sched = one_cycle(opt, resolve_steps_per_epoch("compat", 0, world > 1))
    return model, net, opt, sched


def build_torch(args, device, world, group=None):
    """Stock PyTorch-ROCm recipe (the baseline to beat): torch.nn model, torch DDP (over RCCL on the GPU,
    ``group``: its process group) at N > 1, foreach SGD, LambdaLR."""
    import torch
    import torch.nn as nn
    from torch.nn.parallel import DistributedDataParallel as TDDP
    from ddpx.optim.schedule import OneCycleLambda, resolve_steps_per_epoch
    torch.manual_seed(args.seed)
    if args.model in ("vgg", "deepnn"):
        from ddpx.models import VGG, DeepNN
        model = (VGG if args.model == "vgg" else DeepNN)().to(device)
        if args.torch_amp:
            model = model.to(memory_format=torch.channels_last)
    else:
        dims = [3072] + [args.hidden] * (args.layers - 1) + [10]
        layers = []
        for i in range(args.layers):
            layers.append(nn.Linear(dims[i], dims[i + 1]))
            if i < args.layers - 1:
                layers.append(nn.ReLU())
        model = nn.Sequential(nn.Flatten(), *layers).to(device)
    net = (TDDP(model, device_ids=[device.index] if device.type == "cuda" else None, process_group=group)
           if (world > 1 or group is not None) else model)
    opt = torch.optim.SGD(model.parameters(), lr=0.4, momentum=0.9, weight_decay=5e-4)
    sched = torch.optim.lr_scheduler.LambdaLR(opt, OneCycleLambda(resolve_steps_per_epoch("compat", 0, world > 1)))
    return model, net, opt, sched


def torch_runner(args, device, world, loader, idx_all, full, group=None):
    """Eager step loop of the stock recipe."""
    import torch
    bs = args.batch_size
    amp = (device.type == "cuda" and (args.model not in ("vgg", "deepnn") or args.torch_amp)
           and getattr(args, "dtype", "auto") != "fp32")
    model, net, opt, sched = build_torch(args, device, world, group=group)

    def one_step(k):
        b = full[k % len(full)]
        x, y = loader.make_batch(idx_all[b * bs:(b + 1) * bs], k)
        opt.zero_grad(set_to_none=True)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = net(x)
        loss = torch.nn.functional.cross_entropy(out.float(), y)
        loss.backward()
        opt.step()
        sched.step()
        return loss

    def run(k, n):
        loss = None
        for i in range(n):
            loss = one_step(k + i)
        return loss

    return model, net, opt, sched, run


def graph_sizes(S: int, warm: int = 0):
    """Training steps per captured graph: 1, S, and ``warm`` = the warm-up steps left after capture: the graph the
    warm-up replays once, so that a short timed window replays only graphs that already ran (a graph's first
    replay is slow; ddpx.runtime.graphs.GraphedSteps.schedule, profiles/r5_window)."""
    extra = os.environ.get("DDPX_GRAPH_SIZES")  # diagnostics (benchmarks/window_probe.py): exact size set
    if extra:
        return sorted({1} | {int(v) for v in extra.split(",") if v.strip()})
    out = {1, S}
    if warm >= 2:
        out.add(min(warm, S))
    return sorted(out)


def make_runner(args, device, world, loader, idx_all, full, comm=None):
    """The engine under test and ``run(k, n)`` for its steps k .. k+n-1 (returns the last loss).

    ddpx on the GPU: every step (batch gather + augment from a device cursor, forward, backward with the
    bucketed collectives, optimizer, LR) is captured in a HIP graph after two eager steps and replayed; if
    capture fails on any rank every rank continues eagerly.  ddpx on the CPU and ``--impl torch``: eager steps.
    Used for the timed run and for each start-up calibration trial (``comm`` is the job's communicator)."""
    import torch
    import torch.distributed as dist
    cpu = device.type == "cpu"
    bs = args.batch_size
    runner = None
    closers = []
    if args.impl == "ddpx" and not cpu:
        from ddpx.runtime.graphs import (CapturedCycle, CapturedStep, GraphedSteps, agree_all_ranks,
                                         pingpong_signature_of, restore_after_failed_capture, step_state_snapshot)
        model, net, opt, sched = build_ddpx(args, device, world, comm)
        static_x, static_y = loader.make_batch(idx_all[:bs], 0)

        # the LR schedule lives on the device: the captured step advances it (no per-step host write)
        opt.attach_device_schedule(sched)
        one = torch.ones((), device=device)  # d(loss)/d(loss): no fill kernel per step

        # the batch comes from a device-side cursor over this epoch's index permutation (gather + crop/flip
        # augment in one kernel that also advances the cursor), so the captured step needs no host work
        # per replay besides the launch: batch k = full batch k % nfull, augmentation seed batch_seed(k),
        # exactly the batches the eager loader would draw
        nfull = len(full)
        idx_dev = idx_all[:nfull * bs].contiguous()

        counter = opt.step_counter()  # read by the batch gather, advanced by the LR-table kernel below

        def step_body(x, y):
            loader.cursor_batch(idx_dev, nfull, x, y, counter=counter)
            opt.device_lr_step()
            opt.zero_grad()
            loss, _ = net.forward_loss(x, y) if hasattr(model, "forward_loss") else (
                torch.nn.functional.cross_entropy(net(x), y), None)
            loss.backward(one)
            opt.step()
            return loss

        use_graph = not args.no_graph
        S = max(1, args.graph_steps) if use_graph else 1
        prefetch = bool(args.prefetch_batch and use_graph and world == 1 and S == 1)
        args.prefetch_batch = int(prefetch)
        if prefetch:
            # double-buffered batches: step k reads bufs[k % 2], filled during step k-1 by the augment kernel on a
            # side stream (forked at the step's start, joined at its end), which draws batch k + 1 into the other
            # buffer from its own device cursor (batch index = augments issued so far)
            bufs = [(static_x, static_y), (torch.empty_like(static_x), torch.empty_like(static_y))]
            side = torch.cuda.Stream(device)
            from ddpx.runtime.graphs import register_side_stream, unregister_side_stream
            pf_name = f"prefetch stream #{next(_PF_SEQ)}"
            register_side_stream(side, pf_name)  # joined back / reset by a failed capture
            closers.append(lambda: unregister_side_stream(pf_name))
            data_ctr = counter.clone()
            loader.cursor_batch(idx_dev, nfull, *bufs[0], counter=data_ctr)  # batch of the first step
            data_ctr.add_(1)
            pstate = {"k": 0}

            def pf_body(par):
                x, y = bufs[par]
                nx, ny = bufs[1 - par]
                cur = torch.cuda.current_stream()
                fork = torch.cuda.Event()
                fork.record(cur)
                side.wait_event(fork)
                with torch.cuda.stream(side):
                    loader.cursor_batch(idx_dev, nfull, nx, ny, counter=data_ctr)
                    data_ctr.add_(1)
                ready = torch.cuda.Event()
                ready.record(side)
                opt.device_lr_step()
                opt.zero_grad()
                loss, _ = net.forward_loss(x, y) if hasattr(model, "forward_loss") else (
                    torch.nn.functional.cross_entropy(net(x), y), None)
                loss.backward(one)
                opt.step()
                cur.wait_event(ready)
                return loss

            def pf_eager():
                loss = pf_body(pstate["k"] % 2)
                pstate["k"] += 1
                return loss

        def multi_body(x, y, m):
            loss = None
            for _ in range(m):
                loss = step_body(x, y)
            return loss

        comm_obj = getattr(net, "comm", None)
        snap = {}

        def make_graphs():
            # host-side step state a failed capture could leave half-done (restored by the fallback)
            snap.update(step_state_snapshot(net, opt))
            if prefetch:
                gp = [CapturedStep(lambda x, y, par=par: pf_body(par), static_x, static_y, use_inputs_as_static=True,
                                   comm=comm_obj) for par in (0, 1)]

                def replay_pf():
                    loss = gp[pstate["k"] % 2]()
                    pstate["k"] += 1
                    return loss
                return {1: replay_pf}
            # one version per state of the step's ping-pong weight copies (CapturedCycle: replays alternate)
            sig = pingpong_signature_of(opt)
            g = {1: CapturedCycle(step_body, static_x, static_y, signature=sig, use_inputs_as_static=True,
                                  comm=comm_obj)}
            # multi-step graphs: S, plus the ramp sizes a timed window starts with (GraphedSteps.schedule)
            for m in graph_sizes(S, warm=args.warmup - 2):
                if m == 1:
                    continue
                g[m] = CapturedCycle(lambda x, y, m=m: multi_body(x, y, m), static_x, static_y, signature=sig,
                                     use_inputs_as_static=True, comm=comm_obj)
                if g[m].period > 1 or g[1].period > 1 and m % g[1].period:
                    g.pop(m)  # m-step graphs only when they leave the copies where the 1-step cycle expects them
            return g

        def fallback():
            # nothing of the aborted capture ran on the device: put the host bookkeeping back to where the
            # last eager step left it and continue eagerly (same process, same communicator)
            restore_after_failed_capture(net, opt, snap)

        runner = GraphedSteps(pf_eager if prefetch else (lambda: step_body(static_x, static_y)), make_graphs,
                              steps_per_graph=S,
                              use_graph=use_graph, agree=agree_all_ranks, on_fallback=fallback,
                              after=lambda m: [sched.step() for _ in range(m)])

        def run(k, n):
            """Steps k .. k+n-1: eager for the first two (allocator / lazy-init warm-up), then replays of an
            S-step graph and of a 1-step graph for the remainder (eager if capture failed on any rank)."""
            return runner.run(k, n)
    elif args.impl == "ddpx":  # CPU: the ddpx engine (flat store, flat SGD, DDP over gloo) on torch CPU kernels
        model, net, opt, sched = build_ddpx(args, device, world, comm)

        def one_step(k):
            b = full[k % len(full)]
            x, y = loader.make_batch(idx_all[b * bs:(b + 1) * bs], k)
            opt.zero_grad()
            loss, _ = net.forward_loss(x, y)
            loss.backward()
            opt.step()
            sched.step()
            return loss

        def run(k, n):
            loss = None
            for i in range(n):
                loss = one_step(k + i)
            return loss
    else:
        model, net, opt, sched, run = torch_runner(args, device, world, loader, idx_all, full)

    def close():
        """Release this engine's reducer and captured graphs (not the shared communicator)."""
        if runner is not None:
            runner.graphs = None
        if net is not model and hasattr(net, "close"):
            net.close()
        for c in closers:
            c()
        closers.clear()

    return argparse.Namespace(model=model, net=net, opt=opt, sched=sched, run=run, runner=runner,
                              close=close)



def calibrate_plan(args, device, world, loader, idx_all, full, comm, rank=0):
    """Start-up calibration (``ddpx.parallel.calibrate``): build every candidate gradient-communication plan for
    real (its own model copy, DDP buckets and optimizer, graph-captured like the timed run), time a few
    training steps of each, and set ``args``' bucket caps / ZeRO-1 choice to the fastest.  Collective."""
    import gc

    import torch
    from ddpx.models import build_model
    from ddpx.parallel.calibrate import calibrate_by_step, candidate_plans
    from ddpx.utils.faults import maybe_inject
    from ddpx.runtime.flat_params import flat_of
    from ddpx.runtime.setup import prepare_model
    cpu = device.type == "cpu"
    fp32 = cpu or args.dtype == "fp32"
    probe = build_model(args.model, hidden=args.hidden, layers=args.layers, dtype="fp32" if fp32 else "bf16",
                        device=device, fp8=bool(args.fp8), kernels=args.kernels)
    prepare_model(probe, device)
    f = flat_of(probe)
    numels = list(f.numels)
    shapes = [tuple(p.shape) for p in f.params]
    shadow_only = [id(p) in f.shadow_only for p in f.params]
    del probe, f
    allow = (args.shard_optimizer is None and any(shadow_only) and args.comm == "rccl" and not cpu) or \
        bool(args.shard_optimizer)
    cand_world = (args.sim_world or max(world, 2)) if args.ddp_single else world
    plans = candidate_plans(numels, shadow_only, cand_world, allow_shard=allow,
                            shapes=None if args.chunk_explicit else shapes)
    if args.shard_optimizer is not None:
        plans = [p for p in plans if p["shard"] == bool(args.shard_optimizer)]
    if args.bucket_cap_mb is not None or args.first_bucket_mb is not None:
        plans = [dict(p, bucket_cap_mb=args.bucket_cap_mb if args.bucket_cap_mb is not None else p["bucket_cap_mb"],
                      first_bucket_mb=(args.first_bucket_mb if args.first_bucket_mb is not None
                                       else p["first_bucket_mb"])) for p in plans]
    sync = (lambda: None) if cpu else torch.cuda.synchronize
    if not plans:  # nothing to choose between: torch's caps
        args.bucket_cap_mb = 25.0 if args.bucket_cap_mb is None else args.bucket_cap_mb
        args.first_bucket_mb = 1.0 if args.first_bucket_mb is None else args.first_bucket_mb
        if args.shard_optimizer is None:
            args.shard_optimizer = 0
        resolve_zero_defaults(args)
        return

    def apply(a, plan):
        a.shard_optimizer = int(plan["shard"])
        a.bucket_cap_mb = plan["bucket_cap_mb"]
        a.first_bucket_mb = plan["first_bucket_mb"]
        a.comm_side_optimizer = args.comm_side_optimizer
        a.side_optimizer = getattr(args, "side_optimizer", None)
        a.defer_gather = args.defer_gather
        if not args.chunk_explicit:
            a.chunk_mb = plan.get("chunk_mb") or 0.0
        resolve_zero_defaults(a)

    def make_trial(plan):
        a = argparse.Namespace(**vars(args))
        apply(a, plan)
        a.calibrate = False
        a.graph_steps = 1  # trials replay one step at a time: no multi-step graph to capture
        eng = make_runner(a, device, world, loader, idx_all, full, comm)
        k = [0]

        def step():
            if k[0] == 0:
                maybe_inject("calib", plan["name"], rank)  # tests: a candidate failing in its first step
            eng.run(k[0], 1)
            k[0] += 1

        def close():
            sync()
            eng.close()
            eng.runner = eng.run = eng.net = eng.model = eng.opt = eng.sched = None
            gc.collect()
            if not cpu:
                torch.cuda.empty_cache()
        return step, close

    try:
        chosen, table = calibrate_by_step(plans, make_trial, sync=sync, warm=3, reps=3 if cpu else 5,
                                          rounds=1 if cpu else 3)
    except RuntimeError as e:
        # every candidate failed on some rank (agreed): torch's default plan, replicated optimizer
        args.bucket_cap_mb = 25.0 if args.bucket_cap_mb is None else args.bucket_cap_mb
        args.first_bucket_mb = 1.0 if args.first_bucket_mb is None else args.first_bucket_mb
        if args.shard_optimizer is None:
            args.shard_optimizer = 0
        resolve_zero_defaults(args)
        args.calibration = {"chosen": None, "error": str(e)[:600], "fallback": "torch default caps (25/1 MiB)"}
        return
    apply(args, chosen)
    dropped = sorted(k for k, v in table.items() if isinstance(v, dict))
    args.calibration = {"chosen": chosen["name"], "objective": "training step ms (max over ranks)",
                        "step_ms": table, "dropped": dropped or None}


def measure_stock_same_run(args, device, world, rank, idx_all, full):
    """The stock PyTorch-ROCm recipe timed in this job, on the same data: torch.nn model + bf16 autocast (fp32
    when --dtype fp32) + foreach SGD, and at N > 1 torch DDP over its own RCCL process group (the reference's
    ``DDP(model, device_ids=[gpu_id])``, multigpu.py:89).  Same timing rule as the ddpx line: barrier +
    synchronize on both sides, max over ranks.  Collective.

    Never raises: any failure on any rank is agreed over the CPU group at the phase boundaries and returned as
    ``{"error": ...}`` on every rank (an optional comparison must not cost the job its line).
    Phase 1 (local: data, fault injection) is always met by every rank; a rank failing later, inside the stock
    DDP's own collectives, is covered by the bounded tail (:func:`_arm_tail_watchdog`) when the stock run comes
    after the ddpx line."""
    import torch
    import torch.distributed as dist
    from ddpx.runtime.graphs import agree_all_ranks
    from ddpx.utils.faults import maybe_inject
    a = argparse.Namespace(**vars(args))
    a.impl, a.torch_amp = "torch", args.dtype != "fp32"
    cuda = device.type == "cuda"
    use_ddp = world > 1 or bool(getattr(args, "stock_ddp", 0))
    err, group, loader = None, None, None

    def fail(e):
        return f"{type(e).__name__}: {e}"[:400]

    def sync():
        if cuda:
            torch.cuda.synchronize()

    try:  # phase 1: local only
        maybe_inject("stock", rank=rank)
        loader = make_data(a, device, rank, world)  # the stock model's own (NCHW / flat fp32) input layout
    except Exception as e:  # noqa: BLE001
        err = fail(e)
    if not agree_all_ranks(err is None):
        return {"error": err or "another rank failed the stock recipe"}
    dt = None
    try:  # phase 2: the stock process group, model, DDP and its warm-up steps
        if use_ddp:
            import datetime
            group = dist.new_group(backend="nccl" if cuda else "gloo", timeout=datetime.timedelta(seconds=120))
        _, _, _, _, run = torch_runner(a, device, world, loader, idx_all, full, group=group)
        maybe_inject("stock_run", rank=rank)
        run(0, 5)
        sync()
    except Exception as e:  # noqa: BLE001
        err = fail(e)
    ok = agree_all_ranks(err is None)
    if ok:
        try:  # phase 3: the timed steps
            sync()
            t0 = time.perf_counter()
            run(5, args.stock_steps)
            sync()
            dt = time.perf_counter() - t0
        except Exception as e:  # noqa: BLE001
            err = fail(e)
        ok = agree_all_ranks(err is None)
    if group is not None and ok:  # a failed group is left alone: tearing it down could block on its peers
        try:
            dist.destroy_process_group(group)
        except Exception:  # noqa: BLE001
            pass
    if not ok:
        return {"error": err or "another rank failed the stock recipe"}
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    dt /= args.stock_steps
    recipe = "torch.nn + " + ("fp32" if args.dtype == "fp32" or not cuda else "bf16 autocast") + " + foreach SGD"
    if use_ddp:
        recipe += " + torch DDP (" + ("RCCL" if cuda else "gloo") + ", 25/1 MiB buckets)"
    return {"ms_per_step": round(dt * 1000.0, 4), "samples_per_sec": round(world * args.batch_size / dt, 2),
            "recipe": recipe, "steps": args.stock_steps}


def _vs_stock(value, stock):
    return round(value / stock["samples_per_sec"], 4) if (stock and "samples_per_sec" in stock) else None


def _arm_tail_watchdog(seconds: float):
    """After the headline line is out: end this rank with status 0 if the optional tail (the stock torch-DDP
    comparison, teardown) has not finished within ``seconds`` — a stuck stock collective must not turn a
    measured job into a failed one."""
    import threading

    def fire():
        print(f"bench.py: optional tail (stock comparison / teardown) exceeded {seconds:.0f} s; exiting 0 "
              "(the ddpx line was already printed)", file=sys.stderr, flush=True)
        sys.stdout.flush()
        os._exit(0)
    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


def replica_digest(net, flat=None):
    """SHA-256 of this rank's fp32 master weights and optimizer state, byte for byte (after consolidate)."""
    import hashlib
    f = flat if flat is not None else net.flat
    h = hashlib.sha256()
    for t in [f.master] + [f.state_tensors[k] for k in sorted(f.state_tensors)]:
        h.update(t.detach().cpu().contiguous().numpy().tobytes())
    return h.hexdigest()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    if needs_self_launch(args):
        sys.exit(self_launch(args, argv))

    import torch
    import torch.distributed as dist

    rank, world, local = setup_dist(args)
    resolve_defaults(args, world)
    cpu = args.device == "cpu"
    if args.comm == "host" or cpu:
        args.no_graph = True
    from ddpx.models import native_kernels_for
    if args.impl == "ddpx" and not native_kernels_for(args.model, "fp32" if args.dtype == "fp32" else "bf16",
                                                      args.kernels):
        # torch ops under the ddpx engine (--kernels torch: MIOpen / hipBLASLt) run eagerly: capturing torch's
        # autograd with AccumulateGrad nodes made by the eager warm-up steps crashed the process (exit -11)
        args.no_graph = True
    device = torch.device("cpu") if cpu else torch.device("cuda", local)
    loader = make_data(args, device, rank, world)
    idx_all = loader._epoch_indices()
    nb = len(loader)
    full = [i for i in range(nb) if (i + 1) * args.batch_size <= idx_all.numel()]
    bs = args.batch_size

    def sync():
        if not cpu:
            torch.cuda.synchronize()

    comm = make_comm(args, device, world)
    if getattr(args, "calibrate", False):
        calibrate_plan(args, device, world, loader, idx_all, full, comm, rank=rank)
    if not cpu:
        from ddpx.runtime.graphs import assert_no_capture
        assert_no_capture("before building the timed engine")
    eng = make_runner(args, device, world, loader, idx_all, full, comm)
    model, net, opt, sched, run, runner = eng.model, eng.net, eng.opt, eng.sched, eng.run, eng.runner

    stock = None
    if args.stock_ref and args.stock_first:
        # the baseline first (same process, same data), then the ddpx warm-up and timed steps
        stock = measure_stock_same_run(args, device, world, rank, idx_all, full)
    # warm-up (includes graph capture for ddpx).  The stock recipe is timed between the capture and the last
    # warm-up replays (--stock_between, default): the GPU's clocks ramp for ~10 ms of sustained load
    # (profiles/r5_window: per-step GPU time falls from ~0.26 to ~0.245 ms over a 60-step window), and a capture
    # leaves the GPU idle for a while; this way the timed window starts on a GPU that has just been busy.  The
    # ddpx engine still runs exactly --warmup untimed steps before its --steps timed ones.
    loss = None
    w1 = min(args.warmup, 2)
    if w1:
        loss = run(0, w1)
    if runner is not None and args.warmup > w1:
        runner.capture_now()
    if args.stock_ref and not args.stock_first and args.stock_between:
        stock = measure_stock_same_run(args, device, world, rank, idx_all, full)
    if args.warmup > w1:
        loss = run(w1, args.warmup - w1)
    sync()
    if world > 1:
        dist.barrier()
    sync()
    trace = os.environ.get("DDPX_STEP_TRACE") == "1" and not cpu
    evs = []
    t0 = time.perf_counter()
    if trace:
        # diagnostics only: one event per step (no host sync inside the window) -> per-step GPU time on stderr
        evs.append(torch.cuda.Event(enable_timing=True))
        evs[-1].record()
        for i in range(args.steps):
            loss = run(args.warmup + i, 1)
            evs.append(torch.cuda.Event(enable_timing=True))
            evs[-1].record()
    else:
        loss = run(args.warmup, args.steps)
    sync()
    t1 = time.perf_counter()
    if trace:
        print(json.dumps({"step_ms": [round(a.elapsed_time(b), 4) for a, b in zip(evs, evs[1:])],
                          "host_ms": round((t1 - t0) * 1000, 3)}), file=sys.stderr)
    if world > 1:
        dist.barrier()
    elapsed = t1 - t0
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device="cpu" if (args.impl == "ddpx" or cpu) else device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    final_loss = float(loss.float().item()) if loss is not None else float("nan")
    multi = world > 1 or args.ddp_single
    ddpx_ddp = multi and args.impl == "ddpx"
    cstats = net.comm_stats() if (ddpx_ddp and hasattr(net, "comm_stats")) else None
    consistent = None
    buckets_mb = None
    if ddpx_ddp:
        # outside the timed region: replicas must hold bit-identical fp32 weights and optimizer state
        net.consolidate()
        allck = [None] * world
        dist.all_gather_object(allck, replica_digest(net))
        consistent = all(c == allck[0] for c in allck)
        esz = net.flat.grad.element_size()
        buckets_mb = [round((e - s) * esz / 2 ** 20, 3) for s, e in net.bucket_ranges]
    digest = None
    if args.digest and args.impl == "ddpx":
        from ddpx.runtime.flat_params import flat_of
        digest = allck[rank] if ddpx_ddp else replica_digest(None, flat=flat_of(model))
    stock_after = bool(args.stock_ref and not args.stock_first and not args.stock_between)
    if stock_after and not multi:  # one process: no second communicator, the line can carry the comparison
        stock = measure_stock_same_run(args, device, world, rank, idx_all, full)
        stock_after = False
    value = world * bs * args.steps / elapsed
    ms = elapsed / args.steps * 1000.0
    metric = "samples_per_sec_whole_node"
    model_name = {"mlp": f"toy-mlp-3072x{args.hidden}x{args.layers}",
                  "mlp_wide": f"wide-mlp-3072x{args.hidden}x{args.layers}",
                  "vgg": "vgg11-cifar", "deepnn": "deepnn-cifar"}[args.model]
    base = baseline_value(f"{args.model}_x{world}") if args.impl == "ddpx" else None
    if cpu or (args.impl == "ddpx" and args.dtype == "fp32"):
        dtype = "fp32"
    elif args.model.startswith("mlp"):
        dtype = "mxfp8/bf16" if (args.fp8 and args.impl == "ddpx") else "bf16"
    else:
        dtype = "bf16" if (args.impl == "ddpx" or args.torch_amp) else "fp32"
    if ddpx_ddp:
        grad_comm = f"{args.grad_dtype} {'reduce-scatter+all-gather (ZeRO-1)' if args.shard_optimizer else 'all-reduce'} avg"
    elif multi:
        grad_comm = "fp32 all-reduce avg (torch DDP)"
    else:
        grad_comm = None
    rec = {
        "metric": metric, "value": round(value, 2), "unit": "samples/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms, 4), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": (round(value / base, 4) if base else None), "dtype": dtype,
        "data": ("synthetic (CIFAR-shaped uint8, " + ("host" if cpu else "GPU") +
                 "-resident, crop+flip augment per step; random-init weights)"),
        "config": {"model": model_name, "global_batch": bs * world, "per_gpu_batch": bs, "seq_len": None,
                   "parallelism": f"dp{world}", "device": args.device, "impl": args.impl,
                   "kernels": (args.kernels if args.impl == "ddpx" else None),
                   "launcher": os.environ.get(LAUNCHER_ENV, "torchrun/external" if world > 1 else "none"),
                   "comm": (args.comm if ddpx_ddp else None),
                   "comm_fallback": getattr(args, "comm_fallback", None),
                   "rccl": ({"channels": args.rccl_channels, "proto": os.environ.get("NCCL_PROTO")}
                            if (ddpx_ddp and args.comm == "rccl") else None),
                   "sim_world": (args.sim_world if (args.ddp_single and args.sim_world) else None),
                   "graph": bool(runner is not None and runner.use_graph),
                   "graph_steps": (args.graph_steps if (runner is not None and runner.use_graph) else None),
                   "graph_schedule": (runner.schedule(args.steps) if (runner is not None and runner.use_graph)
                                      else None),
                   "prefetch_batch": bool(getattr(args, "prefetch_batch", 0)),
                   "graph_error": (runner.graph_error if runner is not None else None),
                   "optimizer": "sgd(lr=0.4 one-cycle, m=0.9, wd=5e-4)" + (
                       " fused-into-backward" if (args.impl == "ddpx" and not multi and args.fused_optimizer
                                                  and not cpu) else "") + (
                       " ZeRO-1 (fp32 master + momentum sharded over ranks, bf16 compute copy all-gathered; same "
                       "update arithmetic as the replicated step)" if (ddpx_ddp and args.shard_optimizer) else ""),
                   "grad_comm": grad_comm, "grad_dtype": args.grad_dtype if args.impl == "ddpx" else "fp32",
                   "bucket_cap_mb": args.bucket_cap_mb, "first_bucket_mb": args.first_bucket_mb,
                   "bucket_plan": (("calibrated" if getattr(args, "calibration", None) else "explicit")
                                   if ddpx_ddp else None),
                   "calibration": getattr(args, "calibration", None),
                   "buckets_mb": buckets_mb, "chunk_mb": args.chunk_mb or None,
                   "sharded_optimizer": bool(args.shard_optimizer) if ddpx_ddp else None,
                   "defer_gather": bool(args.defer_gather) if (ddpx_ddp and args.shard_optimizer) else None,
                   "comm_side_optimizer": (bool(args.comm_side_optimizer)
                                           if (ddpx_ddp and args.shard_optimizer) else None),
                   "overlap_optimizer": bool(args.overlap_optimizer) if multi else None,
                   "side_stream_optimizer": (bool(getattr(args, "side_optimizer", 0))
                                             if (ddpx_ddp and not args.shard_optimizer) else None),
                   "final_loss": round(final_loss, 4), "ddp": bool(multi),
                   "replicas_consistent": consistent,
                   "master_digest": digest,
                   "comm_ms_per_step": round(cstats["comm_ms"], 4) if cstats else None,
                   "comm_exposed_ms_per_step": round(cstats["comm_exposed_ms"], 4) if cstats else None,
                   "stock_same_run": (stock if not stock_after else
                                      {"placement": "after this line (DDP job): result on stderr / --json_out"}),
                   "vs_stock_same_run": _vs_stock(value, stock)},
    }
    if rank == 0:
        line = json.dumps(rec)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "a") as f:
                f.write(line + "\n")
    if stock_after:
        # the headline line is out; the stock torch-DDP comparison (a second NCCL communicator) runs now, bounded
        _arm_tail_watchdog(float(os.environ.get("DDPX_BENCH_TAIL_S", "300")))
        stock = measure_stock_same_run(args, device, world, rank, idx_all, full)
        if rank == 0:
            tail = json.dumps({"stock_same_run": stock, "vs_stock_same_run": _vs_stock(value, stock),
                               "for_metric": metric, "n_gpus": world})
            print("STOCK " + tail, file=sys.stderr, flush=True)
            if args.json_out:
                with open(args.json_out, "a") as f:
                    f.write(tail + "\n")
    if multi:
        if args.impl == "ddpx" and hasattr(net, "close"):
            net.close()
        if comm is not None:
            comm.close()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
