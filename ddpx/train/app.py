"""Orchestration shared by ``singlegpu.py`` and ``multigpu.py``.

Mirrors the reference's ``load_train_objs`` / ``prepare_dataloader`` /
``main`` / ``ddp_setup`` / ``__main__`` (``/root/reference/singlegpu.py:132-263``,
``multigpu.py:24-33,122-263``), keeping the positional CLI
(``TOTAL_EPOCHS SAVE_EVERY [--batch_size 512]``), the stdout lines and the
``checkpoint.pt`` format, and adding the SURVEY §5.6 flags.
"""
from __future__ import annotations

import argparse
import os
import subprocess
import sys
import time

import torch
import torch.distributed as dist

from ..data.datasets import get_datasets
from ..data.loader import DeviceLoader
from ..data.sampler import DistributedIndexSampler
from ..models import build_model
from ..optim.schedule import one_cycle, resolve_steps_per_epoch
from ..optim.sgd import SGD
from ..parallel.comm import HostStagedComm, RcclComm, TorchComm, set_rccl_protocol
from ..parallel.sync_bn import convert_sync_batchnorm
from ..parallel.ddp import DistributedDataParallel
from ..runtime.setup import prepare_model
from ..utils.metrics import MetricsWriter
from ..utils.size import MiB, get_model_size
from .checkpoint import FULL_CKPT_PATH, load_full_checkpoint
from .evaluate import evaluate
from .trainer import Trainer

REF_LR = 0.4
REF_MOMENTUM = 0.9
REF_WD = 5e-4


def build_parser(description: str) -> argparse.ArgumentParser:
    p = argparse.ArgumentParser(description=description)
    p.add_argument("total_epochs", type=int, help="Total epochs to train the model")
    p.add_argument("save_every", type=int, help="How often to save a snapshot")
    p.add_argument("--batch_size", default=512, type=int, help="Input batch size on each device (default: 512)")
    p.add_argument("--model", default="vgg", choices=["vgg", "deepnn", "mlp", "mlp_wide"])
    p.add_argument("--hidden", type=int, default=None, help="MLP hidden width (default 4096, wide 16384)")
    p.add_argument("--layers", type=int, default=3, help="MLP Linear layers (default 3)")
    p.add_argument("--data", default="auto", choices=["auto", "cifar10", "synthetic"])
    p.add_argument("--data_root", default="data/cifar10")
    p.add_argument("--train_size", type=int, default=50000, help="synthetic train-set size")
    p.add_argument("--test_size", type=int, default=10000, help="synthetic test-set size")
    p.add_argument("--dtype", default="fp32", choices=["fp32", "bf16", "auto"],
                   help="compute precision: fp32 (default: the reference's recipe, /root/reference/singlegpu.py:134-141 "
                        "trains without autocast) or bf16 (MFMA bf16 with fp32 master weights; auto = bf16 on a GPU)")
    p.add_argument("--device", default="auto", choices=["auto", "cuda", "cpu"])
    p.add_argument("--kernels", default="auto", choices=["auto", "native", "torch"],
                   help="auto / native: the hand-written HIP kernels for every model and precision (measured faster "
                        "than MIOpen / hipBLASLt, profiles/r4_f32); torch: torch ops (MIOpen / hipBLASLt) under the "
                        "ddpx engine (flat store, fused SGD, native DDP)")
    p.add_argument("--bucket_cap_mb", type=float, default=None,
                   help="DDP bucket cap (default: calibrated on the node at start-up, see --bucket_plan)")
    p.add_argument("--first_bucket_mb", type=float, default=None)
    p.add_argument("--bucket_plan", default="calibrated", choices=["calibrated", "default"],
                   help="distributed: time a few training steps of every candidate gradient-communication plan "
                        "(bucket caps; replicated vs --shard_optimizer) on this node before training and use the "
                        "fastest (ddpx.parallel.calibrate); default = torch DDP's 25 / 1 MiB caps")
    p.add_argument("--steps_per_epoch", default="compat", help="'compat' (98/49 as the reference), 'auto' or N")
    p.add_argument("--seed", type=int, default=None, help="seed model init (reference: unseeded)")
    p.add_argument("--lr", type=float, default=REF_LR, help="peak LR of the one-cycle schedule (reference 0.4)")
    p.add_argument("--graph", action="store_true",
                   help="capture the training step in a HIP graph (default on the GPU for the native kernels)")
    p.add_argument("--no_graph", action="store_true", help="eager training steps")
    p.add_argument("--grad_dtype", default="fp32", choices=["fp32", "bf16"], help="gradient buffer / all-reduce dtype")
    p.add_argument("--overlap_optimizer", action="store_true",
                   help="per-bucket SGD as all-reduces land (default when distributed)")
    p.add_argument("--no_overlap_optimizer", action="store_true", help="one SGD pass after all buckets landed")
    p.add_argument("--no_fused_optimizer", action="store_true",
                   help="single GPU: run SGD as its own pass instead of inside the backward kernels")
    p.add_argument("--comm", default="rccl", choices=["rccl", "torch", "host"],
                   help="GPU collective backend (host: gloo-staged, lets several ranks share one GPU)")
    p.add_argument("--rccl_channels", default=None,
                   help="RCCL channel (CTA) bounds of the gradient communicator: N or MIN:MAX (default RCCL's)")
    p.add_argument("--rccl_proto", default=None, help="NCCL_PROTO for this job (Simple, LL, LL128)")
    p.add_argument("--shard_optimizer", action="store_true",
                   help="ZeRO-1: reduce-scatter grads, each rank updates its shard, all-gather params")
    p.add_argument("--chunk_mb", type=float, default=None,
                   help="split weights larger than this (MB of gradient) into row-chunk DDP buckets")
    p.add_argument("--side_optimizer", type=int, default=0,
                   help="DDP with optimizer overlap, replicated optimizer: each bucket's SGD update on a side stream "
                        "behind its all-reduce and its weights' last read in backward (0: on the compute stream)")
    p.add_argument("--comm_side_optimizer", action="store_true",
                   help="with --shard_optimizer on the RCCL path: shard updates on the communicator stream behind "
                        "each reduce-scatter (one join per step instead of one per bucket)")
    p.add_argument("--defer_gather", action="store_true",
                   help="with --shard_optimizer: all-gather updated shards at the start of the next forward, "
                        "overlapped with it (MLP native path)")
    p.add_argument("--sync_bn", action="store_true", help="SyncBatchNorm (reference: commented out)")
    p.add_argument("--resume", action="store_true", help=f"resume from {FULL_CKPT_PATH}")
    p.add_argument("--full_checkpoint", action="store_true", help=f"also write {FULL_CKPT_PATH}")
    p.add_argument("--metrics", default=None, help="JSON-lines metrics file")
    p.add_argument("--eval_batch", type=int, default=512)
    p.add_argument("--no_eval", action="store_true")
    p.add_argument("--nprocs", type=int, default=None, help="multigpu: processes to spawn (default: #GPUs)")
    p.add_argument("--fp8", action="store_true", help="MLP: MX-FP8 hidden-layer forward / weight-gradient GEMMs")
    p.add_argument("--profile", default=None, metavar="DIR",
                   help="re-run this command under rocprofv3 --kernel-trace --stats, output in DIR")
    p.add_argument("--debug", action="store_true",
                   help="serialised kernels (AMD_SERIALIZE_KERNEL=3, HIP_LAUNCH_BLOCKING=1) and DDP "
                        "bucket-order validation across ranks on every step")
    p.add_argument("--fault_step", type=int, default=None,
                   help="fault injection: rank --fault_rank raises at this global step")
    p.add_argument("--fault_rank", type=int, default=0)
    return p


def maybe_profile(args, argv=None) -> None:
    """``--profile DIR``: run this same command as a CHILD under rocprofv3 and exit with its code.

    Done before anything touches the GPU (rocprofv3's library initialises it in the child; this
    process never does), per SURVEY §5.1.  Output: DIR/<pid>/..._kernel_stats.csv etc.
    """
    if not getattr(args, "profile", None):
        return
    argv = list(sys.argv if argv is None else argv)
    rest, skip = [], False
    for a in argv[1:]:
        if skip:
            skip = False
            continue
        if a == "--profile":
            skip = True
            continue
        if a.startswith("--profile="):
            continue
        rest.append(a)
    out = os.path.abspath(args.profile)
    os.makedirs(out, exist_ok=True)
    cmd = ["rocprofv3", "--kernel-trace", "--stats", "--output-format", "csv", "-d", out, "--", sys.executable,
           os.path.abspath(argv[0]), *rest]
    env = dict(os.environ, TMPDIR="/tmp")
    print("profiling:", " ".join(cmd), flush=True)
    rc = subprocess.run(cmd, env=env).returncode
    sys.exit(rc)


def apply_debug_env(args) -> None:
    """``--debug``: kernel serialisation for fault localisation (must precede GPU initialisation)."""
    if getattr(args, "debug", False):
        os.environ.setdefault("AMD_SERIALIZE_KERNEL", "3")
        os.environ.setdefault("HIP_LAUNCH_BLOCKING", "1")
        os.environ.setdefault("DDPX_DEBUG", "1")


def resolve_device(args, local_rank: int = 0) -> torch.device:
    if args.device == "cpu" or (args.device == "auto" and not torch.cuda.is_available()):
        return torch.device("cpu")
    return torch.device("cuda", local_rank)


def resolve_data(args):
    kind = args.data
    if kind == "auto":
        have = os.path.isdir(os.path.join(args.data_root, "cifar-10-batches-bin")) or os.path.isdir(
            os.path.join(args.data_root, "cifar-10-batches-py"))
        kind = "cifar10" if have else "synthetic"
    return kind


def input_layout(model, device, dtype):
    if getattr(model, "input_layout", None):
        return model.input_layout(device)
    return "nchw_f32"


_CONFIG = None  # module-level run configuration the reference-signature helpers default to


def set_config(args) -> None:
    """Make ``args`` the configuration ``load_train_objs()`` / ``prepare_dataloader(ds, bs)`` use."""
    global _CONFIG
    _CONFIG = args


def current_config():
    """The active configuration: the one ``run()`` / ``set_config`` installed, else the reference's defaults
    (``TOTAL_EPOCHS=20 SAVE_EVERY=5``, VGG, lr 0.4, batch 512)."""
    global _CONFIG
    if _CONFIG is None:
        _CONFIG = build_parser("ddpx").parse_args(["20", "5"])
    return _CONFIG


def load_train_objs(args=None, device=None, distributed: bool = False, world_size: int = 1,
                    loader_len_hint: int | None = None, comm=None):
    """(train_set, model, optimizer, test_set, scheduler) — the reference's factory, ddpx engine underneath.

    Callable exactly as the reference does, ``load_train_objs()`` (``/root/reference/singlegpu.py:132``):
    every argument defaults from :func:`current_config` (device: the first GPU, else the CPU).

    ``--sync_bn`` (reference: the commented-out ``convert_sync_batchnorm`` at
    ``/root/reference/multigpu.py:127``): the native VGG merges BatchNorm statistics across ranks inside its
    own kernels' sequence (``model.sync_bn_comm``); the torch-op path swaps every BatchNorm2d for
    :class:`SyncBatchNorm2d` on ``comm`` before the flat parameter store is built.
    """
    if args is None:
        args = current_config()
    if device is None:
        device = resolve_device(args)
    if loader_len_hint is None:
        train_n = args.train_size if resolve_data(args) == "synthetic" else 50000
        loader_len_hint = _loader_len(train_n, args.batch_size, world_size)
    kind = resolve_data(args)
    train_set, test_set = get_datasets(kind, args.data_root, seed=0, train_size=args.train_size,
                                       test_size=args.test_size)
    if args.seed is not None:
        torch.manual_seed(args.seed)
    model, optimizer = build_model_and_optimizer(args, device, distributed, comm)
    spe = resolve_steps_per_epoch(args.steps_per_epoch, loader_len_hint, distributed)
    scheduler = one_cycle(optimizer, spe)
    return train_set, model, optimizer, test_set, scheduler


def build_model_and_optimizer(args, device, distributed: bool = False, comm=None):
    """The model (native kernels where ``build_model`` puts them, SyncBatchNorm on request) in a flat parameter
    store, and its ddpx SGD (the reference's lr 0.4 / momentum 0.9 / wd 5e-4)."""
    model = build_model(args.model, hidden=args.hidden, layers=args.layers, dtype=args.dtype, device=device,
                        kernels=args.kernels, fp8=getattr(args, "fp8", False))
    if getattr(args, "sync_bn", False) and distributed:
        if getattr(model, "use_native", False) and device.type == "cuda":
            # native path, bf16 and fp32: the BN kernels merge statistics across ranks themselves
            # (ops/vgg_native.py, ops/f32.py bn_forward / bn_backward with comm)
            model.sync_bn_comm = comm
        else:
            model = convert_sync_batchnorm(model, comm)
    if args.graph and device.type == "cuda" and not getattr(model, "use_native", True):
        # torch-op models (--kernels torch: MIOpen / hipBLASLt ops) step eagerly: capturing torch's autograd with
        # AccumulateGrad nodes created by the eager warm-up steps is not supported (it crashed in bench.py)
        if getattr(args, "graph_explicit", True):
            print("note: --graph ignored for the torch-op model path", flush=True)
        args.graph = False
    prepare_model(model, device, grad_dtype=torch.bfloat16 if args.grad_dtype == "bf16" else torch.float32)
    optimizer = SGD(model.parameters(), lr=args.lr, momentum=REF_MOMENTUM, weight_decay=REF_WD,
                    capturable=bool(args.graph and device.type == "cuda"),
                    fused_backward=bool(not distributed and device.type == "cuda" and not args.no_fused_optimizer))
    return model, optimizer


def resolve_run_defaults(args, device, distributed: bool):
    """Defaults that depend on where the run happens (``run()``): HIP-graph steps on the GPU, and when
    distributed the per-bucket optimizer overlap and the node-calibrated bucket plan — the tuned path the
    benchmark measures, behind the reference's own entry points."""
    args.graph_explicit = bool(getattr(args, "graph", False))
    args.graph = bool(device.type == "cuda" and not getattr(args, "no_graph", False))
    if distributed:
        args.overlap_optimizer = bool(args.overlap_optimizer or not getattr(args, "no_overlap_optimizer", False))
    args.calibrate = bool(distributed and getattr(args, "bucket_plan", "default") == "calibrated"
                          and (args.bucket_cap_mb is None or args.first_bucket_mb is None))
    if not args.calibrate:
        if args.bucket_cap_mb is None:
            args.bucket_cap_mb = 25.0
        if args.first_bucket_mb is None:
            args.first_bucket_mb = 1.0


def make_ddp(args, model, optimizer, comm):
    net = DistributedDataParallel(model, comm=comm, bucket_cap_mb=args.bucket_cap_mb,
                                  first_bucket_mb=args.first_bucket_mb,
                                  overlap_optimizer=args.overlap_optimizer,
                                  shard_optimizer=args.shard_optimizer, chunk_mb=args.chunk_mb,
                                  defer_gather=args.defer_gather,
                                  comm_side_optimizer=args.comm_side_optimizer,
                                  side_stream_optimizer=bool(getattr(args, "side_optimizer", 0)))
    if args.overlap_optimizer or args.shard_optimizer:
        net.attach_optimizer(optimizer)
    return net


def _loss_of(net, model, x, y):
    if hasattr(model, "forward_loss"):
        loss, _ = net.forward_loss(x, y)
        return loss
    return torch.nn.functional.cross_entropy(net(x), y)


def calibrate_bucket_plan(args, device, comm, batch, world_size):
    """Start-up calibration of the DDP bucket plan (``ddpx.parallel.calibrate``), the same as ``bench.py``'s:
    every candidate (bucket caps; replicated, or ZeRO-1 when ``--shard_optimizer`` is given) is built for real
    on this node and a few training steps of it are timed (graph-captured when the run's steps are), and the
    fastest one's caps are written into ``args``.  Collective.  Returns {name, step_ms}."""
    import gc
    from ..parallel.calibrate import calibrate_by_step, candidate_plans
    from ..runtime.flat_params import flat_of
    from ..runtime.graphs import try_capture
    probe, _ = build_model_and_optimizer(args, device, True, comm)
    f = flat_of(probe)
    numels = list(f.numels)
    shapes = [tuple(p.shape) for p in f.params]
    shadow_only = [id(p) in f.shadow_only for p in f.params]
    del probe, f
    plans = [p for p in candidate_plans(numels, shadow_only, world_size, allow_shard=bool(args.shard_optimizer),
                                        shapes=None if args.chunk_mb else shapes)
             if p["shard"] == bool(args.shard_optimizer)]
    if not plans:
        args.bucket_cap_mb = 25.0 if args.bucket_cap_mb is None else args.bucket_cap_mb
        args.first_bucket_mb = 1.0 if args.first_bucket_mb is None else args.first_bucket_mb
        return {"chosen": "default", "step_ms": {}}
    x, y = batch
    cuda = device.type == "cuda"
    sync = torch.cuda.synchronize if cuda else (lambda: None)

    def make_trial(plan):
        a = argparse.Namespace(**vars(args))
        a.bucket_cap_mb = plan["bucket_cap_mb"] if args.bucket_cap_mb is None else args.bucket_cap_mb
        a.first_bucket_mb = plan["first_bucket_mb"] if args.first_bucket_mb is None else args.first_bucket_mb
        if not args.chunk_mb:
            a.chunk_mb = plan.get("chunk_mb")
        model, opt = build_model_and_optimizer(a, device, True, comm)
        net = make_ddp(a, model, opt, comm)
        one = torch.ones((), device=device)
        st = {"k": 0, "g": None}

        def body(xx, yy):
            opt.zero_grad()
            loss = _loss_of(net, model, xx, yy)
            loss.backward(one)
            opt.step()
            return loss

        def step():
            if a.graph and st["k"] >= 2 and st["g"] is None:
                st["g"], _ = try_capture(body, x, y, net, opt, comm=comm)
                if st["g"] is None:
                    a.graph = False
            if st["g"] is not None:
                st["g"]()
            else:
                body(x, y)
            st["k"] += 1

        def close():
            sync()
            st["g"] = None
            net.close()
            gc.collect()
            if cuda:
                torch.cuda.empty_cache()
        return step, close

    chosen, table = calibrate_by_step(plans, make_trial, sync=sync, warm=3, reps=5 if cuda else 2,
                                      rounds=3 if cuda else 1)
    if args.bucket_cap_mb is None:
        args.bucket_cap_mb = chosen["bucket_cap_mb"]
    if args.first_bucket_mb is None:
        args.first_bucket_mb = chosen["first_bucket_mb"]
    if not args.chunk_mb:
        args.chunk_mb = chosen.get("chunk_mb")
    return {"chosen": chosen["name"], "step_ms": table}


def prepare_dataloader(dataset, batch_size: int, device=None, layout: str = "nchw_f32", rank: int = 0,
                       world_size: int = 1, seed: int = 0):
    """Shuffled training batches (``/root/reference/singlegpu.py:174``: ``DataLoader(dataset, batch_size,
    pin_memory=True, shuffle=True)``) produced on ``device`` by the GPU-resident loader.  Callable as
    ``prepare_dataloader(dataset, batch_size)``: NCHW fp32 batches on the configured device."""
    if device is None:
        device = resolve_device(current_config())
    sampler = DistributedIndexSampler(len(dataset), world_size, rank, shuffle=True, seed=seed)
    return DeviceLoader(dataset, batch_size, device, sampler=sampler, train=True, layout=layout, seed=seed + rank)


def _loader_len(n, batch_size, world_size):
    per_rank = -(-n // world_size)
    return -(-per_rank // batch_size)


def run(args, rank: int = 0, world_size: int = 1, local_rank: int = 0, distributed: bool = False):
    set_config(args)
    device = resolve_device(args, local_rank)
    if device.type == "cuda":
        torch.cuda.set_device(device)
    train_n = args.train_size if resolve_data(args) == "synthetic" else 50000
    comm = None
    if distributed:
        if device.type == "cuda" and args.comm == "rccl":
            set_rccl_protocol(getattr(args, "rccl_proto", None))
            comm = RcclComm(device, channels=getattr(args, "rccl_channels", None))
        elif device.type == "cuda" and args.comm == "host":
            comm = HostStagedComm()
        else:
            comm = TorchComm()
    resolve_run_defaults(args, device, distributed)
    dataset, model, optimizer, testdata, scheduler = load_train_objs(
        args, device, distributed, world_size, _loader_len(train_n, args.batch_size, world_size), comm)
    layout = input_layout(model, device, args.dtype)
    train_data = prepare_dataloader(dataset, args.batch_size, device, layout, rank, world_size)
    net = model
    if distributed:
        if args.calibrate:
            bs = min(args.batch_size, len(dataset))
            batch = train_data.make_batch(train_data._epoch_indices()[:bs], 0)
            cal = calibrate_bucket_plan(args, device, comm, batch, world_size)
            if rank == 0:
                print(f"bucket plan: calibrated {cal['chosen']} (first {args.first_bucket_mb:g} MB, cap "
                      f"{args.bucket_cap_mb:g} MB; training step ms per candidate: {cal['step_ms']})", flush=True)
        net = make_ddp(args, model, optimizer, comm)
    metrics = MetricsWriter(args.metrics, rank) if args.metrics else None
    trainer = Trainer(net, train_data, optimizer, local_rank if device.type == "cuda" else rank, args.save_every,
                      scheduler, distributed=distributed, rank=rank, graph=args.graph, metrics=metrics,
                      full_checkpoint=args.full_checkpoint)
    if args.fault_step is not None and rank == args.fault_rank:
        trainer.fault_step = args.fault_step
    if args.resume and os.path.exists(FULL_CKPT_PATH):
        trainer.start_epoch = load_full_checkpoint(FULL_CKPT_PATH, model, optimizer, scheduler,
                                                   map_location=device)
        if distributed:
            net._broadcast_state()

    start_time = time.time()
    trainer.train(args.total_epochs)
    if isinstance(net, DistributedDataParallel):
        net.consolidate()  # sharded optimizer: complete fp32 weights for eval / final state
    end_time = time.time()
    training_time = end_time - start_time
    print(f"Total training time: {training_time:.2f} seconds")

    fp32_model_size = get_model_size(model)
    print(f"fp32 model has size={fp32_model_size / MiB:.2f} MiB")
    if not args.no_eval:
        test_data = DeviceLoader(testdata, args.eval_batch, device, train=False, layout=layout)
        fp32_model_accuracy = evaluate(model, test_data)
        print(f"fp32 model has accuracy={fp32_model_accuracy:.2f}%")
    if metrics is not None:
        metrics.log(event="done", training_time=training_time)
        metrics.close()
    if comm is not None:
        if device.type == "cuda":
            torch.cuda.synchronize()
        if isinstance(net, DistributedDataParallel):
            net.close()
        comm.close()
    return model


# ------------------------------------------------------------------ multi
def ddp_setup(rank: int, world_size: int, device_type: str, comm: str = "rccl"):
    """Rendezvous (reference: multigpu.py:24-33).  Env MASTER_ADDR/PORT win over the defaults.

    With the native RCCL communicator the c10d group only bootstraps it (TCPStore) and carries
    CPU-side metadata, so it is gloo; ``--comm torch`` uses stock ProcessGroupNCCL (RCCL) instead.
    """
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "12355")
    if device_type == "cuda":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", rank)))
        backend = "gloo" if comm == "rccl" else "cpu:gloo,cuda:nccl"
    else:
        backend = "gloo"
    dist.init_process_group(backend=backend, rank=rank, world_size=world_size)


def main_multi(rank: int, world_size: int, args):
    """Per-process entry (mp.spawn target or torchrun worker)."""
    device_type = resolve_device(args).type
    ddp_setup(rank, world_size, device_type, args.comm)
    local_rank = int(os.environ.get("LOCAL_RANK", rank))
    try:
        run(args, rank=rank, world_size=world_size, local_rank=local_rank, distributed=True)
    finally:
        dist.destroy_process_group()
