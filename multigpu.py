"""Multi-GPU data-parallel entry point (same CLI as the reference's multigpu.py).

    python multigpu.py TOTAL_EPOCHS SAVE_EVERY [--batch_size 512] [ddpx flags]

Spawns one process per MI355X with ``mp.spawn`` exactly like the reference
(/root/reference/multigpu.py:254-263), or — when launched by torchrun
(``RANK``/``WORLD_SIZE``/``LOCAL_RANK`` in the environment) — runs as that
worker.  Each rank: rendezvous over the c10d TCPStore, native RCCL
communicator, ddpx DistributedDataParallel (bucketed all-reduce overlapped with
backward), DistributedSampler-identical sharding, rank-0 checkpointing, and a
full (unsharded) evaluation per rank as in the reference.  ``--device cpu``
runs the same program over gloo for testing.
"""
from __future__ import annotations

import os

import torch
import torch.multiprocessing as mp

from ddpx.data.datasets import get_datasets as getTrainingData  # noqa: F401  (reference name)
from ddpx.models import VGG, DeepNN, MLP  # noqa: F401
from ddpx.train.app import (apply_debug_env, build_parser, ddp_setup, load_train_objs, main_multi,  # noqa: F401
                            maybe_profile, prepare_dataloader)
from ddpx.train.evaluate import evaluate  # noqa: F401
from ddpx.train.trainer import Trainer  # noqa: F401
from ddpx.utils.size import Byte, GiB, KiB, MiB, get_model_size  # noqa: F401


def main(rank: int, world_size: int, save_every: int, total_epochs: int, batch_size: int, args=None):
    """Reference signature main(rank, world_size, save_every, total_epochs, batch_size)."""
    if args is None:
        args = build_parser("simple distributed training job").parse_args([str(total_epochs), str(save_every)])
    args.total_epochs, args.save_every, args.batch_size = total_epochs, save_every, batch_size
    main_multi(rank, world_size, args)


if __name__ == "__main__":
    parser = build_parser("simple distributed training job")
    args = parser.parse_args()
    maybe_profile(args)  # --profile: re-run as a child under rocprofv3 (before any GPU use)
    apply_debug_env(args)
    if "RANK" in os.environ and "WORLD_SIZE" in os.environ:  # torchrun / elastic launch
        main(int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"]), args.save_every, args.total_epochs,
             args.batch_size, args)
    else:
        if args.nprocs:
            world_size = args.nprocs
        else:
            # the reference's world_size = torch.cuda.device_count() (multigpu.py:262), counted without
            # initialising HIP here (environment / KFD topology, ddpx.utils.devices): the ranks are fork+exec'd,
            # which must not happen from a process that touched the GPU
            from ddpx.utils.devices import visible_gpu_count
            if args.device == "cpu":
                world_size = 2  # CPU/gloo rehearsal: two processes unless --nprocs says otherwise
            else:
                world_size = visible_gpu_count()
                if world_size < 1:
                    raise SystemExit("multigpu.py: no GPU is visible (the reference's torch.cuda.device_count() "
                                     "would be 0); pass --device cpu for the gloo rehearsal or --nprocs N")
        if args.device != "cpu":
            from ddpx.utils.devices import assert_hip_uninitialised
            assert_hip_uninitialised("multigpu.py: mp.spawn")
        mp.spawn(main, args=(world_size, args.save_every, args.total_epochs, args.batch_size, args),
                 nprocs=world_size)
