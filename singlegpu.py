"""Single-device training entry point (same CLI as the reference's singlegpu.py).

    python singlegpu.py TOTAL_EPOCHS SAVE_EVERY [--batch_size 512] [ddpx flags]

Reference: /root/reference/singlegpu.py (VGG on CIFAR-10, SGD lr 0.4 momentum 0.9
wd 5e-4, one-cycle LambdaLR, checkpoint.pt every SAVE_EVERY epochs, final
time / size / accuracy prints).  The engine underneath is ddpx (MI355X-native
kernels, GPU-resident data); ``--device cpu`` runs the same recipe on the CPU.
"""
from __future__ import annotations

from ddpx.data.datasets import get_datasets as getTrainingData  # noqa: F401  (reference name)
from ddpx.models import VGG, DeepNN, MLP  # noqa: F401
from ddpx.train.app import (apply_debug_env, build_parser, load_train_objs, maybe_profile,  # noqa: F401
                            prepare_dataloader, run)
from ddpx.train.evaluate import evaluate  # noqa: F401
from ddpx.train.trainer import Trainer  # noqa: F401
from ddpx.utils.size import Byte, GiB, KiB, MiB, get_model_size  # noqa: F401


def main(device, total_epochs: int, save_every: int, batch_size: int, args=None):
    """Reference signature main(device, total_epochs, save_every, batch_size)."""
    if args is None:
        args = build_parser("simple single-device training job").parse_args([str(total_epochs), str(save_every)])
    args.total_epochs, args.save_every, args.batch_size = total_epochs, save_every, batch_size
    return run(args, rank=0, world_size=1, local_rank=device if isinstance(device, int) else 0, distributed=False)


if __name__ == "__main__":
    parser = build_parser("simple single-device training job")
    args = parser.parse_args()
    maybe_profile(args)  # --profile: re-run as a child under rocprofv3 (before any GPU use)
    apply_debug_env(args)
    device = 0
    main(device, args.total_epochs, args.save_every, args.batch_size, args)
