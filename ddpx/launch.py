"""torchrun-compatible launcher with single-node MI355X defaults.

    python -m ddpx.launch [--nproc-per-node N] SCRIPT [ARGS...]

Equivalent to ``python -m torch.distributed.run --nnodes 1 --nproc-per-node N --master-addr
127.0.0.1 --master-port P SCRIPT ARGS`` where N defaults to the number of visible GPUs (counted
without initialising HIP in the launcher) and P to a free port.  Every rank reads
RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* from the environment, as ``multigpu.py`` and
``bench.py`` do.  Options torchrun understands may be passed before SCRIPT and are forwarded.
"""
from __future__ import annotations

import socket
import sys


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def build_argv(argv):
    argv = list(argv)
    opts, i = [], 0
    while i < len(argv) and argv[i].startswith("-"):
        opts.append(argv[i])
        if "=" not in argv[i] and i + 1 < len(argv) and not argv[i + 1].startswith("-") and argv[i] not in (
                "--standalone", "--no-python", "--no_python", "--module", "-m"):
            opts.append(argv[i + 1])
            i += 1
        i += 1
    rest = argv[i:]
    joined = " ".join(opts)
    if "--nproc-per-node" not in joined and "--nproc_per_node" not in joined:
        from .utils.devices import visible_gpu_count
        n = visible_gpu_count() or 1
        opts = ["--nproc-per-node", str(n)] + opts
    if "--nnodes" not in joined:
        opts = ["--nnodes", "1"] + opts
    if "--master-addr" not in joined and "--master_addr" not in joined and "--standalone" not in joined:
        opts += ["--master-addr", "127.0.0.1"]
    if "--master-port" not in joined and "--master_port" not in joined and "--standalone" not in joined:
        opts += ["--master-port", str(_free_port())]
    return opts + rest


def main(argv=None):
    from torch.distributed.run import main as torchrun_main
    torchrun_main(build_argv(sys.argv[1:] if argv is None else argv))


if __name__ == "__main__":
    main()
