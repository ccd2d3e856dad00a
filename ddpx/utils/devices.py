"""Counting the node's GPUs WITHOUT initialising HIP in the calling process.

The reference launches with ``world_size = torch.cuda.device_count(); mp.spawn(...)``
(/root/reference/multigpu.py:262-263).  On torch-ROCm ``device_count()`` stays HIP-free only while amdsmi
enumeration succeeds; otherwise it calls ``hipGetDeviceCount``, which initialises HIP, and the launcher then
fork+execs its ranks from a process that touched the GPU.  :func:`visible_gpu_count` answers from the
environment (``HIP_VISIBLE_DEVICES`` / ``ROCR_VISIBLE_DEVICES`` / ``CUDA_VISIBLE_DEVICES``) or from the KFD
topology in sysfs, keeping only GPUs whose render node this process may open, and falls back to asking a child
process.  The launcher asserts afterwards that HIP is still uninitialised here.
"""
from __future__ import annotations

import glob
import os
import subprocess
import sys

KFD_NODES = "/sys/class/kfd/kfd/topology/nodes"
_ENV_VARS = ("HIP_VISIBLE_DEVICES", "ROCR_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES")


def _env_count(env) -> int | None:
    counts = []
    for k in _ENV_VARS:
        v = env.get(k)
        if v is None:
            continue
        v = v.strip()
        counts.append(0 if v in ("", "-1") else len([x for x in v.split(",") if x.strip()]))
    return min(counts) if counts else None


def _props(path):
    out = {}
    try:
        with open(path) as f:
            for line in f:
                parts = line.split()
                if len(parts) == 2:
                    try:
                        out[parts[0]] = int(parts[1])
                    except ValueError:
                        pass
    except OSError:
        return None
    return out


def kfd_gpu_count(nodes_dir: str = KFD_NODES, dev_dir: str = "/dev/dri") -> int | None:
    """GPUs in the KFD topology (nodes with SIMDs) whose DRM render node exists and is read/writable here;
    None if the topology is unreadable."""
    paths = sorted(glob.glob(os.path.join(nodes_dir, "*", "properties")))
    if not paths:
        return None
    n = 0
    for p in paths:
        pr = _props(p)
        if not pr or pr.get("simd_count", 0) <= 0:
            continue  # CPU node
        minor = pr.get("drm_render_minor")
        if minor is not None and minor > 0:
            node = os.path.join(dev_dir, f"renderD{minor}")
            if not (os.path.exists(node) and os.access(node, os.R_OK | os.W_OK)):
                continue  # not granted to this container
        n += 1
    return n


def _child_count() -> int:
    r = subprocess.run([sys.executable, "-c", "import torch; print(torch.cuda.device_count())"],
                       stdout=subprocess.PIPE, stderr=subprocess.DEVNULL, text=True, timeout=600)
    try:
        return int(r.stdout.strip().splitlines()[-1])
    except (ValueError, IndexError):
        return 0


def visible_gpu_count(env=None) -> int:
    """Number of GPUs a rank of this job could use, without initialising HIP in this process."""
    env = os.environ if env is None else env
    kfd = kfd_gpu_count()
    n = _env_count(env)
    if n is not None:
        return min(n, kfd) if kfd is not None else n
    if kfd is not None:
        return kfd
    return _child_count()


def assert_hip_uninitialised(what: str):
    """Fail before ``what`` (a fork+exec of ranks) if this process initialised HIP."""
    import torch
    if torch.cuda.is_initialized():
        raise RuntimeError(f"{what}: HIP is already initialised in the launching process; ranks must not be "
                           "started from a process that touched the GPU")
