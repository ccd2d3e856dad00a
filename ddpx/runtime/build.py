"""In-tree build of the ddpx native libraries for MI355X (gfx950).

Two shared objects are produced next to the Python package so that they travel
with the repository snapshot to a GPU box:

* ``ddpx/_native/libddpx_kernels.so`` — every HIP kernel in ``csrc/kernels``
  (MFMA GEMM, fused SGD, head/xent, data augmentation, conv/BN/pool ...),
  compiled with ``hipcc --offload-arch=gfx950``.
* ``ddpx/_native/libddpx_rt.so`` — the C++ runtime in ``csrc/runtime`` (RCCL
  communicator, gradient-bucket reducer, watchdog), linked against RCCL.

Both expose a plain C ABI consumed through :mod:`ctypes` (``ddpx.runtime.native``);
no torch headers are needed, so a rebuild takes seconds.  Objects are rebuilt
only when a source or header is newer than the library.
"""
from __future__ import annotations

import concurrent.futures as cf
import glob
import os
import re
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CSRC = os.path.join(ROOT, "csrc")
OUT_DIR = os.path.join(ROOT, "ddpx", "_native")
OBJ_DIR = os.path.join(ROOT, "build", "obj")
ARCH = os.environ.get("DDPX_OFFLOAD_ARCH", "gfx950")

KERNELS_LIB = os.path.join(OUT_DIR, "libddpx_kernels.so")
RT_LIB = os.path.join(OUT_DIR, "libddpx_rt.so")


def _hipcc() -> str:
    for cand in (os.environ.get("HIPCC"), "/opt/rocm/bin/hipcc", shutil.which("hipcc")):
        if cand and os.path.exists(cand):
            return cand
    raise RuntimeError("hipcc not found (set HIPCC or install ROCm)")


def _newest(paths) -> float:
    return max((os.path.getmtime(p) for p in paths), default=0.0)


def _run(cmd, verbose):
    if verbose:
        print(" ".join(cmd), flush=True)
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"command failed ({r.returncode}): {' '.join(cmd)}\n{r.stdout}")
    return r.stdout


_INCLUDE = re.compile(r'^\s*#\s*include\s*"([^"]+)"', re.M)


def _deps(src, inc_dir, seen=None):
    """``src`` and the csrc/include headers it includes, transitively (quoted includes only)."""
    seen = set() if seen is None else seen
    if src in seen or not os.path.exists(src):
        return seen
    seen.add(src)
    with open(src, errors="replace") as f:
        for name in _INCLUDE.findall(f.read()):
            _deps(os.path.join(inc_dir, name), inc_dir, seen)
    return seen


def _compile_objs(srcs, flags, verbose, jobs):
    os.makedirs(OBJ_DIR, exist_ok=True)
    inc_dir = os.path.join(CSRC, "include")
    hipcc = _hipcc()
    todo, objs = [], []
    for s in srcs:
        o = os.path.join(OBJ_DIR, os.path.basename(s) + ".o")
        objs.append(o)
        if not os.path.exists(o) or os.path.getmtime(o) < _newest(_deps(s, inc_dir)):
            todo.append((s, o))
    with cf.ThreadPoolExecutor(max_workers=max(1, jobs)) as ex:
        futs = [ex.submit(_run, [hipcc, *flags, "-c", s, "-o", o], verbose) for s, o in todo]
        for f in futs:
            f.result()
    return objs, bool(todo)


def build(force: bool = False, verbose: bool = False, jobs: int | None = None) -> dict:
    """Compile (if stale) and return the paths of the native libraries."""
    jobs = jobs or min(8, os.cpu_count() or 4)
    os.makedirs(OUT_DIR, exist_ok=True)
    if force and os.path.isdir(OBJ_DIR):
        shutil.rmtree(OBJ_DIR)
    inc = ["-I" + os.path.join(CSRC, "include")]
    common = ["-O3", "-std=c++17", "-fPIC", *inc]

    ksrcs = sorted(glob.glob(os.path.join(CSRC, "kernels", "*.hip")))
    kobjs, kdirty = _compile_objs(ksrcs, [f"--offload-arch={ARCH}", *common], verbose, jobs)
    if force or kdirty or not os.path.exists(KERNELS_LIB) or os.path.getmtime(KERNELS_LIB) < _newest(kobjs):
        _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-o", KERNELS_LIB, *kobjs], verbose)

    rsrcs = sorted(glob.glob(os.path.join(CSRC, "runtime", "*.cpp")))
    robjs, rdirty = _compile_objs(rsrcs, [*common, "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"], verbose, jobs)
    if force or rdirty or not os.path.exists(RT_LIB) or os.path.getmtime(RT_LIB) < _newest(robjs):
        _run([_hipcc(), "-shared", "-o", RT_LIB, *robjs, "-L/opt/rocm/lib", "-lrccl", "-lamdhip64", "-lpthread"],
             verbose)
    return {"kernels": KERNELS_LIB, "runtime": RT_LIB}


if __name__ == "__main__":
    force = "--force" in sys.argv
    print(build(force=force, verbose=True))
