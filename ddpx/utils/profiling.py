"""Tracing / profiling helpers (the reference has only a wall-clock timer).

* :func:`trace_range` — roctx ranges (``libroctx64``, shipped in torch/lib and /opt/rocm/lib) around
  the phases of a step.  They show up in ``rocprofv3 --marker-trace`` timelines.  Enabled with
  ``DDPX_ROCTX=1`` (or :func:`enable_roctx`); a no-op otherwise, so the hot loop pays nothing.
* :class:`StepTimer` — HIP-event timing of named phases per step with no host synchronisation inside
  the step (events are read back once, after the loop), for per-phase ms and samples/s reporting.
* :func:`kernel_table` — summarise a ``rocprofv3 --kernel-trace --stats --output-format csv``
  ``*_kernel_stats.csv`` into a compact table (used for ``profiles/``).
"""
from __future__ import annotations

import contextlib
import csv
import ctypes
import os

import torch

_roctx = None
_roctx_enabled = os.environ.get("DDPX_ROCTX", "0") == "1"


def _load_roctx():
    global _roctx
    if _roctx is not None:
        return _roctx
    cands = [os.path.join(os.path.dirname(torch.__file__), "lib", "libroctx64.so"), "/opt/rocm/lib/libroctx64.so",
             "libroctx64.so.4"]
    for c in cands:
        try:
            lib = ctypes.CDLL(c)
            lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
            lib.roctxRangePushA.restype = ctypes.c_int
            lib.roctxRangePop.restype = ctypes.c_int
            lib.roctxMarkA.argtypes = [ctypes.c_char_p]
            _roctx = lib
            return lib
        except OSError:
            continue
    _roctx = False
    return _roctx


def enable_roctx(flag: bool = True):
    global _roctx_enabled
    _roctx_enabled = flag


@contextlib.contextmanager
def trace_range(name: str):
    lib = _load_roctx() if _roctx_enabled else None
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


def mark(name: str):
    lib = _load_roctx() if _roctx_enabled else None
    if lib:
        lib.roctxMarkA(name.encode())


class StepTimer:
    """Per-phase GPU time with HIP events; ``summary()`` synchronises once."""

    def __init__(self, enabled: bool = True):
        self.enabled = enabled and torch.cuda.is_available()
        self.records = []  # (phase, start_event, end_event)

    @contextlib.contextmanager
    def phase(self, name: str):
        if not self.enabled:
            with trace_range(name):
                yield
            return
        s = torch.cuda.Event(enable_timing=True)
        e = torch.cuda.Event(enable_timing=True)
        s.record()
        with trace_range(name):
            yield
        e.record()
        self.records.append((name, s, e))

    def summary(self):
        if not self.records:
            return {}
        torch.cuda.synchronize()
        out = {}
        for name, s, e in self.records:
            out.setdefault(name, []).append(s.elapsed_time(e))
        return {k: {"mean_ms": sum(v) / len(v), "n": len(v)} for k, v in out.items()}


def kernel_table(stats_csv: str, steps: int | None = None, top: int = 30):
    rows = list(csv.DictReader(open(stats_csv)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    out = []
    for r in rows[:top]:
        out.append({
            "kernel": r["Name"][:120],
            "calls": int(r["Calls"]),
            "avg_us": round(float(r["AverageNs"]) / 1e3, 2),
            "pct": round(float(r["Percentage"]), 2),
        })
    res = {"total_ms": round(total / 1e6, 3), "kernels": out}
    if steps:
        res["per_step_us"] = round(total / steps / 1e3, 1)
    return res
