"""Test-only fault injection for the optional phases of a multi-rank job (``DDPX_BENCH_INJECT``).

The bench's headline line must survive a failure in anything that is not the timed ddpx run itself: the stock
torch-DDP comparison and each start-up calibration candidate.  Tests provoke those failures through this
hook.  ``DDPX_BENCH_INJECT`` is a comma-separated list of ``site[:match][@rankR]`` entries:

* ``stock`` — the stock recipe raises after building its model (every rank, or rank R);
* ``calib:zero1`` — every calibration candidate whose name contains ``zero1`` raises in its first training
  step (every rank, or rank R);
* ``rccl`` — the native RCCL communicator of an N > 1 job cannot be created (every rank: the agreed gloo-staged
  fallback; a single rank would leave the others inside RCCL's collective init).

Unset (the default) it does nothing.
"""
from __future__ import annotations

import os


class InjectedFault(RuntimeError):
    pass


def _entries():
    spec = os.environ.get("DDPX_BENCH_INJECT", "")
    for ent in spec.split(","):
        ent = ent.strip()
        if not ent:
            continue
        rank = None
        if "@rank" in ent:
            ent, r = ent.split("@rank", 1)
            rank = int(r)
        site, _, match = ent.partition(":")
        yield site, match, rank


def maybe_inject(site: str, name: str = "", rank: int = 0) -> None:
    """Raise :class:`InjectedFault` if ``DDPX_BENCH_INJECT`` names ``site`` (and ``name`` contains its match,
    and the entry's rank, if any, is ``rank``)."""
    for s, match, r in _entries():
        if s == site and (not match or match in name) and (r is None or r == rank):
            raise InjectedFault(f"injected fault at {site}{(':' + name) if name else ''} on rank {rank}")
