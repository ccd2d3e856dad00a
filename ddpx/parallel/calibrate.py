"""Start-up calibration of the gradient-communication plan on the node the job actually runs on.

The reference inherits torch DDP's bucket caps (25 MiB, first bucket 1 MiB: ``DDP(model, device_ids=[gpu_id])``
at ``/root/reference/multigpu.py:89``), which were tuned for NVSwitch crossbars.  MI355X nodes are a
point-to-point xGMI mesh (7 links per GPU), where a ring collective is per-link bound and small messages pay
the per-collective latency several times over.  Instead of guessing, every candidate
plan is built for real — its own model copy, the DistributedDataParallel wrapper with that plan's buckets (so
the collectives are exactly the ones DDP issues: same layout code, chunking and padding), its optimizer — and
a few TRAINING STEPS are timed on the node (graph-captured when the job's steps are), before the first real
step.  The objective is therefore what the job pays: backward compute with the buckets' collectives
overlapping it, the exposed tail, the optimizer (replicated: the whole fp32 stream on every rank, applied per
bucket as each lands; ZeRO-1: 1/N of it plus the parameter all-gathers).

Timing the collective sequence alone on an idle GPU (round 3) favoured few large buckets: one bucket has the
fewest latencies but serialises all traffic after backward.  That candidate is no longer offered, and any
plan is judged by the step it produces (``tests/test_calibrate.py`` pins this with a delayed fake
communicator on which the isolated-fastest plan loses).

Candidates (deduplicated by the collective sequence they produce for the model):

* replicated (stock DDP): fp32 all-reduce (``ncclAvg``) per bucket, torch's greedy size rule over the
  gradient-ready order with (first, cap) in {(1, 25) torch default, (1, 8), (4, 16), (16, 64)} MiB;
* ZeRO-1 (when the model's weights are read only through the bf16 compute shadow, i.e. the native MLP):
  fp32 reduce-scatter of each weight bucket + bf16 all-gather of the updated shadow, biases in one
  replicated all-reduced bucket — 0.75x the all-reduce's bytes on the wire and 1/N of the optimizer's
  HBM stream per rank.  Same fp32 gradients and fp32 update as the replicated plan;
* either of the two with row-chunked big weights (16 / 32 MB chunks, torch's caps otherwise).

Every rank times every candidate in the same order (the trials are collective); the per-candidate time is
the max over ranks, so every rank derives the same choice (rank 0's is broadcast as a safeguard).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from ..runtime.flat_params import ALIGN
from ..runtime.graphs import assert_no_capture
from .ddp import plan_buckets

_CANDIDATE_CAPS = [(1.0, 25.0), (1.0, 8.0), (4.0, 16.0), (16.0, 64.0)]
# row-chunk buckets (DDP chunk_mb): a weight bigger than this is split into row chunks, each its own bucket,
# reduced as soon as its slice of the weight gradient is written (the toy MLP's 67 / 50 MB weights would
# otherwise be one bucket each whatever the caps)
_CANDIDATE_CHUNKS = [16.0, 32.0]


def _round_up(x, a):
    return (x + a - 1) // a * a


def _spans(order, numels, limits, esz, pad):
    """Element counts of the buckets torch's rule forms over ``order`` (each bucket padded to ``pad``)."""
    sizes = {i: numels[i] * esz for i in order}
    out = []
    for kind, idx in plan_buckets(order, sizes, limits):
        n = 0
        for i in idx:
            n = _round_up(n + numels[i], ALIGN)
        out.append(_round_up(max(n, pad), pad))
    return out


def candidate_plans(numels, shadow_only, world, allow_shard=True, caps=None, shapes=None, chunks=None):
    """[{name, shard, first_bucket_mb, bucket_cap_mb, chunk_mb, colls: [(kind, count, dtype)]}] for a model whose
    parameters have ``numels`` in gradient-ready order; ``shadow_only[i]``: parameter i is read only
    through the bf16 shadow (eligible for the ZeRO-1 shadow gather).  ``colls`` only deduplicates plans that
    would issue the same collectives.  With ``shapes``, row-chunked variants (torch's default caps, each
    ``chunks`` MB) are added when some matrix parameter is bigger than the chunk."""
    n = len(numels)
    plans, seen = [], set()
    combos = [(first, cap, None) for first, cap in (caps or _CANDIDATE_CAPS)]
    if shapes is not None:
        for ch in (_CANDIDATE_CHUNKS if chunks is None else chunks):
            if any(len(sh) >= 2 and k * 4 > ch * 2 ** 20 for sh, k in zip(shapes, numels)):
                combos.append((1.0, 25.0, ch))
    for first, cap, chunk in combos:
        limits = [int(first * 2 ** 20), int(cap * 2 ** 20)]
        rep = [("all_reduce", c, torch.float32) for c in _spans(list(range(n)), numels, limits, 4, ALIGN)]
        variants = [(False, rep)]
        S = [i for i in range(n) if shadow_only[i]]
        R = [i for i in range(n) if not shadow_only[i]]
        if allow_shard and world > 1:
            # ZeRO-1 gathers the bf16 shadow of the shadow-only parameters (the rest stay replicated), or the
            # fp32 master of every parameter when no parameter is shadow-only (ddp.py _shard_layout)
            gdt = torch.bfloat16 if S else torch.float32
            if not S:
                S, R = R, []
            colls = []
            for c in _spans(S, numels, limits, 4, world * ALIGN):
                colls += [("reduce_scatter", c, torch.float32), ("all_gather", c, gdt)]
            if R:
                rn = 0
                for i in R:
                    rn = _round_up(rn + numels[i], ALIGN)
                colls.append(("all_reduce", _round_up(max(rn, world * ALIGN), world * ALIGN), torch.float32))
            variants.append((True, colls))
        for shard, colls in variants:
            key = (shard, chunk, tuple((k, c, str(d)) for k, c, d in colls))
            if key in seen:
                continue
            seen.add(key)
            name = f"{'zero1' if shard else 'allreduce'}:{first:g}/{cap:g}MB" + (f"+chunk{chunk:g}MB" if chunk else "")
            plans.append({"name": name, "shard": shard, "first_bucket_mb": first, "bucket_cap_mb": cap,
                          "chunk_mb": chunk, "colls": colls})
    return plans


def _max_over_ranks(vals):
    t = torch.tensor(vals, dtype=torch.float64)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)  # the c10d group carries CPU tensors (gloo)
    return [float(v) for v in t]


def _barrier():
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.barrier()


class PeerFailed(RuntimeError):
    """Another rank reported a failure at an agreement point of the current trial."""


def _all_ok(ok: bool) -> bool:
    """Agreement point: True iff ``ok`` on every rank (MIN over the CPU group; the local value without one)."""
    if not (dist.is_initialized() and dist.get_world_size() > 1):
        return ok
    t = torch.tensor([1 if ok else 0], dtype=torch.int32)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return bool(t.item())


def _check():
    """A barrier that also fails the trial on every rank when one rank has already failed it."""
    if not _all_ok(True):
        raise PeerFailed("another rank failed this calibration trial")


def time_trial(step, sync, warm=3, reps=5, rounds=3):
    """Median over ``rounds`` of the mean wall time (ms) of ``reps`` back-to-back ``step()`` calls, after
    ``warm`` untimed ones; every round is bracketed by an agreement point (barrier) and ``sync()`` on both
    sides."""
    for _ in range(warm):
        step()
    sync()
    out = []
    for _ in range(rounds):
        _check()
        sync()
        t0 = time.perf_counter()
        for _ in range(reps):
            step()
        sync()
        out.append((time.perf_counter() - t0) * 1e3 / reps)
    out.sort()
    return out[len(out) // 2]


def _err(e: BaseException) -> str:
    return f"{type(e).__name__}: {e}"[:300]


def run_trial(plan, make_trial, sync, warm, reps, rounds):
    """One candidate's timing, agreed over ranks: (step ms, None) or (inf, error string) on EVERY rank.

    The agreement protocol makes a failed candidate cost the job nothing but its time: a rank whose trial
    raises goes straight to an agreement point with "failed"; the other ranks meet it at their next agreement
    point (every barrier of :func:`time_trial` is one, and so is the end of the trial), see the failure and stop
    this trial too.  Every rank therefore leaves the trial after the same number of CPU-group collectives.  (A
    rank failing *inside* a training step after its peers issued that step's RCCL collectives cannot be met
    this way; the communicator watchdog reports that case.)"""
    err = None
    close = None
    t = float("inf")
    try:
        step, close = make_trial(plan)
        t = time_trial(step, sync, warm=warm, reps=reps, rounds=rounds)
    except PeerFailed as e:
        err = _err(e)
        peer = True
    except Exception as e:  # noqa: BLE001 - any failure of an optional candidate is survivable
        err = _err(e)
        peer = False
    else:
        peer = False
    if close is not None:
        try:
            sync()
            close()
        except Exception as e:  # noqa: BLE001
            err = err or _err(e)
            peer = False
    try:
        # a trial's graph capture must leave no stream capturing: the next trial (or the timed engine) would
        # otherwise have its work recorded instead of run (profiles/r5_capture/NOTES.md)
        assert_no_capture(f"after calibration trial {plan.get('name', '?')}")
    except Exception as e:  # noqa: BLE001
        err = err or _err(e)
        peer = False
    if not peer:  # the final agreement point (a rank that saw PeerFailed already consumed it)
        if not _all_ok(err is None):
            err = err or "another rank failed this calibration trial"
    if err is not None:
        t = float("inf")
    return t, err


def calibrate_by_step(plans, make_trial, sync=lambda: None, warm=3, reps=5, rounds=3, tie=0.01):
    """Pick the plan whose training step is fastest on this node.  Returns (chosen plan, {name: step ms}).

    ``make_trial(plan) -> (step, close)``: a fresh model + DDP + optimizer for ``plan``; ``step()`` runs one
    whole training step, ``close()`` releases the trial (reducer, graphs, memory).  Collective: every rank
    calls this with the same plans.  Ties (within ``tie``) go to the earlier candidate (torch's default caps
    come first).  A candidate that fails on any rank is dropped on every rank (:func:`run_trial`); its error is
    the table entry.  Raises :class:`RuntimeError` only when every candidate failed."""
    if not plans:
        raise ValueError("calibrate_by_step: no candidate plans")
    local, errors = [], {}
    for p in plans:
        t, err = run_trial(p, make_trial, sync, warm, reps, rounds)
        local.append(t)
        if err is not None:
            errors[p["name"]] = err
    ms = _max_over_ranks(local)
    best = min(ms)
    if best == float("inf"):
        raise RuntimeError("calibrate_by_step: every candidate failed: " + "; ".join(
            f"{k}: {v}" for k, v in errors.items()))
    pick = min(i for i, v in enumerate(ms) if v <= best * (1.0 + tie))
    obj = [pick]
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast_object_list(obj, src=0)
    chosen = dict(plans[obj[0]])
    chosen.pop("colls", None)
    table = {p["name"]: (round(v, 4) if v != float("inf") else {"error": errors.get(p["name"], "failed")})
             for p, v in zip(plans, ms)}
    return chosen, table


def isolated_collective_ms(comm, plans, device, reps=3):
    """Diagnostics: median ms of each plan's collective sequence alone on the communicator stream (no
    backward to overlap with).  Collective: every rank must call."""
    maxc = {torch.float32: 0, torch.bfloat16: 0}
    for p in plans:
        for _, c, dt in p["colls"]:
            maxc[dt] = max(maxc[dt], c)
    bufs = {dt: torch.zeros(max(c, 1), dtype=dt, device=device) for dt, c in maxc.items()}
    cuda = device.type == "cuda"
    stream = getattr(comm, "stream", None) if cuda else None
    world = comm.world_size
    out = []
    for p in plans:
        ts = []
        for r in range(reps + 1):  # first pass: warm-up (connection setup, first-touch)
            _barrier()
            if cuda:
                torch.cuda.synchronize()
            t0 = time.perf_counter()
            for kind, count, dt in p["colls"]:
                t = bufs[dt][:count]
                sh = count // world
                if kind == "all_reduce":
                    comm.allreduce_(t, op="avg", stream=stream)
                elif kind == "reduce_scatter":
                    comm.reduce_scatter(t[comm.rank * sh:(comm.rank + 1) * sh], t, op="avg", stream=stream)
                else:
                    src = t[comm.rank * sh:(comm.rank + 1) * sh]
                    comm.allgather(t, src if t.is_cuda else src.clone(), stream=stream)
            if cuda:
                torch.cuda.synchronize()
            if r:
                ts.append((time.perf_counter() - t0) * 1e3)
        ts.sort()
        out.append(ts[len(ts) // 2])
    return _max_over_ranks(out)
