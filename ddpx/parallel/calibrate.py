"""Start-up calibration of the gradient-communication plan on the node the job actually runs on.

The reference inherits torch DDP's bucket caps (25 MiB, first bucket 1 MiB: ``DDP(model, device_ids=[gpu_id])``
at ``/root/reference/multigpu.py:89``), which were tuned for NVSwitch crossbars.  MI355X nodes are a
point-to-point xGMI mesh (7 links per GPU), where a ring collective is per-link bound and small messages pay
the per-collective latency several times over.  Instead of guessing, every candidate
plan's collective sequence — exactly the collectives one training step issues for it, with the step's bucket
sizes and dtypes — is timed on the communicator's own stream before the first training step, and rank 0's
choice is broadcast so every rank builds the same bucket layout.

Candidates (deduplicated by the collective sequence they produce for the model):

* replicated (stock DDP): fp32 all-reduce (``ncclAvg``) per bucket, torch's greedy size rule over the
  gradient-ready order with (first, cap) in {(1, 25) torch default, (4, 16), (16, 64), (one bucket)};
* ZeRO-1 (when the model's weights are read only through the bf16 compute shadow, i.e. the native MLP):
  fp32 reduce-scatter of each weight bucket + bf16 all-gather of the updated shadow, biases in one
  replicated all-reduced bucket — 0.75x the all-reduce's bytes on the wire and 1/N of the optimizer's
  HBM stream per rank.  Same fp32 gradients and fp32 update as the replicated plan.

The collective-sequence time is a lower bound of what the step exposes; ties within ``tie`` go to the plan
with more buckets (more of its traffic can hide behind the backward that produces the later buckets).
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist

from ..runtime.flat_params import ALIGN
from .ddp import plan_buckets

_CANDIDATE_CAPS = [(1.0, 25.0), (4.0, 16.0), (16.0, 64.0), (1e6, 1e6)]


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


def candidate_plans(numels, shadow_only, world, allow_shard=True):
    """[{name, shard, first_bucket_mb, bucket_cap_mb, colls: [(kind, count, dtype)]}] for a model whose
    parameters have ``numels`` in gradient-ready order; ``shadow_only[i]``: parameter i is read only
    through the bf16 shadow (eligible for the ZeRO-1 shadow gather)."""
    n = len(numels)
    plans, seen = [], set()
    for first, cap in _CANDIDATE_CAPS:
        limits = [int(first * 2 ** 20), int(cap * 2 ** 20)]
        rep = [("all_reduce", c, torch.float32) for c in _spans(list(range(n)), numels, limits, 4, ALIGN)]
        variants = [(False, rep)]
        S = [i for i in range(n) if shadow_only[i]]
        R = [i for i in range(n) if not shadow_only[i]]
        if allow_shard and world > 1 and S:
            colls = []
            for c in _spans(S, numels, limits, 4, world * ALIGN):
                colls += [("reduce_scatter", c, torch.float32), ("all_gather", c, torch.bfloat16)]
            if R:
                rn = 0
                for i in R:
                    rn = _round_up(rn + numels[i], ALIGN)
                colls.append(("all_reduce", _round_up(max(rn, world * ALIGN), world * ALIGN), torch.float32))
            variants.append((True, colls))
        for shard, colls in variants:
            key = (shard, tuple((k, c, str(d)) for k, c, d in colls))
            if key in seen:
                continue
            seen.add(key)
            name = f"{'zero1' if shard else 'allreduce'}:{first:g}/{cap:g}MB" if cap < 1e6 else \
                f"{'zero1' if shard else 'allreduce'}:one-bucket"
            plans.append({"name": name, "shard": shard, "first_bucket_mb": first, "bucket_cap_mb": cap,
                          "colls": colls})
    return plans


def _issue(comm, colls, bufs, stream):
    world = comm.world_size
    for kind, count, dt in colls:
        t = bufs[dt][:count]
        if kind == "all_reduce":
            comm.allreduce_(t, op="avg", stream=stream)
        elif kind == "reduce_scatter":
            sh = count // world
            comm.reduce_scatter(t[comm.rank * sh:(comm.rank + 1) * sh], t, op="avg", stream=stream)
        else:
            sh = count // world
            comm.allgather(t, t[comm.rank * sh:(comm.rank + 1) * sh].clone() if not t.is_cuda else
                           t[comm.rank * sh:(comm.rank + 1) * sh], stream=stream)


def time_plans(comm, plans, device, reps=3):
    """Median ms of each plan's collective sequence on this rank (collective: every rank must call)."""
    maxc = {torch.float32: 0, torch.bfloat16: 0}
    for p in plans:
        for _, c, dt in p["colls"]:
            maxc[dt] = max(maxc[dt], c)
    bufs = {dt: torch.zeros(max(c, 1), dtype=dt, device=device) for dt, c in maxc.items()}
    cuda = device.type == "cuda"
    stream = getattr(comm, "stream", None) if cuda else None
    out = []
    for p in plans:
        ts = []
        for r in range(reps + 1):  # first pass: warm-up (connection setup, first-touch)
            if dist.is_initialized() and dist.get_world_size() > 1:
                dist.barrier()
            if cuda:
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                s = stream if stream is not None else torch.cuda.current_stream()
                e0.record(s)
                _issue(comm, p["colls"], bufs, stream)
                e1.record(s)
                e1.synchronize()
                dt_ms = e0.elapsed_time(e1)
            else:
                t0 = time.perf_counter()
                _issue(comm, p["colls"], bufs, None)
                dt_ms = (time.perf_counter() - t0) * 1e3
            if r:
                ts.append(dt_ms)
        ts.sort()
        out.append(ts[len(ts) // 2])
    del bufs
    return out


def calibrate(comm, numels, shadow_only, device, allow_shard=True, reps=3, tie=0.03):
    """Pick the gradient-communication plan for this node.  Returns (chosen plan dict, {name: ms}).

    Every rank times every candidate (the max over ranks is what a step would see); rank 0 decides and the
    decision is broadcast, so all ranks build identical buckets."""
    world = comm.world_size
    plans = candidate_plans(numels, shadow_only, world, allow_shard=allow_shard)
    local = time_plans(comm, plans, device, reps=reps)
    t = torch.tensor(local, dtype=torch.float64)
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    ms = [float(v) for v in t]
    best = min(ms)
    # ties (within `tie`) go to the plan with the most collectives: its later buckets overlap more backward
    ok = [i for i, v in enumerate(ms) if v <= best * (1.0 + tie)]
    pick = max(ok, key=lambda i: (len(plans[i]["colls"]), -ms[i]))
    obj = [pick]
    if dist.is_initialized() and dist.get_world_size() > 1:
        dist.broadcast_object_list(obj, src=0)
    chosen = dict(plans[obj[0]])
    chosen.pop("colls")
    return chosen, {p["name"]: round(v, 4) for p, v in zip(plans, ms)}
