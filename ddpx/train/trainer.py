"""Trainer — the reference's hot loop, MI355X-native underneath.

Same structure, prints and checkpoint rule as ``Trainer`` in
``/root/reference/singlegpu.py:85-128`` / ``multigpu.py:74-119``:

* ``_run_batch``: zero_grad → forward → cross-entropy → backward →
  optimizer.step → scheduler.step (per batch);
* ``_run_epoch``: prints ``[GPU{id}] Epoch {e} | Batchsize: {b} | Steps: {n}``,
  sets the sampler epoch (distributed), iterates the loader;
* ``train``: saves ``checkpoint.pt`` when ``epoch % save_every == 0`` (rank 0
  only when distributed).

Differences (all deliberate):
* batches are produced on the GPU (no H2D copy, no CPU augmentation);
* the batch size for the print is computed, not by loading a throw-away batch
  (the reference's ``len(next(iter(loader))[0])`` augments one extra batch);
* the loss uses the model's fused ``forward_loss`` when it has one;
* ``graph=True`` captures the full-size step into a HIP graph after
  ``graph_warmup`` eager steps and replays it (partial last batch runs eager); if the capture
  fails on any rank, every rank continues eagerly (``graph_error`` says why);
* optional JSON-lines metrics (``metrics``) and full-state checkpoints.
"""
from __future__ import annotations

import time

import torch
import torch.distributed as dist
import torch.nn.functional as F
from torch import nn

from ..runtime.graphs import try_capture
from ..utils.profiling import trace_range
from . import checkpoint as ckpt


class Trainer:
    def __init__(self, model: nn.Module, train_data, optimizer, gpu_id, save_every: int, scheduler,
                 distributed: bool = False, rank: int = 0, graph: bool = False, graph_warmup: int = 2,
                 metrics=None, full_checkpoint: bool = False, ckpt_path: str = ckpt.CKPT_PATH) -> None:
        self.gpu_id = gpu_id
        self.model = model
        self.train_data = train_data
        self.optimizer = optimizer
        self.save_every = save_every
        self._one = None
        self._device_lr = False  # LR schedule tabulated on the device (set at train start)
        self.fault_step = None  # fault injection
        self.scheduler = scheduler
        self.distributed = distributed
        self.rank = rank
        self.use_graph = graph and torch.cuda.is_available() and next(model.parameters()).is_cuda
        self.graph_warmup = graph_warmup
        self.metrics = metrics
        self.full_checkpoint = full_checkpoint
        self.ckpt_path = ckpt_path
        self._graph = None
        self._graph_batch = None
        self.graph_error = None
        self.global_step = 0
        self.last_loss = None
        self.start_epoch = 0

    # ------------------------------------------------------------- one step
    def _forward_loss(self, source, targets):
        if hasattr(ckpt.unwrap(self.model), "forward_loss"):
            loss, _ = self.model.forward_loss(source, targets)
            return loss
        output = self.model(source)
        return F.cross_entropy(output, targets)

    def _step_body(self, source, targets):
        if self._device_lr:
            self.optimizer.device_lr_step()
        self.optimizer.zero_grad()
        with trace_range("forward"):
            loss = self._forward_loss(source, targets)
        with trace_range("backward"):
            if self._one is None or self._one.device != loss.device:
                self._one = torch.ones((), device=loss.device, dtype=loss.dtype)
            loss.backward(self._one)  # preallocated seed gradient: no fill kernel inside the step
        with trace_range("optimizer"):
            self.optimizer.step()
        return loss

    def _run_batch(self, source, targets):
        if self.fault_step is not None and self.global_step == self.fault_step:
            raise RuntimeError(f"injected fault at step {self.global_step} (--fault_step)")
        bs = source.shape[0]
        if self.use_graph and self._graph is None and self.global_step >= self.graph_warmup \
                and self._graph_batch is None:
            self._graph_batch = bs
        if self.use_graph and self._graph_batch == bs and self._graph is None:
            self.optimizer.sync_lr()
            self._graph, err = try_capture(self._step_body, source, targets, self.model, self.optimizer,
                                           comm=getattr(self.model, "comm", None))
            if self._graph is None:
                # capture failed on some rank: every rank steps eagerly from here on (same process)
                self.use_graph = False
                self.graph_error = err
                if self.rank == 0:
                    print(f"note: HIP-graph capture failed, training continues eagerly ({err})", flush=True)
        if self.use_graph and self._graph_batch == bs:
            self._graph.load(source, targets)
            self.optimizer.sync_lr()
            loss = self._graph()
        else:
            if hasattr(self.optimizer, "sync_lr"):
                self.optimizer.sync_lr()
            loss = self._step_body(source, targets)
        self.scheduler.step()
        self.global_step += 1
        self.last_loss = loss
        return loss

    def _batch_size_for_print(self):
        n = len(self.train_data.sampler) if hasattr(self.train_data, "sampler") else None
        bs = self.train_data.batch_size
        return min(bs, n) if n is not None else bs

    def _run_epoch(self, epoch):
        b_sz = self._batch_size_for_print()
        print(f"[GPU{self.gpu_id}] Epoch {epoch} | Batchsize: {b_sz} | Steps: {len(self.train_data)}")
        if hasattr(self.train_data, "set_epoch"):
            self.train_data.set_epoch(epoch)
        t0 = time.time()
        n = 0
        it = iter(self.train_data)
        while True:
            with trace_range("data"):
                batch = next(it, None)
            if batch is None:
                break
            source, targets = batch
            with trace_range("step"):
                self._run_batch(source, targets)
            n += source.shape[0]
        if self.metrics is not None:
            loss = float(self.last_loss.detach().float().item()) if self.last_loss is not None else float("nan")
            dt = time.time() - t0
            extra = {}
            if self.distributed and torch.distributed.is_initialized():
                t = torch.tensor([loss, float(n)], dtype=torch.float64)
                torch.distributed.all_reduce(t)  # CPU tensor: the c10d (gloo) group
                ws = torch.distributed.get_world_size()
                extra["loss_mean_ranks"] = float(t[0]) / ws
                extra["samples_all_ranks"] = int(t[1])
            if hasattr(self.model, "comm_stats"):
                cs = self.model.comm_stats()
                if cs:
                    extra.update(cs)
            self.metrics.log(epoch=epoch, step=self.global_step, loss=loss, samples=n, seconds=dt,
                             samples_per_s=n / max(dt, 1e-9), lr=self.optimizer.param_groups[0]["lr"], **extra)

    def _save_checkpoint(self, epoch):
        path = ckpt.save_checkpoint(self.model, self.ckpt_path)
        print(f"Epoch {epoch} | Training checkpoint saved at {path}")
        if self.full_checkpoint:
            ckpt.save_full_checkpoint(ckpt.FULL_CKPT_PATH, self.model, self.optimizer, self.scheduler, epoch)

    def train(self, max_epochs: int):
        if (not self._device_lr and hasattr(self.optimizer, "attach_device_schedule")
                and hasattr(self.scheduler, "lr_lambdas")):
            self._device_lr = bool(self.optimizer.attach_device_schedule(self.scheduler))
        for epoch in range(self.start_epoch, max_epochs):
            self._run_epoch(epoch)
            if self.distributed and epoch % self.save_every == 0 and hasattr(self.model, "consolidate"):
                self.model.consolidate()  # collective: sharded optimizer -> complete fp32 state on every rank
            if (not self.distributed or self.rank == 0) and epoch % self.save_every == 0:
                self._save_checkpoint(epoch)
            if self.distributed and epoch % self.save_every == 0 and dist.is_initialized():
                # no rank runs ahead of a half-written checkpoint (the reference has no
                # barrier here, multigpu.py:118); one CPU barrier per save
                dist.barrier()
        if torch.cuda.is_available() and next(self.model.parameters()).is_cuda:
            torch.cuda.synchronize()
