"""GPU-resident batch loader: sampler indices → gather + augment kernel → batch.

Replaces ``DataLoader(ds, batch_size, pin_memory=True, shuffle|sampler)``
(``/root/reference/singlegpu.py:174-180``, ``multigpu.py:147-154``) and the
blocking per-batch ``.to(gpu_id)`` copies (``singlegpu.py:114-115``).  The uint8
dataset lives on the device once; each batch is produced by ONE kernel
(``ddpx_augment``: gather, RandomCrop(32, pad 4), RandomHorizontalFlip,
ToTensor scaling) directly in the layout the model consumes.

On CPU the same transform runs with vectorised torch indexing and the *same*
counter-based random stream, so CPU and GPU batches are bit-identical (tested).

``len(loader)`` and the last partial batch follow the reference
(``drop_last=False``): 98 steps of 512 (last 336) for 50k samples on one rank.
"""
from __future__ import annotations

import math

import numpy as np
import torch

from ..runtime import native
from .datasets import ImageDataset
from .sampler import DistributedIndexSampler

LAYOUTS = {"nchw_f32": 0, "nchw_bf16": 1, "nhwc_bf16": 2, "nhwc_f32": 3, "flat_bf16": 1, "flat_f32": 0,
           "nhwc8_bf16": 4, "nhwc4_f32": 5}

_M64 = (1 << 64) - 1


def _splitmix64_np(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(_M64)
    x = ((x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(_M64)
    x = ((x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(_M64)
    return x ^ (x >> np.uint64(31))


def crop_flip_params(seed: int, batch: int, pad: int = 4):
    """(dy, dx, flip) per sample — identical to the HIP kernel's stream."""
    b = np.arange(1, batch + 1, dtype=np.uint64)
    with np.errstate(over="ignore"):
        key = (np.uint64(seed & _M64) ^ ((np.uint64(0xD1B54A32D192ED03) * b) & np.uint64(_M64)))
        r = _splitmix64_np(key)
    m = np.uint64(2 * pad + 1)
    dy = (r % m).astype(np.int64)
    dx = ((r >> np.uint64(16)) % m).astype(np.int64)
    flip = ((r >> np.uint64(40)) & np.uint64(1)).astype(np.int64)
    return torch.from_numpy(dy), torch.from_numpy(dx), torch.from_numpy(flip)


def augment_cpu(images_u8, labels, idx, seed, train=True, pad=4, layout="nchw_f32"):
    x = images_u8[idx]  # [B,C,H,W] uint8
    B, C, H, W = x.shape
    y = labels[idx]
    if train:
        dy, dx, flip = crop_flip_params(seed, B, pad)
        xp = torch.nn.functional.pad(x.float(), (pad, pad, pad, pad))
        rows = dy[:, None] + torch.arange(H)[None, :]                      # [B,H]
        cols = dx[:, None] + torch.arange(W)[None, :]                      # [B,W]
        cols = torch.where(flip[:, None].bool(), cols.flip(1), cols)
        bi = torch.arange(B)[:, None, None, None]
        ci = torch.arange(C)[None, :, None, None]
        out = xp[bi, ci, rows[:, None, :, None], cols[:, None, None, :]]
    else:
        out = x.float()
    out = out * (1.0 / 255.0)  # same fp32 constant multiply as the HIP kernel (bit-identical)
    if layout in ("nhwc_bf16", "nhwc_f32", "nhwc8_bf16", "nhwc4_f32"):
        out = out.permute(0, 2, 3, 1).contiguous()
    if layout == "nhwc8_bf16":
        out = torch.nn.functional.pad(out, (0, 8 - C))
    if layout == "nhwc4_f32":
        out = torch.nn.functional.pad(out, (0, 4 - C))
    if layout in ("flat_bf16", "flat_f32"):
        out = out.reshape(B, -1)
    if "bf16" in layout:
        out = out.to(torch.bfloat16)
    return out, y


def augment_gpu(images_u8, labels, idx, seed, train=True, pad=4, layout="nchw_f32", out=None, tgt=None):
    B = idx.numel()
    _, C, H, W = images_u8.shape
    code = LAYOUTS[layout]
    dt = torch.bfloat16 if "bf16" in layout else torch.float32
    shape = {"nchw_f32": (B, C, H, W), "nchw_bf16": (B, C, H, W), "nhwc_bf16": (B, H, W, C),
             "nhwc_f32": (B, H, W, C), "flat_bf16": (B, C * H * W), "flat_f32": (B, C * H * W),
             "nhwc8_bf16": (B, H, W, 8), "nhwc4_f32": (B, H, W, 4)}[layout]
    if out is None:
        out = torch.empty(shape, dtype=dt, device=images_u8.device)
    if tgt is None:
        tgt = torch.empty((B,), dtype=torch.int64, device=images_u8.device)
    if out.numel() < B * C * H * W or tgt.numel() < B:
        raise ValueError("augment: output buffers too small")
    if idx.dtype != torch.int64 or not idx.is_cuda:
        raise ValueError("augment: idx must be an int64 device tensor")
    lib = native.kernels()
    rc = lib.ddpx_augment(images_u8.data_ptr(), labels.data_ptr(), idx.data_ptr(), B, C, H, W, pad,
                          seed & _M64, int(train), code, out.data_ptr(), tgt.data_ptr(), native.stream_handle())
    native.check(rc, "ddpx_augment")
    return out, tgt


class DeviceLoader:
    """Iterable of (inputs, targets) batches produced on ``device``."""

    def __init__(self, dataset: ImageDataset, batch_size: int, device, sampler: DistributedIndexSampler | None = None,
                 train: bool = True, layout: str = "nchw_f32", seed: int = 0, pad: int = 4):
        self.device = torch.device(device)
        self.ds = dataset.to(self.device)
        self.batch_size = batch_size
        self.sampler = sampler or DistributedIndexSampler(len(dataset), 1, 0, shuffle=train, seed=seed)
        self.train = train
        self.layout = layout
        self.seed = seed
        self.pad = pad
        self.epoch = 0
        self._idx = None
        self._idx_epoch = None

    def set_epoch(self, epoch: int):
        self.epoch = epoch
        self.sampler.set_epoch(epoch)

    def __len__(self):
        return math.ceil(len(self.sampler) / self.batch_size)

    def _epoch_indices(self):
        if self._idx is None or self._idx_epoch != self.epoch:
            self._idx = self.sampler.indices().to(self.device)
            self._idx_epoch = self.epoch
        return self._idx

    def batch_seed(self, step: int) -> int:
        return (self.seed * 1_000_003 + self.epoch * 65_537 + step) & _M64

    def make_batch(self, idx: torch.Tensor, step: int, out=None, tgt=None):
        seed = self.batch_seed(step)
        if self.device.type == "cuda":
            return augment_gpu(self.ds.images, self.ds.labels, idx, seed, self.train, self.pad, self.layout, out, tgt)
        x, y = augment_cpu(self.ds.images, self.ds.labels, idx, seed, self.train, self.pad, self.layout)
        if out is not None:
            out.copy_(x)
            tgt.copy_(y)
            return out, tgt
        return x, y

    def cursor_batch(self, idx_all: torch.Tensor, nbatch: int, out, tgt, counter: torch.Tensor | None = None):
        """Batch k of ``idx_all`` (nbatch x batch_size indices) with augmentation seed ``batch_seed(k)``, k read
        on the device from ``counter`` (int32 [1]), written into the static ``out`` / ``tgt``.

        ``counter`` is the training step's own step counter (``SGD.step_counter()``: the LR-table kernel
        advances it once per step), so a captured step draws the next batch on every replay with no
        host work.  Without one, the loader keeps a private counter and advances it after the launch."""
        if self.device.type != "cuda":
            raise RuntimeError("cursor_batch needs the GPU-resident pipeline")
        own = counter is None
        if own:
            if getattr(self, "_cursor", None) is None:
                self._cursor = torch.zeros(1, dtype=torch.int32, device=self.device)
            counter = self._cursor
        if counter.dtype != torch.int32 or not counter.is_cuda:
            raise ValueError("cursor_batch: counter must be an int32 device tensor")
        B = self.batch_size
        if idx_all.numel() < nbatch * B or idx_all.dtype != torch.int64 or not idx_all.is_cuda:
            raise ValueError("cursor_batch: idx_all must hold nbatch x batch_size int64 device indices")
        _, C, H, W = self.ds.images.shape
        if out.numel() < B * C * H * W or tgt.numel() < B:
            raise ValueError("cursor_batch: output buffers too small")
        lib = native.kernels()
        rc = lib.ddpx_augment_cursor(self.ds.images.data_ptr(), self.ds.labels.data_ptr(), idx_all.data_ptr(), nbatch,
                                     B, C, H, W, self.pad, self.batch_seed(0), int(self.train), LAYOUTS[self.layout],
                                     out.data_ptr(), tgt.data_ptr(), counter.data_ptr(), native.stream_handle())
        native.check(rc, "ddpx_augment_cursor")
        if own:
            counter.add_(1)
        return out, tgt

    def __iter__(self):
        idx = self._epoch_indices()
        for step in range(len(self)):
            yield self.make_batch(idx[step * self.batch_size:(step + 1) * self.batch_size], step)

    @property
    def dataset(self):
        return self.ds
