"""Datasets: CIFAR-10 from disk (no torchvision) and CIFAR-shaped synthetic data.

The reference downloads CIFAR-10 through torchvision at run time
(``/root/reference/singlegpu.py:153-171``).  There is no torchvision and no
network here or on the GPU boxes, so:

* :func:`load_cifar10` reads an already-present copy under ``data/cifar10``:
  the binary distribution (``cifar-10-batches-bin/*.bin``, read with numpy) or
  torchvision's python distribution (``cifar-10-batches-py``, read through a
  restricted unpickler that only admits numpy array reconstruction);
* :func:`synthetic_cifar` makes a CIFAR-shaped dataset (uint8 [N,3,32,32],
  int64 labels) whose labels are *learnable* (class prototype + noise), so
  training curves and accuracy are meaningful in tests and benchmarks.

Both return :class:`ImageDataset` — raw uint8 CHW images plus labels — which
``ddpx.data.loader`` keeps resident on the GPU and augments there.
"""
from __future__ import annotations

import io
import os
import pickle
from dataclasses import dataclass

import numpy as np
import torch

CIFAR_TRAIN = 50000
CIFAR_TEST = 10000


@dataclass
class ImageDataset:
    images: torch.Tensor  # uint8 [N, C, H, W]
    labels: torch.Tensor  # int64 [N]
    num_classes: int = 10
    name: str = "dataset"

    def __len__(self):
        return int(self.images.shape[0])

    def __getitem__(self, i):
        """(float CHW in [0,1], label) — ToTensor semantics, for DataLoader-style use."""
        return self.images[i].float().div_(255.0), int(self.labels[i])

    def to(self, device):
        return ImageDataset(self.images.to(device), self.labels.to(device), self.num_classes, self.name)


class _NumpyOnlyUnpickler(pickle.Unpickler):
    _ALLOWED = {
        ("numpy.core.multiarray", "_reconstruct"),
        ("numpy._core.multiarray", "_reconstruct"),
        ("numpy", "ndarray"),
        ("numpy", "dtype"),
        ("numpy.core.multiarray", "scalar"),
        ("numpy._core.multiarray", "scalar"),
    }

    def find_class(self, module, name):
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load {module}.{name} from a CIFAR batch file")


def _read_py_batch(path):
    with open(path, "rb") as f:
        d = _NumpyOnlyUnpickler(io.BytesIO(f.read()), encoding="bytes").load()
    data = np.asarray(d[b"data"], dtype=np.uint8).reshape(-1, 3, 32, 32)
    labels = np.asarray(d[b"labels"], dtype=np.int64)
    return data, labels


def _read_bin_batch(path):
    raw = np.fromfile(path, dtype=np.uint8).reshape(-1, 3073)
    return raw[:, 1:].reshape(-1, 3, 32, 32).copy(), raw[:, 0].astype(np.int64)


def load_cifar10(root: str = "data/cifar10", train: bool = True) -> ImageDataset:
    bin_dir = os.path.join(root, "cifar-10-batches-bin")
    py_dir = os.path.join(root, "cifar-10-batches-py")
    if os.path.isdir(bin_dir):
        names = [f"data_batch_{i}.bin" for i in range(1, 6)] if train else ["test_batch.bin"]
        parts = [_read_bin_batch(os.path.join(bin_dir, n)) for n in names]
    elif os.path.isdir(py_dir):
        names = [f"data_batch_{i}" for i in range(1, 6)] if train else ["test_batch"]
        parts = [_read_py_batch(os.path.join(py_dir, n)) for n in names]
    else:
        raise FileNotFoundError(
            f"CIFAR-10 not found under {root!r} (expected cifar-10-batches-bin/ or cifar-10-batches-py/). "
            "There is no network access to download it; use --data synthetic.")
    imgs = torch.from_numpy(np.concatenate([p[0] for p in parts]))
    labels = torch.from_numpy(np.concatenate([p[1] for p in parts]))
    return ImageDataset(imgs, labels, 10, "cifar10-train" if train else "cifar10-test")


def synthetic_cifar(n: int, seed: int = 0, num_classes: int = 10, noise: float = 60.0,
                    shape=(3, 32, 32), split_seed_offset: int = 0) -> ImageDataset:
    """Learnable CIFAR-shaped data: per-class smooth prototype + Gaussian noise, uint8."""
    g = torch.Generator().manual_seed(1234 + seed)  # prototypes shared by train/test
    c, h, w = shape
    base = torch.rand((num_classes, c, h // 4, w // 4), generator=g) * 255.0
    protos = torch.nn.functional.interpolate(base, size=(h, w), mode="bilinear", align_corners=False)
    g2 = torch.Generator().manual_seed(99991 + seed + split_seed_offset)
    labels = torch.randint(0, num_classes, (n,), generator=g2, dtype=torch.int64)
    imgs = torch.empty((n, c, h, w), dtype=torch.uint8)
    chunk = 4096
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        x = protos[labels[s:e]] + torch.randn((e - s, c, h, w), generator=g2) * noise
        imgs[s:e] = x.clamp_(0, 255).round_().to(torch.uint8)
    return ImageDataset(imgs, labels, num_classes, f"synthetic-{n}")


def get_datasets(kind: str = "synthetic", root: str = "data/cifar10", seed: int = 0,
                 train_size: int = CIFAR_TRAIN, test_size: int = CIFAR_TEST):
    """(train, test) — the reference's ``getTrainingData()`` (singlegpu.py:153-171)."""
    if kind == "cifar10":
        return load_cifar10(root, True), load_cifar10(root, False)
    if kind == "synthetic":
        return (synthetic_cifar(train_size, seed=seed),
                synthetic_cifar(test_size, seed=seed, split_seed_offset=7))
    raise ValueError(f"unknown dataset kind {kind!r}")
