"""Distributed sampler with index math bit-identical to torch's DistributedSampler.

Reference: ``DistributedSampler(dataset)`` at ``/root/reference/multigpu.py:153``
(``torch/utils/data/distributed.py:98-141``): per epoch
``g.manual_seed(seed + epoch); randperm(N)``; pad to ``ceil(N/ws)*ws`` by
repeating the head (``drop_last=False``); take ``indices[rank::ws]``.
The single-GPU reference uses ``shuffle=True`` (an unseeded RandomSampler);
here world_size=1 gives the same seeded permutation so runs are reproducible.

The indices are materialised once per epoch as an int64 tensor on the device
that holds the dataset, so the GPU loader can gather a batch without any host
round trip.
"""
from __future__ import annotations

import math

import torch


class DistributedIndexSampler:
    def __init__(self, n: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True, seed: int = 0,
                 drop_last: bool = False):
        if rank < 0 or rank >= num_replicas:
            raise ValueError(f"invalid rank {rank} for {num_replicas} replicas")
        self.n = n
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.epoch = 0
        if drop_last and n % num_replicas != 0:
            self.num_samples = math.ceil((n - num_replicas) / num_replicas)
        else:
            self.num_samples = math.ceil(n / num_replicas)
        self.total_size = self.num_samples * num_replicas

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def indices(self) -> torch.Tensor:
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            idx = torch.randperm(self.n, generator=g)
        else:
            idx = torch.arange(self.n)
        if not self.drop_last:
            pad = self.total_size - idx.numel()
            if pad > 0:
                if pad <= idx.numel():
                    idx = torch.cat([idx, idx[:pad]])
                else:
                    reps = math.ceil(pad / idx.numel())
                    idx = torch.cat([idx, idx.repeat(reps)[:pad]])
        else:
            idx = idx[:self.total_size]
        out = idx[self.rank:self.total_size:self.num_replicas]
        assert out.numel() == self.num_samples
        return out

    def __iter__(self):
        return iter(self.indices().tolist())

    def __len__(self):
        return self.num_samples
