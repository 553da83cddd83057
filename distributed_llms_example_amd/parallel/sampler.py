"""Data sharding across data-parallel ranks.

* :class:`ShardedBatchSampler` — Accelerate's ``BatchSamplerShard`` semantics that both the HF Trainer
  path and the custom loop get from ``accelerator.prepare(DataLoader)``
  (accelerate/data_loader.py:110-271): the global sequence of batches is dealt round-robin to ranks;
  with ``even_batches`` the tail wraps to the start so every rank runs the same number of steps
  (818 eval rows on 4 ranks → 820 predictions).  Shuffling uses one seed shared by all
  ranks (Accelerate syncs the generator, data_loader.py:576-595), re-drawn per epoch.
* :class:`DataPartitioner` / :class:`Partition` — train-task's seeded (1234) shuffle-and-split into
  per-rank fractions (ref/train-task.py:32-62), reproduced exactly (``random.Random(seed).shuffle``).
"""
from __future__ import annotations

import math
import random

import torch


class ShardedBatchSampler(torch.utils.data.Sampler):
    def __init__(self, n: int, batch_size: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = False,
                 seed: int = 0, drop_last: bool = False, even_batches: bool = True):
        self.n = n
        self.batch_size = batch_size
        self.num_replicas = num_replicas
        self.rank = rank
        self.shuffle = shuffle
        self.seed = seed
        self.drop_last = drop_last
        self.even_batches = even_batches
        self.epoch = 0

    def set_epoch(self, epoch: int):
        self.epoch = epoch

    def _global_batches(self):
        if self.shuffle:
            g = torch.Generator()
            g.manual_seed(self.seed + self.epoch)
            order = torch.randperm(self.n, generator=g).tolist()
        else:
            order = list(range(self.n))
        batches = [order[i:i + self.batch_size] for i in range(0, self.n, self.batch_size)]
        if self.drop_last and batches and len(batches[-1]) < self.batch_size:
            batches.pop()
        return batches, order

    def __iter__(self):
        batches, order = self._global_batches()
        R = self.num_replicas
        if self.even_batches and batches:
            # complete the last partial batch and the last round with samples from the start
            if not self.drop_last and len(batches[-1]) < self.batch_size:
                need = self.batch_size - len(batches[-1])
                batches[-1] = batches[-1] + [order[i % len(order)] for i in range(need)]
            k = 0
            while len(batches) % R:
                batches.append(batches[k % len(batches)])
                k += 1
        for i in range(self.rank, len(batches), R):
            yield batches[i]

    def __len__(self):
        nb = (self.n // self.batch_size) if self.drop_last else math.ceil(self.n / self.batch_size)
        if self.even_batches:
            return math.ceil(nb / self.num_replicas)
        return len(range(self.rank, nb, self.num_replicas))


class Partition:
    """View of ``data`` at the given indices (ref/train-task.py:32-43)."""

    def __init__(self, data, index):
        self.data = data
        self.index = index

    def __len__(self):
        return len(self.index)

    def __getitem__(self, i):
        return self.data[self.index[i]]


class DataPartitioner:
    """Seeded shuffle, then consecutive fractions (ref/train-task.py:46-62)."""

    def __init__(self, data, sizes=(0.7, 0.2, 0.1), seed: int = 1234):
        self.data = data
        self.partitions = []
        rng = random.Random()
        rng.seed(seed)
        idx = list(range(len(data)))
        rng.shuffle(idx)
        for frac in sizes:
            n = int(frac * len(data))
            self.partitions.append(idx[:n])
            idx = idx[n:]

    def use(self, partition: int) -> Partition:
        return Partition(self.data, self.partitions[partition])
