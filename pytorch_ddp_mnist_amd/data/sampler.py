"""Index streams bit-equal to ``torch.utils.data.DistributedSampler``.

Reference use: ``DistributedSampler(ds, num_replicas=W, rank=r, shuffle=True,
seed=42)`` + ``sampler.set_epoch(i)`` (ddp_tutorial_multi_gpu.py:26-30,81).
Semantics (survey App. C): permutation = ``randperm(N, generator(seed+epoch))``,
padded by repeating its head to ``ceil(N/W)*W``, then ``[rank::W]``.

The native engine does not iterate a Python sampler per batch: it uploads one
int32 index vector per epoch into HBM and every training kernel reads its
batch slice from there (``device_loader``).  ``epoch_indices`` builds that
vector (the next epoch's is computed on the host while the current one trains).
"""
from __future__ import annotations

import math
from typing import Iterator, List

import torch


def num_samples(n: int, world_size: int, drop_last: bool = False) -> int:
    if drop_last and n % world_size != 0:
        return math.ceil((n - world_size) / world_size)
    return math.ceil(n / world_size)


def epoch_indices(n: int, world_size: int = 1, rank: int = 0, epoch: int = 0, seed: int = 42,
                  shuffle: bool = True, drop_last: bool = False) -> torch.Tensor:
    """int64 tensor of this rank's sample order for ``epoch`` (== list(DistributedSampler))."""
    if shuffle:
        g = torch.Generator()
        g.manual_seed(seed + epoch)
        indices = torch.randperm(n, generator=g)
    else:
        indices = torch.arange(n)
    ns = num_samples(n, world_size, drop_last)
    total = ns * world_size
    if not drop_last:
        pad = total - n
        if pad > 0:
            if pad <= n:
                indices = torch.cat([indices, indices[:pad]])
            else:
                reps = math.ceil(pad / n)
                indices = torch.cat([indices, indices.repeat(reps)[:pad]])
    else:
        indices = indices[:total]
    assert indices.numel() == total
    return indices[rank:total:world_size]


class ShardedSampler:
    """Drop-in iterable with ``set_epoch`` (same API surface the reference uses)."""

    def __init__(self, n: int, num_replicas: int = 1, rank: int = 0, shuffle: bool = True,
                 seed: int = 0, drop_last: bool = False):
        self.n, self.num_replicas, self.rank = n, num_replicas, rank
        self.shuffle, self.seed, self.drop_last = shuffle, seed, drop_last
        self.epoch = 0

    def set_epoch(self, epoch: int) -> None:
        self.epoch = epoch

    def indices(self) -> torch.Tensor:
        return epoch_indices(self.n, self.num_replicas, self.rank, self.epoch, self.seed,
                             self.shuffle, self.drop_last)

    def __iter__(self) -> Iterator[int]:
        return iter(self.indices().tolist())

    def __len__(self) -> int:
        return num_samples(self.n, self.num_replicas, self.drop_last)


def batch_slices(count: int, batch_size: int, drop_last: bool = False) -> List[tuple]:
    """(start, size) pairs of DataLoader batches over ``count`` indices (last batch partial)."""
    out = []
    for s in range(0, count, batch_size):
        b = min(batch_size, count - s)
        if b < batch_size and drop_last:
            break
        out.append((s, b))
    return out
