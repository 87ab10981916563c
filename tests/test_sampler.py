"""Sampler order bit-equal to torch.utils.data.DistributedSampler (survey App. C, N18)."""
import pytest
import torch
from torch.utils.data import DistributedSampler

from pytorch_ddp_mnist_amd.data.sampler import ShardedSampler, batch_slices, epoch_indices, num_samples


class _DS:
    def __init__(self, n):
        self.n = n

    def __len__(self):
        return self.n


@pytest.mark.parametrize("n", [60000, 1000, 37])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("drop_last", [False, True])
def test_bit_equal_to_distributed_sampler(n, world, drop_last):
    for rank in range(world):
        ref = DistributedSampler(_DS(n), num_replicas=world, rank=rank, shuffle=True, seed=42, drop_last=drop_last)
        ours = ShardedSampler(n, world, rank, shuffle=True, seed=42, drop_last=drop_last)
        for epoch in range(3):
            ref.set_epoch(epoch)
            ours.set_epoch(epoch)
            assert list(ref) == list(ours)
            assert len(ref) == len(ours)


def test_unshuffled_and_counts():
    assert epoch_indices(10, 4, 1, shuffle=False).tolist() == [1, 5, 9]
    assert num_samples(60000, 8) == 7500
    assert epoch_indices(60000, 8, 7, 0).numel() == 7500


def test_batches_match_dataloader():
    assert batch_slices(7500, 128)[-1] == (7424, 76)
    assert len(batch_slices(60000, 128)) == 469
    assert batch_slices(10, 4, drop_last=True) == [(0, 4), (4, 4)]


def test_steps_per_epoch_table():  # survey §6
    for w, steps in ((1, 469), (2, 235), (4, 118), (8, 59)):
        assert len(batch_slices(num_samples(60000, w), 128)) == steps
