"""Device batch loaders (data/loaders.py): DataLoader/DistributedSampler semantics, native gather."""
import numpy as np
import pytest
import torch
from torch.utils.data import DistributedSampler

from pytorch_ddp_mnist_amd.data.datasets import normalize_batch
from pytorch_ddp_mnist_amd.data.loaders import DeviceBatchLoader, create_data_loaders
from pytorch_ddp_mnist_amd.data.sampler import ShardedSampler
from pytorch_ddp_mnist_amd.data.synthetic import make_split


def _data(n=1000):
    x, y = make_split(n, seed=11)
    return torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y)


@pytest.mark.parametrize("world,rank", [(1, 0), (3, 2)])
def test_loader_matches_distributed_sampler(world, rank):
    x, y = _data()
    s = ShardedSampler(len(y), world, rank, shuffle=True, seed=42)
    ld = DeviceBatchLoader(x, y, 128, s, layout="image")
    ref = DistributedSampler(list(range(len(y))), num_replicas=world, rank=rank, shuffle=True, seed=42)
    for epoch in (0, 1):
        ld.sampler.set_epoch(epoch)
        ref.set_epoch(epoch)
        order = list(ref)
        got = list(ld)
        assert len(got) == len(ld) == -(-len(order) // 128)
        xs = torch.cat([b[0] for b in got])
        ys = torch.cat([b[1] for b in got])
        assert got[0][0].shape[1:] == (1, 28, 28) and ys.dtype == torch.int64
        assert torch.equal(ys, y[order].long())
        assert torch.allclose(xs.view(-1, 784), normalize_batch(x[order]))


def test_plain_shuffle_reshuffles_each_pass():
    x, y = _data(300)
    ld = DeviceBatchLoader(x, y, 100)
    a = torch.cat([b[1] for b in ld])
    b = torch.cat([b[1] for b in ld])
    assert sorted(a.tolist()) == sorted(b.tolist()) and not torch.equal(a, b)


def test_create_data_loaders_synthetic():
    tr, te = create_data_loaders(batch_size=256, world_size=2, rank=1, fmt="synthetic", limit=2000)
    assert len(tr) == -(-1000 // 256) and len(te) == -(-10000 // 256)
    x, y = next(iter(tr))
    assert x.shape == (256, 784) and x.dtype == torch.float32


@pytest.mark.gpu
@pytest.mark.parametrize("dtype,tol", [(torch.float32, 1e-6), (torch.bfloat16, 1e-2)])
def test_native_gather_normalize(native, dtype, tol):
    x, y = _data()
    dev = torch.device("cuda", 0)
    s = ShardedSampler(len(y), 2, 1, shuffle=True, seed=42)
    ld = DeviceBatchLoader(x.to(dev), y.to(dev), 96, s, dtype=dtype)
    assert ld._C is native, "the GPU loader must use the native gather kernel"
    order = s.indices()
    xs = torch.cat([b[0].float().cpu() for b in ld])
    ys = torch.cat([b[1].cpu() for b in ld])
    assert torch.equal(ys, y[order].long())
    ref = normalize_batch(x[order])
    assert float((xs - ref).abs().max()) <= tol * max(1.0, float(ref.abs().max()))
