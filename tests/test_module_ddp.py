"""Bring-your-own-model DDP wrapper (parallel/module_ddp.py) vs torch's DistributedDataParallel.

gloo, world_size 2 on CPU: both wrappers train the same model from different per-rank seeds for
three SGD steps (zero_grad(set_to_none=True) between them, so the grad-view re-binding path
runs); parameters must match torch DDP to fp32 round-off.  Also covers unused parameters and
``no_sync`` accumulation.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from pytorch_ddp_mnist_amd.models import build_model
from pytorch_ddp_mnist_amd.parallel.module_ddp import DistributedDataParallel, assign_buckets


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_assign_buckets():
    # backward-order sizes (floats); 1 MiB first cap = 262144 floats, then 4 MiB
    assert assign_buckets([10, 20, 30], 4, 1 << 20, 4 << 20) == [[0, 1, 2]]
    b = assign_buckets([200000, 100000, 500000, 600000, 5], 4, 1 << 20, 4 << 20)
    assert b == [[0], [1, 2], [3, 4]]
    assert assign_buckets([2_000_000], 4, 1 << 20, 4 << 20) == [[0]]


class WithUnused(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(784, 32)
        self.b = torch.nn.Linear(32, 10)
        self.unused = torch.nn.Linear(4, 4)

    def forward(self, x):
        return self.b(torch.relu(self.a(x)))


def _make(name):
    if name == "unused":
        return WithUnused()
    m = build_model(name)
    if name == "mlp":
        m[2].p = 0.0
    return m


def _worker(rank, world, port, name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    results = []
    for kind in ("ours", "torch"):
        torch.manual_seed(10 + rank)  # different init per rank: construction must broadcast rank 0's
        m = _make(name)
        if kind == "ours":
            dm = DistributedDataParallel(m, bucket_cap_mb=0.05, first_bucket_mb=0.02)
        else:
            dm = torch.nn.parallel.DistributedDataParallel(m, find_unused_parameters=(name == "unused"))
        opt = torch.optim.SGD(dm.parameters(), lr=0.1, momentum=0.9)
        g = torch.Generator().manual_seed(3)
        for step in range(3):
            x = torch.randn(16 * world, 784, generator=g)
            y = torch.randint(0, 10, (16 * world,), generator=g)
            xs, ys = x[rank * 16:(rank + 1) * 16], y[rank * 16:(rank + 1) * 16]
            if name == "lenet5":
                xs = xs.view(-1, 1, 28, 28)
            opt.zero_grad()
            out = dm(xs)
            loss = F.nll_loss(out, ys) if name == "lenet5" else F.cross_entropy(out, ys)
            loss.backward()
            opt.step()
        results.append({k: v.detach().clone() for k, v in m.state_dict().items()})
    # no_sync: two accumulated micro-batches then one synced == torch DDP with the same pattern
    accum = []
    for kind in ("ours", "torch"):
        torch.manual_seed(20 + rank)
        m = _make("mlp")
        dm = DistributedDataParallel(m) if kind == "ours" else torch.nn.parallel.DistributedDataParallel(m)
        g = torch.Generator().manual_seed(5 + rank)
        with dm.no_sync():
            F.cross_entropy(dm(torch.randn(8, 784, generator=g)), torch.randint(0, 10, (8,), generator=g)).backward()
        F.cross_entropy(dm(torch.randn(8, 784, generator=g)), torch.randint(0, 10, (8,), generator=g)).backward()
        accum.append(torch.cat([p.grad.reshape(-1) for p in m.parameters()]))
    # numpy payloads are pickled by value (tensors would travel as shared-memory fds that die with us)
    q.put((rank, [{k: v.numpy() for k, v in r.items()} for r in results], [a.numpy() for a in accum]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("name", ["mlp", "lenet5", "unused"])
def test_module_ddp_matches_torch_ddp(name):
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, name, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=180) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank in range(world):
        ours, ref = res[rank][1]
        for k in ref:
            assert np.allclose(ours[k], ref[k], rtol=1e-5, atol=1e-6), (rank, k, np.abs(ours[k] - ref[k]).max())
        a_ours, a_ref = res[rank][2]
        assert np.allclose(a_ours, a_ref, rtol=1e-5, atol=1e-6)
    for k in res[0][1][0]:
        assert np.array_equal(res[0][1][0][k], res[1][1][0][k]), "replicas must stay bit-identical"
