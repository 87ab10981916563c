"""T4: distributed logic on CPU with gloo, world_size 2 (bucketing, averaging, broadcast, order)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
import torch.nn.functional as F

from pytorch_ddp_mnist_amd.models import build_model, flatten_grads
from pytorch_ddp_mnist_amd.parallel.ddp import GlooReducer, model_phases, plan_buckets


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bucket_plans():
    assert plan_buckets(model_phases("mlp")) == [(100480, 118272, 0), (0, 100480, 1)]
    assert plan_buckets(model_phases("lenet5")) == [(2572, 61706, 0), (0, 2572, 1)]
    b = plan_buckets(model_phases("lenet5"), cap_bytes=64 * 1024)
    assert b[0] == (61706 - 16384, 61706, 0)  # backward produces the last layers first
    covered = sorted((a, e) for a, e, _ in b)
    assert covered[0][0] == 0 and covered[-1][1] == 61706
    assert all(covered[i][1] == covered[i + 1][0] for i in range(len(covered) - 1))


def _worker(rank, world, port, model_name, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.manual_seed(100 + rank)  # different init per rank: the reducer must broadcast rank 0's
    m = build_model(model_name)
    if model_name == "mlp":
        m[2].p = 0.0
    red = GlooReducer(m, world, plan_buckets(model_phases(model_name), cap_bytes=32 * 1024))
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8 * world, 784, generator=g)
    y = torch.randint(0, 10, (8 * world,), generator=g)
    xs = x[rank * 8:(rank + 1) * 8]
    if model_name == "lenet5":
        xs = xs.view(-1, 1, 28, 28)
    out = m(xs)
    loss = F.nll_loss(out, y[rank * 8:(rank + 1) * 8]) if model_name == "lenet5" else F.cross_entropy(out, y[rank * 8:(rank + 1) * 8])
    loss.backward()
    red.sync_grads()
    # numpy, not torch tensors: torch's queue pickler shares storage through fds/shm that can
    # vanish when this process exits before the parent has unpickled them (flaky at W=4)
    q.put((rank, {k: v.detach().numpy().copy() for k, v in m.state_dict().items()},
           flatten_grads(m).detach().numpy().copy()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("model_name", ["mlp", "lenet5"])
def test_ddp_equivalence(model_name, world):
    """W ranks x B samples == 1 rank x W*B samples (mean loss), starting from rank 0's weights."""
    port = _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, model_name, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps], key=lambda t: t[0])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    res = [(r, {k: torch.from_numpy(v) for k, v in sd.items()}, torch.from_numpy(g)) for r, sd, g in res]
    sd0, g0 = res[0][1], res[0][2]
    for r in range(1, world):
        sdr, gr = res[r][1], res[r][2]
        for k in sd0:
            assert torch.equal(sd0[k], sdr[k]), "parameters must be broadcast from rank 0 at construction"
        assert torch.allclose(g0, gr)
    # single-process oracle on the full batch from rank 0's initial weights
    torch.manual_seed(100)
    m = build_model(model_name)
    if model_name == "mlp":
        m[2].p = 0.0
    m.load_state_dict(sd0)
    g = torch.Generator().manual_seed(7)
    x = torch.randn(8 * world, 784, generator=g)
    y = torch.randint(0, 10, (8 * world,), generator=g)
    if model_name == "lenet5":
        x = x.view(-1, 1, 28, 28)
    out = m(x)
    (F.nll_loss(out, y) if model_name == "lenet5" else F.cross_entropy(out, y)).backward()
    assert torch.allclose(g0, flatten_grads(m), atol=1e-6, rtol=1e-4)
