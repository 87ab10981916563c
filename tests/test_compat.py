"""Reference-shaped ``distributed`` wire-up object (parallel/compat.py), gloo world 2 on CPU."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q):
    # OpenMPI-style launcher variables, as `mpirun` would export them (gloo method, mnist_cpu_mp.py:147-188)
    os.environ.update(OMPI_COMM_WORLD_SIZE=str(world), OMPI_COMM_WORLD_RANK=str(rank),
                      OMPI_COMM_WORLD_LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    from pytorch_ddp_mnist_amd.parallel import distributed
    assert distributed.get_size() == 1 and distributed.get_rank() == 0  # before init: fallbacks
    d = distributed("gloo", device="cpu")
    out = (d.get_size(), d.get_rank(), d.reduceMAX(np.array([rank, -rank, 3.5]), 0).tolist(), str(d.device))
    d.barrier()
    d.finalize()
    q.put((rank, out))


def test_distributed_helpers_w2():
    world, port = 2, _port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=120) for _ in ps])
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    for rank, (size, r, mx, dev) in res:
        assert (size, r, dev) == (2, rank, "cpu")
        assert mx == [1.0, 0.0, 3.5]
