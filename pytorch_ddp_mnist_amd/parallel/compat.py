"""Reference-shaped ``distributed`` wire-up object (mnist_cpu_mp.py:14-206).

The reference scripts construct ``distributed(method)`` and (optionally) use its helpers.  This
class keeps that surface on top of :func:`~pytorch_ddp_mnist_amd.parallel.comm.init_distributed`:

  ``get_size()`` / ``get_rank()``   world size / rank, 1 / 0 before initialisation (ref :15-27)
  ``get_local_rank()``              ``LOCAL_RANK`` env, else ``rank % device_count`` on GPUs, else
                                    -1 on CPU (ref :29-39; survey Q21 prefers the env variable)
  ``reduceMAX(src, root=0)``        element-wise MAX over ranks of a vector as float64 (ref :193-199:
                                    ``MPI.COMM_WORLD.Reduce(src, dst, op=MAX, root=root)``).  The
                                    value on ``root`` is the reference's; the other ranks get the same
                                    result instead of the reference's uninitialised ``numpy.empty``
  ``barrier()`` / ``finalize()``    ref :201-206 (never called upstream; here they work, Q16)

No mpi4py: rank/size come from the launcher environment and the control plane is c10d gloo.
"""
from __future__ import annotations

import os
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from .comm import DistContext, init_distributed


class distributed:  # noqa: N801  (reference class name)
    def __init__(self, method: str = "gloo", device: str = "auto", comm: str = "rccl"):
        self.method = method
        self.ctx: DistContext = init_distributed(method, parallel=True, device=device, comm=comm)

    @staticmethod
    def get_size() -> int:
        return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1

    @staticmethod
    def get_rank() -> int:
        return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0

    @staticmethod
    def get_local_rank() -> int:
        if "LOCAL_RANK" in os.environ:
            return int(os.environ["LOCAL_RANK"])
        n = torch.cuda.device_count()
        return distributed.get_rank() % n if n > 0 else -1

    @staticmethod
    def reduceMAX(src, root: int = 0) -> np.ndarray:  # noqa: N802  (reference method name and signature)
        a = np.array(src, dtype=np.float64).reshape(-1)
        world = distributed.get_size()
        if not 0 <= int(root) < world:
            raise ValueError(f"reduceMAX: root {root} outside [0, {world})")
        if not (dist.is_available() and dist.is_initialized()) or world == 1:
            return a.copy()
        t = torch.from_numpy(a.copy())
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return t.numpy()

    @staticmethod
    def barrier() -> None:
        if dist.is_available() and dist.is_initialized():
            dist.barrier()

    def finalize(self) -> None:
        self.ctx.finalize()

    @property
    def device(self) -> torch.device:
        return self.ctx.device

    @property
    def rccl(self) -> Optional[object]:
        return self.ctx.rccl
