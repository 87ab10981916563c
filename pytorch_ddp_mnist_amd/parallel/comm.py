"""Process-group bring-up: control plane (c10d gloo + TCPStore) and data plane (native RCCL).

Reference equivalents: ``torch.distributed.init_process_group(NCCL, env://)``
(ddp_tutorial_multi_gpu.py:132-134) and ``class distributed`` (mnist_cpu_mp.py:14-206).

Design (MI355X-first):
  * ``torch.distributed`` is initialised with the **gloo** backend over ``env://``: it carries
    only control traffic — the TCPStore rendezvous, the 128-byte RCCL unique id, barriers and
    the max-reduction of timings.  It never touches gradients.
  * On GPUs the gradient all-reduce goes through the native :class:`RcclComm`
    (``csrc/runtime/rccl_comm.cpp``): one communicator per process, collectives enqueued on the
    trainer's side HIP stream inside the captured step graph (RCCL over xGMI on an MI355X
    node).  ``comm="torch"`` instead initialises ``cpu:gloo,cuda:nccl`` and lets c10d's NCCL
    (= RCCL) process group do the all-reduce (kept for A/B comparison).
  * On CPU (no GPU, or ``device=cpu``) everything is gloo, as the reference forces
    (mnist_cpu_mp.py:247-250).
"""
from __future__ import annotations

import datetime
import os
import sys
from dataclasses import dataclass
from typing import Optional

import torch
import torch.distributed as dist

from . import wireup as W

UID_KEY = "mnist_amd/rccl_uid"


@dataclass
class DistContext:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    device: torch.device = torch.device("cpu")
    backend: str = "none"          # "none" | "gloo" | "cpu:gloo,cuda:nccl"
    rccl: Optional[object] = None  # native RcclComm
    method: Optional[str] = None

    @property
    def is_distributed(self) -> bool:
        return self.world > 1 and dist.is_available() and dist.is_initialized()

    def barrier(self) -> None:
        if self.is_distributed:
            dist.barrier()

    def all_reduce_max(self, value: float) -> float:
        if not self.is_distributed:
            return value
        t = torch.tensor([value], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def all_reduce_sum(self, values):
        if not self.is_distributed:
            return list(values)
        t = torch.tensor(list(values), dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return t.tolist()

    def finalize(self, *trainers) -> None:
        """Clean teardown in a fixed order (the reference never calls its finalize(), survey Q16):
        1. every trainer drops its graphs (they captured collectives), detaches and destroys its native streams
           and events (``close``; ``release`` for objects without one);
        2. the RCCL communicator is flushed and destroyed (``ncclCommFinalize`` -> ``ncclCommDestroy``,
           bounded; aborted if the flush does not complete);
        3. the gloo control plane: barrier, ``destroy_process_group``."""
        for tr in trainers:
            if tr is not None and hasattr(tr, "close"):
                tr.close()
            elif tr is not None and hasattr(tr, "release"):
                tr.release()
        if self.rccl is not None:
            err = self.rccl.destroy(comm_timeout())
            if err:
                print(f"[rank {self.rank}] RCCL teardown: {err}", file=sys.stderr, flush=True)
        self.rccl = None
        if dist.is_available() and dist.is_initialized():
            try:
                dist.barrier()
            except Exception:
                pass
            dist.destroy_process_group()


def _want_gpu(device: str) -> bool:
    if device == "cpu":
        return False
    # counting devices does not initialise HIP on this image; is_available() does
    return torch.cuda.device_count() > 0


def init_distributed(method: Optional[str] = None, parallel: bool = True, device: str = "auto",
                     comm: str = "rccl", timeout_s: float = 600.0, share_device: bool = False) -> DistContext:
    """Bring up rank/world/device and the communicators.

    ``method=None`` uses plain ``env://`` variables (torchrun / torch.distributed.launch); a
    reference wire-up name derives them from the scheduler environment first.
    ``comm``: ``rccl`` (gloo control plane + native RCCL data plane), ``torch`` (c10d nccl data
    plane) or ``gloo`` (everything over gloo).  ``share_device`` (only with ``comm="gloo"``) maps local
    rank r to GPU r % device_count, so several ranks can share one GPU (RCCL refuses that).
    """
    if share_device and comm != "gloo":
        raise ValueError("share_device needs comm='gloo' (RCCL refuses two ranks on one device)")
    use_gpu = _want_gpu(device)
    if not parallel:
        lr = int(os.environ.get("LOCAL_RANK", 0)) if use_gpu else 0
        dev = torch.device("cuda", lr) if use_gpu else torch.device("cpu")
        if use_gpu:
            torch.cuda.set_device(dev)
        return DistContext(0, 1, lr, dev, "none", None, method)

    if method is not None:
        w = W.apply(method)
    else:
        w = W.resolve("gloo", os.environ)
        w.export(os.environ)
    ndev = torch.cuda.device_count() if use_gpu else 1
    local_rank = W.pick_local_rank(w, ndev)
    if use_gpu and local_rank >= ndev:
        if not share_device:
            raise RuntimeError(f"local rank {local_rank} but only {ndev} GPU(s) visible (one rank per GPU; "
                               f"--comm gloo lets ranks share a GPU)")
    dev = torch.device("cuda", local_rank % ndev) if use_gpu else torch.device("cpu")
    if use_gpu:
        torch.cuda.set_device(dev)
    backend = "cpu:gloo,cuda:nccl" if (use_gpu and comm == "torch") else "gloo"
    if w.world_size > 1 or method is not None:
        if not dist.is_initialized():
            kw = {}
            if backend != "gloo":
                kw["device_id"] = dev
            dist.init_process_group(backend=backend, init_method="env://", world_size=w.world_size,
                                    rank=w.rank, timeout=datetime.timedelta(seconds=timeout_s), **kw)
    ctx = DistContext(w.rank, w.world_size, local_rank, dev, backend if dist.is_initialized() else "none",
                      None, method)
    if use_gpu and comm == "rccl" and w.world_size > 1:
        ctx.rccl = make_rccl(ctx)
    return ctx


def comm_timeout() -> float:
    """Collective watchdog deadline in seconds (``MNIST_AMD_COMM_TIMEOUT``, default 600 = c10d's NCCL default)."""
    return float(os.environ.get("MNIST_AMD_COMM_TIMEOUT", "600"))


def comm_init_timeout() -> float:
    """Deadline of the RCCL bring-up (unique-id exchange + communicator init), ``MNIST_AMD_COMM_INIT_TIMEOUT``
    seconds, default 180.  A healthy 8-GPU init takes about a second; past the deadline the rank aborts its
    half-built communicator and raises, naming itself, so the launcher tears the job down instead of every
    rank hanging inside ncclCommInitRank (reference: init_process_group's c10d timeout,
    ddp_tutorial_multi_gpu.py:133-134)."""
    return float(os.environ.get("MNIST_AMD_COMM_INIT_TIMEOUT", "180"))


class CommInitError(RuntimeError):
    """The RCCL bring-up did not complete (peer missing, stalled or failed)."""


def make_rccl(ctx: DistContext, timeout_s: Optional[float] = None):
    """Native RCCL communicator; the unique id travels over the c10d TCPStore.  Bounded: see
    :func:`comm_init_timeout`."""
    from ..ops.native import load_c
    from ..utils.logging import native_stdout_to_stderr
    C = load_c()
    timeout_s = comm_init_timeout() if timeout_s is None else float(timeout_s)
    store = dist.distributed_c10d._get_default_store()
    with native_stdout_to_stderr():  # RCCL's init banner goes to stderr
        if ctx.rank == 0:
            uid = C.RcclComm.make_unique_id()
            store.set(UID_KEY, uid)
        else:
            try:
                store.wait([UID_KEY], datetime.timedelta(seconds=timeout_s))
            except Exception as e:  # noqa: BLE001 -- c10d raises its own store timeout types
                raise CommInitError(f"rank {ctx.rank} of {ctx.world}: no RCCL unique id from rank 0 within "
                                    f"{timeout_s:.0f} s ({e})") from e
            uid = store.get(UID_KEY)
        try:
            return C.RcclComm(bytes(uid), ctx.rank, ctx.world, ctx.local_rank, init_timeout=timeout_s)
        except RuntimeError as e:
            raise CommInitError(str(e)) from e
