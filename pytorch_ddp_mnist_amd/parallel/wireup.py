"""Scheduler environment -> (MASTER_ADDR, MASTER_PORT, WORLD_SIZE, RANK, LOCAL_RANK).

Re-design of the reference ``class distributed`` (mnist_cpu_mp.py:14-206,
mnist_pnetcdf_cpu_mp.py:51-272).  The reference mutates ``os.environ`` and
calls ``dist.init_process_group`` in one go and needs mpi4py for fallbacks; here
the env derivation is a pure function (:func:`resolve`) over a mapping, so every
launcher convention is unit-testable with fake environments, and no MPI is
required (rank/size come from PMI/OMPI/SLURM variables, or a world of one).

Methods (same names/choices as the reference):
  nccl-slurm    SLURM_LAUNCH_NODE_IPADDR / SLURM_SRUN_COMM_PORT / SLURM_NTASKS |
                SLURM_JOB_NUM_NODES x SLURM_(N)TASKS_PER_NODE / SLURM_PROCID
                (mnist_cpu_mp.py:47-92; quirk Q2 fixed: ints are parsed and the
                ``"4(x2),3"`` tasks-per-node form is expanded)
  nccl-openmpi  PMIX_SERVER_URI2 host / OMPI_COMM_WORLD_{SIZE,RANK}
                (mnist_cpu_mp.py:94-116; quirk Q1 fixed: the env mapping is
                subscripted and ``:port`` stripped)
  nccl-mpich    PMI_SIZE / PMI_RANK, defaults localhost:29500, world of one
                (mnist_cpu_mp.py:118-145)
  gloo          OMPI_* then PMI_* (mnist_cpu_mp.py:147-188)
  mpich         PMI_* (mnist_pnetcdf_cpu_mp.py:184-211).  Upstream asks for the
                c10d "mpi" backend which stock PyTorch lacks (Q6); here it maps
                to the same data plane as the other methods.

Data plane: on a GPU the gradient all-reduce runs on the native RCCL
communicator (``parallel.comm``); ``torch.distributed`` is initialised with
the ``gloo`` backend and used only as the control plane (TCPStore rendezvous,
unique-id exchange, barriers, timing reductions).  On CPU, gloo is both.
"""
from __future__ import annotations

import os
import re
from dataclasses import dataclass
from typing import Mapping, MutableMapping, Optional

DEFAULT_PORT = "29500"


class WireupError(RuntimeError):
    """Missing or malformed launcher environment (reference raises bare Exception)."""


@dataclass(frozen=True)
class WireupEnv:
    method: str
    master_addr: str
    master_port: int
    world_size: int
    rank: int
    local_rank: Optional[int]

    def export(self, env: MutableMapping[str, str]) -> None:
        env["MASTER_ADDR"] = self.master_addr
        env["MASTER_PORT"] = str(self.master_port)
        env["WORLD_SIZE"] = str(self.world_size)
        env["RANK"] = str(self.rank)
        if self.local_rank is not None:
            env["LOCAL_RANK"] = str(self.local_rank)


def parse_slurm_tasks_per_node(spec: str) -> list:
    """Expand SLURM's compressed list: ``"4(x2),3"`` -> ``[4, 4, 3]``."""
    out = []
    for part in spec.split(","):
        part = part.strip()
        if not part:
            continue
        m = re.fullmatch(r"(\d+)(?:\(x(\d+)\))?", part)
        if not m:
            raise WireupError(f"cannot parse SLURM tasks-per-node spec {spec!r}")
        out += [int(m.group(1))] * int(m.group(2) or 1)
    return out


def pmix_host(uri: str) -> str:
    """``"pmix-server.1;tcp4://10.1.2.3:4242"`` -> ``"10.1.2.3"`` (fixes Q1)."""
    if "//" not in uri:
        raise WireupError(f"unexpected PMIX_SERVER_URI2 {uri!r}")
    host = uri.split("//", 1)[1]
    if host.startswith("["):               # IPv6 literal
        return host[1:host.index("]")]
    return host.split(":")[0]


def _local_rank(env: Mapping[str, str]) -> Optional[int]:
    for k in ("LOCAL_RANK", "SLURM_LOCALID", "OMPI_COMM_WORLD_LOCAL_RANK", "MPI_LOCALRANKID",
              "PMI_LOCAL_RANK", "MV2_COMM_WORLD_LOCAL_RANK"):
        if k in env:
            return int(env[k])
    return None


def resolve(method: str, env: Mapping[str, str]) -> WireupEnv:
    """Derive the rendezvous parameters for ``method`` from ``env`` (pure)."""
    def first(*keys):
        for k in keys:
            if k in env and env[k] != "":
                return env[k]
        return None

    if method == "nccl-slurm":
        addr = first("MASTER_ADDR", "SLURM_LAUNCH_NODE_IPADDR")
        if addr is None:
            raise WireupError("nccl-slurm: neither MASTER_ADDR nor SLURM_LAUNCH_NODE_IPADDR is set")
        port = first("MASTER_PORT", "SLURM_SRUN_COMM_PORT") or DEFAULT_PORT
        ws = first("WORLD_SIZE", "SLURM_NTASKS")
        if ws is None:
            nodes = first("SLURM_JOB_NUM_NODES")
            if nodes is None:
                raise WireupError("nccl-slurm: SLURM_JOB_NUM_NODES is not set")
            per = first("SLURM_NTASKS_PER_NODE")
            if per is not None:
                ws = int(per.split("(")[0]) * int(nodes)
            else:
                tpn = first("SLURM_TASKS_PER_NODE")
                if tpn is None:
                    raise WireupError("nccl-slurm: SLURM_(N)TASKS_PER_NODE is not set")
                counts = parse_slurm_tasks_per_node(tpn)
                ws = sum(counts) if len(counts) > 1 else counts[0] * int(nodes)
        rank = first("RANK", "SLURM_PROCID")
        if rank is None:
            raise WireupError("nccl-slurm: SLURM_PROCID is not set")
    elif method == "nccl-openmpi":
        addr = first("MASTER_ADDR")
        if addr is None:
            uri = first("PMIX_SERVER_URI2")
            if uri is None:
                raise WireupError("nccl-openmpi: PMIX_SERVER_URI2 is not set")
            addr = pmix_host(uri)
        port = first("MASTER_PORT") or DEFAULT_PORT
        ws = first("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE")
        if ws is None:
            raise WireupError("nccl-openmpi: OMPI_COMM_WORLD_SIZE is not set")
        rank = first("RANK", "OMPI_COMM_WORLD_RANK")
        if rank is None:
            raise WireupError("nccl-openmpi: OMPI_COMM_WORLD_RANK is not set")
    elif method in ("nccl-mpich", "mpich"):
        addr = first("MASTER_ADDR") or "localhost"
        port = first("MASTER_PORT") or DEFAULT_PORT
        ws = first("WORLD_SIZE", "PMI_SIZE") or 1
        rank = first("RANK", "PMI_RANK") or 0
    elif method == "gloo":
        addr = first("MASTER_ADDR")
        if addr is None:
            uri = first("PMIX_SERVER_URI2")
            addr = pmix_host(uri) if uri is not None else "localhost"
        port = first("MASTER_PORT") or DEFAULT_PORT
        ws = first("WORLD_SIZE", "OMPI_COMM_WORLD_SIZE", "PMI_SIZE") or 1
        rank = first("RANK", "OMPI_COMM_WORLD_RANK", "PMI_RANK") or 0
    else:
        raise NotImplementedError(f"wireup method {method!r}")

    ws, rank = int(ws), int(rank)
    if not (0 <= rank < ws):
        raise WireupError(f"{method}: rank {rank} outside world of size {ws}")
    return WireupEnv(method, str(addr), int(port), ws, rank, _local_rank(env))


def pick_local_rank(w: WireupEnv, n_devices: int) -> int:
    """``LOCAL_RANK``-style env first (Q21), else ``rank % n_devices`` (mnist_cpu_mp.py:34)."""
    if w.local_rank is not None:
        return w.local_rank
    return w.rank % max(1, n_devices)


def is_gpu_method(method: str) -> bool:
    return method.startswith("nccl") or method == "mpich"


def apply(method: str, env: Optional[MutableMapping[str, str]] = None) -> WireupEnv:
    """Resolve and export into ``env`` (defaults to ``os.environ``)."""
    env = os.environ if env is None else env
    w = resolve(method, env)
    w.export(env)
    return w
