"""Typed configuration and reference-compatible command lines.

Reference behaviour reproduced here:
  * ``configure()`` of ``mnist_cpu_mp.py:208-243`` / ``mnist_pnetcdf_cpu_mp.py:274-309``:
    flags --wireup_method, --data_path, --data_limit, --batch_size, --n_epochs,
    --num_workers, --parallel, --hdf5; result is a nested dict
    ``config["trainer"] / config["data"]`` with defaults batch_size=128,
    device=0, n_epochs=1, num_workers=0, limit=None, label_map=[0,1,0,0,2,3,1,4].
  * ``--local_rank`` of ``ddp_tutorial_multi_gpu.py:122-124`` (plus the dashed
    ``--local-rank`` that torch>=2 launchers pass, survey quirk Q5, and the
    ``LOCAL_RANK`` env var).

Additive flags (survey §5.6): --model, --dtype, --momentum, --lr, --synthetic,
--bucket_cap_kb, --profile, --seed, --no_save, --comm, --no_graph, --plan, --allreduce, --tqdm, --progress_every,
--resume, --io_mode.
"""
from __future__ import annotations

import argparse
import os
from dataclasses import dataclass, field, asdict
from typing import List, Optional

WIREUP_METHODS = ["nccl-slurm", "nccl-openmpi", "nccl-mpich", "gloo"]
WIREUP_METHODS_PNETCDF = WIREUP_METHODS + ["mpich"]
MODELS = ["mlp", "lenet5"]
DTYPES = ["fp32", "bf16"]


@dataclass
class TrainConfig:
    """Flat typed view of everything a training run needs."""
    model: str = "mlp"
    dtype: str = "fp32"
    batch_size: int = 128
    n_epochs: int = 1
    lr: float = 0.01
    momentum: float = 0.0
    dropout: float = 0.2
    seed: int = 42              # DistributedSampler seed (ddp_tutorial_multi_gpu.py:30)
    init_seed: Optional[int] = None
    wireup_method: str = "nccl-slurm"
    parallel: bool = False
    device: str = "auto"       # "cpu" | "cuda" | "auto"
    num_workers: int = 0
    data_path: Optional[str] = None
    data_limit: Optional[int] = None
    data_format: str = "auto"  # "idx" | "netcdf" | "synthetic" | "auto"
    hdf5: bool = False
    label_map: List[int] = field(default_factory=lambda: [0, 1, 0, 0, 2, 3, 1, 4])
    save_path: Optional[str] = "model.pt"
    bucket_cap_kb: Optional[int] = None
    comm: str = "rccl"          # "rccl" (native communicator) | "torch" (c10d)
    graph: bool = True          # capture the training step in a hipGraph
    profile: bool = False
    disable_tqdm: bool = True
    metrics_jsonl: Optional[str] = None
    local_rank: Optional[int] = None
    shard_eval: bool = False
    progress_every: int = 0     # --tqdm update period in batches (0 = ~20 updates per epoch)
    plan: str = "auto"          # multi-GPU step plan: "auto" (timed at start-up) | "join" | "split" | "overlap"
    allreduce: str = "rccl"     # gradient data plane with --comm rccl: "rccl" | "oneshot" (parallel/oneshot.py)
    io_mode: str = "bulk"       # netCDF: "bulk" (one pread per variable) | "per_sample" (reference __getitem__
                                # reads, whole epoch first) | "interleaved" (each batch read before its step)
    resume: Optional[str] = None  # params + momentum + epoch file: loaded if present, rewritten each epoch

    def to_nested(self) -> dict:
        """Nested dict in the reference layout (mnist_cpu_mp.py:223-241)."""
        return {
            "trainer": {
                "batch_size": self.batch_size,
                "wireup_method": self.wireup_method,
                "parallel": self.parallel,
                "device": 0 if self.device in ("auto", "cuda") else self.device,
                "n_epochs": self.n_epochs,
                "num_workers": self.num_workers,
            },
            "data": {
                "limit": self.data_limit,
                "label_map": list(self.label_map),
                "hdf5": self.hdf5,
                **({"path": self.data_path} if self.data_path is not None else {}),
            },
        }

    def as_dict(self) -> dict:
        return asdict(self)


def _add_extra_flags(p: argparse.ArgumentParser, defaults: TrainConfig) -> None:
    add = p.add_argument
    add("--model", type=str, default=None, choices=MODELS, help="network: reference MLP or LeNet-5")
    add("--dtype", type=str, default=None, choices=DTYPES, help="MFMA input dtype (master weights stay fp32)")
    add("--lr", type=float, default=None, help="SGD learning rate (reference: 0.01)")
    add("--momentum", type=float, default=None, help="SGD momentum (reference: 0)")
    add("--dropout", type=float, default=None, help="MLP dropout probability (reference: 0.2)")
    add("--seed", type=int, default=None, help="sampler seed (reference: 42)")
    add("--init_seed", type=int, default=None, help="torch.manual_seed before model init")
    add("--synthetic", action="store_true", help="use the deterministic synthetic MNIST generator")
    add("--data_format", type=str, default=None, choices=["auto", "idx", "netcdf", "synthetic"])
    add("--device", type=str, default=None, choices=["auto", "cpu", "cuda"])
    add("--bucket_cap_kb", type=int, default=None, help="DDP gradient bucket cap (KiB)")
    add("--comm", type=str, default=None, choices=["rccl", "torch", "gloo"],
        help="gradient all-reduce path: native RCCL, c10d nccl, or c10d gloo via host memory (ranks may share a GPU)")
    add("--no_graph", action="store_true", help="launch the step eagerly instead of replaying a hipGraph")
    add("--profile", action="store_true", help="emit roctx ranges and per-phase timers")
    add("--no_save", action="store_true", help="do not write model.pt")
    add("--save_path", type=str, default=None)
    add("--metrics_jsonl", type=str, default=None, help="append per-epoch metrics as JSON lines")
    add("--tqdm", action="store_true", help="rank-0 progress bars with the batch loss (reference: tqdm per batch)")
    add("--progress_every", type=int, default=None, help="--tqdm update period in batches (one device sync each)")
    add("--shard_eval", action="store_true", help="shard the test set across ranks (reference: every rank evaluates all)")
    add("--plan", type=str, default=None, choices=["auto", "join", "split", "overlap", "fixed"],
        help="step plan (auto: time the candidate schedules at start-up; join/split: multi-GPU plan; overlap: LeNet, "
             "one-shot all-reduces inside the backward branches; fixed: defaults)")
    add("--allreduce", type=str, default=None, choices=["rccl", "oneshot"],
        help="gradient data plane with --comm rccl: RCCL, or the one-shot all-reduce over IPC-mapped peer slots "
             "(validated at start-up; RCCL still broadcasts the initial parameters)")
    add("--io_mode", type=str, default=None, choices=["bulk", "per_sample", "interleaved"],
        help="netCDF input: bulk pread (default), or the reference's per-sample __getitem__ reads, timed (MB/s): "
             "per_sample reads the epoch first, interleaved reads each batch beside the training steps")
    add("--resume", type=str, default=None,
        help="resume file (params + momentum + epoch): loaded when it exists, rewritten after every epoch")


def _apply_extra(cfg: TrainConfig, a: argparse.Namespace) -> None:
    for name in ("model", "dtype", "lr", "momentum", "dropout", "seed", "init_seed", "data_format",
                 "device", "bucket_cap_kb", "comm", "save_path", "metrics_jsonl", "plan", "resume", "progress_every",
                 "io_mode", "allreduce"):
        v = getattr(a, name, None)
        if v is not None:
            setattr(cfg, name, v)
    if getattr(a, "synthetic", False):
        cfg.data_format = "synthetic"
    if getattr(a, "no_graph", False):
        cfg.graph = False
    if getattr(a, "profile", False):
        cfg.profile = True
    if getattr(a, "no_save", False):
        cfg.save_path = None
    if getattr(a, "tqdm", False):
        cfg.disable_tqdm = False
    if getattr(a, "shard_eval", False):
        cfg.shard_eval = True


def mp_parser(pnetcdf: bool = False) -> argparse.ArgumentParser:
    """The reference ``configure()`` parser (mnist_cpu_mp.py:210-221) plus additive flags."""
    p = argparse.ArgumentParser(description="Evaluate cost of reading input files")
    add = p.add_argument
    add("--wireup_method", type=str, default="nccl-slurm",
        choices=WIREUP_METHODS_PNETCDF if pnetcdf else WIREUP_METHODS,
        help="Choose backend for distributed environment initialization")
    add("--data_path", type=str, default=None, help="File path to training samples")
    add("--data_limit", type=int, default=None, help="Max number of samples to be used")
    add("--batch_size", type=int, default=None, help="Batch size")
    add("--n_epochs", type=int, default=None, help="Number of epochs")
    add("--num_workers", type=int, default=None, help="Number of subprocesses to use for data loading")
    add("--parallel", action="store_true", help="To run in parallel")
    add("--hdf5", action="store_true", help="Read from HDF5 files")
    _add_extra_flags(p, TrainConfig())
    return p


def configure(argv: Optional[List[str]] = None, pnetcdf: bool = False,
              base: Optional[TrainConfig] = None) -> TrainConfig:
    """Parse the reference multi-process CLI into a :class:`TrainConfig`.

    CLI values override defaults only when given (``!= None``), exactly like
    mnist_cpu_mp.py:237-241.
    """
    a = mp_parser(pnetcdf).parse_args(argv)
    cfg = base if base is not None else TrainConfig()
    cfg.wireup_method = a.wireup_method
    cfg.parallel = a.parallel
    cfg.hdf5 = a.hdf5
    if a.data_path is not None:
        cfg.data_path = a.data_path
    if a.data_limit is not None:
        cfg.data_limit = a.data_limit
    if a.batch_size is not None:
        cfg.batch_size = a.batch_size
    if a.n_epochs is not None:
        cfg.n_epochs = a.n_epochs
    if a.num_workers is not None:
        cfg.num_workers = a.num_workers
    _apply_extra(cfg, a)
    return cfg


def gpu_tutorial_parser() -> argparse.ArgumentParser:
    """``ddp_tutorial_multi_gpu.py:122-124`` parser, accepting both rank spellings (Q5)."""
    p = argparse.ArgumentParser()
    p.add_argument("--local_rank", "--local-rank", dest="local_rank", type=int, default=None)
    p.add_argument("--batch_size", type=int, default=None)
    p.add_argument("--n_epochs", "--epochs", dest="n_epochs", type=int, default=None)
    _add_extra_flags(p, TrainConfig())
    return p


def configure_gpu_tutorial(argv: Optional[List[str]] = None) -> TrainConfig:
    """Config for ddp_tutorial_multi_gpu.py: B=128, epochs=10 (:126-127)."""
    a = gpu_tutorial_parser().parse_args(argv)
    cfg = TrainConfig(batch_size=128, n_epochs=10, parallel=True, device="cuda")
    lr = a.local_rank
    if lr is None and "LOCAL_RANK" in os.environ:
        lr = int(os.environ["LOCAL_RANK"])
    cfg.local_rank = lr
    if a.batch_size is not None:
        cfg.batch_size = a.batch_size
    if a.n_epochs is not None:
        cfg.n_epochs = a.n_epochs
    _apply_extra(cfg, a)
    return cfg


def simple_parser(description: str = "") -> argparse.ArgumentParser:
    """Parser for the no-argument reference scripts (ddp_tutorial_cpu.py, mnist_pnetcdf_cpu.py):
    they take no flags upstream; we accept only the additive ones."""
    p = argparse.ArgumentParser(description=description)
    p.add_argument("--batch_size", type=int, default=None)
    p.add_argument("--n_epochs", "--epochs", dest="n_epochs", type=int, default=None)
    p.add_argument("--data_path", type=str, default=None)
    p.add_argument("--data_limit", type=int, default=None)
    _add_extra_flags(p, TrainConfig())
    return p


def configure_simple(argv: Optional[List[str]] = None, base: Optional[TrainConfig] = None,
                     description: str = "") -> TrainConfig:
    a = simple_parser(description).parse_args(argv)
    cfg = base if base is not None else TrainConfig()
    for name in ("batch_size", "n_epochs", "data_path", "data_limit"):
        v = getattr(a, name)
        if v is not None:
            setattr(cfg, name, v)
    _apply_extra(cfg, a)
    return cfg
