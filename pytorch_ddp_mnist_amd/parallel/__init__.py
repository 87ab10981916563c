"""Data-parallel layer: wire-up, communicators, native DDP bucketing, launchers."""
from .compat import distributed
from .module_ddp import DDP, DistributedDataParallel

__all__ = ["distributed", "DistributedDataParallel", "DDP"]
