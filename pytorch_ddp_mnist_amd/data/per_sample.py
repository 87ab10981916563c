"""The reference's I/O-cost experiment: every sample of every epoch read through the Dataset.

Reference: ``MNISTNetCDF.__getitem__`` issues two independent reads per sample -- the 784-byte
image row and the 1-byte label (``mnist_pnetcdf_cpu_mp.py:39-49``) -- from a DataLoader over a
DistributedSampler, which is what the argparse description "Evaluate cost of reading input
files" (``mnist_cpu_mp.py:210``) measures.  ``--io_mode per_sample`` reproduces that access
pattern (same ``Dataset`` class, same per-sample calls, sampler order, every epoch) and times it,
instead of the default bulk ``pread`` of the whole variable.

Two schedules:
  * ``per_sample`` -- the samples of an epoch are gathered on the host in sampler order and then handed
    to the engine as that epoch's resident data, so the measured read cost is isolated from the step;
  * ``interleaved`` -- :class:`InterleavedLoader` reads each batch right before the step that consumes
    it, as the reference's DataLoader with ``num_workers=0`` does (mnist_pnetcdf_cpu_mp.py:39-49 called
    from the loader of :370-409, inside the training loop).  On the GPU the batch's host read overlaps
    the previous (asynchronous) step; its rows go through a pinned two-slot ring into the resident
    buffer.  Same batches, same order: the training is bitwise that of ``per_sample``.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Optional, Tuple

import numpy as np
import torch

from .datasets import MNISTNetCDF


@dataclass
class ReadStats:
    samples: int = 0
    bytes: int = 0
    seconds: float = 0.0

    @property
    def mb_per_s(self) -> float:
        return self.bytes / 1e6 / self.seconds if self.seconds > 0 else 0.0

    @property
    def samples_per_s(self) -> float:
        return self.samples / self.seconds if self.seconds > 0 else 0.0

    def line(self, what: str) -> str:
        return (f"{what}: {self.samples} samples, {self.bytes / 1e6:.2f} MB in {self.seconds:.3f} s "
                f"= {self.mb_per_s:.2f} MB/s ({self.samples_per_s:,.0f} samples/s, 2 reads per sample)")


class InterleavedLoader:
    """``loader(s, b)``: read the samples at positions [s, s+b) of this epoch's sampler order through
    ``reader`` (one ``__getitem__`` each) and hand them to ``write_rows(x, y, s)`` -- called by the
    engine right before the step that trains on rows [s, s+b).  ``stats`` sums the read time."""

    def __init__(self, reader: "PerSampleReader", order, write_rows):
        self.reader, self.write_rows = reader, write_rows
        self.order = order.tolist() if isinstance(order, torch.Tensor) else list(order)
        self.stats = ReadStats()

    def __call__(self, s: int, b: int) -> None:
        x, y, st = self.reader.read(self.order[s:s + b])
        self.stats.samples += st.samples
        self.stats.bytes += st.bytes
        self.stats.seconds += st.seconds
        self.write_rows(x, y, s)


class PerSampleReader:
    """Wraps a reference-API :class:`MNISTNetCDF` (no transform: raw uint8 rows, the kernels
    normalise on the device) and reads index lists one ``__getitem__`` at a time."""

    def __init__(self, root: str, is_train: bool, comm=None):
        self.ds = MNISTNetCDF(root, is_train, transforms=None, comm=comm)

    def __len__(self) -> int:
        return len(self.ds)

    def read(self, indices, limit: Optional[int] = None) -> Tuple[np.ndarray, np.ndarray, ReadStats]:
        idx = indices.tolist() if isinstance(indices, torch.Tensor) else list(indices)
        if limit is not None:
            idx = idx[:limit]
        n = len(idx)
        x = np.empty((n, 784), np.uint8)
        y = np.empty(n, np.uint8)
        t0 = time.perf_counter()
        for j, i in enumerate(idx):
            img, lab = self.ds[i]
            x[j] = np.asarray(img, np.uint8).reshape(784)
            y[j] = lab
        dt = time.perf_counter() - t0
        return x, y, ReadStats(n, n * 785, dt)
