"""DataLoader-compatible device batch iterators over an HBM-resident MNIST split.

Reference: ``create_data_loaders(batch_size)`` (ddp_tutorial_cpu.py:12-40), its distributed
variant with ``DistributedSampler(num_replicas, rank, shuffle=True, seed=42)``
(ddp_tutorial_multi_gpu.py:13-49, mnist_cpu_mp.py:304-341) and the PnetCDF loaders
(mnist_pnetcdf_cpu.py:141-151, mnist_pnetcdf_cpu_mp.py:370-409).  There, every batch costs 128
Python ``__getitem__`` calls + PIL decode + ToTensor/Normalize in worker processes, a pin-memory
thread and a host->device copy (survey N13/N14).

Here the split is uploaded once (47 MB uint8; pinned staging + ``hipMemcpyAsync``,
``device_loader``), each epoch's sample order (bit-equal to ``DistributedSampler``) is uploaded as
ONE int32 vector, and every batch is produced on the device by the native ``gather_normalize``
kernel: ``x[r] = ((images[idx[r]] / 255) - 0.1307) / 0.3081`` in fp32 or bf16.  The loader has
the surface the reference's training loops use — ``len()``, iteration yielding ``(x, y)``, and
``loader.sampler.set_epoch(i)`` — so a bring-your-own-model loop (with
:class:`~pytorch_ddp_mnist_amd.parallel.module_ddp.DistributedDataParallel`) switches over
unchanged.  On CPU the same batches come from torch indexing (plumbing / tests).
"""
from __future__ import annotations

from typing import Iterator, Optional, Tuple

import numpy as np
import torch

from .datasets import load_arrays, normalize_batch
from .device_loader import upload_arrays, upload_netcdf
from .sampler import ShardedSampler, batch_slices


class DeviceBatchLoader:
    """Iterable of ``(x, y)`` batches; ``x`` is ``[B,784]`` (``layout="flat"``) or ``[B,1,28,28]``."""

    def __init__(self, images: torch.Tensor, labels: torch.Tensor, batch_size: int = 128,
                 sampler: Optional[ShardedSampler] = None, shuffle: bool = True, seed: int = 0,
                 layout: str = "flat", dtype: torch.dtype = torch.float32, drop_last: bool = False):
        if layout not in ("flat", "image"):
            raise ValueError("layout must be 'flat' or 'image'")
        if dtype not in (torch.float32, torch.bfloat16):
            raise ValueError("dtype must be float32 or bfloat16")
        self.images = images.view(-1, 784)
        self.labels = labels.view(-1)
        self.device = self.images.device
        self.batch_size = int(batch_size)
        self.sampler = sampler or ShardedSampler(self.images.shape[0], 1, 0, shuffle=shuffle, seed=seed)
        self.layout, self.dtype, self.drop_last = layout, dtype, drop_last
        self._auto_epoch = sampler is None  # plain shuffle=True loaders reshuffle every pass
        self._C = None
        if self.device.type == "cuda":
            from ..ops.native import require_gpu
            self._C = require_gpu()
            self._zero = torch.zeros(1, dtype=torch.int32, device=self.device)
            self._labels_i64 = self.labels.to(torch.int64)

    def __len__(self) -> int:
        return len(batch_slices(len(self.sampler), self.batch_size, self.drop_last))

    def _shape(self, x: torch.Tensor) -> torch.Tensor:
        return x if self.layout == "flat" else x.view(-1, 1, 28, 28)

    def __iter__(self) -> Iterator[Tuple[torch.Tensor, torch.Tensor]]:
        order = self.sampler.indices()
        if self._auto_epoch:
            self.sampler.set_epoch(self.sampler.epoch + 1)
        slices = batch_slices(order.numel(), self.batch_size, self.drop_last)
        if self._C is None:
            for s, b in slices:
                idx = order[s:s + b]
                x = normalize_batch(self.images[idx]).to(self.dtype)
                yield self._shape(x), self.labels[idx].to(torch.int64)
            return
        stream = torch.cuda.current_stream(self.device)
        idx_dev = order.to(torch.int32).pin_memory().to(self.device, non_blocking=True)
        did = 0 if self.dtype == torch.float32 else 1
        for s, b in slices:
            x = torch.empty(b, 784, dtype=self.dtype, device=self.device)
            self._C.gather_normalize(did, self.images.data_ptr(), idx_dev.data_ptr() + 4 * s,
                                     self._zero.data_ptr(), b, x.data_ptr(), 784, stream.cuda_stream)
            y = self._labels_i64.index_select(0, idx_dev[s:s + b].long())
            yield self._shape(x), y


def _split_loaders(xtr, ytr, xte, yte, batch_size, world_size, rank, device, layout, dtype, seed,
                   test_shuffle) -> Tuple[DeviceBatchLoader, DeviceBatchLoader]:
    dev = torch.device(device)
    if dev.type == "cuda":
        dx, dy = upload_arrays(xtr, ytr, dev)
        tx, ty = upload_arrays(xte, yte, dev)
    else:
        dx, dy = torch.from_numpy(np.ascontiguousarray(xtr).reshape(-1, 784)), torch.from_numpy(ytr)
        tx, ty = torch.from_numpy(np.ascontiguousarray(xte).reshape(-1, 784)), torch.from_numpy(yte)
    sampler = ShardedSampler(dx.shape[0], world_size, rank, shuffle=True, seed=seed) if world_size > 1 else None
    train = DeviceBatchLoader(dx, dy, batch_size, sampler, True, seed, layout, dtype)
    test = DeviceBatchLoader(tx, ty, batch_size, None, test_shuffle, seed, layout, dtype)  # test is not sharded (Q8)
    return train, test


def create_data_loaders(batch_size: int = 128, world_size: int = 1, rank: int = 0, device="cpu",
                        fmt: str = "auto", root: Optional[str] = None, limit: Optional[int] = None,
                        layout: str = "flat", dtype: torch.dtype = torch.float32, seed: int = 42,
                        test_shuffle: bool = True) -> Tuple[DeviceBatchLoader, DeviceBatchLoader]:
    """(train_loader, test_loader) over idx-ubyte / netCDF / synthetic MNIST.

    ``world_size > 1`` shards the train split exactly like ``DistributedSampler(seed=42)``; call
    ``train_loader.sampler.set_epoch(i)`` each epoch as the reference does.  The test split is
    not sharded (reference behaviour, survey Q8) and is shuffled like the reference's test loader
    (``shuffle=True``, Q20).
    """
    xtr, ytr, xte, yte, _ = load_arrays(fmt, root, limit, verbose=False)
    return _split_loaders(xtr, ytr, xte, yte, batch_size, world_size, rank, device, layout, dtype, seed,
                          test_shuffle)


def create_netcdf_loaders(root_dir: str = ".", batch_size: int = 128, world_size: int = 1, rank: int = 0,
                          device="cpu", layout: str = "flat", dtype: torch.dtype = torch.float32,
                          seed: int = 42, limit: Optional[int] = None
                          ) -> Tuple[DeviceBatchLoader, DeviceBatchLoader]:
    """PnetCDF-path loaders over ``root_dir/mnist_{train,test}_images.nc`` (CDF-1/2/5).

    On a GPU the file bytes go pread -> pinned host memory -> HBM without an intermediate copy.
    """
    import os
    dev = torch.device(device)
    tr = os.path.join(root_dir, "mnist_train_images.nc")
    te = os.path.join(root_dir, "mnist_test_images.nc")
    dx, dy = upload_netcdf(tr, dev, limit)
    tx, ty = upload_netcdf(te, dev)
    sampler = ShardedSampler(dx.shape[0], world_size, rank, shuffle=True, seed=seed) if world_size > 1 else None
    return (DeviceBatchLoader(dx, dy, batch_size, sampler, True, seed, layout, dtype),
            DeviceBatchLoader(tx, ty, batch_size, None, True, seed, layout, dtype))
