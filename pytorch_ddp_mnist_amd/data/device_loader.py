"""HBM-resident dataset staging: pinned host buffer -> hipMemcpyAsync on a copy stream.

Replaces the reference's per-batch input pipeline (4 DataLoader worker processes decoding PIL
images + a pin-memory thread + ``.to(device, non_blocking=True)`` per batch, survey N13/N14 and
CS1) with a one-time upload: MNIST is 47 MB of uint8 — nothing against 288 GB of HBM — so the
whole split lives on the device and kernels gather rows by index every step.

For netCDF sources the bytes go file -> pinned host memory directly (native ``pread`` into the
pinned tensor's address, no intermediate numpy copy) -> device.
"""
from __future__ import annotations

from typing import Optional, Tuple

import numpy as np
import torch

from . import cdf5


def _pinned_u8(n: int) -> torch.Tensor:
    t = torch.empty(n, dtype=torch.uint8)
    try:
        return t.pin_memory()
    except RuntimeError:       # no GPU (CPU tests): plain memory
        return t


def upload_arrays(images: np.ndarray, labels: np.ndarray, device: torch.device,
                  stream: Optional[torch.cuda.Stream] = None) -> Tuple[torch.Tensor, torch.Tensor]:
    """uint8 images [N,784] and labels [N] on ``device`` via pinned staging + async copy."""
    x = np.ascontiguousarray(images, dtype=np.uint8).reshape(-1, 784)
    y = np.ascontiguousarray(labels, dtype=np.uint8).reshape(-1)
    if device.type != "cuda":
        return torch.from_numpy(x.copy()), torch.from_numpy(y.copy())
    hx = _pinned_u8(x.size)
    hx.numpy()[:] = x.reshape(-1)
    hy = _pinned_u8(y.size)
    hy.numpy()[:] = y
    stream = stream or torch.cuda.Stream(device=device)
    with torch.cuda.stream(stream):
        dx = torch.empty(x.shape, dtype=torch.uint8, device=device)
        dy = torch.empty(y.shape, dtype=torch.uint8, device=device)
        dx.view(-1).copy_(hx, non_blocking=True)
        dy.copy_(hy, non_blocking=True)
    stream.synchronize()
    return dx, dy


def upload_netcdf(path: str, device: torch.device, limit: Optional[int] = None,
                  threads: int = 8) -> Tuple[torch.Tensor, torch.Tensor]:
    """Read a PnetCDF-format MNIST file straight into pinned memory and copy it to HBM."""
    f = cdf5.open_nc(path)
    n = int(f.shape("images")[0]) if limit is None else min(int(limit), int(f.shape("images")[0]))
    if hasattr(f, "read_rows_into"):
        hx = _pinned_u8(n * 784)
        hy = _pinned_u8(n)
        f.read_rows_into("images", 0, n, hx.data_ptr(), hx.numel(), threads)
        f.read_rows_into("labels", 0, n, hy.data_ptr(), hy.numel(), 1)
        if device.type != "cuda":
            return hx.view(n, 784).clone(), hy.clone()
        s = torch.cuda.Stream(device=device)
        with torch.cuda.stream(s):
            dx = torch.empty((n, 784), dtype=torch.uint8, device=device)
            dy = torch.empty(n, dtype=torch.uint8, device=device)
            dx.view(-1).copy_(hx, non_blocking=True)
            dy.copy_(hy, non_blocking=True)
        s.synchronize()
        return dx, dy
    x, y = f.read_rows("images", 0, n), f.read_rows("labels", 0, n)
    return upload_arrays(x, y, device)
