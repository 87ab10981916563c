"""MNIST sources: idx-ubyte files, PnetCDF-format netCDF files, or the synthetic generator.

Reference sources:
  * torchvision ``datasets.MNIST('./mnist_data', download=True, transform=...)``
    (ddp_tutorial_cpu.py:17-35) — here :class:`MNISTIdx`; with no network, a missing dataset is
    *synthesised* into the same file layout instead of downloaded (and the run says so);
  * ``MNISTNetCDF`` (mnist_pnetcdf_cpu.py:20-50, mnist_pnetcdf_cpu_mp.py:18-49) — same class name,
    same ``(root_dir, is_train, transforms, comm)`` signature, same two log lines, per-sample
    ``__getitem__`` returning ``(image, uint8 label)``, backed by the native CDF-5 reader.

The engines do not iterate these per sample: :func:`load_arrays` returns whole uint8 arrays
(bulk ``pread``), which ``device_loader`` stages into HBM once.
"""
from __future__ import annotations

import os
from typing import Callable, Optional, Tuple

import numpy as np
import torch
from torch.utils.data import Dataset

from . import cdf5, idx
from .synthetic import make_mnist

MEAN, STD = 0.1307, 0.3081
IDX_NAMES = {
    ("train", "images"): "train-images-idx3-ubyte", ("train", "labels"): "train-labels-idx1-ubyte",
    ("test", "images"): "t10k-images-idx3-ubyte", ("test", "labels"): "t10k-labels-idx1-ubyte",
}
NC_NAMES = {"train": "mnist_train_images.nc", "test": "mnist_test_images.nc"}


def mnist_transform(img_u8) -> torch.Tensor:
    """``transforms.Compose([ToTensor(), Normalize((0.1307,), (0.3081,))])`` on a 28x28 uint8 image."""
    x = torch.as_tensor(np.asarray(img_u8), dtype=torch.uint8).float().div_(255.0)
    return x.sub_(MEAN).div_(STD).view(1, 28, 28)


def normalize_batch(x_u8: torch.Tensor) -> torch.Tensor:
    return (x_u8.float() / 255.0 - MEAN) / STD


# ----------------------------------------------------------------------------- discovery
def find_idx(root: str) -> Optional[dict]:
    """Locate the four idx files under ``root`` (torchvision, Kaggle/notebook, or flat layout)."""
    out = {}
    for key, name in IDX_NAMES.items():
        cands = [os.path.join(root, "MNIST", "raw", name), os.path.join(root, name, name), os.path.join(root, name)]
        hit = next((c for c in cands if os.path.isfile(c)), None)
        if hit is None:
            return None
        out[key] = hit
    return out


def find_netcdf(root: str) -> Optional[dict]:
    out = {s: os.path.join(root, n) for s, n in NC_NAMES.items()}
    return out if all(os.path.isfile(p) for p in out.values()) else None


def synthesize_idx(root: str, seed: int = 0, verbose: bool = True) -> dict:
    (xtr, ytr), (xte, yte) = make_mnist(seed)
    paths = idx.write_mnist_idx(root, (xtr, ytr), (xte, yte), layout="torchvision")
    if verbose:
        print(f"=> no network / no local MNIST: wrote synthetic MNIST-format idx files under {root}/MNIST/raw")
    return paths


def synthesize_netcdf(root: str, seed: int = 0, verbose: bool = True) -> dict:
    (xtr, ytr), (xte, yte) = make_mnist(seed)
    os.makedirs(root or ".", exist_ok=True)
    out = {}
    for split, (x, y) in (("train", (xtr, ytr)), ("test", (xte, yte))):
        p = os.path.join(root, NC_NAMES[split])
        cdf5.write_mnist_nc(p, x, y)
        out[split] = p
    if verbose:
        print(f"=> no MNIST netCDF files found: wrote synthetic CDF-5 files {out['train']}, {out['test']}")
    return out


# ----------------------------------------------------------------------------- bulk arrays
def load_arrays(fmt: str = "auto", root: Optional[str] = None, limit: Optional[int] = None,
                seed: int = 0, create: bool = True, verbose: bool = True
                ) -> Tuple[np.ndarray, np.ndarray, np.ndarray, np.ndarray, str]:
    """(x_train [N,28,28] u8, y_train [N] u8, x_test, y_test, source description)."""
    if fmt == "synthetic":
        (xtr, ytr), (xte, yte) = make_mnist(seed)
        src = "synthetic"
    elif fmt in ("idx", "auto"):
        r = root or "./mnist_data"
        paths = find_idx(r)
        if paths is None and fmt == "auto" and find_netcdf(root or ".") is not None:
            return load_arrays("netcdf", root or ".", limit, seed, create, verbose)
        if paths is None:
            if not create:
                raise FileNotFoundError(f"no MNIST idx files under {r}")
            paths = synthesize_idx(r, seed, verbose)
        xtr = idx.read_idx(paths[("train", "images")], limit)
        ytr = idx.read_idx(paths[("train", "labels")], limit)
        xte = idx.read_idx(paths[("test", "images")])
        yte = idx.read_idx(paths[("test", "labels")])
        src = f"idx-ubyte ({os.path.dirname(paths[('train', 'images')])})"
    elif fmt == "netcdf":
        r = root or "."
        paths = find_netcdf(r)
        if paths is None:
            if not create:
                raise FileNotFoundError(f"no mnist_*_images.nc under {r}")
            paths = synthesize_netcdf(r, seed, verbose)
        xtr, ytr = cdf5.read_mnist_nc(paths["train"], limit)
        xte, yte = cdf5.read_mnist_nc(paths["test"])
        src = f"netCDF CDF-5 ({paths['train']})"
    else:
        raise ValueError(f"unknown data format {fmt!r}")
    if limit is not None and fmt == "synthetic":
        xtr, ytr = xtr[:limit], ytr[:limit]
    return (np.ascontiguousarray(xtr).reshape(-1, 28, 28), np.ascontiguousarray(ytr).reshape(-1),
            np.ascontiguousarray(xte).reshape(-1, 28, 28), np.ascontiguousarray(yte).reshape(-1), src)


# ----------------------------------------------------------------------------- Dataset classes
class MNISTIdx(Dataset):
    """torchvision.datasets.MNIST-compatible dataset over idx files (root layout as torchvision)."""

    def __init__(self, root: str = "./mnist_data", train: bool = True, transform: Optional[Callable] = None,
                 download: bool = True, limit: Optional[int] = None):
        paths = find_idx(root)
        if paths is None:
            if not download:
                raise FileNotFoundError(f"MNIST idx files not found under {root}")
            paths = synthesize_idx(root)
        split = "train" if train else "test"
        self.data = idx.read_idx(paths[(split, "images")], limit)
        self.targets = idx.read_idx(paths[(split, "labels")], limit).astype(np.int64)
        self.transform = transform

    def __len__(self) -> int:
        return len(self.targets)

    def __getitem__(self, i):
        img = self.data[i]
        return (self.transform(img) if self.transform else img), int(self.targets[i])


class MNISTNetCDF(Dataset):
    """Reference-compatible netCDF dataset (mnist_pnetcdf_cpu_mp.py:18-49) without MPI.

    ``comm`` is accepted for signature parity; reads are independent per-sample ``pread``s
    (the reference's ``begin_indep()`` + ``get_var`` mode).  Labels come back as 0-d uint8 arrays
    exactly like the reference's ``buff = np.empty((), np.uint8)`` (survey Q11).
    """

    def __init__(self, root_dir: str, is_train: bool = True, transforms: Optional[Callable] = None, comm=None):
        self.transforms = transforms
        print("=> Reading NetCDF File...")
        nc_path = os.path.join(root_dir, "mnist_{}_images.nc".format("train" if is_train else "test"))
        self.nc = cdf5.open_nc(nc_path)
        self.comm = comm
        print("=> Dataset created, image nc file is : {}".format(nc_path))

    def __len__(self) -> int:
        return int(self.nc.shape("images")[0])

    def __getitem__(self, index):
        image = np.array(self.nc.read_row("images", int(index))[0])
        buff = np.empty((), np.uint8)
        buff[()] = self.nc.read_row("labels", int(index))[0]
        if self.transforms:
            image = self.transforms(image)
        return image, buff
