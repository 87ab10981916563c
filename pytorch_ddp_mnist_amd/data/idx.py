"""idx-ubyte reader/writer (MNIST's native format).

Reference: the notebook's ``MnistDataloader.read_images_labels`` (mnist_to_netcdf.ipynb cell 2,
lines 24-45: ``>II`` magic 2049 for labels, ``>IIII`` magic 2051 for images) and torchvision's
decoder used by every training script.  Fast path: the native ``_io.idx_read`` (parallel
``pread``); fallback: numpy.
"""
from __future__ import annotations

import os
import struct
from typing import Optional

import numpy as np

from ..ops.native import load_io

LABEL_MAGIC, IMAGE_MAGIC = 2049, 2051


def read_idx(path: str, limit: Optional[int] = None, native: bool = True) -> np.ndarray:
    io = load_io() if native else None
    if io is not None:
        return io.idx_read(path, -1 if limit is None else int(limit))
    with open(path, "rb") as f:
        head = f.read(4)
        if len(head) < 4 or head[0] != 0 or head[1] != 0:
            raise ValueError(f"{path}: bad idx magic")
        if head[2] != 0x08:
            raise ValueError(f"{path}: only unsigned-byte idx files are supported")
        nd = head[3]
        dims = list(struct.unpack(">" + "I" * nd, f.read(4 * nd)))
        if limit is not None:
            dims[0] = min(dims[0], int(limit))
        count = int(np.prod(dims))
        data = np.frombuffer(f.read(count), dtype=np.uint8)
        if data.size != count:
            raise ValueError(f"{path}: truncated")
        return data.reshape(dims).copy()


def write_idx(path: str, array: np.ndarray, native: bool = True) -> None:
    a = np.ascontiguousarray(array, dtype=np.uint8)
    io = load_io() if native else None
    if io is not None:
        io.idx_write(path, a)
        return
    with open(path, "wb") as f:
        f.write(bytes([0, 0, 0x08, a.ndim]))
        f.write(struct.pack(">" + "I" * a.ndim, *a.shape))
        f.write(a.tobytes())


def read_images_labels(images_path: str, labels_path: str, limit: Optional[int] = None):
    """Same contract as the notebook's read_images_labels (magic-checked)."""
    with open(labels_path, "rb") as f:
        magic, _ = struct.unpack(">II", f.read(8))
        if magic != LABEL_MAGIC:
            raise ValueError(f"Magic number mismatch, expected {LABEL_MAGIC}, got {magic}")
    with open(images_path, "rb") as f:
        magic, _, _, _ = struct.unpack(">IIII", f.read(16))
        if magic != IMAGE_MAGIC:
            raise ValueError(f"Magic number mismatch, expected {IMAGE_MAGIC}, got {magic}")
    return read_idx(images_path, limit), read_idx(labels_path, limit)


def write_mnist_idx(root: str, train, test, layout: str = "torchvision") -> dict:
    """Write (x, y) splits as the four MNIST idx files.  layout: 'torchvision'
    (<root>/MNIST/raw/<name>) or 'kaggle' (<root>/<name>/<name>, the notebook's layout)."""
    names = {("train", "images"): "train-images-idx3-ubyte", ("train", "labels"): "train-labels-idx1-ubyte",
             ("test", "images"): "t10k-images-idx3-ubyte", ("test", "labels"): "t10k-labels-idx1-ubyte"}
    out = {}
    for split, (x, y) in (("train", train), ("test", test)):
        for kind, arr in (("images", x), ("labels", y)):
            name = names[(split, kind)]
            if layout == "torchvision":
                d = os.path.join(root, "MNIST", "raw")
                p = os.path.join(d, name)
            else:
                d = os.path.join(root, name)
                p = os.path.join(d, name)
            os.makedirs(d, exist_ok=True)
            write_idx(p, arr)
            out[(split, kind)] = p
    return out
