"""Deterministic synthetic MNIST.

No network exists on either side of this project (and torchvision is not installed), so real
MNIST is only used when idx files are already on disk (``datasets.find_mnist``).  Otherwise
this generator provides data of the exact MNIST shape/dtype — uint8 [N,28,28] images and uint8
labels — that is *learnable*: each class has a fixed stroke template (seeded), every sample is
its class template with a random sub-pixel shift, stroke-thickness jitter and pixel noise.
Top-1 accuracy on it is therefore meaningful (a linear model reaches >90 %, the reference MLP
>97 % within an epoch), unlike uniform noise.
"""
from __future__ import annotations

from typing import Tuple

import numpy as np

TRAIN_N, TEST_N = 60000, 10000


def _templates(seed: int) -> np.ndarray:
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:28, 0:28].astype(np.float32)
    out = np.zeros((10, 28, 28), np.float32)
    for c in range(10):
        img = np.zeros((28, 28), np.float32)
        nstroke = 2 + c % 3
        for _ in range(nstroke):
            # a random quadratic Bezier stroke inside the central 20x20 box
            p = rng.uniform(5, 23, size=(3, 2)).astype(np.float32)
            for t in np.linspace(0, 1, 24, dtype=np.float32):
                q = (1 - t) ** 2 * p[0] + 2 * (1 - t) * t * p[1] + t ** 2 * p[2]
                img += np.exp(-((yy - q[0]) ** 2 + (xx - q[1]) ** 2) / 2.2)
        out[c] = img / img.max()
    return out


def make_split(n: int, seed: int, template_seed: int = 20250114) -> Tuple[np.ndarray, np.ndarray]:
    """(images uint8 [n,28,28], labels uint8 [n])."""
    tpl = _templates(template_seed)
    rng = np.random.default_rng(seed)
    labels = rng.integers(0, 10, size=n).astype(np.uint8)
    shifts = rng.integers(-2, 3, size=(n, 2))
    gain = rng.uniform(0.75, 1.0, size=n).astype(np.float32)
    images = np.empty((n, 28, 28), np.uint8)
    chunk = 8192
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        base = tpl[labels[s:e]]
        shifted = np.empty_like(base)
        for i in range(e - s):
            shifted[i] = np.roll(base[i], shift=(int(shifts[s + i, 0]), int(shifts[s + i, 1])), axis=(0, 1))
        noise = rng.normal(0.0, 0.08, size=base.shape).astype(np.float32)
        x = np.clip(shifted * gain[s:e, None, None] + noise, 0.0, 1.0)
        images[s:e] = (x * 255.0 + 0.5).astype(np.uint8)
    return images, labels


def make_mnist(seed: int = 0, train_n: int = TRAIN_N, test_n: int = TEST_N):
    """((x_train, y_train), (x_test, y_test)) in the MNIST layout, like the notebook's load_data()."""
    return make_split(train_n, seed * 2 + 1), make_split(test_n, seed * 2 + 2)
