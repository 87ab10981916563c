"""Loader for the native extensions.

``_C`` (HIP) is REQUIRED on a GPU: there is no silent eager-PyTorch fallback for the training
kernels.  If the in-tree ``.so`` is missing or fails to load while a GPU is visible, importing
it raises with the build command.  ``_io`` (CPU C++ IO) is optional; the pure-Python readers in
``data/`` are used when it is absent.
"""
from __future__ import annotations

import importlib
import os
from types import ModuleType
from typing import Optional

import torch  # noqa: F401  (HIP runtime / RCCL must be mapped by torch first)

_C: Optional[ModuleType] = None
_IO: Optional[ModuleType] = None
BUILD_HINT = "build it with:  python -m pytorch_ddp_mnist_amd.ops.build   (or __graft_entry__.build())"


class NativeExtensionError(ImportError):
    pass


def load_c() -> ModuleType:
    """Import ``pytorch_ddp_mnist_amd._C``; build it first if the sources are newer/missing and
    MNIST_AMD_AUTOBUILD=1."""
    global _C
    if _C is not None:
        return _C
    alt = os.environ.get("MNIST_AMD_C_PATH")
    if alt:
        # same-box A/B of another build of the extension (scripts/build_ab.sh): the file's module init is
        # PyInit__C, so it is loaded under the package module name from the given path
        from importlib import util as _iu
        spec = _iu.spec_from_file_location("pytorch_ddp_mnist_amd._C", alt)
        if spec is None or spec.loader is None:
            raise NativeExtensionError(f"MNIST_AMD_C_PATH={alt}: not a loadable extension")
        mod = _iu.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _C = mod
        return _C
    try:
        _C = importlib.import_module("pytorch_ddp_mnist_amd._C")
    except ImportError as e:
        if os.environ.get("MNIST_AMD_AUTOBUILD", "0") == "1":
            from .build import build_c
            build_c()
            _C = importlib.import_module("pytorch_ddp_mnist_amd._C")
        else:
            raise NativeExtensionError(f"native HIP extension not loadable ({e}); {BUILD_HINT}") from e
    return _C


def load_io() -> Optional[ModuleType]:
    global _IO
    if _IO is not None:
        return _IO
    try:
        _IO = importlib.import_module("pytorch_ddp_mnist_amd._io")
    except ImportError:
        _IO = None
    return _IO


def require_gpu() -> ModuleType:
    """The native module, and a check that the visible device is the gfx950 target."""
    C = load_c()
    if not torch.cuda.is_available():
        raise RuntimeError("no ROCm GPU visible (torch.cuda.is_available() is False)")
    arch = torch.cuda.get_device_properties(torch.cuda.current_device()).gcnArchName
    if not arch.startswith("gfx950") and os.environ.get("MNIST_AMD_ALLOW_ARCH", "0") != "1":
        raise RuntimeError(f"kernels are built for gfx950 only, device is {arch}")
    return C
