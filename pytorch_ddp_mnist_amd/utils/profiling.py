"""Tracing: roctx ranges around training phases + host-side phase timers (survey §5.1).

roctx ranges appear in ``rocprofv3 --marker-trace`` timelines; they are no-ops unless enabled
(``--profile`` or ``MNIST_AMD_ROCTX=1``) so the hot loop pays nothing by default.  The library is
loaded with ctypes from the already-mapped ``libroctx64.so.4`` (torch ships it) or /opt/rocm.
"""
from __future__ import annotations

import contextlib
import ctypes
import os
import time
from collections import defaultdict
from typing import Dict, List

_lib = None
_enabled = os.environ.get("MNIST_AMD_ROCTX", "0") == "1"


def enable(on: bool = True) -> None:
    global _enabled
    _enabled = on


def _roctx():
    global _lib
    if _lib is None:
        for name in ("libroctx64.so.4", "libroctx64.so", "/opt/rocm/lib/libroctx64.so.4"):
            try:
                _lib = ctypes.CDLL(name)
                _lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                break
            except OSError:
                continue
        else:
            _lib = False
    return _lib


@contextlib.contextmanager
def range_(name: str):
    lib = _roctx() if _enabled else None
    if lib:
        lib.roctxRangePushA(name.encode())
    try:
        yield
    finally:
        if lib:
            lib.roctxRangePop()


class PhaseTimer:
    """Wall-clock seconds per named phase (``--profile`` prints them per epoch).  ``sync`` (e.g. the
    trainer's stream synchronize) runs before a phase's clock stops, so device work is included."""

    def __init__(self, sync=None):
        self.t: Dict[str, List[float]] = defaultdict(list)
        self.sync = sync

    @contextlib.contextmanager
    def __call__(self, name: str):
        t0 = time.perf_counter()
        with range_(name):
            yield
            if self.sync is not None:
                self.sync()
        self.t[name].append(time.perf_counter() - t0)

    def summary(self) -> Dict[str, float]:
        return {k: sum(v) for k, v in self.t.items()}
