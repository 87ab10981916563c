"""Test-only fault injection and numeric guards (survey §5.2 / §5.3).

``MNIST_AMD_FAIL_AT_STEP=k`` makes the training loop raise at its k-th optimizer step (0-based,
counted across epochs) -- on every rank, or only on ``MNIST_AMD_FAIL_RANK=r``.  Used to check
that one failing rank takes the whole job down promptly (the launcher kills the survivors that
would otherwise block in the next collective) with a non-zero exit code.
"""
from __future__ import annotations

import math
import os


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, rank: int = 0, env=None):
        env = os.environ if env is None else env
        at = env.get("MNIST_AMD_FAIL_AT_STEP")
        only = env.get("MNIST_AMD_FAIL_RANK")
        self.at = int(at) if at not in (None, "") else None
        self.active = self.at is not None and (only in (None, "") or int(only) == rank)
        self.rank = rank
        self.step = 0

    def tick(self) -> None:
        """Call once per optimizer step."""
        if self.active and self.step == self.at:
            raise InjectedFault(f"injected failure at step {self.step} on rank {self.rank} (MNIST_AMD_FAIL_AT_STEP)")
        self.step += 1


def check_finite(what: str, *values: float) -> None:
    """NaN/Inf guard on the device-accumulated loss (read once per epoch, so it costs nothing per step)."""
    for v in values:
        if not math.isfinite(v):
            raise FloatingPointError(f"{what} is not finite ({v}): training diverged")
