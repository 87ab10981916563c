"""Console output compatible with the reference, plus structured metrics.

* the per-epoch line ``Epoch={i}, train_loss={:.4f}, val_loss={:.4f}`` printed by every rank,
  with the reference's loss bookkeeping (sum over batches of ``mean_batch_loss / batch_size``,
  survey quirk Q7) — kept byte-compatible;
* the rank-0 banner of ``init_parallel`` (mnist_cpu_mp.py:278-299, ``"%-32s: %s"`` fields) with
  accurate labels (Q15);
* an additional rank-0 line with the true global mean loss, top-1 accuracy and images/sec, and
  an optional JSON-lines metrics file.
"""
from __future__ import annotations

import contextlib
import os
import json
import socket
import sys
import time
from typing import Optional


def epoch_line(i: int, train_loss: float, val_loss: float) -> str:
    return f"Epoch={i}, train_loss={train_loss:.4f}, val_loss={val_loss:.4f}"


def banner(rank: int, world: int, n_gpus: int, device, fmt: str, num_workers: int, n_epochs: int,
           parallel: bool, model: str, dtype: str, engine: str, out=sys.stdout) -> None:
    if rank != 0:
        return
    p = lambda k, v: print("%-32s: %s" % (k, v), file=out)  # noqa: E731
    print("------------------------------------------------------------------", file=out)
    print("\n======== MNIST %s training (%s) ========" % ("data-parallel" if parallel else "serial", engine), file=out)
    p("Host name", socket.gethostname())
    p("Number of processes", world)
    p("number of GPUs per node", n_gpus)
    if getattr(device, "type", "cpu") == "cuda":
        p("Rank 0 GPU device", device)
    else:
        print("Rank 0 is Using CPU device", file=out)
    p("Input file format", fmt)
    p("DataLoader num_workers", num_workers)
    p("Number of epochs", n_epochs)
    p("Model / compute dtype", f"{model} / {dtype}")
    print("------------------------------------------------------------------", file=out)


def reference_epoch_loss(full_sum: float, n_full: int, batch: int, last_sum: float, last_b: int) -> float:
    """sum_b mean_b / B_b  ==  full_sum / B^2 + last_sum / B_last^2 (Q7 formula)."""
    v = full_sum / float(batch * batch) if n_full else 0.0
    if last_b:
        v += last_sum / float(last_b * last_b)
    return v


class MetricsWriter:
    def __init__(self, path: Optional[str], rank: int = 0):
        self.f = open(path, "a") if (path and rank == 0) else None

    def write(self, **kw) -> None:
        if self.f:
            kw.setdefault("time", time.time())
            self.f.write(json.dumps(kw) + "\n")
            self.f.flush()

    def close(self) -> None:
        if self.f:
            self.f.close()


class ProgressBar:
    """Rank-0 per-batch progress (``--tqdm``): the reference's ``tqdm(loader)`` with
    ``set_description(f'training batch_loss={:.4f}')`` / ``validation …`` (ddp_tutorial_multi_gpu.py:85,98,
    104,114; ddp_tutorial_cpu.py:69,79,85,93).  The native engine accumulates the loss on the device,
    so the bar is fed every ``every`` batches with the mean loss of that window (one device sync
    per update instead of the reference's ``.item()`` per batch).  Uses tqdm when importable."""

    def __init__(self, total_batches: int, kind: str, every: int, out=sys.stderr):
        self.kind, self.every, self.total = kind, max(1, every), total_batches
        self.n = 0
        self.t0 = time.perf_counter()
        self.out = out
        try:
            from tqdm import tqdm
            self.bar = tqdm(total=total_batches, file=out, leave=False, dynamic_ncols=True)
        except ImportError:  # pragma: no cover - tqdm ships with the image
            self.bar = None
        self.last = None

    @classmethod
    def make(cls, cfg, rank: int, n_samples: int, kind: str) -> Optional["ProgressBar"]:
        if cfg.disable_tqdm or rank != 0:
            return None
        nb = -(-int(n_samples) // int(cfg.batch_size))
        every = cfg.progress_every or max(1, nb // 20)
        return cls(nb, kind, every)

    def __call__(self, batch_loss: float, n: int = 1) -> None:
        self.n += n
        self.last = float(batch_loss)
        desc = f"{self.kind} batch_loss={self.last:.4f}"
        if self.bar is not None:
            self.bar.set_description(desc)
            self.bar.update(n)
        else:
            rate = self.n / max(1e-9, time.perf_counter() - self.t0)
            print(f"\r{desc} {self.n}/{self.total} [{rate:.1f}it/s]", end="", file=self.out, flush=True)

    def close(self) -> None:
        if self.bar is not None:
            self.bar.close()
        else:
            print(file=self.out)


@contextlib.contextmanager
def native_stdout_to_stderr():
    """Route file-descriptor-level stdout to stderr for the duration (RCCL prints a version banner on
    stdout when it initialises, which would corrupt the one-JSON-line contract of bench.py and
    interleave with the epoch lines)."""
    sys.stdout.flush()
    saved = os.dup(1)
    try:
        os.dup2(2, 1)
        yield
    finally:
        try:
            sys.stdout.flush()
        finally:
            os.dup2(saved, 1)
            os.close(saved)
