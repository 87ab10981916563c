"""Torch-CPU engine: the reference training loop, kept as the plumbing path and test oracle.

It reproduces ``main()`` of ddp_tutorial_cpu.py:56-97 / mnist_cpu_mp.py:357-418 step for step —
``zero_grad`` -> forward -> CrossEntropy (NLL for LeNet's log-softmax head) -> ``backward`` ->
gradient all-reduce (``GlooReducer``, DDP semantics, only when world > 1) -> ``SGD.step`` — on
pre-normalised in-memory tensors (no per-sample PIL/ToTensor work; identical values).
"""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Optional

import numpy as np
import torch
import torch.nn.functional as F

from ..data.datasets import normalize_batch
from ..data.sampler import batch_slices
from ..models import build_model
from ..parallel.ddp import GlooReducer, model_phases, plan_buckets
from ..utils.fault import FaultInjector


@dataclass
class EpochResult:
    loss_sum: float = 0.0        # sum of per-sample losses
    correct: float = 0.0
    count: float = 0.0
    full_sum: float = 0.0        # loss sum over full batches (for the reference's epoch_loss)
    n_full: int = 0
    last_sum: float = 0.0
    last_b: int = 0
    seconds: float = 0.0
    steps: int = 0
    next_indices: object = None  # the prefetch callback's result (next epoch's sampler order), if any

    @property
    def mean_loss(self) -> float:
        return self.loss_sum / max(1.0, self.count)

    @property
    def accuracy(self) -> float:
        return self.correct / max(1.0, self.count)


class TorchCPUEngine:
    name = "torch-cpu"

    def __init__(self, model: str, batch: int, lr: float, momentum: float, dropout: float,
                 xtr: np.ndarray, ytr: np.ndarray, xte: np.ndarray, yte: np.ndarray, world: int = 1,
                 bucket_cap_kb: Optional[int] = None, init: Optional[torch.nn.Module] = None):
        self.model_name, self.batch = model, batch
        # share the host's cores between co-located ranks instead of oversubscribing them
        local = int(os.environ.get("LOCAL_WORLD_SIZE", world if world > 1 else 1))
        torch.set_num_threads(max(1, (os.cpu_count() or 1) // max(1, local)))
        self.module = init if init is not None else build_model(model)
        if model == "mlp":
            self.module[2].p = dropout
        shape = self.shape = (-1, 784) if model == "mlp" else (-1, 1, 28, 28)
        self.x = normalize_batch(torch.from_numpy(np.ascontiguousarray(xtr))).reshape(shape)
        self.y = torch.from_numpy(ytr.astype(np.int64))
        self.xt = normalize_batch(torch.from_numpy(np.ascontiguousarray(xte))).reshape(shape)
        self.yt = torch.from_numpy(yte.astype(np.int64))
        self.opt = torch.optim.SGD(self.module.parameters(), lr=lr, momentum=momentum)
        cap = None if bucket_cap_kb is None else bucket_cap_kb * 1024
        self.reducer = GlooReducer(self.module, world, plan_buckets(model_phases(model), cap))
        self.crit = F.nll_loss if model == "lenet5" else F.cross_entropy
        self.fault = FaultInjector(int(os.environ.get("RANK", "0")))
        self.global_step = 0

    def load_train_arrays(self, x: np.ndarray, y: np.ndarray) -> None:
        """Per-sample I/O mode: this epoch's rows (sampler order) become the resident training data."""
        self.x = normalize_batch(torch.from_numpy(np.ascontiguousarray(x))).reshape(self.shape)
        self.y = torch.from_numpy(y.astype(np.int64))

    def write_train_rows(self, x: np.ndarray, y: np.ndarray, row0: int) -> None:
        """Interleaved I/O: one batch's rows become resident rows [row0, row0+b)."""
        b = len(y)
        self.x[row0:row0 + b] = normalize_batch(torch.from_numpy(np.ascontiguousarray(x))).reshape(self.shape)
        self.y[row0:row0 + b] = torch.from_numpy(y.astype(np.int64))

    def load_test_arrays(self, x: np.ndarray, y: np.ndarray) -> None:
        self.xt = normalize_batch(torch.from_numpy(np.ascontiguousarray(x))).reshape(self.shape)
        self.yt = torch.from_numpy(y.astype(np.int64))

    def train_epoch(self, indices: torch.Tensor, progress=None, prefetch=None, batch_loader=None) -> EpochResult:
        r = EpochResult()
        self.module.train()
        t0 = time.perf_counter()
        slices = batch_slices(indices.numel(), self.batch)
        for s, b in slices:
            if batch_loader is not None:  # interleaved I/O: this batch's rows are read now
                batch_loader(s, b)
            idx = indices[s:s + b]
            x, y = self.x[idx], self.y[idx]
            self.fault.tick()  # before the step, as NativeEngine._step: FAIL_AT_STEP=k -> k completed steps
            self.opt.zero_grad()
            out = self.module(x)
            loss = self.crit(out, y)
            loss.backward()
            self.reducer.sync_grads()
            self.opt.step()
            self.global_step += 1
            lv = float(loss.item()) * b
            r.loss_sum += lv
            r.correct += float((out.argmax(1) == y).sum())
            r.count += b
            if b == self.batch:
                r.full_sum += lv
                r.n_full += 1
            else:
                r.last_sum, r.last_b = lv, b
            r.steps += 1
            if progress is not None:
                progress(lv / b, 1)
        r.seconds = time.perf_counter() - t0
        if prefetch is not None:
            r.next_indices = prefetch()
        return r

    @torch.no_grad()
    def evaluate(self, indices: torch.Tensor, progress=None) -> EpochResult:
        r = EpochResult()
        self.module.eval()
        for s, b in batch_slices(indices.numel(), self.batch):
            idx = indices[s:s + b]
            out = self.module(self.xt[idx])
            y = self.yt[idx]
            lv = float(self.crit(out, y, reduction="sum"))
            if progress is not None:
                progress(lv / b, 1)
            r.loss_sum += lv
            r.correct += float((out.argmax(1) == y).sum())
            r.count += b
            if b == self.batch:
                r.full_sum += lv
                r.n_full += 1
            else:
                r.last_sum, r.last_b = lv, b
        return r

    def state_dict(self):
        return {k: v.detach().clone() for k, v in self.module.state_dict().items()}

    # resume: flat params (state_dict order) + flat SGD momentum buffers (zeros before the first step)
    def get_state(self):
        params = torch.cat([p.detach().reshape(-1) for p in self.module.parameters()])
        bufs = [self.opt.state.get(p, {}).get("momentum_buffer") for p in self.module.parameters()]
        mom = torch.cat([(b if b is not None else torch.zeros_like(p)).reshape(-1)
                         for b, p in zip(bufs, self.module.parameters())])
        return params, mom, self.global_step

    def set_state(self, params: torch.Tensor, mom, global_step: int = 0) -> None:
        self.global_step = int(global_step)
        off = 0
        with torch.no_grad():
            for p in self.module.parameters():
                n = p.numel()
                p.copy_(params[off:off + n].view_as(p))
                if mom is not None and self.opt.defaults.get("momentum", 0) != 0:
                    self.opt.state[p]["momentum_buffer"] = mom[off:off + n].view_as(p).clone()
                off += n

    def finish(self) -> None:
        pass
