"""Data-parallel gradient exchange: bucket planning + a gloo reducer for the CPU path.

Reference: ``DistributedDataParallel(model[, device_ids])`` (ddp_tutorial_multi_gpu.py:72,
mnist_cpu_mp.py:371) — parameter broadcast from rank 0 at construction, bucketed SUM
all-reduce of gradients during backward (first bucket <= 1 MiB, then 25 MiB caps, grads divided
by the world size), ``model.module`` unwrap.  For both reference models every gradient fits the
first bucket, so the reference does ONE 473,088-byte (MLP) all-reduce per step with no overlap
(survey §2.7, CS5).

MI355X design (GPU path, csrc/runtime/trainer.cpp): gradients are written by the kernels into
ONE flat fp32 slab; a bucket is a contiguous range of it.  :func:`plan_buckets` decides the ranges
(one per backward phase by default: LeNet-5 FC head 236.5 KB | conv 10 KB, MLP layers 2+3 71 KB |
layer 1 402 KB; ``bucket_cap_kb`` forces further splits).  For messages this small the all-reduce is latency-bound
on xGMI (7 point-to-point links, ~153 GB/s each: a 247 KB ring step is ~2 us of wire time), so
WHEN the buckets go out matters more than how many there are.  Two step plans exist (trainer.h):

  * ``join``  -- the FC and conv backward branches join, then ONE all-reduce of the coalesced
    slab (one ring latency per step, fully exposed);
  * ``split`` -- phase 0's buckets go out on the comm stream as soon as its grads are reduced
    (LeNet: the FC buckets beside conv_bwd, whose grid can be capped to leave whole CUs free for
    RCCL's kernels; MLP: layers 2+3 beside the layer-1 weight gradient) and phase 0's parameters are
    updated right behind them on the same stream; phase 1's buckets and update follow its reduce
    (LeNet: only the 10 KB conv bucket and its 2,572-parameter update are exposed).

Which one is faster depends on the xGMI latency at the actual world size and on whether RCCL's
kernels find CU room beside conv_bwd, so it is not hard-coded: at start-up every candidate of
:func:`default_plan_candidates` is timed on the real communicator (NativeTrainer.autotune_plan)
and :func:`choose_plan` keeps the fastest, preferring ``join`` unless another plan wins by a
margin (rank-max timings, so every rank decides the same).

:class:`GlooReducer` is the same contract for the CPU path (plumbing / oracle): it broadcasts
parameters at construction and all-reduces the flattened gradients in the same bucket plan.
"""
from __future__ import annotations

from typing import Dict, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist

Range = Tuple[int, int, int]  # (p0, p1, phase)


def plan_buckets(phases: Sequence[Tuple[int, int]], cap_bytes: Optional[int] = None,
                 elem_bytes: int = 4) -> List[Range]:
    """Split each backward phase's contiguous parameter range into <= cap-sized buckets.

    ``phases`` lists (p0, p1) ranges in the order backward produces them; bucket k of phase i is
    launched when phase i's gradients are complete.
    """
    out: List[Range] = []
    for ph, (p0, p1) in enumerate(phases):
        if cap_bytes is None or cap_bytes <= 0:
            out.append((p0, p1, ph))
            continue
        step = max(1, cap_bytes // elem_bytes)
        # later parameters of a phase are produced first in backward: cut from the end
        e = p1
        while e > p0:
            s = max(p0, e - step)
            out.append((s, e, ph))
            e = s
    return out


def default_plan_candidates(default_grid: int, n_cu: int, reserve_cus=(16,)) -> Dict[str, dict]:
    """Multi-GPU candidates: name -> {plan, bwd_blocks (conv_bwd target workgroups; 0 = default one
    full round)}.  ``split_rN`` caps conv_bwd to the workgroups that fit on ``n_cu - N`` CUs at the
    default workgroups-per-CU, so N CUs stay free for RCCL's kernels while conv_bwd runs."""
    out: Dict[str, dict] = {"join": dict(plan="join", bwd_blocks=0), "split": dict(plan="split", bwd_blocks=0)}
    per_cu = max(1, round(default_grid / max(1, n_cu)))
    for r in reserve_cus:
        if 0 < r < n_cu and default_grid >= n_cu:
            out[f"split_r{r}"] = dict(plan="split", bwd_blocks=per_cu * (n_cu - r))
    return out


def mlp_plan_candidates() -> Dict[str, dict]:
    """MLP multi-GPU candidates: one coalesced all-reduce after the whole weight gradient, or layers 2+3
    sent beside the layer-1 weight gradient."""
    return {"join": dict(plan="join"), "split": dict(plan="split")}


def local_plan_candidates(fwd_head: bool = False) -> Dict[str, dict]:
    """Single-GPU LeNet schedules: the FC weight gradient + FC update on an aux stream beside
    conv_bwd (``concurrent``, the default) or after it (``serial``).  ``fwd_head`` (bf16, large
    batches: the fused forward + FC head kernel applies): also the same schedule with the two separate
    kernels (``separate``), so the calibration measures what the fusion is worth on this box."""
    c = {"concurrent": dict(concurrent=True), "serial": dict(concurrent=False)}
    if fwd_head:
        c["separate"] = dict(concurrent=True, fwd_head=False)
    return c


def choose_plan(timings_ms: Dict[str, float], prefer: str = "join", margin: float = 0.015) -> str:
    """Fastest candidate, but keep ``prefer`` unless the winner beats it by more than ``margin``
    (relative): the simpler schedule wins ties and timing noise."""
    if not timings_ms:
        raise ValueError("choose_plan: no timings")
    best = min(timings_ms, key=lambda k: (timings_ms[k], k != prefer))
    if prefer in timings_ms and timings_ms[best] > timings_ms[prefer] * (1.0 - margin):
        return prefer
    return best


def model_phases(model: str) -> List[Tuple[int, int]]:
    """The two backward phases of a model, in the order backward produces them: phase 0 = the late
    layers (LeNet-5 FC head ``7.*,9.*,11.*``; MLP ``3.*,5.*``), phase 1 = the early ones (LeNet-5 convs;
    MLP ``0.*``).  Reference gradient-ready order: survey §2.7."""
    from ..models import NPARAM, PHASE_SPLIT
    n, c = NPARAM[model], PHASE_SPLIT[model]
    return [(c, n), (0, c)]


def coalesce_buckets(buckets: Sequence[Range]) -> List[Range]:
    """Merge a bucket into the previous one when they are contiguous and belong to different backward
    phases (the JOIN plan's one all-reduce of the coalesced slab; csrc/runtime/trainer.cpp
    ``coalesced_buckets``).  Splits inside a phase come from an explicit cap and are kept."""
    out: List[List[int]] = []
    for p0, p1, ph in sorted(buckets, key=lambda b: b[0]):
        if out and out[-1][1] == p0 and out[-1][2] != ph:
            out[-1][1], out[-1][2] = p1, ph
        else:
            out.append([p0, p1, ph])
    return [tuple(b) for b in out]


class GlooReducer:
    """DDP semantics for the torch-CPU engine: broadcast at init, bucketed mean all-reduce.  With the
    default per-phase plan the two phases are coalesced into ONE all-reduce per step, as the reference's
    single 1 MiB-capped DDP bucket does (survey §2.7); a capped plan keeps its cap splits."""

    def __init__(self, module: torch.nn.Module, world: int, buckets: Optional[List[Range]] = None):
        self.module = module
        self.world = world
        self.params = [p for p in module.parameters()]
        self.numel = sum(p.numel() for p in self.params)
        self.buckets = coalesce_buckets(buckets) if buckets else [(0, self.numel, 0)]
        if world > 1 and dist.is_initialized():
            with torch.no_grad():
                flat = torch.cat([p.detach().reshape(-1) for p in self.params])
                dist.broadcast(flat, 0)
                self._unflatten(flat, grads=False)

    def _unflatten(self, flat: torch.Tensor, grads: bool) -> None:
        off = 0
        for p in self.params:
            n = p.numel()
            v = flat[off:off + n].view_as(p)
            if grads:
                if p.grad is None:
                    p.grad = v.clone()
                else:
                    p.grad.copy_(v)
            else:
                p.data.copy_(v)
            off += n

    def sync_grads(self) -> None:
        if self.world <= 1 or not dist.is_initialized():
            return
        flat = torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1) for p in self.params])
        works = [dist.all_reduce(flat[a:b], async_op=True) for a, b, _ in self.buckets]
        for wk in works:
            wk.wait()
        flat.div_(self.world)
        self._unflatten(flat, grads=True)
