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


# ------------------------------------------------------------------------------------------------------------
# Link-aware bucket groups: WHICH gradients leave together, chosen from the measured RCCL latency
# curve of the real communicator and the measured backward cost of each gradient-producing unit.
#
# A plan is a partition of the model's units (models.UNITS, backward-ready order) into contiguous GROUPS; group g's
# gradients are produced by one weight-gradient launch (+ reduce) and all-reduced as soon as they are ready, on the
# comm stream, in group order (csrc/runtime/trainer.cpp launch_lenet_split_tail / launch_mlp_comm_tail).  The
# default SPLIT plan is two groups (LeNet: FC head | conv; MLP: layers 3+2 | layer 1).  On xGMI every collective
# of these sizes (1 KB - 400 KB) is latency-bound -- a ring's per-hop synchronisation, not the ~153 GB/s of a link,
# sets its time -- so a group is worth cutting off only when its all-reduce can start early enough to hide under
# the remaining backward work AND the extra launches and collective latencies it adds stay hidden as well.  The
# model below prices exactly that; the start-up calibration then times the best modelled plans for real.
# ------------------------------------------------------------------------------------------------------------
class LatencyCurve:
    """All-reduce latency (us) vs message bytes, piecewise linear through measured points (rank-max medians of
    standalone collectives on the job's communicator); flat below the smallest point, extended with the last
    segment's slope above the largest."""

    def __init__(self, points: Sequence[Tuple[int, float]]):
        pts = sorted((int(b), float(t)) for b, t in points)
        if not pts:
            raise ValueError("LatencyCurve: no points")
        self.pts = pts

    def __call__(self, nbytes: float) -> float:
        p = self.pts
        if nbytes <= p[0][0] or len(p) == 1:
            return p[0][1]
        for (b0, t0), (b1, t1) in zip(p, p[1:]):
            if nbytes <= b1:
                return t0 + (t1 - t0) * (nbytes - b0) / max(1, b1 - b0)
        (b0, t0), (b1, t1) = p[-2], p[-1]
        return t1 + max(0.0, (t1 - t0) / max(1, b1 - b0)) * (nbytes - b1)

    def as_dict(self) -> Dict[str, float]:
        return {str(b): round(t, 2) for b, t in self.pts}


# message sizes the start-up sweep times (4 KB .. 1 MB: every bucket either model can form lies inside)
LATENCY_SWEEP_BYTES = (4096, 16384, 32768, 65536, 131072, 262144, 524288, 1048576)


def partitions(n: int) -> List[List[List[int]]]:
    """Every split of units 0..n-1 (in order) into non-empty contiguous groups (2**(n-1) of them)."""
    out = []
    for mask in range(1 << max(0, n - 1)):
        groups, cur = [], [0]
        for i in range(1, n):
            if mask >> (i - 1) & 1:
                groups.append(cur)
                cur = [i]
            else:
                cur.append(i)
        groups.append(cur)
        out.append(groups)
    return out


def fc_unit_count(model: str) -> int:
    """Units produced by FC weight-gradient launches (all of the MLP's; LeNet's without the conv unit)."""
    from ..models import UNITS
    return sum(1 for name, _, _ in UNITS[model] if name != "conv")


def groups_to_buckets(model: str, groups: Sequence[Sequence[int]], cap_bytes: Optional[int] = None,
                      elem_bytes: int = 4) -> List[Range]:
    """Bucket ranges (p0, p1, group) of a partition of the FC units (indices into models.UNITS); LeNet's conv unit
    is appended as the last group.  ``cap_bytes`` splits a group into several collectives (cut from the end, as
    :func:`plan_buckets`), all issued when the group is ready."""
    from ..models import UNITS
    units = UNITS[model]
    nfc = fc_unit_count(model)
    flat = [i for g in groups for i in g]
    if flat != list(range(nfc)):
        raise ValueError(f"groups_to_buckets: {groups} is not an ordered partition of the {nfc} FC units")
    spans = [(min(units[i][1] for i in g), max(units[i][2] for i in g)) for g in groups]
    if nfc < len(units):
        spans.append((units[-1][1], units[-1][2]))
    out: List[Range] = []
    for gi, (p0, p1) in enumerate(spans):
        for a, b, _ in plan_buckets([(p0, p1)], cap_bytes, elem_bytes):
            out.append((a, b, gi))
    return out


def default_groups(model: str) -> List[List[int]]:
    """The two-group default (LeNet: the whole FC head, then conv; MLP: layers 3+2, then layer 1)."""
    n = fc_unit_count(model)
    return [list(range(n))] if model == "lenet5" else [list(range(n - 1)), [n - 1]]


def model_split_tail_us(model: str, groups: Sequence[Sequence[int]], lat: LatencyCurve, unit_us: Sequence[float],
                        fc_all_us: float, main_us: float = 0.0, update_us: float = 2.0, elem_bytes: int = 4) -> float:
    """Modelled time from the start of the weight gradients to the end of the step's last update under SPLIT with
    these groups.  ``unit_us``: each FC unit's weight gradient + reduce as its own launches (ready order);
    ``fc_all_us``: all FC units as ONE launch + reduce (merging k units into a group saves (k-1) x the measured
    per-launch saving); ``main_us`` (LeNet): conv_bwd + its reduce, on the main stream beside the FC groups.
    Groups run back to back (LeNet: aux stream; MLP: main stream); the comm stream sends group g when it is ready
    and its previous collective is done (one all-reduce + one update each); LeNet's conv group goes last."""
    from ..models import UNITS
    units = UNITS[model]
    nfc = fc_unit_count(model)
    save = max(0.0, (sum(unit_us[:nfc]) - fc_all_us) / (nfc - 1)) if nfc > 1 else 0.0
    t = comm = 0.0
    for g in groups:
        t += sum(unit_us[i] for i in g) - save * (len(g) - 1)
        nbytes = elem_bytes * sum(units[i][2] - units[i][1] for i in g)
        comm = max(comm, t) + lat(nbytes) + update_us
    if nfc < len(units):  # LeNet: the conv group after conv_bwd + reduce on the main stream
        nbytes = elem_bytes * (units[-1][2] - units[-1][1])
        comm = max(comm, main_us) + lat(nbytes) + update_us
    return comm


def model_join_tail_us(model: str, lat: LatencyCurve, fc_all_us: float, main_us: float = 0.0,
                       update_us: float = 2.0, elem_bytes: int = 4) -> float:
    """The JOIN plan on the same clock: both branches reduced, then ONE all-reduce of every gradient and one update."""
    from ..models import NPARAM
    return max(fc_all_us, main_us) + lat(elem_bytes * NPARAM[model]) + update_us


def choose_bucket_groups(model: str, lat: LatencyCurve, unit_us: Sequence[float], fc_all_us: float,
                         main_us: float = 0.0, update_us: float = 2.0) -> List[Tuple[List[List[int]], float]]:
    """Every partition of the FC units ranked by :func:`model_split_tail_us` (fastest first; ties: fewer groups)."""
    ranked = [(g, model_split_tail_us(model, g, lat, unit_us, fc_all_us, main_us, update_us))
              for g in partitions(fc_unit_count(model))]
    ranked.sort(key=lambda x: (round(x[1], 3), len(x[0])))
    return ranked


def bucket_plan_candidates(model: str, ranked: Sequence[Tuple[List[List[int]], float]], base: Optional[dict] = None
                           ) -> Dict[str, dict]:
    """SPLIT candidates from a ranking: the modelled best plan (``split_bm``) unless it is the default grouping, and
    the best plan with at least two FC groups (``split_mb``: LeNet >= 3 buckets, MLP >= 3), so the calibration
    always measures one multi-bucket plan against the default.  Each candidate carries its bucket ranges."""
    base = dict(base or {"plan": "split", "bwd_blocks": 0})
    out: Dict[str, dict] = {}
    dflt = default_groups(model)
    if ranked and ranked[0][0] != dflt:
        out["split_bm"] = dict(base, buckets=groups_to_buckets(model, ranked[0][0]), groups=ranked[0][0])
    multi = [g for g, _ in ranked if len(g) >= (2 if model == "lenet5" else 3)]
    if multi and multi[0] != dflt and ("split_bm" not in out or out["split_bm"]["groups"] != multi[0]):
        out["split_mb"] = dict(base, buckets=groups_to_buckets(model, multi[0]), groups=multi[0])
    return out


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
