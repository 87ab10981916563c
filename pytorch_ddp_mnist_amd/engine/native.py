"""Python façade of the native MI355X trainer (``csrc/runtime/trainer.cpp``).

Owns every device buffer of a training run (allocated once through torch's HBM caching
allocator, never re-allocated per step) and exposes epoch-level operations:

  * the train set lives in HBM as uint8 ``[N,784]`` + uint8 labels (47 MB for MNIST — the
    reference instead re-decodes PIL images in 4 DataLoader workers every epoch, survey N13/N14);
  * one int32 index vector per epoch (bit-equal to DistributedSampler) is uploaded with a single
    async copy; kernels address their batch through a device step counter, so the captured
    hipGraph of a step is replayed unchanged for every full batch;
  * loss / accuracy are accumulated on the device and read back once per epoch (the reference
    syncs with ``.item()`` every batch, survey K16);
  * with a communicator attached, every host wait goes through the RCCL watchdog
    (``RcclComm.wait_stream``: async-error polling + deadline -> ``ncclCommAbort`` ->
    :class:`CollectiveError`), the behaviour the reference inherits from ProcessGroupNCCL's
    timeout (ddp_tutorial_multi_gpu.py:133-134, survey N10/§5.3);
  * the multi-GPU step plan (JOIN / SPLIT, ``csrc/runtime/trainer.h``) is chosen at start-up by
    timing the candidates on the real communicator (:meth:`NativeTrainer.autotune_plan`).
"""
from __future__ import annotations

import atexit
import math
import os
import sys
import time
import weakref
from dataclasses import dataclass
from typing import Dict, Optional, Tuple

import torch

from ..models import MODEL_IDS, build_model, flatten_state, unflatten_state
from ..ops.native import require_gpu
from ..parallel.comm import comm_timeout  # noqa: F401  (re-exported: watchdog deadline)

PLANS = {"join": 0, "split": 1, "overlap": 2}
# standalone collective latencies (comm_profile) are timed as graphs of this many back-to-back calls: one call per
# graph measured the host's graph-launch rate (~15 us per replay) instead of the collective -- the one-shot kernel's
# in-kernel span is ~4.5 us at world 1 (profiles/r5_session1/prof1/oneshot_lat.txt)
STANDALONE_CALLS_PER_GRAPH = 8

# Every live trainer is closed (graphs -> streams / events / device counters, NativeTrainer.close) by an atexit hook
# when a script ends without DistContext.finalize: Python runs atexit handlers in reverse registration order, and this
# one is registered after `import torch`, so it runs before torch's own exit handlers and long before the C++ static
# destructors that tear the HIP runtime down -- the native teardown never runs against a dead runtime (the failure
# mode suspected behind the round-4 rank exit 139; PARITY.md §5.3).
_LIVE_TRAINERS: "weakref.WeakSet" = weakref.WeakSet()


def _close_live_trainers() -> None:
    for tr in list(_LIVE_TRAINERS):
        if getattr(tr, "comm", None) is not None or getattr(tr, "oneshot", None) is not None:
            continue  # collectives attached: DistContext.finalize's bounded teardown owns it (a dead peer must not
            #           turn the exit of a failing rank into a wait on a collective that never completes)
        try:
            tr.close()
        except Exception as e:  # teardown must not raise at exit; report and go on
            print(f"[mnist_amd] trainer teardown at exit: {e}", file=sys.stderr, flush=True)


atexit.register(_close_live_trainers)


def resolve_plan(name: Optional[str]) -> Optional[str]:
    """CLI ``--plan`` value -> the plan to pin, or None for the start-up calibration.

    ``auto`` (or None) = calibrate; ``fixed`` = no calibration, keep the default ``join`` plan; a plan
    name pins it.  Anything else is rejected here, before any device work."""
    if name is None or name == "auto":
        return None
    if name == "fixed":
        return "join"
    if name not in PLANS:
        raise ValueError(f"unknown step plan {name!r} (choices: auto, fixed, {', '.join(sorted(PLANS))})")
    return name


def split_allowed(world: int) -> bool:
    """SPLIT-family plans (per-group collectives on a comm stream beside the backward) are calibration candidates at
    world 1 (tests, --comm-world1) and, at world >= 2, only with ``MNIST_AMD_SPLIT=1``: they have not run across real
    GPUs yet, and a replay that hangs at world >= 2 can only end in the calibration watchdog's abort, while JOIN is
    the schedule every multi-rank run can fall back on (advisor, round 5).  ``MNIST_AMD_NO_SPLIT=1`` removes them
    everywhere."""
    if os.environ.get("MNIST_AMD_NO_SPLIT", "0") == "1":
        return False
    return world <= 1 or os.environ.get("MNIST_AMD_SPLIT", "0") == "1"


def forced_plan() -> Optional[str]:
    """``MNIST_AMD_MG_SCHED`` pins the multi-GPU plan (validated: a typo must not silently calibrate)."""
    v = os.environ.get("MNIST_AMD_MG_SCHED")
    if not v:
        return None
    if v not in PLANS:
        raise ValueError(f"MNIST_AMD_MG_SCHED={v!r}: expected one of {sorted(PLANS)}")
    return v
PLAN_NAMES = {v: k for k, v in PLANS.items()}


def calib_blocks(avail: int, k: int, multi: bool):
    """Sample shape of :meth:`NativeTrainer.time_schedules`: (multi, replays per sample, samples per
    segment, steps per sample).  A sample replays from the rewound step counter, so it must never run
    past the ``avail`` loaded steps: at most 4 k-step replays and no more than fit (a 4 x 20-step block
    over a 28-step order once read past the index buffer -- a GPU memory fault)."""
    blk = min(4, avail // k) if multi and k > 1 else 1
    if blk < 1:
        multi, blk = False, 1
    seg = 4 if multi else 12
    per = blk * (k if multi else 1)
    if per > avail:
        raise RuntimeError(f"time_schedules: a sample of {per} steps exceeds the {avail} loaded steps")
    return bool(multi), blk, seg, per


# (Rounds 3-4 pinned the serial schedule for single-GPU LeNet batches <= 1024 because the calibration had timed
#  it wrong at B = 128 (profiles/r3_session3/calib_probe_b128.txt).  Round 5, same box: the calibration now picks
#  serial at B = 128 itself (bf16 0.0301 vs 0.0345 ms, fp32 0.0498 vs 0.0547) and concurrent at B = 1024, where
#  the pinned serial schedule was 10 % slower (47.7 vs 52.4 us per step): profiles/r5_session1/calib_b128_auto.jsonl.
#  The rule is gone; every single-GPU LeNet batch is calibrated.)


class CollectiveError(RuntimeError):
    """A gradient collective failed or exceeded the watchdog deadline; the communicator is aborted.
    ``detected_after`` = seconds from the start of the wait to the detection (before the abort)."""

    def __init__(self, msg: str, detected_after: float = 0.0):
        super().__init__(msg)
        self.detected_after = detected_after


HEAD_DIMS = {  # K0P, N1P, N2P  (csrc/kernels/models.h)
    "mlp": (800, 128, 128),
    "lenet5": (416, 128, 96),
}


def _rup(x: int, m: int) -> int:
    return (x + m - 1) // m * m


GUARD_BYTES = 4096   # per side of a guarded buffer (MNIST_AMD_GUARD)
GUARD_FILL = 0xA5


def _alloc(shape, dt, dev, guards):
    """Zeroed device buffer; with a guard list, carved out of a larger allocation whose bytes before and after
    the buffer hold GUARD_FILL (recorded in ``guards`` for NativeTrainer.check_guards)."""
    if guards is None:
        return torch.zeros(*shape, dtype=dt, device=dev)
    n = 1
    for d in shape:
        n *= int(d)
    nb = n * torch.empty((), dtype=dt).element_size()
    raw = torch.full((2 * GUARD_BYTES + _rup(nb, 256),), GUARD_FILL, dtype=torch.uint8, device=dev)
    body = raw[GUARD_BYTES:GUARD_BYTES + nb]
    body.zero_()
    guards.append((raw, nb))
    return body.view(dt).view(*shape)


@dataclass
class EpochStats:
    loss_sum: float
    correct: float
    count: float

    @property
    def mean_loss(self) -> float:
        return self.loss_sum / max(self.count, 1.0)

    @property
    def accuracy(self) -> float:
        return self.correct / max(self.count, 1.0)


class NativeTrainer:
    def __init__(self, model: str, dtype: str, batch: int, images: torch.Tensor, labels: torch.Tensor,
                 device: Optional[torch.device] = None, lr: float = 0.01, momentum: float = 0.0,
                 dropout: float = 0.2, seed: int = 1234, fc_splits: Optional[int] = None,
                 init: Optional[torch.nn.Module] = None, max_indices: Optional[int] = None):
        C = require_gpu()
        self.C = C
        self.model_name = model
        self.dtype_name = dtype
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.batch = int(batch)
        mid = MODEL_IDS[model]
        tdt = torch.float32 if dtype == "fp32" else torch.bfloat16
        did = 0 if dtype == "fp32" else 1
        dev = self.device
        self.nparam = C.model_nparam(mid)
        self.images = images.to(dev, torch.uint8).contiguous().view(-1, 784)
        self.labels = labels.to(dev, torch.uint8).contiguous().view(-1)
        n_max = max_indices or self.images.shape[0]
        self.ld_b = _rup(self.batch, 64)
        KC = 16 if dtype == "fp32" else 32
        if fc_splits is None:
            fc_splits = int(os.environ.get("MNIST_AMD_FC_SPLITS", "0")) or max(1, min(16, _rup(self.batch, KC) // 512))
        K0P, N1P, N2P = HEAD_DIMS[model]
        # MNIST_AMD_GUARD=1: every buffer the kernels address sits between two guard regions of a known byte
        # pattern; check_guards() names the buffers whose guards a launch wrote (an out-of-bounds store)
        self._guards = [] if os.environ.get("MNIST_AMD_GUARD", "0") not in ("", "0") else None
        z = lambda *s, dt=tdt: _alloc(s, dt, dev, self._guards)  # noqa: E731
        self.params = z(self.nparam, dt=torch.float32)
        self.grad = z(self.nparam, dt=torch.float32)
        self.mom = z(self.nparam, dt=torch.float32)
        self.pack_buf = z(C.model_pack_size(mid))
        self.idx = torch.zeros(n_max, dtype=torch.int32, device=dev)
        # device counters: [0] step within the epoch (batch addressing), [1] global step (dropout stream),
        # [2] loaded indices of the epoch (look-ahead gather bound)
        self.step_ctr = torch.zeros(4, dtype=torch.int32, device=dev)
        # per-head-workgroup metric rows [loss_sum, correct, count, 0], summed when read (no atomics)
        self.metrics = z(C.metric_rows(self.batch), 4, dt=torch.float32)
        self.eval_metrics = z(C.metric_rows(self.batch), 4, dt=torch.float32)
        self.xT, self.h1T, self.h2T = z(K0P, self.ld_b), z(N1P, self.ld_b), z(N2P, self.ld_b)
        self.dy1T, self.dy2T, self.dy3T = z(N1P, self.ld_b), z(N2P, self.ld_b), z(16, self.ld_b)
        self.slab_fc = z(fc_splits, _rup(self.nparam, 4), dt=torch.float32)  # rows 16-byte aligned (Trainer::fc_ld)
        # rows for any batch <= self.batch (a partial last batch can need more workgroups than a full one).
        # (Round 5 measured the transposed layout -- one slab column per workgroup, one wave per parameter in the
        # conv update -- and reverted it: conv_bwd's scattered column stores cost 50.7 -> 54.4 us at B = 8192
        # and the update did not get faster (5.5 -> 5.1 us; B = 128 4.6 -> 4.7 us): profiles/r5_session1/NOTES.md.)
        conv_slabs = C.conv_bwd_max_blocks(self.batch) if model == "lenet5" else 0
        ncp = C.model_conv_params(mid)
        self.slab_conv = z(max(conv_slabs, 1), max(ncp, 1), dt=torch.float32)
        if model == "lenet5":
            self.p1 = z(self.ld_b * 196 * 8)
            self.m1 = z(self.ld_b * 196 * 8, dt=torch.uint8)
            self.p2 = z(self.ld_b, 416)
            self.m2 = z(self.ld_b * 400, dt=torch.uint8)
            self.dp2 = z(self.ld_b, 416)
        else:
            self.p1 = self.m1 = self.p2 = self.m2 = self.dp2 = None
        # layer-1 K-split partials for the small-batch path (csrc/kernels/head.hip l1_split_kernel)
        self.z1p = z(C.L1_KSPLIT * N1P * self.ld_b, dt=torch.float32) if self.batch <= C.L1_SPLIT_MAX_B else None
        # small-batch MLP: the next step's pixels / labels, gathered one step ahead by the head kernel (rows
        # padded to the tiles that read them).  (At B=8192 the same look-ahead -- the head kernel supports
        # it at every tile size -- measured no gain: 35.4-35.6 vs 35.2-35.8 us per step, same box; the
        # staging phase is not bound by the random dataset rows.)
        look = model == "mlp" and self.z1p is not None and not os.environ.get("MNIST_AMD_NO_LOOKAHEAD")
        self.xnext = z(_rup(self.batch, 64) * 784, dt=torch.uint8) if look else None
        self.ynext = z(_rup(self.batch, 64), dt=torch.uint8) if look else None
        # LeNet small batches: conv_fwd's pixel rows in batch order for conv_bwd (no index chain at its start)
        xbm = getattr(C, "XB_MAX_B", 0)
        self.xb = z(self.batch * 785, dt=torch.uint8) if model == "lenet5" and self.batch <= xbm else None  # rows | labels

        P = C.TrainerPtrs()
        ptr = lambda t: 0 if t is None else t.data_ptr()  # noqa: E731
        P.images, P.labels, P.idx, P.step = ptr(self.images), ptr(self.labels), ptr(self.idx), ptr(self.step_ctr)
        P.params, P.grad, P.mom, P.pack = ptr(self.params), ptr(self.grad), ptr(self.mom), ptr(self.pack_buf)
        P.slab_fc, P.slab_conv, P.metrics = ptr(self.slab_fc), ptr(self.slab_conv), ptr(self.metrics)
        P.xT, P.h1T, P.h2T = ptr(self.xT), ptr(self.h1T), ptr(self.h2T)
        P.dy1T, P.dy2T, P.dy3T = ptr(self.dy1T), ptr(self.dy2T), ptr(self.dy3T)
        P.p1, P.m1, P.p2, P.m2, P.dp2 = ptr(self.p1), ptr(self.m1), ptr(self.p2), ptr(self.m2), ptr(self.dp2)
        P.z1p = ptr(self.z1p)
        P.xnext, P.ynext = ptr(self.xnext), ptr(self.ynext)
        if hasattr(P, "xb"):
            P.xb = ptr(self.xb)
        # MNIST_AMD_STAMPS=1: per-workgroup phase timestamps (wall clock, 100 MHz), 16 slots per workgroup,
        # one row range per kernel (csrc/kernels/launch.h STAMP_*; later workgroups skip)
        self.stamps = z(C.STAMP_ROWS * 16, dt=torch.int64) if os.environ.get("MNIST_AMD_STAMPS") else None
        P.stamps = ptr(self.stamps)
        self._ptrs = P
        self.rt = C.Trainer(mid, did, self.batch, self.ld_b, fc_splits, P)
        self.rt.set_optimizer(float(lr), float(momentum))
        self.rt.set_dropout(float(dropout), int(seed) & 0xFFFFFFFF)
        self._base_buckets = [(b.p0, b.p1, b.phase) for b in self.rt.buckets()]  # the native default (2 groups)
        _LIVE_TRAINERS.add(self)
        self.stream = torch.cuda.Stream(device=dev)
        self.world = 1
        self.comm = None
        self.oneshot = None         # one-shot xGMI all-reduce data plane (attach_oneshot)
        self.overlap = None         # (FC, conv) one-shot instances of the OVERLAP plan (attach_overlap)
        self.ext_allreduce = None   # external data plane (attach_external_allreduce)
        self.capture_failures = {}  # candidate schedules the runtime refused to capture (time_schedules)
        self.module_template = build_model(model)
        if init is not None:
            self.load_module(init)
        else:
            self.load_module(self.module_template)

    # ------------------------------------------------------------------ parameters
    def _sync_in(self):
        """Order our stream after torch's current stream (tensors written by torch ops)."""
        self.stream.wait_stream(torch.cuda.current_stream(self.device))

    def _sync_out(self):
        torch.cuda.current_stream(self.device).wait_stream(self.stream)

    def load_flat(self, flat: torch.Tensor) -> None:
        self.params.copy_(flat.to(self.device, torch.float32).view(-1))
        self._sync_in()
        self.rt.pack(self.stream.cuda_stream)
        self._sync_out()

    def load_module(self, module: torch.nn.Module) -> None:
        self.load_flat(flatten_state(module))

    def state_dict(self) -> Dict[str, torch.Tensor]:
        self.synchronize()
        return unflatten_state(self.module_template, self.params)

    def to_module(self) -> torch.nn.Module:
        m = build_model(self.model_name)
        m.load_state_dict(self.state_dict())
        return m

    # ------------------------------------------------------------------ distributed
    def attach_comm(self, comm, world: int, plan: str = "join", bwd_blocks: int = 0) -> None:
        """Use a native RcclComm for the gradient all-reduce (None = local only)."""
        self.comm, self.world = comm, world
        if comm is not None:
            self.rt.set_comm(comm)
        self.rt.set_world(world)
        self.set_plan(plan, bwd_blocks)

    def attach_oneshot(self, oneshot, world: int, plan: str = "join") -> None:
        """Use the one-shot xGMI all-reduce (parallel/oneshot.py) for the step's gradient collectives instead of
        RCCL.  An RCCL communicator may stay attached (parameter broadcast, comm_profile comparison)."""
        self.oneshot = oneshot
        self.world = int(world)
        self.rt.set_oneshot(oneshot)
        self.rt.set_world(self.world)
        self.set_plan(plan, 0)

    def attach_overlap(self, fc, conv, world: int) -> None:
        """LeNet: the OVERLAP plan's two one-shot instances (``make_oneshot`` each; FC range and conv range) --
        the concurrent single-GPU schedule with each branch's all-reduce inside it (csrc/runtime/trainer.h
        Plan::OVERLAP).  The installed plan is not changed: ``set_plan('overlap')`` / the calibration picks it."""
        if self.model_name != "lenet5":
            raise ValueError("the overlap plan is LeNet-only")
        self.overlap = (fc, conv)
        self.world = int(world)
        self.rt.set_overlap(fc, conv)
        self.rt.set_world(self.world)

    def set_plan(self, plan: str, bwd_blocks: int = 0) -> None:
        if plan not in PLANS:
            raise ValueError(f"unknown step plan {plan!r} (choices: {sorted(PLANS)})")
        self.rt.set_plan(PLANS[plan])
        if self.model_name == "lenet5":
            self.rt.set_bwd_blocks(int(bwd_blocks))

    def fwd_head_applies(self, B: Optional[int] = None) -> bool:
        """LeNet bf16: a full step of B rows (default: the trainer batch) can run conv_fwd + the FC head as
        ONE kernel (fwd_head_kernel); the installed schedule uses it unless ``fwd_head: False``."""
        return self.model_name == "lenet5" and bool(self.C.fwd_head_applies(1 if self.dtype_name == "bf16" else 0,
                                                                               int(B or self.batch)))

    @property
    def plan(self) -> str:
        return PLAN_NAMES[self.rt.plan]

    def plan_info(self) -> dict:
        """What a full-batch step runs: plan, conv_bwd grid, and the collectives in issue order."""
        coll = [(b.p0, b.p1) for b in self.rt.issued_collectives()]
        dp = self.comm is not None or self.oneshot is not None or self.overlap is not None
        ov = self.plan == "overlap"
        groups = {(b.p0, b.p1): b.phase for b in self.rt.buckets()}
        return {"plan": self.plan if dp else ("local" if self.rt.concurrent else "local-serial"),
                "allreduce": "oneshot" if (self.oneshot is not None or ov) else ("rccl" if self.comm is not None else None),
                "conv_bwd_grid": self.rt.bwd_grid if self.model_name == "lenet5" else None,
                "collectives": [{"params": [a, b], "bytes": 4 * (b - a),
                                 **({"group": groups[(a, b)]} if self.plan == "split" and (a, b) in groups else {})}
                                for a, b in coll]}

    def set_buckets(self, ranges) -> None:
        """Install a bucket plan (ranges (p0, p1, group), groups in backward-ready order: csrc Trainer::set_buckets)
        as the trainer's base plan; calibration candidates that carry their own ``buckets`` switch to theirs."""
        self._base_buckets = [tuple(int(v) for v in r) for r in ranges]
        self._install_buckets(self._base_buckets)

    def _install_buckets(self, ranges) -> None:
        self.rt.set_buckets([self.C.Bucket(int(a), int(b), int(ph)) for a, b, ph in ranges])

    def current_buckets(self):
        return [(b.p0, b.p1, b.phase) for b in self.rt.buckets()]

    def bucket_model(self, reduce_max=None, iters: int = 24, warmup: int = 4) -> dict:
        """Inputs of the link-aware bucket plan (parallel/ddp.py choose_bucket_groups), measured on this job:
        the RCCL all-reduce latency at LATENCY_SWEEP_BYTES on the real communicator (standalone collectives, 8 per
        graph, rank-max median) and each gradient-producing unit's backward cost (Trainer::time_units, rank-max).
        Collective: every rank calls it at the same point.  Gradients and slabs are scratch here (restored)."""
        from ..parallel.ddp import LATENCY_SWEEP_BYTES, LatencyCurve, choose_bucket_groups, fc_unit_count
        if self.comm is None:
            raise RuntimeError("bucket_model: needs an RCCL communicator")
        rmax = reduce_max if reduce_max is not None else (lambda v: v)
        pts = []
        nmax = max(LATENCY_SWEEP_BYTES) // 4
        buf = torch.zeros(nmax, dtype=torch.float32, device=self.device)
        self._sync_in()
        for nb in LATENCY_SWEEP_BYTES:
            try:
                ts = self.comm.time_all_reduce(buf.data_ptr(), nb // 4, warmup, iters, self.stream.cuda_stream,
                                               comm_timeout(), per_graph=STANDALONE_CALLS_PER_GRAPH)
            except RuntimeError as e:
                self.comm.abort()
                raise CollectiveError(f"rank {self.comm.rank}: {e} (communicator aborted)") from e
            ts = sorted(ts)
            pts.append((nb, rmax(ts[len(ts) // 2] * 1000.0)))
        lat = LatencyCurve(pts)
        saved = self.grad.clone()
        with torch.cuda.stream(self.stream):
            us = [rmax(float(v)) for v in self.rt.time_units(iters, warmup, self.stream.cuda_stream)]
            self.grad.copy_(saved)
        self.synchronize()
        nfc = fc_unit_count(self.model_name)
        unit_us, fc_all = us[:nfc], us[nfc]
        main = us[nfc + 1] if len(us) > nfc + 1 else 0.0
        ranked = choose_bucket_groups(self.model_name, lat, unit_us, fc_all, main)
        return {"latency_us": lat.as_dict(), "unit_us": [round(v, 2) for v in unit_us], "fc_all_us": round(fc_all, 2),
                "main_us": round(main, 2),
                "ranked": [{"groups": g, "modelled_us": round(t, 2)} for g, t in ranked], "_ranked": ranked,
                "note": "comm-stream timeline model used to pick which bucket plans to time; it does not price the "
                        "extra groups' kernels contending with the main stream -- the calibration's measured "
                        "timings_ms decide"}

    def broadcast_params(self, root: int = 0) -> None:
        """DDP construction semantics: every rank starts from rank 0's parameters (over RCCL, or over the
        c10d control plane when only the one-shot data plane is attached)."""
        if self.comm is None:
            if self.oneshot is not None and self.world > 1:
                import torch.distributed as dist
                p = self.params.detach().cpu()
                dist.broadcast(p, root)
                self.load_flat(p)
            return
        self._sync_in()
        self.comm.broadcast_f32(self.params.data_ptr(), self.nparam, root, self.stream.cuda_stream)
        self.rt.pack(self.stream.cuda_stream)
        self.synchronize()

    def attach_external_allreduce(self, fn, world: int, host: bool = True) -> None:
        """Exchange gradients through an EXTERNAL collective instead of the native RCCL communicator:
        ``fn(t)`` must SUM ``t`` in place across the ranks (c10d gloo / c10d nccl all_reduce).

        Every step then runs the phase API: forward/backward + slab reduce on the device, the gradient
        slab into ``fn`` (staged through pinned host memory when ``host``, else the device tensor on the
        trainer stream), then the SGD update with the 1/W average folded in.  No graphs: the collective
        is a host call.  This is the plumbing / test path -- with a host collective several processes
        can share ONE GPU (RCCL refuses two ranks on one device), so the whole multi-process chain
        (launch, rendezvous, broadcast, rank-max calibration, sharded training) runs on a one-GPU box."""
        self.ext_allreduce = (fn, bool(host))
        self.world = int(world)
        self.rt.set_world(self.world)
        self._host_grad = torch.empty(self.nparam, dtype=torch.float32, pin_memory=True) if host else None

    def _external_step(self, B: int) -> None:
        fn, host = self.ext_allreduce
        self.forward_backward(B)
        if host:
            with torch.cuda.stream(self.stream):
                self._host_grad.copy_(self.grad, non_blocking=True)
            self.stream.synchronize()
            fn(self._host_grad)
            with torch.cuda.stream(self.stream):
                self.grad.copy_(self._host_grad, non_blocking=True)
        else:
            with torch.cuda.stream(self.stream):
                fn(self.grad)
        self.optimizer_step(1.0 / self.world)

    def check_comm(self) -> None:
        """Health poll (once per epoch): abort + raise on an asynchronous RCCL error; raise if a one-shot
        all-reduce flag wait timed out (also raised by every :meth:`synchronize`)."""
        self._check_oneshot()
        if self.comm is None:
            return
        err = self.comm.async_error()
        if err:
            self.comm.abort()
            raise CollectiveError(f"RCCL communicator error on rank {self.comm.rank}: {err}")

    def current_schedule(self) -> dict:
        """The installed schedule as a complete :meth:`apply_plan` candidate."""
        return {"plan": self.plan, "bwd_blocks": int(self.rt.bwd_blocks) if self.model_name == "lenet5" else 0,
                "concurrent": bool(self.rt.concurrent), "fwd_head": bool(self.rt.fwd_head),
                "buckets": self.current_buckets()}

    def apply_plan(self, cfg: dict) -> None:
        """Install one candidate of :meth:`autotune_plan` ({plan, bwd_blocks, concurrent, fwd_head, comm}).
        Keys a candidate leaves out take their defaults (join, default conv_bwd grid, concurrent, fused
        forward + head kernel, comm on), so a candidate names ONE cached graph whatever was installed
        before it.  ``comm: False`` (timing only) runs the local schedule without collectives."""
        self.rt.comm_enabled = bool(cfg.get("comm", True))
        self.rt.set_concurrent(bool(cfg.get("concurrent", True)))
        self.rt.set_fwd_head(bool(cfg.get("fwd_head", True)))
        self._install_buckets(cfg.get("buckets") or self._base_buckets)
        self.set_plan(cfg.get("plan", "join"), int(cfg.get("bwd_blocks", 0)))

    def time_schedules(self, candidates: Dict[str, dict], iters: int = 48, warmup: int = 8,
                       reduce_max=None, multi: Optional[bool] = None) -> Dict[str, float]:
        """Median step time (ms) of each candidate schedule, state restored afterwards.

        Every candidate's step graph (and its k-step graph) is captured first -- graphs are cached
        per schedule.  What is timed is what training replays: blocks of k-step graph replays
        (``multi``, when the loaded order holds k + 1 batches; per-step time = block time / steps),
        else single-step replays.  Each candidate runs in segments of consecutive samples: one
        untimed round over all candidates, then two timed rounds, the second in reverse order (the
        GPU clock ramps up during the first milliseconds of work; the reverse round hands no
        candidate the faster clock), with no host sync in between.  Replays train on consecutive
        batches of the loaded epoch order from batch 0, the device step counter rewound when the
        order runs out, identically on every rank, so all ranks issue the same collectives in the
        same order; GPU times come from events on the step stream and ``reduce_max`` (e.g. a gloo
        MAX all-reduce) makes the result identical on every rank.  Parameters, momentum, gradients,
        counters and metrics are restored afterwards (the operand images are re-packed); the
        schedule installed before the call is re-installed.  ``iters`` / ``warmup`` are accepted
        for API compatibility (the segment plan fixes the sample counts)."""
        if getattr(self, "n_epoch", 0) < max(2, self.host_step + 1) * self.batch:
            raise RuntimeError("time_schedules: the loaded epoch order needs >= 2 full batches beyond the current step")
        # time what training replays: the k-step graph (run_steps) when the loaded order holds k + 1 batches
        # (per-replay time / k).  Single-step replays ranked the LeNet B=128 schedules the wrong way round:
        # concurrent 0.0485 vs serial 0.0490 ms, but 35.4 vs 33.0 us per step in 8-step graphs.
        k = self.graph_steps()
        can = k > 1 and self.ext_allreduce is None and getattr(self, "n_epoch", 0) >= (k + 1) * self.batch
        multi = can if multi is None else (bool(multi) and can)
        avail = getattr(self, "n_epoch", 0) // self.batch  # steps the loaded order holds
        multi, blk, seg, per = calib_blocks(avail, k, multi)
        self.last_timing = {"graph_steps": k if multi else 1, "replays": 2 * (seg - 1) * blk}
        before = self.current_schedule()
        self.synchronize()
        saved = [t.clone() for t in (self.params, self.mom, self.grad, self.step_ctr, self.metrics)]
        self._sync_in()
        st = self.stream
        names = list(candidates)
        failed = {}
        for name in names:                 # all captures (host work) before any timed replay
            try:
                self.apply_plan(candidates[name])
                self.prepare_graphs()
                if multi and self.rt.multi_steps != k:
                    self.rt.capture_multi(st.cuda_stream, k)
            except RuntimeError as e:      # a capture the runtime refuses drops that candidate, not the run
                failed[name] = str(e)
        # every rank drops the same candidates (a captured collective has not run yet: dropping one is safe)
        agree = reduce_max if reduce_max is not None else (lambda v: v)
        names = [n for n in names if not agree(1.0 if n in failed else 0.0)]
        self.capture_failures = failed
        if not names:
            raise RuntimeError(f"time_schedules: no candidate could be captured: {failed}")
        self.apply_plan(candidates[names[0]])
        ev = {name: [] for name in names}
        with torch.cuda.stream(st):
            self.step_ctr[0].zero_()       # every replay trains on batch 0 of the loaded order
        # Each candidate runs in SEGMENTS of consecutive samples (the first sample of a segment untimed), in
        # one untimed round and two timed rounds, the second in reverse order so the GPU clock ramp favours
        # no candidate.  Interleaving candidates replay by replay slowed the graphs that followed a different
        # graph: LeNet B=128 serial measured 38.7 us/step interleaved with the concurrent schedule but 33.0 in
        # its own segment and in run_steps (same box), which ranked the schedules the wrong way round.
        # A k-step sample is a block of `blk` back-to-back replays between one pair of events; the step
        # counter is rewound only when the next block would run past the loaded order.
        pos = 0
        rounds = [names, names, names[::-1]]
        for r, order in enumerate(rounds):
            for name in order:
                self.apply_plan(candidates[name])   # host-side switch to the cached graph
                for j in range(seg):
                    if pos + per > avail or not multi:
                        with torch.cuda.stream(st):
                            self.step_ctr[0].zero_()
                        pos = 0
                    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    a.record(st)
                    for _ in range(blk):
                        if multi:
                            self.rt.replay_multi(st.cuda_stream)
                        else:
                            self.rt.replay(st.cuda_stream)
                    b.record(st)
                    pos += per
                    if r > 0 and j > 0:
                        ev[name].append((a, b))
        # the calibration's own watchdog: a candidate whose collectives never complete fails the start-up within
        # minutes, naming the calibration, instead of after the step loop's full deadline
        self.synchronize(timeout=min(comm_timeout(), float(os.environ.get("MNIST_AMD_CALIB_TIMEOUT", "180"))))
        timings = {}
        if os.environ.get("MNIST_AMD_CALIB_DEBUG"):
            for name in names:
                print(f"calib {name}: " + " ".join(f"{a.elapsed_time(b) / (blk * k if multi else 1) * 1000:.1f}"
                                                  for a, b in ev[name]), file=sys.stderr, flush=True)
        for name in names:
            ts = sorted(a.elapsed_time(b) / (blk * k if multi else 1) for a, b in ev[name])
            med = ts[len(ts) // 2]
            timings[name] = reduce_max(med) if reduce_max is not None else med
        with torch.cuda.stream(st):
            for dst, src in zip((self.params, self.mom, self.grad, self.step_ctr, self.metrics), saved):
                dst.copy_(src)
        self.rt.pack(st.cuda_stream)
        # the replays advanced the MLP look-ahead rows (xnext / ynext) past the restored step counter
        self.rt.prime_next(st.cuda_stream)
        self.apply_plan(before)
        return timings

    def autotune_plan(self, candidates=None, iters: int = 48, warmup: int = 8, reduce_max=None,
                      margin: float = 0.015, log=None) -> dict:
        """Time each candidate step schedule (:meth:`time_schedules`) and keep the fastest (a start-up
        calibration, like cudnn.benchmark).

        With a communicator the candidates are the multi-GPU plans -- LeNet: JOIN / SPLIT / SPLIT
        with a capped conv_bwd grid (:func:`~pytorch_ddp_mnist_amd.parallel.ddp.default_plan_candidates`);
        MLP: JOIN / SPLIT (:func:`~pytorch_ddp_mnist_amd.parallel.ddp.mlp_plan_candidates`) -- timed on
        the real communicator, plus the timing-only ``nocomm`` schedule (the local single-GPU step, no
        collective), so ``exposed_comm_ms`` = chosen plan - nocomm is measured in the same interleaved
        run.  Without a communicator, the single-GPU LeNet schedules
        (:func:`~pytorch_ddp_mnist_amd.parallel.ddp.local_plan_candidates`).
        ``MNIST_AMD_MG_SCHED=join|split`` pins the multi-GPU plan.

        Sample plan (:meth:`time_schedules`, :func:`calib_blocks`): every candidate runs in segments of
        consecutive k-step graph replays (blocks of up to 4 replays between two events, k =
        ``MNIST_AMD_GRAPH_STEPS``) -- one untimed round over all candidates, then two timed rounds, the
        second in reverse order -- so each candidate gets 2 x (segment - 1) timed samples (``replays_per_
        candidate`` in the result; ``iters`` / ``warmup`` are accepted for API compatibility only).  The
        median per candidate is max-reduced over the ranks.  The run also brings the GPU from idle to its
        sustained clock before the caller's warm-up steps (measured: steps 1-20 after a cold start run ~6 %
        slower than steps 100+, scripts/step_times.py).

        At world >= 2 the SPLIT plans are candidates too (``MNIST_AMD_NO_SPLIT=1`` keeps JOIN only): their
        collectives and updates run on ONE comm stream in a fixed order (FC buckets beside conv_bwd, then the
        conv buckets), and only the main stream consumes the comm stream's completion, once, at the end of the
        step -- the capture pattern that made hipStreamEndCapture fail on ROCm 7.0 (a stream waiting on an event
        recorded behind a captured RCCL call) is not used, and a world-1 test replays that pattern on the box's
        runtime (``RcclComm.probe_cross_stream_capture``).  A candidate whose capture the runtime refuses is
        dropped on every rank (:meth:`time_schedules`), and the calibration waits under its own watchdog
        (``MNIST_AMD_CALIB_TIMEOUT``, default 180 s).
        ``exposed_comm_ms`` is measured against the local schedule with the chosen plan's fwd_head /
        conv_bwd-grid settings and the faster of the concurrent / serial single-GPU branch.
        """
        from ..parallel.ddp import (bucket_plan_candidates, choose_plan, default_plan_candidates,
                                    local_plan_candidates, mlp_plan_candidates)
        forced = forced_plan()
        bmodel = None
        dp = self.comm is not None or self.oneshot is not None  # a gradient data plane is attached
        ovl = dp and self.overlap is not None and self.model_name == "lenet5"  # + the one-shot OVERLAP plan
        if dp and forced:
            self.set_plan(forced, 0)
            return {"chosen": forced, "timings_ms": {}, "forced": True}
        if candidates is None:
            if dp:
                if self.model_name == "lenet5":
                    ncu = torch.cuda.get_device_properties(self.device).multi_processor_count
                    candidates = default_plan_candidates(self.C.conv_bwd_blocks(self.batch), ncu)
                else:
                    candidates = mlp_plan_candidates()
                if not split_allowed(self.world):
                    candidates = {k: v for k, v in candidates.items() if v.get("plan", "join") == "join"}
                elif self.comm is not None and self.oneshot is None and os.environ.get("MNIST_AMD_BUCKET_MODEL", "1") != "0":
                    # link-aware bucket groups: the modelled best plan and the best multi-bucket plan join the
                    # candidates (parallel/ddp.py choose_bucket_groups; inputs measured on this communicator)
                    bmodel = self.bucket_model(reduce_max=reduce_max)
                    candidates.update(bucket_plan_candidates(self.model_name, bmodel.pop("_ranked"),
                                                             base=candidates.get("split")))
                if ovl:
                    candidates["overlap"] = dict(plan="overlap")
            elif self.model_name == "lenet5":
                candidates = local_plan_candidates(fwd_head=self.fwd_head_applies())
            else:
                return {"chosen": "local", "timings_ms": {}}
        prefer = "join" if dp else "concurrent"
        extra = {}
        if dp:
            # the local step without collectives, in both single-GPU branch forms: exposed communication is
            # measured against the faster one (the concurrent branch is not the local best at every batch)
            for conc in (True, False):
                extra[f"nocomm{'' if conc else '_serial'}"] = {"comm": False, "concurrent": conc}
        if len(candidates) == 1 and not extra:
            chosen = next(iter(candidates))
            self.apply_plan(candidates[chosen])
            return {"chosen": chosen, "timings_ms": {}, "candidates": candidates, "single_candidate": True}
        timings = self.time_schedules({**candidates, **extra}, iters=iters, warmup=warmup, reduce_max=reduce_max)
        ok = {k: timings[k] for k in candidates if k in timings}
        if not ok:
            raise RuntimeError(f"autotune_plan: no candidate could be captured: {self.capture_failures}")
        chosen = choose_plan(ok, prefer=prefer, margin=margin)
        self.apply_plan(candidates[chosen])
        out = {"chosen": chosen, "timings_ms": {k: round(v, 4) for k, v in timings.items()},
               "candidates": candidates, "replays_per_candidate": self.last_timing["replays"],
               "steps_per_replay": self.last_timing["graph_steps"], "interleaved": True}
        if self.capture_failures:
            out["capture_failures"] = self.capture_failures
        if bmodel is not None:
            out["bucket_model"] = bmodel
        if extra and any(k in timings for k in extra):
            local = min(timings[k] for k in extra if k in timings)
            out["nocomm_ms"] = round(local, 4)
            out["exposed_comm_ms"] = round(timings[chosen] - local, 4)
        if log is not None:
            log(out)
        return out

    def comm_profile(self, reduce_max=None, iters: int = 48, warmup: int = 8, tune: Optional[dict] = None,
                     probe=None) -> dict:
        """Attributable communication figures of the installed plan (bench JSON ``comm_profile``).

        * ``rccl_world`` -- ranks of the RCCL communicator;
        * per collective the step issues: its size and the latency of ONE standalone all-reduce of that
          size, captured in its own graph and replayed back to back (median of ``iters``, rank-max);
        * ``step_plan_ms`` / ``step_local_ms`` / ``exposed_comm_us`` -- the captured step with the plan's
          collectives vs the local single-GPU schedule without any, interleaved replays (taken from
          ``tune`` when the calibration already timed both);
        * ``probe``: a validated one-shot all-reduce that the step does NOT use (measure-only): its standalone
          latency per collective is reported next to RCCL's (``oneshot_us``).
        Collective: every rank calls it at the same point."""
        if self.comm is None and self.oneshot is None and self.overlap is None:
            return {"rccl_world": None}
        colls = []
        for c in self.plan_info()["collectives"]:
            a, b = c["params"]
            row = {"params": [a, b], "bytes": 4 * (b - a)}
            if self.comm is not None:
                buf = torch.zeros(b - a, dtype=torch.float32, device=self.device)
                self._sync_in()
                try:
                    # 8 calls per graph: the per-call figure, not the host's graph-launch rate
                    ts = self.comm.time_all_reduce(buf.data_ptr(), b - a, warmup, iters, self.stream.cuda_stream,
                                                   comm_timeout(), per_graph=STANDALONE_CALLS_PER_GRAPH)
                except RuntimeError as e:
                    self.comm.abort()
                    raise CollectiveError(f"rank {self.comm.rank}: {e} (communicator aborted)") from e
                ts = sorted(ts)
                med = ts[len(ts) // 2]
                med = reduce_max(med) if reduce_max is not None else med
                row["allreduce_us"] = round(med * 1000.0, 2)
            os_ = self.oneshot if self.oneshot is not None else (probe if probe is not None else
                                                                  (self.overlap[0] if self.overlap else None))
            if os_ is not None:
                from ..parallel.oneshot import time_oneshot
                med = time_oneshot(os_, b - a, self.device, iters=iters, warmup=warmup,
                                   per_graph=STANDALONE_CALLS_PER_GRAPH)
                med = reduce_max(med) if reduce_max is not None else med
                row["oneshot_us"] = round(med * 1000.0, 2)
            colls.append(row)
        tm = (tune or {}).get("timings_ms", {})
        chosen = (tune or {}).get("chosen")
        if chosen in tm and "nocomm_ms" in (tune or {}):
            plan_ms, local_ms = tm[chosen], tune["nocomm_ms"]
        else:
            cur = self.current_schedule()
            loc = {"nocomm": {**cur, "comm": False, "concurrent": True},
                   "nocomm_serial": {**cur, "comm": False, "concurrent": False}}
            t = self.time_schedules({"plan": cur, **loc}, iters=iters, warmup=warmup, reduce_max=reduce_max)
            plan_ms, local_ms = t["plan"], min(t["nocomm"], t["nocomm_serial"])
        return {"rccl_world": int(self.comm.world) if self.comm is not None else None,
                "allreduce": self.plan_info()["allreduce"], "collectives": colls,
                "step_plan_ms": round(plan_ms, 4), "step_local_ms": round(local_ms, 4),
                "exposed_comm_us": round((plan_ms - local_ms) * 1000.0, 2)}

    def close(self) -> None:
        """Final teardown (DistContext.finalize): :meth:`release`, then the native runtime's streams, events and
        device counters are destroyed here, while HIP is certainly up -- not by the pybind destructor, which can run
        during interpreter shutdown after torch's HIP teardown (verdict r4, weak #1).  The trainer is unusable
        afterwards; a second call does nothing."""
        if self.rt is None:
            return
        self.release()
        self.rt.destroy()
        self.rt = None

    def check_guards(self) -> list:
        """MNIST_AMD_GUARD=1 runs: the buffers (attribute names) whose guard bytes no longer hold the fill
        pattern after the queued work drained -- a kernel stored outside them.  [] when none, or no guards."""
        if self._guards is None:
            return []
        self.synchronize()
        names = {}
        for k, v in vars(self).items():
            if isinstance(v, torch.Tensor) and v.is_cuda:
                names.setdefault(v.data_ptr(), k)
        bad = []
        for raw, nb in self._guards:
            lo = raw[:GUARD_BYTES]
            hi = raw[GUARD_BYTES + nb:]
            if bool((lo != GUARD_FILL).any()) or bool((hi != GUARD_FILL).any()):
                bad.append(names.get(raw.data_ptr() + GUARD_BYTES, f"buffer@{raw.data_ptr() + GUARD_BYTES:#x}"))
        return bad

    def release(self) -> None:
        """Teardown (before the communicator is destroyed): drain the streams, drop every cached graph --
        they captured collectives -- and detach the communicator.  The trainer can still run local steps."""
        if self.rt is None:
            return
        try:
            if self.comm is not None and not self.comm.aborted:
                self.synchronize()
            else:
                self.stream.synchronize()
        except CollectiveError:
            pass  # already raised to the caller at its last wait; teardown goes on
        self.rt.release()
        self.comm = None
        self.oneshot = None
        self.overlap = None

    # ------------------------------------------------------------------ training
    def set_epoch_indices(self, indices: torch.Tensor) -> None:
        n = indices.numel()
        if n > self.idx.numel():
            raise ValueError(f"epoch has {n} indices, buffer holds {self.idx.numel()}")
        src = indices.to(torch.int32)
        if src.device.type == "cpu":
            src = src.pin_memory()
        with torch.cuda.stream(self.stream):
            self.idx[:n].copy_(src, non_blocking=True)
            self.step_ctr[0].zero_()
            self.step_ctr[2].fill_(n)
        self.rt.prime_next(self.stream.cuda_stream)  # look-ahead rows of step 0 (no-op without it)
        self.n_epoch = n
        self.host_step = 0  # mirror of the device step counter: every launch is bounds-checked on the host

    def _check_rows(self, B: int) -> None:
        """The kernels read idx[step * batch + r], r < B, through the DEVICE step counter: refuse on the
        host any step that would index past the loaded order (an out-of-bounds gather faults the GPU)."""
        if B <= 0 or B > self.batch:
            raise ValueError(f"batch of {B} rows outside (0, {self.batch}]")
        if getattr(self, "n_epoch", 0) < self.host_step * self.batch + B:
            raise RuntimeError(f"step {self.host_step} of {B} rows would read past the {getattr(self, 'n_epoch', 0)} "
                               f"loaded indices; call set_epoch_indices first")

    def reset_metrics(self) -> None:
        with torch.cuda.stream(self.stream):
            self.metrics.zero_()

    def read_metrics(self, which: str = "train") -> EpochStats:
        self.synchronize()
        m = (self.metrics if which == "train" else self.eval_metrics).double().sum(0).tolist()
        return EpochStats(*m[:3])

    def capture(self) -> None:
        self.rt.capture(self.stream.cuda_stream)

    def step(self, B: Optional[int] = None, use_graph: bool = True) -> None:
        B = self.batch if B is None else B
        if self.ext_allreduce is not None:
            self._external_step(B)   # counts the step itself (optimizer_step)
            return
        self._check_rows(B)
        self.host_step += 1
        if use_graph and B == self.batch:
            if not self.rt.captured:
                self.capture()
            self.rt.replay(self.stream.cuda_stream)
        else:
            self.rt.train_step(B, self.stream.cuda_stream)

    @staticmethod
    def graph_steps() -> int:
        # 10: the 20-step driver shape is two whole graphs (0.1081-0.1098 vs 0.1097-0.1103 ms with 8, same box;
        # equal at 2000 steps)
        return int(os.environ.get("MNIST_AMD_GRAPH_STEPS", "10"))

    def prepare_graphs(self, k: Optional[int] = None, extra=()) -> None:
        """Capture + instantiate the single-step and the k-step graph now (setup, not step time), and a graph
        of each ``extra`` step count >= 2 (the remainders run_steps will need: 20 steps = 8 + 8 + a 4-step
        graph instead of 4 single-step launches)."""
        k = self.graph_steps() if k is None else int(k)
        if not self.rt.captured:
            self.capture()
        if k > 1 and self.rt.multi_steps != k:
            self.rt.capture_multi(self.stream.cuda_stream, k)
        for e in extra:
            e = int(e)
            if e >= 2 and e != k and not self.rt.has_graph(e):
                self.rt.capture_n(self.stream.cuda_stream, e)

    def run_steps(self, n: int, use_graph: bool = True, k: Optional[int] = None) -> None:
        """``n`` consecutive full-batch steps.  With graphs, runs of ``k`` steps are ONE hipGraph launch
        (``MNIST_AMD_GRAPH_STEPS``, default 10; the graph launch gap is paid once per k steps), the
        remainder single-step graphs.  Same kernels, same order, same results as ``n`` x :meth:`step`."""
        k = self.graph_steps() if k is None else int(k)
        if not use_graph or k <= 1 or self.ext_allreduce is not None:
            for _ in range(n):
                self.step(self.batch, use_graph)
            return
        while n >= k:
            if getattr(self, "n_epoch", 0) < (self.host_step + k) * self.batch:
                break  # the k-step window would run past the loaded order: finish with single steps
            if self.rt.multi_steps != k:
                self.rt.capture_multi(self.stream.cuda_stream, k)
            self.rt.replay_multi(self.stream.cuda_stream)
            self.host_step += k
            n -= k
        # the remainder as ONE graph when one of that length was prepared (prepare_graphs(extra=...))
        if (n >= 2 and self.rt.has_graph(n) and getattr(self, "n_epoch", 0) >= (self.host_step + n) * self.batch):
            self.rt.replay_n(self.stream.cuda_stream, n)
            self.host_step += n
            n = 0
        for _ in range(n):
            self.step(self.batch, use_graph)

    def train_epoch(self, indices: torch.Tensor, use_graph: bool = True, progress=None) -> EpochStats:
        self.set_epoch_indices(indices)
        self.reset_metrics()
        n = indices.numel()
        nfull, last = divmod(n, self.batch)
        if progress is None:
            self.run_steps(nfull, use_graph)
        for i in range(nfull if progress is not None else 0):
            self.step(self.batch, use_graph)
            progress(i)
        if last:
            self.step(last, use_graph=False)
        return self.read_metrics("train")

    def evaluate(self, images: torch.Tensor, labels: torch.Tensor, indices: torch.Tensor) -> EpochStats:
        """Forward-only loss/accuracy over ``indices`` (device int32) of (images, labels)."""
        with torch.cuda.stream(self.stream):
            self.eval_metrics.zero_()
        idx = indices.to(self.device, torch.int32).contiguous()
        imgs = images.to(self.device, torch.uint8).contiguous()
        labs = labels.to(self.device, torch.uint8).contiguous()
        n = idx.numel()
        for s in range(0, n, self.batch):
            b = min(self.batch, n - s)
            self.rt.eval_batch(imgs.data_ptr(), labs.data_ptr(), idx.data_ptr() + 4 * s, b,
                               self.eval_metrics.data_ptr(), self.stream.cuda_stream)
        self._keep = (imgs, labs, idx)
        return self.read_metrics("eval")

    # ------------------------------------------------------------------ phases (tests / torch comm)
    def forward_backward(self, B: Optional[int] = None) -> None:
        B = self.batch if B is None else B
        self._check_rows(B)
        self.rt.forward_backward(B, self.stream.cuda_stream)
        self.rt.reduce_grads(B, self.stream.cuda_stream)

    def optimizer_step(self, gscale: float = 1.0) -> None:
        self.rt.optimizer_step(float(gscale), self.stream.cuda_stream)
        self.host_step += 1  # the SGD kernel bumps the device counter

    def grads(self) -> torch.Tensor:
        self.synchronize()
        return self.grad.detach().cpu().clone()

    def synchronize(self, timeout: Optional[float] = None) -> None:
        """Wait for the step stream.  With a communicator this is the collective watchdog: RCCL async
        errors are polled while waiting and a deadline (``MNIST_AMD_COMM_TIMEOUT``) aborts the
        communicator and raises :class:`CollectiveError` instead of hanging in hipStreamSynchronize."""
        t0 = time.perf_counter()
        if self.comm is None:
            self.stream.synchronize()
        else:
            err = self.comm.wait_stream(self.stream.cuda_stream, comm_timeout() if timeout is None else timeout)
            if err:
                detected = time.perf_counter() - t0
                self.comm.abort()  # ncclCommAbort: RCCL kernels still waiting on peers exit
                raise CollectiveError(f"rank {self.comm.rank}: RCCL collective failed: {err} (communicator aborted)",
                                      detected)
        self._check_oneshot(t0)

    def _oneshot_instances(self):
        return ([self.oneshot] if self.oneshot is not None else []) + list(self.overlap or ())

    def agree_oneshot(self, reduce_max) -> None:
        """Collective end-of-run check of the one-shot data plane: a latched failure is one-sided (a late peer that
        arrives after another rank timed out still finds every flag raised, sums and updates), so before a
        successful return every rank reports its latch over the control plane (``reduce_max``, e.g. a gloo MAX
        all-reduce) and ALL ranks raise :class:`CollectiveError` if any rank failed (advisor, round 5).  No-op
        without one-shot instances.  Collective: every rank calls it at the same point."""
        insts = self._oneshot_instances()
        if not insts:
            return
        self.stream.synchronize()
        local = next((e for e in (o.check() for o in insts) if e), "")
        if reduce_max(1.0 if local else 0.0) > 0.0:
            raise CollectiveError(local or "one-shot all-reduce failed on a peer rank (its latched error; this rank's "
                                  "parameters may differ from that rank's)")

    def _check_oneshot(self, t0: Optional[float] = None) -> None:
        """One-shot data plane: a flag wait that timed out is latched on the device (no sum written, later calls
        and the updates behind them skipped, csrc/kernels/oneshot.hip); raise it at this host wait."""
        for o in self._oneshot_instances():
            err = o.check()
            if err:
                raise CollectiveError(err, 0.0 if t0 is None else time.perf_counter() - t0)
