"""Bring-up of the one-shot xGMI all-reduce (csrc/runtime/oneshot.h, csrc/kernels/oneshot.hip).

The alternative gradient data plane to RCCL's ring (survey §5.8-3): every rank exports one uncached device
region over IPC (``hipIpcGetMemHandle``), the handles travel over the control-plane TCPStore, every rank maps
its peers' regions, and a step's all-reduce becomes ONE kernel that pushes the local slice into every peer's
slot over the point-to-point xGMI links and sums the W slots of its own region in a fixed rank order (bitwise
identical replicas).  Reference call site it replaces: the DDP bucket all-reduce of
``ddp_tutorial_multi_gpu.py:94`` (one NCCL all-reduce per step).  RCCL stays the default
(``bench.py --allreduce rccl``); ``--allreduce oneshot`` selects this one.
"""
from __future__ import annotations

import datetime
import os
from typing import Optional

import torch
import torch.distributed as dist

KEY = "mnist_amd/oneshot/{gen}/{rank}"
_GEN = [0]


def oneshot_timeout() -> float:
    """In-kernel bound of a flag wait (``MNIST_AMD_ONESHOT_TIMEOUT`` seconds, default 5): it bounds how far a
    rank may run ahead of its slowest peer inside the step loop.  A rank whose peer does not arrive in time
    LATCHES the error word (csrc/kernels/oneshot.hip): that call writes no sum, every later call does nothing,
    the parameter updates behind them are skipped, and the next host wait raises :class:`CollectiveError`
    (``NativeTrainer.synchronize`` polls ``check()``).  A few seconds, not the RCCL watchdog's 600: a kernel
    must not spin for minutes on a dead peer."""
    return float(os.environ.get("MNIST_AMD_ONESHOT_TIMEOUT", "5"))


def make_oneshot(ctx, max_count: int, nblk: int = 64, timeout_s: Optional[float] = None, init_timeout_s: float = 180.0):
    """Collective (every rank of ``ctx``): create this rank's region, exchange the IPC handles, map the peers.
    World 1 needs no exchange."""
    from ..ops.native import load_c
    C = load_c()
    dev = ctx.device.index if ctx.device.type == "cuda" and ctx.device.index is not None else torch.cuda.current_device()
    if ctx.world == 1:
        return C.OneShotAllReduce(ctx.rank, ctx.world, int(dev), int(max_count), int(nblk),
                                  oneshot_timeout() if timeout_s is None else float(timeout_s))
    _GEN[0] += 1
    store = dist.distributed_c10d._get_default_store()
    mine = KEY.format(gen=_GEN[0], rank=ctx.rank)
    try:
        o = C.OneShotAllReduce(ctx.rank, ctx.world, int(dev), int(max_count), int(nblk),
                               oneshot_timeout() if timeout_s is None else float(timeout_s))
        h = o.handle()
    except Exception:
        store.set(mine, b"")  # tell the peers at once instead of letting them wait out the deadline
        raise
    store.set(mine, h)
    keys = [KEY.format(gen=_GEN[0], rank=r) for r in range(ctx.world)]
    store.wait(keys, datetime.timedelta(seconds=init_timeout_s))
    handles = [bytes(store.get(k)) for k in keys]
    if any(not x for x in handles):
        raise RuntimeError(f"rank {ctx.rank}: a peer failed to create its one-shot region")
    err = ""
    try:
        o.open_peers(handles)
    except Exception as e:  # noqa: BLE001 -- agreed below, so every rank issues the same collectives
        err = f"rank {ctx.rank}: mapping the peers' regions failed: {e}"
    # one agreement (also the barrier: every rank has mapped every region before the first call)
    if ctx.all_reduce_sum([1.0 if err else 0.0])[0]:
        raise RuntimeError(err or "a peer failed to map the one-shot regions")
    return o


def time_oneshot(o, count: int, device, iters: int = 48, warmup: int = 8, per_graph: int = 1):
    """Latency (ms) of ONE one-shot all-reduce of ``count`` floats, as the step graph issues it: ``per_graph`` calls
    captured back to back into a graph, replayed back to back (median per call; collective -- every rank calls it).
    With one call per graph the figure is the host's graph-launch rate (~15 us), not the kernel."""
    buf = torch.zeros(count, dtype=torch.float32, device=device)
    s = torch.cuda.Stream(device=device)
    s.wait_stream(torch.cuda.current_stream(device))
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        for _ in range(max(1, per_graph)):
            o.all_reduce_sum_f32(buf.data_ptr(), count, torch.cuda.current_stream(device).cuda_stream)
    with torch.cuda.stream(s):
        for _ in range(warmup):
            g.replay()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(iters + 1)]
        ev[0].record(s)
        for i in range(iters):
            g.replay()
            ev[i + 1].record(s)
    s.synchronize()
    err = o.check()
    if err:
        raise RuntimeError(err)
    ts = sorted(ev[i].elapsed_time(ev[i + 1]) / max(1, per_graph) for i in range(iters))
    return ts[len(ts) // 2]


def validate_oneshot(ctx, o, count: int) -> str:
    """Collective correctness check of a freshly built one-shot all-reduce against the exact host sum: rank r
    contributes (r + 1) * (i % 97 + 1) / 8 at element i (exact in fp32 for W <= 8, any summation order), two
    calls (both buffer parities).  Returns "" on every rank if every rank matched, else the failures.  The
    verdict is agreed over the control plane, so all ranks take the same decision."""
    try:
        i = torch.arange(count, dtype=torch.float32, device=ctx.device) % 97 + 1
        expect = i * (ctx.world * (ctx.world + 1) / 2) / 8
        ok = True
        for _ in range(2):
            x = i * (ctx.rank + 1) / 8
            s = torch.cuda.current_stream(ctx.device)
            o.all_reduce_sum_f32(x.data_ptr(), count, s.cuda_stream)
            s.synchronize()
            ok = ok and bool(torch.equal(x, expect)) and o.check() == ""
        err = "" if ok else f"rank {ctx.rank}: one-shot all-reduce result differs from the exact sum"
    except Exception as e:  # noqa: BLE001 -- any failure disqualifies the probe
        err = f"rank {ctx.rank}: {e}"
    bad = ctx.all_reduce_sum([0.0 if not err else 1.0])[0] if ctx.world > 1 else (1.0 if err else 0.0)
    if bad:
        return err or f"{int(bad)} rank(s) failed the one-shot check"
    return ""


def probe_oneshot(ctx, max_count: int):
    """Measure-only one-shot all-reduce next to RCCL (bench.py at world > 1 with ``--allreduce rccl``): built,
    exchanged and validated, or None with the reason -- never fatal, and agreed by every rank."""
    err = ""
    o = None
    try:
        o = make_oneshot(ctx, max_count)
    except Exception as e:  # noqa: BLE001
        err = f"rank {ctx.rank}: {e}"
    failed = ctx.all_reduce_sum([1.0 if err else 0.0])[0] if ctx.world > 1 else (1.0 if err else 0.0)
    if failed:
        return None, err or "one-shot bring-up failed on another rank"
    err = validate_oneshot(ctx, o, max_count)
    return (None, err) if err else (o, "")


def attach_overlap_plan(ctx, tr, fc_inst, world: int) -> str:
    """LeNet: make the one-shot OVERLAP plan available (csrc/runtime/trainer.h Plan::OVERLAP) -- ``fc_inst`` (a
    validated one-shot instance, >= the FC range) carries the FC range on the aux stream, a second instance,
    built and validated here, the conv range on the main stream.  Collective; never fatal: returns "" or why
    the plan is unavailable (agreed by every rank)."""
    if tr.model_name != "lenet5":
        return "LeNet-only plan"
    conv, err = probe_oneshot(ctx, int(tr.rt.conv_params))
    if conv is None:
        return err
    tr.attach_overlap(fc_inst, conv, world)
    return ""


def setup_oneshot(ctx, tr, world: int, mode: str, pinned: Optional[str] = None):
    """The one-shot data plane of a trainer with an RCCL communicator attached (bench.py and the entry-script
    runner).  ``mode == "oneshot"``: the step's collectives run on a validated one-shot instance (failure is
    fatal: RuntimeError); ``"rccl"``: at world > 1, only when ``MNIST_AMD_PROBE_ONESHOT=1`` (opt-in: the one-shot
    plane has not moved a byte over real xGMI links yet, so a default multi-GPU run must not pick it up), a
    measure-only instance is probed and, when it validates, the OVERLAP plan becomes a calibration candidate.  A
    pinned ``overlap`` plan without it is fatal.  Collective.  Returns (step instance or None, probe instance or
    None, reason)."""
    oneshot = probe = None
    why = ""
    if mode == "oneshot":
        oneshot = make_oneshot(ctx, tr.nparam)
        err = validate_oneshot(ctx, oneshot, tr.nparam)  # exact-sum check, agreed by every rank
        if err:
            raise RuntimeError(f"one-shot all-reduce failed its check: {err}")
        tr.attach_oneshot(oneshot, world)
        why = attach_overlap_plan(ctx, tr, oneshot, world)
    elif world > 1 and os.environ.get("MNIST_AMD_PROBE_ONESHOT", "0") == "1":
        probe, why = probe_oneshot(ctx, tr.nparam)
        if probe is not None:
            why = attach_overlap_plan(ctx, tr, probe, world)
            why = f"overlap plan unavailable: {why}" if why else ""
    else:
        why = "not probed (MNIST_AMD_PROBE_ONESHOT=1 opts in)"
    if pinned == "overlap" and why:
        raise RuntimeError(f"--plan overlap: {why}")
    return oneshot, probe, why

