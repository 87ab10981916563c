"""Epoch driver shared by every entry script.

``run(cfg, entry)`` = the reference's ``__main__`` blocks + ``main()`` re-designed once:
wire-up -> data (idx / netCDF / synthetic) -> engine (native MI355X trainer on a GPU, torch-CPU
reference loop otherwise) -> per epoch {DistributedSampler-equivalent order, train, full test-set
eval, reference epoch line} -> rank-0 ``model.pt``.
"""
from __future__ import annotations

import os
import time
from typing import Optional, Tuple

import numpy as np
import torch

from ..config import TrainConfig
from ..data.datasets import find_netcdf, load_arrays, synthesize_netcdf
from ..data.device_loader import upload_netcdf
from ..data.per_sample import InterleavedLoader, PerSampleReader
from ..data.sampler import epoch_indices
from ..models import build_model
from ..parallel.comm import DistContext, init_distributed
from ..parallel.ddp import model_phases, plan_buckets
from ..utils.checkpoint import load_resume, save_model, save_resume
from ..utils.fault import FaultInjector, check_finite
from ..utils.logging import MetricsWriter, ProgressBar, banner, epoch_line, reference_epoch_loss
from ..utils.profiling import PhaseTimer, enable as enable_roctx, range_
from .reference import EpochResult, TorchCPUEngine


class NativeEngine:
    """Adapter of :class:`NativeTrainer` to the epoch driver (GPU path)."""
    name = "native-hip"

    def __init__(self, cfg: TrainConfig, ctx: DistContext, xtr, ytr, xte, yte, init: torch.nn.Module):
        from ..data.device_loader import upload_arrays
        from .native import NativeTrainer, resolve_plan
        dev = ctx.device

        def on_device(x, y):  # numpy arrays are staged (pinned -> async copy); device tensors used as is
            if isinstance(x, torch.Tensor) and x.device.type == "cuda":
                return x.view(-1, 784), y.view(-1)
            return upload_arrays(x, y, dev)
        images, labels = on_device(xtr, ytr)
        self.test_images, self.test_labels = on_device(xte, yte)
        self.batch = cfg.batch_size
        self.cfg, self.ctx = cfg, ctx
        self.tr = NativeTrainer(cfg.model, cfg.dtype, cfg.batch_size, images, labels, device=dev, lr=cfg.lr,
                                momentum=cfg.momentum, dropout=cfg.dropout if cfg.model == "mlp" else 0.0,
                                seed=cfg.seed * 7919 + ctx.rank, init=init)
        cap = None if cfg.bucket_cap_kb is None else cfg.bucket_cap_kb * 1024
        self.tr.set_buckets(plan_buckets(model_phases(cfg.model), cap))
        self.torch_comm = ctx.world > 1 and ctx.rccl is None
        self.plan_pinned = cfg.plan != "auto"
        self.plan_forced = resolve_plan(cfg.plan)  # 'fixed' = no calibration, default join plan
        if cfg.allreduce == "oneshot" and not (ctx.world > 1 and ctx.rccl is not None):
            raise SystemExit("--allreduce oneshot needs world > 1 and the native RCCL communicator (--comm rccl)")
        self.oneshot_note = None
        if ctx.world > 1 and ctx.rccl is not None:
            self.tr.attach_comm(ctx.rccl, ctx.world)
            self.tr.broadcast_params(0)
            # one-shot data plane (--allreduce oneshot), or a validated measure-only probe that makes the LeNet
            # OVERLAP plan a calibration candidate (parallel/oneshot.py setup_oneshot; collective)
            from ..parallel.oneshot import setup_oneshot
            try:
                _, _, why = setup_oneshot(ctx, self.tr, ctx.world, cfg.allreduce,
                                          self.plan_forced if self.plan_pinned else None)
            except RuntimeError as e:
                raise SystemExit(f"[rank{ctx.rank}] {e}") from e
            self.oneshot_note = why or "available"
        elif self.torch_comm:
            # c10d data plane: the all-reduce is enqueued behind the backward on the trainer stream and the
            # SGD kernel that follows on the same stream waits for it (c10d makes the current stream wait);
            # a gloo-only group stages the slab through pinned host memory
            import torch.distributed as dist
            host = dist.get_backend() == "gloo"
            p = self.tr.params.cpu() if host else self.tr.params
            dist.broadcast(p, 0)
            self.tr.load_flat(p.clone())
            self.tr.attach_external_allreduce(lambda t: dist.all_reduce(t), ctx.world, host=host)
        self.use_graph = cfg.graph and not self.torch_comm
        self.fault = FaultInjector(ctx.rank)
        self.tuned = not self.use_graph  # the calibration times captured steps
        self.tune = None

    def _load_rows(self, dst_x: torch.Tensor, dst_y: torch.Tensor, x: np.ndarray, y: np.ndarray) -> None:
        """Per-sample I/O mode: this epoch's rows replace the resident data (stream-ordered after the
        steps that read the previous contents)."""
        n = len(y)
        hx = torch.from_numpy(np.ascontiguousarray(x).reshape(n, 784)).pin_memory()
        hy = torch.from_numpy(np.ascontiguousarray(y).reshape(n)).pin_memory()
        with torch.cuda.stream(self.tr.stream):
            dst_x[:n].copy_(hx, non_blocking=True)
            dst_y[:n].copy_(hy, non_blocking=True)
        self._staged = (hx, hy)  # alive until the copy has run (the epoch ends with a sync)

    def load_train_arrays(self, x: np.ndarray, y: np.ndarray) -> None:
        self._load_rows(self.tr.images, self.tr.labels, x, y)

    def write_train_rows(self, x: np.ndarray, y: np.ndarray, row0: int) -> None:
        """Interleaved I/O: one batch's rows -> resident rows [row0, row0+b), through a two-slot pinned ring
        (a slot is refilled only after its previous copy ran: the host read of batch j+1 overlaps step j)."""
        b = len(y)
        if not hasattr(self, "_ring"):
            self._ring = [(torch.empty(self.batch, 784, dtype=torch.uint8, pin_memory=True),
                           torch.empty(self.batch, dtype=torch.uint8, pin_memory=True), torch.cuda.Event())
                          for _ in range(2)]
            self._slot = 0
        hx, hy, ev = self._ring[self._slot]
        self._slot ^= 1
        ev.synchronize()
        hx[:b].copy_(torch.from_numpy(np.ascontiguousarray(x).reshape(b, 784)))
        hy[:b].copy_(torch.from_numpy(np.ascontiguousarray(y).reshape(b)))
        with torch.cuda.stream(self.tr.stream):
            self.tr.images[row0:row0 + b].copy_(hx[:b], non_blocking=True)
            self.tr.labels[row0:row0 + b].copy_(hy[:b], non_blocking=True)
            ev.record(self.tr.stream)

    def load_test_arrays(self, x: np.ndarray, y: np.ndarray) -> None:
        self._load_rows(self.test_images, self.test_labels, x, y)

    def get_state(self):
        self.tr.synchronize()
        return (self.tr.params.detach().cpu().clone(), self.tr.mom.detach().cpu().clone(),
                int(self.tr.step_ctr[1].item()))

    def set_state(self, params: torch.Tensor, mom, global_step: int = 0) -> None:
        self.tr.load_flat(params)
        with torch.cuda.stream(self.tr.stream):  # ordered before the next step on the trainer stream
            if mom is not None:
                self.tr.mom.copy_(mom.to(self.tr.mom.device), non_blocking=True)
            self.tr.step_ctr[1].fill_(int(global_step))  # dropout stream continues, not replayed
        self.tr.synchronize()

    def _step(self, b: int) -> None:
        self.fault.tick()
        self.tr.step(b, use_graph=self.use_graph)

    def _maybe_tune(self, nfull: int) -> None:
        """First epoch: pick the step schedule by timing the candidates (multi-GPU plans on the
        communicator, or the single-GPU schedules)."""
        if self.tuned or nfull < 2:
            return
        self.tuned = True
        if self.plan_pinned:
            if self.tr.comm is not None:
                self.tr.set_plan(self.plan_forced)
            return
        self.tune = self.tr.autotune_plan(reduce_max=self.ctx.all_reduce_max)
        if self.ctx.rank == 0:
            print(f"[rank0] step plan: {self.tune['chosen']} (ms/step {self.tune['timings_ms']})", flush=True)

    def _window_loss(self, prev: float, steps: int, B: int) -> Tuple[float, float]:
        cur = self.tr.read_metrics().loss_sum
        return cur, (cur - prev) / max(1, steps * B)

    def train_epoch(self, indices: torch.Tensor, progress=None, prefetch=None, batch_loader=None) -> EpochResult:
        """``prefetch`` (optional) runs on the host while the epoch's steps execute on the GPU: the
        next epoch's sampler order is ready when this one ends (no host gap between epochs).
        ``progress`` (optional, --tqdm) gets the mean batch loss of the last ``progress.every``
        batches; reading it is a device sync, so it happens only every ``every`` steps.
        ``batch_loader(s, b)`` (optional, interleaved I/O) is called before the step on rows [s, s+b)."""
        tr, B = self.tr, self.batch
        r = EpochResult()
        t0 = time.perf_counter()
        tr.set_epoch_indices(indices)
        n = indices.numel()
        nfull, last = divmod(n, B)
        nsteps = nfull + (1 if last else 0)

        def load(j):  # interleaved I/O, one batch AHEAD of the step that trains on it: the small-batch MLP
            if batch_loader is not None and j < nsteps:  # head gathers the next step's rows during this one
                batch_loader(j * B, min(B, n - j * B))
        if batch_loader is not None:
            load(0)
            load(1)
            tr.rt.prime_next(tr.stream.cuda_stream)  # look-ahead rows of step 0, now that they are resident
        self._maybe_tune(nfull)
        tr.reset_metrics()
        every = getattr(progress, "every", 0) if progress is not None else 0
        prev = 0.0
        with range_("train_full_batches"):
            if not every and not self.torch_comm and not self.fault.active and batch_loader is None:
                if self.use_graph:
                    tr.prepare_graphs()
                tr.run_steps(nfull, use_graph=self.use_graph)   # k-step graph launches
                self.fault.step += nfull
                nfull_loop = 0
            else:
                nfull_loop = nfull
            for i in range(nfull_loop):
                self._step(B)
                load(i + 2)
                if every and ((i + 1) % every == 0 or i + 1 == nfull):
                    k = (i % every) + 1
                    prev, bl = self._window_loss(prev, k, B)
                    progress(bl, k)
        if prefetch is not None:
            r.next_indices = prefetch()
        m = tr.read_metrics()
        r.full_sum, r.n_full = m.loss_sum, nfull
        if last:
            self._step(last)
            m2 = tr.read_metrics()
            r.last_sum, r.last_b = m2.loss_sum - m.loss_sum, last
            m = m2
            if every:
                progress(r.last_sum / last, 1)
        tr.synchronize()
        tr.check_comm()
        r.loss_sum, r.correct, r.count = m.loss_sum, m.correct, m.count
        r.seconds, r.steps = time.perf_counter() - t0, nfull + (1 if last else 0)
        return r

    def evaluate(self, indices: torch.Tensor, progress=None) -> EpochResult:
        tr, B = self.tr, self.batch
        r = EpochResult()
        idx = indices.to(self.ctx.device, torch.int32).contiguous()
        with torch.cuda.stream(tr.stream):
            tr.eval_metrics.zero_()
        n = idx.numel()
        nfull, last = divmod(n, B)

        def run(s, b):
            tr.rt.eval_batch(self.test_images.data_ptr(), self.test_labels.data_ptr(), idx.data_ptr() + 4 * s, b,
                             tr.eval_metrics.data_ptr(), tr.stream.cuda_stream)
        every = getattr(progress, "every", 0) if progress is not None else 0
        prev = 0.0
        for i in range(nfull):
            run(i * B, B)
            if every and ((i + 1) % every == 0 or i + 1 == nfull):
                k = (i % every) + 1
                cur = tr.read_metrics("eval").loss_sum
                progress((cur - prev) / (k * B), k)
                prev = cur
        m = tr.read_metrics("eval")
        r.full_sum, r.n_full = m.loss_sum, nfull
        if last:
            run(nfull * B, last)
            m2 = tr.read_metrics("eval")
            r.last_sum, r.last_b = m2.loss_sum - m.loss_sum, last
            m = m2
            if every:
                progress(r.last_sum / last, 1)
        r.loss_sum, r.correct, r.count = m.loss_sum, m.correct, m.count
        return r

    def state_dict(self):
        return self.tr.state_dict()

    def finish(self) -> None:
        self.tr.synchronize()


def _uses_oneshot(engine) -> bool:
    """A one-shot xGMI all-reduce plane (data plane or the OVERLAP plan's instances) is attached."""
    tr = getattr(engine, "tr", None)
    return getattr(tr, "oneshot", None) is not None or getattr(tr, "overlap", None) is not None


def make_engine(cfg: TrainConfig, ctx: DistContext, xtr, ytr, xte, yte):
    if cfg.init_seed is not None:
        torch.manual_seed(cfg.init_seed)
    init = build_model(cfg.model)
    if ctx.device.type == "cuda":
        return NativeEngine(cfg, ctx, xtr, ytr, xte, yte, init)
    return TorchCPUEngine(cfg.model, cfg.batch_size, cfg.lr, cfg.momentum, cfg.dropout, xtr, ytr, xte, yte,
                          world=ctx.world, bucket_cap_kb=cfg.bucket_cap_kb, init=init)


def _data_format(cfg: TrainConfig, entry: str) -> str:
    if cfg.data_format != "auto":
        return cfg.data_format
    return "netcdf" if "pnetcdf" in entry else "idx"


def run(cfg: TrainConfig, entry: str = "ddp_tutorial_cpu", show_banner: bool = False,
        ctx: Optional[DistContext] = None) -> dict:
    if cfg.profile:
        enable_roctx(True)
    own_ctx = ctx is None
    if ctx is None:
        world_env = int(os.environ.get("WORLD_SIZE", "1"))
        parallel = cfg.parallel or world_env > 1
        method = cfg.wireup_method if (cfg.parallel and entry.startswith("mnist_")) else None
        # The method only decides how rank/world/master are derived from the launcher env; the
        # backend follows the device: no GPU -> gloo (the reference forces "gloo" here, which
        # also drops the SLURM/PMI variables: mnist_cpu_mp.py:247-249 -- we keep them).
        ctx = init_distributed(method, parallel=parallel, device=cfg.device, comm=cfg.comm,
                               share_device=cfg.comm == "gloo")
    fmt = _data_format(cfg, entry)
    root = cfg.data_path if cfg.data_path else ("." if fmt == "netcdf" else "./mnist_data")
    per_sample = cfg.io_mode in ("per_sample", "interleaved")
    if per_sample and fmt != "netcdf":
        raise ValueError(f"--io_mode {cfg.io_mode} is the netCDF read-cost experiment: use it with the netCDF format")
    if fmt == "netcdf" and ctx.rank == 0:
        print("=> Reading NetCDF File...")
    # rank 0 creates missing files first, the others wait, then every rank reads
    direct_nc = fmt == "netcdf" and ctx.device.type == "cuda" and cfg.io_mode == "bulk"
    if fmt == "netcdf" and (direct_nc or per_sample):
        if ctx.rank == 0 and find_netcdf(root) is None:
            synthesize_netcdf(root, verbose=True)
        ctx.barrier()
        paths = find_netcdf(root)
        if per_sample:
            readers = (PerSampleReader(root, True), PerSampleReader(root, False))
            n_tr = len(readers[0]) if cfg.data_limit is None else min(len(readers[0]), int(cfg.data_limit))
            xtr, ytr = np.zeros((n_tr, 28, 28), np.uint8), np.zeros(n_tr, np.uint8)
            xte, yte = np.zeros((len(readers[1]), 28, 28), np.uint8), np.zeros(len(readers[1]), np.uint8)
            src = f"netCDF CDF-5 ({paths['train']}), per-sample reads"
        else:  # file -> pinned host memory (threaded pread) -> HBM, no intermediate numpy copy
            xtr, ytr = upload_netcdf(paths["train"], ctx.device, cfg.data_limit)
            xte, yte = upload_netcdf(paths["test"], ctx.device)
            src = f"netCDF CDF-5 ({paths['train']}), pread -> pinned -> HBM"
    else:
        if ctx.rank == 0:
            xtr, ytr, xte, yte, src = load_arrays(fmt, root, cfg.data_limit, create=True, verbose=True)
        ctx.barrier()
        if ctx.rank != 0:
            xtr, ytr, xte, yte, src = load_arrays(fmt, root, cfg.data_limit, create=False, verbose=False)
    if fmt == "netcdf" and ctx.rank == 0:
        print("=> Dataset created, image nc file is : {}".format(os.path.join(root, "mnist_train_images.nc")))
    n_gpus = torch.cuda.device_count() if ctx.device.type == "cuda" else 0
    engine = make_engine(cfg, ctx, xtr, ytr, xte, yte)
    if show_banner:
        banner(ctx.rank, ctx.world, n_gpus, ctx.device, src, cfg.num_workers, cfg.n_epochs, cfg.parallel,
               cfg.model, cfg.dtype if ctx.device.type == "cuda" else "fp32", engine.name)
    metrics = MetricsWriter(cfg.metrics_jsonl, ctx.rank)
    ntest = len(yte)
    history = []
    start = 0
    if cfg.resume and os.path.exists(cfg.resume):
        st = load_resume(cfg.resume)
        if st.get("model") != cfg.model:
            raise ValueError(f"resume file {cfg.resume} holds a {st.get('model')} model, not {cfg.model}")
        engine.set_state(st["params"], st.get("momentum"), int(st.get("global_step", 0)))
        start = int(st["epoch"]) + 1
        if ctx.rank == 0:
            print(f"=> resumed from {cfg.resume} after epoch {st['epoch']}", flush=True)
    timer = PhaseTimer(sync=engine.finish)
    idx = None
    for i in range(start, cfg.n_epochs):
        if idx is None:
            idx = epoch_indices(len(ytr), ctx.world, ctx.rank, i, cfg.seed)
        nxt = None
        if i + 1 < cfg.n_epochs:
            nxt = lambda e=i + 1: epoch_indices(len(ytr), ctx.world, ctx.rank, e, cfg.seed)  # noqa: E731
        io = {}
        order = idx
        if cfg.io_mode == "per_sample":  # read this epoch's samples one __getitem__ at a time
            x_ep, y_ep, st = readers[0].read(idx)
            engine.load_train_arrays(x_ep, y_ep)
            order = torch.arange(len(y_ep))
            io["train"] = st
        loader = None
        if cfg.io_mode == "interleaved":  # each batch read right before its step (reference num_workers=0 loop)
            loader = InterleavedLoader(readers[0], idx, engine.write_train_rows)
            order = torch.arange(len(idx))
        bar = ProgressBar.make(cfg, ctx.rank, len(order), "training")
        if ctx.world > 1 and _uses_oneshot(engine):
            # the one-shot data plane's flag waits are bounded (MNIST_AMD_ONESHOT_TIMEOUT, 5 s) and a timeout is
            # latched as fatal: per-rank host work before the epoch (per-sample reads, rank 0's resume save) must not
            # put one rank's first collective that far ahead of another's (advisor, round 5)
            ctx.barrier()
        with range_(f"epoch{i}.train"), timer("train"):
            tr = engine.train_epoch(order, progress=bar, prefetch=nxt, batch_loader=loader)
        if loader is not None:
            io["train"] = loader.stats
        if bar is not None:
            bar.close()
        idx = tr.next_indices
        if cfg.shard_eval and ctx.world > 1:
            tidx = torch.arange(ctx.rank, ntest, ctx.world)
        else:
            tidx = torch.arange(ntest)
        if cfg.io_mode in ("per_sample", "interleaved"):
            x_te, y_te, st = readers[1].read(tidx)
            engine.load_test_arrays(x_te, y_te)
            tidx = torch.arange(len(y_te))
            io["test"] = st
        bar = ProgressBar.make(cfg, ctx.rank, len(tidx), "validation")
        with range_(f"epoch{i}.eval"), timer("eval"):
            ev = engine.evaluate(tidx, progress=bar)
        if bar is not None:
            bar.close()
        check_finite(f"epoch {i} training loss", tr.loss_sum)
        train_loss = reference_epoch_loss(tr.full_sum, tr.n_full, cfg.batch_size, tr.last_sum, tr.last_b)
        val_loss = reference_epoch_loss(ev.full_sum, ev.n_full, cfg.batch_size, ev.last_sum, ev.last_b)
        print(epoch_line(i, train_loss, val_loss), flush=True)
        g = ctx.all_reduce_sum([tr.loss_sum, tr.correct, tr.count, ev.loss_sum, ev.correct, ev.count])
        secs = ctx.all_reduce_max(tr.seconds)
        ips = g[2] / secs if secs > 0 else 0.0
        rec = dict(epoch=i, train_loss_mean=g[0] / max(g[2], 1), train_acc=g[1] / max(g[2], 1),
                   val_loss_mean=g[3] / max(g[5], 1), val_acc=g[4] / max(g[5], 1), images_per_sec=ips,
                   epoch_seconds=secs, world=ctx.world, engine=engine.name)
        for k, st in io.items():
            rec[f"io_{k}_MBps"], rec[f"io_{k}_samples_per_s"] = st.mb_per_s, st.samples_per_s
            if ctx.rank == 0:
                print("[rank0] per-sample netCDF " + st.line(k), flush=True)
        history.append(rec)
        if ctx.rank == 0:
            print(f"[rank0] epoch={i} global_train_loss={rec['train_loss_mean']:.4f} train_acc={rec['train_acc']:.4f} "
                  f"val_loss={rec['val_loss_mean']:.4f} val_acc={rec['val_acc']:.4f} "
                  f"images/s={ips:,.0f} ({engine.name}, world={ctx.world})", flush=True)
        metrics.write(**rec)
        if cfg.profile and ctx.rank == 0:
            print("[rank0] phase seconds: " + ", ".join(f"{k}={v:.4f}" for k, v in timer.summary().items()), flush=True)
        if cfg.resume:
            params, mom, gstep = engine.get_state()  # every rank holds the same replica
            if ctx.rank == 0:
                save_resume(cfg.resume, params, mom, i, cfg.model, cfg.dtype, global_step=gstep)
    engine.finish()
    if ctx.world > 1 and _uses_oneshot(engine):
        engine.tr.agree_oneshot(ctx.all_reduce_max)  # every rank raises if any rank latched a one-shot failure
    sd = engine.state_dict()
    if ctx.rank == 0 and cfg.save_path:
        save_model(sd, cfg.save_path)
    metrics.close()
    if own_ctx:
        ctx.finalize(getattr(engine, "tr", None))  # trainer graphs -> RCCL communicator -> process group
    return {"history": history, "state_dict": sd, "rank": ctx.rank, "world": ctx.world}
