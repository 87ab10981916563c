#!/usr/bin/env python3
"""Headline benchmark: whole-node training images/sec of LeNet-5 MNIST DDP on MI355X (+ top-1).

Metric/config from BASELINE.json: "images/sec (whole node) MNIST ConvNet DDP at 1/2/4/8 MI355X;
top-1 acc", config "LeNet-5 MNIST DDP 8xMI355X large-batch 8192/GPU bf16".  Weak scaling:
8192 images per GPU per step, global batch = 8192 * N.

Each timed step is a COMPLETE data-parallel training step through the native path: gather +
normalise of the step's samples from the HBM-resident uint8 dataset, LeNet-5 forward and
backward (hand-written CDNA4 MFMA kernels, bf16 inputs / fp32 accumulate / fp32 master
weights), at N > 1 the gradient all-reduce over the native RCCL communicator (the step plan --
one coalesced all-reduce after the backward join, or the FC bucket + FC update sent beside
conv_bwd -- is chosen at start-up by timing both on the real communicator and is reported in the
JSON), and the SGD-momentum update, replayed as hipGraphs.  The reference MLP (``--model mlp``)
runs with the reference's Dropout(0.2) in the timed step.
The DistributedSampler(seed=42) order of every epoch the run touches is computed
before timing and kept in HBM (the step counter crosses epoch boundaries on the device).
Data: synthetic 28x28 uint8 images of the MNIST shape (no network), random init.

Timing: W untimed warm-up steps; then every rank passes a barrier, synchronises its device and
times exactly K steps ending with its own device synchronisation; the reported time is the MAX of
the per-rank times (one gloo max-reduction AFTER the clock stops -- no collective or barrier inside
the timed region other than the step's own gradient all-reduces).
With a communicator the JSON carries ``comm_profile``: the RCCL world, the latency of each bucket's
standalone all-reduce, and the exposed communication (step with the plan's collectives minus the
local schedule without any, interleaved replays).

Launch:
  ``python bench.py`` (1 GPU);
  ``python bench.py --gpus N`` spawns N rank processes itself (one per GPU, torchrun-style env,
  before this parent touches a GPU) and relays rank 0's JSON line;
  ``python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1
  --master-port P bench.py --gpus N --steps K --warmup W`` runs the ranks under torchrun.
  ``--comm gloo`` exchanges gradients over c10d gloo through host memory instead of RCCL; ranks may
  then share one GPU (test path: the multi-process chain on a one-GPU box).
Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import importlib.util
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec (whole node) MNIST ConvNet DDP at 1/2/4/8 MI355X; top-1 acc"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=50)
    ap.add_argument("--model", default="lenet5", choices=["lenet5", "mlp"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--batch", type=int, default=8192, help="per-GPU batch")
    ap.add_argument("--lr", type=float, default=0.05)
    ap.add_argument("--momentum", type=float, default=0.9)
    ap.add_argument("--dropout", type=float, default=None,
                    help="dropout after layer 1 (default: the reference's 0.2 for --model mlp; LeNet-5 has none)")
    ap.add_argument("--comm", default="rccl", choices=["rccl", "torch", "gloo"],
                    help="gradient data plane: native RCCL (default), c10d nccl, or c10d gloo via host memory")
    ap.add_argument("--allreduce", default="rccl", choices=["rccl", "oneshot"],
                    help="gradient data plane of the captured step: RCCL (default) or the one-shot xGMI all-reduce "
                         "(every rank pushes its slice into every peer's IPC-mapped slot, then sums its own slots in "
                         "rank order; parallel/oneshot.py).  With --comm gloo the ranks may share one GPU")
    ap.add_argument("--plan", default="auto", choices=["auto", "join", "split", "overlap", "fixed"],
                    help="step plan: auto = time the candidates at start-up and keep the fastest "
                         "(multi-GPU plans, or the single-GPU schedules); join/split = that multi-GPU plan; "
                         "overlap = LeNet, one-shot all-reduces inside the concurrent schedule's branches "
                         "(needs a validated one-shot data plane); fixed = no calibration, defaults")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--comm-world1", action="store_true",
                    help="attach a world-1 RCCL communicator (runs the multi-GPU step schedule on one GPU)")
    ap.add_argument("--data", default="synthetic", choices=["synthetic", "netcdf"],
                    help="synthetic: the split is built in host memory and uploaded; netcdf (BASELINE config 3, the "
                         "PnetCDF loader path): rank 0 writes the same split as CDF-5 files (native writer, the "
                         "notebook's layout) into --data-dir, every rank loads them through the bulk reader "
                         "(threaded pread -> pinned host memory -> hipMemcpyAsync) and the JSON reports load_s / "
                         "load_GBps; the timed steps are the same")
    ap.add_argument("--data-dir", default=None,
                    help="directory of the --data netcdf files (default: $TMPDIR/mnist_amd_bench_nc)")
    ap.add_argument("--synthetic-mode", default="hard", choices=["easy", "hard"],
                    help="synthetic data generator (hard, the default: stronger noise / affine jitter, so the top-1 "
                         "read-out carries information; easy saturates at 1.0)")
    ap.add_argument("--eval", action="store_true", default=True)
    ap.add_argument("--acc-steps", type=int, default=500,
                    help="untimed training steps after the timed region and before the top-1 read-out (so the "
                         "accuracy in the JSON is that of a trained model, not of warm-up + K steps)")
    ap.add_argument("--no-eval", dest="eval", action="store_false")
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--digest", action="store_true",
                    help="every rank prints a sha256 of its final parameters to stderr (replica consistency check)")
    ap.add_argument("--dump-params", default=None,
                    help="every rank saves its final parameter slab to PATH.rank<r>.pt (tests)")
    ap.add_argument("--rank-logs", default=None,
                    help="--gpus N self-launch: also write each rank's stderr to DIR/rank<r>.stderr")
    ap.add_argument("--dry-run", action="store_true",
                    help="check the launch wiring only: every rank validates its env, rank 0 prints a JSON line, no GPU")
    return ap.parse_args(argv)


def _launcher():
    """parallel/launch.py loaded by path: the parent must not import torch / touch a GPU."""
    spec = importlib.util.spec_from_file_location("_mnist_launch", os.path.join(ROOT, "pytorch_ddp_mnist_amd",
                                                                                 "parallel", "launch.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def spawn_ranks(a) -> int:
    """``--gpus N`` without a launcher: start N rank processes and relay rank 0's JSON line."""
    L = _launcher()
    cmd = [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]
    # crash evidence of every rank: the native backtrace of a host fault (MNIST_AMD_SEGV_TRACE), then the
    # Python stacks of every thread (faulthandler); the launcher keeps each rank's stderr separately
    env = {k: os.environ.get(k, "1") for k in ("MNIST_AMD_SEGV_TRACE", "PYTHONFAULTHANDLER")}
    rc, lines = L.launch_relay(cmd, a.gpus, style="torch", relay_rank=0, extra_env=env, log_dir=a.rank_logs,
                               timeout=float(os.environ.get("MNIST_AMD_LAUNCH_TIMEOUT", "0")))
    if rc == 0 and not any(l.lstrip().startswith("{") for l in lines):
        print("[bench] rank 0 printed no result line", file=sys.stderr)
        return 1
    if rc != 0:
        print(f"[bench] a rank failed with exit code {rc}", file=sys.stderr)
    return rc


def dry_run(a) -> int:
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    lrank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus or not (0 <= rank < world) or lrank != rank or (world > 1 and not os.environ.get("MASTER_PORT")):
        print(f"[bench] bad rank env: RANK={rank} WORLD_SIZE={world} LOCAL_RANK={lrank}", file=sys.stderr)
        return 3
    if os.environ.get("MNIST_AMD_DRYRUN_FAIL_RANK") == str(rank):
        return 7
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "n_gpus": world, "dry_run": True,
                          "master": f"{os.environ.get('MASTER_ADDR')}:{os.environ.get('MASTER_PORT')}"}), flush=True)
    return 0


def bench_data(world: int, rank: int, batch: int, total_steps: int, mode: str = "hard"):
    """The run's data: the MNIST-shaped synthetic train split (repeated so every rank has >= 8 full
    batches per epoch), the test split, and this rank's DistributedSampler(seed=42) order of every epoch
    the run touches, each cut to its full batches and laid end to end (the device step counter walks
    from one epoch straight into the next, so no index upload or counter reset sits between timed
    steps).  Deterministic: tests rebuild it to emulate the ranks in one process."""
    import numpy as np
    import torch

    from pytorch_ddp_mnist_amd.data.sampler import epoch_indices, num_samples
    from pytorch_ddp_mnist_amd.data.synthetic import make_split
    base_x, base_y = make_split(60000, seed=1, mode=mode)
    reps = max(1, -(-(world * batch * 8) // 60000))
    n = 60000 * reps
    images = np.tile(base_x.reshape(-1, 784), (reps, 1))
    labels = np.tile(base_y, reps)
    ns = num_samples(n, world)
    steps_per_epoch = ns // batch
    n_epochs = -(-total_steps // steps_per_epoch)
    idx_all = torch.cat([epoch_indices(n, world, rank, e, seed=42)[: steps_per_epoch * batch]
                         for e in range(n_epochs)]).to(torch.int32)
    test_x, test_y = make_split(10000, seed=2, mode=mode)
    return torch.from_numpy(images), torch.from_numpy(labels), idx_all, test_x, test_y


def netcdf_data(ctx, images, labels, data_dir, mode: str):
    """BASELINE config 3 (the PnetCDF loader path): rank 0 writes the run's train split as a CDF-5 file (the
    notebook's to_nc() layout, nb#c2:83-104, through the native writer), every rank then loads it through the
    bulk reader -- threaded pread straight into pinned host memory, one hipMemcpyAsync to HBM
    (data/device_loader.py upload_netcdf; reference: MNISTNetCDF + DataLoader per-sample reads,
    mnist_pnetcdf_cpu_mp.py:18-49,370-409).  Returns the device tensors and the load figures (timed on every
    rank, the max reported)."""
    import torch

    from pytorch_ddp_mnist_amd.data.cdf5 import write_mnist_nc
    from pytorch_ddp_mnist_amd.data.device_loader import upload_netcdf
    d = data_dir or os.path.join(os.environ.get("TMPDIR", "/tmp"), "mnist_amd_bench_nc")
    path = os.path.join(d, f"mnist_train_images_{images.shape[0]}_{mode}.nc")
    if ctx.rank == 0:
        os.makedirs(d, exist_ok=True)
        t0 = time.perf_counter()
        tmp = f"{path}.tmp{os.getpid()}"
        write_mnist_nc(tmp, images.numpy().reshape(-1, 28, 28), labels.numpy())
        os.replace(tmp, path)
        write_s = time.perf_counter() - t0
    else:
        write_s = 0.0
    ctx.barrier()
    sync = (lambda: torch.cuda.synchronize(ctx.device)) if ctx.device.type == "cuda" else (lambda: None)
    sync()
    t0 = time.perf_counter()
    dx, dy = upload_netcdf(path, ctx.device)
    sync()
    load_s = ctx.all_reduce_max(time.perf_counter() - t0)
    if dx.shape[0] != images.shape[0]:
        raise RuntimeError(f"{path}: {dx.shape[0]} rows, expected {images.shape[0]}")
    nbytes = dx.numel() + dy.numel()
    info = {"source": "netCDF CDF-5 (native writer) -> threaded pread -> pinned -> hipMemcpyAsync",
            "file": path, "rows": int(dx.shape[0]), "bytes": int(nbytes), "write_s": round(write_s, 4),
            "load_s": round(load_s, 4), "load_GBps": round(nbytes / max(load_s, 1e-9) / 1e9, 3)}
    return dx, dy, info


def timed_region(ctx, tr, run, steps: int, cuda_sync, clock=time.perf_counter) -> float:
    """Time exactly ``steps`` steps on every rank; returns the max over ranks (seconds).

    A barrier + device sync puts every rank at the start line; each rank's clock stops after its own
    stream drained (the trainer's synchronize() is the collective watchdog with a communicator).  The
    rank-max reduction runs after both clock reads: nothing but the steps themselves (and their
    gradient all-reduces) is inside the timed region."""
    tr.synchronize()
    ctx.barrier()
    cuda_sync()
    t0 = clock()
    run(steps)
    tr.synchronize()
    cuda_sync()
    t1 = clock()
    return ctx.all_reduce_max(t1 - t0)


def main(argv=None) -> int:
    a = parse(argv)
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return spawn_ranks(a)
    if a.dry_run:
        return dry_run(a)

    import torch

    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer, resolve_plan
    from pytorch_ddp_mnist_amd.models import build_model
    from pytorch_ddp_mnist_amd.parallel.comm import init_distributed
    from pytorch_ddp_mnist_amd.parallel.ddp import model_phases, plan_buckets

    pinned = resolve_plan(a.plan)   # validates --plan before any device work
    dropout = a.dropout if a.dropout is not None else (0.2 if a.model == "mlp" else 0.0)
    if a.model == "lenet5" and dropout:
        raise SystemExit("LeNet-5 has no dropout layer")
    world_env = int(os.environ.get("WORLD_SIZE", "1"))
    from pytorch_ddp_mnist_amd.parallel.comm import CommInitError
    try:
        ctx = init_distributed(None, parallel=world_env > 1, device="cuda", comm=a.comm,
                               share_device=a.comm == "gloo")
    except CommInitError as e:
        # bounded RCCL bring-up failed (MNIST_AMD_COMM_INIT_TIMEOUT): name the rank and leave at once -- the
        # launcher tears the other ranks down; no interpreter teardown that could wait on the dead peers
        print(f"[bench] {e}", file=sys.stderr, flush=True)
        os._exit(3)
    if ctx.world != a.gpus and ctx.rank == 0:
        print(f"[bench] note: --gpus {a.gpus} but WORLD_SIZE={ctx.world}; using {ctx.world}", file=sys.stderr)
    W, rank, dev = ctx.world, ctx.rank, ctx.device

    acc_steps = max(0, a.acc_steps) if a.eval else 0
    images, labels, idx_all, test_x, test_y = bench_data(W, rank, a.batch, a.warmup + a.steps + acc_steps,
                                                         a.synthetic_mode)
    load = None
    if a.data == "netcdf":
        images, labels, load = netcdf_data(ctx, images, labels, a.data_dir, a.synthetic_mode)
    else:
        images, labels = images.to(dev), labels.to(dev)

    torch.manual_seed(0)
    tr = NativeTrainer(a.model, a.dtype, a.batch, images, labels, device=dev, lr=a.lr,
                       momentum=a.momentum, dropout=dropout, init=build_model(a.model), max_indices=idx_all.numel())
    tr.set_buckets(plan_buckets(model_phases(a.model)))
    tr.set_epoch_indices(idx_all)
    comm, rccl_version, tune, prof = None, None, None, None
    oneshot, probe, probe_err = None, None, None
    if a.allreduce == "oneshot" and a.comm == "torch":
        raise SystemExit("--allreduce oneshot needs --comm rccl (RCCL kept for broadcast / comparison) or gloo")
    external = a.comm in ("torch", "gloo") and W > 1 and a.allreduce != "oneshot"
    if external:
        import torch.distributed as dist
        if a.comm == "gloo":
            p = tr.params.cpu()
            dist.broadcast(p, 0)
            tr.load_flat(p)
        else:
            dist.broadcast(tr.params, 0)
            tr.load_flat(tr.params.clone())
        tr.attach_external_allreduce(lambda t: dist.all_reduce(t), W, host=a.comm == "gloo")
    elif (W > 1 or a.comm_world1) and a.comm == "rccl":
        from pytorch_ddp_mnist_amd.ops.native import load_c
        C = load_c()
        comm = ctx.rccl
        if comm is None:  # --comm-world1: a world-1 RCCL communicator, no rendezvous needed
            from pytorch_ddp_mnist_amd.utils.logging import native_stdout_to_stderr
            with native_stdout_to_stderr():  # RCCL's init banner must not reach the JSON stdout
                comm = C.RcclComm(bytes(C.RcclComm.make_unique_id()), 0, 1, ctx.local_rank)
        rccl_version = C.rccl_version()
        tr.attach_comm(comm, W)
    elif a.comm_world1:
        raise SystemExit("--comm-world1 needs --comm rccl")
    if not external and (a.allreduce == "oneshot" or comm is not None):
        # the one-shot data plane, exactly as the entry scripts set it up (parallel/oneshot.py setup_oneshot):
        # --allreduce oneshot = the step's collectives (validated against the exact sum; RCCL, when attached,
        # broadcasts and is timed for comparison); with RCCL at world > 1 an opt-in measure-only probe
        from pytorch_ddp_mnist_amd.parallel.oneshot import setup_oneshot
        try:
            oneshot, probe, probe_err = setup_oneshot(ctx, tr, W, a.allreduce, pinned)
        except RuntimeError as e:
            raise SystemExit(f"[bench] {e}")
    if comm is not None or oneshot is not None:
        tr.broadcast_params(0)  # over RCCL, or over the c10d control plane with only the one-shot plane
        if pinned is not None:
            tr.set_plan(pinned)

    use_graph = not a.no_graph and not external
    # start-up schedule calibration (multi-GPU plan on the communicator, or the single-GPU
    # schedule): interleaved captured-step replays per candidate, state restored, choice in the JSON.
    # With an external data plane the step is not a graph: the local schedules are still timed (rank-max)
    if a.plan == "auto" and use_graph:
        tune = tr.autotune_plan(reduce_max=ctx.all_reduce_max)
    elif a.plan == "auto" and external:
        # the external data plane runs the eager phase API (forward_backward -> host all-reduce -> SGD), not
        # the captured schedules a calibration would time: nothing to choose
        tune = {"chosen": "eager-phases", "timings_ms": {}, "note": "external data plane: no graph schedules"}
    if (comm is not None or oneshot is not None) and use_graph:
        prof = tr.comm_profile(reduce_max=ctx.all_reduce_max, tune=tune, probe=probe)
        if oneshot is None and W > 1:
            prof["oneshot_probe"] = "validated (measure-only)" if probe is not None else (probe_err or "not probed")

    def run(n):
        tr.run_steps(n, use_graph=use_graph)  # k-step graphs (MNIST_AMD_GRAPH_STEPS), then single steps

    if use_graph:
        # capture + instantiate the 1-step and k-step graphs before the clock.  (A graph of the timed run's
        # remainder -- 20 steps = 8 + 8 + one 4-step graph -- measured SLOWER than 4 single-step launches,
        # 0.118-0.132 vs 0.110-0.113 ms/step even when the warm-up launched it first: not used.)
        tr.prepare_graphs()
    tr.reset_metrics()
    run(a.warmup)
    elapsed = timed_region(ctx, tr, run, a.steps, lambda: torch.cuda.synchronize(dev))
    train = tr.read_metrics()
    tr.check_comm()

    top1 = None
    if a.eval:
        if acc_steps:
            run(acc_steps)  # untimed: the model the top-1 describes has trained warm-up + K + acc_steps steps
        ev = tr.evaluate(torch.from_numpy(test_x.reshape(-1, 784)), torch.from_numpy(test_y),
                         torch.arange(10000, dtype=torch.int32))
        top1 = ev.accuracy

    n_gpus = comm.world if comm is not None else W
    info = tr.plan_info()
    if oneshot is not None or info["plan"] == "overlap":
        colls = " + ".join(f"{c['bytes'] // 1024} KiB" for c in info["collectives"])
        where = " inside the backward branches" if info["plan"] == "overlap" else ""
        comm_desc = (f"one-shot xGMI all-reduce (IPC peer slots, fixed rank order){where}, plan={info['plan']}: "
                     f"{colls} per step" + (f" (RCCL {rccl_version} attached: broadcast, comparison)" if comm else ""))
    elif comm is not None:
        colls = " + ".join(f"{c['bytes'] // 1024} KiB" for c in info["collectives"])
        comm_desc = f"native RCCL {rccl_version}, plan={info['plan']}: all-reduce {colls} per step"
    elif external:
        comm_desc = ("c10d gloo all_reduce of the grad slab via pinned host memory" if a.comm == "gloo"
                     else "c10d nccl (RCCL) all_reduce of the whole grad slab")
    else:
        comm_desc = "none (single process, no gradient exchange)"
    ms = elapsed / a.steps * 1e3
    value = n_gpus * a.batch * a.steps / elapsed
    from pytorch_ddp_mnist_amd.ops.native import load_c as _load_c
    from pytorch_ddp_mnist_amd.ops.precision import dtype_label, fp32_products
    split = getattr(_load_c(), "F32_SPLIT", 0) if a.dtype == "fp32" else 0
    out = {
        "metric": METRIC,
        "value": round(value, 1),
        "unit": "images/s",
        "n_gpus": n_gpus,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        # fp32: which products run as exact 3-part bf16 splits (ops/precision.py; every one with the opt-in
        # MNIST_AMD_F32_SPLIT build) -- config.fp32_products lists both kinds
        "dtype": dtype_label(a.dtype, a.model, a.batch, split),
        "data": f"synthetic (MNIST-shaped 28x28 uint8, class-template + noise, mode={a.synthetic_mode}; "
                "random-init weights)" + ("; loaded from a CDF-5 netCDF file" if load else ""),
        "config": {
            "model": "LeNet-5" if a.model == "lenet5" else "MLP-784-128-128-10",
            "global_batch": n_gpus * a.batch,
            "per_gpu_batch": a.batch,
            "seq_len": None,
            "image_shape": [1, 28, 28],
            "parallelism": f"dp{n_gpus}",
            "optimizer": f"SGD(lr={a.lr}, momentum={a.momentum})",
            "dropout": dropout,
            "comm": comm_desc,
            "plan": info,
            "plan_autotune": tune,
            "hipgraph": use_graph,
            **({"fp32_products": fp32_products(a.model, a.batch, split)} if a.dtype == "fp32" else {}),
        },
        "rccl_world": comm.world if comm is not None else None,
        "allreduce": "oneshot" if oneshot is not None else ("rccl" if comm is not None else None),
        "input": load or {"source": "in-memory synthetic split -> HBM (one copy)"},
        "comm_profile": prof,
        "top1": None if top1 is None else round(top1, 4),
        # what the top-1 above measures: the 10000-image synthetic test split after warm-up + timed steps
        "top1_eval": None if top1 is None else {
            "split": f"synthetic test (10000, mode={a.synthetic_mode})",
            "steps_trained": a.warmup + a.steps + acc_steps,
            "untimed_steps_after_timing": acc_steps,
            "epochs_trained": round((a.warmup + a.steps + acc_steps) * a.batch * n_gpus / 60000, 2)},
        "train_loss_mean": round(train.mean_loss, 4),
    }
    if n_gpus > 1:
        tr.agree_oneshot(ctx.all_reduce_max)  # one-shot data plane: every rank raises if any rank latched a failure
    if a.digest or a.dump_params:
        tr.synchronize()
        p = tr.params.detach().cpu()
        if a.digest:
            import hashlib
            print(f"digest rank={rank} {hashlib.sha256(p.numpy().tobytes()).hexdigest()}", file=sys.stderr, flush=True)
        if a.dump_params:
            torch.save(p, f"{a.dump_params}.rank{rank}.pt")
    if rank == 0:
        line = json.dumps(out)
        print(line, flush=True)
        if a.json_out:
            with open(a.json_out, "w") as f:
                f.write(line + "\n")
    ctx.finalize(tr)
    return 0


if __name__ == "__main__":
    sys.exit(main())
