"""The multi-process chain of bench.py on ONE GPU, and its communication report.

RCCL refuses two ranks on one device, but nothing else in the multi-GPU chain needs two GPUs:
``bench.py --gpus 2 --comm gloo`` self-launches two rank processes that share the GPU, rendezvous over
the TCPStore, broadcast rank 0's parameters and train on their
DistributedSampler shards with the gradient slab summed by c10d gloo through pinned host memory.
Both replicas must end bitwise identical, and equal to the same two shards trained by two trainers in
ONE process whose gradients are summed on the host (the DDP arithmetic, reference
ddp_tutorial_multi_gpu.py:72,94 / train_multi_gpu.sh:3).
"""
import json
import os
import re
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, timeout=540, log_dir=None):
    """Run bench.py in a subprocess.  The pytest process drains its own device work first (nothing of ours
    runs beside the ranks), the ranks carry the crash tracers (native backtrace + faulthandler, bench.py
    spawn_ranks), the launcher bounds the whole job below ``timeout`` and terminates every rank on its way
    out, and a failure reports each rank's exit status and stderr tail (``log_dir``: full per-rank logs)."""
    if torch.cuda.is_available():
        torch.cuda.synchronize()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MNIST_AMD_SEGV_TRACE="1", PYTHONFAULTHANDLER="1", MNIST_AMD_LAUNCH_TIMEOUT=str(max(60, timeout - 60)))
    extra = ["--rank-logs", str(log_dir)] if log_dir is not None and "--gpus" in args else []
    r = subprocess.run([sys.executable, "-u", os.path.join(ROOT, "bench.py")] + args + extra, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=timeout)
    if r.returncode != 0:
        print(r.stderr[-20000:], file=sys.stderr)  # every rank's block (launch_relay) -- shown by pytest on failure
    assert r.returncode == 0, r.stderr[-6000:]
    lines = [l for l in r.stdout.splitlines() if l.lstrip().startswith("{")]
    assert len(lines) == 1, r.stdout
    return json.loads(lines[0]), r.stderr


def _emulate(model, dtype, batch, steps, dropout):
    """Two trainers in one process on the two shards, gradients summed on the host, 1/2 in the update."""
    sys.path.insert(0, ROOT)
    import bench
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    shards = [bench.bench_data(2, r, batch, steps) for r in range(2)]
    torch.manual_seed(0)
    init = build_model(model)
    trs = []
    for images, labels, idx, _, _ in shards:
        tr = NativeTrainer(model, dtype, batch, images.cuda(), labels.cuda(), lr=0.05, momentum=0.9, dropout=dropout,
                           init=init, max_indices=idx.numel())
        tr.set_epoch_indices(idx)
        trs.append(tr)
    for _ in range(steps):
        for tr in trs:
            tr.forward_backward(batch)
        g = trs[0].grads() + trs[1].grads()
        for tr in trs:
            tr.grad.copy_(g.to(tr.grad.device))
            torch.cuda.current_stream().synchronize()
            tr.optimizer_step(0.5)
    for tr in trs:
        tr.synchronize()
    return [tr.params.cpu() for tr in trs]


@pytest.mark.timeout(600)
@pytest.mark.parametrize("model,dtype,batch", [("lenet5", "bf16", 2048), ("mlp", "fp32", 128)])
def test_two_ranks_share_one_gpu(native, tmp_path, model, dtype, batch):
    steps, warmup = 4, 2
    out, err = _bench(["--gpus", "2", "--comm", "gloo", "--model", model, "--dtype", dtype, "--batch", str(batch),
                       "--steps", str(steps), "--warmup", str(warmup), "--no-eval", "--digest",
                       "--dump-params", str(tmp_path / "p")], log_dir=tmp_path / "ranks")
    assert out["n_gpus"] == 2 and out["config"]["parallelism"] == "dp2" and out["value"] > 0
    assert "gloo" in out["config"]["comm"]
    # the host (gloo) data plane runs the eager phase API, not the captured schedules: nothing is calibrated
    assert out["config"]["plan_autotune"]["chosen"] == "eager-phases"
    # (the two ranks share stderr: their lines can interleave without a newline between them)
    digests = dict(re.findall(r"digest rank=(\d) ([0-9a-f]{64})", err))
    assert set(digests) == {"0", "1"} and digests["0"] == digests["1"], err[-2000:]
    p = [torch.load(tmp_path / f"p.rank{r}.pt", weights_only=True) for r in range(2)]
    assert torch.equal(p[0], p[1])
    dropout = out["config"]["dropout"]
    assert dropout == (0.2 if model == "mlp" else 0.0)
    emu = _emulate(model, dtype, batch, steps + warmup, dropout)
    assert torch.equal(emu[0], emu[1])
    rel = ((p[0] - emu[0]).norm() / emu[0].norm()).item()
    assert rel <= 1e-6, rel


@pytest.mark.timeout(300)
@pytest.mark.parametrize("model", ["lenet5", "mlp"])
def test_comm_profile_world1(native, model):
    """With a (world-1) RCCL communicator the JSON attributes the communication: RCCL world, each
    collective's standalone all-reduce latency and the exposed comm (plan step - local step)."""
    out, _ = _bench(["--comm-world1", "--model", model, "--batch", "1024", "--steps", "8", "--warmup", "2",
                     "--no-eval"])
    assert out["rccl_world"] == 1
    prof = out["comm_profile"]
    assert prof["rccl_world"] == 1
    colls = prof["collectives"]
    assert colls and sum(c["bytes"] for c in colls) == 4 * (61706 if model == "lenet5" else 118272)
    assert all(0 < c["allreduce_us"] < 10000 for c in colls)
    assert prof["step_plan_ms"] > 0 and prof["step_local_ms"] > 0
    assert abs(prof["exposed_comm_us"] - 1000 * (prof["step_plan_ms"] - prof["step_local_ms"])) < 0.1
    tune = out["config"]["plan_autotune"]
    assert "nocomm" in tune["timings_ms"] and tune["chosen"] in ("join", "split", "split_r16", "split_bm", "split_mb")
    # link-aware bucket plan: the latency sweep and unit costs measured on this communicator, every partition of
    # the FC units ranked, and a multi-bucket SPLIT candidate timed beside the default plans
    bm = tune["bucket_model"]
    assert len(bm["latency_us"]) == 8 and all(v > 0 for v in bm["latency_us"].values())
    assert len(bm["unit_us"]) == 3 and bm["fc_all_us"] > 0 and len(bm["ranked"]) == 4
    assert any(k in tune["timings_ms"] for k in ("split_bm", "split_mb"))
    multi = [k for k in ("split_bm", "split_mb") if k in tune["candidates"]]
    assert any(len({b[2] for b in tune["candidates"][k]["buckets"]}) >= 3 for k in multi)
