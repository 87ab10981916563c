"""bench.py's timed region, plan-argument handling and the synthetic generator modes, on CPU."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import forced_plan, resolve_plan  # noqa: E402


class _Log(list):
    def clock(self):
        self.append("clock")
        return float(len(self))


class FakeCtx:
    """Records every control-plane call; all_reduce_max returns a fixed 'slowest rank' time."""

    def __init__(self, log):
        self.log = log

    def barrier(self):
        self.log.append("barrier")

    def all_reduce_max(self, v):
        self.log.append("all_reduce_max")
        return max(v, 123.0)

    def all_reduce_sum(self, vals):
        self.log.append("all_reduce_sum")
        return vals


class FakeTrainer:
    def __init__(self, log):
        self.log = log

    def synchronize(self):
        self.log.append("sync")


def test_timed_region_has_no_collective_inside():
    log = _Log()
    ctx, tr = FakeCtx(log), FakeTrainer(log)
    run = lambda n: log.append(f"run{n}")  # noqa: E731
    out = bench.timed_region(ctx, tr, run, 20, cuda_sync=lambda: log.append("cuda_sync"), clock=log.clock)
    assert out == 123.0                                   # the rank-max is what is reported
    t0, t1 = [i for i, e in enumerate(log) if e == "clock"]
    inside = log[t0 + 1:t1]
    assert inside == ["run20", "sync", "cuda_sync"], inside
    assert "barrier" in log[:t0] and "cuda_sync" in log[:t0]   # ranks start together, device idle
    assert log[t1 + 1:] == ["all_reduce_max"]             # the only collective after the clock stops


def test_timed_region_elapsed_is_per_rank_clock():
    seen = []

    class Ctx(FakeCtx):
        def all_reduce_max(self, v):
            seen.append(v)
            return v

    log = _Log()
    out = bench.timed_region(Ctx(log), FakeTrainer(log), lambda n: None, 5, cuda_sync=lambda: None, clock=log.clock)
    assert seen == [out] and out > 0


def test_resolve_plan():
    assert resolve_plan("auto") is None and resolve_plan(None) is None
    assert resolve_plan("fixed") == "join"              # no calibration, default plan (no KeyError)
    assert resolve_plan("join") == "join" and resolve_plan("split") == "split"
    assert resolve_plan("overlap") == "overlap"          # LeNet one-shot plan (needs a validated data plane)
    with pytest.raises(ValueError):
        resolve_plan("bogus")


def test_forced_plan_env(monkeypatch):
    monkeypatch.delenv("MNIST_AMD_MG_SCHED", raising=False)
    assert forced_plan() is None
    monkeypatch.setenv("MNIST_AMD_MG_SCHED", "split")
    assert forced_plan() == "split"
    monkeypatch.setenv("MNIST_AMD_MG_SCHED", "splt")
    with pytest.raises(ValueError, match="MNIST_AMD_MG_SCHED"):
        forced_plan()


def test_bench_parses_plan_fixed_and_mlp_dropout_default():
    a = bench.parse(["--plan", "fixed", "--model", "mlp"])
    assert a.plan == "fixed" and a.dropout is None      # main() turns None into the reference's 0.2
    assert bench.parse(["--comm", "gloo"]).comm == "gloo"


def test_bench_data_is_deterministic_and_sharded():
    x0, y0, i0, _, _ = bench.bench_data(2, 0, 256, 10)
    x1, y1, i1, _, _ = bench.bench_data(2, 1, 256, 10)
    assert np.array_equal(x0.numpy(), x1.numpy()) and i0.numel() == i1.numel() >= 10 * 256
    a, b = set(i0[:30000].tolist()), set(i1[:30000].tolist())
    assert not (a & b)                                   # disjoint shards within an epoch
    _, _, j0, _, _ = bench.bench_data(2, 0, 256, 10)
    assert np.array_equal(i0.numpy(), j0.numpy())


def test_synthetic_hard_mode():
    from pytorch_ddp_mnist_amd.data.synthetic import make_split
    xe, ye = make_split(2000, seed=3)
    xh, yh = make_split(2000, seed=3, mode="hard")
    assert xh.shape == xe.shape and xh.dtype == np.uint8 and yh.dtype == np.uint8
    xh2, _ = make_split(2000, seed=3, mode="hard")
    assert np.array_equal(xh, xh2)
    # noisier than the default set: nearest-centroid accuracy well below the easy set's
    def centroid_acc(x, y):
        X = x.reshape(len(x), -1).astype(np.float32) / 255
        C = np.stack([X[y == c].mean(0) for c in range(10)])
        return (np.argmin(((X[:, None] - C[None]) ** 2).sum(-1), 1) == y).mean()
    assert centroid_acc(xh, yh) < centroid_acc(xe, ye) - 0.2
    with pytest.raises(ValueError):
        make_split(10, seed=0, mode="nope")


def test_calibration_samples_stay_inside_the_loaded_order():
    """time_schedules replays samples from a rewound step counter: a sample must never need more steps
    than the loaded order holds (a 4 x 20-step block over 28 loaded steps read past the index buffer)."""
    from pytorch_ddp_mnist_amd.engine.native import calib_blocks
    for avail in (1, 2, 9, 14, 20, 21, 28, 40, 468):
        for k in (1, 2, 8, 10, 20, 32):
            for multi in (True, False):
                m, blk, seg, per = calib_blocks(avail, k, multi and avail >= k + 1)
                assert per <= avail and blk >= 1 and seg >= 2
                assert per == blk * (k if m else 1)
    assert calib_blocks(28, 8, True) == (True, 3, 4, 24)
    assert calib_blocks(28, 20, True) == (True, 1, 4, 20)
    assert calib_blocks(468, 8, True) == (True, 4, 4, 32)
    assert calib_blocks(10, 8, False) == (False, 1, 12, 1)


def test_bench_netcdf_data_roundtrip(tmp_path):
    """bench.py --data netcdf: the split written as CDF-5 and read back through the bulk loader is the
    in-memory split, byte for byte (CPU device: the same write + pread path, no HBM copy)."""
    import torch

    import bench
    from pytorch_ddp_mnist_amd.parallel.comm import DistContext
    images, labels, idx, _, _ = bench.bench_data(1, 0, 512, 20)
    ctx = DistContext(0, 1, 0, torch.device("cpu"))
    dx, dy, info = bench.netcdf_data(ctx, images, labels, str(tmp_path), "easy")
    assert torch.equal(dx.view(-1, 784), images.view(-1, 784)) and torch.equal(dy, labels)
    assert info["rows"] == images.shape[0] and info["bytes"] == images.numel() + labels.numel()
    assert info["load_s"] > 0 and info["load_GBps"] > 0
