"""Real multi-process RCCL runs of the native step (needs >= 2 GPUs; skipped on a one-GPU box).

bench.py --gpus 2 spawns two ranks (one per GPU), attaches the native RCCL communicator, calibrates
the plan on it and trains; every rank then prints a digest of its parameters.  DDP keeps replicas
bitwise identical (same all-reduced gradient, same update), so the digests must match -- for the
calibrated plan and for both pinned plans, LeNet and the MLP.
"""
import os
import re
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _two_gpus():
    return torch.cuda.device_count() >= 2


@pytest.mark.skipif(not _two_gpus(), reason="needs >= 2 GPUs")
@pytest.mark.timeout(600)
@pytest.mark.parametrize("args", [["--plan", "auto"], ["--plan", "join"], ["--plan", "split"],
                                  ["--model", "mlp", "--dtype", "fp32", "--batch", "128"]])
def test_two_rank_replicas_bitwise_equal(args):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "6", "--warmup", "2",
           "--no-eval", "--digest"] + args
    if "--batch" not in args:
        cmd += ["--batch", "1024"]
    r = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    digests = dict(re.findall(r"digest rank=(\d) (\w+)", r.stderr))
    assert set(digests) == {"0", "1"}, r.stderr[-2000:]
    assert digests["0"] == digests["1"]
    assert '"n_gpus": 2' in r.stdout
