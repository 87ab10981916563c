"""One-shot xGMI all-reduce (csrc/kernels/oneshot.hip, parallel/oneshot.py; survey §5.8-3) on one MI355X.

* world 1: the kernel is the identity on random data (push to the own slot, wait the own flag, sum one slot),
  over many calls (parities, per-block sequence numbers), and a trainer whose captured step issues its gradient
  all-reduce through it trains bitwise like the local step;
* two rank PROCESSES on the one GPU (``bench.py --gpus 2 --comm gloo --allreduce oneshot``): the ranks export
  their regions over IPC, map each other's, and every step's all-reduce is the one-shot kernel.  Both replicas
  must end bitwise identical and equal to the same two shards trained with the gradient sum done on the host
  (the DDP arithmetic, reference ddp_tutorial_multi_gpu.py:72,94).
(A real 8-GPU node exercises the xGMI links themselves; here the peer "remote" stores go to the same device.)
"""
import os
import re
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_oneshot_world1_identity(native):
    C = native
    n = 61706
    o = C.OneShotAllReduce(0, 1, 0, n)
    assert o.ready and o.world == 1
    g = torch.Generator(device="cuda").manual_seed(3)
    s = torch.cuda.current_stream()
    for it in range(5):
        cnt = n - 3 * it  # also counts that are not a multiple of 4 (tail path)
        x = torch.randn(n, device="cuda", generator=g)
        ref = x.clone()
        o.all_reduce_sum_f32(x.data_ptr(), cnt, s.cuda_stream)
        s.synchronize()
        assert torch.equal(x, ref)
    assert o.check() == ""


def test_oneshot_world1_trainer_matches_local(native, small_mnist):
    from pytorch_ddp_mnist_amd.engine.native import NativeTrainer
    from pytorch_ddp_mnist_amd.models import build_model
    from pytorch_ddp_mnist_amd.parallel.comm import DistContext
    from pytorch_ddp_mnist_amd.parallel.oneshot import make_oneshot
    x, y, _, _ = small_mnist
    order = torch.randperm(4096, generator=torch.Generator().manual_seed(1)).to(torch.int32)
    out = []
    for use in (False, True):
        torch.manual_seed(0)
        tr = NativeTrainer("lenet5", "bf16", 512, torch.from_numpy(x.reshape(-1, 784)), torch.from_numpy(y), lr=0.05,
                           momentum=0.9, dropout=0.0, init=build_model("lenet5"))
        if use:
            o = make_oneshot(DistContext(0, 1, 0, torch.device("cuda", 0)), tr.nparam)
            tr.attach_oneshot(o, 1)
            assert tr.plan_info()["allreduce"] == "oneshot"
        tr.set_epoch_indices(order)
        tr.run_steps(6, use_graph=True, k=3)
        tr.synchronize()
        tr.check_comm()
        out.append(tr.params.cpu())
    assert torch.equal(out[0], out[1])


def _bench(args, timeout=540, log_dir=None):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_shared_gpu_ranks import _bench as run
    return run(args, timeout=timeout, log_dir=log_dir)


@pytest.mark.timeout(600)
@pytest.mark.parametrize("plan", ["fixed", "overlap"])
def test_oneshot_two_ranks_share_one_gpu(native, tmp_path, plan):
    """``fixed`` = JOIN (one all-reduce of the whole slab after the backward join); ``overlap`` = Plan::OVERLAP
    (two one-shot instances, the FC range's all-reduce + update inside the aux branch beside conv_bwd)."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from test_shared_gpu_ranks import _emulate
    steps, warmup, batch = 4, 2, 2048
    out, err = _bench(["--gpus", "2", "--comm", "gloo", "--allreduce", "oneshot", "--batch", str(batch),
                       "--steps", str(steps), "--warmup", str(warmup), "--no-eval", "--digest", "--plan", plan,
                       "--dump-params", str(tmp_path / "p")], log_dir=tmp_path / "ranks")
    assert out["n_gpus"] == 2 and out["allreduce"] == "oneshot" and out["value"] > 0
    assert "one-shot" in out["config"]["comm"]
    assert out["config"]["plan"]["plan"] == ("join" if plan == "fixed" else "overlap")
    prof = out["comm_profile"]
    assert prof["allreduce"] == "oneshot" and all(0 < c["oneshot_us"] < 10000 for c in prof["collectives"])
    digests = dict(re.findall(r"digest rank=(\d) ([0-9a-f]{64})", err))
    assert set(digests) == {"0", "1"} and digests["0"] == digests["1"], err[-2000:]
    p = [torch.load(tmp_path / f"p.rank{r}.pt", weights_only=True) for r in range(2)]
    assert torch.equal(p[0], p[1])
    emu = _emulate("lenet5", "bf16", batch, steps + warmup, 0.0)
    rel = ((p[0] - emu[0]).norm() / emu[0].norm()).item()
    assert rel <= 1e-6, rel


@pytest.mark.timeout(300)
def test_oneshot_missing_peer_call_latches(native, tmp_path):
    """A rank that does not issue one all-reduce (fault injection) makes its peer's flag wait run out: the peer
    raises CollectiveError at its next host wait within the in-kernel bound + 1 s, and the update behind the
    failed call leaves its parameters untouched (no partial sum is ever applied)."""
    import json
    import subprocess
    torch.cuda.synchronize()
    bound = 2.0
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env.update(MNIST_AMD_ONESHOT_SKIP_CALL="1:3", MNIST_AMD_ONESHOT_TIMEOUT=str(bound), MNIST_AMD_SEGV_TRACE="1",
               PYTHONFAULTHANDLER="1")
    code = ("import sys; sys.path.insert(0, %r); from pytorch_ddp_mnist_amd.parallel.launch import launch_relay; "
            "rc, _ = launch_relay([sys.executable, %r], 2, style='torch', timeout=200, log_dir=%r); sys.exit(rc)"
            % (ROOT, os.path.join(ROOT, "tests", "_oneshot_fault_rank.py"), str(tmp_path / "ranks")))
    r = subprocess.run([sys.executable, "-c", code], env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                       text=True, timeout=260)
    assert r.returncode == 0, r.stderr[-8000:]
    res = {}
    for line in (r.stdout + "\n" + r.stderr).splitlines():
        line = line.strip()
        if line.startswith("{") and '"rank"' in line:
            d = json.loads(line)
            res[d["rank"]] = d
    assert set(res) == {0, 1}, r.stdout + r.stderr[-4000:]
    assert res[0]["raised"] and "timed out" in res[0]["msg"], res[0]
    assert res[0]["seconds"] <= bound + 1.0, res[0]
    assert res[0]["params_unchanged"], res[0]
    assert res[1]["calls"] == 4 and res[0]["calls"] == 4


@pytest.mark.timeout(300)
def test_oneshot_and_rccl_profile_world1(native):
    """World 1 with both data planes: the step runs the one-shot kernel, and comm_profile reports the standalone
    latency of each collective on BOTH (RCCL all-reduce and one-shot)."""
    out, _ = _bench(["--comm-world1", "--allreduce", "oneshot", "--batch", "1024", "--steps", "8", "--warmup", "2",
                     "--no-eval"])
    prof = out["comm_profile"]
    assert prof["rccl_world"] == 1 and prof["allreduce"] == "oneshot"
    for c in prof["collectives"]:
        assert 0 < c["allreduce_us"] < 10000 and 0 < c["oneshot_us"] < 10000
