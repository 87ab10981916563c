"""bench.py's self-launch (``--gpus N`` without torchrun) and the multi-GPU plan decision, on CPU."""
import json
import os
import subprocess
import sys

import pytest

from pytorch_ddp_mnist_amd.parallel.ddp import choose_plan, default_plan_candidates

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    e.update(env)
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=e, stdout=subprocess.PIPE,
                          stderr=subprocess.PIPE, text=True, timeout=120)


@pytest.mark.parametrize("n", [2, 4])
def test_bench_spawns_n_ranks_and_prints_one_line(n):
    r = _bench(["--gpus", str(n), "--dry-run"])
    assert r.returncode == 0, r.stderr
    lines = [l for l in r.stdout.splitlines() if l.strip()]
    assert len(lines) == 1, r.stdout               # only rank 0's JSON line reaches stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == n and d["dry_run"] and d["master"].startswith("127.0.0.1:")


def test_bench_failing_rank_propagates():
    r = _bench(["--gpus", "4", "--dry-run"], MNIST_AMD_DRYRUN_FAIL_RANK="2")
    assert r.returncode == 7
    assert "a rank failed" in r.stderr


def test_bench_under_torchrun_does_not_respawn():
    """With WORLD_SIZE in the env (torchrun) bench.py is a rank itself."""
    r = _bench(["--gpus", "2", "--dry-run"], WORLD_SIZE="2", RANK="1", LOCAL_RANK="1", MASTER_ADDR="127.0.0.1",
               MASTER_PORT="29999")
    assert r.returncode == 0 and r.stdout.strip() == ""   # rank 1 prints nothing


def test_choose_plan_prefers_join_within_margin():
    assert choose_plan({"join": 0.150, "split": 0.149}) == "join"            # < 1.5 % faster: keep join
    assert choose_plan({"join": 0.150, "split": 0.140}) == "split"
    assert choose_plan({"join": 0.150, "split": 0.140, "split_r16": 0.120}) == "split_r16"
    assert choose_plan({"split": 0.2, "split_r16": 0.3}) == "split"          # no join candidate
    with pytest.raises(ValueError):
        choose_plan({})


def test_choose_plan_is_rank_consistent():
    """Each rank passes rank-max timings, so every rank sees the same dict and decides the same."""
    per_rank = [{"join": 0.150, "split": 0.131}, {"join": 0.149, "split": 0.160}]
    agreed = {k: max(r[k] for r in per_rank) for k in per_rank[0]}
    assert {choose_plan(agreed) for _ in per_rank} == {"join"}


def test_default_plan_candidates():
    c = default_plan_candidates(512, 256)
    assert c["join"] == dict(plan="join", bwd_blocks=0) and c["split"] == dict(plan="split", bwd_blocks=0)
    assert c["split_r16"] == dict(plan="split", bwd_blocks=2 * (256 - 16))
    assert set(default_plan_candidates(64, 256)) == {"join", "split"}   # small batch: no capped variant
    assert choose_plan({"concurrent": 0.13, "serial": 0.1285}, prefer="concurrent") == "concurrent"
