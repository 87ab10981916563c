"""Step-schedule equivalence on one MI355X (csrc/runtime/trainer.cpp launch_step).

The FC weight gradient runs on an aux stream beside conv_bwd (default) or after it
(MNIST_AMD_CONCURRENT=0); with a
communicator the gradient exchange follows the JOIN plan (one coalesced all-reduce after the backward
join) or the SPLIT plan (phase-0 buckets + their update on the comm stream beside the rest of the
backward, then phase 1's).  All of them reduce in the same fixed order, so the trained parameters must
be bitwise identical; a capped conv_bwd grid changes the summation order, so capped variants are
compared among themselves.  The ``_w2`` variants check the 1/W averaging of both plans against a local
run at half the learning rate; ``_k4`` variants run the steps as one 4-step graph (deferred aux join).
The MLP has the same plans (layers 2+3 sent beside the layer-1 weight gradient).  ``overlap`` (LeNet): world-1
one-shot all-reduces inside the concurrent schedule's two branches (Plan::OVERLAP).
"""
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _digests(env_extra, variants, model="lenet5", extra=(), dump=None):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    dump_arg = ["--dump", str(dump)] if dump else []
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "sched_equiv.py"), "--model", model, *extra, *dump_arg]
                       + variants,
                       env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    return dict(re.findall(r"digest (\S+) (\w+)", r.stdout))


@pytest.mark.timeout(900)  # two fresh interpreters (torch import + GPU init each)
def test_schedules_bitwise_equal(native):
    serial = _digests({"MNIST_AMD_CONCURRENT": "0"}, ["local", "local_halflr"])
    d = _digests({"MNIST_AMD_CONCURRENT": "1"},
                 ["local", "join", "split", "join_w2", "split_w2", "local_b480", "join_b480", "split_b480",
                  "local_k4", "join_k4", "split_k4", "overlap", "overlap_w2", "overlap_k4"])
    ref = serial["local"]
    for k in ("local", "join", "split", "local_k4", "join_k4", "split_k4", "overlap", "overlap_k4"):
        assert d[k] == ref, k
    assert d["join_w2"] == serial["local_halflr"] and d["split_w2"] == serial["local_halflr"]
    assert d["overlap_w2"] == serial["local_halflr"]
    assert d["join_b480"] == d["local_b480"] and d["split_b480"] == d["local_b480"]


@pytest.mark.timeout(600)
def test_bucket_groups_bitwise_equal(native):
    """Link-aware bucket plans (parallel/ddp.py choose_bucket_groups): SPLIT with the FC head cut into 2 or 3 bucket
    groups -- each its own weight-gradient launch (job mask), reduce, all-reduce and update -- gives the parameters of
    the local step, bitwise (world-1 communicator; _w2: the 1/W arithmetic of two ranks)."""
    serial = _digests({"MNIST_AMD_CONCURRENT": "0"}, ["local", "local_halflr"])
    d = _digests({"MNIST_AMD_CONCURRENT": "1"}, ["split_g0.1.2", "split_g01.2", "split_g0.12", "split_g0.1.2_w2",
                                                  "split_g0.1.2_k4", "join_g0.1.2"])
    for k in ("split_g0.1.2", "split_g01.2", "split_g0.12", "split_g0.1.2_k4", "join_g0.1.2"):
        assert d[k] == serial["local"], k
    assert d["split_g0.1.2_w2"] == serial["local_halflr"]
    m = _digests({}, ["local", "split_g0.1.2", "split_g012", "split_g0.12_k4"], model="mlp")
    for k in ("split_g0.1.2", "split_g012", "split_g0.12_k4"):
        assert m[k] == m["local"], k


@pytest.mark.timeout(900)
def test_large_batch_schedules_bitwise_equal(native):
    """The headline batch (8192: fused forward + head, split-K-in-workgroup weight gradient, 16 FC splits): serial,
    concurrent, JOIN / SPLIT and multi-group SPLIT steps give bitwise-identical parameters."""
    extra = ("--batch", "8192", "--steps", "2")
    serial = _digests({"MNIST_AMD_CONCURRENT": "0"}, ["local"], extra=extra)
    d = _digests({"MNIST_AMD_CONCURRENT": "1"}, ["local", "join", "split", "split_g0.1.2", "split_g01.2"], extra=extra)
    for k in ("local", "join", "split", "split_g0.1.2", "split_g01.2"):
        assert d[k] == serial["local"], k
    m = _digests({}, ["local", "join", "split", "split_g0.1.2"], model="mlp", extra=extra)
    for k in ("join", "split", "split_g0.1.2"):
        assert m[k] == m["local"], k


@pytest.mark.timeout(600)
@pytest.mark.parametrize("dtype,batch", [("fp32", 128), ("bf16", 128)])
def test_small_batch_serial_equals_concurrent(native, dtype, batch):
    """Small batches (one FC batch split): the serial schedule runs conv_bwd and the SGD-fused FC weight
    gradient as ONE kernel (launch_lenet_conv_bwd_fc); the concurrent one runs them on two streams."""
    extra = ("--dtype", dtype, "--batch", str(batch))
    serial = _digests({"MNIST_AMD_CONCURRENT": "0"}, ["local", "local_k4", "local_t69"], extra=extra)
    conc = _digests({"MNIST_AMD_CONCURRENT": "1"}, ["local", "local_t69"], extra=extra)
    assert serial["local"] == conc["local"] and serial["local_k4"] == conc["local"]
    assert serial["local_t69"] == conc["local_t69"]  # + a partial last batch of 69 rows


@pytest.mark.timeout(300)
def test_mlp_schedules_bitwise_equal(native):
    d = _digests({}, ["local", "local_halflr", "join", "split", "join_w2", "split_w2", "split_k4"], model="mlp")
    for k in ("join", "split", "split_k4"):
        assert d[k] == d["local"], k
    assert d["join_w2"] == d["local_halflr"] and d["split_w2"] == d["local_halflr"]

