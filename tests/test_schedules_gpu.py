"""Step-schedule equivalence on one MI355X (csrc/runtime/trainer.cpp launch_step).

The FC weight gradient runs on an aux stream beside conv_bwd (default) or after it
(MNIST_AMD_CONCURRENT=0); with a communicator the two gradient reductions join into one whole-slab
all-reduce (default) or the FC bucket goes out first (MNIST_AMD_MG_SCHED=split).  All of them
reduce in the same fixed order, so the trained parameters must be bitwise identical.
"""
import os
import re
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _digest(env_extra, args):
    env = dict(os.environ, PYTHONPATH=ROOT, **env_extra)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "sched_equiv.py")] + args, env=env,
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout[-3000:]
    return re.search(r"digest (\w+)", r.stdout).group(1)


@pytest.mark.timeout(900)  # five fresh interpreters (torch import + GPU init each)
def test_schedules_bitwise_equal(native):
    ref = _digest({"MNIST_AMD_CONCURRENT": "0"}, [])
    assert _digest({"MNIST_AMD_CONCURRENT": "1"}, []) == ref
    assert _digest({"MNIST_AMD_CONCURRENT": "1", "MNIST_AMD_SPLIT_BWD": "1"}, []) == ref  # conv_bwd halves
    assert _digest({"MNIST_AMD_CONCURRENT": "1"}, ["--comm"]) == ref
    assert _digest({"MNIST_AMD_CONCURRENT": "1", "MNIST_AMD_MG_SCHED": "split"}, ["--comm"]) == ref
