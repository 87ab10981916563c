"""native_stdout_to_stderr: native (fd-level) writes inside the guard land on stderr, so RCCL's init
banner cannot corrupt bench.py's one-JSON-line stdout."""
import subprocess
import sys

CODE = r"""
import os, sys
from pytorch_ddp_mnist_amd.utils.logging import native_stdout_to_stderr
print("before", flush=True)
with native_stdout_to_stderr():
    os.write(1, b"banner from native code\n")
    print("python print inside", flush=True)
print('{"json": 1}', flush=True)
"""


def test_native_stdout_goes_to_stderr():
    r = subprocess.run([sys.executable, "-c", CODE], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                       timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.splitlines() == ["before", '{"json": 1}']
    assert "banner from native code" in r.stderr and "python print inside" in r.stderr
