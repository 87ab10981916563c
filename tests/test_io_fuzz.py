"""Hostile-input hardening of the native header parsers (survey §5.2: sanitizers on host code).

* ``csrc/io/fuzz_headers.cpp`` -- the exact parsers of the ``_io`` extension (csrc/io/formats.h) --
  is compiled with ``-fsanitize=address,undefined -fno-sanitize-recover=all`` and fed valid idx /
  CDF-5 / CDF-1 seed files plus thousands of deterministic mutations (bit flips, truncations, 0xFF
  length fields, lies about the file size): any out-of-bounds access, overflow or UB aborts it.
* hand-built malicious headers through the real ``_io`` module: every one must raise a Python
  exception (no crash, no huge allocation, no read outside the file).
"""
import os
import shutil
import struct
import subprocess

import numpy as np
import pytest

from pytorch_ddp_mnist_amd.data import cdf5, idx
from pytorch_ddp_mnist_amd.ops.native import load_io

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _seeds(d):
    rng = np.random.default_rng(0)
    x = rng.integers(0, 256, (64, 28, 28), dtype=np.uint8)
    y = rng.integers(0, 10, 64, dtype=np.uint8)
    idx.write_idx(os.path.join(d, "img.idx"), x)
    idx.write_idx(os.path.join(d, "lab.idx"), y)
    cdf5.write_mnist_nc(os.path.join(d, "mnist.nc"), x, y)
    # a CDF-1 file with a global attribute and a variable attribute (32-bit fields, other branches)
    h = bytearray(b"CDF\x01") + struct.pack(">I", 0)
    h += struct.pack(">II", 0x0A, 1) + struct.pack(">I", 1) + b"n\0\0\0" + struct.pack(">I", 4)
    h += struct.pack(">II", 0x0C, 1) + struct.pack(">I", 1) + b"t\0\0\0" + struct.pack(">II", 2, 3) + b"abc\0"
    h += struct.pack(">II", 0x0B, 1) + struct.pack(">I", 1) + b"v\0\0\0" + struct.pack(">II", 1, 0)
    h += struct.pack(">II", 0x0C, 1) + struct.pack(">I", 1) + b"u\0\0\0" + struct.pack(">II", 5, 1) + struct.pack(">f", 1.0)
    h += struct.pack(">III", 5, 16, len(h) + 12) + struct.pack(">4f", 1, 2, 3, 4)
    with open(os.path.join(d, "cdf1.nc"), "wb") as f:
        f.write(bytes(h))
    return [os.path.join(d, n) for n in ("img.idx", "lab.idx", "mnist.nc", "cdf1.nc")]


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_header_parsers_under_asan_ubsan(tmp_path):
    exe = str(tmp_path / "fuzz_headers")
    r = subprocess.run(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined", "-fno-sanitize-recover=all",
                        "-fno-omit-frame-pointer", "-I", os.path.join(ROOT, "csrc", "io"),
                        os.path.join(ROOT, "csrc", "io", "fuzz_headers.cpp"), "-o", exe],
                       stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True, timeout=300)
    assert r.returncode == 0, r.stdout
    seeds = _seeds(str(tmp_path))
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="print_stacktrace=1")
    r = subprocess.run([exe] + seeds + ["--mutations", "3000", "--seed", "7"], env=env, stdout=subprocess.PIPE,
                       stderr=subprocess.STDOUT, text=True, timeout=600)
    assert r.returncode == 0 and "fuzz_headers:" in r.stdout, r.stdout[-4000:]
    parsed = int(r.stdout.split("fuzz_headers:")[1].split()[0])
    assert parsed >= 2 * len(seeds)          # the unmutated seeds parse (both formats tried on each)


def _nc_header(name_len=None, dim_len=28, nvars=1, begin=None, ndims=1, dimid=0, vtype=7):
    """CDF-5 header with one dim and one variable; fields overridable with hostile values."""
    h = bytearray(b"CDF\x05") + struct.pack(">Q", 0)
    h += struct.pack(">IQ", 0x0A, 1) + struct.pack(">Q", 1 if name_len is None else name_len) + b"d\0\0\0"
    h += struct.pack(">Q", dim_len)
    h += struct.pack(">IQ", 0, 0)
    h += struct.pack(">IQ", 0x0B, nvars) + struct.pack(">Q", 1) + b"v\0\0\0" + struct.pack(">Q", ndims)
    h += struct.pack(">Q", dimid) * ndims + struct.pack(">IQ", 0, 0) + struct.pack(">I", vtype)
    h += struct.pack(">Q", dim_len) + struct.pack(">Q", len(h) + 16 if begin is None else begin)
    return bytes(h) + b"\0" * 64


@pytest.mark.parametrize("case", [
    dict(name_len=2 ** 63),                   # name length that wraps p + n
    dict(name_len=2 ** 64 - 2),               # (n + 3) & ~3 wraps to 0
    dict(dim_len=2 ** 62, ndims=3),           # product of dims overflows
    dict(begin=2 ** 64 - 8),                  # begin + size wraps
    dict(begin=10 ** 9),                      # data past the end of the file
    dict(nvars=2 ** 60),                      # absurd variable count (header runs out)
    dict(dimid=7),                            # unknown dimension id
    dict(vtype=99),                           # unknown type
])
def test_hostile_netcdf_headers_raise(tmp_path, case):
    io = load_io()
    if io is None:
        pytest.skip("_io not built")
    p = tmp_path / "bad.nc"
    p.write_bytes(_nc_header(**case))
    with pytest.raises(Exception):
        f = io.NcFile(str(p))
        f.read_rows("v", 0, -1)


@pytest.mark.parametrize("hdr", [
    b"\0\0\x08\x04" + struct.pack(">IIII", 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF, 0xFFFFFFFF),  # size overflow
    b"\0\0\x08\x03" + struct.pack(">III", 60000, 28, 28),   # claims 47 MB, file has a few bytes
    b"\0\0\x08\x09" + b"\0" * 36,                          # rank 9
    b"\0\0\x08",                                           # truncated magic
    b"\0\0\x0d\x01" + struct.pack(">I", 4) + b"\0" * 16,   # float idx (unsupported)
])
def test_hostile_idx_headers_raise(tmp_path, hdr):
    io = load_io()
    if io is None:
        pytest.skip("_io not built")
    p = tmp_path / "bad.idx"
    p.write_bytes(hdr)
    with pytest.raises(Exception):
        io.idx_read(str(p), -1)
