"""In-tree build of the native extensions (no JIT cache, no pip install).

* ``_C``  : HIP kernels (``csrc/kernels/*.hip``, compiled by hipcc for gfx950 only) + the C++
            step runtime / RCCL communicator / pybind11 bindings; linked against
            ``libamdhip64.so.7`` and ``librccl.so.1`` (resolved at import time to the copies
            torch already mapped, see ``pytorch_ddp_mnist_amd/__init__.py``).
* ``_io`` : CPU-only C++ idx-ubyte / CDF-5 reader-writer (g++), importable without a GPU.

Both land next to this package (``pytorch_ddp_mnist_amd/*.so``) so they travel with the repo
snapshot to the GPU box.  Objects are cached under ``build/`` keyed on source + header hashes.
Usage: ``python -m pytorch_ddp_mnist_amd.ops.build [--force] [--only _C|_io]``.
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import hashlib
import os
import shutil
import subprocess
import sys
import sysconfig
from pathlib import Path
from typing import List

ROOT = Path(__file__).resolve().parents[2]
CSRC = ROOT / "csrc"
PKG = ROOT / "pytorch_ddp_mnist_amd"
BUILD = ROOT / "build" / "native"
ARCH = os.environ.get("PYTORCH_ROCM_ARCH", "gfx950")
ROCM = Path(os.environ.get("ROCM_PATH", "/opt/rocm"))
EXT = sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def _pybind_includes() -> List[str]:
    import pybind11
    return [f"-I{pybind11.get_include()}", f"-I{sysconfig.get_paths()['include']}"]


def _hipcc() -> str:
    p = shutil.which("hipcc") or str(ROCM / "bin" / "hipcc")
    return p


def _digest(paths: List[Path], extra: str) -> str:
    h = hashlib.sha1(extra.encode())
    for p in sorted(paths):
        h.update(p.read_bytes())
    return h.hexdigest()[:16]


def _run(cmd: List[str]) -> None:
    r = subprocess.run(cmd, stdout=subprocess.PIPE, stderr=subprocess.STDOUT, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"native build failed:\n{' '.join(cmd)}\n{r.stdout}")


def _compile(src: Path, headers: List[Path], cmd_prefix: List[str], force: bool) -> Path:
    tag = _digest([src] + headers, " ".join(cmd_prefix))
    obj = BUILD / f"{src.stem}.{tag}.o"
    if obj.exists() and not force:
        return obj
    BUILD.mkdir(parents=True, exist_ok=True)
    tmp = obj.with_suffix(".tmp.o")
    _run(cmd_prefix + ["-c", str(src), "-o", str(tmp)])
    tmp.replace(obj)
    return obj


def build_c(force: bool = False, jobs: int = 8, csrc: Path = CSRC, out: Path = None) -> Path:
    """``csrc`` / ``out``: build another source tree (e.g. a previous revision's ``csrc``, scripts/build_ab.sh)
    into another file, for same-box A/B runs (ops/native.py ``MNIST_AMD_C_PATH``)."""
    csrc = Path(csrc)
    headers = list(csrc.rglob("*.h"))
    hip_srcs = sorted((csrc / "kernels").glob("*.hip"))
    cpp_srcs = sorted((csrc / "runtime").glob("*.cpp")) + [csrc / "bindings.cpp"]
    # MNIST_AMD_BUILD_DEFINES: extra -D flags of a diagnostic build (e.g. -DMNIST_AMD_ABLATION_BUILD for
    # scripts/ablate.sh); part of the object-cache key, so switching back rebuilds the normal objects
    defs = os.environ.get("MNIST_AMD_BUILD_DEFINES", "").split()
    # MNIST_AMD_HIP_FLAGS: extra hipcc-only flags of a diagnostic build (code-generation options)
    hip_extra = os.environ.get("MNIST_AMD_HIP_FLAGS", "").split()
    hip_cmd = [_hipcc(), f"--offload-arch={ARCH}", "-O3", "-std=c++17", "-fPIC", f"-I{csrc}",
               "-Wno-unused-result"] + defs + hip_extra
    cpp_cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-D__HIP_PLATFORM_AMD__", f"-I{ROCM / 'include'}",
               f"-I{csrc}", "-fvisibility=hidden"] + defs + _pybind_includes()
    with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
        futs = [ex.submit(_compile, s, headers, hip_cmd, force) for s in hip_srcs]
        futs += [ex.submit(_compile, s, headers, cpp_cmd, force) for s in cpp_srcs]
        objs = [f.result() for f in futs]
    out = Path(out) if out else PKG / f"_C{EXT}"
    tmp = out.with_name(out.name + ".tmp")
    _run([_hipcc(), f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(tmp)] + [str(o) for o in objs]
         + [f"-L{ROCM / 'lib'}", "-lamdhip64", "-lrccl"])
    tmp.replace(out)
    return out


def build_io(force: bool = False) -> Path:
    src = CSRC / "io" / "mnist_io.cpp"
    cmd = ["g++", "-O2", "-std=c++17", "-fPIC", "-fvisibility=hidden"] + _pybind_includes()
    obj = _compile(src, [CSRC / "io" / "formats.h"], cmd, force)
    out = PKG / f"_io{EXT}"
    tmp = out.with_name(out.name + ".tmp")
    _run(["g++", "-shared", "-fPIC", "-o", str(tmp), str(obj), "-lpthread"])
    tmp.replace(out)
    return out


def build_all(force: bool = False) -> List[Path]:
    return [build_io(force), build_c(force)]


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__)
    ap.add_argument("--force", action="store_true")
    ap.add_argument("--only", choices=["_C", "_io"], default=None)
    ap.add_argument("--csrc", default=str(CSRC), help="_C source tree (default: the repo's csrc)")
    ap.add_argument("--out", default=None, help="_C output file (default: the in-tree package module)")
    a = ap.parse_args(argv)
    if a.only == "_io":
        print(build_io(a.force))
    elif a.only == "_C":
        print(build_c(a.force, csrc=Path(a.csrc), out=Path(a.out) if a.out else None))
    else:
        for p in build_all(a.force):
            print(p)
    return 0


if __name__ == "__main__":
    sys.exit(main())
