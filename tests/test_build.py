"""The in-tree native build's object cache (ops/build.py): cached objects are reused, a source change
compiles a new object, and --force recompiles even when the cache is warm."""
import time

from pytorch_ddp_mnist_amd.ops import build as B


def test_build_cache_and_force(tmp_path, monkeypatch):
    monkeypatch.setattr(B, "BUILD", tmp_path / "native")
    src = tmp_path / "t.cpp"
    src.write_text("int f() { return 1; }\n")
    cmd = ["g++", "-O0", "-fPIC"]
    o1 = B._compile(src, [], cmd, False)
    m1 = o1.stat().st_mtime_ns
    o2 = B._compile(src, [], cmd, False)
    assert o2 == o1 and o2.stat().st_mtime_ns == m1          # cache hit: not recompiled
    time.sleep(0.02)
    o3 = B._compile(src, [], cmd, True)
    assert o3 == o1 and o3.stat().st_mtime_ns > m1           # --force: recompiled in place
    src.write_text("int f() { return 2; }\n")
    assert B._compile(src, [], cmd, False) != o1             # new source -> new cache key


def test_build_cli_parses_force():
    import argparse
    called = {}
    orig = B.build_io
    try:
        B.build_io = lambda force=False: called.setdefault("force", force) or "x"
        B.main(["--only", "_io", "--force"])
    finally:
        B.build_io = orig
    assert called["force"] is True
