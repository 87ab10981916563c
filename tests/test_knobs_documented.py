"""Every MNIST_AMD_* switch the code reads is listed in docs/KNOBS.md (knob hygiene, verdict r5 weak item 10)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC_DIRS = ("csrc", "pytorch_ddp_mnist_amd")
SRC_FILES = ("bench.py", "__graft_entry__.py")
NAME = re.compile(r"MNIST_AMD_[A-Z0-9_]*[A-Z0-9]")


def _source_names():
    names = set()
    paths = [os.path.join(ROOT, f) for f in SRC_FILES]
    for d in SRC_DIRS:
        for dp, _, fs in os.walk(os.path.join(ROOT, d)):
            paths += [os.path.join(dp, f) for f in fs if f.endswith((".py", ".cpp", ".h", ".hip"))]
    for p in paths:
        if os.path.exists(p):
            with open(p, encoding="utf-8") as fh:
                names.update(NAME.findall(fh.read()))
    return names


def test_every_knob_is_documented():
    with open(os.path.join(ROOT, "docs", "KNOBS.md"), encoding="utf-8") as fh:
        doc = set(NAME.findall(fh.read()))
    missing = sorted(_source_names() - doc)
    assert not missing, f"undocumented switches (add them to docs/KNOBS.md): {missing}"
