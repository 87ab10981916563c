"""CPU checks of the LDS bank models used to choose the conv kernels' LDS layouts.

scripts/lds_model.py (conv_bwd) and scripts/lds_model_fwd.py (conv_fwd) replay every LDS access of one
image with the kernels' lane mappings.  Their conflict shares were validated against the measured
SQ_LDS_BANK_CONFLICT share (conv_bwd 38.5 % vs 38.9 % at the old pitches; conv_fwd 36.5 % vs 38.2 %,
profiles/r2_session3/pmc_table.md); these tests pin the bank rules and the current layouts' results.
"""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))

import lds_model  # noqa: E402
import lds_model_fwd  # noqa: E402


def test_b128_rules():
    # 64 lanes reading consecutive 16-byte chunks: every 16-lane group covers the 64 banks once (ideal:
    # one cycle per group)
    c, ideal = lds_model.cycles("r128", {lane: 16 * lane for lane in range(64)})
    assert (c, ideal) == (4, 4)
    # all lanes on the same 16 bytes: one distinct dword per bank -> ideal
    c, _ = lds_model.cycles("r128", {lane: 0 for lane in range(64)})
    assert c == 4
    # two lanes of one group 256 bytes apart (same banks, different dwords): 2-way conflict in that group
    addrs = {0: 0, 1: 256}
    c, _ = lds_model.cycles("r128", addrs)
    assert c == 2


def test_sub_dword_stores_merge():
    # 16-bit stores of two lanes into one dword are not a conflict; into two dwords of one bank they are
    assert lds_model.cycles("w16", {0: 0, 1: 2})[0] == 1
    assert lds_model.cycles("w16", {0: 0, 1: 128})[0] == 2


def test_conv_fwd_model_current_layout():
    acc = lds_model_fwd.model({"XP": 1048, "P1CP": 232, "M1CP": 240})
    total = sum(v[1] for v in acc.values())
    ideal = sum(v[2] for v in acc.values())
    assert (total, ideal) == (1064, 676)
    # the staging stores and the pool2 / copy-out accesses are conflict-free at the chosen pitches
    assert acc["stage xs (w128)"][1] <= acc["stage xs (w128)"][2]
    assert acc["conv2 epi p2s (w16)"][1] <= acc["conv2 epi p2s (w16)"][2]


@pytest.mark.parametrize("xp", [1040, 1056, 1072])
def test_conv_fwd_plane_pitch_is_a_local_optimum(xp):
    cur = sum(v[1] for v in lds_model_fwd.model({"XP": 1048, "P1CP": 232, "M1CP": 240}).values())
    alt = sum(v[1] for v in lds_model_fwd.model({"XP": xp, "P1CP": 232, "M1CP": 240}).values())
    assert alt > cur


def test_conv_bwd_phase_c_layout():
    """conv1 wgrad as one packed tile (lenet.hip C_AMAP / C_BMAP, XP 1048, D1P 944): conflict-free
    DY1T reads, at most 1.5-way XS reads, and fewer LDS cycles per image than the two-tile layout."""
    acc, _ = lds_model.model(lds_model.CUR)
    n, c, i, _ = acc["C.dy1t"]
    assert (n, c) == (29, i)
    n, c, i, _ = acc["C.xs"]
    assert n == 29 and c <= 1.5 * i
    prev, _ = lds_model.model(lds_model.PREV)
    tot = lambda a: sum(v[1] for v in a.values())  # noqa: E731
    assert tot(acc) < tot(prev) - 150
    # round 3 final: the conv2 wgrad A operand read from DYS with transposing reads (no DY2T copy) is cheaper
    r3c, _ = lds_model.model(lds_model.R3C)
    assert "B1.dys_tr" in acc and "B1.dy2t" not in acc and tot(acc) < tot(r3c)
    # the (r, n) map covers every (row shift, channel) once; the column map every (khb, kw) + the bias
    assert sorted(lds_model.CUR["AMAP"]) == [(r, n) for r in range(2) for n in range(8)]
    assert sorted(lds_model.CUR["BMAP"]) == list(range(16))
