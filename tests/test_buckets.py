"""Link-aware bucket plans (parallel/ddp.py): the unit table, the partition -> bucket mapping, the latency
curve, the SPLIT-tail model and the ranking it drives, on synthetic latency curves (CPU only).

Reference: the DDP Reducer cuts buckets by size in backward order (ddp_tutorial_multi_gpu.py:72; torch's first
bucket 1 MiB, then 25 MB), so both reference models send ONE bucket per step (survey §2.7).  Here the groups are
chosen from the measured all-reduce latency curve and per-layer backward cost."""
import pytest
import torch

from pytorch_ddp_mnist_amd.models import NPARAM, UNITS, build_model, param_layout
from pytorch_ddp_mnist_amd.parallel.ddp import (LatencyCurve, bucket_plan_candidates, choose_bucket_groups,
                                                default_groups, fc_unit_count, groups_to_buckets, model_join_tail_us,
                                                model_split_tail_us, partitions)


@pytest.mark.parametrize("model", ["mlp", "lenet5"])
def test_units_tile_the_slab_in_ready_order(model):
    units = UNITS[model]
    assert units[0][2] == NPARAM[model] and units[-1][1] == 0
    for (_, a0, a1), (_, b0, b1) in zip(units, units[1:]):
        assert b1 == a0 and a0 < a1  # each unit ends where the previous (earlier-ready) one starts
    # unit boundaries are layer boundaries of the torch module (weight + bias of one layer never split)
    starts = {off for _, _, off in param_layout(build_model(model))}
    for _, p0, p1 in units:
        assert p0 in starts or p0 == 0
    keys = [k for k, _, _ in param_layout(build_model(model))]
    first = {"mlp": ["5.weight", "3.weight", "0.weight"], "lenet5": ["11.weight", "9.weight", "7.weight", "0.weight"]}[model]
    offs = dict((k, off) for k, _, off in param_layout(build_model(model)))
    assert [offs[k] for k in first] == [p0 for _, p0, _ in units]
    assert set(keys)  # non-empty module


def test_native_job_boundaries_match_units():
    C = pytest.importorskip("pytorch_ddp_mnist_amd.ops.native").load_c()
    if C is None:
        pytest.skip("native extension not built")
    for model, mid in (("mlp", 0), ("lenet5", 1)):
        fc = [u for u in UNITS[model] if u[0] != "conv"]
        # job j = the j-th FC layer from the input side; UNITS lists them last layer first
        for j, (_, p0, p1) in enumerate(reversed(fc)):
            assert C.Trainer.job_begin(mid, j) == p0 and C.Trainer.job_begin(mid, j + 1) == p1


def test_partitions():
    assert partitions(1) == [[[0]]]
    ps = partitions(3)
    assert len(ps) == 4 and [[0, 1, 2]] in ps and [[0], [1], [2]] in ps and [[0, 1], [2]] in ps
    assert len(partitions(4)) == 8
    for p in partitions(4):
        assert [i for g in p for i in g] == [0, 1, 2, 3]


@pytest.mark.parametrize("model", ["mlp", "lenet5"])
def test_groups_to_buckets_cover_every_parameter(model):
    n = fc_unit_count(model)
    for groups in partitions(n):
        b = groups_to_buckets(model, groups)
        # groups in ready order, contiguous, covering [0, nparam) exactly once
        cov = torch.zeros(NPARAM[model], dtype=torch.int32)
        for p0, p1, _ in b:
            cov[p0:p1] += 1
        assert bool((cov == 1).all())
        ng = len(groups) + (1 if model == "lenet5" else 0)
        assert sorted({g for _, _, g in b}) == list(range(ng))
        ends = {}
        for p0, p1, g in b:
            lo, hi = ends.get(g, (p0, p1))
            ends[g] = (min(lo, p0), max(hi, p1))
        assert ends[0][1] == NPARAM[model] and ends[ng - 1][0] == 0
        for g in range(1, ng):
            assert ends[g][1] == ends[g - 1][0]
    with pytest.raises(ValueError):
        groups_to_buckets(model, [[1], [0]] + ([[2]] if n == 3 else []))  # out of ready order


def test_bucket_cap_splits_inside_a_group():
    b = groups_to_buckets("lenet5", [[0, 1], [2]], cap_bytes=64 * 1024)
    assert {g for _, _, g in b} == {0, 1, 2}
    assert all(4 * (p1 - p0) <= 64 * 1024 for p0, p1, _ in b)
    assert sum(p1 - p0 for p0, p1, _ in b) == NPARAM["lenet5"]


def test_latency_curve_interpolates_and_extrapolates():
    lat = LatencyCurve([(4096, 10.0), (65536, 14.0), (1 << 20, 30.0)])
    assert lat(1024) == 10.0  # flat below the smallest point
    assert lat(4096) == 10.0 and lat(65536) == 14.0
    assert abs(lat((4096 + 65536) / 2) - 12.0) < 1e-9
    slope = (30.0 - 14.0) / ((1 << 20) - 65536)
    assert abs(lat(2 << 20) - (30.0 + slope * (1 << 20))) < 1e-6
    assert set(lat.as_dict()) == {"4096", "65536", "1048576"}


def test_latency_bound_curve_keeps_one_fc_group():
    """Pure per-collective latency (no size term) and an FC branch that finishes long before conv_bwd: every extra
    group only adds a collective + update on the comm stream, so the default single FC group wins."""
    lat = LatencyCurve([(4096, 20.0), (1 << 20, 20.0)])
    r = choose_bucket_groups("lenet5", lat, unit_us=[3.0, 3.0, 5.0], fc_all_us=9.0, main_us=50.0)
    assert r[0][0] == [[0, 1, 2]]
    assert [g for g, _ in r][-1] == [[0], [1], [2]]
    assert bucket_plan_candidates("lenet5", r).keys() == {"split_mb"}  # the best multi-bucket plan is still timed


def test_exposed_fc_comm_is_cut_into_early_groups():
    """Bandwidth-dominated collectives and an FC branch that ends AFTER the conv backward (small conv work, a slow
    fc1 weight gradient): sending fc3 + fc2 while fc1's gradient is computed hides their collective, so a
    multi-group plan is modelled faster than one FC group."""
    lat = LatencyCurve([(4096, 5.0), (1 << 20, 5.0 + (1 << 20) / 4000.0)])  # ~4 KB per us
    unit_us = [2.0, 6.0, 40.0]
    one = model_split_tail_us("lenet5", [[0, 1, 2]], lat, unit_us, fc_all_us=46.0, main_us=10.0)
    two = model_split_tail_us("lenet5", [[0, 1], [2]], lat, unit_us, fc_all_us=46.0, main_us=10.0)
    assert two < one
    r = choose_bucket_groups("lenet5", lat, unit_us, fc_all_us=46.0, main_us=10.0)
    assert len(r[0][0]) >= 2
    c = bucket_plan_candidates("lenet5", r)
    assert "split_bm" in c and c["split_bm"]["plan"] == "split"
    assert len({g for _, _, g in c["split_bm"]["buckets"]}) >= 3


def test_split_tail_model_arithmetic():
    """Hand-checked timeline: LeNet, groups [[0],[1,2]], constant 10 us collectives, 1 us updates."""
    lat = LatencyCurve([(1, 10.0)])
    unit_us, fc_all, main = [2.0, 3.0, 7.0], 10.0, 30.0
    save = (2.0 + 3.0 + 7.0 - 10.0) / 2  # per merged unit
    t0 = 2.0                              # group 0 ready
    c0 = t0 + 10.0 + 1.0                  # its collective + update
    t1 = t0 + 3.0 + 7.0 - save            # group 1 ready
    c1 = max(c0, t1) + 10.0 + 1.0
    conv = max(c1, main) + 10.0 + 1.0
    got = model_split_tail_us("lenet5", [[0], [1, 2]], lat, unit_us, fc_all, main, update_us=1.0)
    assert abs(got - conv) < 1e-9
    j = model_join_tail_us("lenet5", lat, fc_all, main, update_us=1.0)
    assert abs(j - (30.0 + 10.0 + 1.0)) < 1e-9


def test_mlp_candidates_and_defaults():
    assert default_groups("mlp") == [[0, 1], [2]] and default_groups("lenet5") == [[0, 1, 2]]
    lat = LatencyCurve([(4096, 8.0), (1 << 20, 12.0)])
    r = choose_bucket_groups("mlp", lat, unit_us=[2.0, 3.0, 12.0], fc_all_us=15.0)
    c = bucket_plan_candidates("mlp", r)
    assert any(len({g for _, _, g in v["buckets"]}) >= 3 for v in c.values())
    for v in c.values():
        assert v["groups"] != default_groups("mlp")
