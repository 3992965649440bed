"""bench.py's report helpers on a synthetic profile (no GPU): the roofline objects and the kernel table read the
per-kernel tuples spg.Context.prof_read(ops=True) returns -- (launches, us, bytes, madds, Fq products) -- whatever
mix of modelled quantities a kernel carries"""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def bench():
    spec = importlib.util.spec_from_file_location("bench_under_test", os.path.join(ROOT, "bench.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def synthetic(bench):
    p = bench.Prof({
        "spark_layer_round": (100, 1000.0, 1.5e8, 0.0, 4.0e7),     # bytes + Fq products
        "msm_bullet_round": (50, 800.0, 5.0e7, 2.5e5, 0.0),         # bytes + madds
        "msm_comb": (2, 5000.0, 0.0, 1.0e8, 0.0),                   # madds only
        "sc_phase1_fold_eval": (10, 900.0, 6.0e8, 0.0, 1.2e8),
        "eq_table": (20, 100.0, 1.0e6, 0.0, 0.0),
    })
    p.busy_us = 7000.0
    p.busy_resident_us = 7000.0
    return p


def test_rooflines_read_five_field_tuples(bench):
    prof = synthetic(bench)
    roof, h, v = bench.rooflines(prof)
    assert h["kernel"] == "spark_layer_round" and h["bound"] == "hbm"
    assert v["kernel"] == "msm_comb" and v["bound"] == "valu"
    assert roof is v  # the kernel with the most device time among the modelled ones
    assert abs(v["achieved"] - 1.0e8 / 5000e-6) < 1.0
    f = bench.roofline_fq(prof)
    assert f["kernel"] == "spark_layer_round" and f["bound"] == "valu_fq"
    assert abs(f["achieved"] - 4.0e7 / 1000e-6) < 1.0
    assert 0 < f["frac"] < 1 and f["hbm_frac"] > 0


def test_rooflines_on_four_field_tuples(bench):
    # a library built before the Fq-product counter reports four fields
    prof = bench.Prof({k: v[:4] for k, v in synthetic(bench).items()})
    roof, h, v = bench.rooflines(prof)
    assert roof is not None and h is not None and v is not None
    assert bench.roofline_fq(prof) is None


def test_kernel_table(bench):
    t = bench.kernel_table(synthetic(bench), steps=2, top=3)
    assert list(t) == ["msm_comb", "spark_layer_round", "sc_phase1_fold_eval"]
    assert t["spark_layer_round"]["fq_products_per_s"] > 0 and t["msm_comb"]["madds_per_s"] > 0
    assert t["msm_comb"]["GBps"] is None
