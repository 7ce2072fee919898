"""Property-based tests (hypothesis): relational operators on random small tables against
pandas / Python-set oracles on the CPU engine, and the HIP paths against their CPU twins on the
same draws (GPU variants).  Keys come from tiny ranges so duplicates, empty sides, all-equal
keys and null payloads are common (reference analogue: python/test/test_table_properties.py,
cpp/test/{join,sorting,groupby,set_op}_test.cpp -- fixed fixtures there, generated ones here)."""
import numpy as np
import pandas as pd
import pyarrow as pa
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from cylon_amd import Table

SETTINGS = settings(max_examples=40, deadline=None, suppress_health_check=[HealthCheck.too_slow])
GPU_SETTINGS = settings(max_examples=15, deadline=None, suppress_health_check=[HealthCheck.too_slow])

small_keys = st.lists(st.integers(-6, 6), min_size=0, max_size=48)
payload = st.one_of(st.none(), st.floats(-100, 100, allow_nan=False, width=32))


@st.composite
def relation(draw, prefix):
    ks = draw(small_keys)
    vs = draw(st.lists(payload, min_size=len(ks), max_size=len(ks)))
    return pa.table({"k": pa.array(ks, pa.int64()), f"{prefix}v": pa.array(vs, pa.float64())})


def _canon(df: pd.DataFrame):
    rows = []
    for r in df.itertuples(index=False):
        rows.append(tuple(None if v is None or v is pd.NA or (isinstance(v, float) and np.isnan(v)) else v
                          for v in r))
    return sorted(rows, key=lambda r: tuple((x is None, 0 if x is None else x) for x in r))


def _pandas_join(a: pa.Table, b: pa.Table, how: str) -> pd.DataFrame:
    x = a.to_pandas().add_prefix("l_")
    y = b.to_pandas().add_prefix("r_")
    return x.merge(y, left_on="l_k", right_on="r_k", how=how)


# ---------------------------------------------------------------------------
# CPU engine vs oracles
# ---------------------------------------------------------------------------
@SETTINGS
@given(relation("a"), relation("b"), st.sampled_from(["inner", "left", "right", "outer"]),
       st.sampled_from(["hash", "sort"]))
def test_join_matches_pandas_merge(ctx, a, b, how, algorithm):
    out = Table(a, ctx).join(Table(b, ctx), how, algorithm, on=["k"], left_prefix="l_",
                             right_prefix="r_").to_pandas()
    ref = _pandas_join(a, b, how)
    assert len(out) == len(ref)
    assert _canon(out) == _canon(ref[list(out.columns)])


@SETTINGS
@given(small_keys, st.booleans())
def test_sort_is_stable_and_ordered(ctx, ks, asc):
    n = len(ks)
    t = pa.table({"k": pa.array(ks, pa.int64()), "p": pa.array(np.arange(n, dtype=np.int64))})
    out = Table(t, ctx).sort("k", ascending=asc).to_pandas()
    ref = t.to_pandas().sort_values("k", ascending=asc, kind="stable").reset_index(drop=True)
    pd.testing.assert_frame_equal(out.reset_index(drop=True), ref, check_dtype=False)


@SETTINGS
@given(relation("a"))
def test_groupby_matches_pandas(ctx, a):
    if a.num_rows == 0:
        return
    g = Table(a, ctx).groupby("k", {"av": ["sum", "min", "max"]}).to_pandas()
    g = g.sort_values(g.columns[0]).reset_index(drop=True)
    ref = a.to_pandas().groupby("k", sort=True)["av"].agg(["sum", "min", "max"]).reset_index()
    assert g.iloc[:, 0].tolist() == ref["k"].tolist()
    for j, op in enumerate(["sum", "min", "max"], start=1):
        got = g.iloc[:, j].to_numpy(dtype=float)
        exp = ref[op].to_numpy(dtype=float)
        if op == "sum":  # an all-null group sums to 0 in both
            np.testing.assert_allclose(got, exp, rtol=1e-9, atol=1e-9)
        else:  # an all-null group has a null min / max
            np.testing.assert_allclose(np.nan_to_num(got, nan=1e300), np.nan_to_num(exp, nan=1e300), rtol=1e-9)


@SETTINGS
@given(small_keys, small_keys)
def test_set_ops_match_python_sets(ctx, xs, ys):
    a = pa.table({"k": pa.array(xs, pa.int64())})
    b = pa.table({"k": pa.array(ys, pa.int64())})
    A, B = Table(a, ctx), Table(b, ctx)
    assert sorted(A.union(B).to_pydict()["k"]) == sorted(set(xs) | set(ys))
    assert sorted(A.subtract(B).to_pydict()["k"]) == sorted(set(xs) - set(ys))
    assert sorted(A.intersect(B).to_pydict()["k"]) == sorted(set(xs) & set(ys))


@SETTINGS
@given(relation("a"), st.sampled_from(["first", "last"]))
def test_unique_keeps_first_or_last(ctx, a, keep):
    out = Table(a, ctx).unique(columns=["k"], keep=keep).to_pandas()
    ref = a.to_pandas().drop_duplicates(subset=["k"], keep=keep)
    assert _canon(out) == _canon(ref)


# ---------------------------------------------------------------------------
# HIP paths vs the CPU twin on the same draws (radix paths forced on tiny inputs)
# ---------------------------------------------------------------------------
@pytest.mark.gpu
@GPU_SETTINGS
@given(relation("a"), relation("b"), st.sampled_from(["hash", "sort"]))
def test_gpu_inner_join_matches_cpu(gpu_ctx, ctx, a, b, algorithm):
    import os
    os.environ["CYLON_RADIX_JOIN_MIN_ROWS"] = "1"
    try:
        g = Table(a, gpu_ctx).join(Table(b, gpu_ctx), "inner", algorithm, on=["k"], left_prefix="l_",
                                   right_prefix="r_").to_pandas()
    finally:
        del os.environ["CYLON_RADIX_JOIN_MIN_ROWS"]
    c = Table(a, ctx).join(Table(b, ctx), "inner", algorithm, on=["k"], left_prefix="l_",
                           right_prefix="r_").to_pandas()
    assert _canon(g) == _canon(c)


@pytest.mark.gpu
@GPU_SETTINGS
@given(small_keys, st.booleans())
def test_gpu_row_sort_matches_cpu(gpu_ctx, ctx, ks, asc):
    import os
    n = len(ks)
    t = pa.table({"k": pa.array(ks, pa.int64()), "p": pa.array(np.arange(n, dtype=np.int64))})
    os.environ["CYLON_RADIX_SORT_MIN_ROWS"] = "1"
    try:
        g = Table(t, gpu_ctx).sort("k", ascending=asc).to_pandas()
    finally:
        del os.environ["CYLON_RADIX_SORT_MIN_ROWS"]
    c = Table(t, ctx).sort("k", ascending=asc).to_pandas()
    pd.testing.assert_frame_equal(g, c)
