"""Group-by and aggregate tests (reference: cpp/test/groupby_test.cpp,
cpp/test/aggregate_test.cpp) plus pandas oracles."""
import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

from cylon_amd import Table

from dist_utils import run_distributed

OPS = ["sum", "count", "min", "max", "mean", "var", "std", "nunique", "median"]
PD = {"sum": "sum", "count": "count", "min": "min", "max": "max", "mean": "mean", "var": "var", "std": "std",
      "nunique": "nunique", "median": "median"}
PREFIX = {"sum": "sum_", "count": "count_", "min": "min_", "max": "max_", "mean": "mean_", "var": "var_",
          "std": "std_", "nunique": "nunique_", "median": "quantile_"}


def _ref_table():
    # reference groupby_test.cpp:30-37
    return pa.table({"col0": pa.array([0, 0, 1, 1, 2, 2, 3, 3, 4, 4], pa.int64()),
                     "col1": pa.array([0, 0, 1, 1, 2, 2, 3, 3, 4, 4], pa.float64())})


def _ref_invariants(ctx):
    w = ctx.get_world_size()
    t = Table(_ref_table(), ctx)
    out = {}
    for op in ("sum", "count", "mean", "var", "std", "nunique", "median", "min", "max"):
        g = t.groupby(0, {1: op})
        out[op] = (g.sum(0).to_pydict()["col0"][0], g.sum(1).to_pydict()[g.column_names[1]][0])
    p = t.groupby(0, {1: "sum"}, algorithm="pipeline")
    out["pipeline"] = (p.sum(0).to_pydict()["col0"][0], p.sum(1).to_pydict()[p.column_names[1]][0])
    return w, out


@pytest.mark.parametrize("world", [1, 2, 4])
def test_reference_groupby_invariants(world):
    for w, out in run_distributed(_ref_invariants, world):
        assert out["sum"] == (10, 2 * 10.0 * w)
        assert out["count"] == (10, 5 * 2 * w)
        assert out["mean"] == (10, 10.0)
        assert out["var"][1] == pytest.approx(0.0)
        assert out["std"][1] == pytest.approx(0.0)
        assert out["nunique"] == (10, 5)
        assert out["median"] == (10, 10.0)
        assert out["min"] == (10, 10.0) and out["max"] == (10, 10.0)
        assert out["pipeline"] == (10, 2 * 10.0 * w)


def _frame(seed=0, n=2000, nulls=False):
    rng = np.random.default_rng(seed)
    v = rng.normal(size=n)
    df = pd.DataFrame({"k": rng.integers(0, 37, n), "s": [f"g{x}" for x in rng.integers(0, 5, n)], "v": v,
                       "i": rng.integers(-1000, 1000, n)})
    if nulls:
        df.loc[rng.random(n) < 0.1, "v"] = np.nan
    return df


def _check(got: pd.DataFrame, df: pd.DataFrame, keys, col, ops):
    exp = df.groupby(keys)[col].agg([PD[o] for o in ops]).reset_index()
    got = got.sort_values(keys).reset_index(drop=True)
    exp = exp.sort_values(keys).reset_index(drop=True)
    assert len(got) == len(exp)
    for k in keys:
        assert got[k].tolist() == exp[k].tolist()
    for o in ops:
        g = got[PREFIX[o] + col].to_numpy(dtype=float)
        e = exp[PD[o]].to_numpy(dtype=float)
        np.testing.assert_allclose(g, e, rtol=1e-9, atol=1e-9, equal_nan=True)


@pytest.mark.parametrize("nulls", [False, True])
@pytest.mark.parametrize("keys", [["k"], ["s"], ["k", "s"]])
def test_local_groupby_vs_pandas(ctx, keys, nulls):
    df = _frame(1, nulls=nulls)
    t = Table.from_pandas(ctx, df)
    for alg in ("hash", "pipeline"):
        tt = t.sort(keys) if alg == "pipeline" else t
        got = tt.local_groupby(keys, {"v": OPS}, algorithm=alg).to_pandas()
        _check(got, df, keys, "v", OPS)
    got = t.local_groupby(keys, {"i": ["sum", "min", "max", "count"]}).to_pandas()
    _check(got, df, keys, "i", ["sum", "min", "max", "count"])


def test_groupby_first_occurrence_order(ctx):
    t = Table(pa.table({"k": [5, 3, 5, 9, 3, 1], "v": [1, 2, 3, 4, 5, 6]}), ctx)
    assert t.local_groupby("k", {"v": "sum"}).to_pydict() == {"k": [5, 3, 9, 1], "sum_v": [4, 7, 4, 6]}


def _dist_groupby(ctx, ops, keys):
    df = _frame(10 + ctx.get_rank(), n=700, nulls=True)
    t = Table.from_pandas(ctx, df)
    return t.groupby(keys, {"v": ops}).to_pandas(), df


@pytest.mark.parametrize("ops", [["sum", "count", "min", "max", "mean", "var", "std"],
                                 ["nunique", "median", "sum"]])
def test_distributed_groupby_vs_pandas(ops):
    for keys in (["k"], ["k", "s"]):
        res = run_distributed(_dist_groupby, 3, ops, keys)
        got = pd.concat([r[0] for r in res])
        df = pd.concat([r[1] for r in res])
        _check(got, df, keys, "v", ops)


def _dist_groupby_simple(ctx, keys):
    df = _frame(20 + ctx.get_rank(), n=900, nulls=False)
    t = Table.from_pandas(ctx, df)
    ops = ["sum", "count", "min", "max", "mean"]
    return t.groupby(keys, {"v": ops, "i": ["sum", "mean", "max"]}).to_pandas(), df


@pytest.mark.parametrize("keys", [["k"], ["k", "s"]])
def test_distributed_groupby_partial_states_fast_form(keys):
    """SUM / COUNT / MIN / MAX / MEAN over non-null columns: the local group-by emits the
    partial states directly (phase 1 fast form)."""
    res = run_distributed(_dist_groupby_simple, 3, keys)
    got = pd.concat([r[0] for r in res])
    df = pd.concat([r[1] for r in res])
    _check(got, df, keys, "v", ["sum", "count", "min", "max", "mean"])
    exp = df.groupby(keys)["i"].agg(["sum", "mean", "max"]).reset_index()
    m = got.merge(exp, on=keys)
    assert len(m) == len(exp) == len(got)
    assert (m["sum_i"] == m["sum"]).all() and (m["max_i"] == m["max"]).all()
    np.testing.assert_allclose(m["mean_i"], m["mean"], rtol=1e-12)


def _dist_aggs(ctx):
    rng = np.random.default_rng(ctx.get_rank())
    df = pd.DataFrame({"a": rng.integers(-50, 50, 100), "f": rng.random(100)})
    t = Table.from_pandas(ctx, df)
    out = {op: [getattr(t, op)(c).to_pydict()[c][0] for c in ("a", "f")]
           for op in ("sum", "count", "min", "max", "mean", "var", "std", "nunique")}
    out["median"] = [t.quantile(c, 0.5).to_pydict()[c][0] for c in ("a", "f")]
    return out, df


def test_distributed_scalar_aggregates():
    res = run_distributed(_dist_aggs, 4)
    df = pd.concat([r[1] for r in res])
    for out, _ in res:
        for c, col in enumerate(("a", "f")):
            s = df[col]
            assert out["sum"][c] == pytest.approx(s.sum())
            assert out["count"][c] == len(s)
            assert out["min"][c] == s.min() and out["max"][c] == s.max()
            assert out["mean"][c] == pytest.approx(s.mean())
            assert out["var"][c] == pytest.approx(s.var())
            assert out["std"][c] == pytest.approx(s.std())
            assert out["nunique"][c] == s.nunique()
            assert out["median"][c] == pytest.approx(s.median())
