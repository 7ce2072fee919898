"""Set operations and unique: reference golden files (cpp/test/set_op_test.cpp,
data/output/{union,subtract,intersect}_{world}_{rank}.csv) and pandas oracles."""
import os

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.csv as pacsv
import pytest

from cylon_amd import Table
from cylon_amd.io import CSVReadOptions, read_csv

from dist_utils import run_distributed


def _rows(df):
    return sorted(tuple(round(float(x), 6) for x in r) for r in df.itertuples(index=False))


def _golden_setop(ctx, data_dir, op):
    rank, world = ctx.get_rank(), ctx.get_world_size()
    opts = CSVReadOptions().use_threads(False).with_column_types({"0": pa.int64(), "1": pa.float64()})
    t1 = read_csv(ctx, os.path.join(data_dir, "input", f"csv1_{rank}.csv"), opts)
    t2 = read_csv(ctx, os.path.join(data_dir, "input", f"csv2_{rank}.csv"), opts)
    exp = pacsv.read_csv(os.path.join(data_dir, "output", f"{op}_{world}_{rank}.csv")).to_pandas()
    res = getattr(t1, f"distributed_{op}")(t2).to_pandas()
    return _rows(res) == _rows(exp), len(res), len(exp)


@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("op", ["union", "subtract", "intersect"])
def test_set_ops_golden(data_dir, world, op):
    for ok, got, exp in run_distributed(_golden_setop, world, data_dir, op):
        assert ok, f"{op}: rows got={got} expected={exp}"


def _frames():
    rng = np.random.default_rng(5)
    a = pd.DataFrame({"x": rng.integers(0, 6, 300), "s": [f"v{v}" for v in rng.integers(0, 4, 300)]})
    b = pd.DataFrame({"x": rng.integers(3, 9, 200), "s": [f"v{v}" for v in rng.integers(0, 4, 200)]})
    return a, b


def _set(df):
    return set(map(tuple, df.itertuples(index=False)))


def test_local_set_ops_vs_python_sets(ctx):
    a, b = _frames()
    ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
    u, s, i = ta.union(tb).to_pandas(), ta.subtract(tb).to_pandas(), ta.intersect(tb).to_pandas()
    assert len(u) == len(_set(u)) and _set(u) == _set(a) | _set(b)
    assert len(s) == len(_set(s)) and _set(s) == _set(a) - _set(b)
    assert len(i) == len(_set(i)) and _set(i) == _set(a) & _set(b)


def test_set_op_schema_mismatch(ctx):
    a = Table(pa.table({"x": [1, 2]}), ctx)
    b = Table(pa.table({"x": [1.0, 2.0]}), ctx)
    with pytest.raises(Exception):
        a.union(b)


def test_unique_first_last(ctx, data_dir):
    at = pacsv.read_csv(os.path.join(data_dir, "input", "indexing_data.csv"))
    t = Table(at, ctx)
    df = at.to_pandas()
    for keep in ("first", "last"):
        got = t.unique(columns=["a", "b"], keep=keep).to_pandas().reset_index(drop=True)
        exp = df.drop_duplicates(subset=["a", "b"], keep=keep).reset_index(drop=True)
        pd.testing.assert_frame_equal(got, exp)


def test_unique_with_nulls_and_strings(ctx):
    at = pa.table({"a": pa.array([1, None, 1, None, 2]), "s": ["x", "y", "x", "y", None]})
    got = Table(at, ctx).unique().to_pandas()
    assert len(got) == 3


def _numeric(df):
    return df.assign(s=df["s"].str[1:].astype(np.int64))


def _dist_set_ops(ctx, numeric=False):
    a, b = _frames()
    if numeric:
        a, b = _numeric(a), _numeric(b)
    r = ctx.get_rank()
    a = a.iloc[r::ctx.get_world_size()]
    b = b.iloc[r::ctx.get_world_size()]
    ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
    return (ta.distributed_union(tb).to_pandas(), ta.distributed_subtract(tb).to_pandas(),
            ta.distributed_intersect(tb).to_pandas(), ta.distributed_unique(["x"]).to_pandas())


def _dist_set_ops_chunked(ctx):
    from cylon_amd._lib import C
    ctx.add_config("shuffle_chunks", "3")
    C.trace_enable(True)
    out = _dist_set_ops(ctx, numeric=True)
    assert C.trace_counters().get("shuffle.chunks", 0) >= 3
    C.trace_enable(False)
    return out


@pytest.mark.parametrize("chunked", [False, True])
def test_distributed_set_ops_vs_sets(chunked):
    a, b = _frames()
    if chunked:
        a, b = _numeric(a), _numeric(b)
    res = run_distributed(_dist_set_ops_chunked if chunked else _dist_set_ops, 3)
    u = pd.concat([r[0] for r in res])
    s = pd.concat([r[1] for r in res])
    i = pd.concat([r[2] for r in res])
    q = pd.concat([r[3] for r in res])
    assert len(u) == len(_set(u)) and _set(u) == _set(a) | _set(b)
    assert _set(s) == _set(a) - _set(b) and len(s) == len(_set(s))
    assert _set(i) == _set(a) & _set(b) and len(i) == len(_set(i))
    assert sorted(q["x"].tolist()) == sorted(a["x"].unique().tolist())


def test_unique_and_sort_with_nulls_over_varying_payload(ctx):
    """Null entries whose underlying buffer values differ are still equal (and adjacent in
    multi-column sorts): nulls get a constant sort image."""
    import numpy as np
    import pyarrow as pa
    from cylon_amd import Table
    f = pa.array([0.5, 1.25, 0.5, 7.0, 2.0], mask=np.array([True, False, False, True, False]))
    t = Table(pa.table({"f": f, "i": pa.array([1, 2, 1, 1, 2], pa.int32())}), ctx)
    assert t.unique(None).to_pydict() == {"f": [None, 1.25, 0.5, 2.0], "i": [1, 2, 1, 2]}
    s = t.sort(["f", "i"]).to_pydict()
    assert s == {"f": [0.5, 1.25, 2.0, None, None], "i": [1, 2, 2, 1, 1]}
    u = Table(pa.table({"f": pa.array([3.0], type=pa.float64(), mask=np.array([True])), "i": pa.array([1], pa.int32())}), ctx)
    assert t.union(u).row_count == 4
    assert t.subtract(u).to_pydict() == {"f": [1.25, 0.5, 2.0], "i": [2, 1, 2]}
