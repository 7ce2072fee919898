"""DataFrame / CylonEnv frontend (reference: python/test/test_frame.py) and the indexing
golden files (cpp/test/indexing_test.cpp, data/output/indexing_loc_{hl,r}_{1..9}.csv)."""
import os

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.csv as pacsv
import torch
import pytest

from cylon_amd import CylonEnv, DataFrame, GlooConfig, IndexingSchema, Table

from dist_utils import run_distributed


def _rows(at):
    return sorted(tuple(r.values()) for r in at.to_pylist())


# indexing_test.cpp: index built on column 'a' (hash/linear) or a range index; data = b, c, d
LOC_CASES = {
    1: lambda t: t.loc[0:5, 0],
    2: lambda t: t.loc[0:5, 0:1],
    3: lambda t: t.loc[0:5, [0, 2]],
    4: lambda t: t.loc[10, 1],
    5: lambda t: t.loc[[4, 10], 1:2],
    6: lambda t: t.loc[[4, 10], [0, 2]],
    7: lambda t: t.loc[4, [0, 1]],
    8: lambda t: t.loc[4, 1:2],
    9: lambda t: t.loc[[4, 10], 0],
}


@pytest.mark.parametrize("schema", [IndexingSchema.HASH, IndexingSchema.LINEAR, IndexingSchema.RANGE])
@pytest.mark.parametrize("case", sorted(LOC_CASES))
def test_loc_golden(ctx, data_dir, schema, case):
    at = pacsv.read_csv(os.path.join(data_dir, "input", "indexing_data.csv"))
    t = Table(at, ctx)
    if schema == IndexingSchema.RANGE:
        t = t.drop(["a"])
        t.set_index(list(range(t.row_count)), IndexingSchema.RANGE)
        tag = "r"
    else:
        t.set_index("a", schema, drop=True)
        tag = "hl"
    got = LOC_CASES[case](t).to_arrow()
    exp = pacsv.read_csv(os.path.join(data_dir, "output", f"indexing_loc_{tag}_{case}.csv"))
    assert _rows(got.rename_columns(exp.column_names)) == _rows(exp)


def test_indexing_schema_switch(ctx):
    t = Table(pa.table({"k": [5, 6, 7], "v": [1, 2, 3]}), ctx)
    t.set_index("k", IndexingSchema.HASH, drop=True)
    assert t.indexing_schema == IndexingSchema.HASH
    t.indexing_schema = IndexingSchema.LINEAR
    assert t.loc[6].to_pydict() == {"v": [2]}


def test_dataframe_basics(ctx):
    df = DataFrame({"a": [3, 1, 2, 1], "b": [0.5, 1.5, None, 2.5]}, context=ctx)
    assert df.shape == (4, 2) and df.columns == ["a", "b"]
    assert df.sort_values(by="a").to_dict()["a"] == [1, 1, 2, 3]
    assert df.drop_duplicates(subset=["a"]).to_dict()["a"] == [3, 1, 2]
    assert df.drop_duplicates(subset=["a"], keep="last").to_dict()["b"] == [0.5, None, 2.5]
    assert df.fillna(0).to_dict()["b"] == [0.5, 1.5, 0.0, 2.5]
    assert df[df["a"] > 1].shape == (2, 2)
    assert (df + 1).to_dict()["a"] == [4, 2, 3, 2]
    df["c"] = 1
    assert df.columns == ["a", "b", "c"]
    assert df.isnull().to_dict()["b"][2] is True
    cpu = df.to_cpu()
    assert cpu.is_cpu() and cpu.device == "cpu"
    assert df.groupby("a", {"c": "sum"}).sort_values(by="a").to_dict() == {"a": [1, 2, 3], "sum_c": [2, 1, 1]}


def test_dataframe_merge_join_concat(ctx):
    l = DataFrame({"k": [1, 2, 3], "x": ["a", "b", "c"]}, context=ctx)
    r = DataFrame({"k": [2, 3, 4], "y": [20, 30, 40]}, context=ctx)
    m = l.merge(r, how="inner", on=["k"], suffixes=("l_", "r_")).to_pandas()
    assert sorted(m["l_k"].tolist()) == [2, 3]
    m = l.merge(r, how="outer", algorithm="hash", left_on=["k"], right_on=["k"]).to_pandas()
    assert len(m) == 4
    r2 = r.set_index("k", drop=False)
    j = l.join(r2, on="k", how="left").to_pandas()
    assert len(j) == 3
    c = DataFrame.concat([l, l], axis=0)
    assert c.shape == (3, 2)  # reference concat(axis=0) is a set union
    c1 = DataFrame.concat([l, r], axis=1)
    assert c1.shape[0] == 3


def _dist_frame(ctx):
    env = CylonEnv.__new__(CylonEnv)
    env._context, env._distributed, env._finalized = ctx, True, True
    rank = ctx.get_rank()
    l = DataFrame({"k": np.arange(rank * 10, rank * 10 + 10) % 7, "x": np.arange(10) + rank * 100})
    r = DataFrame({"k": np.arange(7), "y": np.arange(7) * 10})
    j = l.merge(r, on=["k"], env=env).to_pandas()
    s = l.sort_values(by=["k", "x"], env=env).to_pandas()
    u = l.drop_duplicates(subset=["k"], env=env).to_pandas()
    g = l.groupby("k", {"x": "sum"}, env=env).to_pandas()
    return j, s, u, g, l.to_pandas(), r.to_pandas()


def test_dataframe_distributed_env():
    res = run_distributed(_dist_frame, 2)
    j = pd.concat([r[0] for r in res])
    l = pd.concat([r[4] for r in res])
    r = res[0][5]
    exp = l.merge(r, on="k")
    assert len(j) == 2 * len(exp)  # r is replicated on both ranks
    s = pd.concat([x[1] for x in res]).reset_index(drop=True)
    assert s["k"].is_monotonic_increasing
    u = pd.concat([x[2] for x in res])
    assert sorted(u["k"].tolist()) == sorted(l["k"].unique().tolist())
    g = pd.concat([x[3] for x in res]).sort_values("k")
    assert g["sum_x"].tolist() == l.groupby("k")["x"].sum().sort_index().tolist()


def test_reference_indexer_entry_points(ctx):
    """pycylon's LocIndexer.loc_with_* and PyLocIndexer entry points."""
    import pyarrow as pa
    from cylon_amd import Table
    from cylon_amd.indexing import ILocIndexer, IndexingSchema, LocIndexer, PyLocIndexer
    t = Table(pa.table({"a": [10, 20, 30, 40], "b": [1.0, 2.0, 3.0, 4.0], "c": ["w", "x", "y", "z"]}), ctx)
    li = LocIndexer(IndexingSchema.LINEAR)
    assert li.loc_with_single_column(slice(1, 2), "b", t).to_pydict() == {"b": [2.0, 3.0]}
    assert li.loc_with_multi_column([0, 3], ["a", "c"], t).to_pydict() == {"a": [10, 40], "c": ["w", "z"]}
    assert li.loc_with_range_column(slice(2, 3), slice("b", "c"), t).to_pydict() == {"b": [3.0, 4.0],
                                                                                     "c": ["y", "z"]}
    assert ILocIndexer(t).loc_with_single_column(slice(0, 2), 0).to_pydict() == {"a": [10, 20]}
    assert PyLocIndexer(t, "iloc")[1:3, ["a"]].to_pydict() == {"a": [20, 30]}
    assert PyLocIndexer(t, "loc")[2, "c"].to_pydict() == {"c": ["y"]}


# ---- persistent native indexes (cylon/indexing/index.hpp) -----------------------



def _loc_oracle(vals, labels):
    return [i for l in labels for i, v in enumerate(vals) if v == l]


@pytest.mark.parametrize("schema", ["HASH", "BINARYTREE", "BTREE", "LINEAR"])
@pytest.mark.parametrize("kind", ["int64", "int32", "float64", "nullable"])
def test_persistent_index_lookups(ctx, schema, kind):
    """Built once, then probed: label order then row order, duplicates, misses, nulls never match."""
    from cylon_amd._lib import C
    from cylon_amd.indexing import IndexingSchema, build_index
    rng = np.random.default_rng(3)
    vals = rng.integers(-50, 50, 3000)
    if kind == "float64":
        arr = pa.array(vals.astype(np.float64) / 4)
    elif kind == "int32":
        arr = pa.array(vals.astype(np.int32))
    elif kind == "nullable":
        arr = pa.array(vals, mask=rng.random(3000) < 0.1)
    else:
        arr = pa.array(vals)
    C.trace_enable(True)
    C.trace_reset()
    idx = build_index(arr, IndexingSchema[schema], ctx.device)
    pyvals = arr.to_pylist()
    labels = [pyvals[5], 1000, pyvals[17], pyvals[5]]
    for _ in range(3):  # repeated lookups reuse the built structure
        got = idx.positions_of_list(labels).tolist()
    assert got == _loc_oracle(pyvals, labels)
    built = dict(C.trace_counters()).get("index.built_rows", 0)
    if schema != "LINEAR":
        assert idx.persistent_rows == sum(v is not None for v in pyvals)
        assert built == idx.persistent_rows  # one build, not one per lookup
    C.trace_enable(False)


@pytest.mark.parametrize("kind", ["string", "nullable_string", "binary", "fixed_binary"])
def test_persistent_string_hash_index(ctx, kind):
    """A string / binary Hash index is built once (hash runs + byte verification on probe):
    label order then row order, duplicates, misses, nulls never match, and 64-bit hash
    collisions cannot merge distinct values (the probe compares bytes)."""
    from cylon_amd._lib import C
    from cylon_amd.indexing import IndexingSchema, build_index
    rng = np.random.default_rng(4)
    words = [f"w{int(x)}" for x in rng.integers(0, 300, 4000)]
    if kind == "string":
        arr = pa.array(words)
    elif kind == "nullable_string":
        arr = pa.array(words, mask=rng.random(4000) < 0.1)
    elif kind == "binary":
        arr = pa.array([w.encode() for w in words], pa.binary())
    else:
        arr = pa.array([w.encode().ljust(6, b"_") for w in words], pa.binary(6))
    pyvals = arr.to_pylist()
    C.trace_enable(True)
    C.trace_reset()
    idx = build_index(arr, IndexingSchema.HASH, ctx.device)
    labels = [pyvals[3], "nope" if kind in ("string", "nullable_string") else b"nope__", pyvals[11], pyvals[3]]
    labels = [l for l in labels if l is not None] or labels
    for _ in range(3):
        got = idx.positions_of_list(labels).tolist()
    assert got == _loc_oracle(pyvals, labels)
    assert idx.persistent_rows == sum(v is not None for v in pyvals)
    assert dict(C.trace_counters()).get("index.built_rows", 0) == idx.persistent_rows
    C.trace_enable(False)


def test_index_labels_must_convert_exactly(ctx):
    """A label that does not convert exactly to the index type matches nothing (2.5 is not 2)."""
    from cylon_amd.indexing import IndexingSchema, build_index
    arr = pa.array(np.array([1, 2, 3, 2, 127], dtype=np.int8))
    for schema in ("HASH", "BTREE", "LINEAR"):
        idx = build_index(arr, IndexingSchema[schema], ctx.device)
        assert idx.positions_of_list([2.0]).tolist() == [1, 3]
        assert idx.positions_of_list([2.5]).tolist() == []
        assert idx.positions_of_list([383]).tolist() == []  # 383 = 127 mod 256
    fidx = build_index(pa.array([0.5, 1.0, 2.0]), IndexingSchema.HASH, ctx.device)
    assert fidx.positions_of_list([1]).tolist() == [1]
    big = build_index(pa.array(np.array([2 ** 53], dtype=np.float64)), IndexingSchema.HASH, ctx.device)
    assert big.positions_of_list([2 ** 53 + 1]).tolist() == []


def test_native_loc_indexer_and_set_index(ctx):
    """C++ LocIndexer / ILocIndexer over a table whose index was set once (Set_Index)."""
    from cylon_amd._lib import C
    from cylon_amd.data import arrow_bridge as ab
    t = Table(pa.table({"k": [5, 3, 9, 3, 7, 1], "v": [0.5, 0.3, 0.9, 0.35, 0.7, 0.1]}), ctx)
    nidx = C.build_index(t.native, 0, C.IndexingSchema.HASH)
    C.table_set_index(t.native, nidx)
    assert C.table_get_index(t.native) is not None
    lab = ab.column_from_arrow("l", pa.array([3, 7]), ctx.device)
    out = Table(None, ctx, _native=C.loc(t.native, lab, [1], C.IndexingSchema.HASH)).to_pydict()
    assert out == {"v": [0.3, 0.35, 0.7]}
    s = ab.column_from_arrow("s", pa.array([3]), ctx.device)
    e = ab.column_from_arrow("e", pa.array([7]), ctx.device)
    rng = Table(None, ctx, _native=C.loc_range(t.native, s, e, [], C.IndexingSchema.HASH)).to_pydict()
    assert rng["k"] == [3, 9, 3, 7]
    il = Table(None, ctx, _native=C.iloc(t.native, torch.tensor([5, 0]), [0])).to_pydict()
    assert il == {"k": [1, 5]}
    C.table_reset_index(t.native)
    assert C.table_get_index(t.native) is None


@pytest.mark.parametrize("kind", ["int", "float_nan", "string_nulls", "range"])
@pytest.mark.parametrize("skip_null", [True, False])
def test_base_index_isin_matches_arrow(kind, skip_null):
    """BaseIndex.isin (reference indexing/index.pyx:81): per label membership, against Arrow's is_in
    (the reference's compare_array_like_values) as the oracle."""
    import pyarrow.compute as pc
    from cylon_amd.indexing.index import BaseIndex, HashIndex, RangeIndex
    if kind == "int":
        labels, values, idx = pa.array([5, 1, 9, 1, 7]), [1, 7, 2.5, 100], HashIndex([5, 1, 9, 1, 7])
    elif kind == "float_nan":
        labels, values = pa.array([1.5, float("nan"), 2.0, -0.5]), np.array([2.0, np.nan])
        idx = BaseIndex(np.array([1.5, np.nan, 2.0, -0.5]))
    elif kind == "string_nulls":
        labels, values = pa.array(["a", None, "c", "a", "d"]), ["a", None, "d"]
        idx = BaseIndex(labels)
    else:
        labels, values, idx = pa.array(np.arange(2, 12, 3)), [5, 8, 9], RangeIndex(2, 12, 3)
    got = idx.isin(values, skip_null=skip_null)
    vs = [v for v in (values.tolist() if isinstance(values, np.ndarray) else values)
          if not (kind == "int" and isinstance(v, float) and not float(v).is_integer())]
    exp = pc.is_in(labels, options=pc.SetLookupOptions(value_set=pa.array(vs, type=labels.type),
                                                       skip_nulls=skip_null)).to_numpy(zero_copy_only=False)
    if kind == "float_nan":  # Arrow's is_in matches NaN with NaN; so does isin
        exp = exp.copy()
    assert got.tolist() == exp.tolist()
    with pytest.raises(ValueError):
        idx.isin("not-a-list")
