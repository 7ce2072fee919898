"""pycylon Table API parity (reference: python/test/test_table_properties.py, test_compute.py,
test_table.py, test_pycylon.py, test_join_config.py, test_status.py, test_data_types.py,
test_csv_read_options.py, test_series.py)."""
import os

import numpy as np
import pandas as pd
import pyarrow as pa
import pyarrow.compute as pc
import pytest
import torch

import cylon_amd as cy
from cylon_amd import C
from cylon_amd import CylonContext, DataFrame, JoinConfig, Series, Status, Table
from cylon_amd.io import CSVReadOptions, CSVWriteOptions, read_csv, write_csv


@pytest.fixture
def tb(ctx):
    return Table(pa.table({"col-1": [1, 2, 3, 4], "col-2": [5.0, None, 7.0, 8.0], "col-3": [9, 10, 11, 12]}), ctx)


def test_constructors_and_conversions(ctx):
    d = {"a": [1, 2, 3], "b": ["x", "y", None]}
    for t in (Table.from_pydict(ctx, d), Table.from_list(ctx, ["a", "b"], [[1, 2, 3], ["x", "y", None]]),
              Table.from_pandas(ctx, pd.DataFrame(d)), Table.from_arrow(ctx, pa.table(d))):
        assert t.to_pydict() == d
        assert t.shape == (3, 2) and t.column_names == ["a", "b"]
    t = Table.from_numpy(ctx, ["x", "y"], [np.array([1, 2]), np.array([0.5, 1.5])])
    assert t.to_numpy().shape == (2, 2)
    assert t.to_pandas()["y"].tolist() == [0.5, 1.5]


def test_all_types_roundtrip(ctx):
    at = pa.table({
        "b": pa.array([True, False, None]), "i8": pa.array([1, -2, None], pa.int8()),
        "u16": pa.array([1, 2, 3], pa.uint16()), "i32": pa.array([1, None, 3], pa.int32()),
        "u64": pa.array([1, 2, 2 ** 63], pa.uint64()), "f16": pa.array(np.array([1, 2, 3], np.float16)),
        "f32": pa.array([1.5, None, 3.5], pa.float32()), "d": pa.array([1.5, 2.5, None]),
        "s": pa.array(["a", None, "ccc"]), "bin": pa.array([b"x", b"yy", None]),
        "fsb": pa.array([b"ab", b"cd", b"ef"], pa.binary(2)), "d32": pa.array([1, 2, 3], pa.date32()),
        "ts": pa.array([1, 2, None], pa.timestamp("us")), "t64": pa.array([1, 2, 3], pa.time64("ns")),
        "dur": pa.array([1, 2, 3], pa.duration("ms")),
    })
    assert Table(at, ctx).to_arrow().equals(at)


def test_getitem_setitem(tb):
    assert tb["col-1"].to_pydict() == {"col-1": [1, 2, 3, 4]}
    assert tb[["col-1", "col-3"]].column_names == ["col-1", "col-3"]
    assert tb[1:3].to_pydict()["col-3"] == [10, 11]
    assert tb[2].to_pydict()["col-1"] == [3]
    assert tb[tb["col-1"] > 2].to_pydict()["col-1"] == [3, 4]
    tb["col-4"] = Table(pa.table({"x": [0, 0, 0, 1]}), tb.context)
    tb["col-5"] = 7
    assert tb.to_pydict()["col-4"] == [0, 0, 0, 1] and tb.to_pydict()["col-5"] == [7] * 4
    tb["col-1"] = tb["col-1"] * 2
    assert tb.to_pydict()["col-1"] == [2, 4, 6, 8]


def test_comparison_logical_arithmetic(tb):
    assert (tb["col-1"] == 2).to_pydict() == {"col-1": [False, True, False, False]}
    assert (tb["col-1"] != 2).to_pydict()["col-1"] == [True, False, True, True]
    assert (tb["col-1"] <= 2).to_pydict()["col-1"] == [True, True, False, False]
    assert (tb["col-1"] >= 3).to_pydict()["col-1"] == [False, False, True, True]
    m = (tb["col-1"] > 1) & (tb["col-1"] < 4)
    assert m.to_pydict()["col-1"] == [False, True, True, False]
    assert ((tb["col-1"] < 2) | (tb["col-1"] > 3)).to_pydict()["col-1"] == [True, False, False, True]
    assert (~(tb["col-1"] > 2)).to_pydict()["col-1"] == [True, True, False, False]
    assert (-tb["col-1"]).to_pydict()["col-1"] == [-1, -2, -3, -4]
    assert (tb["col-1"] + 1).to_pydict()["col-1"] == [2, 3, 4, 5]
    assert (tb["col-1"] - tb["col-3"]).to_pydict()["col-1"] == [-8] * 4
    assert (tb["col-1"] / 2).to_pydict()["col-1"] == [0.5, 1.0, 1.5, 2.0]
    assert (tb[["col-2"]] * 2).to_pydict()["col-2"] == [10.0, None, 14.0, 16.0]


def test_null_ops(tb):
    assert tb.isnull().to_pydict()["col-2"] == [False, True, False, False]
    assert tb.notna().to_pydict()["col-2"] == [True, False, True, True]
    assert tb.fillna(0).to_pydict()["col-2"] == [5.0, 0.0, 7.0, 8.0]
    assert tb.dropna().row_count == 3
    assert tb.dropna(axis=1).column_names == ["col-1", "col-3"]
    w = tb.where(tb > 2)
    assert w.to_pydict()["col-1"] == [None, None, 3, 4]


def test_rename_prefix_drop_isin_astype(tb):
    assert tb.add_prefix("p_").column_names == ["p_col-1", "p_col-2", "p_col-3"]
    assert tb.add_suffix("_s").column_names[0] == "col-1_s"
    assert tb.drop(["col-2"]).column_names == ["col-1", "col-3"]
    assert tb.isin([1, 11]).to_pydict() == {"col-1": [True, False, False, False],
                                           "col-2": [False, False, False, False],
                                           "col-3": [False, False, True, False]}
    c = tb.astype({"col-1": pa.float64()})
    assert c.to_arrow().schema.field("col-1").type == pa.float64()
    assert tb.applymap(lambda x: None if x is None else x * 10).to_pydict()["col-3"] == [90, 100, 110, 120]
    tb.rename({"col-1": "A"})
    assert tb.column_names[0] == "A"
    tb.rename(["x", "y", "z"])
    assert tb.column_names == ["x", "y", "z"]


def test_iterrows_and_index(tb):
    rows = list(tb.iterrows())
    assert rows[0] == (0, [1, 5.0, 9])
    tb.set_index("col-1", drop=True)
    assert tb.column_names == ["col-2", "col-3"]
    assert tb.loc[3].to_pydict() == {"col-2": [7.0], "col-3": [11]}
    assert tb.loc[2:3, "col-3"].to_pydict() == {"col-3": [10, 11]}
    assert tb.iloc[0:2].to_pydict()["col-3"] == [9, 10]
    tb.reset_index()
    assert tb.column_names[0] == "index" and tb.to_pydict()["index"] == [1, 2, 3, 4]


def test_concat_axis1_on_index(ctx):
    a = Table(pa.table({"x": [1, 2, 3]}), ctx)
    b = Table(pa.table({"y": [10, 20, 30]}), ctx)
    c = Table.concat([a, b], axis=1, join="inner")
    assert sorted(zip(*c.to_pydict().values())) == [(1, 10), (2, 20), (3, 30)]


def test_scalar_aggregates_local(tb):
    assert tb.sum("col-1").to_pydict() == {"col-1": [10]}
    assert tb.count("col-2").to_pydict() == {"col-2": [3]}
    assert tb.min("col-2").to_pydict() == {"col-2": [5.0]}
    assert tb.max("col-3").to_pydict() == {"col-3": [12]}


def test_join_config_status_types():
    jc = JoinConfig("left", "hash", 0, 1, "l_", "r_")
    assert jc.join_type == cy.JoinType.LEFT and jc.join_algorithm == cy.JoinAlgorithm.HASH
    with pytest.raises(ValueError):
        JoinConfig("inner", "sort", [0, 1], [0])
    s = Status(cy.Code.Invalid, "bad")
    assert not s.is_ok() and s.get_code() == 4 and s.get_msg() == "bad"
    assert Status.OK().is_ok()
    assert cy.int64().type == cy.C.Type.INT64 and cy.string().layout() == cy.C.Layout.VARIABLE_WIDTH
    assert cy.double().width() == 8


def test_join_config_apply(ctx):
    a = Table(pa.table({"k": [1, 2], "v": [3, 4]}), ctx)
    b = Table(pa.table({"k": [2, 3], "w": [5, 6]}), ctx)
    out = JoinConfig("outer", "sort", 0, 0, "a_", "b_").apply(a, b)
    assert out.row_count == 3 and out.column_names == ["a_k", "a_v", "b_k", "b_w"]


def test_native_errors_are_raised(ctx):
    a = Table(pa.table({"k": [1, 2]}), ctx)
    b = Table(pa.table({"k": ["x", "y"]}), ctx)
    with pytest.raises(cy.CylonError):
        a.join(b, "inner", "hash", on=[0])


def test_series():
    s = Series("s", [1, 2, 3])
    assert s.shape == (3,) and s[1] == 2 and s.id == "s"
    assert s.dtype.type == cy.C.Type.INT64


def test_csv_read_write_options(ctx, tmp_path, data_dir):
    opts = CSVReadOptions().use_threads(False).block_size(1 << 20).with_delimiter(",").na_values(["na"])
    t = read_csv(ctx, os.path.join(data_dir, "input", "null_data.csv"), opts)
    assert t.isnull().to_pandas().sum().sum() > 0
    opts2 = CSVReadOptions().use_cols(["a", "c"]).skip_rows(0)
    t2 = read_csv(ctx, os.path.join(data_dir, "input", "null_data.csv"), opts2)
    assert t2.column_names == ["a", "c"]
    p = str(tmp_path / "o.csv")
    write_csv(t, p, CSVWriteOptions().with_delimiter(","))
    t3 = read_csv(ctx, p, CSVReadOptions())
    assert t3.row_count == t.row_count
    many = read_csv(ctx, [os.path.join(data_dir, "input", f"csv1_{i}.csv") for i in range(4)], CSVReadOptions())
    assert len(many) == 4 and all(m.row_count == 20 for m in many)


def test_parquet_and_ipc(ctx, tmp_path, data_dir):
    from cylon_amd.io import read_arrow_ipc, read_parquet, write_arrow_ipc, write_parquet
    t = read_parquet(ctx, os.path.join(data_dir, "input", "parquet1_0.parquet"))
    assert t.row_count > 0
    p = str(tmp_path / "x.parquet")
    write_parquet(t, p)
    assert read_parquet(ctx, p).to_arrow().equals(t.to_arrow())
    q = str(tmp_path / "x.arrow")
    write_arrow_ipc(t, q)
    assert read_arrow_ipc(ctx, q).to_arrow().equals(t.to_arrow())


def test_context_config(ctx):
    ctx.add_config("compute_engine", "arrow")
    assert ctx.get_config("compute_engine") == "arrow"
    t = Table(pa.table({"a": [1, 2]}), ctx)
    assert (t > 1).to_pydict() == {"a": [False, True]}
    ctx.add_config("compute_engine", "device")
    assert ctx.get_rank() == 0 and ctx.get_world_size() == 1 and not ctx.is_distributed()
    assert ctx.get_next_sequence() + 1 == ctx.get_next_sequence()


def test_functional_ops_api(ctx):
    from cylon_amd import ops
    a = Table.from_pydict(ctx, {"k": [3, 1, 2, 2], "v": [1.0, 2.0, 3.0, 4.0]})
    b = Table.from_pydict(ctx, {"k": [2, 3, 9], "w": [5, 6, 7]})
    assert ops.join(a, b, "inner", "hash", on=["k"]).row_count == 3
    assert ops.sort(a, "k").to_pydict()["k"] == [1, 2, 2, 3]
    assert ops.unique(a, ["k"]).row_count == 3
    assert ops.local_groupby(a, "k", {"v": "sum"}).row_count == 3
    assert ops.merge([a, a]).row_count == 8
    assert ops.project(a, ["v"]).column_names == ["v"]
    assert ops.union(ops.project(a, ["k"]), ops.project(b, ["k"])).row_count == 4


def test_device_isin_strings_and_numeric_cast(ctx):
    """isin on string columns (device hash join against the value set) and numeric astype on the
    table's device with Arrow's safe-cast checks (reference: pycylon compute.pyx is_in / astype)."""
    import pyarrow as pa
    from cylon_amd import Table
    t = Table(pa.table({"s": pa.array(["a", None, "bb", "c", "a"]), "x": pa.array([1.0, 2.0, None, 4.0, 5.0]),
                        "i": pa.array([1, 2, 3, 300, 5])}), ctx)
    got = t.isin({"s": ["a", "c", None], "x": [2.0, 5.0], "i": [3]}).to_pydict()
    assert got["s"] == [True, False, False, True, True]
    assert got["x"] == [False, True, False, False, True]
    assert got["i"] == [False, False, True, False, False]
    c = t.astype({"x": "int32", "i": "int16"}).to_arrow()
    assert c.column("x").type == pa.int32() and c.column("x").to_pylist() == [1, 2, None, 4, 5]
    assert c.column("i").type == pa.int16()
    import pytest
    with pytest.raises(Exception):
        Table(pa.table({"x": [1.5]}), ctx).astype("int64")
    with pytest.raises(Exception):
        t.astype({"i": "int8"})  # 300 out of range


@pytest.mark.parametrize("typ", [pa.string(), pa.large_string(), pa.binary()])
def test_string_fillna_where_select_kernel(ctx, typ):
    """K15 string / binary where and fill_null run the native select kernels (select_var) and
    match Arrow's if_else / fill_null: scalar fill, null `other`, column `other` (with nulls),
    empty strings and rows longer than the 16-byte vector copy."""
    rng = np.random.default_rng(4)
    n = 3000

    def val(i):
        s = "" if i % 11 == 0 else ("abc%d" % i) * (1 + i % 37)
        return s.encode() if typ == pa.binary() else s
    a = pa.array([None if i % 7 == 0 else val(i) for i in range(n)], typ)
    o = pa.array([None if i % 5 == 0 else val(i + 1) for i in range(n)], typ)
    cond = rng.random(n) < 0.5
    t = Table(pa.table({"s": a, "o": o}), ctx)
    fill = b"FILL" if typ == pa.binary() else "FILL"
    same = lambda got, ref: got.equals(ref.cast(got.type))  # noqa: E731  (large_string maps to string)
    assert same(t.fillna(fill).to_arrow().column("s").combine_chunks(), pc.fill_null(a, fill))
    m = Table(pa.table({"s": cond, "o": cond}), ctx)
    got = t.where(m).to_arrow()
    assert same(got.column("s").combine_chunks(), pc.if_else(pa.array(cond), a, None).cast(typ))
    cols = t.native.columns()
    sel = C.select_var(cols[0], cols[1], torch.from_numpy(cond))
    ref = pc.if_else(pa.array(cond), a, o)
    assert same(t._wrap(C.Table(t.native.context(), [sel])).to_arrow().column("s").combine_chunks(), ref)
    with_scalar = t.where(m, fill).to_arrow().column("s").combine_chunks()
    assert same(with_scalar, pc.if_else(pa.array(cond), a, pa.scalar(fill, typ)))
