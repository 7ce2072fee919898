"""list<numeric> and fixed_size_list<numeric> columns (reference: cpp/src/cylon/arrow/arrow_types.cpp:83-111
validates them, util/copy_arrray.cpp:113-139,222-281 gathers them): they travel through gather, sort,
join materialisation, set operations and the distributed shuffle like binary values."""
import numpy as np
import pyarrow as pa
import pytest

from cylon_amd import Table

from dist_utils import run_distributed


def _lists(rng, n, nullable=True):
    lens = rng.integers(0, 4, n)
    vals = [list(map(int, rng.integers(-9, 9, L))) for L in lens]
    mask = (rng.random(n) < 0.15) if nullable else np.zeros(n, bool)
    return pa.array([None if m else v for v, m in zip(vals, mask)], pa.list_(pa.int32()))


def _fsl(rng, n):
    vals = rng.standard_normal((n, 3))
    mask = rng.random(n) < 0.1
    return pa.array([None if m else list(map(float, v)) for v, m in zip(vals, mask)], pa.list_(pa.float64(), 3))


def _key(row):
    return tuple(tuple(x) if isinstance(x, list) else x for x in row)


def _rows(t: pa.Table):
    return sorted((_key(r) for r in zip(*[t.column(i).to_pylist() for i in range(t.num_columns)])),
                  key=lambda r: repr(r))


def test_list_roundtrip_and_types(ctx):
    rng = np.random.default_rng(1)
    t = pa.table({"k": pa.array(rng.integers(0, 50, 300)), "l": _lists(rng, 300), "f": _fsl(rng, 300)})
    T = Table(t, ctx)
    back = T.to_arrow()
    assert back.column("l").type == pa.list_(pa.int32())
    assert back.column("f").type == pa.list_(pa.float64(), 3)
    assert back.column("l").to_pylist() == t.column("l").to_pylist()
    assert back.column("f").to_pylist() == t.column("f").to_pylist()
    with pytest.raises(Exception):
        Table(pa.table({"x": pa.array([[1, None]], pa.list_(pa.int64()))}), ctx)  # null elements in a valid row
    with pytest.raises(Exception):
        Table(pa.table({"x": pa.array([["a"]], pa.list_(pa.string()))}), ctx)  # non-numeric elements


def _oracle_join(a, b, how, acols, bcols):
    """pandas merge on the key with row ids, then the python values of every column."""
    import pandas as pd
    da = pd.DataFrame({"k": a.column("k").to_pylist(), "ra": range(a.num_rows)})
    db = pd.DataFrame({"k": b.column("k").to_pylist(), "rb": range(b.num_rows)})
    m = da.merge(db, on="k", how=how)
    av = {c: a.column(c).to_pylist() for c in acols}
    bv = {c: b.column(c).to_pylist() for c in bcols}
    out = []
    for ra, rb in zip(m["ra"], m["rb"]):
        left = [None if pd.isna(ra) else av[c][int(ra)] for c in acols]
        right = [None if pd.isna(rb) else bv[c][int(rb)] for c in bcols]
        out.append(_key(left + right))
    return sorted(out, key=repr)


@pytest.mark.parametrize("how", ["inner", "left", "outer"])
def test_list_columns_through_join(ctx, how):
    rng = np.random.default_rng(2)
    a = pa.table({"k": pa.array(rng.integers(0, 40, 200)), "l": _lists(rng, 200)})
    b = pa.table({"k": pa.array(rng.integers(0, 40, 150)), "f": _fsl(rng, 150)})
    got = Table(a, ctx).join(Table(b, ctx), how, "hash", on=["k"], left_prefix="l_", right_prefix="r_").to_arrow()
    g = _rows(got.select(["l_k", "l_l", "r_k", "r_f"]))
    assert g == _oracle_join(a, b, how, ["k", "l"], ["k", "f"])


def test_list_columns_sort_and_setops(ctx):
    rng = np.random.default_rng(3)
    a = pa.table({"k": pa.array(rng.integers(0, 10, 120)), "l": _lists(rng, 120, nullable=False)})
    T = Table(a, ctx)
    s = T.sort("k").to_arrow()
    order = np.argsort(a.column("k").to_numpy(), kind="stable")
    assert s.column("l").to_pylist() == [a.column("l").to_pylist()[i] for i in order]
    u = T.union(T).to_arrow()
    assert len(_rows(u)) == len(set(_rows(a)))


def _dist_lists(ctx):
    rng = np.random.default_rng(20 + ctx.get_rank())
    a = pa.table({"k": pa.array(rng.integers(0, 30, 150)), "l": _lists(rng, 150), "f": _fsl(rng, 150)})
    b = pa.table({"k": pa.array(rng.integers(0, 30, 100)), "w": pa.array(rng.random(100))})
    out = Table(a, ctx).distributed_join(Table(b, ctx), "inner", "hash", on=["k"], left_prefix="l_",
                                         right_prefix="r_").to_arrow()
    return out, a, b


def test_list_columns_distributed_join():
    res = run_distributed(_dist_lists, 2)
    got = pa.concat_tables([r[0] for r in res])
    a = pa.concat_tables([r[1] for r in res])
    b = pa.concat_tables([r[2] for r in res])
    g = _rows(got.select(["l_k", "l_l", "l_f", "r_k", "r_w"]))
    assert g == _oracle_join(a, b, "inner", ["k", "l", "f"], ["k", "w"])


@pytest.mark.gpu
@pytest.mark.parametrize("how", ["inner", "outer"])
def test_list_columns_join_on_device(gpu_ctx, how):
    rng = np.random.default_rng(5)
    a = pa.table({"k": pa.array(rng.integers(0, 400, 3000)), "l": _lists(rng, 3000)})
    b = pa.table({"k": pa.array(rng.integers(0, 400, 2000)), "f": _fsl(rng, 2000)})
    got = Table(a, gpu_ctx).join(Table(b, gpu_ctx), how, "hash", on=["k"], left_prefix="l_",
                                 right_prefix="r_").to_arrow()
    assert _rows(got.select(["l_k", "l_l", "r_k", "r_f"])) == _oracle_join(a, b, how, ["k", "l"], ["k", "f"])


@pytest.mark.gpu
def test_list_columns_distributed_join_on_device():
    res = run_distributed(_dist_lists, 2, device="cuda:0")
    got = pa.concat_tables([r[0] for r in res])
    a = pa.concat_tables([r[1] for r in res])
    b = pa.concat_tables([r[2] for r in res])
    assert _rows(got.select(["l_k", "l_l", "l_f", "r_k", "r_w"])) == _oracle_join(a, b, "inner", ["k", "l", "f"],
                                                                                 ["k", "w"])


def test_list_columns_native_parquet_roundtrip(ctx, tmp_path):
    """The C++ Parquet writer / reader (io/arrow_io.cpp) map list and fixed-size-list columns.
    (Fixed-size lists without null rows: Arrow's own Parquet round trip of a null fixed-size
    list row fails, pyarrow 25 included.)"""
    import pyarrow.parquet as pq
    from cylon_amd.io import read_parquet, write_parquet
    rng = np.random.default_rng(9)
    f = pa.array([list(map(float, v)) for v in rng.standard_normal((80, 3))], pa.list_(pa.float64(), 3))
    t = pa.table({"k": pa.array(rng.integers(0, 9, 80)), "l": _lists(rng, 80), "f": f})
    p = tmp_path / "lists.parquet"
    write_parquet(Table(t, ctx), str(p))
    assert pq.read_table(p).column("l").to_pylist() == t.column("l").to_pylist()
    back = read_parquet(ctx, str(p)).to_arrow()
    assert back.column("l").to_pylist() == t.column("l").to_pylist()
    assert back.column("f").to_pylist() == t.column("f").to_pylist()
