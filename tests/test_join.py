"""Join tests: local joins vs a pandas oracle, and the reference's distributed
golden files (cpp/test/join_test.cpp, data/output/join_inner_{world}_{rank}.csv)."""
import os

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

from cylon_amd import Table
from cylon_amd.io import CSVReadOptions, read_csv

from dist_utils import run_distributed

JOIN_TYPES = ["inner", "left", "right", "outer"]


def _canon(df: pd.DataFrame):
    rows = [tuple(None if (isinstance(v, float) and np.isnan(v)) or v is None or v is pd.NA else v
                  for v in r) for r in df.itertuples(index=False)]
    return sorted(rows, key=lambda r: tuple((x is None, str(type(x)), x if x is not None else 0) for x in r))


def _oracle(a: pd.DataFrame, b: pd.DataFrame, how, lk, rk, lp="l_", rp="r_"):
    a2 = a.add_prefix(lp)
    b2 = b.add_prefix(rp)
    return a2.merge(b2, left_on=[lp + k for k in lk], right_on=[rp + k for k in rk], how=how)


@pytest.mark.parametrize("algorithm", ["hash", "sort"])
@pytest.mark.parametrize("how", JOIN_TYPES)
def test_single_key_int(ctx, algorithm, how):
    rng = np.random.default_rng(1)
    a = pd.DataFrame({"k": rng.integers(-20, 60, 500), "v": rng.random(500)})
    b = pd.DataFrame({"k": rng.integers(0, 80, 300), "w": rng.integers(0, 9, 300)})
    out = Table.from_pandas(ctx, a).join(Table.from_pandas(ctx, b), how, algorithm, on=["k"], left_prefix="l_",
                                         right_prefix="r_").to_pandas()
    ref = _oracle(a, b, how, ["k"], ["k"])
    assert list(out.columns) == ["l_k", "l_v", "r_k", "r_w"]
    assert _canon(out) == _canon(ref[out.columns])


@pytest.mark.parametrize("algorithm", ["hash", "sort"])
@pytest.mark.parametrize("how", JOIN_TYPES)
def test_multi_key_and_strings(ctx, algorithm, how):
    rng = np.random.default_rng(2)
    n, m = 400, 250
    a = pd.DataFrame({"k1": rng.integers(0, 6, n), "k2": [f"s{x}" for x in rng.integers(0, 7, n)],
                      "v": rng.random(n)})
    b = pd.DataFrame({"k1": rng.integers(0, 6, m), "k2": [f"s{x}" for x in rng.integers(0, 7, m)],
                      "w": [f"p{x}" for x in range(m)]})
    out = Table.from_pandas(ctx, a).join(Table.from_pandas(ctx, b), how, algorithm, on=["k1", "k2"],
                                         left_prefix="l_", right_prefix="r_").to_pandas()
    ref = _oracle(a, b, how, ["k1", "k2"], ["k1", "k2"])
    assert _canon(out) == _canon(ref[out.columns])


def test_float_and_mixed_width_keys(ctx):
    a = pa.table({"k": pa.array([1, 2, 3, -4], pa.int32()), "x": [1.5, 2.5, 3.5, 4.5]})
    b = pa.table({"k": pa.array([3, 1, -4, 9, 1], pa.int64()), "y": [0.25, -0.0, 0.0, 1.0, 2.0]})
    out = Table(a, ctx).join(Table(b, ctx), "inner", "hash", left_on=[0], right_on=[0]).to_pandas()
    assert sorted(out["k"].iloc[:, 0].tolist()) == [-4, 1, 1, 3]
    fa = pa.table({"f": [0.0, 1.5, float("nan")]})
    fb = pa.table({"f": [-0.0, 1.5, 2.0]})
    out = Table(fa, ctx).join(Table(fb, ctx), "inner", "hash", on=[0], left_prefix="a", right_prefix="b")
    assert out.row_count == 2


def test_null_keys_match_each_other(ctx):
    a = pa.table({"k": pa.array([1, None, 3]), "v": [1, 2, 3]})
    b = pa.table({"k": pa.array([None, 3, 4]), "w": [7, 8, 9]})
    out = Table(a, ctx).join(Table(b, ctx), "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")
    d = out.to_pandas()
    assert sorted(d["l_v"].tolist()) == [2, 3]


def test_empty_tables(ctx):
    a = pa.table({"k": pa.array([], pa.int64()), "v": pa.array([], pa.float64())})
    b = pa.table({"k": pa.array([1, 2], pa.int64()), "w": pa.array([1.0, 2.0])})
    for how in JOIN_TYPES:
        out = Table(a, ctx).join(Table(b, ctx), how, "hash", on=[0], left_prefix="l_", right_prefix="r_")
        expect = 2 if how in ("right", "outer") else 0
        assert out.row_count == expect


# --------------------------------------------------------------------------
# distributed golden files (partition-sensitive: validates bit-exact K1 hashing)
# --------------------------------------------------------------------------
def _golden_join(ctx, data_dir, algorithm):
    rank, world = ctx.get_rank(), ctx.get_world_size()
    opts = CSVReadOptions().use_threads(False).with_column_types({"0": pa.int64(), "1": pa.float64()})
    t1 = read_csv(ctx, os.path.join(data_dir, "input", f"csv1_{rank}.csv"), opts)
    t2 = read_csv(ctx, os.path.join(data_dir, "input", f"csv2_{rank}.csv"), opts)
    exp_opts = CSVReadOptions().use_threads(False)
    exp = pa.csv.read_csv(os.path.join(data_dir, "output", f"join_inner_{world}_{rank}.csv"))
    res = t1.distributed_join(t2, "inner", algorithm, on=[0])
    got = res.to_pandas()
    got_rows = sorted(tuple(round(float(x), 6) for x in r) for r in got.itertuples(index=False))
    exp_rows = sorted(tuple(round(float(x), 6) for x in r) for r in exp.to_pandas().itertuples(index=False))
    return got_rows == exp_rows, len(got_rows), len(exp_rows)


@pytest.mark.parametrize("world", [1, 2, 4])
@pytest.mark.parametrize("algorithm", ["hash", "sort"])
def test_distributed_join_golden(data_dir, world, algorithm):
    import pyarrow.csv  # noqa: F401
    res = run_distributed(_golden_join, world, data_dir, algorithm)
    for ok, got, exp in res:
        assert ok, f"rows got={got} expected={exp}"


@pytest.mark.parametrize("world", [2, 4])
def test_distributed_join_golden_native_tcp(data_dir, world):
    """Same golden files with the context brought up natively (TCPConfig: C++ bootstrap over a
    TCPStore, native TCP mesh transport; no torch.distributed process group)."""
    import pyarrow.csv  # noqa: F401
    res = run_distributed(_golden_join, world, data_dir, "hash", env={"CYLON_TEST_COMM": "tcp"})
    for ok, got, exp in res:
        assert ok, f"rows got={got} expected={exp}"


def _dist_vs_oracle(ctx, how, algorithm):
    rank, world = ctx.get_rank(), ctx.get_world_size()
    rng = np.random.default_rng(100 + rank)
    a = pd.DataFrame({"k": rng.integers(0, 40, 150), "s": [f"x{v}" for v in rng.integers(0, 5, 150)]})
    b = pd.DataFrame({"k": rng.integers(0, 40, 120), "v": rng.random(120)})
    out = Table.from_pandas(ctx, a).distributed_join(Table.from_pandas(ctx, b), how, algorithm, on=["k"],
                                                     left_prefix="l_", right_prefix="r_")
    return out.to_pandas(), a, b


@pytest.mark.parametrize("how", JOIN_TYPES)
def test_distributed_join_all_types(how):
    res = run_distributed(_dist_vs_oracle, 2, how, "hash")
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    ref = _oracle(a, b, how, ["k"], ["k"])
    assert _canon(got) == _canon(ref[got.columns])


def _golden_join_chunked(ctx, data_dir, algorithm, chunks):
    ctx.add_config("shuffle_chunks", str(chunks))
    return _golden_join(ctx, data_dir, algorithm)


@pytest.mark.parametrize("world", [2, 4])
@pytest.mark.parametrize("chunks", [2, 3])
def test_distributed_join_chunked_golden(data_dir, world, chunks):
    """Pipelined (chunked) shuffle: every rank ends with exactly the reference's per-rank join rows."""
    res = run_distributed(_golden_join_chunked, world, data_dir, "hash", chunks)
    for ok, got, exp in res:
        assert ok, f"rows got={got} expected={exp}"


def _dist_chunked_vs_oracle(ctx, how, algorithm, chunks):
    ctx.add_config("shuffle_chunks", str(chunks))
    rank = ctx.get_rank()
    rng = np.random.default_rng(300 + rank)
    a = pd.DataFrame({"k": rng.integers(0, 60, 400), "x": rng.integers(0, 9, 400).astype(np.int32),
                      "f": rng.random(400)})
    a.loc[a.index % 7 == 0, "f"] = np.nan  # nullable payload
    b = pd.DataFrame({"k": rng.integers(0, 60, 300), "v": rng.random(300)})
    from cylon_amd._lib import C
    C.trace_enable(True)
    out = Table.from_pandas(ctx, a).distributed_join(Table.from_pandas(ctx, b), how, algorithm, on=["k"],
                                                     left_prefix="l_", right_prefix="r_")
    assert C.trace_counters().get("shuffle.chunks") == chunks
    C.trace_enable(False)
    return out.to_pandas(), a, b


@pytest.mark.parametrize("how", JOIN_TYPES)
@pytest.mark.parametrize("algorithm", ["hash", "sort"])
def test_distributed_join_chunked_all_types(how, algorithm):
    res = run_distributed(_dist_chunked_vs_oracle, 2, how, algorithm, 4)
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    ref = _oracle(a, b, how, ["k"], ["k"])
    assert _canon(got) == _canon(ref[got.columns])


def _narrow_join(ctx, chunks):
    from cylon_amd._lib import C
    ctx.add_config("shuffle_chunks", str(chunks))
    rank = ctx.get_rank()
    rng = np.random.default_rng(40 + rank)
    n = 500
    # key: negative, range < 2^32 (narrowed); w: range > 2^32 (not narrowed); z: nullable, narrowed
    a = pd.DataFrame({"k": rng.integers(-2_000_000_000, -1_999_999_900, n),
                      "w": rng.integers(-(1 << 60), 1 << 60, n),
                      "z": pd.array(rng.integers(5, 50, n), dtype="Int64")})
    a.loc[a.index % 5 == 0, "z"] = pd.NA
    b = pd.DataFrame({"k": rng.integers(-2_000_000_000, -1_999_999_900, n // 2), "v": rng.random(n // 2)})
    if rank == 1:
        b = b.iloc[:0]  # an empty relation on one rank
    C.trace_enable(True)
    C.trace_reset()
    out = Table.from_pandas(ctx, a).distributed_join(Table.from_pandas(ctx, b), "inner", "hash", on=["k"],
                                                     left_prefix="l_", right_prefix="r_")
    narrowed = C.trace_counters().get("shuffle.narrowed_columns", 0)
    C.trace_enable(False)
    return out.to_pandas(), a, b, narrowed


@pytest.mark.parametrize("chunks", [1, 2])
def test_distributed_join_narrowed_wire(chunks):
    """int64 columns with a global range < 2^32 travel as uint32 offsets (negative values, nulls, an empty
    rank); wider columns travel as is; the result is exact."""
    res = run_distributed(_narrow_join, 2, chunks)
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    ref = _oracle(a, b, "inner", ["k"], ["k"])
    assert len(got) == len(ref) > 0
    assert _canon(got) == _canon(ref[got.columns])
    assert all(r[3] == 3 for r in res)  # l.k, l.z, r.k (l.w spans > 2^32)


@pytest.mark.parametrize("how", JOIN_TYPES)
def test_global_hash_join_hot_keys_directory(ctx, how):
    """The global-table join's directory holds each distinct build key once (ops/join.cpp
    hash_join_pairs): hot keys with thousands of duplicates on both sides, next to unique keys."""
    from cylon_amd._lib import C
    rng = np.random.default_rng(9)
    n = 20_000
    ka = rng.integers(0, 5_000, n)
    kb = rng.integers(0, 5_000, n)
    ka[rng.random(n) < 0.02] = 77  # ~400 x ~3000 rows of key 77
    kb[rng.random(n) < 0.15] = 77
    kb[rng.random(n) < 0.05] = -3  # only on the build side
    a = pd.DataFrame({"k": ka, "v": rng.random(n)})
    b = pd.DataFrame({"k": kb[: n // 2], "w": rng.random(n // 2)})
    C.trace_enable(True)
    C.trace_reset()
    out = Table.from_pandas(ctx, a).join(Table.from_pandas(ctx, b), how, "hash", on=["k"], left_prefix="l_",
                                         right_prefix="r_").to_pandas()
    c = dict(C.trace_counters())
    C.trace_enable(False)
    ref = _oracle(a, b, how, ["k"], ["k"])
    assert len(out) == len(ref)
    assert _canon(out) == _canon(ref[out.columns])
