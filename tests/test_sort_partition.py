"""Sorting and partitioning tests (reference: cpp/test/partition_test.cpp,
sorting_test.cpp, quick_sort_test.cpp)."""
import struct

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest
import torch

from cylon_amd import C, SortOptions, Table

from dist_utils import run_distributed


def murmur3_32(data: bytes, seed: int = 0) -> int:
    """Plain-python MurmurHash3_x86_32 oracle."""
    c1, c2 = 0xCC9E2D51, 0x1B873593
    h = seed
    n = len(data)
    for i in range(0, n - n % 4, 4):
        k = struct.unpack_from("<I", data, i)[0]
        k = (k * c1) & 0xFFFFFFFF
        k = ((k << 15) | (k >> 17)) & 0xFFFFFFFF
        k = (k * c2) & 0xFFFFFFFF
        h ^= k
        h = ((h << 13) | (h >> 19)) & 0xFFFFFFFF
        h = (h * 5 + 0xE6546B64) & 0xFFFFFFFF
    tail = data[n - n % 4:]
    k = 0
    if len(tail) >= 3:
        k ^= tail[2] << 16
    if len(tail) >= 2:
        k ^= tail[1] << 8
    if len(tail) >= 1:
        k ^= tail[0]
        k = (k * c1) & 0xFFFFFFFF
        k = ((k << 15) | (k >> 17)) & 0xFFFFFFFF
        k = (k * c2) & 0xFFFFFFFF
        h ^= k
    h ^= n
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    h ^= h >> 16
    return h


@pytest.mark.parametrize("nparts", [1, 2, 3, 4, 7, 8, 16])
def test_modulo_partition_spec(ctx, nparts):
    # partition_test.cpp:32-53: int keys -> (uint32)v % P
    vals = np.arange(-50, 200, dtype=np.int64)
    t = Table(pa.table({"v": vals}), ctx)
    pid, counts = C.map_to_hash_partitions(t.native, [0], nparts)
    exp = (vals.astype(np.uint32) % nparts)
    assert np.array_equal(pid.numpy().astype(np.uint32), exp)
    assert counts == np.bincount(exp, minlength=nparts).tolist()


@pytest.mark.parametrize("nparts", [2, 5, 8])
def test_murmur_partition_spec(ctx, nparts):
    # partition_test.cpp:55-79: doubles -> MurmurHash3_x86_32(&v, 8, 0) % P
    vals = np.random.default_rng(3).normal(size=300)
    t = Table(pa.table({"d": vals, "s": [f"str{i}" for i in range(300)]}), ctx)
    pid, _ = C.map_to_hash_partitions(t.native, [0], nparts)
    exp = [murmur3_32(struct.pack("<d", v)) % nparts for v in vals]
    assert pid.numpy().astype(np.uint32).tolist() == exp
    pid, _ = C.map_to_hash_partitions(t.native, [1], nparts)
    exp = [murmur3_32(f"str{i}".encode()) % nparts for i in range(300)]
    assert pid.numpy().astype(np.uint32).tolist() == exp
    # multi-column chain: h = 31 * h + f(v)
    pid, _ = C.map_to_hash_partitions(t.native, [0, 1], nparts)
    exp = [((31 * murmur3_32(struct.pack("<d", v))) + murmur3_32(f"str{i}".encode())) % (1 << 32) % nparts
           for i, v in enumerate(vals)]
    assert pid.numpy().astype(np.uint32).tolist() == exp


def test_split_is_stable(ctx):
    t = Table(pa.table({"k": np.arange(1000) % 7, "i": np.arange(1000)}), ctx)
    parts = t.hash_partition(["k"], 4)
    for p in parts:
        assert np.all(np.diff(p.to_pandas()["i"].to_numpy()) > 0)
    assert sum(p.row_count for p in parts) == 1000


@pytest.mark.parametrize("asc", [True, False])
def test_local_sort_vs_pandas(ctx, asc):
    rng = np.random.default_rng(0)
    n = 3000
    df = pd.DataFrame({"a": rng.integers(-5, 5, n), "b": rng.normal(size=n), "s": [f"s{x % 13}" for x in range(n)],
                       "i": np.arange(n)})
    t = Table.from_pandas(ctx, df)
    for cols in (["a"], ["a", "b"], ["s", "a"], ["b"]):
        got = t.sort(cols, ascending=asc).to_pandas()
        exp = df.sort_values(cols, ascending=asc, kind="stable").reset_index(drop=True)
        pd.testing.assert_frame_equal(got, exp)
    got = t.sort(["a", "s"], ascending=[True, False]).to_pandas()
    exp = df.sort_values(["a", "s"], ascending=[True, False], kind="stable").reset_index(drop=True)
    pd.testing.assert_frame_equal(got, exp)


def test_sort_nulls_last(ctx):
    t = Table(pa.table({"a": pa.array([3, None, 1, None, 2])}), ctx)
    assert t.sort("a").to_pydict()["a"] == [1, 2, 3, None, None]
    assert t.sort("a", ascending=False).to_pydict()["a"] == [3, 2, 1, None, None]


def _dist_sort(ctx, asc):
    rng = np.random.default_rng(ctx.get_rank())
    n = 2000
    df = pd.DataFrame({"a": rng.integers(0, 10000, n), "b": rng.random(n)})
    t = Table.from_pandas(ctx, df)
    s = t.distributed_sort(["a", "b"], ascending=asc, sort_options=SortOptions(num_bins=0, num_samples=0))
    total = s.count("a").to_pydict()["a"][0]
    return s.to_pandas(), df, total


@pytest.mark.parametrize("asc", [True, False])
def test_distributed_sort_global_order(asc):
    world = 4
    res = run_distributed(_dist_sort, world, asc)
    parts = [r[0] for r in res]
    allin = pd.concat([r[1] for r in res])
    for r in res:
        assert r[2] == len(allin)  # row count preserved (distributed Count)
    got = pd.concat(parts).reset_index(drop=True)
    exp = allin.sort_values(["a", "b"], ascending=asc).reset_index(drop=True)
    pd.testing.assert_frame_equal(got, exp)


def test_range_partition_monotonic(ctx):
    vals = np.random.default_rng(1).integers(0, 1 << 40, 5000)
    t = Table(pa.table({"v": vals}), ctx)
    pid, counts = C.map_to_sort_partitions(t.native, 0, 4, True, 0, 0)
    pid = pid.numpy().astype(np.int64)
    order = np.argsort(vals, kind="stable")
    assert np.all(np.diff(pid[order]) >= 0)
    assert sum(counts) == 5000


def _dist_sort_case(ctx, case):
    rank = ctx.get_rank()
    rng = np.random.default_rng(40 + rank)
    n = 3000 + 500 * rank
    if case == "wide_int64":  # keys spanning +-2^62 (beyond double precision)
        a = rng.integers(-(1 << 62), 1 << 62, n, dtype=np.int64)
        a[: n // 10] = (1 << 62) + np.arange(n // 10)  # neighbours 1 apart near 2^62
        df = pd.DataFrame({"a": a, "i": np.arange(n) + 100000 * rank})
        cols, asc = ["a"], True
    elif case == "one_key":  # every row the same key: balance must come from the tie-break
        df = pd.DataFrame({"a": np.full(n, 7, dtype=np.int64), "i": np.arange(n) + 100000 * rank})
        cols, asc = ["a"], True
    elif case == "skew_desc":  # 90% of the rows on one key, descending
        a = np.where(rng.random(n) < 0.9, 123, rng.integers(0, 1000, n)).astype(np.int64)
        df = pd.DataFrame({"a": a, "i": np.arange(n) + 100000 * rank})
        cols, asc = ["a"], False
    elif case == "multi_nulls":  # two sort columns, nulls in the first, float second
        a = pd.array(rng.integers(0, 20, n), dtype="Int64")
        a[rng.random(n) < 0.1] = pd.NA
        df = pd.DataFrame({"a": a, "b": rng.standard_normal(n), "i": np.arange(n) + 100000 * rank})
        cols, asc = ["a", "b"], [True, False]
    t = Table.from_pandas(ctx, df)
    s = t.distributed_sort(cols, ascending=asc)
    return s.to_pandas(), df, cols, asc


@pytest.mark.parametrize("case", ["wide_int64", "one_key", "skew_desc", "multi_nulls"])
def test_distributed_sort_exact_splitters(case):
    """Exact composite-key splitters: global order equals a stable sort of the rank-ordered
    concatenation (ties keep input order across ranks), and per-rank loads stay within 1.5x
    of the mean even when one key holds every row (reference: table.cpp:338-382)."""
    world = 4
    res = run_distributed(_dist_sort_case, world, case)
    cols, asc = res[0][2], res[0][3]
    allin = pd.concat([r[1] for r in res]).reset_index(drop=True)
    got = pd.concat([r[0] for r in res]).reset_index(drop=True)
    exp = allin.sort_values(cols, ascending=asc, kind="mergesort", na_position="last").reset_index(drop=True)
    assert len(got) == len(exp)
    pd.testing.assert_frame_equal(got.astype(exp.dtypes.to_dict()), exp, check_dtype=False)
    loads = [len(r[0]) for r in res]
    assert max(loads) <= 1.5 * len(allin) / world, loads


def test_verify_sort_config_cpu(ctx):
    """config verify_sort=1 on the CPU engine: sorted results pass the order-image check."""
    import numpy as np
    import pyarrow as pa
    from cylon_amd import Table
    from cylon_amd._lib import C
    rng = np.random.default_rng(3)
    t = Table(pa.table({"k": pa.array(rng.standard_normal(5000), mask=rng.random(5000) < 0.05),
                        "i": rng.integers(0, 9, 5000)}), ctx)
    ctx.add_config("verify_sort", "1")
    C.trace_enable(True)
    C.trace_reset()
    try:
        t.sort("k")
        t.sort(["i", "k"], ascending=[False, True])
        c = dict(C.trace_counters())
    finally:
        ctx.add_config("verify_sort", "0")
        C.trace_enable(False)
    assert c.get("sort.verified", 0) == 2


def _pipelined_sort_case(ctx, chunks, delay_us, asc):
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    if delay_us:
        ctx._ctx.use_async_delay_transport(delay_us)
    if chunks:
        ctx.add_config("sort_chunks", str(chunks))
    rng = np.random.default_rng(70 + rank)
    n = 4000 + 700 * rank
    a = rng.integers(-(1 << 40), 1 << 40, n, dtype=np.int64)
    a[: n // 5] = 17  # a heavy tie: balance and stability come from the global row tie-break
    df = pd.DataFrame({"a": a, "x": rng.standard_normal(n), "i": np.arange(n) + 100000 * rank})
    C.trace_enable(True)
    C.trace_reset()
    s = Table.from_pandas(ctx, df).distributed_sort("a", ascending=asc)
    return s.to_pandas(), df, dict(C.trace_counters())


@pytest.mark.parametrize("world,chunks,delay_us,asc", [(3, 3, 0, True), (4, 1, 0, False), (2, 4, 300.0, True)])
def test_pipelined_distributed_sort(world, chunks, delay_us, asc):
    """Sort locally, split by exact (image, global row) splitters into contiguous ranges, exchange
    K key sub-range chunks (one plan all-gather), merge each chunk's W sorted runs with the merge
    path kernel: the result equals a stable sort of the rank-ordered concatenation, also over
    the asynchronous delay transport (chunk k merges while chunk k+1 is in flight)."""
    res = run_distributed(_pipelined_sort_case, world, chunks, delay_us, asc)
    allin = pd.concat([r[1] for r in res]).reset_index(drop=True)
    got = pd.concat([r[0] for r in res]).reset_index(drop=True)
    exp = allin.sort_values("a", ascending=asc, kind="mergesort").reset_index(drop=True)
    pd.testing.assert_frame_equal(got, exp, check_dtype=False)
    for r in res:
        c = r[2]
        assert c.get("sort.dist.pipelined", 0) == 1
        assert c.get("shuffle.chunks", 0) == chunks
        assert c.get("shuffle.plan_collectives", 0) == 1
        assert c.get("sort.dist.merge_rounds", 0) >= 1  # every chunk receives >= 2 non-empty runs here
    loads = [len(r[0]) for r in res]
    assert max(loads) <= 1.5 * len(allin) / world, loads


def _one_rank_nulls_case(ctx):
    import pyarrow as pa
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    rng = np.random.default_rng(90 + rank)
    n = 3000 + 500 * rank
    a = rng.integers(-1000, 1000, n)
    # only rank 1's key column carries a validity tensor (with nulls): every rank must still
    # take the same sort path (the pipelined sort's eligibility is agreed across ranks)
    arr = pa.array(a, mask=(rng.random(n) < 0.1)) if rank == 1 else pa.array(a)
    t = Table(pa.table({"a": arr, "i": np.arange(n) + 100000 * rank}), ctx)
    C.trace_enable(True)
    C.trace_reset()
    s = t.distributed_sort("a")
    return s.to_pandas(), t.to_pandas(), dict(C.trace_counters())


def test_distributed_sort_nulls_on_one_rank_only():
    """a key column nullable on one rank only must not split the ranks between
    the pipelined and the splitter sort (different collectives: a hang).  Result: globally sorted,
    nulls last, every row once, and no rank took the pipelined path."""
    res = run_distributed(_one_rank_nulls_case, 3)
    allin = pd.concat([r[1] for r in res]).reset_index(drop=True)
    got = pd.concat([r[0] for r in res]).reset_index(drop=True)
    assert len(got) == len(allin)
    assert sorted(got["i"].tolist()) == sorted(allin["i"].tolist())
    keys = got["a"].tolist()
    nn = [k for k in keys if not pd.isna(k)]
    assert nn == sorted(nn)
    first_null = next((j for j, k in enumerate(keys) if pd.isna(k)), len(keys))
    assert all(pd.isna(k) for k in keys[first_null:])
    for r in res:
        assert r[2].get("sort.dist.pipelined", 0) == 0


@pytest.mark.parametrize("nruns", [1, 2, 3, 8])
def test_merge_sorted_runs_stable(ctx, nruns):
    """MergeSortedRuns (merge-path rounds) equals a stable sort of the concatenated runs:
    equal keys keep run order, then row order; empty runs are skipped."""
    from cylon_amd._lib import C
    rng = np.random.default_rng(nruns)
    sizes = [int(x) for x in rng.integers(0, 3000, nruns)]
    if nruns > 2:
        sizes[1] = 0
    frames = [pd.DataFrame({"k": np.sort(rng.integers(-50, 50, s)), "src": np.full(s, r), "j": np.arange(s)})
              for r, s in enumerate(sizes)]
    allin = pd.concat(frames).reset_index(drop=True)
    t = Table.from_pandas(ctx, allin)
    got = t._wrap(C.merge_sorted_runs(t.native, sizes, 0, True)).to_pandas()
    exp = allin.sort_values("k", kind="mergesort").reset_index(drop=True)
    pd.testing.assert_frame_equal(got, exp, check_dtype=False)
