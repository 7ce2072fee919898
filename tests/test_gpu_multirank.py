"""Multi-rank device paths on the single-GPU box: 2 ranks share cuda:0, tables live
in HBM, collectives go over gloo.  This runs the device kernels of every
world > 1 code path (hash partition into W / W*K parts, chunked pipelined join
writing into one output sink, distributed group-by / sort / set ops) against a
pandas oracle of the gathered inputs.  RCCL itself needs one GPU per rank, so
the RCCL transport at world > 1 is exercised by the driver's 8-GPU bench only."""
import numpy as np
import pandas as pd
import pytest

from dist_utils import run_distributed

pytestmark = pytest.mark.gpu

DEV = "cuda:0"
SMALL_RADIX = {"CYLON_RADIX_JOIN_MIN_ROWS": "1024"}  # radix join (and its sink) on small chunks


def _canon(df):
    # nulls / NaN -> one sortable sentinel (the test data has no infinities)
    return sorted(tuple(float("-inf") if (isinstance(x, float) and np.isnan(x)) else x for x in r)
                  for r in df.itertuples(index=False))


def _join_chunks(ctx, chunks, n):
    from cylon_amd import Table
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    rng = np.random.default_rng(7 + rank)
    a = pd.DataFrame({"k": rng.integers(0, int(0.99 * 2 * n), n), "x": rng.integers(-9, 9, n).astype(np.int32),
                      "f": rng.random(n)})
    b = pd.DataFrame({"k": rng.integers(0, int(0.99 * 2 * n), n), "v": rng.random(n)})
    ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
    assert ta.device == ctx.device
    ctx.add_config("shuffle_chunks", str(chunks))
    C.trace_enable(True)
    C.trace_reset()
    out = ta.distributed_join(tb, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")
    counters = dict(C.trace_counters())
    return out.to_pandas(), a, b, counters


@pytest.mark.parametrize("chunks", [1, 3])
def test_chunked_distributed_join_on_device(chunks):
    n = 60_000
    res = run_distributed(_join_chunks, 2, chunks, n, device=DEV, env=SMALL_RADIX)
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    ref = a.add_prefix("l_").merge(b.add_prefix("r_"), left_on="l_k", right_on="r_k")
    assert len(got) == len(ref) > 0
    assert _canon(got[sorted(got.columns)]) == _canon(ref[sorted(got.columns)])
    for r in res:
        c = r[3]
        assert c.get("join.radix.rows_out", 0) > 0, c  # the LDS radix join ran (into the sink when chunked)
        if chunks > 1:
            assert c.get("shuffle.chunks") == chunks
            assert c.get("shuffle.fast_partition") == 2  # one LDS-staged pass per relation


def _dist_ops(ctx):
    from cylon_amd import Table
    rank = ctx.get_rank()
    rng = np.random.default_rng(11 + rank)
    n = 50_000
    df = pd.DataFrame({"k": rng.integers(0, 3000, n), "v": rng.random(n), "i": rng.integers(-100, 100, n)})
    t = Table.from_pandas(ctx, df)
    g = t.groupby("k", {"v": "sum", "i": "max"}).to_pandas()
    s = t.distributed_sort("v").to_pandas()
    u1 = pd.DataFrame({"a": rng.integers(0, 500, 4000), "b": rng.integers(0, 3, 4000)})
    u2 = pd.DataFrame({"a": rng.integers(0, 500, 3000), "b": rng.integers(0, 3, 3000)})
    tu1, tu2 = Table.from_pandas(ctx, u1), Table.from_pandas(ctx, u2)
    sets = {op: getattr(tu1, f"distributed_{op}")(tu2).to_pandas() for op in ("union", "intersect", "subtract")}
    return df, g, s, u1, u2, sets


@pytest.mark.parametrize("shape", ["mixed_widths", "nullable_8byte"])
def test_shuffle_partition_fast_pass_matches_generic(shape):
    """The shuffle's one-pass partition of an int64-keyed table equals the generic
    pid + stable scatter path (rows, order within partitions, counts).  nullable_8byte:
    validity and bool bytes travel packed 8 per word through the pass (radix.cpp
    PackByteColumns) and are unpacked back to their columns."""
    import pyarrow as pa
    import torch
    from cylon_amd import CylonContext, Table
    from cylon_amd._lib import C
    ctx = CylonContext(device=DEV)
    g = torch.Generator(device="cuda").manual_seed(3)
    n = 300_000
    if shape == "mixed_widths":
        t = Table.from_torch(ctx, {"k": torch.randint(-2**40, 2**40, (n,), generator=g, device="cuda"),
                                   "x": torch.randint(0, 100, (n,), generator=g, device="cuda", dtype=torch.int32),
                                   "f": torch.rand(n, generator=g, device="cuda", dtype=torch.float64)})
    else:
        rng = np.random.default_rng(4)
        t = Table(pa.table({"k": rng.integers(-2**40, 2**40, n),
                            "f": pa.array(rng.random(n), mask=rng.random(n) < 0.3),
                            "i": pa.array(rng.integers(0, 9, n), mask=rng.random(n) < 0.1),
                            "b": pa.array(rng.random(n) < 0.5, mask=rng.random(n) < 0.2)}), ctx)
        assert t.device.startswith("cuda")
    for P in (2, 8, 24, 1024):
        fast, cf = C.shuffle_partition(t.native, [0], P)
        pid, _ = C.map_to_hash_partitions(t.native, [0], P)
        slow, cs = C.partition_reorder(t.native, pid, P)
        assert list(cf) == list(cs)
        a, b = Table(None, ctx, _native=fast).to_arrow(), Table(None, ctx, _native=slow).to_arrow()
        assert a.equals(b), P


def test_distributed_ops_on_device():
    res = run_distributed(_dist_ops, 2, device=DEV)
    df = pd.concat([r[0] for r in res])
    g = pd.concat([r[1] for r in res]).sort_values("k").reset_index(drop=True)
    ref = df.groupby("k").agg(sum_v=("v", "sum"), max_i=("i", "max")).reset_index()
    assert np.array_equal(g["k"].to_numpy(), ref["k"].to_numpy())
    np.testing.assert_allclose(g["sum_v"].to_numpy(), ref["sum_v"].to_numpy(), rtol=1e-9)
    assert np.array_equal(g["max_i"].to_numpy(), ref["max_i"].to_numpy())
    # distributed sort: every rank sorted, rank 0's max <= rank 1's min, rows conserved
    s0, s1 = res[0][2]["v"].to_numpy(), res[1][2]["v"].to_numpy()
    assert np.all(np.diff(s0) >= 0) and np.all(np.diff(s1) >= 0)
    assert len(s0) + len(s1) == len(df) and (len(s0) == 0 or len(s1) == 0 or s0[-1] <= s1[0])
    u1 = pd.concat([r[3] for r in res])
    u2 = pd.concat([r[4] for r in res])
    A = set(map(tuple, u1.to_numpy().tolist()))
    B = set(map(tuple, u2.to_numpy().tolist()))
    expect = {"union": A | B, "intersect": A & B, "subtract": A - B}
    for op, rows in expect.items():
        got = [tuple(x) for r in res for x in r[5][op].to_numpy().tolist()]
        assert len(got) == len(set(got)) and set(got) == rows, op


def _join_edge_cases(ctx, case):
    import torch
    from cylon_amd import Table
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    g = torch.Generator(device="cuda").manual_seed(50 + rank)
    n = 40_000
    if case == "skew":  # one hot key on the (smaller) build side overflows the LDS capacity -> split items
        k = torch.randint(0, 5000, (n,), generator=g, device="cuda")
        m = n // 4
        kb = torch.where(torch.rand(m, generator=g, device="cuda") < 0.3, torch.zeros(m, dtype=torch.int64, device="cuda"),
                         torch.randint(1, 5000, (m,), generator=g, device="cuda"))
    else:
        k = torch.randint(0, 60_000, (n,), generator=g, device="cuda")
        kb = torch.randint(0, 60_000, (n if rank == 0 else 0,), generator=g, device="cuda")  # rank 1: empty right
    v = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
    a = Table.from_torch(ctx, {"k": k, "v": v})
    if case == "nulls":  # nullable payload through the radix sink
        import pyarrow as pa
        at = a.to_arrow()
        mask = (at.column("v").to_numpy() < 0.2)
        a = Table(pa.table({"k": at.column("k"), "v": pa.array(at.column("v").to_numpy(), mask=mask)}), ctx)
    b = Table.from_torch(ctx, {"k": kb, "w": torch.rand(kb.numel(), generator=g, device="cuda", dtype=torch.float64)})
    ctx.add_config("shuffle_chunks", "3")
    C.trace_enable(True)
    C.trace_reset()
    out = a.distributed_join(b, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")
    c = dict(C.trace_counters())
    return out.to_pandas(), a.to_pandas(), b.to_pandas(), c


@pytest.mark.parametrize("case", ["skew", "empty_rank", "nulls"])
def test_chunked_join_edge_cases_on_device(case):
    res = run_distributed(_join_edge_cases, 2, case, device=DEV, env=SMALL_RADIX)
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    ref = a.add_prefix("l_").merge(b.add_prefix("r_"), left_on="l_k", right_on="r_k")
    assert len(got) == len(ref)
    assert _canon(got[sorted(got.columns)]) == _canon(ref[sorted(got.columns)])
    if case == "skew":  # the hot key's partition runs as split work items (no global-table fallback)
        assert any(r[3].get("join.radix.split_partitions", 0) > 0 for r in res)
        assert all(r[3].get("join.radix.overflow_fallback", 0) == 0 for r in res)


# ---------------------------------------------------------------------------
# Asynchronous exchange on the device (net/async_delay_communicator.hpp): every posted
# all-to-all completes on a side HIP stream after a spin delay into a poisoned buffer,
# with event-backed requests (Test = event query, Wait = stream wait) -- RCCL's completion
# semantics, so the chunk-k-consumed-while-k+1-in-flight ordering runs for real.
# ---------------------------------------------------------------------------
def _async_join(ctx, chunks, n, delay_us):
    from cylon_amd import Table
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    ctx._ctx.use_async_delay_transport(float(delay_us))
    rng = np.random.default_rng(70 + rank)
    a = pd.DataFrame({"k": rng.integers(0, int(0.99 * 2 * n), n), "x": rng.integers(-9, 9, n).astype(np.int32),
                      "f": rng.random(n)})
    b = pd.DataFrame({"k": rng.integers(0, int(0.99 * 2 * n), n), "v": rng.random(n)})
    ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
    ctx.add_config("shuffle_chunks", str(chunks))
    C.trace_enable(True)
    C.trace_reset()
    out = ta.distributed_join(tb, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")
    got = out.to_pandas()
    join_counters = dict(C.trace_counters())
    u1 = pd.DataFrame({"a": rng.integers(0, 500, 4000), "b": rng.integers(0, 3, 4000)})
    u2 = pd.DataFrame({"a": rng.integers(0, 500, 3000), "b": rng.integers(0, 3, 3000)})
    tu1, tu2 = Table.from_pandas(ctx, u1), Table.from_pandas(ctx, u2)
    sets = {op: getattr(tu1, f"distributed_{op}")(tu2).to_pandas() for op in ("union", "intersect", "subtract")}
    posted, in_flight = ctx._ctx.async_transport_stats()
    return got, a, b, u1, u2, sets, posted, in_flight, join_counters


@pytest.mark.parametrize("chunks", [1, 4])
def test_async_exchange_join_and_setops_on_device(chunks):
    res = run_distributed(_async_join, 2, chunks, 60_000, 3000, device=DEV, env=SMALL_RADIX)
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    ref = a.add_prefix("l_").merge(b.add_prefix("r_"), left_on="l_k", right_on="r_k")
    assert len(got) == len(ref) > 0
    assert _canon(got[sorted(got.columns)]) == _canon(ref[sorted(got.columns)])
    u1 = pd.concat([r[3] for r in res])
    u2 = pd.concat([r[4] for r in res])
    A = set(map(tuple, u1.to_numpy().tolist()))
    B = set(map(tuple, u2.to_numpy().tolist()))
    for op, rows in {"union": A | B, "intersect": A & B, "subtract": A - B}.items():
        g = [tuple(x) for r in res for x in r[5][op].to_numpy().tolist()]
        assert len(g) == len(set(g)) and set(g) == rows, op
    for r in res:
        posted, in_flight, c = r[6], r[7], r[8]
        assert posted > 0
        assert in_flight > 0, "no posted exchange was still in flight when its consumer reached it"
        if chunks > 1:
            assert c.get("shuffle.chunks") == chunks


def _dev_sort(ctx, case):
    import torch
    from cylon_amd import Table
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    g = torch.Generator(device="cuda").manual_seed(90 + rank)
    n = 200_000 + 30_000 * rank
    if case == "wide_chunked":  # pipelined sort: 4 key sub-range chunks, merge-path merges on the device
        ctx.add_config("sort_chunks", "4")
    if case.startswith("wide"):
        k = torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, device="cuda")
    else:  # one key everywhere
        k = torch.full((n,), 5, dtype=torch.int64, device="cuda")
    i = torch.arange(n, device="cuda") + 1_000_000 * rank
    t = Table.from_torch(ctx, {"k": k, "i": i})
    C.trace_enable(True)
    C.trace_reset()
    s = t.distributed_sort("k", ascending=case.startswith("wide"))
    return s.to_pandas(), t.to_pandas(), dict(C.trace_counters())


@pytest.mark.parametrize("case", ["wide", "wide_chunked", "one_key"])
def test_distributed_sort_exact_splitters_on_device(case):
    res = run_distributed(_dev_sort, 2, case, device=DEV)
    allin = pd.concat([r[1] for r in res]).reset_index(drop=True)
    got = pd.concat([r[0] for r in res]).reset_index(drop=True)
    for r in res:
        assert r[2].get("sort.dist.pipelined", 0) == 1
        assert r[2].get("shuffle.chunks", 0) == (4 if case == "wide_chunked" else 1)
    exp = allin.sort_values("k", ascending=case.startswith("wide"), kind="mergesort").reset_index(drop=True)
    assert got["k"].tolist() == exp["k"].tolist() and got["i"].tolist() == exp["i"].tolist()
    loads = [len(r[0]) for r in res]
    assert max(loads) <= 1.5 * len(allin) / 2, loads


def _graph_async(ctx):
    from cylon_amd import Table
    from cylon_amd._lib import C
    from cylon_amd.parallel import DisJoinOp
    rank = ctx.get_rank()
    ctx._ctx.use_async_delay_transport(500.0)
    rng = np.random.default_rng(20 + rank)
    lefts = [pd.DataFrame({"k": rng.integers(0, 5000, 20_000), "v": rng.random(20_000)}) for _ in range(4 - 2 * rank)]
    rights = [pd.DataFrame({"k": rng.integers(0, 5000, 15_000), "w": rng.random(15_000)}) for _ in range(2)]
    C.trace_enable(True)
    C.trace_reset()
    op = DisJoinOp(ctx, "inner", "hash", [0], [0], "l_", "r_", num_splits=4)
    for d in lefts:
        op.insert_table(DisJoinOp.LEFT, Table.from_pandas(ctx, d))
    for d in rights:
        op.insert_table(DisJoinOp.RIGHT, Table.from_pandas(ctx, d))
    got = pd.concat([r.to_pandas() for r in op.execute()])
    return got, pd.concat(lefts), pd.concat(rights), dict(C.trace_counters())


def test_dis_join_op_streaming_on_device_async():
    """Streaming op-graph exchange on HBM tables with event-backed asynchronous transfers."""
    res = run_distributed(_graph_async, 2, device=DEV)
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    ref = a.add_prefix("l_").merge(b.add_prefix("r_"), left_on="l_k", right_on="r_k")
    assert len(got) == len(ref) and _canon(got[sorted(got.columns)]) == _canon(ref[sorted(got.columns)])
    for r in res:
        assert r[3].get("graph.alltoall.rounds") == 6, r[3]  # 4 left rounds (rank 0's batches) + 2 right


def _string_join_chunks(ctx, chunks, n):
    """String key + string payload through the planned, chunked exchange (var columns as lengths in
    the gapped row layout and bytes in their own gapped byte layouts)."""
    from cylon_amd import Table
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    rng = np.random.default_rng(70 + rank)
    ka, kb = rng.integers(0, n, n), rng.integers(0, n, n)
    a = pd.DataFrame({"s": [f"id{x:07d}" for x in ka], "x": rng.integers(-9, 9, n),
                      "p": [("p" * int(x % 5)) + str(x) for x in ka]})
    b = pd.DataFrame({"s": [f"id{x:07d}" for x in kb], "v": rng.random(n)})
    ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
    ctx.add_config("shuffle_chunks", str(chunks))
    C.trace_enable(True)
    C.trace_reset()
    out = {"join": ta.distributed_join(tb, "inner", "hash", on=["s"], left_prefix="l_", right_prefix="r_"),
           "left": ta.distributed_join(tb, "left", "hash", on=["s"], left_prefix="l_", right_prefix="r_"),
           "union": ta[["s"]].distributed_union(tb[["s"]])}
    counters = dict(C.trace_counters())
    C.trace_enable(False)
    return {k: v.to_pandas() for k, v in out.items()}, a, b, counters


def _check_string_join(res, chunks):
    A = pd.concat([r[1] for r in res]).reset_index(drop=True)
    B = pd.concat([r[2] for r in res]).reset_index(drop=True)
    la, rb = A.add_prefix("l_"), B.add_prefix("r_")
    for how in ("join", "left"):
        got = pd.concat([r[0][how] for r in res])
        exp = la.merge(rb, left_on="l_s", right_on="r_s", how="inner" if how == "join" else "left")
        cols = sorted(got.columns)
        key = lambda df: sorted(map(lambda t: tuple("~nan" if (x is None or (isinstance(x, float) and x != x)) else x
                                                    for x in t), df[cols].itertuples(index=False)), key=str)
        assert len(got) == len(exp) and key(got) == key(exp), how
    un = sorted(pd.concat([r[0]["union"] for r in res])["s"].tolist())
    assert un == sorted(set(A["s"]) | set(B["s"]))
    for r in res:
        assert r[3].get("shuffle.var_columns_planned", 0) > 0, r[3]
        assert r[3].get("shuffle.chunks", 0) == 3 * chunks, r[3]  # three operators, each chunked


def test_string_join_chunked_gloo_gpu():
    """2 ranks, tables in HBM, gloo collectives: a string-key join runs chunked (shuffle.chunks > 1)
    through the planned var-width exchange, and the device radix join on the row hash."""
    res = run_distributed(_string_join_chunks, 2, 3, 40_000, device=DEV, env=SMALL_RADIX)
    _check_string_join(res, 3)
