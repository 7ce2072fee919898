"""force_shuffle on a distributed world-1 context (CPU, gloo): every distributed
operator takes its shuffle + exchange path instead of the world-1 shortcut and must
give the local operator's result.  The GPU twin over RCCL is
tests/test_gpu_rccl_forced.py."""
import numpy as np
import pandas as pd
import pytest

from dist_utils import run_distributed


def _frame(df):
    df = df[sorted(df.columns)]
    return df.sort_values(list(df.columns), kind="mergesort").reset_index(drop=True)


def _ops(ctx, chunks, self_wire):
    from cylon_amd import CylonContext, Table
    from cylon_amd._lib import C
    rng = np.random.default_rng(1)
    n = 20_000
    a = pd.DataFrame({"k": rng.integers(0, 15_000, n), "x": rng.integers(-5, 5, n), "f": rng.random(n)})
    b = pd.DataFrame({"k": rng.integers(0, 15_000, n), "v": rng.random(n), "s": [f"s{i % 17}" for i in range(n)]})
    local = CylonContext()
    res = {}
    ctx.add_config("shuffle_self_rccl", "1" if self_wire else "0")
    for forced in (False, True):
        ctx.add_config("force_shuffle", "1" if forced else "0")
        ctx.add_config("shuffle_chunks", str(chunks))
        C.trace_enable(True)
        C.trace_reset()
        ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
        r = {"join": ta.distributed_join(tb, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_"),
             "ljoin": ta.distributed_join(tb, "left", "sort", on=["k"], left_prefix="l_", right_prefix="r_"),
             "union": ta[["k"]].distributed_union(tb[["k"]]),
             "subtract": ta[["k"]].distributed_subtract(tb[["k"]]),
             "intersect": ta[["k"]].distributed_intersect(tb[["k"]]),
             "unique": tb.distributed_unique(["s"]),
             "groupby": ta.groupby("x", {"f": ["sum", "mean"], "k": "max"}),
             "sort": ta.distributed_sort(["x", "k"], ascending=[False, True])}
        res[forced] = ({k: v.to_pandas() for k, v in r.items()}, dict(C.trace_counters()))
    la, lb = Table.from_pandas(local, a), Table.from_pandas(local, b)
    ref = la.join(lb, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_").to_pandas()
    return res, ref


@pytest.mark.parametrize("chunks,self_wire", [(1, True), (3, True), (3, False)])
def test_force_shuffle_world1_matches_local(chunks, self_wire):
    """self_wire (config shuffle_self_rccl=1): the own partition goes through the communicator
    too, so a world-1 context exercises the posted exchanges; without it the own rows stay in
    place (reference table.cpp:89-106) and nothing is posted for the fixed-width operators."""
    res, ref = run_distributed(_ops, 1, chunks, self_wire)[0]
    plain, pc = res[False]
    forced, fc = res[True]
    assert pc.get("shuffle.requests_waited", 0) == 0  # world-1 shortcut: no exchange
    if self_wire:
        assert fc.get("shuffle.requests_waited", 0) > 0, fc  # forced: every op went through the exchange
    else:
        assert fc.get("shuffle.self_rows_kept_local", 0) > 0, fc
    if chunks > 1:
        assert fc.get("shuffle.chunks", 0) >= chunks and fc["shuffle.chunks"] % chunks == 0  # summed over ops
    pd.testing.assert_frame_equal(_frame(forced["join"]), _frame(ref), check_dtype=False)
    for op in plain:
        g, e = forced[op], plain[op]
        if op == "sort":
            assert g[["x", "k"]].equals(e[["x", "k"]])
        if op == "groupby":
            g, e = g.sort_values("x").reset_index(drop=True), e.sort_values("x").reset_index(drop=True)
            np.testing.assert_allclose(g["sum_f"], e["sum_f"], rtol=1e-12)
            np.testing.assert_allclose(g["mean_f"], e["mean_f"], rtol=1e-12)
            g, e = g.drop(columns=["sum_f", "mean_f"]), e.drop(columns=["sum_f", "mean_f"])
        pd.testing.assert_frame_equal(_frame(g), _frame(e), check_dtype=False, obj=op)


def _prologue(ctx, chunks):
    from cylon_amd import Table
    from cylon_amd._lib import C
    rng = np.random.default_rng(5 + ctx.get_rank())
    n = 30_000
    a = pd.DataFrame({"k": rng.integers(0, 40_000, n), "v": rng.random(n)})
    b = pd.DataFrame({"k": rng.integers(0, 40_000, n), "w": rng.random(n), "i": rng.integers(0, 9, n)})
    ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
    ctx.add_config("shuffle_chunks", str(chunks))
    C.trace_enable(True)
    C.trace_reset()
    out = ta.distributed_join(tb, "inner", "hash", on=["k"])
    c = dict(C.trace_counters())
    C.trace_enable(False)
    return out.row_count, c, len(a.merge(b, on="k"))


@pytest.mark.parametrize("chunks", [1, 3])
def test_exchange_prologue_is_one_collective(chunks):
    """A distributed join agrees on chunk count, per-chunk counts of both tables, nullability and
    the narrowed wire format with ONE all-gather; the only other collectives are the posted
    payload all-to-alls (reference exchanged headers per buffer, table.cpp:67-131)."""
    res = run_distributed(_prologue, 2, chunks)
    for rows, c, _ in res:
        assert c.get("comm.allgather") == 1, c
        assert c.get("comm.allreduce", 0) == 0 and c.get("comm.alltoall_blocking", 0) == 0, c
        assert c.get("comm.alltoall_posted", 0) == chunks * (2 + 3), c  # one per column buffer per chunk
    assert sum(r[0] for r in res) > 0
