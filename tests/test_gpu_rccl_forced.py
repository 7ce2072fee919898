"""The RCCL exchange path on one MI355X.

A world-1 RCCL context (torch.distributed backend nccl, one rank) with config
force_shuffle=1 runs every distributed operator through its shuffle path instead of
the world-1 local shortcut: partition -> posted RCCL all-to-alls (ProcessGroupNCCL
self all-to-all: a real asynchronous RCCL kernel on the communicator's stream) ->
PGRequest Test()/Wait() (event query / stream wait) -> local operator.  Results
are compared against the CPU twin of the same operator on the same data.

Reference: cpp/src/cylon/table.cpp:67-131 (all_to_all_arrow_tables), :482-502
(DistributedJoin), :727-767 (distributed set ops), :338-382 (DistributedSort),
groupby/groupby.cpp:33-83 (DistributedHashGroupBy)."""
import numpy as np
import pandas as pd
import pytest

from dist_utils import run_distributed

pytestmark = pytest.mark.gpu

RCCL = {"CYLON_TEST_COMM": "rccl", "CYLON_RADIX_JOIN_MIN_ROWS": "4096"}


def _sorted_frame(df):
    df = df[sorted(df.columns)]
    return df.sort_values(list(df.columns), kind="mergesort").reset_index(drop=True)


def _forced(ctx, chunks, n, self_wire=True):
    import torch
    from cylon_amd import CylonContext, Table
    from cylon_amd._lib import C
    assert ctx.get_world_size() == 1 and ctx.on_gpu and ctx.is_distributed()
    ctx.add_config("force_shuffle", "1")
    # the own partition normally stays in place (nothing to send at world 1); the knob routes it
    # through RCCL so these tests keep driving real RCCL kernels on one GPU
    ctx.add_config("shuffle_self_rccl", "1" if self_wire else "0")
    ctx.add_config("shuffle_chunks", str(chunks))
    cpu = CylonContext(device="cpu")
    g = torch.Generator(device="cuda").manual_seed(5)
    kr = int(0.99 * n)
    a = {"k": torch.randint(0, kr, (n,), generator=g, device="cuda"),
         "x": torch.randint(-9, 9, (n,), generator=g, device="cuda", dtype=torch.int32),
         "f": torch.rand(n, generator=g, device="cuda", dtype=torch.float64)}
    b = {"k": torch.randint(0, kr, (n,), generator=g, device="cuda"),
         "v": torch.rand(n, generator=g, device="cuda", dtype=torch.float64)}
    ta, tb = Table.from_torch(ctx, a), Table.from_torch(ctx, b)
    ca, cb = Table(ta.to_arrow(), cpu), Table(tb.to_arrow(), cpu)
    out = {}
    C.trace_enable(True)
    C.trace_reset()
    out["join"] = (ta.distributed_join(tb, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_").to_pandas(),
                   ca.join(cb, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_").to_pandas())
    join_counters = dict(C.trace_counters())
    C.trace_reset()
    m = n // 8
    s1 = Table.from_torch(ctx, {"a": torch.randint(0, 5000, (m,), generator=g, device="cuda"),
                                "b": torch.randint(0, 3, (m,), generator=g, device="cuda")})
    s2 = Table.from_torch(ctx, {"a": torch.randint(2000, 7000, (m,), generator=g, device="cuda"),
                                "b": torch.randint(0, 3, (m,), generator=g, device="cuda")})
    c1, c2 = Table(s1.to_arrow(), cpu), Table(s2.to_arrow(), cpu)
    for op in ("union", "intersect", "subtract"):
        out[op] = (getattr(s1, f"distributed_{op}")(s2).to_pandas(), getattr(c1, op)(c2).to_pandas())
    out["unique"] = (s1.distributed_unique(["a"]).to_pandas(), c1.unique(["a"]).to_pandas())
    out["groupby"] = (ta.groupby("x", {"f": ["sum", "max"], "k": "count"}).to_pandas(),
                      ca.groupby("x", {"f": ["sum", "max"], "k": "count"}).to_pandas())
    out["sort"] = (ta.distributed_sort(["k", "x"]).to_pandas(), ca.sort(["k", "x"]).to_pandas())
    return out, join_counters, dict(C.trace_counters())


@pytest.mark.parametrize("chunks,self_wire", [(1, True), (4, True), (4, False)])
def test_forced_rccl_shuffle_matches_cpu_twin(chunks, self_wire):
    out, jc, oc = run_distributed(_forced, 1, chunks, 2_000_000, self_wire, device="cuda:0", env=RCCL)[0]
    for op, (got, exp) in out.items():
        assert len(got) == len(exp) > 0, op
        if op == "sort":  # globally ordered by (k, x); ties in any order
            assert got[["k", "x"]].equals(exp[["k", "x"]]), op
            got, exp = _sorted_frame(got), _sorted_frame(exp)
        elif op == "groupby":
            got, exp = got.sort_values("x").reset_index(drop=True), exp.sort_values("x").reset_index(drop=True)
            np.testing.assert_allclose(got["sum_f"], exp["sum_f"], rtol=1e-9)
            got, exp = got.drop(columns="sum_f"), exp.drop(columns="sum_f")
        else:
            got, exp = _sorted_frame(got), _sorted_frame(exp)
        pd.testing.assert_frame_equal(got, exp, check_dtype=False, obj=op)
    if not self_wire:  # the own rows never left the layout: the join read them in place
        assert jc.get("shuffle.self_rows_kept_local", 0) == 4_000_000, jc
        assert jc.get("shuffle.requests_waited", 0) == 0, jc
        assert jc.get("join.radix.rows_out", 0) == len(out["join"][0]), jc
        return
    # the exchange ran through RCCL work handles: requests were posted, were still running on
    # the RCCL stream after posting (PGRequest::Test() == false: asynchronous to the host), and
    # were waited on by their consumers.  (Whether one is still running when its consumer
    # arrives -- shuffle.requests_in_flight_at_wait -- depends on how fast the self-exchange
    # is relative to the host's posting, so it is reported, not asserted.)
    assert jc.get("shuffle.requests_waited", 0) > 0, jc
    assert jc.get("shuffle.requests_pending_after_post", 0) > 0, jc
    assert jc.get("join.radix.rows_out", 0) == len(out["join"][0]), jc
    if chunks > 1:
        assert jc.get("shuffle.chunks") == chunks, jc
    assert oc.get("shuffle.requests_waited", 0) > 0, oc
