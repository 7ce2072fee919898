"""GPU tests for group-by, set operations, unique, aggregates and the RCCL
communicator (world size 1 on the single-GPU box; the 8-GPU path is exercised
by the driver's scaling bench)."""
import os

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest
import torch

from cylon_amd import Table

pytestmark = pytest.mark.gpu


def _frame(n=200_000, seed=0):
    rng = np.random.default_rng(seed)
    v = rng.normal(size=n)
    v[rng.random(n) < 0.05] = np.nan
    return pd.DataFrame({"k": rng.integers(0, 5000, n), "s": [f"g{x}" for x in rng.integers(0, 40, n)], "v": v,
                         "i": rng.integers(-10**6, 10**6, n)})


def _sorted(df, keys):
    return df.sort_values(keys).reset_index(drop=True)


@pytest.mark.parametrize("keys", [["k"], ["s"], ["k", "s"]])
def test_groupby_gpu_vs_cpu(gpu_ctx, ctx, keys):
    df = _frame()
    ops = ["sum", "count", "min", "max", "mean", "var", "std", "nunique", "median"]
    g = Table.from_pandas(gpu_ctx, df).local_groupby(keys, {"v": ops, "i": ["sum", "min", "max"]}).to_pandas()
    c = Table.from_pandas(ctx, df).local_groupby(keys, {"v": ops, "i": ["sum", "min", "max"]}).to_pandas()
    g, c = _sorted(g, keys), _sorted(c, keys)
    assert list(g.columns) == list(c.columns)
    for col in g.columns:
        if g[col].dtype.kind == "f":
            np.testing.assert_allclose(g[col].to_numpy(), c[col].to_numpy(), rtol=1e-9, atol=1e-9, equal_nan=True)
        else:
            assert g[col].tolist() == c[col].tolist()


def test_groupby_small_group_count_lds_path(gpu_ctx):
    n = 1_000_000
    k = torch.randint(0, 7, (n,), device="cuda")
    v = torch.rand(n, device="cuda", dtype=torch.float64)
    t = Table.from_torch(gpu_ctx, {"k": k, "v": v})
    out = t.local_groupby("k", {"v": ["sum", "count", "min", "max"]}).sort("k").to_pandas()
    df = pd.DataFrame({"k": k.cpu().numpy(), "v": v.cpu().numpy()})
    exp = df.groupby("k")["v"].agg(["sum", "count", "min", "max"]).reset_index()
    np.testing.assert_allclose(out["sum_v"], exp["sum"], rtol=1e-9)
    assert out["count_v"].tolist() == exp["count"].tolist()
    assert np.array_equal(out["min_v"], exp["min"]) and np.array_equal(out["max_v"], exp["max"])


def test_set_ops_and_unique_gpu_vs_cpu(gpu_ctx, ctx):
    rng = np.random.default_rng(3)
    a = pa.table({"x": rng.integers(0, 300, 50_000), "s": [f"v{v}" for v in rng.integers(0, 9, 50_000)]})
    b = pa.table({"x": rng.integers(200, 500, 30_000), "s": [f"v{v}" for v in rng.integers(0, 9, 30_000)]})
    for op in ("union", "subtract", "intersect"):
        g = getattr(Table(a, gpu_ctx), op)(Table(b, gpu_ctx)).to_arrow()
        c = getattr(Table(a, ctx), op)(Table(b, ctx)).to_arrow()
        assert g.equals(c), op
    for keep in ("first", "last"):
        g = Table(a, gpu_ctx).unique(["x"], keep=keep).to_arrow()
        c = Table(a, ctx).unique(["x"], keep=keep).to_arrow()
        assert g.equals(c)


def test_scalar_aggregates_gpu(gpu_ctx):
    df = _frame(100_000, 9)
    t = Table.from_pandas(gpu_ctx, df)
    assert t.sum("i").to_pydict()["i"][0] == df["i"].sum()
    assert t.count("v").to_pydict()["v"][0] == df["v"].count()
    assert t.min("v").to_pydict()["v"][0] == df["v"].min()
    assert t.max("i").to_pydict()["i"][0] == df["i"].max()
    assert t.mean("v").to_pydict()["v"][0] == pytest.approx(df["v"].mean())
    assert t.std("v").to_pydict()["v"][0] == pytest.approx(df["v"].std())
    assert t.quantile("v", 0.5).to_pydict()["v"][0] == pytest.approx(df["v"].median())


def test_rccl_communicator_world1():
    """Exercises the ProcessGroup communicator on RCCL (backend nccl) on one GPU."""
    import torch.distributed as dist
    from cylon_amd import CylonContext, RCCLConfig
    os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
    os.environ.setdefault("MASTER_PORT", "29533")
    os.environ["RANK"] = "0"
    os.environ["WORLD_SIZE"] = "1"
    os.environ["LOCAL_RANK"] = "0"
    ctx = CylonContext(config=RCCLConfig(), distributed=True)
    try:
        assert ctx.get_world_size() == 1 and ctx.on_gpu
        x = torch.arange(10, device="cuda", dtype=torch.int64)
        assert torch.equal(ctx._ctx.alltoallv(x, [10]), x)
        y = torch.ones(4, device="cuda")
        assert torch.equal(ctx.allreduce(y.clone(), "sum"), y)
        assert torch.equal(ctx.allgather(x), x)
        ctx.barrier()
        t = Table(pa.table({"k": [1, 2, 3], "v": [1.0, 2.0, 3.0]}), ctx)
        j = t.distributed_join(t, "inner", "hash", on=[0], left_prefix="l_", right_prefix="r_")
        assert j.row_count == 3
        g = t.groupby("k", {"v": "sum"})
        assert g.row_count == 3
    finally:
        ctx.finalize()
        if dist.is_initialized():
            dist.destroy_process_group()


def test_device_memory_pool(gpu_ctx):
    pool = gpu_ctx.memory_pool()
    assert pool.backend_name() == "hip_caching_allocator" and pool.device().startswith("cuda")
    before = pool.bytes_allocated()
    x = pool.empty([1 << 20], "int64")
    assert x.is_cuda and pool.bytes_allocated() == before + 8 * (1 << 20)
    x.fill_(3)
    assert int(x.sum()) == 3 * (1 << 20)
    del x
    assert pool.bytes_allocated() == before


def test_native_index_lookup_on_gpu(gpu_ctx, ctx):
    import numpy as np
    from cylon_amd.indexing.index import IndexingSchema
    rng = np.random.default_rng(3)
    keys = rng.integers(0, 500, 20000)
    res = []
    for cx in (gpu_ctx, ctx):
        t = Table(pa.table({"k": keys, "v": np.arange(20000)}), cx)
        t.set_index("k", IndexingSchema.HASH, drop=True)
        res.append(t.loc[[7, 3, 499, 1000], "v"].to_pandas()["v"].tolist())
    assert res[0] == res[1] and len(res[0]) == int(np.isin(keys, [7, 3, 499]).sum())
