"""Aux subsystems: tracing, fault injection, checkpointing, utils, interop, determinism."""
import os

import numpy as np
import pandas as pd
import pyarrow as pa
import pytest
import torch

from cylon_amd import CylonError, Table
from cylon_amd.utils import (MiniBatcher, benchmark_with_repitions, generate_numeric_csv, random_table, traced)
from cylon_amd.utils import trace as tr
from cylon_amd.utils.checkpoint import load_table, save_table
from cylon_amd.utils.interop import from_dlpack, to_dlpack, to_tensor

from dist_utils import run_distributed


def test_tracing_phases(ctx):
    t = random_table(ctx, 5000, 2, seed=1)
    with traced():
        t.join(t, "inner", "hash", on=[0])
        t.sort("v0")
        t.local_groupby("k", {"v1": "sum"})
        ph = tr.phases()
    assert "join.materialize" in ph and "sort.indices" in ph and "groupby.group_ids" in ph
    assert all(v[0] >= 0 and v[1] >= 1 for v in ph.values())
    assert "phase" in tr.report()


def _fault(ctx):
    t = Table(pa.table({"k": np.arange(100), "v": np.arange(100)}), ctx)
    ctx._ctx.inject_faults(2)  # fail on the 2nd collective of the shuffle
    try:
        t.shuffle(["k"])
    except CylonError as e:
        return ("injected" in str(e), e.args[1] if len(e.args) > 1 else None)
    return (False, None)


def test_fault_injection_surfaces_as_error():
    for ok, code in run_distributed(_fault, 2):
        assert ok and code == 42  # Code::ExecutionError


def _ckpt(ctx, d):
    t = Table(pa.table({"k": np.arange(10) + 100 * ctx.get_rank()}), ctx)
    save_table(t, d, "tbl")
    ctx.barrier()
    back = load_table(ctx, d, "tbl")
    return back.to_pydict() == t.to_pydict()


def test_checkpoint_roundtrip(tmp_path):
    assert all(run_distributed(_ckpt, 2, str(tmp_path)))


def test_benchutils_datagen_minibatch(ctx, tmp_path):
    @benchmark_with_repitions(repititions=3, time_type="ms")
    def f(x):
        return x + 1

    t, r = f(1)
    assert r == 2 and t >= 0
    p = generate_numeric_csv(100, 4, str(tmp_path / "g.csv"), seed=0)
    df = pd.read_csv(p)
    assert df.shape == (100, 4) and df["0"].max() < 99
    mb = MiniBatcher.generate_minibatches(np.arange(15000), 32)
    assert mb.shape == (469, 32)
    mt = MiniBatcher.generate_minibatches(torch.arange(10), 4)
    assert mt.shape == (3, 4)


def test_dlpack_interop(ctx):
    t = random_table(ctx, 100, 2)
    back = from_dlpack(ctx, to_dlpack(t))
    assert back.to_arrow().equals(t.to_arrow())
    x = to_tensor(t, ["v0", "v1"])
    assert x.shape == (100, 2)


def test_join_is_deterministic(ctx):
    rng = np.random.default_rng(0)
    a = Table(pa.table({"k": rng.integers(0, 100, 3000), "v": rng.random(3000)}), ctx)
    r1 = a.join(a, "inner", "hash", on=[0]).to_arrow()
    r2 = a.join(a, "inner", "hash", on=[0]).to_arrow()
    assert r1.equals(r2)


def test_memory_pool_accounting(ctx):
    from cylon_amd.ctx import host_memory_pool
    pool = ctx.memory_pool()
    assert pool.backend_name() == "host" and pool.device() == "cpu"
    p = host_memory_pool()
    x = p.empty([1000, 4], "float64")
    assert tuple(x.shape) == (1000, 4) and p.bytes_allocated() == 32000
    x.fill_(1.5)
    assert float(x.sum()) == 6000.0
    del x
    assert p.bytes_allocated() == 0 and p.max_memory() == 32000
    ctx.set_memory_pool(p)
    assert ctx.memory_stats()["pool_max_memory"] == 32000


# ---- K15 string <-> number casts (kernels/strcast.hip; CPU twin here, GPU in test_gpu_ops.py)
def _cast_cases():
    import pyarrow as pa
    return [
        (["1", "-25", None, "007", "-0", "9223372036854775807", "-9223372036854775808"], pa.int64()),
        (["12", None, "-128", "127"], pa.int8()),
        (["1.5", ".5", "5.", "+1e3", "1E-3", None, "-0", "123456789.125", "0.1", "1e22", "3.14159"], pa.float64()),
        (["0.1", "2.5e-3", "7"], pa.float32()),
        (["inf", "1.5", "nan", "1e400", "0.12345678901234567890123"], pa.float64()),  # host parser
        (["0x10", "5"], pa.int64()),  # hex: host parser
    ]


@pytest.mark.parametrize("case", range(6))
def test_string_to_number_cast_matches_arrow(ctx, case):
    import math
    import pyarrow as pa
    import pyarrow.compute as pc
    from cylon_amd import Table
    vals, typ = _cast_cases()[case]
    arr = pa.array(vals, pa.string())
    got = Table(pa.table({"s": arr}), ctx).astype({"s": typ}).to_arrow().column(0).to_pylist()
    exp = pc.cast(arr, typ).to_pylist()
    assert len(got) == len(exp)
    for g, e in zip(got, exp):
        if e is None or g is None:
            assert g is None and e is None
        elif isinstance(e, float) and math.isnan(e):
            assert math.isnan(g)
        else:
            assert g == e and (not isinstance(e, float) or math.copysign(1, g) == math.copysign(1, e)), (g, e)


@pytest.mark.parametrize("bad,typ", [("+5", "int64"), ("1_000", "int64"), ("", "int64"), (" 1", "int64"),
                                     ("300", "int8"), ("-1", "uint8"), (".", "float64"), ("1e", "float64"),
                                     ("e5", "float64"), ("1.5x", "float64")])
def test_string_to_number_cast_rejects_like_arrow(ctx, bad, typ):
    import pyarrow as pa
    from cylon_amd import Table
    with pytest.raises(pa.ArrowInvalid):
        pa.compute.cast(pa.array([bad]), getattr(pa, typ)())
    with pytest.raises(pa.ArrowInvalid):
        Table(pa.table({"s": pa.array(["1", bad])}), ctx).astype({"s": getattr(pa, typ)()})


@pytest.mark.parametrize("typ", ["int64", "int32", "int8", "uint16", "uint32"])
def test_integer_to_string_cast_matches_arrow(ctx, typ):
    import numpy as np
    import pyarrow as pa
    import pyarrow.compute as pc
    from cylon_amd import Table
    info = np.iinfo(typ)
    rng = np.random.default_rng(1)
    v = list(rng.integers(info.min, info.max, 200, dtype=typ, endpoint=True)) + [info.min, info.max, 0]
    arr = pa.array(v, getattr(pa, typ)(), mask=np.arange(len(v)) % 17 == 3)
    got = Table(pa.table({"x": arr}), ctx).astype({"x": pa.string()}).to_arrow().column(0)
    assert got.to_pylist() == pc.cast(arr, pa.string()).to_pylist()


def test_knob_registry_matches_docs():
    """docs/knobs.md lists exactly the knobs of the native registry (knobs.cpp), and no native source
    reads a CYLON_* variable around the registry."""
    import glob
    import re
    from cylon_amd._lib import C
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    reg = {f"CYLON_{name}" for name, _, _ in C.knob_registry()}
    doc = open(os.path.join(root, "docs", "knobs.md")).read()
    tables = doc[doc.index("## Runtime"):]  # the tables (the intro names deleted knobs)
    assert set(re.findall(r"`(CYLON_[A-Z0-9_]+)`", tables)) == reg
    srcs = glob.glob(os.path.join(root, "cylon_amd", "csrc", "**", "*.cpp"), recursive=True) + \
        glob.glob(os.path.join(root, "cylon_amd", "csrc", "**", "*.hip"), recursive=True)
    offenders = [p for p in srcs if 'getenv("CYLON_' in open(p).read() and not p.endswith("knobs.cpp")]
    assert offenders == []
    assert len(reg) <= 27
