"""The Python examples (examples/python/) run end to end on the CPU and print the results their
operators must give (pandas oracles recomputed here); the distributed one runs as 2 gloo ranks."""
import os
import socket
import subprocess
import sys

import numpy as np
import pandas as pd
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EX = os.path.join(ROOT, "examples", "python")


def _run(args, timeout=300):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    r = subprocess.run(args, cwd=ROOT, env=env, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    out = {}
    for line in r.stdout.splitlines():
        parts = line.split(" ", 1)
        if len(parts) == 2 and not line.startswith("["):
            out[parts[0]] = parts[1]
    return out


def test_table_initialize_example():
    out = _run([sys.executable, os.path.join(EX, "table_initialize.py"), "--device", "cpu"])
    for name in ("dict", "list", "numpy", "pandas", "arrow", "torch"):
        assert out[f"rows_{name}"] == "4"
    assert float(out["pandas_sum"]) == 8.0 and out["numpy_shape"] == "4x2" and out["arrow_columns"] == "id,score"


def test_relational_algebra_example():
    n = 20_000
    out = _run([sys.executable, os.path.join(EX, "table_relational_algebra.py"), "--device", "cpu", "--rows", str(n)])
    rng = np.random.default_rng(0)
    left = pd.DataFrame({"k": rng.integers(0, n // 2, n), "x": rng.random(n)})
    right = pd.DataFrame({"k": rng.integers(0, n // 2, n), "y": rng.random(n)})
    a, b = set(left.k), set(right.k)
    assert int(out["join_rows"]) == len(left.merge(right, on="k"))
    assert int(out["left_join_rows"]) == len(left.merge(right, on="k", how="left"))
    assert int(out["union_rows"]) == len(a | b)
    assert int(out["intersect_rows"]) == len(a & b)
    assert int(out["subtract_rows"]) == len(a - b)
    assert int(out["unique_rows"]) == len(a) == int(out["groups"])
    assert abs(float(out["sorted_first"]) - round(left.x.max(), 6)) < 1e-6


def test_dataframe_example():
    out = _run([sys.executable, os.path.join(EX, "dataframe_ops.py"), "--device", "cpu"])
    assert out["merge_rows"] == "3" and out["left_merge_rows"] == "5" and out["concat_rows"] == "6"
    assert out["sort_first_a"] == "50" and out["group_sums"] == "3.0,12.0" and out["dedup_rows"] == "2"
    assert out["index_join_rows"] == "3" and out["on_host"] == "True"


def test_distributed_example_two_ranks():
    n = 5_000
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = _run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(EX, "distributed_ops.py"),
                "--device", "cpu", "--rows", str(n)], timeout=600)
    assert out["world"] == "2"
    frames = []
    for r in range(2):
        rng = np.random.default_rng(100 + r)
        frames.append((pd.DataFrame({"k": rng.integers(0, 4 * n, n), "x": rng.random(n)}),
                       pd.DataFrame({"k": rng.integers(0, 4 * n, n), "y": rng.random(n)})))
    L = pd.concat([f[0] for f in frames])
    R = pd.concat([f[1] for f in frames])
    tot = lambda key: sum(int(out[f"rank{r}_{key}"]) for r in range(2))
    assert tot("join_rows") == len(L.merge(R, on="k"))
    assert tot("union_rows") == len(set(L.k) | set(R.k))
    assert tot("sorted_rows") == 2 * n
    assert tot("groups") == L.k.nunique()
