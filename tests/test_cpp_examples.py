"""The native C++ API without Python: examples/cpp/relational_example.cpp links only
cylon_amd/libcylon_amd.so (+ libtorch) and must agree with the Python API."""
import os
import subprocess

import pyarrow as pa
import pyarrow.csv  # noqa: F401
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EXE = os.path.join(ROOT, "examples", "cpp", "bin", "relational_example")


def _ensure_built():
    import fcntl
    import glob
    srcs = glob.glob(os.path.join(ROOT, "examples", "cpp", "*.cpp"))
    exes = [os.path.join(ROOT, "examples", "cpp", "bin", os.path.basename(s)[:-4]) for s in srcs]
    os.makedirs(os.path.join(ROOT, "examples", "cpp", "bin"), exist_ok=True)
    # one builder at a time: parallel test workers would otherwise rewrite an executable another runs
    with open(os.path.join(ROOT, "examples", "cpp", "bin", ".build.lock"), "w") as lock:
        fcntl.flock(lock, fcntl.LOCK_EX)
        newest = max(os.path.getmtime(p) for p in srcs + [os.path.join(ROOT, "cylon_amd", "libcylon_amd.so")])
        if any(not os.path.exists(e) or os.path.getmtime(e) < newest for e in exes):
            subprocess.run(["bash", os.path.join(ROOT, "examples", "cpp", "build.sh")], check=True,
                           capture_output=True)
    return EXE


def _run(device, tmp_path, data_dir):
    exe = _ensure_built() if device == "cpu" else EXE
    r = subprocess.run([exe, device, os.path.join(data_dir, "input", "csv1_0.csv"),
                        os.path.join(data_dir, "input", "csv2_0.csv"), str(tmp_path)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict((k, int(v)) for k, v in (line.split() for line in r.stdout.splitlines()))


def _python_counts(ctx, data_dir):
    from cylon_amd import Table
    from cylon_amd.io import read_csv
    a = read_csv(ctx, os.path.join(data_dir, "input", "csv1_0.csv"))
    b = read_csv(ctx, os.path.join(data_dir, "input", "csv2_0.csv"))
    return {"left": a.row_count, "right": b.row_count,
            "join_hash": a.join(b, "inner", "hash", on=[0]).row_count,
            "join_sort": a.join(b, "inner", "sort", on=[0]).row_count,
            "union": a.union(b).row_count, "intersect": a.intersect(b).row_count,
            "subtract": a.subtract(b).row_count, "unique_col0": a.unique([a.column_names[0]]).row_count,
            "sort": a.row_count, "sum_col1": 1}


def test_cpp_example_on_cpu(ctx, tmp_path, data_dir):
    got = _run("cpu", tmp_path, data_dir)
    exp = _python_counts(ctx, data_dir)
    for k, v in exp.items():
        assert got[k] == v, (k, got, exp)
    assert got["parquet_roundtrip"] == got["join_hash"]
    assert got["groupby_sum"] == got["unique_col0"]
    assert pa.csv.read_csv(str(tmp_path / "join.csv")).num_rows == got["join_hash"]


@pytest.mark.gpu
def test_cpp_example_on_gpu(tmp_path, data_dir):
    if not os.path.exists(EXE):
        pytest.fail("examples/cpp/bin/relational_example missing: run __graft_entry__.build()")
    from cylon_amd import CylonContext
    got = _run("cuda:0", tmp_path, data_dir)
    exp = _python_counts(CylonContext(device="cpu"), data_dir)
    for k, v in exp.items():
        assert got[k] == v, (k, got, exp)


REG = os.path.join(ROOT, "examples", "cpp", "bin", "registry_example")


def _run_registry(device, tmp_path, data_dir):
    if device == "cpu":
        _ensure_built()
    r = subprocess.run([REG, device, os.path.join(data_dir, "input", "csv1_0.csv"),
                        os.path.join(data_dir, "input", "csv2_0.csv"), str(tmp_path)],
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict((k, int(v)) for k, v in (line.split() for line in r.stdout.splitlines()))


def _check_registry(got, ctx, data_dir):
    from cylon_amd.io import read_csv
    a = read_csv(ctx, os.path.join(data_dir, "input", "csv1_0.csv"))
    b = read_csv(ctx, os.path.join(data_dir, "input", "csv2_0.csv"))
    first = a.to_pandas().iloc[:, 0]
    exp = {"a": a.row_count, "b": b.row_count, "j": a.join(b, "inner", "hash", on=[0]).row_count,
           "s": a.subtract(b).row_count, "i": a.intersect(b).row_count, "m": a.row_count + b.row_count,
           "sel": int((first % 2 == 0).sum()), "partitions": 3, "partition_rows": a.row_count, "p_columns": 2,
           "printed_lines": 1 + min(3, a.join(b, "inner", "hash", on=[0]).row_count)}
    for k, v in exp.items():
        assert got[k] == v, (k, got, exp)
    assert got["p"] == got["j"] == got["j2"]
    if got["sel"]:
        assert got["sel_first_even"] == 1


def test_cpp_registry_example_on_cpu(ctx, tmp_path, data_dir):
    _check_registry(_run_registry("cpu", tmp_path, data_dir), ctx, data_dir)


@pytest.mark.gpu
def test_cpp_registry_example_on_gpu(tmp_path, data_dir):
    from cylon_amd import CylonContext
    if not os.path.exists(REG):
        pytest.fail("examples/cpp/bin/registry_example missing: run __graft_entry__.build()")
    _check_registry(_run_registry("cuda:0", tmp_path, data_dir), CylonContext(device="cpu"), data_dir)


def _rows(path):
    import pandas as pd
    df = pd.read_csv(path)
    return sorted(tuple(round(float(x), 6) for x in r) for r in df.itertuples(index=False))


@pytest.mark.parametrize("world", [2, 4])
def test_cpp_example_native_distributed_tcp(tmp_path, data_dir, world):
    """relational_example brings its context up natively (CylonContext::InitDistributed from the
    torchrun environment, TCPStore rendezvous, native TCP mesh; no Python in the ranks) and every
    rank's distributed join / union / intersect / subtract matches the reference's golden files
    (reference: ctx/cylon_context.cpp:32-43, net/mpi/mpi_communicator.cpp:51-60)."""
    import socket
    exe = _ensure_built()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(world):
        env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC")}
        env.update(RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        procs.append(subprocess.Popen([exe, "tcp", os.path.join(data_dir, "input", "csv1_%r.csv"),
                                       os.path.join(data_dir, "input", "csv2_%r.csv"), str(tmp_path)],
                                      stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
    res = [p.communicate(timeout=180) for p in procs]
    errs = "\n".join(f"rank {r} rc={p.returncode}: {e[-1500:]}" for r, (p, (_, e)) in enumerate(zip(procs, res)))
    assert all(p.returncode == 0 for p in procs), errs
    outs = [dict((k, int(v)) for k, v in (line.split() for line in o.splitlines())) for o, _ in res]
    gold = os.path.join(data_dir, "output")
    for r, got in enumerate(outs):
        assert _rows(tmp_path / f"join_{r}.csv") == _rows(os.path.join(gold, f"join_inner_{world}_{r}.csv"))
        for op in ("union", "intersect", "subtract"):
            assert got[op] == len(_rows(os.path.join(gold, f"{op}_{world}_{r}.csv"))), (r, op)
        assert got["parquet_roundtrip"] == got["join_hash"]
    assert len({o["sum_col1"] for o in outs}) == 1


# ---------------------------------------------------------------------------
# the example programs mirroring the reference's cpp/src/examples (groupby, sorting, unique,
# partition, select / project / table-from-vectors, indexing): every printed result checked
# against the Python API on the same input
# ---------------------------------------------------------------------------
def _run_example(name, device, *args):
    if device == "cpu":
        _ensure_built()
    exe = os.path.join(ROOT, "examples", "cpp", "bin", name)
    if not os.path.exists(exe):
        pytest.fail(f"examples/cpp/bin/{name} missing: run __graft_entry__.build()")
    r = subprocess.run([exe, device, *args], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return dict((k, int(v)) for k, v in (line.split() for line in r.stdout.splitlines()))


def _check_examples(device, data_dir):
    import pandas as pd
    from cylon_amd import CylonContext
    from cylon_amd.io import read_csv
    ctx = CylonContext(device="cpu")
    csv = os.path.join(data_dir, "input", "csv1_0.csv")
    t = read_csv(ctx, csv)
    df = t.to_pandas()
    c0 = df.columns[0]

    got = _run_example("groupby_example", device, csv)
    assert got["hash_groups"] == got["pipeline_groups"] == df[c0].nunique()
    assert got["hash_columns"] == 9 and got["count_col1"] == len(df)
    assert got["pipeline_matches_hash"] == got["group_sums_match_total"] == got["minmax_consistent"] == 1

    got = _run_example("sorting_example", device, csv)
    assert got["sort_asc_rows"] == got["dist_sort_rows"] == len(df)
    assert all(got[k] == 1 for k in ("sort_asc_ok", "sort_desc_ok", "sort_multi_ok", "dist_sort_ok")), got

    got = _run_example("unique_example", device, csv)
    assert got["unique_first"] == got["unique_last"] == got["distributed_unique"] == df[c0].nunique()
    assert got["unique_all_columns"] == len(df.drop_duplicates())
    assert got["unique_first"] == t.unique([c0], keep="first").row_count
    assert got["unique_last"] == t.unique([c0], keep="last").row_count

    got = _run_example("partition_example", device, csv, "4")
    assert got["partition_total"] == got["shuffled"] == len(df)
    for p in range(4):  # reference modulo partition of an int64 key: (uint32)v % 4
        assert got[f"partition_{p}"] == int(((df[c0].to_numpy().astype("uint32")) % 4 == p).sum()), p

    got = _run_example("select_project_example", device, csv)
    assert got["select_even_col0"] == int((df[c0] % 2 == 0).sum())
    assert got["project_columns"] == 1 and got["merge_rows"] == len(df) + got["select_even_col0"]
    assert got["vector_table_rows"] == 5 and got["vector_table_first_id"] == 1 and got["vector_table_sum_x10"] == 125

    icsv = os.path.join(data_dir, "input", "indexing_data.csv")
    idf = pd.read_csv(icsv)
    got = _run_example("indexing_example", device, icsv)
    labels = idf.iloc[:3, 0].tolist()
    want = int(idf.iloc[:, 0].isin(labels).sum())
    assert got["loc_hash"] == got["loc_sorted"] == got["loc_linear"] == want
    assert got["iloc_range"] == 5
    it = read_csv(ctx, icsv)
    it.set_index(it.column_names[0])
    assert got["loc_range"] == it.loc[labels[1]:labels[2]].row_count


def _gen(seed, n, rng):
    import pandas as pd
    import torch
    g = torch.Generator().manual_seed(seed)
    k = torch.randint(rng, (n,), generator=g, dtype=torch.long)
    v = torch.rand(n, generator=g, dtype=torch.float64)
    return pd.DataFrame({"k": k.numpy(), "v": v.numpy()})


def _check_more_examples(device, data_dir):
    """join (4 types x hash/sort + multi-index), scalar aggregates, in-memory datagen."""
    import numpy as np
    import pandas as pd
    from cylon_amd import CylonContext
    from cylon_amd.io import read_csv
    ctx = CylonContext(device="cpu")
    c1, c2 = (os.path.join(data_dir, "input", f) for f in ("csv1_0.csv", "csv2_0.csv"))
    a, b = read_csv(ctx, c1).to_pandas(), read_csv(ctx, c2).to_pandas()
    got = _run_example("join_example", device, c1, c2)
    ka, kb = a.columns[0], b.columns[0]
    for name, how in (("inner", "inner"), ("left", "left"), ("right", "right"), ("outer", "outer")):
        want = len(a.merge(b, left_on=ka, right_on=kb, how=how))
        assert got[f"{name}_hash"] == got[f"{name}_sort"] == want, (name, got)
        assert got[f"{name}_algorithms_agree"] == 1
    assert got["inner_multi_idx"] == len(a.merge(b, left_on=list(a.columns[:2]), right_on=list(b.columns[:2])))

    got = _run_example("compute_example", device, c1)
    assert got["rows"] == len(a)
    for c, col in enumerate(a.columns):
        if not np.issubdtype(a[col].dtype, np.number):
            continue
        assert got[f"col{c}_sum_x1000"] == int(round(a[col].sum() * 1000)), col
        assert got[f"col{c}_count"] == int(a[col].count())
        assert got[f"col{c}_min_x1000"] == int(round(a[col].min() * 1000))
        assert got[f"col{c}_max_x1000"] == int(round(a[col].max() * 1000))
        assert got[f"col{c}_minmax_consistent"] == 1

    n = 20000
    got = _run_example("datagen_join_example", device, str(n))
    l, r = _gen(1000, n, 4 * n), _gen(1001, n, 4 * n)
    assert got["join_rows"] == len(l.merge(r, on="k"))
    assert got["union_rows"] == len(set(l.k) | set(r.k)) and got["intersect_rows"] == len(set(l.k) & set(r.k))
    assert got["sorted_rows"] == n and got["sorted_ok"] == 1


def test_cpp_more_examples_on_cpu(data_dir):
    _check_more_examples("cpu", data_dir)


@pytest.mark.gpu
def test_cpp_more_examples_on_gpu(data_dir):
    _check_more_examples("cuda:0", data_dir)


def test_cpp_datagen_example_distributed_tcp():
    """datagen_join_example as 3 native TCP ranks: per-rank results sum to the pandas totals."""
    import socket
    _ensure_built()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    n, W = 5000, 3
    exe = os.path.join(ROOT, "examples", "cpp", "bin", "datagen_join_example")
    procs = []
    for r in range(W):
        env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC")}
        env.update(RANK=str(r), WORLD_SIZE=str(W), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([exe, "tcp", str(n)], stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True,
                                      env=env))
    res = [p.communicate(timeout=180) for p in procs]
    assert all(p.returncode == 0 for p in procs), [e[-1500:] for _, e in res]
    outs = [dict((k, int(v)) for k, v in (line.split() for line in o.splitlines())) for o, _ in res]
    import pandas as pd
    L = pd.concat([_gen(1000 + 2 * r, n, 4 * n) for r in range(W)])
    R = pd.concat([_gen(1001 + 2 * r, n, 4 * n) for r in range(W)])
    assert sum(o["join_rows"] for o in outs) == len(L.merge(R, on="k"))
    assert sum(o["union_rows"] for o in outs) == len(set(L.k) | set(R.k))
    assert sum(o["intersect_rows"] for o in outs) == len(set(L.k) & set(R.k))
    assert sum(o["sorted_rows"] for o in outs) == W * n and all(o["sorted_ok"] == 1 for o in outs)


def test_cpp_reference_examples_on_cpu(data_dir):
    _check_examples("cpu", data_dir)


@pytest.mark.gpu
def test_cpp_reference_examples_on_gpu(data_dir):
    _check_examples("cuda:0", data_dir)


def test_cpp_examples_distributed_tcp(data_dir):
    """groupby / sorting examples as 2 native TCP ranks: the distributed sort leaves every rank
    ordered and the group-by's pipeline and hash results agree on every rank."""
    import socket
    _ensure_built()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    for name in ("groupby_example", "sorting_example"):
        exe = os.path.join(ROOT, "examples", "cpp", "bin", name)
        procs = []
        for r in range(2):
            env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC")}
            env.update(RANK=str(r), WORLD_SIZE="2", LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                       MASTER_PORT=str(port))
            procs.append(subprocess.Popen([exe, "tcp", os.path.join(data_dir, "input", f"csv1_{r}.csv")],
                                          stdout=subprocess.PIPE, stderr=subprocess.PIPE, text=True, env=env))
        res = [p.communicate(timeout=180) for p in procs]
        assert all(p.returncode == 0 for p in procs), [e[-1500:] for _, e in res]
        outs = [dict((k, int(v)) for k, v in (line.split() for line in o.splitlines())) for o, _ in res]
        for o in outs:
            if name == "sorting_example":
                assert o["dist_sort_ok"] == 1 and o["sort_multi_ok"] == 1
            else:
                assert o["pipeline_matches_hash"] == 1 and o["group_sums_match_total"] == 1
        port += 1


def _check_io_graph_examples(device, data_dir, out_dir):
    """parquet_example (CSV -> Parquet -> device round trip, multi-file and column-subset reads,
    join / union of the Parquet tables) and op_graph_example (DisJoinOP / DisUnionOp fed in
    batches vs the one-shot operators), against pandas."""
    import pandas as pd
    c1, c2 = (os.path.join(data_dir, "input", f) for f in ("csv1_0.csv", "csv2_0.csv"))
    l, r = pd.read_csv(c1), pd.read_csv(c2)
    k = l.columns[0]
    join_rows = len(l.merge(r, on=k))
    union_rows = len(pd.concat([l, r]).drop_duplicates())
    got = _run_example("parquet_example", device, c1, c2, str(out_dir))
    assert got["left_rows"] == len(l) and got["right_rows"] == len(r) and got["roundtrip_equal"] == 1, got
    assert got["multi_file_rows"] == len(l) + len(r) and got["subset_columns"] == 1, got
    assert got["join_rows"] == join_rows and got["union_rows"] == union_rows, got
    got = _run_example("op_graph_example", device, c1, c2, "4")
    assert got["op_join_rows"] == got["direct_join_rows"] == join_rows, got
    assert got["op_union_rows"] == got["direct_union_rows"] == union_rows, got


def test_cpp_io_graph_examples_on_cpu(data_dir, tmp_path):
    _check_io_graph_examples("cpu", data_dir, tmp_path)


@pytest.mark.gpu
def test_cpp_io_graph_examples_on_gpu(data_dir, tmp_path):
    _check_io_graph_examples("cuda:0", data_dir, tmp_path)


def test_cpp_io_graph_examples_distributed_tcp(data_dir, tmp_path):
    """parquet_example and op_graph_example as 2 native TCP ranks (rank r reads csv{1,2}_r):
    per-rank join / union rows of the streamed op graph equal the one-shot distributed operators',
    and their sums equal pandas on the concatenated inputs."""
    import socket
    import pandas as pd
    _ensure_built()
    W = 2
    files = [[os.path.join(data_dir, "input", f"csv{s}_{r}.csv") for s in (1, 2)] for r in range(W)]
    L = pd.concat([pd.read_csv(f[0]) for f in files])
    R = pd.concat([pd.read_csv(f[1]) for f in files])
    k = L.columns[0]
    for name, extra in (("parquet_example", [str(tmp_path)]), ("op_graph_example", ["3"])):
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        exe = os.path.join(ROOT, "examples", "cpp", "bin", name)
        procs = []
        for r in range(W):
            env = {k2: v for k2, v in os.environ.items() if not k2.startswith("TORCHELASTIC")}
            env.update(RANK=str(r), WORLD_SIZE=str(W), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
            procs.append(subprocess.Popen([exe, "tcp", *files[r], *extra], stdout=subprocess.PIPE,
                                          stderr=subprocess.PIPE, text=True, env=env))
        res = [p.communicate(timeout=180) for p in procs]
        assert all(p.returncode == 0 for p in procs), [e[-1500:] for _, e in res]
        outs = [dict((a, int(b)) for a, b in (line.split() for line in o.splitlines())) for o, _ in res]
        if name == "parquet_example":
            assert all(o["roundtrip_equal"] == 1 for o in outs)
            assert sum(o["join_rows"] for o in outs) == len(L.merge(R, on=k))
            assert sum(o["union_rows"] for o in outs) == len(pd.concat([L, R]).drop_duplicates())
        else:
            assert all(o["op_join_rows"] == o["direct_join_rows"] and o["op_union_rows"] == o["direct_union_rows"]
                       for o in outs), outs
            assert sum(o["op_join_rows"] for o in outs) == len(L.merge(R, on=k))
