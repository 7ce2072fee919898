"""Op-graph runtime, table all-to-all, task all-to-all and the registry
(reference: cpp/src/examples/ops/join_op_example.cpp, task_test.cpp, table_api)."""
import numpy as np
import pandas as pd
import pyarrow as pa
import pytest

from cylon_amd import Table
from cylon_amd.parallel import DisJoinOp, DisUnionOp, TableAllToAll, TableRegistry, TaskAllToAll

from dist_utils import run_distributed


def _rows(df):
    return sorted(map(tuple, df.itertuples(index=False)))


def _op_graph(ctx, nbatches):
    rank = ctx.get_rank()
    rng = np.random.default_rng(rank)
    lefts = [pd.DataFrame({"k": rng.integers(0, 50, 40), "v": rng.random(40)}) for _ in range(nbatches)]
    rights = [pd.DataFrame({"k": rng.integers(0, 50, 30), "w": rng.random(30)}) for _ in range(nbatches + rank)]
    op = DisJoinOp(ctx, "inner", "hash", [0], [0], "l_", "r_", num_splits=8)
    for d in lefts:
        op.insert_table(DisJoinOp.LEFT, Table.from_pandas(ctx, d))
    for d in rights:
        op.insert_table(DisJoinOp.RIGHT, Table.from_pandas(ctx, d))
    res = op.execute()
    got = pd.concat([r.to_pandas() for r in res]) if res else pd.DataFrame()
    u = DisUnionOp(ctx)
    for d in lefts:
        u.insert_table(0, Table.from_pandas(ctx, d))
    un = pd.concat([r.to_pandas() for r in u.execute()])
    return got, pd.concat(lefts), pd.concat(rights), un


@pytest.mark.parametrize("world", [1, 3])
def test_dis_join_op_graph(world):
    res = run_distributed(_op_graph, world, 2)
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    exp = a.add_prefix("l_").merge(b.add_prefix("r_"), left_on="l_k", right_on="r_k")
    assert _rows(got) == _rows(exp[got.columns])
    un = pd.concat([r[3] for r in res])
    assert _rows(un) == _rows(a.drop_duplicates())


def _a2a(ctx):
    rank, world = ctx.get_rank(), ctx.get_world_size()
    seen = []
    a2a = TableAllToAll(ctx, lambda src, t, ref: seen.append((src, ref, t.to_pydict()["x"])) or True)
    for target in range(world):
        a2a.insert(Table(pa.table({"x": [rank * 10 + target]}), ctx), target, reference=rank * 100 + target)
        a2a.insert(Table(pa.table({"x": [rank * 10 + target, -1]}), ctx), target, reference=7)
    a2a.finish()
    while not a2a.is_complete():
        pass
    tasks = TaskAllToAll(ctx, [t % world for t in range(2 * world)])
    for task in range(2 * world):
        tasks.insert(Table(pa.table({"x": [task]}), ctx), task)
    got = [(s, r, t.to_pydict()["x"]) for s, t, r in tasks.wait_for_completion()]
    return seen, got


def test_table_all_to_all_protocol():
    world = 3
    res = run_distributed(_a2a, world)
    for rank, (seen, tasks) in enumerate(res):
        exp = []
        for src in range(world):
            exp.append((src, src * 100 + rank, [src * 10 + rank]))
            exp.append((src, 7, [src * 10 + rank, -1]))
        assert sorted(seen) == sorted(exp)
        mine = sorted(t for t in range(2 * world) if t % world == rank)
        assert sorted(r for _, r, _ in tasks) == sorted(mine * world)


def test_registry(ctx):
    reg = TableRegistry(ctx)
    reg.put("a", Table(pa.table({"k": [1, 2, 3], "v": [1, 2, 3]}), ctx))
    reg.put("b", Table(pa.table({"k": [2, 3, 4], "w": [5, 6, 7]}), ctx))
    reg.join("a", "b", "j", "inner", "hash")
    assert reg.row_count("j") == 2 and reg.column_count("j") == 4
    reg.union("a", "a", "u")
    assert reg.get("u").row_count == 3
    assert set(reg.ids()) >= {"a", "b", "j", "u"}
    reg.remove("j")
    assert "j" not in reg.ids()


def _channel(ctx):
    import torch
    from cylon_amd.net import Channel, ChannelReceiveCallback, ChannelSendCallback, TxRequest
    rank, world = ctx.get_rank(), ctx.get_world_size()
    got, sent = [], []

    class R(ChannelReceiveCallback):
        def received_header(self, source, finished, header):
            got.append(("h", source, finished, list(header[:2])))

        def received_data(self, source, buffer):
            got.append(("d", source, buffer.view(torch.int64).tolist()))

    class S(ChannelSendCallback):
        def send_complete(self, req):
            sent.append(req.header[0])

        def send_finish_complete(self, req):
            sent.append("fin")

    rcb, scb = R(), S()
    peers = [r for r in range(world) if r != rank]
    ch = Channel(ctx)
    ch.init(7, peers, peers, rcb, scb)
    for p in peers:
        for m in range(3):
            ch.send(TxRequest(p, torch.arange(m + 1, dtype=torch.int64) + 100 * rank, [m, rank]))
        ch.send(TxRequest(p, None, [9, 9]))  # header-only message
        ch.send_fin(TxRequest(p))
    import time
    t0 = time.time()
    while not ch.is_complete() and time.time() - t0 < 60:
        ch.progress_sends()
        ch.progress_receives()
    ch.close()
    return got, sent


def test_channel_point_to_point():
    res = run_distributed(_channel, 2)
    for rank, (got, sent) in enumerate(res):
        other = 1 - rank
        assert sent == [0, 1, 2, 9, "fin"]
        datas = [g[2] for g in got if g[0] == "d"]
        assert datas[:3] == [[100 * other + i for i in range(m + 1)] for m in range(3)]
        heads = [g for g in got if g[0] == "h"]
        assert heads[0][3] == [0, other] and heads[-1][2] == 1 and len(heads) == 5


def _etl(ctx, data_dir):
    import os
    import torch
    from cylon_amd.io import read_csv
    from cylon_amd.models import join_features, train_ddp
    r = ctx.get_rank() + 1
    dev = read_csv(ctx, os.path.join(data_dir, f"user_device_tm_{r}.csv"))
    use = read_csv(ctx, os.path.join(data_dir, f"user_usage_tm_{r}.csv"))
    x, y = join_features(dev, use)
    model, loss = train_ddp(x, y, epochs=2, train_rows=50)
    # DDP keeps replicas identical
    w = torch.cat([p.detach().reshape(-1) for p in model.parameters()])
    return x.shape[0], x.shape[1], loss, w.tolist()


def test_etl_to_ddp_pipeline():
    import os
    d = os.path.join(os.path.dirname(__file__), "data", "tutorial")
    res = run_distributed(_etl, 2, d)
    for rows, feats, loss, _ in res:
        assert rows > 50 and feats == 4 and loss == loss
    assert np.allclose(res[0][3], res[1][3])


def test_bench_contract_multirank_cpu_rehearsal():
    """bench.py under torch.distributed.run (2 ranks, gloo): one JSON line with the driver's fields."""
    import json
    import os
    import socket
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ, CYLON_BENCH_BACKEND="gloo")
    out = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                          "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.join(root, "bench.py"),
                          "--gpus", "2", "--steps", "2", "--warmup", "1", "--rows", "100000"],
                         capture_output=True, text=True, timeout=240, env=env, cwd="/tmp")
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode == 0 and len(lines) == 1, out.stderr[-2000:]
    rec = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config"):
        assert k in rec
    assert rec["n_gpus"] == 2 and rec["steps"] == 2 and rec["config"]["output_rows"] > 0
    # self-validating multi-rank record: verified by default, one entry per rank with its world size
    assert rec["verify"]["ok"] and rec["verify"]["rows"] == rec["config"]["output_rows"]
    assert [r["rank"] for r in rec["ranks"]] == [0, 1] and all(r["world_size_pg"] == 2 for r in rec["ranks"])


def test_bench_self_launch_four_ranks_cpu():
    """bench.py --gpus 4 with no torchrun environment starts 4 ranks itself (child torchrun) and
    reports n_gpus == 4, per-phase timings and a passing verify of a FULL OUTER join; a WORLD_SIZE that disagrees
    with --gpus exits non-zero (reference launch: cpp/src/experiments/run_dist_scaling.py:115-154)."""
    import json
    import os
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["CYLON_BENCH_BACKEND"] = "gloo"
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--steps", "2",
                          "--warmup", "1", "--rows", "80000", "--how", "outer"],
                         capture_output=True, text=True, timeout=300, env=env, cwd="/tmp")
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert out.returncode == 0 and len(lines) == 1, out.stderr[-2000:]
    rec = json.loads(lines[0])
    assert rec["n_gpus"] == 4 and rec["steps"] == 2 and rec["warmup"] == 1
    assert rec["verify"]["ok"] and rec["verify"]["rows"] == rec["config"]["output_rows"]
    ph = rec["phases_ms_max_over_ranks"]
    assert "shuffle.plan" in ph and "shuffle.reorder+post" in ph, ph  # one planning collective, then posts
    bad = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "4", "--rows", "1000"],
                         capture_output=True, text=True, timeout=120, cwd="/tmp",
                         env=dict(env, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0"))
    assert bad.returncode == 2 and "WORLD_SIZE" in bad.stderr


def _op_graph_uneven(ctx):
    """Ranks feed different numbers of batches; the streaming exchange keeps rounds matched."""
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    rng = np.random.default_rng(10 + rank)
    nb_left = 5 if rank == 0 else 1
    lefts = [pd.DataFrame({"k": rng.integers(0, 60, 50), "v": rng.random(50)}) for _ in range(nb_left)]
    rights = [pd.DataFrame({"k": rng.integers(0, 60, 35), "w": rng.random(35)}) for _ in range(2 + rank)]
    C.trace_enable(True)
    C.trace_reset()
    op = DisJoinOp(ctx, "inner", "hash", [0], [0], "l_", "r_", num_splits=4)
    for d in lefts:
        op.insert_table(DisJoinOp.LEFT, Table.from_pandas(ctx, d))
    for d in rights:
        op.insert_table(DisJoinOp.RIGHT, Table.from_pandas(ctx, d))
    res = op.execute()
    got = pd.concat([r.to_pandas() for r in res]) if res else pd.DataFrame()
    return got, pd.concat(lefts), pd.concat(rights), dict(C.trace_counters())


def test_dis_join_op_streaming_rounds():
    """AllToAllOp streams (reference all_to_all_op.cpp:40-62): one collective round per batch,
    empty rounds for ranks whose inputs ended, results equal to pandas."""
    res = run_distributed(_op_graph_uneven, 2)
    got = pd.concat([r[0] for r in res])
    a = pd.concat([r[1] for r in res])
    b = pd.concat([r[2] for r in res])
    exp = a.add_prefix("l_").merge(b.add_prefix("r_"), left_on="l_k", right_on="r_k")
    assert len(got) == len(exp) and _rows(got) == _rows(exp[got.columns])
    for r in res:
        c = r[3]
        # left: 5 rounds (rank 0's batches), right: 3 rounds -- identical on both ranks
        assert c.get("graph.alltoall.rounds") == 8, c


def _eight_rank_ops(ctx):
    """One rank of the 8-rank rehearsal: chunked planned joins (inner, left) with the gapped
    exchange layout, a two-key join, a distributed group-by and a distributed sort."""
    import numpy as np
    import pandas as pd
    from cylon_amd import Table
    from cylon_amd._lib import C
    rank = ctx.get_rank()
    rng = np.random.default_rng(800 + rank)
    n = 3000 + 250 * rank
    a = pd.DataFrame({"k": rng.integers(0, 9000, n), "g": rng.integers(0, 3, n), "v": rng.random(n)})
    b = pd.DataFrame({"k": rng.integers(0, 9000, n), "g": rng.integers(0, 3, n), "w": rng.random(n)})
    ctx.add_config("shuffle_chunks", "3")
    ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
    C.trace_enable(True)
    C.trace_reset()
    out = {"inner": ta.distributed_join(tb, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_"),
           "left": ta.distributed_join(tb, "left", "hash", on=["k"], left_prefix="l_", right_prefix="r_"),
           "two": ta.distributed_join(tb, "inner", "hash", on=["k", "g"], left_prefix="l_", right_prefix="r_")}
    counters = dict(C.trace_counters())
    out["gb"] = ta.groupby("k", {"v": ["sum", "count"]})
    out["sort"] = ta.distributed_sort("k")
    return {k: v.to_pandas() for k, v in out.items()}, a, b, counters


def test_eight_rank_distributed_rehearsal():
    """8 ranks over gloo (the driver's 8-GPU shape on CPUs): every rank's results together equal
    pandas on the concatenated inputs; the own partition of each chunk stays in place."""
    import pandas as pd
    from dist_utils import run_distributed
    res = run_distributed(_eight_rank_ops, 8)
    A = pd.concat([r[1] for r in res]).reset_index(drop=True)
    B = pd.concat([r[2] for r in res]).reset_index(drop=True)

    def canon(df):
        df = df[sorted(df.columns)]
        return df.sort_values(list(df.columns), kind="mergesort", na_position="last").reset_index(drop=True)

    la, rb = A.add_prefix("l_"), B.add_prefix("r_")
    exp_inner = la.merge(rb, left_on="l_k", right_on="r_k")
    exp_left = la.merge(rb, left_on="l_k", right_on="r_k", how="left")
    exp_two = la.merge(rb, left_on=["l_k", "l_g"], right_on=["r_k", "r_g"])
    for name, exp in (("inner", exp_inner), ("left", exp_left), ("two", exp_two)):
        got = pd.concat([r[0][name] for r in res])
        pd.testing.assert_frame_equal(canon(got), canon(exp), check_dtype=False, obj=name)
    gb = pd.concat([r[0]["gb"] for r in res]).sort_values("k").reset_index(drop=True)
    eg = A.groupby("k")["v"].agg(["sum", "count"]).reset_index()
    assert gb["k"].tolist() == eg["k"].tolist() and gb["count_v"].tolist() == eg["count"].tolist()
    srt = pd.concat([r[0]["sort"] for r in res])["k"].tolist()
    assert srt == sorted(A["k"].tolist())
    for r in res:
        assert r[3].get("shuffle.self_rows_kept_local", 0) > 0, r[3]
        assert r[3].get("shuffle.plan_collectives", 0) == 3, r[3]


def _idle_rank_ops(ctx, chunks):
    """Rank 2 holds empty tables and no key of ranks 0 / 1 hashes to it: in every chunk its own
    sends and receives are all zero while the other ranks exchange (the collective
    must still be posted on every rank, or the busy ranks block)."""
    from cylon_amd import CylonContext
    from cylon_amd._lib import C
    rank, world = ctx.get_rank(), ctx.get_world_size()
    ctx.add_config("shuffle_chunks", str(chunks))
    # keys whose planned-shuffle partition (hash % (world * chunks)) maps to rank 0 or 1
    local = CylonContext()
    cand = Table.from_pandas(local, pd.DataFrame({"k": np.arange(600, dtype=np.int64)}))
    parts = cand.hash_partition(["k"], world * chunks)
    keys = np.concatenate([t.to_pandas()["k"].to_numpy() for p, t in enumerate(parts) if p % world != 2])
    rng = np.random.default_rng(rank)
    n = 0 if rank == 2 else 300
    a = pd.DataFrame({"k": rng.choice(keys, n).astype(np.int64), "v": rng.random(n)})
    b = pd.DataFrame({"k": rng.choice(keys, n).astype(np.int64), "w": rng.random(n)})
    C.trace_enable(True)
    C.trace_reset()
    ta, tb = Table.from_pandas(ctx, a), Table.from_pandas(ctx, b)
    out = {"join": ta.distributed_join(tb, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_"),
           "union": ta[["k"]].distributed_union(tb[["k"]]),
           "gb": ta.groupby("k", {"v": ["sum"]})}
    counters = dict(C.trace_counters())
    C.trace_enable(False)
    return {k: v.to_pandas() for k, v in out.items()}, a, b, counters


@pytest.mark.parametrize("chunks", [1, 2])
def test_idle_rank_still_posts_collectives(chunks):
    res = run_distributed(_idle_rank_ops, 3, chunks, timeout=120.0)
    A = pd.concat([r[1] for r in res]).reset_index(drop=True)
    B = pd.concat([r[2] for r in res]).reset_index(drop=True)
    assert len(res[2][0]["join"]) == 0 and len(res[2][0]["union"]) == 0  # rank 2 stayed idle
    exp = A.add_prefix("l_").merge(B.add_prefix("r_"), left_on="l_k", right_on="r_k")
    got = pd.concat([r[0]["join"] for r in res])
    assert _rows(got[sorted(got.columns)]) == _rows(exp[sorted(exp.columns)])
    un = sorted(pd.concat([r[0]["union"] for r in res])["k"].tolist())
    assert un == sorted(set(A["k"]) | set(B["k"]))
    gb = pd.concat([r[0]["gb"] for r in res]).sort_values("k")
    assert gb["k"].tolist() == sorted(set(A["k"]))
    assert all(r[3].get("shuffle.plan_collectives", 0) >= 1 for r in res)


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


@pytest.mark.parametrize("world,chunks", [(2, 3), (3, 2)])
def test_planned_shuffle_var_width_chunked(world, chunks):
    """Tables with string columns take the planned, chunked exchange (not the unplanned ShufflePair):
    a string-key join, a LEFT join and a union, against pandas on the gathered inputs."""
    res = run_distributed(_string_join_chunks, world, chunks, 3_000, timeout=200.0)
    _check_string_join(res, chunks)
