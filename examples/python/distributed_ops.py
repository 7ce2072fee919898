"""Distributed operators, one process per device (reference: python/examples/experiments/
table_join_dist_test.py).  Each rank holds its share of both relations; every operator hash-
or range-shuffles over the communicator (RCCL on GPUs, gloo on CPUs) and runs locally.

    torchrun --nproc-per-node 2 --master-addr 127.0.0.1 examples/python/distributed_ops.py [--device cpu]
"""
import os

import numpy as np

from _common import device_from_argv, report, rows_from_argv
from cylon_amd import CylonEnv, Table

dev = device_from_argv()
if dev.startswith("cuda"):
    dev = f"cuda:{int(os.environ.get('LOCAL_RANK', '0'))}"
env = CylonEnv(distributed=True, device=dev)
ctx = env.context
rank, world = env.rank, env.world_size
n = rows_from_argv(50_000)
rng = np.random.default_rng(100 + rank)
left = Table.from_numpy(ctx, ["k", "x"], [rng.integers(0, 4 * n, n), rng.random(n)])
right = Table.from_numpy(ctx, ["k", "y"], [rng.integers(0, 4 * n, n), rng.random(n)])


j = left.distributed_join(right, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")
u = left.project(["k"]).distributed_union(right.project(["k"]))
s = left.distributed_sort("k")
g = left.groupby("k", {"x": "sum"})  # distributed when the context is
ks = s.to_pandas()["k"].to_numpy()
assert np.all(np.diff(ks) >= 0)
if rank == 0:
    report("world", world)
report(f"rank{rank}_join_rows", j.row_count)
report(f"rank{rank}_union_rows", u.row_count)
report(f"rank{rank}_sorted_rows", s.row_count)
report(f"rank{rank}_groups", g.row_count)
env.barrier()
env.finalize()
