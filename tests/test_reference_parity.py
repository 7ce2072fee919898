"""Per-rank result parity with the reference's distributed pycylon tests.

The expected numbers are the reference's own assertions, which encode its partition
functions (Murmur3_x86_32 of the double key for the hash join on a float column,
modulo of the int64 key for the sort join), so matching them per rank checks that
rows land on the same ranks as in the reference, not just that the global result
is right:
  * /root/reference/python/test/test_dist_rl.py:30-98 -- world 4, each rank reads
    user_usage_tm_{rank+1}.csv twice; inner hash join on column 0 (float64),
    union / subtract / intersect of the table with itself;
  * /root/reference/python/test/test_cylon_simple_table_join.py:30-70 -- world 4,
    every rank reads user_usage_tm_1.csv and user_device_tm_1.csv; inner sort join
    left_on=[3] (use_id) right_on=[0] (use_id).
Run over torch.distributed gloo and over the native TCP mesh (CommType TCP)."""
import os

import pytest

from dist_utils import run_distributed

DATA = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data", "tutorial")

# rank -> (join rows, subtract rows, union rows, intersect rows), test_dist_rl.py:76-98
DIST_RL = {0: (1424, 0, 62, 62), 1: (1648, 0, 53, 53), 2: (2704, 0, 53, 53), 3: (1552, 0, 72, 72)}
# rank -> sort-join rows, test_cylon_simple_table_join.py:57-68
SIMPLE_JOIN = {0: 640, 1: 624, 2: 592, 3: 688}


def _dist_rl(ctx):
    from cylon_amd.io import CSVReadOptions, read_csv
    rank = ctx.get_rank()
    opts = CSVReadOptions().use_threads(True).block_size(1 << 30)
    path = os.path.join(DATA, f"user_usage_tm_{rank + 1}.csv")
    tb1, tb2 = read_csv(ctx, path, opts), read_csv(ctx, path, opts)
    tb3 = tb1.distributed_join(table=tb2, join_type="inner", algorithm="hash", left_on=[0], right_on=[0])
    tb4 = tb1.distributed_union(tb2)
    tb5 = tb1.distributed_subtract(tb2)
    tb6 = tb1.distributed_intersect(tb2)
    ctx.barrier()
    return [(t.row_count, t.column_count) for t in (tb3, tb5, tb4, tb6)]


def _simple_join(ctx):
    from cylon_amd.io import CSVReadOptions, read_csv
    opts = CSVReadOptions().use_threads(True).block_size(1 << 30)
    tb1 = read_csv(ctx, os.path.join(DATA, "user_usage_tm_1.csv"), opts)
    tb2 = read_csv(ctx, os.path.join(DATA, "user_device_tm_1.csv"), opts)
    tb3 = tb1.distributed_join(table=tb2, join_type="inner", algorithm="sort", left_on=[3], right_on=[0])
    return tb3.row_count, tb3.column_count


@pytest.mark.parametrize("comm", ["gloo", "tcp"])
def test_dist_rl_per_rank_counts(comm):
    env = {"CYLON_TEST_COMM": comm} if comm == "tcp" else None
    res = run_distributed(_dist_rl, 4, env=env)
    for rank, got in enumerate(res):
        join, sub, uni, inter = DIST_RL[rank]
        assert got == [(join, 8), (sub, 4), (uni, 4), (inter, 4)], (rank, got)


@pytest.mark.parametrize("comm", ["gloo", "tcp"])
def test_simple_table_sort_join_per_rank_counts(comm):
    env = {"CYLON_TEST_COMM": comm} if comm == "tcp" else None
    res = run_distributed(_simple_join, 4, env=env)
    assert [r for r in res] == [(SIMPLE_JOIN[r], 8) for r in range(4)]
