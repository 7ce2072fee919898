"""Local relational operators on one device: join (hash and sort), union, intersect, subtract,
unique, sort, group-by and projection (reference: python/examples/table_relational_algebra.py,
cylon_operators.py).

    python examples/python/table_relational_algebra.py [--device cpu|cuda:0] [--rows N]
"""
import numpy as np

from _common import device_from_argv, report, rows_from_argv
from cylon_amd import CylonContext, Table

dev = device_from_argv()
n = rows_from_argv(100_000)
ctx = CylonContext(device=dev)
rng = np.random.default_rng(0)
left = Table.from_numpy(ctx, ["k", "x"], [rng.integers(0, n // 2, n), rng.random(n)])
right = Table.from_numpy(ctx, ["k", "y"], [rng.integers(0, n // 2, n), rng.random(n)])

hj = left.join(right, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")
sj = left.join(right, "inner", "sort", on=["k"], left_prefix="l_", right_prefix="r_")
assert hj.row_count == sj.row_count
report("join_rows", hj.row_count)
report("left_join_rows", left.join(right, "left", "hash", on=["k"], left_prefix="l_", right_prefix="r_").row_count)

a = left.project(["k"])
b = right.project(["k"])
report("union_rows", a.union(b).row_count)
report("intersect_rows", a.intersect(b).row_count)
report("subtract_rows", a.subtract(b).row_count)
report("unique_rows", a.unique().row_count)

s = left.sort("x", ascending=False)
xs = s.to_pandas()["x"].to_numpy()
assert np.all(np.diff(xs) <= 0)
report("sorted_first", round(float(xs[0]), 6))

g = left.groupby("k", {"x": ["sum", "count"]})
report("groups", g.row_count)
