"""Secondary BASELINE.json configs (the headline distributed join is bench.py).

  1. local inner join of two 10k-row CSV tables on the CPU (plumbing path)
  2. single-GPU hash inner join 100M x 100M, int64 keys + int64/float64 payload
  4. hash groupby + sum, 1B rows / 10M int64 groups (whole problem on one GPU, and
     the 125M-row per-GPU share of the 8-GPU config)
  5. radix sort of 2B int64 rows (whole problem on one GPU, and the 250M per-GPU share)
  6. union of two join-shaped relations (the reference's second headline chart)
  7. the headline join with the sort algorithm

Prints one JSON line per config.  Synthetic data generated in HBM (CSV files for 1).
Usage: python tools/bench_suite.py [--configs 1,2,4,5] [--reps 3] [--scale 1.0]
"""
import argparse
import json
import os
import statistics
import sys
import tempfile
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd.io import CSVReadOptions, read_csv  # noqa: E402
from cylon_amd.utils import generate_numeric_csv  # noqa: E402


def timed(fn, reps, warmup=1, sync=True):
    for _ in range(warmup):
        fn()
    ts = []
    for _ in range(reps):
        if sync:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if sync:
            torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts), ts


def verify_sorted(orig, k):
    """Non-decreasing and the same multiset as the input (count, wrapping sum and sum of squares)."""
    if orig.numel() != k.numel():
        return False
    mono = bool((k[1:] >= k[:-1]).all().item())
    same = all(int(a.item()) == int(b.item()) for a, b in ((orig.sum(), k.sum()), ((orig * orig).sum(), (k * k).sum())))
    return mono and same


def verify_groupby(t, res, groups):
    """Group sums against torch index_add over the group ids (outside the timed region)."""
    c = t.to_torch()
    g, x = c["g"], c["x"]
    ref = torch.zeros(groups, dtype=torch.float64, device=g.device).index_add_(0, g, x)
    present = torch.bincount(g, minlength=groups) > 0
    cols = list(res.to_torch().values())
    keys, sums = cols[0], cols[1]
    if keys.numel() != int(present.sum().item()):
        return False
    return bool(torch.allclose(sums, ref[keys], rtol=1e-9, atol=1e-9))


def emit(**kw):
    print(json.dumps(kw), flush=True)


def cfg1(reps):
    ctx = CylonContext()
    d = tempfile.mkdtemp()
    p1 = generate_numeric_csv(10_000, 4, os.path.join(d, "a.csv"), seed=1)
    p2 = generate_numeric_csv(10_000, 4, os.path.join(d, "b.csv"), seed=2)
    opts = CSVReadOptions().use_threads(True)

    def run():
        a = read_csv(ctx, p1, opts)
        b = read_csv(ctx, p2, opts)
        return a.join(b, "inner", "hash", on=[0]).row_count

    med, ts = timed(run, max(reps, 5), warmup=2, sync=False)
    emit(config="1: local CSV inner join 10k x 10k (read_csv + join), CPU", ms=med * 1e3, rows_out=run(),
         all_ms=[t * 1e3 for t in ts])


def rel(n, hi, seed, payload):
    g = torch.Generator(device="cuda").manual_seed(seed)
    cols = {"k": torch.randint(0, hi, (n,), generator=g, device="cuda")}
    for i, dt in enumerate(payload):
        cols[f"v{i}"] = (torch.randint(0, 1 << 40, (n,), generator=g, device="cuda") if dt == "int64"
                         else torch.rand(n, generator=g, device="cuda", dtype=torch.float64))
    return cols


def cfg2(reps, scale):
    ctx = CylonContext(device="cuda:0")
    n = int(100_000_000 * scale)
    hi = int(0.99 * n)
    L = Table.from_torch(ctx, rel(n, hi, 1, ["int64", "float64"]))
    R = Table.from_torch(ctx, rel(n, hi, 2, ["int64", "float64"]))
    out = {}

    def run():
        out["rows"] = L.join(R, "inner", "hash", on=[0]).row_count

    med, ts = timed(run, reps)
    emit(config="2: single-GPU hash inner join 100M x 100M int64 keys, int64+float64 payload", n=n, ms=med * 1e3,
         rows_per_s=2 * n / med, rows_out=out["rows"], all_ms=[t * 1e3 for t in ts])


def cfg4(reps, scale):
    ctx = CylonContext(device="cuda:0")
    groups = 10_000_000
    for n in (int(1_000_000_000 * scale), int(125_000_000 * scale)):
        g = torch.Generator(device="cuda").manual_seed(4)
        t = Table.from_torch(ctx, {"g": torch.randint(0, groups, (n,), generator=g, device="cuda"),
                                   "x": torch.rand(n, generator=g, device="cuda", dtype=torch.float64)})
        out = {}

        def run():
            out["res"] = t.local_groupby("g", {"x": "sum"})
            out["groups"] = out["res"].row_count

        med, ts = timed(run, reps)
        ok = verify_groupby(t, out.pop("res"), groups)
        emit(config="4: hash groupby+sum, 10M int64 groups, one GPU", n=n, ms=med * 1e3, rows_per_s=n / med,
             groups_out=out["groups"], verified=ok, all_ms=[x * 1e3 for x in ts])
        assert ok, "config 4 output differs from the torch index_add reference"
        del t


def cfg5(reps, scale):
    ctx = CylonContext(device="cuda:0")
    for n in (int(2_000_000_000 * scale), int(250_000_000 * scale)):
        g = torch.Generator(device="cuda").manual_seed(5)
        t = Table.from_torch(ctx, {"k": torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, device="cuda")})
        out = {}

        def run():
            out["sorted"] = t.sort("k")

        med, ts = timed(run, reps)
        ok = verify_sorted(t.to_torch()["k"], out.pop("sorted").to_torch()["k"])
        emit(config="5: radix sort of int64 rows (table sort, one GPU)", n=n, ms=med * 1e3, rows_per_s=n / med,
             verified=ok, all_ms=[x * 1e3 for x in ts])
        assert ok, "config 5 output is not a sorted permutation of the input"
        del t


def cfg6(reps, scale):
    """Reference headline #2 (docs/src/pages/index.js:118-134): union of two relations of the
    join benchmark's shape (int64 key + 3 float64), distinct rows, on one GPU."""
    ctx = CylonContext(device="cuda:0")
    for n in (int(200_000_000 * scale), int(1_000_000_000 * scale)):
        hi = int(0.99 * n)
        L = Table.from_torch(ctx, rel(n, hi, 1, ["float64"] * 3))
        R = Table.from_torch(ctx, rel(n, hi, 2, ["float64"] * 3))
        out = {}

        def run():
            out["rows"] = L.distributed_union(R).row_count

        med, ts = timed(run, reps)
        emit(config="6: union (distinct rows), int64 key + 3 float64, one GPU", n=n, ms=med * 1e3,
             rows_per_s=2 * n / med, rows_out=out["rows"], all_ms=[x * 1e3 for x in ts])
        del L, R
        torch.cuda.empty_cache()


def cfg7(reps, scale):
    """The join benchmark with the reference's sort algorithm (arch.md reports sort times for w >= 2)."""
    ctx = CylonContext(device="cuda:0")
    for n in (int(200_000_000 * scale), int(1_000_000_000 * scale)):
        hi = int(0.99 * n)
        L = Table.from_torch(ctx, rel(n, hi, 1, ["float64"] * 3))
        R = Table.from_torch(ctx, rel(n, hi, 2, ["float64"] * 3))
        out = {}

        def run():
            out["rows"] = L.distributed_join(R, "inner", "sort", on=[0]).row_count

        med, ts = timed(run, reps)
        emit(config="7: sort-algorithm inner join, int64 key + 3 float64, one GPU", n=n, ms=med * 1e3,
             rows_per_s=2 * n / med, rows_out=out["rows"], all_ms=[x * 1e3 for x in ts])
        del L, R
        torch.cuda.empty_cache()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--configs", default="1,2,4,5")
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--scale", type=float, default=1.0)
    a = ap.parse_args()
    for c in a.configs.split(","):
        {"1": lambda: cfg1(a.reps), "2": lambda: cfg2(a.reps, a.scale), "4": lambda: cfg4(a.reps, a.scale),
         "5": lambda: cfg5(a.reps, a.scale), "6": lambda: cfg6(a.reps, a.scale),
         "7": lambda: cfg7(a.reps, a.scale)}[c.strip()]()
        torch.cuda.empty_cache() if torch.cuda.is_available() else None


if __name__ == "__main__":
    main()
