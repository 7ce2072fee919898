"""Time the join types (inner / left / right / full outer) and a two-int-key inner join on the
headline shape (int64 key + 3 float64 payload per side, keys uniform in [0, 0.99 n)).

usage: python tools/join_types_probe.py <rows per side> [reps] [types, comma separated]
types: inner, left, right, outer, inner2 (two int64 keys), left2
One JSON line per type: median ms over reps (after one warm-up), output rows, path counters."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd._lib import C  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 100_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
types = (sys.argv[3] if len(sys.argv) > 3 else "inner,left,right,outer,inner2").split(",")
ctx = CylonContext(device="cuda:0")
g = torch.Generator(device="cuda").manual_seed(0)
hi = max(1, int(0.99 * n))


def side(p, two):
    cols = {f"{p}k": torch.randint(0, hi, (n,), generator=g, device="cuda")}
    if two:  # second key: a small-range column, so (k, k2) still matches ~ as often as k alone / 4
        cols[f"{p}k2"] = torch.randint(0, 4, (n,), generator=g, device="cuda")
    for i in range(3):
        cols[f"{p}{i}"] = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
    return Table.from_torch(ctx, cols)


tables = {}
for t in types:
    two = t.endswith("2")
    if two not in tables:
        tables.clear()  # one table pair resident at a time (1B x 1B: 64-80 GB per pair)
        torch.cuda.empty_cache()
        tables[two] = (side("a", two), side("b", two))
    torch.cuda.empty_cache()  # each type starts from the same allocator state
    L, R = tables[two]
    how = {"inner": "inner", "left": "left", "right": "right", "outer": "outer"}[t.rstrip("2")]
    on = [0, 1] if two else [0]

    def run():
        return L.join(R, how, "hash", on=on)

    out = run()
    rows = out.row_count
    del out
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = run()
        torch.cuda.synchronize()
        ts.append(1000 * (time.perf_counter() - t0))
        del out
    torch.cuda.reset_peak_memory_stats()
    C.trace_enable(True)
    C.trace_reset()
    out = run()
    torch.cuda.synchronize()
    cnt = {k: v for k, v in dict(C.trace_counters()).items() if k.startswith("join.")}
    C.trace_enable(False)
    del out
    print(json.dumps({"type": t, "rows_per_side": n, "ms": round(statistics.median(ts), 3),
                      "all_ms": [round(x, 2) for x in ts], "out_rows": rows,
                      "peak_gb": round(torch.cuda.max_memory_allocated() / 2**30, 1), "counters": cnt}), flush=True)
