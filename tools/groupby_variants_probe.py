"""Time the LDS radix group-by on the BASELINE config-4 shape (1B rows, 10M int64 groups, float64
values) with richer aggregations and keys:
  sum        {"x": "sum"}                         (the config-4 baseline)
  sum_mean_std {"x": ["sum", "mean", "std"]}      (M2 accumulator: a second in-block pass)
  two_keys   keys (g // 4, g % 4): the same 10M groups as two key columns (exact composite), {"x": "sum"}
  two_keys_4x keys (g, h) with h in [0, 4): 4x the groups (40M), {"x": "sum"}
  float_key  key = g as float64                   (canonical bits), {"x": "sum"}

usage: python tools/groupby_variants_probe.py [rows] [groups] [reps] [variants, comma separated]
One JSON line per variant: median ms over reps after one warm-up, groups out, path counters."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd._lib import C  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
groups = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
variants = (sys.argv[4] if len(sys.argv) > 4 else "sum,sum_mean_std,two_keys,two_keys_4x,float_key").split(",")
ctx = CylonContext(device="cuda:0")
g = torch.Generator(device="cuda").manual_seed(4)
cols = {"g": torch.randint(0, groups, (n,), generator=g, device="cuda"),
        "x": torch.rand(n, generator=g, device="cuda", dtype=torch.float64)}
if "two_keys" in variants:
    cols["g1"] = cols["g"] // 4
    cols["g2"] = cols["g"] % 4
if "two_keys_4x" in variants:
    cols["h"] = torch.randint(0, 4, (n,), generator=g, device="cuda")
if "float_key" in variants:
    cols["f"] = cols["g"].to(torch.float64)
t = Table.from_torch(ctx, cols)
spec = {"sum": (["g"], {"x": "sum"}), "sum_mean_std": (["g"], {"x": ["sum", "mean", "std"]}),
        "two_keys": (["g1", "g2"], {"x": "sum"}), "two_keys_4x": (["g", "h"], {"x": "sum"}),
        "float_key": (["f"], {"x": "sum"})}
for v in variants:
    keys, aggs = spec[v]
    torch.cuda.empty_cache()
    out = t.local_groupby(keys, aggs)
    ngroups = out.row_count
    del out
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = t.local_groupby(keys, aggs)
        torch.cuda.synchronize()
        ts.append(1000 * (time.perf_counter() - t0))
        del out
    C.trace_enable(True)
    C.trace_reset()
    out = t.local_groupby(keys, aggs)
    torch.cuda.synchronize()
    cnt = {k: v for k, v in dict(C.trace_counters()).items() if k.startswith("groupby.")}
    C.trace_enable(False)
    del out
    print(json.dumps({"variant": v, "rows": n, "groups": groups, "ms": round(statistics.median(ts), 3),
                      "all_ms": [round(x, 2) for x in ts], "groups_out": ngroups, "counters": cnt}), flush=True)
