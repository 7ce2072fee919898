"""QUANTILE on the LDS radix group-by: BASELINE config 4 shape (N rows, G int64
groups, one float64 value) timed for {sum} and for {sum, quantile(0.5)}; the radix result is
checked group by group against the global-table path on a 1/64 key subset (exact equality of the
type-2 quantile: same values, same rule).

usage: python tools/quantile_probe.py [rows] [groups] [reps]"""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd._lib import C  # noqa: E402


def timed(fn, reps):
    fn()
    ts = []
    for _ in range(reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = fn()
        torch.cuda.synchronize()
        ts.append(1000 * (time.perf_counter() - t0))
        del out
    return statistics.median(ts), ts


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    groups = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    ctx = CylonContext(device="cuda:0")
    g = torch.Generator(device="cuda").manual_seed(4)
    t = Table.from_torch(ctx, {"g": torch.randint(0, groups, (n,), generator=g, device="cuda"),
                               "x": torch.rand(n, generator=g, device="cuda", dtype=torch.float64)})
    res = {}
    for name, aggs in (("sum", {"x": ["sum"]}), ("sum_median", {"x": ["sum", "median"]})):
        ms, ts = timed(lambda: t.local_groupby("g", aggs), reps)
        C.trace_enable(True)
        C.trace_reset()
        out = t.local_groupby("g", aggs)
        torch.cuda.synchronize()
        cnt = {k: v for k, v in dict(C.trace_counters()).items() if k.startswith("groupby.")}
        C.trace_enable(False)
        res[name] = {"aggs": name, "rows": n, "groups": out.row_count, "ms": round(ms, 3),
                     "all_ms": [round(x, 2) for x in ts], "counters": cnt}
        if name == "sum_median":  # exactness on a key subset against the global path
            tt = out.to_torch()
            sel = tt["g"] % 64 == 0
            sub = Table.from_torch(ctx, {"g": t.to_torch()["g"], "x": t.to_torch()["x"]})
            keep = sub.to_torch()["g"] % 64 == 0
            small = Table.from_torch(ctx, {"g": sub.to_torch()["g"][keep], "x": sub.to_torch()["x"][keep]})
            os.environ["CYLON_RADIX_GROUPBY_MIN_ROWS"] = str(1 << 62)
            ref = small.local_groupby("g", {"x": ["sum", "median"]}).to_torch()
            del os.environ["CYLON_RADIX_GROUPBY_MIN_ROWS"]
            a_o, b_o = torch.argsort(tt["g"][sel]), torch.argsort(ref["g"])
            qa, qb = tt["quantile_x"][sel][a_o], ref["quantile_x"][b_o]
            res[name]["subset_groups"] = int(qb.numel())
            res[name]["subset_keys_equal"] = bool(torch.equal(tt["g"][sel][a_o], ref["g"][b_o]))
            res[name]["subset_quantile_exact"] = bool(torch.equal(qa, qb))
            res[name]["subset_sum_max_rel_err"] = float(((tt["sum_x"][sel][a_o] - ref["sum_x"][b_o]).abs() /
                                                         ref["sum_x"][b_o].abs().clamp_min(1e-300)).max())
        print(json.dumps(res[name]), flush=True)
        del out
    print(json.dumps({"sum_median_over_sum": round(res["sum_median"]["ms"] / res["sum"]["ms"], 3)}), flush=True)


if __name__ == "__main__":
    main()
