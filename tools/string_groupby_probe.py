"""String-key group-by on the LDS radix path (invertible word key, ops/groupby.cpp radix_groupby) vs
the int64-key group-by of the same shape: N rows, G groups, 16-byte string keys ("k" + 15 decimal
digits of the int key) + one float64 value, SUM + MAX, all generated in HBM.

usage: python tools/string_groupby_probe.py <rows> [groups] [reps]
Prints one JSON line per key type (median ms, groups, groupby.* counters) and the ratio; the string
run's per-group sums must equal the int64 run's (groups matched through the key digits)."""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))

from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd._lib import C  # noqa: E402
from string_join_probe import string_column, var_string_column, var_string_ints  # noqa: E402


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--var")]
    var = next((a for a in sys.argv[1:] if a.startswith("--var")), None)  # --var=8,32
    vlo, vhi = (int(x) for x in var.split("=")[1].split(",")) if var else (0, 0)
    n = int(args[0]) if len(args) > 0 else 200_000_000
    groups = int(args[1]) if len(args) > 1 else 10_000_000
    reps = int(args[2]) if len(args) > 2 else 3
    ctx = CylonContext(device="cuda:0")
    res, sums = {}, {}
    for kind in ("int64", "string"):
        torch.cuda.empty_cache()
        g = torch.Generator(device="cuda").manual_seed(0)
        k = torch.randint(0, groups, (n,), generator=g, device="cuda")
        v = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
        t = Table.from_torch(ctx, {"k": k, "v": v})
        if kind == "string":
            kc = var_string_column("k", k, vlo, vhi) if var else string_column("k", k)
            t = Table(context=ctx, _native=C.Table(ctx._ctx, [kc] + [t.native.columns()[1]]))

        def run():
            return t.local_groupby(["k"], {"v": ["sum", "max"]})

        out = run()
        ng = out.row_count
        del out
        ts = []
        for _ in range(reps):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            out = run()
            torch.cuda.synchronize()
            ts.append(1000 * (time.perf_counter() - t0))
            del out
        C.trace_enable(True)
        C.trace_reset()
        out = run()
        torch.cuda.synchronize()
        cnt = {a: b for a, b in dict(C.trace_counters()).items() if a.startswith("groupby.")}
        C.trace_enable(False)
        cols = out.native.columns()
        if kind == "string" and var:
            key = var_string_ints(cols[0])
        elif kind == "string":  # key bytes -> the int key (15 digits after 'k')
            b = cols[0].data.reshape(-1, 16)[:, 1:].to(torch.int64) - 48
            key = torch.zeros(b.shape[0], dtype=torch.int64, device=b.device)
            for d in range(15):
                key = key * 10 + b[:, d]
        else:
            key = cols[0].data
        order = torch.argsort(key)
        sums[kind] = (key[order], cols[1].data[order])
        rec = {"key": kind + (f" var[{vlo},{vhi}]" if var and kind == "string" else ""), "rows": n, "ms": round(statistics.median(ts), 3), "all_ms": [round(x, 2) for x in ts],
               "groups": ng, "counters": cnt}
        if kind == "string":
            rec["keys_equal_int64_run"] = bool(torch.equal(sums["int64"][0], sums["string"][0]))
            rec["sums_max_abs_diff"] = float((sums["int64"][1] - sums["string"][1]).abs().max())
        del out, t, k, v
        res[kind] = rec
        print(json.dumps(rec), flush=True)
    print(json.dumps({"string_over_int64": round(res["string"]["ms"] / res["int64"]["ms"], 3)}), flush=True)


if __name__ == "__main__":
    main()
