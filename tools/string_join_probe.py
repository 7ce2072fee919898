"""String-key join on the LDS radix path vs the int64-key join of the same shape (VERDICT r04 "do
this" 5): N x N rows, 16-byte string keys ("k" + 15 decimal digits of an int key uniform in
[0, 0.99 N)) + 3 float64 payload columns, all generated in HBM.

usage: python tools/string_join_probe.py <rows per side> [reps]
Prints one JSON line per key type: median ms, output rows, join.* counters, and (string run) the
output's key-equality / row-count check against the int64 run."""
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
from cylon_amd.types import DataType, Type  # noqa: E402


def string_column(name, ints):
    """16-byte ASCII keys 'k' + 15 zero-padded digits of ints (device)."""
    n = ints.numel()
    digits = torch.empty((n, 15), dtype=torch.uint8, device=ints.device)
    x = ints.clone()
    for d in range(14, -1, -1):
        digits[:, d] = (x % 10 + 48).to(torch.uint8)
        x //= 10
    b = torch.cat([torch.full((n, 1), ord("k"), dtype=torch.uint8, device=ints.device), digits], 1).reshape(-1)
    offs = torch.arange(0, 16 * n + 1, 16, dtype=torch.int64, device=ints.device)
    return C.Column(name, DataType(Type.STRING), n, b, offs)


def var_string_column(name, ints, lo=8, hi=32):
    """Variable-length ASCII keys of lo..hi bytes (device): 'k' + 5 base-64 digits of ints (< 2^30)
    + filler bytes, the length a function of the int (so equal ints <=> equal keys)."""
    n = ints.numel()
    ln = lo + (ints * 2654435761) % (hi - lo + 1)
    buf = torch.empty((n, hi), dtype=torch.uint8, device=ints.device)
    buf[:, 0] = ord("k")
    x = ints.clone()
    for d in range(5):
        buf[:, 1 + d] = (x % 64 + 48).to(torch.uint8)
        x //= 64
    for j in range(6, hi):
        buf[:, j] = ((buf[:, 1 + j % 5].to(torch.int64) + j) % 64 + 48).to(torch.uint8)
    pos = torch.arange(hi, device=ints.device)[None, :]
    step = 1 << 24  # (one boolean-mask select over all rows overflows inside torch)
    b = torch.cat([buf[i:i + step].masked_select(pos < ln[i:i + step, None]) for i in range(0, n, step)])
    del buf
    offs = torch.zeros(n + 1, dtype=torch.int64, device=ints.device)
    offs[1:] = torch.cumsum(ln, 0)
    return C.Column(name, DataType(Type.STRING), n, b, offs)


def var_string_ints(col):
    """The ints of var_string_column keys (digits 1..5 of each row)."""
    o = col.offsets[:-1]
    key = torch.zeros(o.numel(), dtype=torch.int64, device=o.device)
    for d in range(4, -1, -1):
        key = key * 64 + (col.data[o + 1 + d].to(torch.int64) - 48)
    return key


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--var")]
    var = next((a for a in sys.argv[1:] if a.startswith("--var")), None)  # --var=8,32
    vlo, vhi = (int(x) for x in var.split("=")[1].split(",")) if var else (0, 0)
    n = int(args[0]) if len(args) > 0 else 200_000_000
    reps = int(args[1]) if len(args) > 1 else 3
    ctx = CylonContext(device="cuda:0")
    kr = int(0.99 * n)
    res = {}
    for kind in ("int64", "string"):
        torch.cuda.empty_cache()
        g = torch.Generator(device="cuda").manual_seed(0)  # the same keys for both runs
        sides = []
        for _ in range(2):
            k = torch.randint(0, kr, (n,), generator=g, device="cuda")
            vals = {f"v{i}": torch.rand(n, generator=g, device="cuda", dtype=torch.float64) for i in range(3)}
            t = Table.from_torch(ctx, {"k": k, **vals})
            if kind == "string":
                kc = var_string_column("k", k, vlo, vhi) if var else string_column("k", k)
                cols = [kc] + [c for c in t.native.columns()[1:]]
                t = Table(context=ctx, _native=C.Table(ctx._ctx, cols))
            del k
            sides.append(t)
        L, R = sides

        def run():
            return L.join(R, "inner", "hash", on=["k"], left_prefix="l_", right_prefix="r_")

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
        C.trace_enable(True)
        C.trace_reset()
        out = run()
        torch.cuda.synchronize()
        cnt = {k: v for k, v in dict(C.trace_counters()).items() if k.startswith("join.")}
        phases = {k: round(v[0], 3) for k, v in dict(C.trace_phases()).items()}
        C.trace_enable(False)
        rec = {"key": kind + (f" var[{vlo},{vhi}]" if var and kind == "string" else ""), "rows_per_side": n, "ms": round(statistics.median(ts), 3),
               "all_ms": [round(x, 2) for x in ts], "out_rows": rows, "counters": cnt, "phases_ms": phases}
        if kind == "string":  # the key bytes of both sides are equal row by row (also checked by the join)
            lk, rk = out.native.columns()[0], out.native.columns()[4]
            rec["key_bytes_equal"] = bool(torch.equal(lk.data, rk.data) and torch.equal(lk.offsets, rk.offsets))
            rec["rows_equal_int64_run"] = rows == res["int64"]["out_rows"]
        del out, L, R, sides
        res[kind] = rec
        print(json.dumps(rec), flush=True)
    print(json.dumps({"string_over_int64": round(res["string"]["ms"] / res["int64"]["ms"], 3)}), flush=True)


if __name__ == "__main__":
    main()
