"""Time and verify the 1B x 1B inner join on skewed keys (VERDICT r04 "do this" 2).

usage: python tools/skew_probe.py <rows per side> [reps] [shapes, comma separated]
shapes:
  uniform  the headline shape (keys uniform in [0, 0.99 n)), for the ratio
  hotbuild the build side (right) holds 16 hot keys x 200k duplicates (scaled by n / 1B), the rest
           uniform; the probe side is uniform
  zipf     probe-side (left) keys Zipf(1.1) over the key range (discrete Pareto ranks scattered over
           the keys by a multiplicative hash), build side uniform
Each shape: median ms over reps after one warm-up, output rows, join.* path counters, and the
bincount identities of bench.verify_join on the last output (one JSON line per shape)."""
import json
import os
import statistics
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import verify_join  # noqa: E402
from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd._lib import C  # noqa: E402


def zipf_keys(n, key_range, s, g):
    # P(rank >= k) = k^-(s-1): rank = floor(u^(-1/(s-1))); ranks past the key range wrap around
    u = torch.rand(n, generator=g, device="cuda", dtype=torch.float64).clamp_(min=1e-300)
    r = torch.floor(u.pow_(-1.0 / (s - 1.0))).clamp_(max=2.0**62).to(torch.int64)
    del u
    r.remainder_(key_range)
    # scatter the ranks over the key range (hot keys land in unrelated partitions)
    return (r * 0x9E3779B1).remainder_(key_range)


def side(ctx, keys, g, prefix):
    n = keys.numel()
    cols = {"k": keys}
    for i in range(3):
        cols[f"v{i}"] = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
    return Table.from_torch(ctx, cols)


def make(shape, n, key_range, g):
    lk = torch.randint(0, key_range, (n,), generator=g, device="cuda")
    rk = torch.randint(0, key_range, (n,), generator=g, device="cuda")
    if shape == "hotbuild":
        dup = max(1, 200_000 * n // 1_000_000_000)
        hot = torch.arange(16, device="cuda", dtype=torch.int64) * (key_range // 16) + 7
        pos = torch.randperm(n, generator=g, device="cuda")[:16 * dup]
        rk[pos] = hot.repeat_interleave(dup)
        del pos
    elif shape == "zipf":
        lk = zipf_keys(n, key_range, 1.1, g)
    return lk, rk


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    shapes = (sys.argv[3] if len(sys.argv) > 3 else "uniform,hotbuild,zipf").split(",")
    ctx = CylonContext(device="cuda:0")
    key_range = max(1, int(0.99 * n))
    for shape in shapes:
        torch.cuda.empty_cache()
        g = torch.Generator(device="cuda").manual_seed(0)
        lk, rk = make(shape, n, key_range, g)
        L, R = side(ctx, lk, g, "l"), side(ctx, rk, g, "r")
        del lk, rk

        def run():
            return L.join(R, "inner", "hash", on=[0], left_prefix="l_", right_prefix="r_")

        out = run()
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
        C.trace_enable(False)
        ver = verify_join(ctx, L, R, out, key_range)
        rows = out.row_count
        del out, L, R
        print(json.dumps({"shape": shape, "rows_per_side": n, "ms": round(statistics.median(ts), 3),
                          "all_ms": [round(x, 2) for x in ts], "out_rows": rows, "verify_ok": ver["ok"],
                          "verify": ver, "counters": cnt}), flush=True)


if __name__ == "__main__":
    main()
