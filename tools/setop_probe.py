"""Set-operation timing / kernel-profile driver: <op> of two N-row relations (int64 key + 3
float64), the reference's second headline workload (union).

usage: python tools/setop_probe.py [N] [op] [reps] [digit bits per stable partition pass]
Prints one JSON line: median ms over reps (after one warm-up), output rows."""
import json
import os
import statistics
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd._lib import C  # noqa: E402

n = int(float(sys.argv[1])) if len(sys.argv) > 1 else 1_000_000_000
op = sys.argv[2] if len(sys.argv) > 2 else "union"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
db = int(sys.argv[4]) if len(sys.argv) > 4 else 10
C.partition_digit_bits(db)
ctx = CylonContext(device="cuda:0")
g = torch.Generator(device="cuda").manual_seed(0)
hi = int(0.99 * n)
cols = lambda p: {f"{p}k": torch.randint(0, hi, (n,), generator=g, device="cuda"),
                  **{f"{p}{i}": torch.rand(n, generator=g, device="cuda", dtype=torch.float64) for i in range(3)}}
L, R = Table.from_torch(ctx, cols("a")), Table.from_torch(ctx, cols("a"))
ts, rows = [], 0
for i in range(reps + 1):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = getattr(L, op)(R)
    torch.cuda.synchronize()
    if i:
        ts.append(1000 * (time.perf_counter() - t0))
    rows = out.row_count
    del out
print(json.dumps({"op": op, "n": n, "digit_bits": db, "ms": round(statistics.median(ts), 3),
                  "all_ms": [round(x, 2) for x in ts], "rows": rows}), flush=True)
