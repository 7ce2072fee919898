"""Cost of nullability in the LDS row-moving passes: int64 key + 3 float64 payload (200M rows by
default), once with non-nullable payload and once with every payload column nullable (validity
bytes travel packed 8 per 8-byte word through the passes).  --op join (200M x 200M radix join,
default), sort (radix table sort by the key) or shuffle (one-pass mod partition into 8 parts)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cylon_amd import CylonContext, Table  # noqa: E402
from cylon_amd._lib import C  # noqa: E402
from cylon_amd.data import arrow_bridge as ab  # noqa: E402

args = [a for a in sys.argv[1:] if not a.startswith("--")]
n = int(args[0]) if args else 200_000_000
MODES = (True,) if "--only-nullable" in sys.argv else (False, True)
OP = next((a.split("=", 1)[1] for a in sys.argv if a.startswith("--op=")), "join")
ctx = CylonContext(device="cuda:0")
hi = int(0.99 * n)


def rel(seed, nullable):
    g = torch.Generator(device="cuda").manual_seed(seed)
    cols = [ab.column_from_tensor("k", torch.randint(0, hi, (n,), generator=g, device="cuda"))]
    for i in range(3):
        v = torch.rand(n, generator=g, device="cuda", dtype=torch.float64)
        valid = (torch.rand(n, generator=g, device="cuda") > 0.1).to(torch.uint8) if nullable else None
        cols.append(ab.column_from_tensor(f"v{i}", v, valid))
    return Table(context=ctx, _native=C.Table(ctx._ctx, cols))


def run(L, R):
    if OP == "sort":
        return L.sort("k")
    if OP == "shuffle":
        return C.shuffle_partition(L.native, [0], 8)
    return L.join(R, "inner", "hash", on=[0])


for nullable in MODES:
    L = rel(1, nullable)
    R = rel(2, nullable) if OP == "join" else None
    run(L, R)
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        out = run(L, R)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        del out
    print(f"{OP} nullable={nullable}: median {sorted(ts)[2]:.2f} ms  all {[round(x, 2) for x in ts]}", flush=True)
    del L, R
    torch.cuda.empty_cache()
