"""Cost of nullability in the radix join: 200M x 200M, int64 key + 3 float64 payload, once with
non-nullable payload and once with every payload column nullable (validity bytes travel through
the LDS passes as one more 1-byte column each)."""
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


for nullable in MODES:
    L, R = rel(1, nullable), rel(2, nullable)
    L.join(R, "inner", "hash", on=[0])
    torch.cuda.synchronize()
    ts = []
    for _ in range(5):
        t0 = time.perf_counter()
        out = L.join(R, "inner", "hash", on=[0])
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e3)
        del out
    print(f"nullable={nullable}: median {sorted(ts)[2]:.2f} ms  all {[round(x, 2) for x in ts]}", flush=True)
    del L, R
    torch.cuda.empty_cache()
