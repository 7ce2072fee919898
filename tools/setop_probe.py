"""Driver for kernel profiles of the set-operation path: union of two N-row relations
(int64 key + 3 float64), the reference's second headline workload."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cylon_amd import CylonContext, Table  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
op = sys.argv[2] if len(sys.argv) > 2 else "union"
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
ctx = CylonContext(device="cuda:0")
g = torch.Generator(device="cuda").manual_seed(0)
hi = int(0.99 * n)
cols = lambda p: {f"{p}k": torch.randint(0, hi, (n,), generator=g, device="cuda"),
                  **{f"{p}{i}": torch.rand(n, generator=g, device="cuda", dtype=torch.float64) for i in range(3)}}
L, R = Table.from_torch(ctx, cols("a")), Table.from_torch(ctx, cols("a"))
for _ in range(reps):
    out = getattr(L, op)(R)
    torch.cuda.synchronize()
    print(op, "rows", out.row_count, flush=True)
    del out
