"""Driver for kernel profiles of the sort-algorithm join (1B x 1B by default)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cylon_amd import CylonContext, Table  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
ctx = CylonContext(device="cuda:0")
g = torch.Generator(device="cuda").manual_seed(0)
hi = int(0.99 * n)
cols = lambda p: {f"{p}k": torch.randint(0, hi, (n,), generator=g, device="cuda"),
                  **{f"{p}{i}": torch.rand(n, generator=g, device="cuda", dtype=torch.float64) for i in range(3)}}
L, R = Table.from_torch(ctx, cols("a")), Table.from_torch(ctx, cols("b"))
for _ in range(2):
    out = L.join(R, "inner", "sort", on=[0])
    torch.cuda.synchronize()
    print("rows", out.row_count, flush=True)
    del out
