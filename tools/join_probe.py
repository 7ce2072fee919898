"""Small driver for counter profiles of the join path: N x N int64 keys + 3 float64 payload."""
import sys

import os
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from cylon_amd import CylonContext, Table

n = int(sys.argv[1]) if len(sys.argv) > 1 else 200_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ctx = CylonContext(device="cuda:0")
g = torch.Generator(device="cuda").manual_seed(0)
hi = int(0.99 * n)
cols = lambda p: {f"{p}k": torch.randint(0, hi, (n,), generator=g, device="cuda"),
                  **{f"{p}{i}": torch.rand(n, generator=g, device="cuda", dtype=torch.float64) for i in range(3)}}
L, R = Table.from_torch(ctx, cols("a")), Table.from_torch(ctx, cols("b"))
for _ in range(reps):
    out = L.join(R, "inner", "hash", on=[0])
    torch.cuda.synchronize()
    print("rows", out.row_count, flush=True)
    del out
