"""Driver for kernel profiles of the hash group-by path (BASELINE config 4 shape)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cylon_amd import CylonContext, Table  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1_000_000_000
groups = int(sys.argv[2]) if len(sys.argv) > 2 else 10_000_000
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
ctx = CylonContext(device="cuda:0")
g = torch.Generator(device="cuda").manual_seed(4)
t = Table.from_torch(ctx, {"g": torch.randint(0, groups, (n,), generator=g, device="cuda"),
                           "x": torch.rand(n, generator=g, device="cuda", dtype=torch.float64)})
for _ in range(reps):
    out = t.local_groupby("g", {"x": "sum"})
    torch.cuda.synchronize()
    print("groups", out.row_count, flush=True)
