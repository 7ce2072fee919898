"""Driver for kernel profiles of the table sort path (BASELINE config 5 shape)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from cylon_amd import CylonContext, Table  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ctx = CylonContext(device="cuda:0")
g = torch.Generator(device="cuda").manual_seed(5)
t = Table.from_torch(ctx, {"k": torch.randint(-(1 << 62), 1 << 62, (n,), generator=g, device="cuda")})
for _ in range(reps):
    out = t.sort("k")
    torch.cuda.synchronize()
    print("rows", out.row_count, flush=True)
    del out
