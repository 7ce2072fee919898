#!/bin/bash
# Round-4 call AA: look-back passes for the stable hash partitions (group-by / set ops) behind
# CYLON_PARTITION_LOOKBACK=1: counter check, GPU tests with it on, config 4 / 6 A/B interleaved.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04aa
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
CYLON_PARTITION_LOOKBACK=1 step counter 120 python -c "
import torch
from cylon_amd import CylonContext, Table
from cylon_amd._lib import C
ctx = CylonContext(device='cuda:0')
g = torch.Generator(device='cuda').manual_seed(1)
n = 20_000_000
t = Table.from_torch(ctx, {'g': torch.randint(0, 2_000_000, (n,), generator=g, device='cuda'), 'x': torch.rand(n, generator=g, device='cuda', dtype=torch.float64)})
C.trace_enable(True); C.trace_reset()
r = t.local_groupby('g', {'x': 'sum'})
print(r.row_count, {k: v for k, v in dict(C.trace_counters()).items() if 'lookback' in k or 'groupby.radix' in k})
"
CYLON_PARTITION_LOOKBACK=1 step pytest_plb 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_radix_joins.py tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -k "groupby or nunique or setop or unique or union or distinct or intersect or subtract"
grep -q "pytest_plb rc=0" $O/steps.txt || exit 1
for r in a b; do
  step suite46_off_$r 300 python tools/bench_suite.py --configs 4,6 --reps 3
  CYLON_PARTITION_LOOKBACK=1 step suite46_on_$r 300 python tools/bench_suite.py --configs 4,6 --reps 3
done
echo done
