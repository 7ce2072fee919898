#!/bin/bash
# Round-4 call N: slot kernel v5 (int64 destinations again, next-digit code only in sort instances,
# slot tiles claimed two ahead): targeted tests, interleaved same-box A/B, kernel trace, PMC set.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04n
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_targeted 400 python -u -m pytest tests/test_gpu_radix_joins.py -x -q --timeout 200 --timeout-method thread -k "slot or outer or composite or nunique"
step bench_s1 200 python bench.py --steps 20 --warmup 5
CYLON_RJ_SLOT=0 step bench_x1 200 python bench.py --steps 20 --warmup 5
step bench_s2 200 python bench.py --steps 20 --warmup 5
CYLON_RJ_SLOT=0 step bench_x2 200 python bench.py --steps 20 --warmup 5
step bench_verify 200 python bench.py --steps 3 --warmup 1 --verify
step prof_head 300 rocprofv3 --kernel-trace --stats -d $O/prof_head -o head -- python3 bench.py --steps 2 --warmup 1 --no-phases
CYLON_RJ_SLOT=0 step prof_noslot 300 rocprofv3 --kernel-trace --stats -d $O/prof_noslot -o noslot -- python3 bench.py --steps 2 --warmup 1 --no-phases
step pmc 900 bash tools/gpu/r04_pmc.sh final
echo done
