#!/bin/bash
# Round-4 call M: slot kernel v4 (packed destinations, next-digit code only in sort instances, slot
# tiles claimed two ahead) -- targeted tests, same-box A/B, group-by variants (verdict item 6), sort.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04m
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_targeted 400 python -u -m pytest tests/test_gpu_radix_joins.py tests/test_gpu_kernels.py -x -q --timeout 200 --timeout-method thread -k "slot or ranking_guard or outer or composite or sort or nunique or groupby"
step bench_1 200 python bench.py --steps 20 --warmup 5
CYLON_RJ_SLOT=0 step bench_1_noslot 200 python bench.py --steps 20 --warmup 5
step bench_1b 200 python bench.py --steps 20 --warmup 5
step bench_1_verify 200 python bench.py --steps 3 --warmup 1 --verify
step gb_variants 400 python tools/groupby_variants_probe.py 1000000000 10000000 3
step suite5 400 python tools/bench_suite.py --configs 5 --reps 3
step prof_head 300 rocprofv3 --kernel-trace --stats -d $O/prof_head -o head -- python3 bench.py --steps 2 --warmup 1 --no-phases
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
echo done
