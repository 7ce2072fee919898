#!/bin/bash
# Round-4 call O: slot first pass with XCD-major cursors (slot x * nb + d; the bucket-major order put
# 8 XCDs' claim atomics on each cursor line): targeted tests, interleaved same-box A/B, kernel trace,
# group-by variants with the fused key pass.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04o
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
step gb_variants 600 python -u tools/groupby_variants_probe.py 1000000000 10000000 3
echo done
