#!/bin/bash
# Round-4 call AB: partition look-back passes on by default: the forcing test first, the whole GPU
# suite, then config 4 / 6 interleaved with CYLON_PARTITION_LOOKBACK=0.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04ab
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_plb 240 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 100 --timeout-method thread -k "partition_lookback"
grep -q "pytest_plb rc=0" $O/steps.txt || exit 1
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step suite46_on_a 300 python tools/bench_suite.py --configs 4,6 --reps 3
CYLON_PARTITION_LOOKBACK=0 step suite46_off_a 300 python tools/bench_suite.py --configs 4,6 --reps 3
step suite46_on_b 300 python tools/bench_suite.py --configs 4,6 --reps 3
echo done
