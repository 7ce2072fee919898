#!/bin/bash
# Round-4 call Z: look-back window A/B (CYLON_SORT_LB_WINDOW = 1 / 2 / 4 words per round trip),
# interleaved on one box, after the look-back tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04z
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_lb 240 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 100 --timeout-method thread -k "lookback"
grep -q "pytest_lb rc=0" $O/steps.txt || exit 1
for r in a b; do
  for w in 4 2 1; do
    CYLON_SORT_LB_WINDOW=$w step suite5_w${w}_$r 300 python tools/bench_suite.py --configs 5 --reps 3
  done
done
echo done
