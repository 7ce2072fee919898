#!/bin/bash
# Round-4 final validation on the final tree: the whole GPU suite, smoke(), the driver's bench
# command twice and once with --verify, config 4/5 suite numbers.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/${R04_FINAL_DIR:-r04final}
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_1 200 python bench.py --steps 20 --warmup 5
step bench_2 200 python bench.py --steps 20 --warmup 5
step bench_verify 200 python bench.py --steps 3 --warmup 1 --verify
step suite45 300 python tools/bench_suite.py --configs 4,5 --reps 3
echo done
