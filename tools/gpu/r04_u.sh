#!/bin/bash
# Round-4 call U: nullable integer keys on the radix group-by (null rows as one group under a free
# key value): group-by GPU tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04u
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_gb 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_radix_joins.py -x -q --timeout 200 --timeout-method thread -k "groupby or nunique"
echo done
