#!/bin/bash
# Round-4 call W (after nullable multi-key group-by): nullable integer keys on the radix group-by and (as exact composites with a null
# code) on the radix join; the group-by / join GPU tests.
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04w
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pytest_gbj 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_radix_joins.py -x -q --timeout 200 --timeout-method thread -k "groupby or nunique or join"
echo done
