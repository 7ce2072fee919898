#!/bin/bash
# Round-4 call Y: PMC set of the final 2B-row sort passes (one rocprofv3 --pmc pass per counter group).
set -uo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04y
mkdir -p $O
export TMPDIR=/tmp
. tools/gpu/lib.sh
step pmc_sort 1000 bash tools/gpu/r04_pmc_sort.sh final
echo done
