#!/bin/bash
# Kernel trace of the 2B-row sort (config 5) and the 1B group-by (config 4) on the final tree.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03sortprof
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/sort -o sort -- python3 tools/bench_suite.py --configs 5 --reps 1 > $O/sort.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/gb -o gb -- python3 tools/bench_suite.py --configs 4 --reps 1 > $O/gb.log 2>&1
echo done
