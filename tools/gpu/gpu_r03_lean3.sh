#!/bin/bash
# With the XCD-tile schedule: lean (default for 1-2 column passes) vs classic for sort / group-by / union.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03lean3
mkdir -p $O
timeout -k 10 500 python tools/bench_suite.py --configs 4,5,6 --reps 3 > $O/lean.jsonl 2> $O/lean.err
CYLON_RP_KERNEL=classic timeout -k 10 500 python tools/bench_suite.py --configs 4,5,6 --reps 3 > $O/classic.jsonl 2> $O/classic.err
echo done
