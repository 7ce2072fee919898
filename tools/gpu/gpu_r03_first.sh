#!/bin/bash
# Round-3 first GPU call: forced RCCL exchange tests, interleaved A/B headline bench of the
# round-1 tree (ab_r1/, built from 0baca72) and HEAD, forced-shuffle bench and its kernel trace.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_rccl_forced.py -x -v --timeout 300 --timeout-method thread > $O/pytest_forced.txt 2>&1
for i in 1 2; do
  timeout -k 10 150 python bench.py --steps 10 --warmup 3 > $O/head_$i.json 2> $O/head_$i.err
  (cd ab_r1 && timeout -k 10 150 python bench.py --steps 10 --warmup 3) > $O/r1_$i.json 2> $O/r1_$i.err
done
timeout -k 10 200 python bench.py --steps 10 --warmup 3 --force-shuffle > $O/forced.json 2> $O/forced.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_forced -o forced -- python3 bench.py --steps 1 --warmup 1 --force-shuffle --no-phases > $O/prof_forced.log 2>&1

bash tools/gpu_pmc_r03.sh base
