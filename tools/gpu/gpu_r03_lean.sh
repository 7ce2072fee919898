#!/bin/bash
# Lean (2 blocks/CU) vs classic radix pass: correctness with the lean kernel forced, then
# interleaved A/B of the headline join and the pass-heavy secondary configs, kernel traces.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03c
mkdir -p $O
export CYLON_RP_KERNEL=lean
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_multirank.py tests/test_properties.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_lean.txt 2>&1
for i in 1 2; do
  CYLON_RP_KERNEL=classic timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/classic_$i.json 2> $O/classic_$i.err
  CYLON_RP_KERNEL=lean timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/lean_$i.json 2> $O/lean_$i.err
done
CYLON_RP_KERNEL=classic timeout -k 10 400 python tools/bench_suite.py --configs 4,5,6 --reps 3 > $O/suite_classic.jsonl 2> $O/suite_classic.err
CYLON_RP_KERNEL=lean timeout -k 10 400 python tools/bench_suite.py --configs 4,5,6 --reps 3 > $O/suite_lean.jsonl 2> $O/suite_lean.err
CYLON_RP_KERNEL=lean timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_lean -o lean -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof_lean.log 2>&1
echo done
