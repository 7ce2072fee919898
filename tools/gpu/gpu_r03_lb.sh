#!/bin/bash
# Chained-scan (decoupled lookback) radix passes: GPU correctness with lookback on (default), then
# interleaved A/B against the per-pass histogram kernels (CYLON_RP_LOOKBACK=0) on the headline join
# and the pass-heavy secondary configs, and kernel traces of both.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03lb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py tests/test_properties.py -x -q --timeout 300 --timeout-method thread -m gpu > $O/pytest_lb.txt 2>&1
for i in 1 2; do
  CYLON_RP_LOOKBACK=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/hist_$i.json 2> $O/hist_$i.err
  CYLON_RP_LOOKBACK=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/lb_$i.json 2> $O/lb_$i.err
done
CYLON_RP_LOOKBACK=0 timeout -k 10 400 python tools/bench_suite.py --configs 4,5,6 --reps 3 > $O/suite_hist.jsonl 2> $O/suite_hist.err
CYLON_RP_LOOKBACK=1 timeout -k 10 400 python tools/bench_suite.py --configs 4,5,6 --reps 3 > $O/suite_lb.jsonl 2> $O/suite_lb.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_lb -o lb -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof_lb.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sort -o sort -- python3 tools/bench_suite.py --configs 5 --reps 1 > $O/prof_sort.log 2>&1
echo done
