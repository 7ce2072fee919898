#!/bin/bash
# Windowed lookback A/B (CYLON_RP_LOOKBACK=0 vs 1) + staged ingest test/bench.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03lb2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ops.py -x -q --timeout 200 --timeout-method thread -m gpu -k "staged_ingest or groupby or set_ops" > $O/pytest_ingest.txt 2>&1
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu -k "sort or join" > $O/pytest_lb.txt 2>&1
CYLON_RP_LOOKBACK=1 timeout -k 10 300 python tools/bench_suite.py --configs 5,4 --reps 3 > $O/suite_lb.jsonl 2> $O/suite_lb.err
CYLON_RP_LOOKBACK=0 timeout -k 10 300 python tools/bench_suite.py --configs 5,4 --reps 3 > $O/suite_hist.jsonl 2> $O/suite_hist.err
CYLON_RP_LOOKBACK=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/lb_1.json 2> $O/lb_1.err
CYLON_RP_LOOKBACK=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/hist_1.json 2> $O/hist_1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sort -o sort -- python3 tools/bench_suite.py --configs 5 --reps 1 > $O/prof_sort.log 2>&1
timeout -k 10 400 python -u tools/ingest_bench.py --rows 1000000000 --reps 2 > $O/ingest.jsonl 2> $O/ingest.err
echo done
