#!/bin/bash
# XCD-tile schedule default on (classic + lean passes): GPU suite, headline and secondary configs
# A/B against CYLON_RP_XT=0, kernel traces of the sort and the join.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03xt2
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
for i in 1 2; do
  CYLON_RP_XT=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/base_$i.json 2> $O/base_$i.err
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/xt_$i.json 2> $O/xt_$i.err
done
CYLON_RP_XT=0 timeout -k 10 500 python tools/bench_suite.py --configs 2,4,5,6,7 --reps 3 > $O/suite_base.jsonl 2> $O/suite_base.err
timeout -k 10 500 python tools/bench_suite.py --configs 2,4,5,6,7 --reps 3 > $O/suite_xt.jsonl 2> $O/suite_xt.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_join -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof_join.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_sort -o sort -- python3 tools/bench_suite.py --configs 5 --reps 1 > $O/prof_sort.log 2>&1
echo done
