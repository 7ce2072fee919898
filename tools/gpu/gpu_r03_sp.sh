#!/bin/bash
# Sort prologue fusion (varying bits + first-pass tile histogram in one read): sort GPU tests, config 5 A/B.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03sp
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "sort" > $O/pytest.txt 2>&1
for i in 1 2; do
  CYLON_SORT_PREHIST=0 timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 3 > $O/off_$i.jsonl 2> $O/off_$i.err
  timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 3 > $O/on_$i.jsonl 2> $O/on_$i.err
done
echo done
