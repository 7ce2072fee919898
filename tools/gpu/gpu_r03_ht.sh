#!/bin/bash
# Software-pipelined per-tile histogram kernel: radix GPU tests, headline x2 (+verify), sort/union/group-by suite,
# kernel trace of the join.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03ht
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_ops.py -x -q --timeout 300 --timeout-method thread -k "join or sort or groupby or set or xcd" > $O/pytest.txt 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_1.json 2> $O/bench_1.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verify > $O/bench_verify.json 2> $O/bench_verify.err
timeout -k 10 500 python tools/bench_suite.py --configs 4,5,6 --reps 3 > $O/suite.jsonl 2> $O/suite.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof.log 2>&1
echo done
