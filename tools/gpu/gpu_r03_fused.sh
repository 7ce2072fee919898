#!/bin/bash
# Fused count+write radix join + high-priority RCCL stream: join GPU tests, headline bench
# (with --verify), forced-shuffle bench + its RCCL/compute overlap, headline kernel trace.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rccl_forced.py tests/test_gpu_multirank.py -x -v --timeout 300 --timeout-method thread > $O/pytest.txt 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/bench_1.json 2> $O/bench_1.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verify > $O/bench_verify.json 2> $O/bench_verify.err
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/bench_2.json 2> $O/bench_2.err
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --force-shuffle > $O/forced.json 2> $O/forced.err
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/prof_forced -o forced -- python3 bench.py --steps 1 --warmup 1 --force-shuffle --no-phases > $O/prof_forced.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_join -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof_join.log 2>&1
echo done
