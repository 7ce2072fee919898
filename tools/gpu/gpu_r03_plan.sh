#!/bin/bash
# Planned pair shuffle (one collective) on the device paths + ranking guard A/B.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_gpu_multirank.py tests/test_gpu_rccl_forced.py tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "multirank or forced or distributed or async or guard or verify or radix_sort or radix_row_sort or chunked" > $O/pytest.txt 2>&1
for i in 1 2; do
  CYLON_RP_GUARD=0 timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 3 > $O/sort_noguard_$i.jsonl 2> $O/sort_noguard_$i.err
  timeout -k 10 300 python tools/bench_suite.py --configs 5 --reps 3 > $O/sort_guard_$i.jsonl 2> $O/sort_guard_$i.err
done
CYLON_RP_GUARD=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/join_noguard.json 2> $O/join_noguard.err
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/join_guard.json 2> $O/join_guard.err
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --force-shuffle > $O/forced.json 2> $O/forced.err
echo done
