#!/bin/bash
# Join write kernel staging A/B: all build-column loads in flight vs column by column (+ phase stamps).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03rj
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -m gpu -k "join" > $O/pytest_join.txt 2>&1
for m in all column; do
  CYLON_RJ_STAGE=$m CYLON_RJ_STAMPS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/stamps_$m.json 2> $O/stamps_$m.err
done
for i in 1 2; do
  for m in all column; do
    CYLON_RJ_STAGE=$m timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench_${m}_$i.json 2> $O/bench_${m}_$i.err
  done
done
echo done
