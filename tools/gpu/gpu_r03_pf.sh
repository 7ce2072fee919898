#!/bin/bash
# Write kernel: next emit round prefetched into registers, count loop two rounds in flight.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03pf
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 300 --timeout-method thread -k "join or narrow or guard" > $O/pytest.txt 2>&1
for i in 1 2 3; do
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/b_$i.json 2> $O/b_$i.err
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verify > $O/verify.json 2> $O/verify.err
CYLON_RJ_STAMPS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/stamps.json 2> $O/stamps.err
echo done
