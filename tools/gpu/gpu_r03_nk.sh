#!/bin/bash
# Narrow-key radix join: join GPU tests, then interleaved headline A/B (CYLON_RJ_NARROW=0 vs default),
# a --verify run and a kernel trace of the default.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03nk
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_kernels.py -x -v --timeout 300 --timeout-method thread -k "join or narrow or guard" > $O/pytest.txt 2>&1
for i in 1 2; do
  CYLON_RJ_NARROW=0 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/wide_$i.json 2> $O/wide_$i.err
  timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/narrow_$i.json 2> $O/narrow_$i.err
done
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --verify > $O/narrow_verify.json 2> $O/narrow_verify.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof.log 2>&1
echo done
