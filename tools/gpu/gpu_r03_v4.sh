#!/bin/bash
# Round-3 validation of the final tree (XCD-tile passes, 512-thread per-tile histograms): full GPU suite,
# secondary configs, kernel trace, write-kernel phase stamps, and PMC passes of the join kernels
# with LDS-DMA build staging (default) and with register staging (CYLON_RJ_DMA=0).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03v4
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_1.json 2> $O/bench_1.err
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_2.json 2> $O/bench_2.err
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --verify > $O/bench_verify.json 2> $O/bench_verify.err
timeout -k 10 500 python tools/bench_suite.py --configs 2,4,5,6,7 --reps 3 > $O/suite.jsonl 2> $O/suite.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof.log 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_3.json 2> $O/bench_3.err
echo done
