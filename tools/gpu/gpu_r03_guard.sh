#!/bin/bash
# Full GPU suite with the in-pass ranking guard, headline bench x2, secondary configs, kernel trace.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/bench_1.json 2> $O/bench_1.err
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/bench_2.json 2> $O/bench_2.err
timeout -k 10 400 python tools/bench_suite.py --configs 2,4,5,6,7 --reps 3 > $O/suite.jsonl 2> $O/suite.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof.log 2>&1
echo done
