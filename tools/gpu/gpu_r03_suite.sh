#!/bin/bash
# Full GPU suite + smoke + headline bench on the current tree.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err
echo done
