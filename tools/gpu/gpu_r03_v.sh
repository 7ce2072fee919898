#!/bin/bash
# Round-3 validation: full GPU suite, smoke, headline bench x2, secondary configs, sort rank model,
# kernel trace of the headline, PMC "after" passes for k_rows_pass / k_rj_write.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r03v
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench_1.json 2> $O/bench_1.err
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench_2.json 2> $O/bench_2.err
timeout -k 10 500 python tools/bench_suite.py --configs 2,4,5,6,7 --reps 3 > $O/suite.jsonl 2> $O/suite.err
timeout -k 10 300 python tools/rank_sim.py --sort 2000000000 2 4 8 > $O/rank_sim_sort.txt 2> $O/rank_sim_sort.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o join -- python3 bench.py --steps 1 --warmup 1 --no-phases > $O/prof.log 2>&1
CYLON_RJ_STAMPS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/rj_stamps.json 2> $O/rj_stamps.err
CYLON_RJ_OWNERMAP=1 CYLON_RJ_STAMPS=1 timeout -k 10 200 python bench.py --steps 1 --warmup 1 --no-phases > $O/rj_stamps_om.json 2> $O/rj_stamps_om.err
CYLON_RJ_OWNERMAP=1 timeout -k 10 200 python bench.py --steps 20 --warmup 3 --verify > $O/bench_om.json 2> $O/bench_om.err
timeout -k 10 200 python bench.py --steps 20 --warmup 3 > $O/bench_3.json 2> $O/bench_3.err
echo done
