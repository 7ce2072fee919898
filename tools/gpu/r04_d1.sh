#!/bin/bash
# Round-4 call D1: new GPU tests (radix outer / multi-key / var-width joins, extended radix group-by,
# string casts), the full GPU suite, headline bench, forced-shuffle benches (own rows local; K=4;
# own rows through RCCL).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r04e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_radix_joins.py -x -v --timeout 300 --timeout-method thread > $O/pytest_new.txt 2>&1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.txt 2>&1
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $O/bench_1.json 2> $O/bench_1.err
timeout -k 10 300 python bench.py --force-shuffle --steps 10 --warmup 3 > $O/bench_forced_k1.json 2> $O/bench_forced_k1.err
CYLON_SHUFFLE_CHUNKS=4 timeout -k 10 300 python bench.py --force-shuffle --steps 10 --warmup 3 --verify > $O/bench_forced_k4.json 2> $O/bench_forced_k4.err
CYLON_SHUFFLE_CHUNKS=4 CYLON_SHUFFLE_SELF_RCCL=1 timeout -k 10 300 python bench.py --force-shuffle --rows 500000000 --steps 10 --warmup 3 > $O/bench_forced_k4_selfrccl_500m.json 2> $O/bench_forced_k4_selfrccl.err
echo done
