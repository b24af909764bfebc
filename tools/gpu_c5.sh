#!/bin/bash
# C5 engine tests, then a short C5 bench at a given edge (default 60) and the 4.02M one
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_c5_engine.py -x -q --timeout 240 --timeout-method thread -m gpu > gpurun_out/c5.log 2>&1 || { grep -E "Error|error|FAILED|passed|failed|assert" gpurun_out/c5.log | head -20; exit 1; }
tail -1 gpurun_out/c5.log
timeout -k 10 200 python3 bench.py --workload c5 --edge ${1:-60} --steps 5 --warmup 2 --no-cpu 2>gpurun_out/c5b.err | tee gpurun_out/c5_small.json || { tail -5 gpurun_out/c5b.err; exit 1; }
[ -n "$2" ] && timeout -k 10 400 python3 bench.py --workload c5 --edge $2 --steps ${3:-10} --warmup 2 2>>gpurun_out/c5b.err | tee gpurun_out/c5_big.json
exit 0
