#!/bin/bash
# engine + brick GPU tests, then the rebuild and pair-pass timings for one block shape
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bricks.py -x -q --timeout 240 --timeout-method thread > gpurun_out/tq.log 2>&1 || { grep -E "FAILED|Error|passed|failed" gpurun_out/tq.log | head; exit 1; }
tail -1 gpurun_out/tq.log
for e in ${BEXPS:-0}; do echo -n "bexp $e: "; SPH_BEXP=$e timeout -k 10 120 python3 tools/build_sweep.py 100 5 || exit 1; done
timeout -k 10 120 python3 tools/kernel_sweep.py 100 20
