#!/bin/bash
# One GPU iteration of the kernel work: engine + brick parity tests, then pair-pass
# timings for the configurations given as arguments (each "VAR=VAL VAR=VAL" string).
# Usage (on the GPU box): tools/gpu_iter.sh TAG "SPH_PATH=1" "SPH_PATH=1 SPH_LP=0" ...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
TAG=$1
shift
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bricks.py -x -q \
  --timeout 120 --timeout-method thread > "gpurun_out/t_$TAG.log" 2>&1 || exit 1
for cfg in "$@"; do
  echo -n "$cfg "
  (for kv in $cfg; do export "$kv"; done; timeout -k 10 150 python3 tools/kernel_sweep.py 100 20) || exit 1
done > "gpurun_out/sweep_$TAG.log" 2>&1
