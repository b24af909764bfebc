#!/bin/bash
# Cluster-path iteration: pair-pass timings for the given configs, then the engine and
# brick parity tests (all cases, no -x).  Usage: tools/gpu_cl.sh TAG "SPH_PATH=3" ...
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
TAG=$1
shift
mkdir -p gpurun_out
for cfg in "$@"; do
  echo -n "$cfg "
  (for kv in $cfg; do export "$kv"; done; timeout -k 10 150 python3 tools/kernel_sweep.py 100 20) || exit 1
done > "gpurun_out/sweep_$TAG.log" 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bricks.py -q \
  --timeout 120 --timeout-method thread > "gpurun_out/t_$TAG.log" 2>&1
