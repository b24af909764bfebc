#!/bin/bash
# A/B bench lines for engine env configurations (each "VAR=VAL ..." string); then the
# engine + brick parity tests.  Usage: tools/bench_ab.sh TAG "SPH_NEIGHCL=0" "SPH_NEIGHCL=8"
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
TAG=$1
shift
mkdir -p gpurun_out
for cfg in "$@"; do
  echo -n "$cfg "
  (for kv in $cfg; do export "$kv"; done; timeout -k 10 150 python3 bench.py --steps 60 --warmup 10 --no-cpu) || exit 1
done > "gpurun_out/ab_$TAG.log" 2> "gpurun_out/ab_$TAG.err" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bricks.py -q \
  --timeout 120 --timeout-method thread > "gpurun_out/t_$TAG.log" 2>&1
