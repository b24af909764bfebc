#!/bin/bash
# One pytest target on the GPU (default: the C5 brick tests): tools/gpu_one.sh [pytest args]
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out
T=${*:-tests/test_c5_bricks.py}
timeout -k 10 600 python -u -m pytest $T -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/one.log 2>&1
rc=$?; grep -E "PASS|FAIL|passed|failed|^E  " gpurun_out/one.log | head -40; exit $rc
