#!/bin/bash
# GPU tests with a heartbeat (gpurun kills a call silent for 180 s): tools/gpu_tests.sh LOG [pytest args]
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
LOG=$1; shift
mkdir -p "$(dirname "$LOG")"
( while true; do sleep 30; date +%T >> "$LOG.hb"; done ) &
HB=$!
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 900 --timeout-method thread "$@" > "$LOG" 2>&1
RC=$?
kill $HB
grep -E "^(FAILED|E   +AssertionError)|passed|failed" "$LOG" | tail -60
exit $RC
