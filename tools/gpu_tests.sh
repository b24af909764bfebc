#!/bin/bash
# The whole -m gpu suite, then the smoke test.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out
TAG=${1:-all}
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 240 --timeout-method thread > "gpurun_out/tests_$TAG.log" 2>&1
rc=$?
grep -E "passed|failed|error" "gpurun_out/tests_$TAG.log" | tail -5
[ $rc -eq 0 ] || { grep -E "FAILED|Error" "gpurun_out/tests_$TAG.log" | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2
