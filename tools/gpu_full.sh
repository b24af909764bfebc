#!/bin/bash
# Round-end style GPU check: full GPU test suite, smoke(), one bench line.
# Usage (on the GPU box): tools/gpu_full.sh TAG [bench args]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
TAG=$1
shift
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  > "gpurun_out/tests_$TAG.log" 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "gpurun_out/smoke_$TAG.log" 2>&1 || exit 1
timeout -k 10 600 python bench.py "$@" > "gpurun_out/bench_$TAG.json" 2> "gpurun_out/bench_$TAG.err"
