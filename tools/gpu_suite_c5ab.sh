#!/bin/bash
# the whole -m gpu suite, then tools/gpu_c5ab.sh's bench lines (NOTEST)
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out/c5ab
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/c5ab/suite.log 2>&1 || { tail -30 gpurun_out/c5ab/suite.log; exit 1; }
tail -2 gpurun_out/c5ab/suite.log
NOTEST=1 bash tools/gpu_c5ab.sh "$@"
