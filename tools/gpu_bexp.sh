#!/bin/bash
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
for e in 0 1 2 4 8 15; do
  SPH_BLK=${1:-2} SPH_BEXP=$e timeout -k 10 120 python3 tools/build_sweep.py 100 5 || exit 1
done
SPH_PATH=1 timeout -k 10 120 python3 tools/build_sweep.py 100 5
