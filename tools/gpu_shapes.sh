#!/bin/bash
# Pair-pass timings (C2 1M) for each block shape given (SPH_BLK); default 0 1 2 3
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
for b in ${@:-0 1 2 3}; do
  echo -n "shape $b: "; SPH_BLK=$b timeout -k 10 150 python3 tools/kernel_sweep.py 100 20 || exit 1
done
