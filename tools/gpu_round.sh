#!/bin/bash
# tests + block-shape sweep (pair passes, rocprof) + rebuild study variants
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
TAG=$1; SHAPES=${2:-"2"}
tools/gpu_blk.sh "$TAG" "$SHAPES" test || exit 1
for e in 0 1 2 4 8 15; do
  echo -n "bexp $e: "; SPH_BLK=$(echo $SHAPES | cut -d' ' -f1) SPH_BEXP=$e timeout -k 10 120 python3 tools/build_sweep.py 100 5 || exit 1
done
echo -n "row path: "; SPH_PATH=1 timeout -k 10 120 python3 tools/build_sweep.py 100 5
