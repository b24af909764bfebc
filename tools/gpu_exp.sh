#!/bin/bash
# Study variants of the block force pass (SPH_EXP) for one shape, then PMC of the real one.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
R=$(pwd); TAG=$1; B=${2:-2}
mkdir -p gpurun_out
for e in 0 1 2 3; do
  echo -n "exp $e: "; SPH_BLK=$B SPH_EXP=$e timeout -k 10 150 python3 tools/kernel_sweep.py 100 20 | cut -c1-220 || exit 1
done | tee gpurun_out/exp_$TAG.log
tools/gpu_pmc.sh "$TAG" SPH_BLK=$B | grep -E "k_blk" 
