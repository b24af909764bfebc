#!/bin/bash
# Pair-pass timings of the row-kernel variants on C2 1M (tools/kernel_sweep.py per config):
# first vs second generation, lane-pair gathers (SPH_LP), the study bounds (SPH_EXP=1
# gathers only, 2 = body only) and the tile shapes of SPH_ROW2_TILES.
# Usage: tools/sweep_row2.sh > gpurun_out/sweep_row2.log
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 1
export SPH_PATH=1
run() {
  local name=$1
  shift
  echo -n "$name "
  (export "$@"; timeout -k 10 150 python3 tools/kernel_sweep.py 100 20) || exit 1
}
run rowk1 SPH_ROWK=1
run row2 SPH_ROWK=2
run row2_lp SPH_ROWK=2 SPH_LP=1
run row2_exp1 SPH_ROWK=2 SPH_EXP=1
run row2_exp2 SPH_ROWK=2 SPH_EXP=2
run row2_lp_exp1 SPH_ROWK=2 SPH_LP=1 SPH_EXP=1
for t in 1 2 3 4; do
  run row2_t$t SPH_ROWK=2 SPH_ROW2TILE=$t
  run row2_lp_t$t SPH_ROWK=2 SPH_LP=1 SPH_ROW2TILE=$t
done
