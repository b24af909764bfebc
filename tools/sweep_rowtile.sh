#!/bin/bash
# Time the engine's row kernels for every instantiated tile shape (SPH_ROWTILE) and the
# generic pair-layer kernels (SPH_ROWK=0) on the C2 1M workload; one process per shape.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/rowtile.log}
: > "$OUT"
SPH_PATH=1 SPH_ROWK=0 timeout -k 10 120 python3 "$R/tools/kernel_sweep.py" 100 20 | sed 's/^/rowk0 /' >> "$OUT"
for t in 0 1 2 3 4 5; do
  SPH_PATH=1 SPH_ROWTILE=$t timeout -k 10 120 python3 "$R/tools/kernel_sweep.py" 100 20 | sed "s/^/tile$t /" >> "$OUT"
done
