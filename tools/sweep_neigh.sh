#!/bin/bash
# Neighbor-build and pair-kernel timings: new half-bin builder vs the original.
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=${1:-$R/gpurun_out/neigh.log}
: > "$OUT"
for nb in 3 2 1; do
  SPH_NEIGH=$nb timeout -k 10 200 python3 "$R/bench.py" --steps 50 --warmup 10 --no-cpu | sed "s/^/neigh$nb /" >> "$OUT"
done
