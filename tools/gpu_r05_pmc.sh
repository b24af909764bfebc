#!/bin/bash
# Round-5 PMC traffic records (tools/pmc_traffic.sh) of the C2 and C5 bench runs.
# Usage: tools/gpu_r05_pmc.sh OUTDIR COMMIT
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
O=$1; C=$2
META="world=1 edge=100 path=0 steps=20 warmup=5 commit=$C" bash tools/pmc_traffic.sh "$O/pmc_c2" --steps 20 --warmup 5 --no-cpu && echo "pmc c2 done" &&
META="world=1 edge=159 path=0 steps=5 warmup=2 commit=$C" bash tools/pmc_traffic.sh "$O/pmc_c5" --workload c5 --steps 5 --warmup 2 --no-cpu && echo "pmc c5 done"
