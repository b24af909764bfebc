#!/bin/bash
# C2 A/B at the driver's 20/5 and on the 125k RCCL-loopback brick: tools/gpu_ab2.sh SPEC ...
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
AB_ARGS="--steps 20 --warmup 5 --no-cpu" bash tools/gpu_ab.sh "$@" || exit 1
echo "--- 125k loopback"
AB_ARGS="--steps 20 --warmup 5 --no-cpu --edge 50 --comm-loopback" bash tools/gpu_ab.sh "$@"
