#!/bin/bash
# Block-path iteration: engine parity tests (optional), pair-pass timings per SPH_BLK
# shape, and rocprofv3 kernel stats of the block kernels for each shape.
# Usage: tools/gpu_blk.sh TAG "shapes" [test]
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
R=$(pwd)
mkdir -p gpurun_out
TAG=${1:-blk}; SHAPES=${2:-"0 1 2 3 4"}
if [ "$3" = "test" ]; then
  timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py -x -q \
    --timeout 120 --timeout-method thread > "gpurun_out/t_$TAG.log" 2>&1 || { tail -30 "gpurun_out/t_$TAG.log"; exit 1; }
  tail -2 "gpurun_out/t_$TAG.log"
fi
export TMPDIR=/tmp
for b in $SHAPES; do
  (cd /tmp && SPH_BLK=$b timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
     -d "$R/gpurun_out/prof_${TAG}_$b" -o run -- python3 "$R/tools/kernel_sweep.py" 100 20) > "$R/gpurun_out/sweep_${TAG}_$b.log" 2>&1 || exit 1
  echo "shape $b: $(tail -1 $R/gpurun_out/sweep_${TAG}_$b.log)"
  f=$(find "$R/gpurun_out/prof_${TAG}_$b" -name '*kernel_stats.csv' | head -1)
  grep -E "k_blk|k_neigh3|Name" "$f" | cut -d, -f1-5 | cut -c1-160
done
