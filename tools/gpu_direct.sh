#!/bin/bash
# Brick + loopback parity with the direct forward comm, then the 125k/GPU proxy (one brick,
# halos through the RCCL loopback) with the dimension-ordered and the direct forward.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_bricks.py tests/test_gpu_engine.py -x -q --timeout 240 --timeout-method thread > gpurun_out/tb.log 2>&1
rc=$?
tail -2 gpurun_out/tb.log
[ $rc -eq 0 ] || { grep -m8 -E "FAILED|Error|error" gpurun_out/tb.log; exit $rc; }
for d in 0 1; do for e in 50 100; do
  echo -n "direct $d edge $e loopback: "
  SPH_DIRECT=$d timeout -k 10 200 python3 bench.py --edge $e --comm-loopback --steps 100 --warmup 20 --no-cpu 2>/dev/null | python3 -c "import json,sys;d=json.load(sys.stdin);print(round(d['ms_per_step'],4), 'ms/step comm', round(d['kernels']['comm_ms_per_step'],4), 'rebuild', round(d['kernels']['neighbor_build_ms'],3))" || exit 1
done; done
