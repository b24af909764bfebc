#!/bin/bash
# Iteration loop: engine/brick/C1 GPU tests, pair-pass and rebuild timings (C2 1M), then a
# driver-shape bench line.  BEXPS: block-build study variants to time as well.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_bricks.py tests/test_water_collapse.py -x -q --timeout 240 --timeout-method thread > gpurun_out/tq.log 2>&1
rc=$?
tail -3 gpurun_out/tq.log
[ $rc -eq 0 ] || { grep -m5 -E "FAILED|Error" gpurun_out/tq.log; exit $rc; }
echo -n "pairs: "; timeout -k 10 120 python3 tools/kernel_sweep.py 100 20 || exit 1
for e in ${BEXPS:-0}; do echo -n "rebuild bexp $e: "; SPH_BEXP=$e timeout -k 10 120 python3 tools/build_sweep.py 100 5 || exit 1; done
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/bench_iter.json 2> gpurun_out/bench_iter.err || { tail -5 gpurun_out/bench_iter.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/bench_iter.json'));print('bench', round(d['value']/1e6,1), 'M p-s/s', round(d['ms_per_step'],4), 'ms/step', {k:(round(v,4) if isinstance(v,float) else v) for k,v in d['kernels'].items() if not isinstance(v,dict)})"
