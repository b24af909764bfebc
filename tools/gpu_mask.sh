#!/bin/bash
# Bricks / C5 tests, then the three bench lines with the pair-pass-only timed region.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out/mask
timeout -k 10 600 python -u -m pytest tests/test_gpu_bricks.py tests/test_c5_bricks.py tests/test_multi_rank.py -m gpu -q \
  --timeout 240 --timeout-method thread > gpurun_out/mask/tests.log 2>&1 || { tail -30 gpurun_out/mask/tests.log; exit 1; }
tail -2 gpurun_out/mask/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu > gpurun_out/mask/c2_20.json 2> gpurun_out/mask/c2_20.err && \
timeout -k 10 300 python -u bench.py --steps 100 --warmup 20 --no-cpu > gpurun_out/mask/c2_100.json 2> gpurun_out/mask/c2_100.err && \
timeout -k 10 300 python -u bench.py --workload c5 --steps 20 --warmup 5 --no-cpu > gpurun_out/mask/c5.json 2> gpurun_out/mask/c5.err && \
timeout -k 10 300 python -u bench.py --workload c3 --steps 20 --warmup 5 --no-cpu > gpurun_out/mask/c3.json 2> gpurun_out/mask/c3.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 --no-cpu --edge 50 --comm-loopback > gpurun_out/mask/c2_e50_lb.json 2> gpurun_out/mask/lb.err
rc=$?
for f in gpurun_out/mask/*.json; do echo "$f"; python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d.get('kernels'), d.get('roofline',{}).get('frac'))"; done
exit $rc
