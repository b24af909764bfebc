#!/bin/bash
# Round-end evidence on one box: the whole -m gpu suite + smoke, then tools/gpu_r02.sh
# (C2 bench lines, rocprofv3 stats, PMC traffic, C5 lines and stats) and the C3 line.
# Usage: tools/gpu_final.sh COMMIT
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/r02/gpu_tests.log 2>&1
rc=$?
tail -1 gpurun_out/r02/gpu_tests.log
[ $rc -eq 0 ] || { grep -m5 -E "FAILED|Error" gpurun_out/r02/gpu_tests.log; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || { tail -3 gpurun_out/r02/smoke.log; exit 1; }
tail -1 gpurun_out/r02/smoke.log
timeout -k 10 300 python3 bench.py --workload c3 --steps 20 --warmup 5 > gpurun_out/r02/bench_c3.json 2> gpurun_out/r02/bench_c3.err || { tail -3 gpurun_out/r02/bench_c3.err; exit 1; }
echo "c3: $(cut -c1-200 gpurun_out/r02/bench_c3.json)"
tools/gpu_r02.sh "$1"
