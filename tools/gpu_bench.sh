#!/bin/bash
# bench.py lines (driver shape and a longer one) + a rocprofv3 kernel-stats pass.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
R=$(pwd); TAG=${1:-b}; shift
mkdir -p gpurun_out
timeout -k 10 400 python bench.py --steps 20 --warmup 5 "$@" > gpurun_out/bench_${TAG}_20.json 2> gpurun_out/bench_${TAG}_20.err || { tail -5 gpurun_out/bench_${TAG}_20.err; exit 1; }
timeout -k 10 400 python bench.py --steps 100 --warmup 20 --no-cpu "$@" > gpurun_out/bench_${TAG}_100.json 2> gpurun_out/bench_${TAG}_100.err || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/prof_bench_$TAG" -o bench -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu "$@" > "$R/gpurun_out/bench_${TAG}_prof.json" 2>/dev/null || exit 1
cd "$R" && python3 tools/kstats.py "$(find gpurun_out/prof_bench_$TAG -name '*kernel_stats.csv' | head -1)" 14
