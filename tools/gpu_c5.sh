#!/bin/bash
# C5 at 4.02M on one GPU: bench line + rocprofv3 kernel stats into gpurun_out/r03.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
R=$(pwd); O=$R/gpurun_out/r03; mkdir -p "$O"
timeout -k 10 600 python3 bench.py --workload c5 --steps 10 --warmup 3 > "$O/bench_c5.json" 2> "$O/bench_c5.err" || { tail -5 "$O/bench_c5.err"; exit 1; }
echo "c5: $(cut -c1-300 "$O/bench_c5.json")"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5" -o c5 -- python3 "$R/bench.py" --workload c5 --steps 5 --warmup 2 --no-cpu > "$O/bench_c5_prof.json" 2> "$O/prof_c5.err" || exit 1
cd "$R" && python3 tools/kstats.py "$(find "$O/prof_c5" -name '*kernel_stats.csv' | head -1)" 25
