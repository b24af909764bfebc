#!/bin/bash
# Round-6 evidence into gpurun_out/r06/final: C2 bench (driver shape with the CPU baseline,
# and 100/20), rocprofv3 kernel stats of the driver shape, PMC traffic (FETCH / WRITE / VALU
# passes) for C2 and C5, C5 4.02M bench + kernel trace, C3, the 125k loopback brick.
# Every GPU step under its own limit; the first failure ends the script.
# Usage: tools/gpu_final6.sh COMMIT
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
R=$(pwd); O=$R/gpurun_out/r06/final; C=${1:-unknown}
mkdir -p "$O"
timeout -k 10 400 python3 bench.py > "$O/bench_c2_default.json" 2> "$O/bench_c2_default.err" || { tail -5 "$O/bench_c2_default.err"; exit 1; }
echo "c2 default: $(cut -c1-160 "$O/bench_c2_default.json")"
timeout -k 10 400 python3 bench.py --steps 100 --warmup 20 --no-cpu > "$O/bench_c2_100.json" 2> "$O/bench_c2_100.err" || exit 1
echo "c2 100/20: $(cut -c1-160 "$O/bench_c2_100.json")"
META="world=1 edge=100 path=0 steps=20 warmup=5 commit=$C" timeout -k 10 700 tools/pmc_traffic.sh "$O/pmc_c2" --steps 20 --warmup 5 --no-cpu || exit 1
echo "pmc c2 done"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c2" -o c2 -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu > "$O/bench_c2_prof.json" 2> "$O/prof_c2.err" || exit 1
cd "$R" && python3 tools/kstats.py "$(find "$O/prof_c2" -name '*kernel_stats.csv' | head -1)" 8
timeout -k 10 600 python3 bench.py --workload c5 --steps 10 --warmup 3 > "$O/bench_c5.json" 2> "$O/bench_c5.err" || { tail -5 "$O/bench_c5.err"; exit 1; }
echo "c5: $(cut -c1-160 "$O/bench_c5.json")"
META="world=1 edge=159 path=0 steps=5 warmup=2 commit=$C" timeout -k 10 900 tools/pmc_traffic.sh "$O/pmc_c5" --workload c5 --steps 5 --warmup 2 --no-cpu || exit 1
echo "pmc c5 done"
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c5" -o c5 -- python3 "$R/bench.py" --workload c5 --steps 5 --warmup 2 --no-cpu > "$O/bench_c5_prof.json" 2> "$O/prof_c5.err" || exit 1
cd "$R" && python3 tools/kstats.py "$(find "$O/prof_c5" -name '*kernel_stats.csv' | head -1)" 10
timeout -k 10 400 python3 bench.py --workload c3 --steps 20 --warmup 5 > "$O/bench_c3.json" 2> "$O/bench_c3.err" || { tail -5 "$O/bench_c3.err"; exit 1; }
echo "c3: $(cut -c1-160 "$O/bench_c3.json")"
timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu --edge 50 --comm-loopback > "$O/bench_lb125k.json" 2> "$O/bench_lb125k.err" || { tail -5 "$O/bench_lb125k.err"; exit 1; }
echo "lb125k: $(cut -c1-160 "$O/bench_lb125k.json")"
