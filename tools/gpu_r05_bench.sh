#!/bin/bash
# Round-5 bench lines on one box: C2 at the driver's 20/5 (with the CPU baselines), C2 100/20,
# C5, the 125k RCCL-loopback proxy, and rocprofv3 --kernel-trace --stats of the C2 20/5 run.
# Usage: tools/gpu_r05_bench.sh OUTDIR
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
O=$1; mkdir -p "$O"
run() {  # name, args...
  local n=$1; shift
  timeout -k 10 400 python3 bench.py "$@" > "$O/$n.json" 2> "$O/$n.err" || { tail -3 "$O/$n.err"; return 1; }
  echo "$n: $(cut -c1-160 "$O/$n.json")"
}
run bench_c2_20 --steps 20 --warmup 5 &&
run bench_c2_100 --steps 100 --warmup 20 --no-cpu &&
run bench_c5 --workload c5 --steps 10 --warmup 3 &&
run bench_lb125k --edge 50 --comm-loopback --steps 100 --warmup 20 --no-cpu &&
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$GRAFT_REPO_ROOT/$O/rocprof_c2" -o c2 -- python3 "$GRAFT_REPO_ROOT/bench.py" --steps 20 --warmup 5 --no-cpu > "$GRAFT_REPO_ROOT/$O/rocprof_c2.log" 2>&1) &&
echo "rocprof c2 done"
