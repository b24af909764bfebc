#!/bin/bash
# Round 6 perf pass: C2 1M bench + kernel trace (step / rebuild timelines), the 125k RCCL
# loopback proxy with and without the halo overlap (+ trace).  Usage: tools/gpu_r06_perf.sh DIR
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
D=$R/gpurun_out/$1
mkdir -p "$D"
export TMPDIR=/tmp
cd /tmp || exit 1
step() {  # name secs cmd...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "$D/$name.log" 2>&1
  local rc=$?
  tail -c 600 "$D/$name.log"; echo; echo "== $name rc=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
}
step c2 200 python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu
step lb 200 python3 -u "$R/bench.py" --edge 50 --comm-loopback --steps 100 --warmup 20 --no-cpu
step lbov 200 python3 -u "$R/bench.py" --edge 50 --comm-loopback --overlap --steps 100 --warmup 20 --no-cpu
[ -n "$R06_MORE" ] && {
step c4ipc 400 python3 -u "$R/bench.py" --gpus 8 --transport ipc --scaling weak --steps 10 --warmup 3 --no-cpu
step c5ipc 400 python3 -u "$R/bench.py" --workload c5 --gpus 8 --transport ipc --steps 6 --warmup 2 --no-cpu
step c2pair 300 python3 -u "$R/bench.py" --workload c2pair --edge 80 --steps 10 --warmup 3 --no-cpu
exit 0
}
step c2trace 300 rocprofv3 --kernel-trace --output-format csv -d "$D/c2prof" -o c2 -- python3 -u "$R/bench.py" --steps 20 --warmup 5 --no-cpu
step lbtrace 300 rocprofv3 --kernel-trace --output-format csv -d "$D/lbprof" -o lb -- python3 -u "$R/bench.py" --edge 50 --comm-loopback --overlap --steps 30 --warmup 5 --no-cpu
cd "$R" || exit 1
python3 tools/step_timeline.py "$(find "$D/c2prof" -name '*kernel_trace.csv' | head -1)" 1 > "$D/c2_step_timeline.txt" 2>&1
python3 tools/rebuild_timeline.py "$(find "$D/c2prof" -name '*kernel_trace.csv' | head -1)" 5 > "$D/c2_rebuild_timeline.txt" 2>&1
python3 tools/step_timeline.py "$(find "$D/lbprof" -name '*kernel_trace.csv' | head -1)" 1 > "$D/lb_step_timeline.txt" 2>&1
python3 tools/rebuild_timeline.py "$(find "$D/lbprof" -name '*kernel_trace.csv' | head -1)" 5 > "$D/lb_rebuild_timeline.txt" 2>&1
tail -3 "$D"/*timeline.txt
