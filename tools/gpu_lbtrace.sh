#!/bin/bash
# rocprofv3 kernel trace of the 125k-particle RCCL-loopback brick (one of 8 GPUs' share of
# C2) and the timeline of its last rebuild
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
R=$(pwd); O=$R/gpurun_out/lb; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o lb -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu --edge 50 --comm-loopback > "$O/bench.json" 2> "$O/bench.err" || { tail -5 "$O/bench.err"; exit 1; }
cd "$R" && python3 tools/rebuild_timeline.py "$(find "$O/prof" -name '*kernel_trace.csv' | head -1)" 0 > "$O/timeline.txt"; tail -80 "$O/timeline.txt"
