#!/bin/bash
# The first-interval slowdown with a clock counter: inner_probe.py's 25
# C2 steps after setup, once plain and once under rocprofv3 with GRBM_GUI_ACTIVE (GPU clock
# cycles while the graphics pipe is busy) and SQ_BUSY_CYCLES per dispatch, beside each
# dispatch's duration: effective clock = cycles / duration.  Usage: tools/clock_probe.sh OUTDIR
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1")
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
timeout -k 10 240 python3 -u "$R/tools/inner_probe.py" > "$OUT/plain.log" 2>&1 || exit $?
timeout -k 10 240 python3 -u "$R/tools/inner_probe.py" --sampler > "$OUT/sampler.log" 2>&1 || exit $?
timeout -s KILL 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_BUSY_CYCLES \
  --output-format csv -d "$OUT/pmc" -o clk -- python3 -u "$R/tools/inner_probe.py" \
  > "$OUT/pmc.log" 2>&1
