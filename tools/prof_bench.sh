#!/bin/bash
# rocprofv3 kernel-trace + stats of a bench.py run (no counters, no API tracing).
# Usage: tools/prof_bench.sh OUTDIR [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o bench -- \
  python3 "$R/bench.py" "$@" > "$OUT/bench.json" 2> "$OUT/bench.err"
