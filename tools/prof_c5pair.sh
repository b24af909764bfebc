#!/bin/bash
# rocprofv3 kernel-trace + stats of the C5 pair-pass workload (bench.py --workload c5pair).
# Usage: tools/prof_c5pair.sh OUTDIR [bench args...]
set -e
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); shift
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o c5pair -- \
  python3 "$R/bench.py" --workload c5pair "$@" > "$OUT/c5pair.json" 2> "$OUT/c5pair.err"
