#!/bin/bash
# Run GPU steps in order on the gpurun box, each under its own time limit, logging to
# gpurun_out/<dir>/<name>.log.  Usage:
#   tools/gpu_steps.sh DIR 'name|seconds|command' ['name|seconds|command' ...]
# A step that FAILS (exit 1: a test failed) does not stop the rest; a step that times out,
# aborts or crashes (any other non-zero status) ends the script there -- nothing more runs
# on the GPU after a fault.
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R" || exit 2
out="gpurun_out/$1"
shift
mkdir -p "$out"
final=0
for step in "$@"; do
  name=${step%%|*}
  rest=${step#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  echo "== $name ($secs s): $cmd"
  timeout -k 10 "$secs" bash -c "$cmd" > "$out/$name.log" 2>&1
  rc=$?
  tail -n 4 "$out/$name.log"
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then
    echo "== stopping after $name (rc $rc)"
    exit $rc
  fi
  [ $rc -ne 0 ] && final=$rc
done
exit $final
