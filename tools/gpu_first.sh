#!/bin/bash
# A session's first call: the new tests, the whole -m gpu suite + smoke, then the driver-shape
# C2 bench and its rocprofv3 kernel stats into gpurun_out/r03.  Test failures (rc 1) do not
# stop the later steps; a crash, abort or time limit does.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
R=$(pwd); O=$R/gpurun_out/r03; mkdir -p "$O"
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
FIRST=${FIRST:-tests/test_c5_bricks.py}
timeout -k 10 600 python -u -m pytest $FIRST -m gpu -v --timeout 240 --timeout-method thread > "$O/tests_first.log" 2>&1
rc=$?; grep -E "passed|failed|PASS|FAIL|Error" "$O/tests_first.log" | tail -25; ok $rc || exit $rc
timeout -k 10 900 python -u -m pytest tests/ -m gpu -v --timeout 240 --timeout-method thread > "$O/tests_all.log" 2>&1
rc=$?; grep -E "FAILED|ERROR| passed| failed" "$O/tests_all.log" | tail -25; ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" 2>&1 | tail -2 || exit 1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > "$O/bench_c2_20.json" 2> "$O/bench_c2_20.err" || { tail -5 "$O/bench_c2_20.err"; exit 1; }
echo "c2 20/5: $(cut -c1-400 "$O/bench_c2_20.json")"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof_c2" -o c2 -- python3 "$R/bench.py" --steps 20 --warmup 5 --no-cpu > "$O/bench_c2_prof.json" 2> "$O/prof_c2.err" || exit 1
cd "$R" && python3 tools/kstats.py "$(find "$O/prof_c2" -name '*kernel_stats.csv' | head -1)" 14
