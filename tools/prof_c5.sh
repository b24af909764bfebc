#!/bin/bash
# rocprofv3 kernel-trace stats of a short C5 run (4.02M by default) + its bench line.
cd "${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}" || exit 1
R=$(pwd); O=$R/gpurun_out/${TAG:-c5prof}; mkdir -p "$O"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o c5 -- python3 "$R/bench.py" --workload c5 --edge ${EDGE:-159} --steps ${STEPS:-5} --warmup 2 --no-cpu > "$O/bench.json" 2> "$O/prof.err" || { tail -5 "$O/prof.err"; exit 1; }
cd "$R" && python3 tools/kstats.py "$(find "$O/prof" -name '*kernel_stats.csv' | head -1)" ${TOP:-22}
python3 -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value']/1e6,1),'M p-s/s',round(d['ms_per_step'],2),'ms/step')"
