#!/bin/bash
# PMC passes over the pair passes of one engine config + summary.  Usage: tools/gpu_pmc.sh TAG [VAR=VAL ...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
"$R/tools/pmc_pass.sh" "$R/gpurun_out/pmc_$TAG" "$@"
python3 "$R/tools/pmc_summary.py" "$R/gpurun_out/pmc_$TAG" > "$R/gpurun_out/pmc_$TAG.json"
cat "$R/gpurun_out/pmc_$TAG/failed.txt" 2>/dev/null
python3 - "$R/gpurun_out/pmc_$TAG.json" <<'PY'
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    print(k, {c: round(x,3) for c,x in v.items()})
PY
