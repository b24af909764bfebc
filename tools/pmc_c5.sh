#!/bin/bash
# PMC counters of the C5 engine kernels (1M-particle bubble, 3 steps): one rocprofv3 --pmc
# pass per counter group.  Usage: tools/pmc_c5.sh OUTDIR [edge]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1"); E=${2:-100}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_INSTS_SALU" \
           "TA_TA_BUSY_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o pmc -- python3 "$R/bench.py" --workload c5 --edge $E --steps 2 --warmup 1 --no-cpu > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed: $grp"; exit 1; }
done
python3 "$R/tools/pmc_table.py" "$OUT" k_mp > "$OUT/table.json"; cat "$OUT/table.json" | head -80
