#!/bin/bash
# PMC counters of the pair passes for one engine configuration: one rocprofv3 --pmc pass
# per counter group over tools/kernel_sweep.py.  Usage: tools/pmc_pass.sh OUTDIR [VAR=VAL ...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1")
shift
mkdir -p "$OUT"
for kv in "$@"; do export "$kv"; done
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU" \
           "TA_TA_BUSY_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o pmc -- python3 "$R/tools/${SWEEP:-kernel_sweep.py}" 100 ${SWEEP_REPS:-5} > "$OUT/pmc$i.log" 2>&1 || echo "pass $i failed: $grp" >> "$OUT/failed.txt"
done
