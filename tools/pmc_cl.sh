#!/bin/bash
# PMC counters of the cluster-pair passes (TA busy, atomics, L2) for one configuration.
# Usage: tools/pmc_cl.sh OUTDIR [VAR=VAL ...]
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1")
shift
mkdir -p "$OUT"
for kv in "$@"; do export "$kv"; done
export TMPDIR=/tmp
cd /tmp || exit 1
i=0
for grp in "TA_TA_BUSY_sum TA_FLAT_ATOMIC_WAVEFRONTS_sum" \
           "TCP_TCC_ATOMIC_WITHOUT_RET_REQ_sum TCP_ATOMIC_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum" \
           "TCC_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o pmc -- python3 "$R/tools/kernel_sweep.py" 100 5 > "$OUT/pmc$i.log" 2>&1 || { echo "pass $i failed: $grp" >> "$OUT/failed.txt"; exit 1; }
done
