#!/bin/bash
# PMC counters of the row2 pair kernels (normal and SPH_EXP=1 gather-only), one
# rocprofv3 --pmc pass per counter group.  Usage: tools/pmc_row2.sh OUTDIR
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
OUT=$(realpath -m "$1")
mkdir -p "$OUT"
export TMPDIR=/tmp
export SPH_PATH=1
cd /tmp || exit 1
timeout -k 10 60 rocprofv3 --list-avail > "$OUT/avail.txt" 2>&1
i=0
for grp in "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_INST_CYCLES_VMEM_RD" \
           "TA_TA_BUSY_sum TA_BUFFER_READ_WAVEFRONTS_sum TD_TD_BUSY_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  for ex in 0 1; do
    SPH_EXP=$ex timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc${i}_exp$ex" -o pmc -- python3 "$R/tools/kernel_sweep.py" 100 5 > "$OUT/pmc${i}_exp$ex.log" 2>&1 || echo "pass $i exp $ex failed: $grp" >> "$OUT/failed.txt"
  done
done
