#!/bin/bash
# PMC counter passes over the rebuild workload (tools/build_sweep.py) + per-kernel summary
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
TAG=$1; shift
OUT="$R/gpurun_out/pmcb_$TAG"; mkdir -p "$OUT"
for kv in "$@"; do export "$kv"; done
export TMPDIR=/tmp; cd /tmp || exit 1
i=0
for grp in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU" \
           "SQ_INSTS_VMEM_RD SQ_WAIT_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$OUT/pmc$i" -o pmc -- python3 "$R/tools/build_sweep.py" 100 3 > "$OUT/pmc$i.log" 2>&1 || echo "pass $i failed"
done
python3 - "$OUT" <<'PY'
import csv,glob,collections,sys
agg=collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(sys.argv[1]+"/pmc*/pmc_counter_collection.csv")):
    for r in csv.DictReader(open(f)):
        n=r["Kernel_Name"]
        for k in ("k_blk_neigh","k_neigh3","k_bin_copy"):
            if k in n:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                agg[k]["_dur_us"].append((float(r["End_Timestamp"])-float(r["Start_Timestamp"]))/1e3)
                agg[k]["_lds"].append(float(r["LDS_Block_Size"])); agg[k]["_vgpr"].append(float(r["VGPR_Count"]))
                agg[k]["_sgpr"].append(float(r.get("SGPR_Count",0) or 0))
                break
for k,d in agg.items():
    print(k, {c:(round(sum(v)/len(v)/1e6,2) if sum(v)/len(v)>1e4 else round(sum(v)/len(v),1)) for c,v in sorted(d.items())})
PY
