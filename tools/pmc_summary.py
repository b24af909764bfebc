"""Summarise rocprofv3 --pmc CSVs (one directory per pass) per kernel family."""
import collections
import csv
import glob
import json
import sys


FAMILIES = ["k_blk_force", "k_blk_rhosum", "k_blk_build", "k_row2_force", "k_row2_rhosum",
            "k_bin_force", "k_bin_rhosum", "k_bin_neigh", "k_blk_neigh", "k_force", "k_rhosum", "k_neigh"]


def family(name):
    for k in FAMILIES:
        if k in name:
            return k
    return None


def main(root):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{root}/pmc*/pmc_counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = family(r["Kernel_Name"])
            if k:
                agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
                agg[k]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
                agg[k]["_lds"].append(float(r["LDS_Block_Size"]))
                agg[k]["_vgpr"].append(float(r["VGPR_Count"]))
    out = {k: {c: sum(v) / len(v) for c, v in sorted(d.items())} for k, d in agg.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1])
