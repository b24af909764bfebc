"""Per-kernel means of rocprofv3 --pmc CSVs under a directory tree (any pass layout)."""
import collections
import csv
import glob
import json
import sys


def main(root, pat=""):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{root}/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            if pat and pat not in k:
                continue
            agg[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
            agg[k]["_dur_us"].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) / 1e3)
    out = {k: {c: sum(v) / len(v) for c, v in sorted(d.items())} for k, d in agg.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "")
