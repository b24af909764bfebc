"""Per-step HBM traffic of each kernel family from two rocprofv3 --pmc passes (FETCH_SIZE,
WRITE_SIZE; both in KB).  gfx950 correction (MI355X_MICROARCH.md, HBM): FETCH_SIZE reports
half the bytes of wide reads, so traffic = 2*FETCH + WRITE.  A family launched more than
once per step with different grids (k_blk_force: the main launch and the large-union one)
is kept per grid and summed into traffic_bytes per step.
Usage: pmc_traffic.py OUTDIR [key=value ...]   (key=value pairs go to _meta)"""
import collections
import csv
import glob
import json
import sys

FAMILIES = ("k_blk_force", "k_blk_rhosum", "k_blk_build", "k_blk_neigh", "k_mp2_gather",
            "k_mp2_rhosum", "k_mp2_colorgradient", "k_mp_gather", "k_mp_rhosum",
            "k_mp_colorgradient", "k_row2_force", "k_row2_rhosum", "k_force", "k_rhosum",
            "k_neigh3")


def family(name):
    for k in FAMILIES:
        if k in name:
            return k
    return None


def load(path, counter):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{path}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = family(r["Kernel_Name"])
            if k:
                agg[k][int(r.get("Grid_Size", 0) or 0)].append(float(r["Counter_Value"]) * 1024.0)
    return agg


def main(root, meta):
    fetch = load(f"{root}/fetch", "FETCH_SIZE")
    write = load(f"{root}/write", "WRITE_SIZE")
    out = {"_meta": meta}
    for k in sorted(set(fetch) | set(write)):
        grids = sorted(set(fetch.get(k, {})) | set(write.get(k, {})))
        per = {}
        tot = 0.0
        ok = True
        for g in grids:
            f = fetch.get(k, {}).get(g)
            w = write.get(k, {}).get(g)
            if not f or not w:
                ok = False
                continue
            fa, wa = sum(f) / len(f), sum(w) / len(w)
            per[str(g)] = {"fetch_bytes": fa, "write_bytes": wa, "launches": len(f),
                           "traffic_bytes": 2.0 * fa + wa}
            tot += (2.0 * fa + wa) * len(f)
        # per step: all launches' bytes over the count of the largest-grid (main) launch
        nmain = per[str(max(grids))]["launches"] if ok and grids else 0
        out[k] = {"grids": per, "traffic_bytes": tot / nmain if ok and nmain else None}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    meta = {}
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        meta[k] = int(v) if v.lstrip("-").isdigit() else v
    main(sys.argv[1], meta)
