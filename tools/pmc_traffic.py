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


def load(path, counter, scale=1024.0, dur=None):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(f"{path}/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            if r["Counter_Name"] != counter:
                continue
            k = family(r["Kernel_Name"])
            if k:
                g = int(r.get("Grid_Size", 0) or 0)
                agg[k][g].append(float(r["Counter_Value"]) * scale)
                if dur is not None:
                    dur[k][g].append((float(r["End_Timestamp"]) - float(r["Start_Timestamp"])) * 1e-9)
    return agg


# fp64 VALU issue peak of the chip: 256 CUs x 4 SIMDs at 2.4 GHz, one wave64 fp64
# instruction per 4 cycles per SIMD (16 lanes/clk: the 78.6 TFLOP/s fp64 vector rate)
FP64_WAVE_INSTR_PER_S = 256 * 4 * 2.4e9 / 4.0


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
        # per step: all launches' bytes over the count of the largest-grid (main) launch; a
        # family with one launch per step whose grid drifts (C5: the atom count grows with
        # the insertions) is averaged over all its launches instead
        nmain = per[str(max(grids))]["launches"] if ok and grids else 0
        if ok and grids and min(grids) > 0.9 * max(grids):
            nmain = sum(v["launches"] for v in per.values())
        out[k] = {"grids": per, "traffic_bytes": tot / nmain if ok and nmain else None}
    dur = collections.defaultdict(lambda: collections.defaultdict(list))
    valu = load(f"{root}/valu", "SQ_INSTS_VALU", 1.0, dur)
    for k, grids in valu.items():
        # the main (largest-grid) launch: VALU wave-instructions per second over its duration,
        # every VALU instruction counted at the fp64 issue cost (an upper bound of the issue
        # time: 32-bit ops issue twice as fast)
        g = max(grids)
        ins = sum(grids[g]) / len(grids[g])
        d = sum(dur[k][g]) / len(dur[k][g])
        out.setdefault(k, {})["valu"] = {"wave_instr_per_launch": ins, "launch_s": d,
                                         "issue_frac_fp64": ins / d / FP64_WAVE_INSTR_PER_S}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    meta = {}
    for kv in sys.argv[2:]:
        k, v = kv.split("=", 1)
        meta[k] = int(v) if v.lstrip("-").isdigit() else v
    main(sys.argv[1], meta)
