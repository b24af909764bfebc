"""Per dispatch of the force / rhosum passes in a rocprofv3 --pmc GRBM_GUI_ACTIVE
SQ_BUSY_CYCLES --kernel-trace run (tools/clock_probe.sh): duration, the counters, and the
clock they imply.  GRBM_GUI_ACTIVE is summed over the 8 XCDs' GRBMs and counts from counter
start to stop (a ~15 us window around the dispatch under --pmc serialisation: the copies of
~3 us read ~300k); clock_GHz = GRBM_GUI_ACTIVE / 8 / duration is therefore an upper figure,
its CHANGE from step to step at equal cycles is what the probe is after.
Usage: python3 tools/clock_summary.py DIR/clk_counter_collection.csv"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = {}
for r in rows:
    k = int(r["Dispatch_Id"])
    e = d.setdefault(k, {"name": r["Kernel_Name"],
                         "dur": int(r["End_Timestamp"]) - int(r["Start_Timestamp"])})
    e[r["Counter_Name"]] = float(r["Counter_Value"])
print(f"{'dispatch':>8} {'kernel':<22} {'dur_us':>8} {'GRBM_GUI_ACTIVE':>16} {'SQ_BUSY_CYCLES':>15} "
      f"{'GRBM/8/dur GHz':>15}")
for k in sorted(d):
    e = d[k]
    nm = e["name"]
    tag = "k_blk_force_w6" if "k_blk_force" in nm else "k_blk_rhosum" if "k_blk_rhosum" in nm else None
    if not tag:
        continue
    g = e["GRBM_GUI_ACTIVE"]
    print(f"{k:8d} {tag:<22} {e['dur'] / 1e3:8.1f} {g:16.0f} {e['SQ_BUSY_CYCLES']:15.0f} "
          f"{g / 8 / e['dur']:15.3f}")
