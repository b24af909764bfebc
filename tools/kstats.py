"""Print a rocprofv3 *_kernel_stats.csv as a compact table (top N kernels)."""
import csv
import sys


def main(path, top=25):
    rows = list(csv.DictReader(open(path)))
    for r in rows[:top]:
        print(f"{r['Name'][:72]:72s} calls={int(r['Calls']):6d} "
              f"total_ms={float(r['TotalDurationNs']) / 1e6:9.3f} "
              f"avg_us={float(r['AverageNs']) / 1e3:9.2f} pct={float(r['Percentage']):5.1f}")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25)
