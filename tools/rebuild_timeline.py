"""Kernel timeline of the last neighbour rebuild in a rocprofv3 kernel trace.

usage: python tools/rebuild_timeline.py trace.csv [min_us]
"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
mn = float(sys.argv[2]) if len(sys.argv) > 2 else 8.0
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'] for r in rows]
i = [k for k, n in enumerate(names) if 'k_blk_build' in n or 'k_blk_neigh' in n][-1]
j = i
while 'k_final_initial' not in names[j] and 'k_initial_integrate' not in names[j]:
    j -= 1
k = i
while 'k_blk_rhosum' not in names[k]:
    k += 1
t0 = int(rows[j]['Start_Timestamp'])
prev = t0
gaps = 0.0
for r in rows[j:k + 1]:
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    g = (s - prev) / 1e3
    if g > mn or (e - s) / 1e3 > 3 * mn:
        print("%8.1f gap %7.1f dur %8.1f  %s" % ((s - t0) / 1e3, g, (e - s) / 1e3, r['Kernel_Name'][:70]))
    gaps += max(g, 0.0)
    prev = e
print("total %.1f us, gaps %.1f us" % ((int(rows[k]['Start_Timestamp']) - t0) / 1e3, gaps))
