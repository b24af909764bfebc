"""Kernel-by-kernel comparison of the neighbour rebuilds in a rocprofv3 kernel trace: for
each k_blk_build, the span from the preceding integrate kernel to the following rhosum, and
the kernels whose duration differs most between the first and the last rebuild.
usage: python tools/rebuild_compare.py trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
names = [r['Kernel_Name'] for r in rows]
idx = [k for k, n in enumerate(names) if 'k_blk_build' in n]
spans = []
for i in idx:
    j = i
    while j > 0 and 'k_final_initial' not in names[j] and 'k_initial_integrate' not in names[j]:
        j -= 1
    k = i
    while k < len(rows) - 1 and 'k_blk_rhosum' not in names[k]:
        k += 1
    t0, t1 = int(rows[j]['Start_Timestamp']), int(rows[k]['Start_Timestamp'])
    busy = sum(int(r['End_Timestamp']) - int(r['Start_Timestamp']) for r in rows[j:k])
    spans.append((j, k))
    print(f"rebuild at trace row {i}: span {(t1 - t0) / 1e3:9.1f} us, kernels {(busy) / 1e3:9.1f} us,"
          f" {k - j} launches")


def per_kernel(j, k):
    d = defaultdict(float)
    for r in rows[j:k]:
        d[r['Kernel_Name'][:60]] += (int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3
    return d


if len(spans) >= 2:
    a, b = per_kernel(*spans[1] if len(spans) > 2 else spans[0]), per_kernel(*spans[-1])
    keys = sorted(set(a) | set(b), key=lambda x: -abs(a.get(x, 0) - b.get(x, 0)))
    for kk in keys[:15]:
        print(f"{a.get(kk, 0):9.1f} {b.get(kk, 0):9.1f}  {kk}")
