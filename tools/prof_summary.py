"""Summarise a rocprofv3 kernel trace: per (kernel, grid) average duration and total."""
import collections
import csv
import re
import sys

path = sys.argv[1]
rows = list(csv.DictReader(open(path)))
agg = collections.defaultdict(list)
for r in rows:
    n = re.sub(r'mt::', '', r['Kernel_Name'])
    n = re.sub(r'\(.*', '', n)[:90]
    g = '%sx%sx%s' % (r['Grid_Size_X'], r['Grid_Size_Y'], r['Grid_Size_Z'])
    agg[(n, g)].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
tot = sum(sum(v) for v in agg.values())
print('%6s %9s %9s %6s  %s' % ('calls', 'avg_us', 'total_ms', 'pct', 'kernel [grid threads]'))
for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
    print('%6d %9.2f %9.3f %6.2f  %s [%s]' % (len(v), sum(v) / len(v) / 1e3, sum(v) / 1e6, 100.0 * sum(v) / tot, k[0], k[1]))
