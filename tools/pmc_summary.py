"""Per-kernel averages of the rocprofv3 PMC passes written by tools/pmc.sh (one directory per
counter). FETCH_SIZE / WRITE_SIZE are KiB per dispatch (counter_defs.yaml); on gfx950
FETCH_SIZE counts half the bytes of 16 B/lane streaming reads (MI355X_MICROARCH.md, HBM), so
hbm_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024. Other access widths are uncalibrated."""
import collections
import csv
import glob
import json
import os
import re
import sys


def short(name):
    n = re.sub(r'mt::', '', name)
    return re.sub(r'\(.*', '', n)


root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for counter in ('FETCH_SIZE', 'WRITE_SIZE'):
    for path in glob.glob(os.path.join(root, counter, '**', '*counter_collection.csv'), recursive=True):
        for r in csv.DictReader(open(path)):
            if r.get('Counter_Name') != counter:
                continue
            vals[short(r['Kernel_Name'])][counter].append(float(r['Counter_Value']))
out = {}
for k, d in vals.items():
    f = d.get('FETCH_SIZE', [])
    w = d.get('WRITE_SIZE', [])
    if not f or not w:
        continue
    fa, wa = sum(f) / len(f), sum(w) / len(w)
    out[k] = dict(dispatches=len(f), FETCH_SIZE_KiB=round(fa, 3), WRITE_SIZE_KiB=round(wa, 3),
                  hbm_bytes=round(2 * fa * 1024 + wa * 1024))
print(json.dumps(out, indent=1, sort_keys=True))
