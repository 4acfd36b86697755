"""Per-kernel averages of every counter in the rocprofv3 PMC passes under a directory
(tools/pmc_any.sh), kernels sorted by dispatch count x first counter."""
import collections
import csv
import glob
import json
import os
import re
import sys

root = sys.argv[1]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for path in glob.glob(os.path.join(root, '**', '*counter_collection.csv'), recursive=True):
    for r in csv.DictReader(open(path)):
        k = re.sub(r'\(.*', '', r['Kernel_Name'].replace('mt::', ''))[:160]
        vals[k][r['Counter_Name']].append(float(r['Counter_Value']))
out = {k: {c: round(sum(v) / len(v), 1) for c, v in d.items()} | {'dispatches': max(len(v) for v in d.values())}
       for k, d in vals.items()}
print(json.dumps(out, indent=1, sort_keys=True))
