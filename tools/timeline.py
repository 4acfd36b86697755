"""Print the device timeline (kernels + memory copies, with gaps) of a few rollout macro-steps from
a rocprofv3 --kernel-trace --memory-copy-trace CSV directory.

    python tools/timeline.py gpurun_out/tl_r01 [--anchor preprocess] [--which 200] [--count 2]
"""
import argparse
import csv
import glob
import os


def load(d):
    ev = []
    for f in glob.glob(os.path.join(d, '**', '*kernel_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'K', r['Kernel_Name'][:90],
                       int(r['Grid_Size_X']) // max(int(r['Workgroup_Size_X']), 1)))
    for f in glob.glob(os.path.join(d, '**', '*memory_copy_trace.csv'), recursive=True):
        for r in csv.DictReader(open(f)):
            kind = r.get('Direction') or r.get('Operation') or 'COPY'
            ev.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), 'C', kind, int(r.get('Size', 0) or 0)))
    ev.sort()
    return ev


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dir')
    ap.add_argument('--anchor', default='preprocess')
    ap.add_argument('--which', type=int, default=200)
    ap.add_argument('--count', type=int, default=2)
    a = ap.parse_args()
    ev = load(a.dir)
    idx = [i for i, e in enumerate(ev) if e[2] == 'K' and a.anchor in e[3]]
    lo, hi = idx[a.which], idx[min(a.which + a.count, len(idx) - 1)]
    t0 = ev[lo][0]
    prev_end = ev[lo - 1][1]
    busy = 0
    for e in ev[lo - 1:hi + 1]:
        s, t, k, name, n = e
        gap = (s - prev_end) / 1e3
        print('%9.1f us  +gap %7.1f  dur %7.1f  %s %-90s %s' % ((s - t0) / 1e3, gap, (t - s) / 1e3, k, name, n))
        prev_end = max(prev_end, t)
        busy += t - s
    span = (ev[hi][1] - ev[lo][0]) / 1e3
    print('span %.1f us over %d anchors, busy %.1f us' % (span, a.count, busy / 1e3))


if __name__ == '__main__':
    main()
