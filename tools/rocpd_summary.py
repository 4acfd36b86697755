"""Kernel summary of a rocprofv3 --kernel-trace database (rocpd SQLite, ROCm 7 default output).

  python tools/rocpd_summary.py <run_results.db> [--bench <bench log or JSON line>] [-o summary.txt]

Prints per-kernel calls / total / mean / median / min / max (us) over the whole run, and — when the
bench line holds "profile_windows" (bench.py: the CLOCK_BOOTTIME span of each labelled hipGraph
measurement, the clock of rocprofv3's timestamps) — the same statistics of the dispatches inside
each window, so a bench number can be checked against the profile of the same command.
"""
import argparse
import json
import re
import sqlite3
import sys

import numpy as np


def short(name, width=150):
    name = name.split('(')[0] if not name.startswith('void mt::group_kernel') else name[:name.find('>(') + 1]
    name = re.sub(r'^void ', '', name)
    name = name.replace('mt::', '')
    return name if len(name) <= width else name[:width - 3] + '...'


def load(db):
    c = sqlite3.connect(db)
    rows = c.execute('select name, start, end from kernels').fetchall()
    return [(n, int(s), int(e)) for n, s, e in rows]


def table(rows, title):
    by = {}
    for n, s, e in rows:
        by.setdefault(n, []).append((e - s) / 1e3)
    tot = sum(sum(v) for v in by.values()) or 1.0
    out = [title, '%6s %10s %9s %9s %9s %9s %6s  %s' % ('calls', 'total_us', 'mean_us', 'median', 'min', 'max', 'pct',
                                                       'kernel')]
    for n, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        a = np.asarray(v)
        out.append('%6d %10.1f %9.3f %9.3f %9.3f %9.3f %6.2f  %s' % (len(a), a.sum(), a.mean(), np.median(a), a.min(),
                                                                     a.max(), 100 * a.sum() / tot, short(n)))
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('db')
    ap.add_argument('--bench', default=None)
    ap.add_argument('-o', '--out', default=None)
    a = ap.parse_args()
    rows = load(a.db)
    lines = table(rows, '== all dispatches (%d) ==' % len(rows))
    if a.bench:
        line = [x for x in open(a.bench) if x.startswith('{')][-1]
        d = json.loads(line)
        for label, (t0, t1, calls) in sorted(d.get('profile_windows', {}).items(), key=lambda kv: kv[1][0]):
            sel = [r for r in rows if r[1] >= t0 and r[2] <= t1]
            lines.append('')
            lines += table(sel, '== window %s: %d dispatches in %.3f ms (%d graph calls timed by bench.py) ==' % (
                label, len(sel), (t1 - t0) / 1e6, calls))
        lines.append('')
        lines.append('bench line: metric %s value %s' % (d.get('metric'), d.get('value')))
    text = '\n'.join(lines) + '\n'
    if a.out:
        open(a.out, 'w').write(text)
    sys.stdout.write(text)


if __name__ == '__main__':
    main()
