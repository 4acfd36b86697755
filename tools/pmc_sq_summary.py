"""Per-kernel summary of a tools/pmc_sq.sh pass: MFMA busy as a fraction of the SIMD cycles the
dispatch spanned (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs), and the wave-state split (active / issue
stall / parked, SQ_* quad-cycles) — averages over the dispatches of each kernel."""
import collections
import csv
import glob
import os
import sys


def main(d):
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)[0]
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for row in csv.DictReader(open(f)):
        k = row['Kernel_Name'][:110]
        acc[k][row['Counter_Name']] += float(row['Counter_Value'])
        if row['Counter_Name'] == 'GRBM_GUI_ACTIVE':
            n[k] += 1
    print('%-110s %5s %8s %8s %7s %7s %7s %8s' % ('kernel', 'n', 'cycles', 'mfma', 'active', 'stall', 'parked',
                                                 'ldsconf'))
    for k, c in sorted(acc.items(), key=lambda kv: -kv[1]['GRBM_GUI_ACTIVE']):
        cyc = c['GRBM_GUI_ACTIVE'] / 8.0 / max(n[k], 1)
        mf = c['SQ_VALU_MFMA_BUSY_CYCLES'] / max(c['GRBM_GUI_ACTIVE'] / 8.0 * 1024, 1)
        wc = max(c['SQ_WAVE_CYCLES'], 1)
        print('%-110s %5d %8.0f %8.3f %7.3f %7.3f %7.3f %8.3f' % (
            k, n[k], cyc, mf, c['SQ_ACTIVE_INST_ANY'] / wc, c['SQ_WAIT_INST_ANY'] / wc, c['SQ_WAIT_ANY'] / wc,
            c['SQ_LDS_BANK_CONFLICT'] / max(c['SQ_BUSY_CYCLES'], 1)))


if __name__ == '__main__':
    main(sys.argv[1])
