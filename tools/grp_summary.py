"""Summed per-kernel time [us per step] of tools/group_probe.py runs under
rocprofv3 --stats (gpurun_out/<tag>/grp_<wl>_<W>/run_kernel_stats.csv)."""
import csv
import glob
import re
import sys

rows = {}
for d in sorted(glob.glob(sys.argv[1] + '/grp_*_[0-9]*/run_kernel_stats.csv')):
    w = int(re.search(r'_(\d+)/run_kernel', d).group(1))
    steps = 12 * 1.0
    for r in csv.DictReader(open(d)):
        name = re.sub(r'\(.*', '', r['Name']).replace('bsa::', '').replace('void ', '')
        name = 'rocprim' if 'rocprim' in name else name
        rows.setdefault(name, {})
        rows[name][w] = rows[name].get(w, 0.0) + float(r['TotalDurationNs']) / 1e3 / steps
ws = sorted({w for v in rows.values() for w in v})
print('%-28s' % 'kernel (us/step, all ranks)' + ''.join('%10s' % ('W=%d' % w) for w in ws))
for k, v in sorted(rows.items(), key=lambda kv: -kv[1].get(1, 0)):
    print('%-28s' % k[:28] + ''.join('%10.1f' % v.get(w, 0.0) for w in ws))
print('%-28s' % 'TOTAL' + ''.join('%10.1f' % sum(v.get(w, 0.0) for v in rows.values()) for w in ws))
