"""Launch gaps of a rocprofv3 kernel trace: for the last `--window` kernels of
the run (the timed steps), the busy time (sum of kernel durations), the span
and the idle gaps between consecutive kernels, by the kernel that follows.
Usage: python tools/trace_gaps.py run_kernel_trace.csv [--window N]"""
import csv
import re
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    window = int(sys.argv[sys.argv.index('--window') + 1]) if '--window' in sys.argv else 400
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']),
                  re.sub(r'\(.*', '', r['Kernel_Name']).replace('bsa::', '').replace('void ', '')[:40])
                 for r in rows), key=lambda x: x[0])[-window:]
    busy = sum(e - s for s, e, _ in ks)
    span = ks[-1][1] - ks[0][0]
    gaps = defaultdict(float)
    cnt = defaultdict(int)
    for (s0, e0, _), (s1, e1, n1) in zip(ks, ks[1:]):
        gaps[n1] += max(0, s1 - e0)
        cnt[n1] += 1
    print('last %d kernels: span %.1f us, busy %.1f us, idle %.1f us (%.0f%%)' %
          (len(ks), span / 1e3, busy / 1e3, (span - busy) / 1e3, 100.0 * (span - busy) / span))
    for n, g in sorted(gaps.items(), key=lambda kv: -kv[1])[:12]:
        print('  gap before %-40s %8.1f us total, %6.2f us avg (%d)' % (n, g / 1e3, g / 1e3 / cnt[n], cnt[n]))


if __name__ == '__main__':
    main()
