#!/usr/bin/env python3
"""Summarise rocprofv3 --pmc passes per kernel.

usage: pmc_summary.py DIR [DIR ...] [--kernels k_prefilter,k_exact,...]

Each DIR holds one pass (run_counter_collection.csv + run_kernel_trace.csv).
Counter values are summed over the dispatches of a kernel (all XCDs / SEs
are already aggregated by rocprofv3 per dispatch) and divided by the number
of dispatches, so every number is PER LAUNCH.  Durations come from the
kernel trace of the same pass (profiled passes run slower than unprofiled
ones; use bench.py's event timings for rates).
"""
import argparse
import collections
import csv
import json
import os
import sys


def short(name):
    n = name.split('(')[0]
    n = n.replace('void ', '').replace('bsa::', '')
    return n[:60]


def load(d):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    with open(os.path.join(d, 'run_counter_collection.csv')) as f:
        for r in csv.DictReader(f):
            k = short(r['Kernel_Name'])
            per[k][r['Counter_Name']] += float(r['Counter_Value'])
            disp[k].add(r['Dispatch_Id'])
    dur = collections.defaultdict(list)
    tr = os.path.join(d, 'run_kernel_trace.csv')
    if os.path.exists(tr):
        with open(tr) as f:
            for r in csv.DictReader(f):
                dur[short(r['Kernel_Name'])].append(int(r['End_Timestamp']) - int(r['Start_Timestamp']))
    out = {}
    for k, cs in per.items():
        nd = max(1, len(disp[k]))
        out[k] = {c: v / nd for c, v in cs.items()}
        out[k]['_dispatches'] = nd
        if dur.get(k):
            out[k]['_dur_ns'] = sum(dur[k]) / len(dur[k])
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('dirs', nargs='+')
    ap.add_argument('--kernels', default='')
    ap.add_argument('--json', default='')
    a = ap.parse_args()
    merged = collections.defaultdict(dict)
    for d in a.dirs:
        for k, cs in load(d).items():
            merged[k].update(cs)
    want = [w for w in a.kernels.split(',') if w]
    keys = [k for k in merged if not want or any(w in k for w in want)]
    for k in sorted(keys, key=lambda k: -merged[k].get('_dur_ns', 0)):
        print('==', k)
        for c, v in sorted(merged[k].items()):
            print('   %-28s %16.1f' % (c, v))
    if a.json:
        with open(a.json, 'w') as f:
            json.dump({k: merged[k] for k in keys}, f, indent=1, sort_keys=True)


if __name__ == '__main__':
    sys.exit(main())
