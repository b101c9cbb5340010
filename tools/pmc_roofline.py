#!/usr/bin/env python3
"""Turn rocprofv3 --pmc passes of the bench into the per-launch figures that
bench.py reports next to its live timings (profiles/pmc_latest.json).

usage: pmc_roofline.py [--bench-json B.json] OUT.json PASSDIR [PASSDIR ...]

The library the counters belong to is recorded in _meta.lib_sha256, taken
from the profiled bench's own output line (bench.py prints the sha256 of the
libbsaccel it actually mapped, BSACCEL_LIB resolved) when --bench-json is
given, else hashed from $BSACCEL_LIB or the in-tree default.  Nothing edits
_meta by hand: bench.py reports the PMC figures only when that sha equals the
sha of the library it mapped itself.

Per kernel and per launch (mean over dispatches):
  hbm_read_bytes   = 2 * FETCH_SIZE[KB] * 1024   (gfx950 FETCH_SIZE counts half of a
                     wide coalesced read: MI355X_MICROARCH.md 'HBM'; Infinity-Cache
                     hits are included, so this is memory-side traffic, an upper
                     bound on HBM bytes)
  hbm_write_bytes  = WRITE_SIZE[KB] * 1024
  lds_bank_conflict_rate = SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE
  valu_insts, lds_insts, salu_insts (wave instructions)
  fp64_flops       = 64 * (2 FMA_F64 + ADD_F64 + MUL_F64 + TRANS_F64)  (per-lane ops)
  dur_ns           = kernel duration in the profiled passes (slower than unprofiled)
"""
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from pmc_summary import load  # noqa: E402


def main():
    args = sys.argv[1:]
    bench_json = None
    if args[:1] == ['--bench-json']:
        bench_json, args = args[1], args[2:]
    out, dirs = args[0], args[1:]
    merged = {}
    for d in dirs:
        for k, cs in load(d).items():
            merged.setdefault(k, {}).update(cs)
    res = {}
    for k, c in merged.items():
        name = k.split('<')[0]
        r = {'dur_ns': c.get('_dur_ns')}
        if 'FETCH_SIZE' in c:
            r['hbm_read_bytes'] = 2.0 * c['FETCH_SIZE'] * 1024.0
        if 'WRITE_SIZE' in c:
            r['hbm_write_bytes'] = c['WRITE_SIZE'] * 1024.0
        if 'SQ_LDS_IDX_ACTIVE' in c and c['SQ_LDS_IDX_ACTIVE'] > 0:
            r['lds_bank_conflict_rate'] = c.get('SQ_LDS_BANK_CONFLICT', 0.0) / c['SQ_LDS_IDX_ACTIVE']
        for src, dst in (('SQ_INSTS_VALU', 'valu_insts'), ('SQ_INSTS_LDS', 'lds_insts'),
                         ('SQ_INSTS_SALU', 'salu_insts'), ('SQ_WAVES', 'waves'),
                         ('SQ_WAVE_CYCLES', 'wave_cycles'), ('SQ_WAIT_ANY', 'wait_any'),
                         ('SQ_ACTIVE_INST_VALU', 'active_valu')):
            if src in c:
                r[dst] = c[src]
        f64 = [c.get(x) for x in ('SQ_INSTS_VALU_FMA_F64', 'SQ_INSTS_VALU_ADD_F64',
                                  'SQ_INSTS_VALU_MUL_F64', 'SQ_INSTS_VALU_TRANS_F64')]
        if all(v is not None for v in f64):
            r['fp64_flops'] = 64.0 * (2 * f64[0] + f64[1] + f64[2] + f64[3])
        res[name] = r
    # the library these counters belong to: bench.py reports them only for the same build
    meta = {'passes': [os.path.basename(os.path.normpath(d)) for d in dirs]}
    if bench_json:
        with open(bench_json) as f:
            line = [x for x in f if x.startswith('{')][-1]
        b = json.loads(line)['build']
        meta.update(lib_sha256=b['lib_sha256'], lib_path=b['lib_path'], sha_source='profiled bench output')
    else:
        lib = os.environ.get('BSACCEL_LIB') or os.path.join(
            os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'bluesky_amd', 'libbsaccel.so')
        with open(lib, 'rb') as f:
            meta.update(lib_sha256=hashlib.sha256(f.read()).hexdigest(), lib_path=lib, sha_source='hashed file')
    res['_meta'] = meta
    with open(out, 'w') as f:
        json.dump(res, f, indent=1, sort_keys=True)
    for k in ('k_prefilter', 'k_exact', 'k_sim_pilot_kin'):
        if k in res:
            print(k, json.dumps(res[k]))


if __name__ == '__main__':
    main()
