"""Full-size oracle fixture of BASELINE configs[3]: the
oracle's StateBasedCD.detect (oracle/statebased.py, pinned bitwise to the
reference by tests/test_oracle_golden.py) over EVERY row of the synthetic
box100k workload (bluesky_amd.synth, seed 7) against all 100k columns --
1e10 pair evaluations, row chunks spread over worker processes on the CPU of
this container (~4 min on 8 cores) -- written as tests/golden/full_box100k.npz:
the conflict pairs (ci, cj) with qdr, dist, tcpa, tinconf, dcpa, the LoS pairs
(li, lj), inconf (bit-packed) and tcpamax of the rows in conflict, plus a
sha256 of the input arrays so the GPU test can check it detects the same
traffic.  tests/test_gpu_fullsize.py compares the HIP detect with it pair for
pair.  Test infrastructure only.

Usage: python tools/make_fullrows.py [workers]"""
import hashlib
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

from bluesky_amd import synth  # noqa: E402
from oracle import statebased as ocd  # noqa: E402

FIELDS = ('lat', 'lon', 'trk', 'gs', 'alt', 'vs')
_T = None


def state_sha(t):
    h = hashlib.sha256()
    for f in FIELDS:
        h.update(np.ascontiguousarray(getattr(t, f), dtype=np.float64).tobytes())
    return h.hexdigest()


def _init():
    global _T
    _T = synth.workload('box100k')


def _rows(span):
    a, b = span
    return ocd.detect_arrays(_T, _T, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, want_dcpa=True,
                             rows=np.arange(a, b), budget_bytes=1 << 30)


def main():
    workers = int(sys.argv[1]) if len(sys.argv) > 1 else min(8, os.cpu_count() or 1)
    t = synth.workload('box100k')
    n = t.ntraf
    spans = [(a, min(n, a + 500)) for a in range(0, n, 500)]
    t0 = time.time()
    with Pool(workers, initializer=_init) as pool:
        parts = []
        for k, p in enumerate(pool.imap(_rows, spans)):
            parts.append(p)
            if k % 20 == 0:
                print('%d / %d row chunks, %.0f s' % (k + 1, len(spans), time.time() - t0), flush=True)
    r = {key: np.concatenate([p[key] for p in parts]) for key in parts[0]}
    inconf = r['inconf'].astype(bool)
    out = dict(ci=r['ci'].astype(np.int32), cj=r['cj'].astype(np.int32),
               li=r['li'].astype(np.int32), lj=r['lj'].astype(np.int32),
               qdr=r['qdr'], dist=r['dist'], tcpa=r['tcpa'], tinconf=r['tinconf'], dcpa=r['dcpa'],
               inconf_bits=np.packbits(inconf), tcpamax_inconf=r['tcpamax'][inconf],
               n=np.int64(n), state_sha256=np.array(state_sha(t)),
               rpz=np.float64(synth.RPZ), hpz=np.float64(synth.HPZ), tla=np.float64(synth.TLOOKAHEAD))
    path = os.path.join(REPO, 'tests', 'golden', 'full_box100k.npz')
    np.savez_compressed(path, **out)
    print('%s: %d conflict pairs, %d LoS pairs, %d rows in conflict, %.0f s, %.1f MB'
          % (path, len(out['ci']), len(out['li']), int(inconf.sum()), time.time() - t0,
             os.path.getsize(path) / 1e6))


if __name__ == '__main__':
    main()
