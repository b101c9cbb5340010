"""Prefilter item timeline (diagnostic build `make trace`, libbsaccel_trace.so).

run:     BSACCEL_LIB=.../libbsaccel_trace.so BSA_PF_TRACE_FILE=f python tools/pf_trace.py run WORKLOAD [ROWS_DIV]
         ... pf_trace.py sim WORKLOAD [SETTLE]  (the resident step)
         ... pf_trace.py probe WORKLOAD R RANK [SETTLE]  (one rank's share, probe_step.py)
analyse: python tools/pf_trace.py show f

`run` steps the resident sim (home order) a few times and, with ROWS_DIV = R,
also detects rank 0's home slice of R ranks; every detect appends one record
set.  `show` prints, per detect: the kernel span (first item start -> last
item end), the item-duration distribution, when the waves ran dry (the tail),
and the busiest waves."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run_sim(name, steps):
    """The resident step itself (the bench's detects: HK, the kept list, the
    listed longest items): one record set per batch -- its last prefilter."""
    from bluesky_amd import _lib, resident, synth
    t = synth.workload(name)
    ctx = _lib.Context(0)
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx)
    path = os.environ.pop('BSA_PF_TRACE_FILE')
    sim.step(1)
    sim.step(steps)   # settle: the list and its listed items in steady state
    os.environ['BSA_PF_TRACE_FILE'] = path
    for _ in range(3):
        sim.step(5)
    ctx.sync()


def run_probe(name, R, rank, steps):
    """One rank's share of the sharded resident step (tools/probe_step.py's
    bsa_sim_probe_rank) in steady state: its last prefilter of 3 batches."""
    from bluesky_amd import _lib, resident, synth
    t = synth.workload(name)
    ctx = _lib.Context(0)
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx)
    path = os.environ.pop('BSA_PF_TRACE_FILE')
    ctx.sim_probe_rank(rank, R)
    sim.step(5)
    sim.step(steps)
    ctx.sync()
    os.environ['BSA_PF_TRACE_FILE'] = path
    for _ in range(3):
        sim.step(5)
    ctx.sync()
    ctx.sim_probe_rank(0, 1)


def run(name, div, rank=0):
    from bluesky_amd import _lib, resident, synth
    t = synth.workload(name)
    ctx = _lib.Context(0)
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx)
    sim.step(3)
    n = t.ntraf
    rpr = ((n + div - 1) // div + 511) // 512 * 512
    for _ in range(2):
        ctx.sim_detect_rows(rank * rpr, min(n, (rank + 1) * rpr))
    ctx.sync()


def show(fn):
    raw = np.fromfile(fn, dtype=np.uint64)
    k = 0
    det = 0
    while k < len(raw):
        assert raw[k] == 0xfeed
        m, groups, tiles = int(raw[k + 1]), int(raw[k + 2]), int(raw[k + 3])
        rec = raw[k + 4:k + 4 + 4 * m].reshape(m, 4)
        k += 4 + 4 * m
        rec = rec[rec[:, 3] > 0]
        t0 = rec[:, 2].min()
        st = (rec[:, 2] - t0) / 100.0     # us (100 MHz)
        en = (rec[:, 3] - t0) / 100.0
        dur = en - st
        subs = (rec[:, 1] & 0xff).astype(np.int64)
        wave = (rec[:, 1] >> 8).astype(np.int64)
        span = en.max()
        print('detect %d: %d items (%d with work), groups %d, tiles %d, span %.1f us' %
              (det, len(rec), int((subs > 0).sum()), groups, tiles, span))
        q = np.percentile(dur, [50, 90, 99, 100])
        print('  item us  p50 %.2f p90 %.2f p99 %.2f max %.2f   (sub-groups of the max item: %d)' %
              (q[0], q[1], q[2], q[3], subs[np.argmax(dur)]))
        # per wave: busy time and last end
        uw, inv = np.unique(wave, return_inverse=True)
        busy = np.bincount(inv, weights=dur)
        last = np.zeros(len(uw))
        np.maximum.at(last, inv, en)
        print('  waves %d: busy us p50 %.1f max %.1f; last end p10 %.1f p50 %.1f p90 %.1f max %.1f' %
              (len(uw), np.median(busy), busy.max(), *np.percentile(last, [10, 50, 90, 100])))
        for frac in (0.5, 0.9, 0.99):
            print('  %.0f%% of item-time done by %.1f us' %
                  (frac * 100, np.interp(frac, np.cumsum(np.sort(dur)[::-1]) / dur.sum(), np.sort(en)) if False else
                   en[np.argsort(en)][np.searchsorted(np.cumsum(dur[np.argsort(en)]) / dur.sum(), frac)]))
        listed = (rec[:, 0] >> np.uint64(63)).astype(bool)
        work_all = subs > 0
        npc = ((rec[:, 0] >> np.uint64(48)) & np.uint64(0x7fff)).astype(np.int64)
        if listed.any():
            print('  listed units %d (pieces %s): max %.1f us; unlisted max %.1f us (sub-groups %d, pieces %d)' %
                  (listed.sum(), np.unique(npc[listed]).tolist(), dur[listed].max(), dur[~listed].max(),
                   subs[~listed][np.argmax(dur[~listed])], npc[~listed][np.argmax(dur[~listed])]))
            for pc in np.unique(npc[listed]).tolist():
                sel = listed & (npc == pc) & work_all
                if sel.any():
                    print('    listed with %d piece(s): %d units, us p50 %.1f max %.1f, sub-groups p50 %d max %d, '
                          'start p90 %.1f' % (pc, sel.sum(), np.median(dur[sel]), dur[sel].max(),
                                              int(np.median(subs[sel])), int(subs[sel].max()),
                                              np.percentile(st[sel], 90)))
            long = dur > 0.6 * dur.max()
            print('  units above 60%% of the max: %d, listed %d; (pieces, sub-groups, us) of the 6 longest: %s' %
                  (long.sum(), (long & listed).sum(),
                   [(int(npc[i]), int(subs[i]), round(float(dur[i]), 1)) for i in np.argsort(-dur)[:6]]))
        else:
            print('  no listed units')
        starts = np.sort(st)
        print('  item starts: first %.1f, 50%% by %.1f, last %.1f us' % (starts[0], starts[len(starts) // 2], starts[-1]))
        work = subs > 0
        edges = np.arange(0.0, span + 5.0, 5.0)
        print('  units with work in flight per 5 us: %s' % [int(((st < e + 5) & (en > e) & work).sum()) for e in edges])
        p90 = np.percentile(last, 90)
        tl = (en > p90) & work
        if tl.any():
            print('  tail (units ending after the p90 wave end, %.1f us): %d, listed %d; start p10/p50/p90 %s; '
                  'us p50 %.1f max %.1f; sub-groups p50 %d max %d' %
                  (p90, tl.sum(), (tl & listed).sum(), np.round(np.percentile(st[tl], [10, 50, 90]), 1).tolist(),
                   np.median(dur[tl]), dur[tl].max(), int(np.median(subs[tl])), int(subs[tl].max())))
        det += 1


if __name__ == '__main__':
    if sys.argv[1] == 'sim':
        run_sim(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 300)
    elif sys.argv[1] == 'probe':
        run_probe(sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]) if len(sys.argv) > 5 else 200)
    elif sys.argv[1] == 'run':
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 1, int(sys.argv[4]) if len(sys.argv) > 4 else 0)
    else:
        show(sys.argv[2])
