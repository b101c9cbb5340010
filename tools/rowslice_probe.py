"""Per-rank detect cost of a row-sharded CD step, probed on one GPU: the stage
times of the resident sim's detect of each rank's home rows (a 512-aligned,
spatially compact slice, bsa_sim_detect_rows) as that rank computes it -- its
own column tiles, the halo plan and the halo tiles it would receive
 -- for R = 1, 2, 4, 8, on the box100k and global1m workloads.
Reports the slowest rank's stages (the step waits for it) and the largest
halo (tiles a rank receives; bytes at 6 fp64 arrays x 512 rows per tile).
Before each rank's detects the device runs BSA_SETTLE (200) untimed sim steps,
so the stage events see it at steady clocks (bench.py's --settle).
Usage: python tools/rowslice_probe.py [workload ...]"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bluesky_amd import _lib, resident, synth  # noqa: E402


def main():
    names = sys.argv[1:] or ['box100k', 'global1m']
    settle = int(os.environ.get('BSA_SETTLE', '200'))
    ctx = _lib.Context(0)
    ctx.set_timing_sample(1)
    for name in names:
        t = synth.workload(name)
        n = t.ntraf
        sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx)
        for R in (1, 2, 4, 8):
            rpr = ((n + R - 1) // R + 511) // 512 * 512
            worst, max_halo, per_rank = None, 0, []
            for r in range(R):
                rb, re = min(n, r * rpr), min(n, (r + 1) * rpr)
                if re <= rb:
                    continue
                if settle > 0:
                    sim.step(settle)
                for _ in range(2):
                    ctx.sim_detect_rows(rb, re)
                ctx.timing_reset()
                for _ in range(6):
                    ctx.sim_detect_rows(rb, re)
                tm, ts = ctx.timing_summary()
                d = max(ts['detects'], 1)
                halo = ctx.sim_halo_stats()['tiles'] if R > 1 else 0
                row = dict(rank=r, rows=re - rb, ms={k: round(v, 4) for k, v in tm.items()},
                           tiles=ts['tiles'] / d, groups=ts['groups'] / d, candidates=ts['candidates'] / d,
                           halo_tiles=halo, halo_MB=halo * 6 * 512 * 8 / 1e6)
                per_rank.append(round(tm['total'], 4))
                if worst is None or tm['total'] > worst['ms']['total']:
                    worst = row
                max_halo = max(max_halo, halo)
            print(name, 'R=%d' % R, json.dumps(worst), 'max halo tiles %d (%.2f MB)'
                  % (max_halo, max_halo * 6 * 512 * 8 / 1e6), 'per-rank total ms %s' % per_rank, flush=True)


if __name__ == '__main__':
    main()
