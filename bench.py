#!/usr/bin/env python3
"""bench.py -- BASELINE.json metric on MI355X:
"CD pair-evals/sec + sim-steps/sec at 100k aircraft; 1/2/4/8 MI355X".

Contract (driver): ``python bench.py --gpus N --steps K --warmup W`` prints ONE
JSON line on rank 0; for N > 1 it is launched by ``torch.distributed.run``
(one process per GPU; RANK / LOCAL_RANK / WORLD_SIZE from the env).

A step = one GPU-resident sim step of the synthetic 100k-aircraft
density-matched box (BASELINE.json configs[3]) with ASAS every
step: [RCCL halo exchange of the column tiles the rank's rows can reach] ->
StateBased detect of the rank's ownship rows against all N intruders -> MVP ->
pilot select + kinematics.  Inputs are
resident in HBM before the timed region.  Each step evaluates all N^2 pairs
(diagonal included), so value = N^2 * K / time (whole job, all ranks);
sim-steps/s = K / time.  Rows are partitioned, total work is fixed:
scaling "strong".
"""
import argparse
import json
import os
import platform
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

from bluesky_amd import _lib, dist, resident, synth  # noqa: E402

FP64_PEAK_TFLOPS = 78.6      # MI355X fp64 vector (spec, FMA = 2 flops)
FP32_PEAK_TFLOPS = 157.3     # MI355X fp32 vector (MI355X_MICROARCH.md)
OPS_PER_PAIR = 110           # algorithmic fp64 ops per pair-eval
PF_FLOPS_PER_PAIR = 9        # prefilter stage-1 fp32 flops per tested pair:
                             # acc = K + k (1) + 3 FMA (6); lo - hi, hi - lo (2)
KIN_BYTES_PER_AC = 234       # K4 algorithmic HBM bytes per aircraft-step
PREP_BYTES_PER_AC = 32 + 16 + 16 + 48 / 8 + 48 / 64   # K4' also writing the next detect's column
                             # records (PFRec, PFVel, position) and sub-group / group boxes (one rank,
                             # DESIGN.md 3.7) ...
PREP_REC_BYTES = 128         # ... plus the 128-B fp64 record when the library stores it (home_records:
                             # rows <= 163840 unless BSA_HOME_REC overrides, bsa_cd.hip)


def prep_bytes_per_ac(n):
    """K4''s next-detect bytes per aircraft for a one-rank sim of n aircraft."""
    env = os.environ.get('BSA_HOME_REC')
    rec = (env == '1') if env in ('0', '1') else n <= 163840
    return PREP_BYTES_PER_AC + (PREP_REC_BYTES if rec else 0)
HBM_PEAK_GBPS = 8000.0       # MI355X HBM3E (spec)
PMC_JSON = os.path.join(REPO, 'profiles', 'pmc_latest.json')
PMC_K24OFF_JSON = os.path.join(REPO, 'profiles', 'pmc_k24off.json')   # the same passes with BSA_K24=0
TIMING_SAMPLE = 20           # detects per HIP-event-timed detect in the warm-up and the secondary lines
                             # (bsa_set_timing_sample; each timed one costs ~24 us of event bubbles,
                             # profiles/r02 kernel trace); the headline batch times ONE detect, its first
                             # (the stage times the roofline uses; ~0.4 us per step at 60 steps)


def pmc_figures(lib_sha, path=PMC_JSON):
    """Per-launch memory-side bytes etc. from the committed rocprofv3 --pmc
    passes of this bench (tools/pmc_roofline.py) -- only if they were taken on
    THE build of libbsaccel this process mapped (the sha256 pmc_roofline.py
    took from the profiled bench's own output); else {}."""
    try:
        with open(path) as f:
            pmc = json.load(f)
    except (OSError, ValueError):
        return {}
    return pmc if pmc.get('_meta', {}).get('lib_sha256') == lib_sha else {}


def cpu_model():
    try:
        with open('/proc/cpuinfo') as f:
            for line in f:
                if line.startswith('model name'):
                    return line.split(':', 1)[1].strip()
    except OSError:
        pass
    return platform.processor() or 'unknown'


def cpu_baseline(t, rows_sample):
    """Oracle (numpy restatement of StateBasedCD.detect, pinned to the
    reference) in this one process on a uniform ownship-row sample, extrapolated
    by N / R (every row scans all N columns).  numpy ufuncs are
    single-threaded; OpenBLAS only serves the k = 1 outer products."""
    from oracle import statebased as ocd
    n = t.ntraf
    rows = np.linspace(0, n - 1, rows_sample).astype(np.int64)
    t0 = time.perf_counter()
    ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, rows=rows, budget_bytes=1 << 30)
    dt = time.perf_counter() - t0
    return dict(value=rows_sample * n / dt, unit='pair-evals/s', cores=1, kind='port',
                detect_s_extrapolated=dt * n / rows_sample,
                sample='oracle detect of %d uniformly spaced ownship rows x %d columns (%.1f s), '
                       'extrapolated by N/R; numpy %s, one process (single-threaded ufuncs), '
                       'OPENBLAS_NUM_THREADS=%s, nproc=%d'
                       % (rows_sample, n, dt, np.__version__,
                          os.environ.get('OPENBLAS_NUM_THREADS', 'unset'), os.cpu_count()),
                cpu_model=cpu_model())


def dropin_detect_line(ctx, t, reps=3):
    """The north-star target is stated on the drop-in ``detect()``: the whole
    StateBasedCD.detect replacement at 100k (host arrays in, the 8-tuple with
    Python id tuples out), wall time per component (SURVEY.md 7 iii): H2D of the
    six state arrays, the detect up to completion, D2H of the results, building
    the confpairs / lospairs lists.  Median of ``reps`` after one warm-up."""
    from bluesky_amd import statebased
    tt = []
    for k in range(reps + 1):
        tm = {}
        res = statebased.detect(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, timings=tm, ctx=ctx)
        if k:
            tt.append(tm)
    med = {key: float(np.median([x[key] for x in tt])) * 1e3 for key in tt[0]}
    return dict(n=t.ntraf, ms=med, n_conf=len(res[0]), n_los=len(res[1]),
                note='wall time of bluesky_amd.statebased.detect (ctypes -> libbsaccel); '
                     'h2d / detect / d2h / tuples / total in ms, median of %d' % reps)


def asas_update_line(ctx, t, calls=6):
    """the user-facing ``ASAS.update`` drop-in
    (bluesky_amd.asas.DeviceASAS.update, asas.py:473-504) at 100k, history off,
    MVP: wall time per phase of one call -- upload of the host simulator's
    traffic (bsa_sim_update), the device CD call (detect + MVP + resopairs +
    ResumeNav + unique / cumulative counts, bsa_sim_cd), the pair lists and
    per-row outputs (bsa_fetch_pairs), the ASAS outputs and counts -- median of
    ``calls`` after the first (which initialises the device sim).  Between
    calls the host traffic moves by one 1 s step (positions along the track),
    as BlueSky's own kinematics would have moved it."""
    import types
    from bluesky_amd import asas as gasas, mvp, statebased
    n = t.ntraf
    st = resident.initial_state(t)
    traf = types.SimpleNamespace(id=['AC%d' % k for k in range(n)], ntraf=n)
    for k in ('lat', 'lon', 'trk', 'gs', 'alt', 'vs', 'tas', 'hdg', 'gseast', 'gsnorth', 'selalt'):
        setattr(traf, k, np.array(st[k]))
    traf.ap = types.SimpleNamespace(trk=st['ap_trk'].copy(), tas=st['ap_tas'].copy(), alt=st['ap_alt'].copy(),
                                    vs=st['ap_vs'].copy())
    a = types.SimpleNamespace(swasas=True, tasas=0.0, dtasas=1.0, asaseval=False, noresolst=[], resoofflst=[],
                              swnoreso=False, swresooff=False, priocode='FF1', R=synth.RPZ, dh=synth.HPZ,
                              dtlookahead=synth.TLOOKAHEAD, Rm=synth.RPZ * 1.05, dhm=synth.HPZ * 1.05,
                              vmin=200.0 * 1852 / 3600., vmax=500.0 * 1852 / 3600., vsmin=-3000. / 60. * 0.3048,
                              vsmax=3000. / 60. * 0.3048, swresohoriz=True, swresospd=False, swresohdg=False,
                              swresovert=False, swprio=False, resopairs=set(), confpairs_all=[], lospairs_all=[],
                              cd=statebased, cr=mvp, alt=np.array(st['asas_alt']))
    dev = gasas.install(a, traf, ctx=ctx)
    tt = []
    for k in range(calls + 1):
        dev.update(float(k))
        if k:
            tt.append(dev.timings)
        dn = traf.gsnorth / 6371000.0 * 57.29577951308232
        traf.lat = traf.lat + dn
        traf.lon = traf.lon + traf.gseast / (6371000.0 * np.cos(np.radians(traf.lat))) * 57.29577951308232
    med = {key: float(np.median([x[key] for x in tt])) * 1e3 for key in tt[0]}
    return dict(n=n, ms=med, n_conf=len(a.confpairs), n_los=len(a.lospairs), resopairs=len(a.resopairs),
                confpairs_all=len(a.confpairs_all),
                note='wall time of bluesky_amd.asas.DeviceASAS.update (ASAS.update drop-in, MVP, resume_nav, '
                     'history off); upload / cd / pairs / asas_outputs / waypoints / total in ms, median of %d'
                     % calls)


def global1m_line(ctx, rank, world, warmup=2, steps=5):
    """BASELINE configs[4]: 1M aircraft uniform on the globe (|lat| <= 70 deg),
    the resident step (ASAS every step) row-sharded over the ranks -- the base
    of the 1 -> 8 GPU curve the north star asks for (>= 6x at 1M) -- plus one
    standalone whole-set detect's stage times (rank 0's rows only with several
    ranks)."""
    t = synth.workload('global1m')
    n = t.ntraf
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx,
                               rank=rank, world=world)
    dt = timed_steps(ctx, sim, warmup, steps)
    tm, ts = ctx.timing_summary()
    st = sim.stats()
    counts = ctx.allreduce_sum([st['n_conf'], st['n_los']])
    halo = halo_line(ctx, sim) if world > 1 else None
    return dict(workload='global1m N=%d (seed 7)' % n, halo=halo, steps=steps, ms_per_step=dt / steps * 1e3,
                sim_steps_per_s=steps / dt, pair_evals_per_s=float(n) * n * steps / dt,
                n_conf=int(counts[0]), n_los=int(counts[1]),
                kernels_ms_rank0=dict(k0_prep=tm['prep'], prefilter=tm['prefilter'], exact=tm['exact'],
                                      k2_sort=tm['sort'], detect_total=tm['total']),
                candidates_rank0=ts['candidates'] / max(ts['detects'], 1))


def halo_line(ctx, sim, cd_steps=None):
    """Bytes each rank exchanged per CD call (max over ranks; collective), and
    the stream-ordered collectives of the timed region per CD step (calls and
    payload bytes, max over ranks: bsa_sim_comm_stats)."""
    h = sim.halo_stats()
    cs = ctx.sim_comm_stats()
    mx = ctx.allreduce_max([h['rx_bytes'], h['tx_bytes'], h['tiles'], h['regrowths'], cs['calls'],
                            cs['tx_bytes'], cs['rx_bytes']])
    tot = ctx.allreduce_sum([h['rx_bytes']])
    out = dict(rx_bytes_per_cd_max_rank=int(mx[0]), tx_bytes_per_cd_max_rank=int(mx[1]),
               rx_bytes_per_cd_all_ranks=int(tot[0]), tiles_received_max_rank=int(mx[2]),
               regrowths=int(mx[3]),
               note='halo exchange (grouped RCCL send/recv of the column tiles a rank\'s rows can reach) '
                    'instead of the full-state all-gather; 512 aircraft x 6 or 8 fp64 per tile')
    if cd_steps:
        out['collectives_per_cd_step'] = dict(
            calls=mx[4] / cd_steps, tx_bytes_max_rank=mx[5] / cd_steps, rx_bytes_max_rank=mx[6] / cd_steps,
            note='box all-gather + grouped halo send/recv + 16-B gate all-reduce per CD step (RCCL over xGMI)')
    return out


PARITY_PAIR_KEYS = ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'li', 'lj', 'inconf', 'tcpamax')


def parity_vs_world1(ctx, init, p, rank, world, device, steps=2, group=None):
    """the first multi-GPU run checks itself.  Every rank
    runs ``steps`` steps of the sharded sim (halo exchange over RCCL, or the
    in-process group in tests); the state is all-gathered and the last CD
    call's pairs are gathered to rank 0 (C2), which runs the same steps at
    world 1 in a second context on its own GPU and compares both BITWISE
    (every state array's bytes, every pair array).  Collective: every rank
    learns the verdict (all-reduce), so a divergence stops every rank."""
    import hashlib
    sim = resident.ResidentSim(init, p, ctx=ctx, rank=rank, world=world, group=group)
    sim.step(steps)
    got = sim.read()                       # collective: the all-gathered state
    gp = sim.gather_pairs(root=0)          # collective: rank-order pair blocks on rank 0
    bad = []
    out = dict(steps=steps, world=world)
    if rank == 0:
        c1 = _lib.Context(device)
        try:
            ref = resident.ResidentSim(init, p, ctx=c1)
            ref.step(steps)
            exp, st = ref.read(), ref.stats()
            ep = c1.fetch_pairs(st['n_conf'], st['n_los'])
        finally:
            c1.close()
        bad = [k for k in sorted(exp) if np.asarray(got[k]).tobytes() != np.asarray(exp[k]).tobytes()]
        bad += ['pairs.' + k for k in PARITY_PAIR_KEYS if np.asarray(gp[k]).tobytes() != np.asarray(ep[k]).tobytes()]
        h = hashlib.sha256()
        for k in sorted(got):
            h.update(np.ascontiguousarray(got[k]).tobytes())
        out.update(state_sha256=h.hexdigest(), n_conf=len(ep['ci']), n_los=len(ep['li']), mismatched=bad)
    flag = ctx.allreduce_max([1.0 if bad else 0.0])
    out['ok'] = bool(flag[0] == 0.0)
    return out


def timed_steps(ctx, sim, warmup, steps):
    """Run warmup + steps resident sim steps; the timed batch's wall time, max over ranks."""
    sim.step(warmup)
    ctx.allreduce_max([0.0])
    ctx.sync()
    ctx.timing_reset()
    t0 = time.perf_counter()
    sim.step(steps)
    ctx.sync()
    ctx.allreduce_max([0.0])
    return float(ctx.allreduce_max([time.perf_counter() - t0])[0])


def variants(ctx, t, rank, world, warmup):
    """Secondary lines on the same workload (not the headline value):
    - reference_cadence: CD + MVP every 20th step (asas_dt 1 s / simdt 0.05 s,
      SURVEY.md 8d), kinematics every step;
    - candidate_reuse: ASAS every step with the candidate list kept across
      detects under per-aircraft drift budgets (bitwise equal
      results, tests/test_gpu_reuse.py)."""
    n = t.ntraf
    out = {}
    steps = 40
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=20), ctx=ctx,
                               rank=rank, world=world)
    dt = timed_steps(ctx, sim, warmup, steps)
    out['reference_cadence'] = dict(cd_every=20, steps=steps, ms_per_step=dt / steps * 1e3,
                                    sim_steps_per_s=steps / dt)
    sh, sv = 1500.0, 300.0
    ctx.set_candidate_reuse(True, sh, sv)
    try:
        sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=1), ctx=ctx,
                                   rank=rank, world=world)
        dt = timed_steps(ctx, sim, warmup, steps)
        out['candidate_reuse'] = dict(sigma_h_m=sh, sigma_v_m=sv, steps=steps, ms_per_step=dt / steps * 1e3,
                                      sim_steps_per_s=steps / dt, pair_evals_per_s=float(n) * n * steps / dt,
                                      **ctx.reuse_stats())
    finally:
        ctx.set_candidate_reuse(False, sh, sv)
    return out


def geo_matrix_line(ctx, t, m=8192):
    """Secondary line: the standalone qdrdist_matrix / kwikqdrdist_matrix
    producers (bsa_qdrdist) on an m x m same-set matrix of the
    workload's first m aircraft.  HBM-write-bound: 16 B algorithmic bytes per
    entry (qdr + dist fp64; the 2 x 8 B point vectors are L2-resident), timed
    with HIP events around the producing kernel alone (the PCIe copy of the
    result to the host is not part of it)."""
    out = {}
    lat, lon = t.lat[:m], t.lon[:m]
    for name, kwik in (('qdrdist_matrix', False), ('kwikqdrdist_matrix', True)):
        ms = []
        for _ in range(3):
            ctx.qdrdist(lat, lon, lat, lon, kwik=kwik)
            ms.append(ctx.geo_last_ms())
        best = min(ms)
        gbps = 16.0 * m * m / (best * 1e-3) / 1e9
        out[name] = dict(m=m, n=m, kernel_ms=best, entries_per_s=m * m / (best * 1e-3),
                         algorithmic_bytes=16 * m * m, achieved_GBps=gbps, peak_GBps=HBM_PEAK_GBPS,
                         frac=gbps / HBM_PEAK_GBPS)
    return out


def spawn_ranks(n, argv, cmd=None):
    """``bench.py --gpus N`` (N > 1) started without torch.distributed.run
    starts its N ranks itself: N fresh child processes, one per GPU, with RANK /
    LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment.  This process has
    not touched HIP (the library loads lazily, _lib.load), and the children are
    started, never exec'd into.  Rank 0's JSON line reaches stdout through the
    inherited descriptor; the exit code is the first failing rank's, and a
    failing rank ends the others (they would wait in a collective forever)."""
    import subprocess
    base = dict(os.environ, WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), MASTER_ADDR='127.0.0.1',
                MASTER_PORT=os.environ.get('MASTER_PORT', str(29500 + os.getpid() % 1000)),
                TORCHELASTIC_RUN_ID='bench%d' % os.getpid())   # the RCCL id file's key (dist._rdv_path)
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + list(argv)
    procs = [subprocess.Popen(cmd, env=dict(base, RANK=str(r), LOCAL_RANK=str(r))) for r in range(n)]
    rc = 0
    try:
        while None in [p.poll() for p in procs]:   # (a list: every child is polled)
            bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
            if bad:
                rc = bad[0]
                break
            time.sleep(0.1)
    finally:
        for p in procs:
            if p.poll() is None:
                p.terminate()
        for p in procs:
            try:
                p.wait(timeout=30)
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc or next((p.returncode for p in procs if p.returncode), 0)


def resolve_world(gpus):
    """(rank, world, local) of this process, or ('spawn', n) when this process
    must start the ranks itself; a launcher world that disagrees with --gpus
    is an error (a silent world-1 line for --gpus 8 would mislabel the run)."""
    if 'WORLD_SIZE' not in os.environ:
        if gpus > 1:
            return 'spawn', gpus
        return dist.env_rank_world()
    rank, world, local = dist.env_rank_world()
    if world != gpus:
        raise SystemExit('bench.py: WORLD_SIZE=%d from the launcher but --gpus %d; refusing to run'
                         % (world, gpus))
    return rank, world, local


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=60)
    ap.add_argument('--warmup', type=int, default=10)
    ap.add_argument('--settle', type=int, default=300,
                    help='untimed steps before the W warm-up steps, so the timed batch sees the GPU at its '
                         'steady clocks (DESIGN.md 5: a cold device is ~15%% slower over its first ~25 ms)')
    ap.add_argument('--n', type=int, default=100000)
    ap.add_argument('--workload', default='box100k', choices=['box10k', 'box100k', 'global1m'])
    ap.add_argument('--cd-every', type=int, default=1)
    ap.add_argument('--cpu-rows', type=int, default=1024)
    ap.add_argument('--no-cpu', action='store_true')
    ap.add_argument('--reuse', type=float, nargs=2, default=None, metavar=('SIGMA_H', 'SIGMA_V'),
                    help='candidate-list reuse budgets [m] (bsa_set_candidate_reuse); default off')
    ap.add_argument('--no-variants', action='store_true',
                    help='skip the secondary lines (reference CD cadence, candidate-list reuse)')
    ap.add_argument('--parity-steps', type=int, default=2,
                    help='with several GPUs: steps of the sharded run checked bitwise against one GPU first '
                         '(0: skip)')
    ap.add_argument('--dry-run', action='store_true',
                    help='resolve the ranks (spawning them if needed), report them, touch no GPU (launcher test)')
    args = ap.parse_args()

    rw = resolve_world(args.gpus)
    if rw[0] == 'spawn':
        sys.exit(spawn_ranks(rw[1], sys.argv[1:]))
    rank, world, local = rw
    if args.dry_run:
        print('bench.py dry run: rank %d of %d (local %d)' % (rank, world, local), file=sys.stderr, flush=True)
        if rank == 0:
            print(json.dumps(dict(dry_run=True, n_gpus=world, rank=rank)), flush=True)
        return
    ctx = _lib.Context(local)
    # HIP-event stage timing of one detect in TIMING_SAMPLE, inside the timed
    # region (each event record leaves a ~5 us gap before the next kernel)
    ctx.set_timing_sample(TIMING_SAMPLE)
    if args.reuse:
        ctx.set_candidate_reuse(True, args.reuse[0], args.reuse[1])
    t = synth.workload(args.workload, n=args.n, seed=7)
    n = t.ntraf
    parity = None
    if world > 1 and args.parity_steps > 0:   # the sharded step equals one GPU's, bitwise, or nothing is timed
        parity = parity_vs_world1(ctx, resident.initial_state(t), resident.params(cd_every=args.cd_every),
                                  rank, world, local, steps=args.parity_steps)
        if not parity['ok']:
            if rank == 0:
                print(json.dumps(dict(metric='CD pair-evals/s at 100k aircraft (GPU-resident sim step, ASAS every '
                                             'step)', value=None, n_gpus=world, parity_vs_world1=False,
                                      parity=parity, error='sharded run differs from one GPU')), flush=True)
            sys.exit(3)
    sim = resident.ResidentSim(resident.initial_state(t), resident.params(cd_every=args.cd_every),
                               ctx=ctx, rank=rank, world=world)
    comm = (ctx.comm_info() if hasattr(ctx.lib, 'bsa_comm_info') else   # with RCCL: ncclCommCount /
            dict(transport='unknown (older build, BSACCEL_AB=1)', ranks=world, rank=rank, device=local))
    # ncclCommUserRank / ncclCommCuDevice
    if world > 1 and (comm['transport'] != 'rccl' or comm['ranks'] != world or comm['rank'] != rank):
        raise SystemExit('bench.py: rank %d of %d but the communicator reports %s' % (rank, world, comm))

    if args.settle > 0:         # same count on every rank (the halo step exchanges)
        sim.step(1)              # the first batch grows the candidate buffers and re-runs: keep it short
        sim.step(args.settle - 1)
        ctx.sync()
    sim.step(args.warmup)
    ctx.allreduce_max([0.0])     # barrier
    ctx.sync()
    ctx.timing_reset()
    ctx.set_timing_sample(max(args.steps, 1))   # the timed batch's first detect carries the stage events
    tr0 = ctx.tile_reuse_stats()
    t0 = time.perf_counter()
    sim.step(args.steps)         # one batch: no host synchronisation between steps
    ctx.sync()
    ctx.allreduce_max([0.0])     # barrier
    dt_local = time.perf_counter() - t0
    dt = float(ctx.allreduce_max([dt_local])[0])   # max over ranks
    tm, ts = ctx.timing_summary()
    ctx.set_timing_sample(TIMING_SAMPLE)
    st = sim.stats()
    counts = ctx.allreduce_sum([st['n_conf'], st['n_los'], ts['candidates'] / max(ts['detects'], 1)])
    tr = ctx.tile_reuse_stats()   # tile-pair list (K0d) builds / detects of this run
    tile_reuse = dict(builds=tr['builds'] - tr0['builds'], detects=tr['detects'] - tr0['detects'],
                      note='K0d tile-pair list rebuilt on the device when a record left its drift budget')

    k0 = max(args.settle, 0) + args.warmup   # sim step index of the timed batch's first step
    cd_steps = sum(1 for k in range(k0, k0 + args.steps) if k % args.cd_every == 0)
    pairs = float(n) * n * cd_steps
    value = pairs / dt
    pf_s = tm['prefilter'] * 1e-3
    tested = ts['groups'] / max(ts['detects'], 1) * _lib.PF_BLOCK_PAIRS    # pair tests the prefilter executed
    lib_path, lib_sha = _lib.mapped_library()
    pmc = pmc_figures(lib_sha)
    prov = dict(file=os.path.relpath(PMC_JSON, REPO), lib_sha256=lib_sha,
                passes=pmc.get('_meta', {}).get('passes')) if pmc else None
    pf = pmc.get('k_prefilter', {})
    fused = ctx.exact_fusion_stats()['last']   # K1b ran inside the prefilter's launch
    stage1 = tested * PF_FLOPS_PER_PAIR
    # fused: the launch also does K1b's fp64 work (PMC SQ_INSTS_VALU_*_F64 of the
    # fused kernel -- the sweep itself is fp32); weighted by the fp32 / fp64 peak
    # ratio, both kinds of work count as time at the vector peak
    ex64 = pf.get('fp64_flops') if fused else None
    n_exact = ts['candidates'] / max(ts['detects'], 1)      # K1b evaluates every candidate pair exactly
    w64 = FP32_PEAK_TFLOPS / FP64_PEAK_TFLOPS
    # algorithmic work: 9 fp32 flops per stage-1 test; fused, also
    # 110 fp64 ops per exact evaluation -- each kind priced at its own vector
    # peak (fp64 ops x the fp32 / fp64 peak ratio in fp32-equivalent flops)
    alg = stage1 + (n_exact * OPS_PER_PAIR * w64 if fused else 0.0)
    roof = dict(bound='valu', kernel=('k_prefilter with K1b fused (fp32 packed VALU stage-1 test + fp64 exact '
                                      'evaluation, dominant)' if fused else
                                      'k_prefilter (fp32 packed VALU stage-1 test, dominant)'),
                achieved=alg / pf_s / 1e12,
                peak=FP32_PEAK_TFLOPS, unit='TFLOP/s' + (' (fp32-equivalent)' if fused else ''))
    roof['frac'] = roof['achieved'] / roof['peak']
    roof['stage1_TFLOPs'] = stage1 / pf_s / 1e12
    roof['duration_us'] = pf_s * 1e6
    if fused:
        roof['exact_evaluations'] = n_exact
        roof['exact_fp64_flops_pmc'] = ex64
        pmc_ach = (stage1 + ex64 * w64) / pf_s / 1e12 if ex64 else None
        roof['achieved_pmc_flops'] = pmc_ach
        roof['frac_pmc_flops'] = pmc_ach / FP32_PEAK_TFLOPS if pmc_ach else None
        roof['note'] = ('fused launch: achieved = (stage-1 tests x %d fp32 flops + exact evaluations x %d fp64 ops '
                        '(SURVEY 8d) x %.1f) / the launch\'s event-timed duration; *_pmc_flops: the same with the '
                        'PMC-counted fp64 flops of the launch (ocml expansions included) instead of the 110 '
                        'algorithmic ops' % (PF_FLOPS_PER_PAIR, OPS_PER_PAIR, w64))
    roof['traffic'] = (pf['hbm_read_bytes'] + pf['hbm_write_bytes']) if 'hbm_write_bytes' in pf else None
    roof['traffic_source'] = ('rocprofv3 --pmc FETCH_SIZE x2 + WRITE_SIZE per launch, from_profile (the '
                              'committed passes of this bench on this very library)' if pmc else
                              'no PMC summary for this build of libbsaccel.so')
    roof['from_profile'] = prov
    if 'lds_bank_conflict_rate' in pf:
        roof['lds_bank_conflict_rate'] = pf['lds_bank_conflict_rate']
    kin = pmc.get('k_sim_pilot_kin', {})
    kin_kernel, kin_note = 'k_sim_pilot_kin', None
    k24 = world == 1 and os.environ.get('BSA_K24', '1') != '0'   # (K2 fused with K4')
    if not kin.get('dur_ns') and k24 and pmc.get('k_rank_rows', {}).get('dur_ns'):
        # one rank: K4' runs inside K2's launch (k_rank_rows<true>)
        kin = pmc['k_rank_rows']
        kin_kernel = "k_rank_rows<true> (K2 fused with K4')"
        kin_note = ("the launch also places the detect's pairs (K2): the kinematics' bytes over the whole "
                    "launch's duration, a lower bound of K4''s own fraction")
    propagation = None
    if kin.get('dur_ns'):
        nrows_r0 = (n + world - 1) // world
        prep = world == 1 and not args.reuse and os.environ.get('BSA_SIM_PREP', '1') != '0'
        pb = prep_bytes_per_ac(n) if prep else 0
        alg = int((KIN_BYTES_PER_AC + pb) * nrows_r0)
        propagation = dict(kernel=kin_kernel, bound='hbm', algorithmic_bytes=alg, from_profile=prov,
                           bytes_per_aircraft=dict(kinematics=KIN_BYTES_PER_AC, next_detect_records=pb),
                           duration_us_profiled=kin['dur_ns'] * 1e-3,
                           achieved_GBps=alg / kin['dur_ns'], peak_GBps=HBM_PEAK_GBPS,
                           frac=alg / kin['dur_ns'] / HBM_PEAK_GBPS,
                           measured_bytes=(kin.get('hbm_read_bytes', 0) + kin.get('hbm_write_bytes', 0)) or None)
        if kin_note:
            propagation['note'] = kin_note
        # VERDICT r04 missing #3: K4' measured on its own (the same PMC passes
        # with BSA_K24=0, K2 and K4' as two launches; gpu_profile.sh)
        k4 = pmc_figures(lib_sha, PMC_K24OFF_JSON).get('k_sim_pilot_kin', {})
        if k4.get('dur_ns'):
            propagation['unfused'] = dict(
                kernel='k_sim_pilot_kin (BSA_K24=0 passes)', duration_us_profiled=k4['dur_ns'] * 1e-3,
                achieved_GBps=alg / k4['dur_ns'], frac=alg / k4['dur_ns'] / HBM_PEAK_GBPS,
                measured_bytes=(k4.get('hbm_read_bytes', 0) + k4.get('hbm_write_bytes', 0)) or None,
                from_profile=dict(file=os.path.relpath(PMC_K24OFF_JSON, REPO), lib_sha256=lib_sha))
    ex = pmc.get('k_exact', {})
    exact_fp64 = None
    if ex.get('fp64_flops') and not fused:
        exact_fp64 = dict(kernel='k_exact', fp64_flops_per_launch=ex['fp64_flops'], from_profile=prov,
                          achieved_TFLOPs=ex['fp64_flops'] / (tm['exact'] * 1e-3) / 1e12,
                          peak_TFLOPs=FP64_PEAK_TFLOPS)
    out = dict(metric='CD pair-evals/s at 100k aircraft (GPU-resident sim step, ASAS every step)',
               value=value, unit='pair-evals/s', n_gpus=world, steps=args.steps, warmup=args.warmup,
               settle_steps=max(args.settle, 0),
               ms_per_step=dt / args.steps * 1e3, higher_is_better=True, scaling='strong',
               vs_baseline=None, dtype='f64', data='synthetic',
               config=dict(workload='%s N=%d (seed 7, density-matched box)' % (args.workload, n),
                           step='detect+MVP+pilot+kinematics, cd_every=%d' % args.cd_every,
                           rpz_m=synth.RPZ, hpz_m=synth.HPZ, tlookahead_s=synth.TLOOKAHEAD,
                           simdt_s=0.05, parallelism='rows%d' % world),
               sim_steps_per_s=args.steps / dt,
               reuse=(dict(sigma_h_m=args.reuse[0], sigma_v_m=args.reuse[1], **ctx.reuse_stats())
                      if args.reuse else None),
               roofline=roof,
               kernels_ms_rank0=dict(k0_prep=tm['prep'], prefilter=tm['prefilter'], exact=tm['exact'],
                                     k2_sort=tm['sort'], detect_total=tm['total'],
                                     timed_detects='the first of %d' % args.steps,
                                     exact_fused=fused),
               prefilter_pair_tests_rank0=tested,
               tile_reuse_rank0=tile_reuse,
               tile_pairs_rank0=ts['tiles'] / max(ts['detects'], 1),
               n_conf=int(counts[0]), n_los=int(counts[1]), n_candidates=int(counts[2]),
               # N^2 x 110 fp64 ops / fp64 peak: what culling buys over evaluating every
               # pair at the ALUs' peak -- a property of the algorithm, not a fraction of peak
               n2_equivalent_speedup_over_fp64_peak=value * OPS_PER_PAIR / (FP64_PEAK_TFLOPS * 1e12),
               propagation=propagation, exact_fp64=exact_fp64,
               build=dict(lib_path=os.path.relpath(lib_path, REPO), lib_sha256=lib_sha),
               parity_vs_world1=None if parity is None else parity['ok'],
               parity=parity,
               rccl_ranks=comm['ranks'] if comm['transport'] == 'rccl' else None, comm=comm)
    if world > 1:   # the halo exchange that replaced the full-state all-gather
        out['halo'] = halo_line(ctx, sim, cd_steps)
    if world > 1:   # C2: the last CD call's pair lists of all ranks to rank 0's host
        g0 = time.perf_counter()
        gp = sim.gather_pairs(root=0)
        gms = float(ctx.allreduce_max([time.perf_counter() - g0])[0]) * 1e3
        if rank == 0:
            out['pair_gather'] = dict(ms=gms, n_conf=len(gp['ci']), n_los=len(gp['li']),
                                      note='bsa_gather_pairs to rank 0 (counts, then rank-order blocks)')
    if not args.no_variants and not args.reuse:
        out['variants'] = variants(ctx, t, rank, world, args.warmup)
        if rank == 0:
            out['variants']['geo_matrix'] = geo_matrix_line(ctx, t)
        if args.workload == 'box100k':
            out['variants']['global1m'] = global1m_line(ctx, rank, world)
    if rank == 0 and world == 1 and not args.no_cpu:
        out['cpu_baseline'] = cpu_baseline(t, args.cpu_rows)
        out['speedup_vs_cpu'] = value / out['cpu_baseline']['value']
        if not args.no_variants:
            d = dropin_detect_line(ctx, t)
            d['speedup_vs_cpu_detect'] = out['cpu_baseline']['detect_s_extrapolated'] * 1e3 / d['ms']['total']
            out['dropin_detect'] = d
    if rank == 0 and world == 1 and not args.no_variants and args.workload == 'box100k':
        out['asas_update'] = asas_update_line(ctx, t)
    if rank == 0:
        print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
