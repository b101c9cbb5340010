"""GPU-resident synthetic sim step over libbsaccel's bsa_sim_*.

State lives in HBM across steps; the host only launches.  One step:
CD + MVP every ``cd_every`` steps (asas.update, asas.py:473-504, with
``asas.active = inconf`` standing in for ResumeNav, or with ``resume_nav`` the
device-side resopairs bookkeeping + ResumeNav), then Pilot.APorASAS
(no wind, constant wind or a 2-D field) fused with the kinematic update
(traffic.py:397-409).  State is kept on the device in home order (the spatial
order of the initial traffic); arrays cross the API in aircraft-index order.
With several ranks (one process per GPU) each rank owns a contiguous,
spatially compact range of home rows; before each CD it receives, over RCCL,
only the column tiles its rows can reach (the halo exchange).
"""
import numpy as np

from . import _lib, dist

FT = 0.3048
KTS = 0.514444
NM = 1852.0
FPM = FT / 60.


def initial_state(traf):
    """Sim state of a freshly created synthetic traffic set (no wind).

    Mirrors Traffic.create (traffic.py:192-312) for what the step reads:
    tas = gs, hdg = trk, gs components, AP targets = the initial values,
    ``ap.vs = 1500 fpm`` (traffic.py:289), ``selalt = alt``, bank 25 deg,
    eps 0.01 (traffic.py:290-308), OpenAP airborne acceleration 0.5 m/s^2
    (perfoap.py:271-280), ``asas.alt = alt`` (asas.py:405-409).
    """
    n = traf.ntraf
    tas = np.array(traf.gs, dtype=np.float64)
    hdg = np.array(traf.trk, dtype=np.float64)
    return dict(lat=np.array(traf.lat, dtype=np.float64), lon=np.array(traf.lon, dtype=np.float64),
                alt=np.array(traf.alt, dtype=np.float64), tas=tas, hdg=hdg,
                vs=np.array(traf.vs, dtype=np.float64), gs=tas.copy(), trk=hdg.copy(),
                gseast=tas * np.sin(np.radians(hdg)), gsnorth=tas * np.cos(np.radians(hdg)),
                ap_trk=hdg.copy(), ap_tas=tas.copy(), ap_alt=np.array(traf.alt, dtype=np.float64),
                ap_vs=np.full(n, 1500. * FPM), selalt=np.array(traf.alt, dtype=np.float64),
                bank=np.full(n, np.radians(25.)), eps=np.full(n, 0.01), accel=np.full(n, 0.5),
                asas_alt=np.array(traf.alt, dtype=np.float64))


def params(simdt=0.05, rpz=5.0 * NM, hpz=1000.0 * FT, tla=300.0, cd_every=1, reso=True, mar=1.05,
           swresohoriz=True, swresospd=False, swresohdg=False, swresovert=False, swprio=False,
           priocode='FF1', wind=None, resume_nav=False, windfield=False):
    """bsa_sim_params; ASAS defaults of asas.py:81-112 with asas_mar from data/default.cfg.
    ``wind=(vnorth, veast)`` [m/s]: constant wind (winddim 1); ``windfield=True``: the
    2-D field handed to ``ResidentSim(windfield=...)`` (winddim 2).  ``resume_nav``: ASAS.update's
    resopairs bookkeeping and ResumeNav's asas.active (asas.py:409-504) instead of
    ``active = inconf``."""
    mvp = _lib.MvpParams(Rm=rpz * mar, dhm=hpz * mar, dtlookahead=tla, vmin=200.0 * NM / 3600.,
                         vmax=500.0 * NM / 3600., vsmin=-3000. / 60. * FT, vsmax=3000. / 60. * FT,
                         swresohoriz=int(swresohoriz), swresospd=int(swresospd),
                         swresohdg=int(swresohdg), swresovert=int(swresovert), swprio=int(swprio),
                         priocode=_lib.PRIO_CODES.get(priocode, 0), swnoreso=0, swresooff=0)
    wn, we = (0.0, 0.0) if wind is None else (float(wind[0]), float(wind[1]))
    return _lib.SimParams(simdt=simdt, rpz=rpz, hpz=hpz, tla=tla, cd_every=int(cd_every),
                          reso=int(bool(reso)), mvp=mvp,
                          winddim=2 if windfield else (0 if wind is None else 1),
                          resume_nav=int(bool(resume_nav)),
                          windnorth=wn, windeast=we)


class ResidentSim:
    """Device-resident traffic; ``rank``/``world`` > 1 shards the rows over GPUs."""

    def __init__(self, state, p, ctx=None, rank=0, world=1, windfield=None, limits=None, group=None):
        """``windfield``: dict(lat, lon, vnorth, veast) of the 2-D field's points
        (Windfield.lat / lon / vnorth[0, :] / veast[0, :]) for ``winddim`` 2.
        ``limits``: per-aircraft OpenAP envelope dict(hmax, vmin, vmax, vsmin,
        vsmax, axmax) for Pilot.applylimits (pilot.py:65-68), or None.
        ``group``: an in-process ``_lib.Group`` to join as ``rank`` instead of
        an RCCL communicator (several ranks in one process, one thread each)."""
        self.ctx = ctx or _lib.default_context()
        self.rank, self.world = rank, world
        if group is not None:
            if getattr(self.ctx, 'comm_rank_world', None) != (rank, group.nranks):
                self.ctx.comm_init_group(group, rank)
        elif world > 1:
            dist.init_comm(self.ctx, rank, world)
        if windfield is not None:
            self.ctx.set_windfield(windfield['lat'], windfield['lon'], windfield['vnorth'],
                                   windfield['veast'])
        self.ctx.sim_init(state, p)
        if limits is not None:
            self.ctx.sim_set_limits(limits)
        self.params = p

    def step(self, nsteps=1):
        self.ctx.sim_step(nsteps)

    def set_params(self, p):
        """New parameters for the running sim (bsa_sim_set_params; e.g. ZONER / DTLOOK)."""
        self.ctx.sim_set_params(p)
        self.params = p

    def halo_stats(self):
        """Halo exchange of the sharded step (bsa_sim_halo_stats): rx / tx bytes per CD
        call, tiles received at the last CD call, capacity regrowths."""
        return self.ctx.sim_halo_stats()

    def update(self, **arrays):
        """Overwrite state arrays (host simulator changed the traffic between
        steps) keeping the ASAS bookkeeping (bsa_sim_update)."""
        self.ctx.sim_update(**arrays)

    def set_perf(self, table=None, type_idx=None):
        """OpenAP.update's flight phase, phase-dependent envelope and
        acceleration in every step (bsa_sim_set_perf; bluesky_amd.perf builds
        ``table`` / ``type_idx``); None switches it off."""
        self.ctx.sim_set_perf(table, type_idx)

    def read_perf(self):
        """(flight phase of the last step, traf.ax) of this rank's rows."""
        return self.ctx.sim_read_perf()

    def create(self, state):
        """Append aircraft (Traffic.create; ``state`` as ``initial_state`` returns,
        m long each): indices n..n+m-1 (bsa_sim_create; collective with several ranks)."""
        self.ctx.sim_create(state)

    def delete(self, idx):
        """Remove aircraft ``idx`` (Traffic.delete: the rest shift down in order),
        keeping the callsign-keyed ASAS bookkeeping of the others (bsa_sim_delete)."""
        self.ctx.sim_delete(idx)

    def read(self):
        return self.ctx.sim_read()

    def stats(self):
        return self.ctx.sim_stats()

    def asas_stats(self):
        return self.ctx.sim_asas_stats()

    def resopairs(self):
        return self.ctx.sim_resopairs()

    def row_ids(self):
        """Aircraft indices of this rank's rows (ascending)."""
        return self.ctx.sim_row_ids()

    def gather_pairs(self, root=0):
        """C2: the last CD call's pairs of all ranks, on ``root`` (collective)."""
        return self.ctx.gather_pairs(root)

    def acdata_request(self):
        """Enqueue an ACDATA snapshot of this rank's rows behind the queued steps
        (screenio.py:194-239; no host synchronisation)."""
        self.ctx.sim_acdata_request()

    def acdata(self, wait=True):
        """The requested snapshot: dict of per-row arrays (lat lon alt tas cas gs
        trk vs tcpamax inconf asasn asase) plus steps, row_begin/row_end and the
        four pair counts; None while in flight when ``wait`` is False."""
        return self.ctx.sim_acdata_poll(wait)
