"""ctypes binding of ``libbsaccel.so`` (declarations in ``include/bsaccel.h``).

The HIP library is the ONLY compute path: if it is missing, or no HIP device
is visible, every call raises ``AccelUnavailable`` -- there is deliberately no
CPU fallback in the product path.
"""
import ctypes
import os
import threading

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('BSACCEL_LIB', os.path.join(_HERE, 'libbsaccel.so'))

ABI_VERSION = 1
PF_BLOCK_PAIRS = 512   # BSA_PF_BLOCK_PAIRS: stage-1 pair tests per swept prefilter block
FLAG_WITH_DCPA = 1
FLAG_NOPRUNE = 2
FLAG_RESORT = 4
FLAG_KWIK = 8
FLAG_STAGE1_T0 = 16
GEO_KWIK = 1
GEO_PAIRWISE = 2

_c_dp = ctypes.POINTER(ctypes.c_double)
_c_fp = ctypes.POINTER(ctypes.c_float)
_c_i32p = ctypes.POINTER(ctypes.c_int32)
_c_u8p = ctypes.POINTER(ctypes.c_uint8)
_c_i64p = ctypes.POINTER(ctypes.c_int64)
_vp = ctypes.c_void_p


class AccelUnavailable(RuntimeError):
    """libbsaccel.so could not be loaded or has no usable HIP device."""


class AccelError(RuntimeError):
    """A libbsaccel call returned an error status."""


# name -> (restype, argtypes); must match include/bsaccel.h exactly
SIGNATURES = {
    'bsa_abi_version': (ctypes.c_int, []),
    'bsa_device_count': (ctypes.c_int, []),
    'bsa_create': (_vp, [ctypes.c_int]),
    'bsa_destroy': (None, [_vp]),
    'bsa_last_error': (ctypes.c_char_p, [_vp]),
    'bsa_sync': (ctypes.c_int, [_vp]),
    'bsa_set_state': (ctypes.c_int, [_vp, ctypes.c_int64] + [_c_dp] * 6),
    'bsa_set_intruder': (ctypes.c_int, [_vp, ctypes.c_int64] + [_c_dp] * 6),
    'bsa_detect': (ctypes.c_int, [_vp, ctypes.c_double, ctypes.c_double, ctypes.c_double,
                                  ctypes.c_int, ctypes.c_int64, ctypes.c_int64, _c_i64p, _c_i64p]),
    'bsa_fetch_pairs': (ctypes.c_int, [_vp, _c_i32p, _c_i32p, _c_dp, _c_dp, _c_dp, _c_dp, _c_dp,
                                       _c_i32p, _c_i32p, _c_u8p, _c_dp]),
    'bsa_last_candidates': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_last_tiles': (ctypes.c_int, [_vp, _c_i64p, _c_i64p, _c_i64p]),
    'bsa_set_candidate_reuse': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double, ctypes.c_double]),
    'bsa_reuse_stats': (ctypes.c_int, [_vp, _c_i64p, _c_i64p]),
    'bsa_set_tile_reuse': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double, ctypes.c_double]),
    'bsa_tile_reuse_stats': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_set_hk': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_double]),
    'bsa_hk_stats': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_set_halo_overlap': (ctypes.c_int, [_vp, ctypes.c_int]),
    'bsa_halo_overlap_count': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_reuse_budget_use': (ctypes.c_int, [_vp, _c_dp]),
    'bsa_last_timings': (ctypes.c_int, [_vp, _c_dp]),
    'bsa_timing_reset': (ctypes.c_int, [_vp]),
    'bsa_set_candidate_capacity': (ctypes.c_int, [_vp, ctypes.c_int64]),
    'bsa_timing_summary': (ctypes.c_int, [_vp, _c_dp, _c_i64p]),
    'bsa_set_timing_sample': (ctypes.c_int, [_vp, ctypes.c_int]),
}

PRIO_CODES = {'FF1': 1, 'FF2': 2, 'FF3': 3, 'LAY1': 4, 'LAY2': 5}


class MvpParams(ctypes.Structure):
    """bsa_mvp_params (include/bsaccel.h)."""
    _fields_ = [('Rm', ctypes.c_double), ('dhm', ctypes.c_double),
                ('dtlookahead', ctypes.c_double), ('vmin', ctypes.c_double),
                ('vmax', ctypes.c_double), ('vsmin', ctypes.c_double), ('vsmax', ctypes.c_double),
                ('swresohoriz', ctypes.c_int32), ('swresospd', ctypes.c_int32),
                ('swresohdg', ctypes.c_int32), ('swresovert', ctypes.c_int32),
                ('swprio', ctypes.c_int32), ('priocode', ctypes.c_int32),
                ('swnoreso', ctypes.c_int32), ('swresooff', ctypes.c_int32)]


class KinIO(ctypes.Structure):
    """bsa_kin_io (include/bsaccel.h)."""
    _fields_ = [(k, _c_dp) for k in ('ptas', 'phdg', 'palt', 'pvs', 'bank', 'eps', 'accel',
                                     'tas', 'hdg', 'alt', 'vs', 'lat', 'lon', 'ax', 'delspd',
                                     'cas', 'mach', 'gsnorth', 'gseast', 'gs', 'trk', 'coslat',
                                     'az')] + [('swhdgsel', _c_u8p), ('swaltsel', _c_u8p)]


SIGNATURES.update({
    'bsa_set_pairs': (ctypes.c_int, [_vp, ctypes.c_int64, _c_i32p, _c_i32p, _c_dp, _c_dp, _c_dp,
                                     _c_dp]),
    'bsa_mvp': (ctypes.c_int, [_vp, ctypes.POINTER(MvpParams), _c_dp, _c_dp, _c_dp, _c_dp, _c_u8p,
                               _c_u8p, _c_dp, _c_dp, _c_dp, _c_dp, _c_fp, _c_fp]),
    'bsa_kinematics': (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_double, ctypes.c_int,
                                      ctypes.c_double, ctypes.c_double, ctypes.POINTER(KinIO)]),
})

class SimParams(ctypes.Structure):
    """bsa_sim_params (include/bsaccel.h)."""
    _fields_ = [('simdt', ctypes.c_double), ('rpz', ctypes.c_double), ('hpz', ctypes.c_double),
                ('tla', ctypes.c_double), ('cd_every', ctypes.c_int32), ('reso', ctypes.c_int32),
                ('mvp', MvpParams), ('winddim', ctypes.c_int32), ('resume_nav', ctypes.c_int32),
                ('windnorth', ctypes.c_double), ('windeast', ctypes.c_double)]


SIM_STATE_FIELDS = ('lat', 'lon', 'alt', 'tas', 'hdg', 'vs', 'gs', 'trk', 'gseast', 'gsnorth',
                    'ap_trk', 'ap_tas', 'ap_alt', 'ap_vs', 'selalt', 'bank', 'eps', 'accel',
                    'asas_alt')
SIM_OUT_FIELDS = ('lat', 'lon', 'alt', 'tas', 'hdg', 'vs', 'gs', 'trk', 'gseast', 'gsnorth',
                  'asas_trk', 'asas_tas', 'asas_vs', 'asas_alt')


class SimState(ctypes.Structure):
    """bsa_sim_state (include/bsaccel.h)."""
    _fields_ = [(k, _c_dp) for k in SIM_STATE_FIELDS]


class SimOut(ctypes.Structure):
    """bsa_sim_out (include/bsaccel.h)."""
    _fields_ = [(k, _c_dp) for k in SIM_OUT_FIELDS] + [('active', _c_u8p)]


ACDATA_F64 = ('lat', 'lon', 'alt', 'tas', 'cas', 'gs', 'trk', 'vs', 'tcpamax')
ACDATA_COUNTS = ('nconf_cur', 'nconf_tot', 'nlos_cur', 'nlos_tot')


class AcData(ctypes.Structure):
    """bsa_acdata (include/bsaccel.h)."""
    _fields_ = ([(k, ctypes.c_int64) for k in ('steps', 'row_begin', 'row_end') + ACDATA_COUNTS] +
                [(k, _c_dp) for k in ACDATA_F64] + [('inconf', _c_u8p), ('asasn', _c_fp), ('asase', _c_fp)])


class PairsOut(ctypes.Structure):
    """bsa_pairs_out (include/bsaccel.h)."""
    _fields_ = [('ci', _c_i32p), ('cj', _c_i32p), ('qdr', _c_dp), ('dist', _c_dp), ('tcpa', _c_dp),
                ('tinconf', _c_dp), ('dcpa', _c_dp), ('li', _c_i32p), ('lj', _c_i32p), ('inconf', _c_u8p),
                ('tcpamax', _c_dp)]


SIGNATURES.update({
    'bsa_group_create': (_vp, [ctypes.c_int]),
    'bsa_group_destroy': (None, [_vp]),
    'bsa_comm_init_group': (ctypes.c_int, [_vp, _vp, ctypes.c_int]),
    'bsa_gather_counts': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_gather_pairs': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(PairsOut)]),
    'bsa_comm_unique_id': (ctypes.c_int, [ctypes.c_char_p]),
    'bsa_comm_init': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_char_p]),
    'bsa_comm_allreduce_max': (ctypes.c_int, [_vp, _c_dp, ctypes.c_int]),
    'bsa_comm_allreduce_sum': (ctypes.c_int, [_vp, _c_dp, ctypes.c_int]),
    'bsa_comm_info': (ctypes.c_int, [_vp, ctypes.POINTER(ctypes.c_int)]),
    'bsa_sim_init': (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.POINTER(SimState),
                                    ctypes.POINTER(SimParams)]),
    'bsa_sim_step': (ctypes.c_int, [_vp, ctypes.c_int]),
    'bsa_sim_update': (ctypes.c_int, [_vp, ctypes.POINTER(SimState)]),
    'bsa_sim_create': (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.POINTER(SimState)]),
    'bsa_sim_delete': (ctypes.c_int, [_vp, ctypes.c_int64, _c_i64p]),
    'bsa_sim_read': (ctypes.c_int, [_vp, ctypes.POINTER(SimOut)]),
    'bsa_sim_stats': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_sim_row_ids': (ctypes.c_int, [_vp, _c_i32p]),
    'bsa_set_row_bucket': (ctypes.c_int, [_vp, ctypes.c_int]),
    'bsa_sim_detect_rows': (ctypes.c_int, [_vp, ctypes.c_int64, ctypes.c_int64, _c_i64p, _c_i64p]),
    'bsa_sim_asas_stats': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_sim_resopairs': (ctypes.c_int, [_vp, _c_i32p, _c_i32p, ctypes.c_int64, _c_i64p]),
    'bsa_qdrdist': (ctypes.c_int, [_vp, ctypes.c_int64, _c_dp, _c_dp, ctypes.c_int64, _c_dp, _c_dp,
                                   ctypes.c_int, _c_dp, _c_dp]),
    'bsa_geo_last_ms': (ctypes.c_int, [_vp, _c_dp]),
    'bsa_sim_acdata_request': (ctypes.c_int, [_vp]),
    'bsa_set_windfield': (ctypes.c_int, [_vp, ctypes.c_int64, _c_dp, _c_dp, _c_dp, _c_dp]),
    'bsa_sim_set_limits': (ctypes.c_int, [_vp] + [_c_dp] * 6),
    'bsa_sim_set_perf': (ctypes.c_int, [_vp, ctypes.c_int64, _c_dp, _c_i32p]),
    'bsa_sim_read_perf': (ctypes.c_int, [_vp, _c_u8p, _c_dp]),
    'bsa_sim_acdata_poll': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.POINTER(AcData)]),
})



class AsasOut(ctypes.Structure):
    """bsa_asas_out (include/bsaccel.h)."""
    _fields_ = [(k, _c_dp) for k in ('trk', 'tas', 'vs', 'alt')] + [('asase', _c_fp), ('asasn', _c_fp),
                                                                   ('active', _c_u8p), ('dropped', _c_u8p)]


SIGNATURES.update({
    'bsa_sim_cd': (ctypes.c_int, [_vp]),
    'bsa_sim_set_params': (ctypes.c_int, [_vp, ctypes.POINTER(SimParams)]),
    'bsa_sim_set_reso_lists': (ctypes.c_int, [_vp, _c_u8p, _c_u8p]),
    'bsa_sim_read_asas': (ctypes.c_int, [_vp, ctypes.POINTER(AsasOut)]),
    'bsa_sim_halo_stats': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_sim_set_halo_cap': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int, ctypes.c_int64]),
    'bsa_sim_halo_recheck': (ctypes.c_int, [_vp]),
    'bsa_sim_probe_rank': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    'bsa_set_exact_fusion': (ctypes.c_int, [_vp, ctypes.c_int, ctypes.c_int]),
    'bsa_exact_fusion_stats': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_sim_comm_stats': (ctypes.c_int, [_vp, _c_i64p]),
    'bsa_sim_set_atmos': (ctypes.c_int, [_vp, ctypes.c_int]),
    'bsa_sim_read_atmos': (ctypes.c_int, [_vp, _c_dp, _c_dp, _c_dp]),
})

UNIQUE_ID_BYTES = 128

_lib = None
_lib_lock = threading.Lock()


def load(path=None):
    """Load and type the library (idempotent).  Raises AccelUnavailable."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        p = path or LIB_PATH
        if not os.path.exists(p):
            raise AccelUnavailable('libbsaccel.so not built (%s); run `make -C bluesky_amd/csrc` '
                                   'or __graft_entry__.build()' % p)
        try:
            lib = ctypes.CDLL(p)
        except OSError as e:
            raise AccelUnavailable('cannot load %s: %s' % (p, e))
        skipped = []
        for name, (res, args) in SIGNATURES.items():
            if not hasattr(lib, name) and p != os.path.join(_HERE, 'libbsaccel.so') \
                    and os.environ.get('BSACCEL_AB') == '1':
                skipped.append(name)   # an older build selected for an A/B measurement
                continue
            if not hasattr(lib, name):
                raise AccelUnavailable('%s lacks %s (stale build? set BSACCEL_AB=1 to load an older '
                                       'build for an A/B measurement)' % (p, name))
            f = getattr(lib, name)
            f.restype = res
            f.argtypes = args
        if skipped:
            import sys
            print('[bsaccel] %s: %d symbols missing (BSACCEL_AB=1): %s' % (p, len(skipped), ' '.join(skipped)),
                  file=sys.stderr)
        v = lib.bsa_abi_version()
        if v != ABI_VERSION:
            raise AccelUnavailable('ABI mismatch: library %d, bindings %d' % (v, ABI_VERSION))
        _lib = lib
        return lib


def mapped_library():
    """(path, sha256) of the libbsaccel this process actually mapped (from
    /proc/self/maps; measurement provenance: bench.py / tools/pmc_roofline.py)."""
    import hashlib
    load()
    path = None
    try:
        with open('/proc/self/maps') as f:
            for line in f:
                q = line.split()
                if len(q) >= 6 and os.path.basename(q[-1]).startswith('libbsaccel'):
                    path = q[-1]
                    break
    except OSError:
        pass
    path = path or os.path.realpath(LIB_PATH)
    with open(path, 'rb') as f:
        return path, hashlib.sha256(f.read()).hexdigest()


def comm_unique_id():
    """128-byte RCCL communicator id (create on one rank, ship to the others)."""
    lib = load()
    buf = ctypes.create_string_buffer(UNIQUE_ID_BYTES)
    if lib.bsa_comm_unique_id(buf) != 0:
        raise AccelError('bsa_comm_unique_id failed')
    return buf.raw


class Group:
    """In-process group of contexts (bsa_group_*): the ranks of a row-sharded
    sim in ONE process, one host thread per rank.  Keep it alive until every
    member context is closed."""

    def __init__(self, nranks):
        self.lib = load()
        self.h = self.lib.bsa_group_create(int(nranks))
        if not self.h:
            raise AccelError('bsa_group_create(%d) failed' % nranks)
        self.nranks = nranks

    def close(self):
        if getattr(self, 'h', None):
            self.lib.bsa_group_destroy(self.h)
            self.h = None


def ptr(a, ctype=_c_dp):
    return None if a is None else a.ctypes.data_as(ctype)


def f64(a):
    return np.ascontiguousarray(a, dtype=np.float64)


class Context:
    """One HIP device + stream + its device buffers (bsa_ctx)."""

    def __init__(self, device=0):
        self.lib = load()
        ndev = self.lib.bsa_device_count()
        if ndev <= 0:
            raise AccelUnavailable('no HIP device visible (bsa_device_count=%d)' % ndev)
        h = self.lib.bsa_create(int(device))
        if not h:
            raise AccelUnavailable('bsa_create(%d) failed: %s'
                                   % (device, self.lib.bsa_last_error(None).decode()))
        self.h = h
        self.device = device
        # bumped by every call that replaces the device-resident state or pairs
        # (set_state / set_intruder / detect / set_pairs / sim_*): the MVP drop-in
        # reuses a detect's device pairs only while it is unchanged
        self.gen = 0

    def close(self):
        if getattr(self, 'h', None):
            self.lib.bsa_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def check(self, status, what):
        if status != 0:
            raise AccelError('%s: %s' % (what, self.lib.bsa_last_error(self.h).decode()))

    # ---------------------------------------------------------------- state
    def set_state(self, lat, lon, trk, gs, alt, vs):
        self.gen += 1
        arrs = [f64(x) for x in (lat, lon, trk, gs, alt, vs)]
        n = len(arrs[0])
        if any(len(a) != n for a in arrs):
            raise ValueError('state arrays differ in length')
        self.check(self.lib.bsa_set_state(self.h, n, *[ptr(a) for a in arrs]), 'bsa_set_state')
        self.n = n

    def set_intruder(self, lat=None, lon=None, trk=None, gs=None, alt=None, vs=None):
        self.gen += 1
        if lat is None:
            self.check(self.lib.bsa_set_intruder(self.h, 0, *([None] * 6)), 'bsa_set_intruder')
            return
        arrs = [f64(x) for x in (lat, lon, trk, gs, alt, vs)]
        self.check(self.lib.bsa_set_intruder(self.h, len(arrs[0]), *[ptr(a) for a in arrs]),
                   'bsa_set_intruder')

    # ---------------------------------------------------------------- detect
    def detect(self, rpz, hpz, tla, flags=0, row_begin=0, row_end=-1):
        self.gen += 1
        nc = ctypes.c_int64()
        nl = ctypes.c_int64()
        self.check(self.lib.bsa_detect(self.h, float(rpz), float(hpz), float(tla), int(flags),
                                       int(row_begin), int(row_end), ctypes.byref(nc),
                                       ctypes.byref(nl)), 'bsa_detect')
        self._rows = (row_begin, self.n if row_end is None or row_end < 0 else row_end)
        return nc.value, nl.value

    def fetch_pairs(self, n_conf, n_los, with_dcpa=False):
        P, L = n_conf, n_los
        R = self._rows[1] - self._rows[0]
        o = dict(ci=np.empty(P, np.int32), cj=np.empty(P, np.int32), qdr=np.empty(P),
                 dist=np.empty(P), tcpa=np.empty(P), tinconf=np.empty(P),
                 dcpa=np.empty(P) if with_dcpa else None, li=np.empty(L, np.int32),
                 lj=np.empty(L, np.int32), inconf=np.empty(R, np.uint8), tcpamax=np.empty(R))
        self.check(self.lib.bsa_fetch_pairs(
            self.h, ptr(o['ci'], _c_i32p), ptr(o['cj'], _c_i32p), ptr(o['qdr']), ptr(o['dist']),
            ptr(o['tcpa']), ptr(o['tinconf']), ptr(o['dcpa']), ptr(o['li'], _c_i32p),
            ptr(o['lj'], _c_i32p), ptr(o['inconf'], _c_u8p), ptr(o['tcpamax'])), 'bsa_fetch_pairs')
        return o

    ENVELOPE_FIELDS = ('hmax', 'vmin', 'vmax', 'vsmin', 'vsmax', 'axmax')

    def sim_set_limits(self, env=None):
        """OpenAP envelope for Pilot.applylimits in the resident step (bsa_sim_set_limits);
        ``env`` = dict of the six per-aircraft arrays, None switches the limits off."""
        if env is None:
            self.check(self.lib.bsa_sim_set_limits(self.h, *([None] * 6)), 'bsa_sim_set_limits')
            return
        arrs = [f64(env[k]).ravel() for k in self.ENVELOPE_FIELDS]
        self.check(self.lib.bsa_sim_set_limits(self.h, *[ptr(a) for a in arrs]), 'bsa_sim_set_limits')

    # ---------------------------------------------------------------- wind field
    def set_windfield(self, lat=None, lon=None, vnorth=None, veast=None):
        """2-D wind field for winddim 2 (bsa_set_windfield); no arguments clears it."""
        if lat is None:
            self.check(self.lib.bsa_set_windfield(self.h, 0, None, None, None, None), 'bsa_set_windfield')
            return
        arrs = [f64(x).ravel() for x in (lat, lon, vnorth, veast)]
        if len({len(a) for a in arrs}) != 1:
            raise ValueError('wind field arrays differ in length')
        self.check(self.lib.bsa_set_windfield(self.h, len(arrs[0]), *[ptr(a) for a in arrs]),
                   'bsa_set_windfield')

    # ---------------------------------------------------------------- ACDATA feed
    def sim_acdata_request(self):
        self.check(self.lib.bsa_sim_acdata_request(self.h), 'bsa_sim_acdata_request')

    def sim_acdata_poll(self, wait=True):
        """The requested snapshot as a dict, or None while it is in flight (wait=False)."""
        probe = AcData()   # NULL arrays: status and row range only (no stream sync)
        st = self.lib.bsa_sim_acdata_poll(self.h, int(bool(wait)), ctypes.byref(probe))
        if st == 1:
            return None
        self.check(st, 'bsa_sim_acdata_poll')
        nr = probe.row_end - probe.row_begin
        arr = {k: np.empty(nr) for k in ACDATA_F64}
        arr.update(inconf=np.empty(nr, np.uint8), asasn=np.empty(nr, np.float32),
                   asase=np.empty(nr, np.float32))
        o = AcData(**{k: ptr(arr[k]) for k in ACDATA_F64}, inconf=ptr(arr['inconf'], _c_u8p),
                   asasn=ptr(arr['asasn'], _c_fp), asase=ptr(arr['asase'], _c_fp))
        self.check(self.lib.bsa_sim_acdata_poll(self.h, 1, ctypes.byref(o)), 'bsa_sim_acdata_poll')
        arr['inconf'] = arr['inconf'].astype(bool)
        arr.update({k: getattr(o, k) for k in ('steps', 'row_begin', 'row_end') + ACDATA_COUNTS})
        return arr

    # ---------------------------------------------------------------- geo matrices
    def qdrdist(self, lat1, lon1, lat2, lon2, kwik=False, pairwise=False):
        """bsa_qdrdist: (qdr, dist) as flat float64 arrays of m*n (outer) or m
        (pairwise) entries, row-major [i, j]."""
        la1, lo1, la2, lo2 = (f64(x).ravel() for x in (lat1, lon1, lat2, lon2))
        m, n = len(la1), len(la2)
        if len(lo1) != m or len(lo2) != n:
            raise ValueError('lat/lon lengths differ')
        total = m if pairwise else m * n
        qdr, dist = np.empty(total), np.empty(total)
        flags = (GEO_KWIK if kwik else 0) | (GEO_PAIRWISE if pairwise else 0)
        self.check(self.lib.bsa_qdrdist(self.h, m, ptr(la1), ptr(lo1), n, ptr(la2), ptr(lo2), flags,
                                        ptr(qdr), ptr(dist)), 'bsa_qdrdist')
        return qdr, dist

    def geo_last_ms(self):
        v = ctypes.c_double()
        self.check(self.lib.bsa_geo_last_ms(self.h, ctypes.byref(v)), 'bsa_geo_last_ms')
        return v.value

    def last_candidates(self):
        v = ctypes.c_int64()
        self.check(self.lib.bsa_last_candidates(self.h, ctypes.byref(v)), 'bsa_last_candidates')
        return v.value

    def set_candidate_capacity(self, capacity):
        """Candidate-list capacity for the next detects (grown on overflow)."""
        self.check(self.lib.bsa_set_candidate_capacity(self.h, int(capacity)),
                   'bsa_set_candidate_capacity')

    def set_candidate_reuse(self, on=True, sigma_h=800.0, sigma_v=60.0):
        """bsa_set_candidate_reuse: keep the candidate list across detects while
        every aircraft's drift stays inside its budgets (exact either way)."""
        self.check(self.lib.bsa_set_candidate_reuse(self.h, int(bool(on)), float(sigma_h), float(sigma_v)),
                   'bsa_set_candidate_reuse')

    def set_tile_reuse(self, on=True, sigma_h=2016.0, sigma_v=300.0):
        """bsa_set_tile_reuse: keep the resident detect's tile-pair list (K0d) while
        every prefilter record stays within the budgets of its build-time record."""
        self.check(self.lib.bsa_set_tile_reuse(self.h, int(bool(on)), float(sigma_h), float(sigma_v)),
                   'bsa_set_tile_reuse')

    def tile_reuse_stats(self):
        v = np.zeros(2, np.int64)
        self.check(self.lib.bsa_tile_reuse_stats(self.h, ptr(v, _c_i64p)), 'bsa_tile_reuse_stats')
        return dict(builds=int(v[0]), detects=int(v[1]))

    def set_hk(self, on=True, f=0.75):
        """Host-known tile-pair list decisions of the resident step (bsa_set_hk)."""
        self.check(self.lib.bsa_set_hk(self.h, 1 if on else 0, float(f)), 'bsa_set_hk')

    def set_halo_overlap(self, mode):
        """Halo exchange overlapped with the own tiles' sweep (bsa_set_halo_overlap):
        0 off, 1 several ranks, 2 also the one-GPU probe."""
        self.check(self.lib.bsa_set_halo_overlap(self.h, int(mode)), 'bsa_set_halo_overlap')

    def halo_overlap_count(self):
        v = np.zeros(1, np.int64)
        self.check(self.lib.bsa_halo_overlap_count(self.h, ptr(v, _c_i64p)), 'bsa_halo_overlap_count')
        return int(v[0])

    def hk_stats(self):
        v = np.zeros(6, np.int64)
        self.check(self.lib.bsa_hk_stats(self.h, ptr(v, _c_i64p)), 'bsa_hk_stats')
        return dict(keeps=int(v[0]), builds=int(v[1]), waits=int(v[2]), stale_aborts=int(v[3]),
                    cooldown=int(v[4]), on=bool(v[5]))

    def reuse_stats(self):
        b, d = ctypes.c_int64(), ctypes.c_int64()
        self.check(self.lib.bsa_reuse_stats(self.h, ctypes.byref(b), ctypes.byref(d)), 'bsa_reuse_stats')
        return dict(builds=b.value, detects=d.value)

    def reuse_budget_use(self):
        u = np.zeros(2)
        self.check(self.lib.bsa_reuse_budget_use(self.h, ptr(u)), 'bsa_reuse_budget_use')
        return float(u[0]), float(u[1])

    def last_tiles(self):
        kept, total, groups = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_int64()
        self.check(self.lib.bsa_last_tiles(self.h, ctypes.byref(kept), ctypes.byref(total),
                                           ctypes.byref(groups)), 'bsa_last_tiles')
        return kept.value, total.value, groups.value

    def last_timings(self):
        t = np.zeros(5)
        self.check(self.lib.bsa_last_timings(self.h, ptr(t)), 'bsa_last_timings')
        return dict(prep=t[0], prefilter=t[1], exact=t[2], sort=t[3], total=t[4])

    def set_timing_sample(self, every):
        """Time one detect in ``every`` (bsa_set_timing_sample; 0 = none)."""
        self.check(self.lib.bsa_set_timing_sample(self.h, int(every)), 'bsa_set_timing_sample')

    def timing_reset(self):
        """Forget recorded detect timings / statistics (bsa_timing_reset)."""
        self.check(self.lib.bsa_timing_reset(self.h), 'bsa_timing_reset')

    def timing_summary(self):
        """Mean stage times [ms] over the detects since the last reset and the
        summed statistics (bsa_timing_summary)."""
        t = np.zeros(5)
        st = np.zeros(4, np.int64)
        self.check(self.lib.bsa_timing_summary(self.h, ptr(t), ptr(st, _c_i64p)), 'bsa_timing_summary')
        return (dict(prep=t[0], prefilter=t[1], exact=t[2], sort=t[3], total=t[4]),
                dict(groups=int(st[0]), candidates=int(st[1]), tiles=int(st[2]), detects=int(st[3])))

    def sync(self):
        self.check(self.lib.bsa_sync(self.h), 'bsa_sync')

    # ---------------------------------------------------------------- MVP
    def set_pairs(self, ci, cj, qdr, dist, tcpa, tlos):
        """bsa_set_pairs: external confpairs (row-major) for bsa_mvp."""
        self.gen += 1
        ci = np.ascontiguousarray(ci, dtype=np.int32)
        cj = np.ascontiguousarray(cj, dtype=np.int32)
        arrs = [f64(x) for x in (qdr, dist, tcpa, tlos)]
        self.check(self.lib.bsa_set_pairs(self.h, len(ci), ptr(ci, _c_i32p), ptr(cj, _c_i32p),
                                          *[ptr(a) for a in arrs]), 'bsa_set_pairs')
        self._rows = (0, self.n)

    def mvp(self, params, gseast, gsnorth, selalt, apvs, asas_alt, noreso=None, resooff=None):
        """bsa_mvp on the last detect's pairs; ``asas_alt`` (detect rows) is
        updated in place.  Returns dict(trk, tas, vs, asase, asasn)."""
        rows = self._rows[1] - self._rows[0]
        ins = [f64(x) for x in (gseast, gsnorth, selalt, apvs)]
        if asas_alt.dtype != np.float64 or not asas_alt.flags.c_contiguous or len(asas_alt) != rows:
            raise ValueError('asas_alt must be a contiguous float64 array of the detect rows')
        nr = None if noreso is None else np.ascontiguousarray(noreso, dtype=np.uint8)
        ro = None if resooff is None else np.ascontiguousarray(resooff, dtype=np.uint8)
        o = dict(trk=np.empty(rows), tas=np.empty(rows), vs=np.empty(rows),
                 asase=np.empty(rows, np.float32), asasn=np.empty(rows, np.float32))
        self.check(self.lib.bsa_mvp(self.h, ctypes.byref(params), *[ptr(a) for a in ins],
                                    ptr(nr, _c_u8p), ptr(ro, _c_u8p), ptr(asas_alt), ptr(o['trk']),
                                    ptr(o['tas']), ptr(o['vs']), ptr(o['asase'], _c_fp),
                                    ptr(o['asasn'], _c_fp)), 'bsa_mvp')
        return o

    # ---------------------------------------------------------------- multi-GPU
    def comm_init(self, nranks, rank, uid):
        if len(uid) != UNIQUE_ID_BYTES:
            raise ValueError('unique id must be %d bytes' % UNIQUE_ID_BYTES)
        self.check(self.lib.bsa_comm_init(self.h, int(nranks), int(rank), uid), 'bsa_comm_init')
        self.comm_rank_world = (int(rank), int(nranks))

    def comm_init_group(self, group, rank):
        """Join an in-process Group as ``rank`` (call from this rank's thread)."""
        self.check(self.lib.bsa_comm_init_group(self.h, group.h, int(rank)), 'bsa_comm_init_group')
        self.comm_rank_world = (rank, group.nranks)
        self.gen += 1

    def comm_info(self):
        """The communicator as its transport reports it (bsa_comm_info): with
        RCCL, ranks / rank / device are ncclCommCount / ncclCommUserRank /
        ncclCommCuDevice."""
        v = (ctypes.c_int * 4)()
        self.check(self.lib.bsa_comm_info(self.h, v), 'bsa_comm_info')
        return dict(transport=('none', 'rccl', 'group')[v[0]], ranks=v[1], rank=v[2], device=v[3])

    def gather_pairs(self, root=0, with_dcpa=False):
        """C2: every rank's last detect gathered to ``root`` in rank order
        (collective; bsa_gather_counts + bsa_gather_pairs).  Returns the
        fetch_pairs-style dict on the root, None elsewhere."""
        tot = np.zeros(3, np.int64)
        self.check(self.lib.bsa_gather_counts(self.h, ptr(tot, _c_i64p)), 'bsa_gather_counts')
        P, L, R = (int(x) for x in tot)
        rank = getattr(self, 'comm_rank_world', (0, 1))[0]
        if rank != root:
            self.check(self.lib.bsa_gather_pairs(self.h, int(root), None), 'bsa_gather_pairs')
            return None
        o = dict(ci=np.empty(P, np.int32), cj=np.empty(P, np.int32), qdr=np.empty(P), dist=np.empty(P),
                 tcpa=np.empty(P), tinconf=np.empty(P), dcpa=np.empty(P) if with_dcpa else None,
                 li=np.empty(L, np.int32), lj=np.empty(L, np.int32), inconf=np.empty(R, np.uint8),
                 tcpamax=np.empty(R))
        po = PairsOut(**{k: ptr(v, _c_i32p if v.dtype == np.int32 else (_c_u8p if v.dtype == np.uint8 else _c_dp))
                         for k, v in o.items() if v is not None})
        self.check(self.lib.bsa_gather_pairs(self.h, int(root), ctypes.byref(po)), 'bsa_gather_pairs')
        return o

    def allreduce_max(self, values):
        v = np.array(values, dtype=np.float64, copy=True).ravel()
        self.check(self.lib.bsa_comm_allreduce_max(self.h, ptr(v), len(v)), 'bsa_comm_allreduce_max')
        return v

    def allreduce_sum(self, values):
        v = np.array(values, dtype=np.float64, copy=True).ravel()
        self.check(self.lib.bsa_comm_allreduce_sum(self.h, ptr(v), len(v)), 'bsa_comm_allreduce_sum')
        return v

    # ---------------------------------------------------------------- resident sim
    def sim_init(self, state, params):
        self.gen += 1
        n = len(state['lat'])
        keep = {k: f64(state[k]) for k in SIM_STATE_FIELDS}
        for k, a in keep.items():
            if len(a) != n:
                raise ValueError('sim state %s has length %d != %d' % (k, len(a), n))
        st = SimState(**{k: ptr(a) for k, a in keep.items()})
        self.check(self.lib.bsa_sim_init(self.h, n, ctypes.byref(st), ctypes.byref(params)),
                   'bsa_sim_init')
        self.n = n
        st = self.sim_stats()
        self._rows = (st['row_begin'], st['row_end'])   # fetch_pairs after steps: this rank's rows

    def sim_set_perf(self, table=None, type_idx=None):
        """bsa_sim_set_perf: OpenAP phase-dependent envelope + acceleration in the
        step (``table``/``type_idx`` from bluesky_amd.perf.type_table); None = off."""
        if table is None:
            self.check(self.lib.bsa_sim_set_perf(self.h, 0, None, None), 'bsa_sim_set_perf')
            return
        tab = np.ascontiguousarray(table, dtype=np.float64)
        idx = np.ascontiguousarray(type_idx, dtype=np.int32).ravel()
        if tab.ndim != 2 or tab.shape[1] != 24:
            raise ValueError('type table must be ntypes x 24')
        if len(idx) != self.n:
            raise ValueError('type index has length %d != %d' % (len(idx), self.n))
        self._perf_keep = (tab, idx)
        self.check(self.lib.bsa_sim_set_perf(self.h, tab.shape[0], ptr(tab), ptr(idx, _c_i32p)),
                   'bsa_sim_set_perf')

    def sim_read_perf(self):
        """(phase uint8, ax float64) of this rank's rows (full-n arrays, other rows 0)."""
        ph = np.zeros(self.n, np.uint8)
        ax = np.zeros(self.n)
        self.check(self.lib.bsa_sim_read_perf(self.h, ptr(ph, _c_u8p), ptr(ax)), 'bsa_sim_read_perf')
        return ph, ax

    def sim_update(self, **arrays):
        """bsa_sim_update: overwrite the given full-n state arrays (SIM_STATE_FIELDS
        names) of the resident sim, keeping its ASAS bookkeeping."""
        bad = set(arrays) - set(SIM_STATE_FIELDS)
        if bad:
            raise ValueError('unknown sim state fields %s' % sorted(bad))
        keep = {k: f64(v) for k, v in arrays.items() if v is not None}
        for k, a in keep.items():
            if len(a) != self.n:
                raise ValueError('sim state %s has length %d != %d' % (k, len(a), self.n))
        st = SimState(**{k: ptr(a) for k, a in keep.items()})
        self.check(self.lib.bsa_sim_update(self.h, ctypes.byref(st)), 'bsa_sim_update')

    def sim_create(self, state):
        """bsa_sim_create: append aircraft (every SIM_STATE_FIELDS array, m long);
        they take indices n..n+m-1 (Traffic.create, traffic.py:192-312)."""
        m = len(state['lat'])
        keep = {k: f64(state[k]) for k in SIM_STATE_FIELDS}
        for k, a in keep.items():
            if len(a) != m:
                raise ValueError('created state %s has length %d != %d' % (k, len(a), m))
        st = SimState(**{k: ptr(a) for k, a in keep.items()})
        self.gen += 1
        self.check(self.lib.bsa_sim_create(self.h, m, ctypes.byref(st)), 'bsa_sim_create')
        self.n += m
        st = self.sim_stats()
        self._rows = (st['row_begin'], st['row_end'])

    def sim_delete(self, idx):
        """bsa_sim_delete: remove aircraft ``idx``; the rest shift down in order
        (Traffic.delete, traffic.py:364-378)."""
        d = np.unique(np.asarray(idx, dtype=np.int64).ravel())
        self.gen += 1
        self.check(self.lib.bsa_sim_delete(self.h, len(d), ptr(d, _c_i64p)), 'bsa_sim_delete')
        self.n -= len(d)
        st = self.sim_stats()
        self._rows = (st['row_begin'], st['row_end'])

    def sim_step(self, nsteps=1):
        self.gen += 1
        self.check(self.lib.bsa_sim_step(self.h, int(nsteps)), 'bsa_sim_step')

    def sim_cd(self):
        """bsa_sim_cd: one CD call (detect -> resolver -> bookkeeping) without kinematics."""
        self.gen += 1
        self.check(self.lib.bsa_sim_cd(self.h), 'bsa_sim_cd')

    def sim_set_params(self, params):
        """bsa_sim_set_params: new rpz / hpz / tla / MVP switches for a running sim."""
        self.check(self.lib.bsa_sim_set_params(self.h, ctypes.byref(params)), 'bsa_sim_set_params')

    def sim_set_reso_lists(self, noreso=None, resooff=None):
        """bsa_sim_set_reso_lists: NORESO / RESOOFF membership (full-n bool-like arrays, None = empty)."""
        keep = [None if a is None else np.ascontiguousarray(a, dtype=np.uint8).ravel() for a in (noreso, resooff)]
        for a in keep:
            if a is not None and len(a) != self.n:
                raise ValueError('membership array has length %d != %d' % (len(a), self.n))
        self.check(self.lib.bsa_sim_set_reso_lists(self.h, ptr(keep[0], _c_u8p), ptr(keep[1], _c_u8p)),
                   'bsa_sim_set_reso_lists')

    def sim_read_asas(self):
        """bsa_sim_read_asas: asas trk / tas / vs / alt, asase / asasn, active and the
        ResumeNav drops of this rank's rows (full-n arrays, other rows 0)."""
        n = self.n
        o = {k: np.zeros(n) for k in ('trk', 'tas', 'vs', 'alt')}
        o.update(asase=np.zeros(n, np.float32), asasn=np.zeros(n, np.float32), active=np.zeros(n, np.uint8),
                 dropped=np.zeros(n, np.uint8))
        ao = AsasOut(**{k: ptr(o[k]) for k in ('trk', 'tas', 'vs', 'alt')}, asase=ptr(o['asase'], _c_fp),
                     asasn=ptr(o['asasn'], _c_fp), active=ptr(o['active'], _c_u8p), dropped=ptr(o['dropped'], _c_u8p))
        self.check(self.lib.bsa_sim_read_asas(self.h, ctypes.byref(ao)), 'bsa_sim_read_asas')
        o['active'] = o['active'].astype(bool)
        o['dropped'] = o['dropped'].astype(bool)
        return o

    def sim_read(self):
        n = self.n
        o = {k: np.empty(n) for k in SIM_OUT_FIELDS}
        o['active'] = np.empty(n, np.uint8)
        so = SimOut(**{k: ptr(o[k]) for k in SIM_OUT_FIELDS}, active=ptr(o['active'], _c_u8p))
        self.check(self.lib.bsa_sim_read(self.h, ctypes.byref(so)), 'bsa_sim_read')
        o['active'] = o['active'].astype(bool)
        return o

    def sim_stats(self):
        v = np.zeros(6, np.int64)
        self.check(self.lib.bsa_sim_stats(self.h, ptr(v, _c_i64p)), 'bsa_sim_stats')
        return dict(steps=int(v[0]), cd_calls=int(v[1]), n_conf=int(v[2]), n_los=int(v[3]),
                    row_begin=int(v[4]), row_end=int(v[5]))

    def set_row_bucket(self, width):
        """bsa_set_row_bucket: K2's per-row bucket width (0 = scatter into segments)."""
        self.check(self.lib.bsa_set_row_bucket(self.h, int(width)), 'bsa_set_row_bucket')

    def sim_row_ids(self):
        """Aircraft indices of this rank's rows, ascending (bsa_sim_row_ids): the
        rows of acdata / fetch_pairs' inconf and tcpamax after resident steps."""
        st = self.sim_stats()
        ids = np.empty(st['row_end'] - st['row_begin'], np.int32)
        self.check(self.lib.bsa_sim_row_ids(self.h, ptr(ids, _c_i32p)), 'bsa_sim_row_ids')
        return ids

    def sim_detect_rows(self, row_begin, row_end):
        """bsa_sim_detect_rows: the sim's detect of home rows [row_begin, row_end)
        (one rank's share, measured on one GPU); returns (n_conf, n_los)."""
        nc, nl = ctypes.c_int64(), ctypes.c_int64()
        self.check(self.lib.bsa_sim_detect_rows(self.h, int(row_begin), int(row_end), ctypes.byref(nc),
                                                ctypes.byref(nl)), 'bsa_sim_detect_rows')
        self.gen += 1
        self._rows = (int(row_begin), int(row_end))
        return nc.value, nl.value

    def sim_set_atmos(self, on=True):
        """bsa_sim_set_atmos: compute traf.p / rho / Temp = vatmos(alt) in every step."""
        self.check(self.lib.bsa_sim_set_atmos(self.h, int(bool(on))), 'bsa_sim_set_atmos')

    def sim_read_atmos(self):
        """(p, rho, Temp) of this rank's rows after the last step (full-n arrays)."""
        o = [np.zeros(self.n) for _ in range(3)]
        self.check(self.lib.bsa_sim_read_atmos(self.h, *[ptr(a) for a in o]), 'bsa_sim_read_atmos')
        return tuple(o)

    def sim_halo_stats(self):
        """bsa_sim_halo_stats: bytes received / sent per CD call, tiles received at the
        last CD call (or needed by the last bsa_sim_detect_rows share), regrowths."""
        v = np.zeros(4, np.int64)
        self.check(self.lib.bsa_sim_halo_stats(self.h, ptr(v, _c_i64p)), 'bsa_sim_halo_stats')
        return dict(rx_bytes=int(v[0]), tx_bytes=int(v[1]), tiles=int(v[2]), regrowths=int(v[3]))

    def sim_comm_stats(self):
        """bsa_sim_comm_stats: collectives since the last timing_reset (calls, bytes sent / received)."""
        v = np.zeros(3, np.int64)
        self.check(self.lib.bsa_sim_comm_stats(self.h, ptr(v, _c_i64p)), 'bsa_sim_comm_stats')
        return dict(calls=int(v[0]), tx_bytes=int(v[1]), rx_bytes=int(v[2]))

    def sim_set_halo_cap(self, sender, receiver, tiles):
        """bsa_sim_set_halo_cap (testing aid): this rank's copy of one tile capacity."""
        self.check(self.lib.bsa_sim_set_halo_cap(self.h, int(sender), int(receiver), int(tiles)),
                   'bsa_sim_set_halo_cap')

    def set_exact_fusion(self, on=True, max_records=64):
        """bsa_set_exact_fusion: K1b fused into the prefilter (default on); max_records < 64
        only to exercise the unfused retry in tests."""
        self.check(self.lib.bsa_set_exact_fusion(self.h, int(bool(on)), int(max_records)), 'bsa_set_exact_fusion')

    def exact_fusion_stats(self):
        """bsa_exact_fusion_stats: fused detects, their unfused retries, whether the last one fused."""
        v = np.zeros(3, np.int64)
        self.check(self.lib.bsa_exact_fusion_stats(self.h, ptr(v, _c_i64p)), 'bsa_exact_fusion_stats')
        return dict(fused=int(v[0]), retries=int(v[1]), last=bool(v[2]))

    def sim_probe_rank(self, rank, nranks):
        """bsa_sim_probe_rank (measurement aid): the one-rank sim's steps play rank `rank` of `nranks`."""
        self.check(self.lib.bsa_sim_probe_rank(self.h, int(rank), int(nranks)), 'bsa_sim_probe_rank')

    def sim_halo_recheck(self):
        """bsa_sim_halo_recheck (collective): the next exchange re-checks the region layout."""
        self.check(self.lib.bsa_sim_halo_recheck(self.h), 'bsa_sim_halo_recheck')

    def sim_asas_stats(self):
        """ASAS bookkeeping counts after the last CD call (resume_nav on); the
        unique / cumulative counts are None with several ranks."""
        v = np.zeros(6, np.int64)
        self.check(self.lib.bsa_sim_asas_stats(self.h, ptr(v, _c_i64p)), 'bsa_sim_asas_stats')
        opt = lambda x: None if x < 0 else int(x)
        return dict(resopairs=int(v[0]), confpairs_unique=opt(v[1]), lospairs_unique=opt(v[2]),
                    confpairs_all=opt(v[3]), lospairs_all=opt(v[4]), active=int(v[5]))

    def sim_resopairs(self):
        """This rank's resopairs as (idx1, idx2) int32 arrays, idx1-major; idx2 is
        -1 for an intruder deleted since the last CD call (bsa_sim_delete)."""
        cnt = np.zeros(1, np.int64)
        a = b = np.empty(0, np.int32)
        while True:
            self.check(self.lib.bsa_sim_resopairs(self.h, ptr(a, _c_i32p), ptr(b, _c_i32p), len(a),
                                                  ptr(cnt, _c_i64p)), 'bsa_sim_resopairs')
            if cnt[0] <= len(a):
                return a[:cnt[0]], b[:cnt[0]]
            a, b = np.empty(int(cnt[0]), np.int32), np.empty(int(cnt[0]), np.int32)

    # ---------------------------------------------------------------- kinematics
    KIN_OUT =('ax', 'delspd', 'cas', 'mach', 'gsnorth', 'gseast', 'gs', 'trk', 'coslat', 'az')

    def kinematics(self, simdt, state, inputs, winddim=0, windnorth=0.0, windeast=0.0):
        """bsa_kinematics.  ``state``: dict of float64 arrays tas, hdg, alt, vs,
        lat, lon (updated in place); ``inputs``: ptas, phdg, palt, pvs, bank,
        eps, accel.  Returns the output dict (incl. swhdgsel/swaltsel bool)."""
        n = len(state['tas'])
        io = KinIO()
        keep = []
        for k in ('ptas', 'phdg', 'palt', 'pvs', 'bank', 'eps', 'accel'):
            a = f64(inputs[k])
            keep.append(a)
            setattr(io, k, ptr(a))
        for k in ('tas', 'hdg', 'alt', 'vs', 'lat', 'lon'):
            a = state[k]
            if a.dtype != np.float64 or not a.flags.c_contiguous or len(a) != n:
                raise ValueError('state %s must be a contiguous float64 array' % k)
            setattr(io, k, ptr(a))
        out = {k: np.empty(n) for k in self.KIN_OUT}
        for k in self.KIN_OUT:
            setattr(io, k, ptr(out[k]))
        sw = {k: np.empty(n, np.uint8) for k in ('swhdgsel', 'swaltsel')}
        io.swhdgsel = ptr(sw['swhdgsel'], _c_u8p)
        io.swaltsel = ptr(sw['swaltsel'], _c_u8p)
        self.check(self.lib.bsa_kinematics(self.h, n, float(simdt), int(winddim), float(windnorth),
                                           float(windeast), ctypes.byref(io)), 'bsa_kinematics')
        out.update({k: v.astype(bool) for k, v in sw.items()})
        return out


_default = {}


def default_context(device=0):
    """Process-wide lazily created context per device (like the sim's single bs.traf)."""
    ctx = _default.get(device)
    if ctx is None:
        ctx = _default[device] = Context(device)
    return ctx
