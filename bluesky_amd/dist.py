"""Row-sharded multi-GPU plumbing: one process per GPU.

* ``home_range(n, rank, world)`` -- the contiguous range of HOME positions a
  rank owns, exactly as bsa_sim_init partitions them (bsa_sim.hip): ``rpr`` =
  ceil(n / world) rounded up to a whole 512-row tile, rank r owns
  ``[r * rpr, min(n, (r + 1) * rpr))``.  Home positions are the spatial (home)
  order of the initial traffic, so the aircraft a rank owns
  are ``h2id[rb:re]`` -- not an index range; ``bsa_sim_row_ids`` lists them.
* ``rendezvous_unique_id(rank, world)`` -- ships the 128-byte RCCL id from
  rank 0 to the other local ranks through a file in /tmp (single node, the
  driver's ``torch.distributed.run`` launch); no PyTorch is imported, so the
  process only ever loads /opt/rocm's HIP runtime and RCCL.
* ``merge_rank_pairs(parts, rows)`` -- the C2 pair gather on the host: each
  rank's pairs are row-major over ITS rows (aircraft-index order), and the rows
  of different ranks interleave in index order, so the reference's global
  row-major order (np.where, StateBasedCD.py:93-101) is the rank-order
  concatenation stably sorted by row (what bsa_gather_pairs does on the root,
  home_pairs_to_ids in bsa_ctx.hip).
"""
import os
import time

import numpy as np


def env_rank_world():
    rank = int(os.environ.get('RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', str(rank)))
    return rank, world, local


HOME_TILE = 512   # kTile: a rank's home range is whole 512-row tiles (bsa_sim.hip, sim_rpr)


def home_range(n, rank, world):
    """Home positions [rb, re) of ``rank``: bsa_sim_init's partition."""
    world = max(int(world), 1)
    rpr = ((n + world - 1) // world + HOME_TILE - 1) // HOME_TILE * HOME_TILE
    rb = min(n, rank * rpr)
    return rb, min(n, rb + rpr)


def _rdv_path():
    key = '%s_%s_%s' % (os.environ.get('TORCHELASTIC_RUN_ID', 'x'), os.environ.get('MASTER_PORT', '0'),
                        os.getppid())
    return os.path.join(os.environ.get('BSACCEL_RDV_DIR', '/tmp'), 'bsaccel_rdv_%s.id' % key)


def rendezvous_unique_id(rank, world, make_id, timeout=300.0):
    """Rank 0 creates the id with ``make_id()`` and publishes it; others poll."""
    path = _rdv_path()
    if world == 1:
        return make_id()
    if rank == 0:
        uid = make_id()
        tmp = path + '.tmp%d' % os.getpid()
        with open(tmp, 'wb') as f:
            f.write(uid)
        os.replace(tmp, path)
        return uid
    t0 = time.time()
    while True:
        try:
            with open(path, 'rb') as f:
                uid = f.read()
            if len(uid) == 128:
                return uid
        except FileNotFoundError:
            pass
        if time.time() - t0 > timeout:
            raise TimeoutError('no RCCL id from rank 0 at %s' % path)
        time.sleep(0.05)


def cleanup_rendezvous(rank):
    if rank == 0:
        try:
            os.remove(_rdv_path())
        except FileNotFoundError:
            pass


def init_comm(ctx, rank, world):
    """Create the RCCL communicator of this rank's context (collective)."""
    from . import _lib
    if world == 1 or getattr(ctx, 'comm_rank_world', None) == (rank, world):
        return                        # one communicator per context, reused by later sims
    uid = rendezvous_unique_id(rank, world, _lib.comm_unique_id)
    ctx.comm_init(world, rank, uid)
    ctx.allreduce_max([0.0])          # everyone has joined
    cleanup_rendezvous(rank)
    ctx.comm_rank_world = (rank, world)


PAIR_KEYS = {'ci': ('ci', 'cj', 'qdr', 'dist', 'tcpa', 'tinconf', 'dcpa'), 'li': ('li', 'lj')}
ROW_KEYS = ('inconf', 'tcpamax')   # per-row arrays, in each rank's row order


def merge_rank_pairs(parts, rows=None):
    """Merge per-rank detect outputs (dicts of arrays as fetch_pairs /
    oracle detect_arrays return them, pairs row-major over the rank's rows)
    into the global row-major result.  ``rows``: each rank's row ids (the
    per-row arrays inconf / tcpamax are in that order); their union must be
    every row once.  Pair arrays are concatenated in rank order and stably
    sorted by row index (a row belongs to one rank, so its pairs stay in order).
    Keys other than PAIR_KEYS' and ROW_KEYS are an error; a key some rank left
    as None is left out."""
    known = set(ROW_KEYS).union(*PAIR_KEYS.values())
    for p in parts:
        extra = set(p) - known
        if extra:
            raise ValueError('merge_rank_pairs: unknown keys %s' % sorted(extra))
    out = {}
    for lead, keys in PAIR_KEYS.items():
        if lead not in parts[0]:
            continue
        order = np.argsort(np.concatenate([p[lead] for p in parts]), kind='stable')
        for k in keys:
            if k in parts[0] and all(p.get(k) is not None for p in parts):
                out[k] = np.concatenate([p[k] for p in parts])[order]
    if rows is not None:
        ids = np.concatenate([np.asarray(r, dtype=np.int64) for r in rows])
        n = len(ids)
        if not np.array_equal(np.sort(ids), np.arange(n)):
            raise ValueError('rank rows do not partition 0..%d' % (n - 1))
        for k in ROW_KEYS:
            if not all(p.get(k) is not None for p in parts):
                continue
            if any(len(p[k]) != len(r) for p, r in zip(parts, rows)):
                raise ValueError('merge_rank_pairs: %s does not have one entry per rank row' % k)
            v = np.concatenate([p[k] for p in parts])
            full = np.empty(n, dtype=v.dtype)
            full[ids] = v
            out[k] = full
    return out
