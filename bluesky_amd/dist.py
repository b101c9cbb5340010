"""Row-sharded multi-GPU plumbing: one process per GPU.

* ``row_range(n, rank, world)`` -- the contiguous ownship rows a rank owns
  (same formula as bsa_sim_init: ceil(n / world) rows per rank).
* ``rendezvous_unique_id(rank, world)`` -- ships the 128-byte RCCL id from
  rank 0 to the other local ranks through a file in /tmp (single node, the
  driver's ``torch.distributed.run`` launch); no PyTorch is imported, so the
  process only ever loads /opt/rocm's HIP runtime and RCCL.
* ``merge_rank_pairs(parts)`` -- the C2 pair gather: concatenating the row
  shards' canonically ordered pair lists in rank order IS the reference's
  global row-major order.
"""
import os
import time

import numpy as np


def env_rank_world():
    rank = int(os.environ.get('RANK', '0'))
    world = int(os.environ.get('WORLD_SIZE', '1'))
    local = int(os.environ.get('LOCAL_RANK', str(rank)))
    return rank, world, local


def row_range(n, rank, world):
    rpr = -(-n // world) if world > 0 else n
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


def merge_rank_pairs(parts):
    """Concatenate per-rank detect outputs (dicts of arrays) in rank order."""
    out = {}
    for k in parts[0]:
        vals = [p[k] for p in parts if p[k] is not None]
        out[k] = np.concatenate(vals) if vals else None
    return out
