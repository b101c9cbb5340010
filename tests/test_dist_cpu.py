"""CPU: the multi-rank host logic (row partition, pair gather, id rendezvous)
with world_size 2 over torch.distributed gloo; the per-shard compute engine
here is the oracle (the GPU path runs the same partition inside libbsaccel)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from bluesky_amd import dist, synth
from oracle import statebased as ocd


@pytest.mark.parametrize('n', [0, 1, 7, 8, 9, 1000, 100001])
@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_row_range_partitions(n, world):
    ranges = [dist.row_range(n, r, world) for r in range(world)]
    covered = np.concatenate([np.arange(a, b) for a, b in ranges]) if n else np.zeros(0)
    assert np.array_equal(covered, np.arange(n))
    rpr = -(-n // world)
    assert all(b - a <= rpr for a, b in ranges)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _gloo_worker(rank, world, port, q):
    import torch.distributed as tdist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    tdist.init_process_group('gloo', rank=rank, world_size=world)
    t = synth.box(600, 40.0, seed=41)
    rb, re = dist.row_range(t.ntraf, rank, world)
    part = ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, rows=np.arange(rb, re))
    parts = [None] * world
    tdist.all_gather_object(parts, part)
    if rank == 0:
        q.put(dist.merge_rank_pairs(parts))
    tdist.barrier()
    tdist.destroy_process_group()


def test_sharded_detect_gloo_world2():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gloo_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    merged = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    t = synth.box(600, 40.0, seed=41)
    full = ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD)
    assert len(full['ci']) > 0
    for k in full:
        assert np.array_equal(merged[k], full[k]), k


def _rdv_worker(rank, world, rdv_dir, q):
    os.environ['BSACCEL_RDV_DIR'] = rdv_dir
    uid = dist.rendezvous_unique_id(rank, world, lambda: bytes(range(128)), timeout=60)
    q.put((rank, uid))


def test_rendezvous_ships_id(tmp_path):
    ctx = mp.get_context('fork')
    q = ctx.Queue()
    procs = [ctx.Process(target=_rdv_worker, args=(r, 3, str(tmp_path), q)) for r in range(3)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=60) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert set(got) == {0, 1, 2}
    assert all(v == bytes(range(128)) for v in got.values())
