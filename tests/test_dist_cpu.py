"""CPU: the multi-rank host logic with world_size 2 over torch.distributed
gloo -- the library's row partition (home ranges of a spatial order, 512-row
tiles), the pair merge into the reference's global row-major order and the
RCCL id rendezvous.  The per-shard compute engine here is the oracle (no GPU:
the GPU path runs the same partition inside libbsaccel, and
tests/test_gpu_multirank.py checks it against this formula)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from bluesky_amd import dist, synth
from oracle import statebased as ocd


@pytest.mark.parametrize('n', [0, 1, 7, 511, 512, 513, 1000, 100000, 100001, 1000000])
@pytest.mark.parametrize('world', [1, 2, 3, 8])
def test_home_range_partitions(n, world):
    ranges = [dist.home_range(n, r, world) for r in range(world)]
    covered = np.concatenate([np.arange(a, b) for a, b in ranges]) if n else np.zeros(0)
    assert np.array_equal(covered, np.arange(n))
    rpr = ((n + world - 1) // world + 511) // 512 * 512
    for r, (a, b) in enumerate(ranges):
        assert a == min(n, r * rpr) and b - a <= rpr
        assert a % 512 == 0 or a == n          # whole 512-row tiles: a rank's row tiles are column tiles


def spatial_order(t):
    """A stand-in home order (any permutation is a valid home order; the
    library's is a 3-D Hilbert key): latitude bands, then
    longitude -- spatially compact ranges, rows of every rank interleaved in
    index order."""
    return np.lexsort((t.lon, np.floor(t.lat / 2.0)))


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
    t = synth.box(1500, 60.0, seed=41)
    h2id = spatial_order(t)
    rb, re = dist.home_range(t.ntraf, rank, world)
    rows = np.sort(h2id[rb:re])                   # the aircraft this rank owns (bsa_sim_row_ids)
    part = ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, rows=rows)
    parts = [None] * world
    tdist.all_gather_object(parts, (rows, part))
    if rank == 0:
        q.put(dist.merge_rank_pairs([p for _, p in parts], rows=[r for r, _ in parts]))
    tdist.barrier()
    tdist.destroy_process_group()


def test_sharded_detect_gloo_world2():
    """Two ranks over gloo, each detecting the rows of its home range (512-row
    tiles of a spatial order, so both ranks' rows interleave in index order);
    the merge is the reference's global row-major 8-tuple bit for bit."""
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
    t = synth.box(1500, 60.0, seed=41)
    full = ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD)
    assert len(full['ci']) > 0 and len(full['li']) > 0
    h2id = spatial_order(t)
    r0 = np.sort(h2id[:dist.home_range(t.ntraf, 0, 2)[1]])
    assert r0[-1] - r0[0] + 1 > len(r0)          # the ranks' rows interleave in index order
    for k in full:
        assert np.array_equal(merged[k], full[k]), k


def test_merge_rank_pairs_interleaved_rows():
    """Rows of the two ranks interleave in index order: a rank-order
    concatenation alone would not be row-major."""
    t = synth.box(700, 40.0, seed=5)
    full = ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD)
    rows = [np.arange(0, 700, 2), np.arange(1, 700, 2)]
    parts = [ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, rows=r) for r in rows]
    assert not np.array_equal(np.concatenate([p['ci'] for p in parts]), full['ci'])
    merged = dist.merge_rank_pairs(parts, rows=rows)
    for k in full:
        assert np.array_equal(merged[k], full[k]), k


def test_merge_rank_pairs_keys_are_explicit():
    """Per-row arrays are named (ROW_KEYS), never inferred from a length: an
    unknown key, or a per-row array of the wrong length, is an error, and a
    pair array some rank left as None is left out rather than scattered."""
    t = synth.box(300, 30.0, seed=3)
    rows = [np.arange(0, 300, 2), np.arange(1, 300, 2)]
    parts = [ocd.detect_arrays(t, t, synth.RPZ, synth.HPZ, synth.TLOOKAHEAD, rows=r) for r in rows]
    with pytest.raises(ValueError, match='unknown keys'):
        dist.merge_rank_pairs([dict(p, extra=np.zeros(len(r))) for p, r in zip(parts, rows)], rows=rows)
    with pytest.raises(ValueError, match='one entry per rank row'):
        dist.merge_rank_pairs([dict(p, inconf=p['inconf'][:-1]) for p in parts], rows=rows)
    half = [dict(parts[0], dcpa=None), dict(parts[1], dcpa=np.zeros(len(parts[1]['ci'])))]
    assert 'dcpa' not in dist.merge_rank_pairs(half, rows=rows)


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
