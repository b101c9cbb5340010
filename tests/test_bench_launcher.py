"""CPU: bench.py's rank launcher.  ``--gpus N`` without a
launcher starts N ranks itself; a launcher world that disagrees with --gpus is
an error.  ``--dry-run`` resolves and reports the ranks without touching HIP."""
import json
import os
import subprocess
import sys
import time

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(REPO, 'bench.py')


def run(args, **env):
    e = {k: v for k, v in os.environ.items() if k not in ('RANK', 'LOCAL_RANK', 'WORLD_SIZE', 'LOCAL_WORLD_SIZE')}
    e.update(env)
    return subprocess.run([sys.executable, BENCH] + args, env=e, capture_output=True, text=True, timeout=120)


@pytest.mark.parametrize('n', [2, 3])
def test_gpus_n_without_launcher_spawns_n_ranks(n):
    r = run(['--gpus', str(n), '--dry-run'])
    assert r.returncode == 0, r.stderr
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1, r.stdout                       # rank 0's line only
    d = json.loads(lines[0])
    assert d['n_gpus'] == n and d['rank'] == 0
    seen = sorted(ln for ln in r.stderr.splitlines() if ln.startswith('bench.py dry run'))
    assert seen == ['bench.py dry run: rank %d of %d (local %d)' % (k, n, k) for k in range(n)]


def test_world_size_disagreeing_with_gpus_exits_nonzero():
    r = run(['--gpus', '8', '--dry-run'], RANK='0', LOCAL_RANK='0', WORLD_SIZE='1')
    assert r.returncode != 0
    assert 'refusing' in r.stderr
    assert r.stdout.strip() == ''


def test_launcher_world_matching_gpus_runs_as_that_rank():
    r = run(['--gpus', '2', '--dry-run'], RANK='1', LOCAL_RANK='1', WORLD_SIZE='2')
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == ''                          # not rank 0: no line
    assert 'rank 1 of 2' in r.stderr


def test_one_gpu_default_is_world_one():
    r = run(['--dry-run'])
    assert r.returncode == 0, r.stderr
    assert json.loads(r.stdout)['n_gpus'] == 1


def test_spawn_ranks_returns_first_failure():
    sys.path.insert(0, REPO)
    import bench
    code = 'import os, sys, time; r = int(os.environ["RANK"]); time.sleep(60 if r == 0 else 0); sys.exit(5)'
    t0 = time.time()
    rc = bench.spawn_ranks(2, ['--dry-run'], cmd=[sys.executable, '-c', code])
    assert rc == 5                      # rank 1 failed ...
    assert time.time() - t0 < 30        # ... and rank 0 (waiting, as in a collective) was ended
