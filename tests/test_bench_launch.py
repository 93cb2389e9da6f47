"""bench.py's N-process contract on the CPU (gloo): ``--gpus N`` without a launcher spawns N ranks
itself, every rank checks WORLD_SIZE == --gpus, and rank 0 prints one JSON line with n_gpus = N.
ANR_BENCH_DRYRUN=1 runs the launch / rendezvous / barrier / max-over-ranks logic with no GPU work."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None):
    env = dict(os.environ, ANR_BENCH_DRYRUN='1', OMP_NUM_THREADS='1')
    for k in ('RANK', 'WORLD_SIZE', 'LOCAL_RANK', 'MASTER_ADDR', 'MASTER_PORT'):
        env.pop(k, None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py')] + args, env=env, capture_output=True,
                          text=True, timeout=240)


def test_gpus_flag_spawns_ranks():
    p = _run(['--gpus', '2', '--steps', '3', '--warmup', '0'])
    assert p.returncode == 0, p.stderr
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    assert len(lines) == 1, p.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d['n_gpus'] == 2 and d['ranks_seen'] == 2 and d['steps'] == 3


def test_world_mismatch_fails():
    p = _run(['--gpus', '2'], {'WORLD_SIZE': '1', 'RANK': '0', 'LOCAL_RANK': '0'})
    assert p.returncode != 0
    assert 'WORLD_SIZE=1' in (p.stderr + p.stdout)
