"""bench.py's multi-rank path on CPU: `--gpus 2` without a launcher spawns two
ranks (gloo, the --stub workload), shards the clip batch, all-gathers it back in
global order, takes the max-over-ranks time and prints n_gpus = 2; the step
accounting rounds the requested steps up to whole generations."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*args):
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    p = subprocess.run([sys.executable, os.path.join(REPO, 'bench.py'), '--stub', *args], env=env,
                       capture_output=True, text=True, timeout=180)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(l) for l in p.stdout.splitlines() if l.startswith('{')]
    return lines


def test_launcher_spawns_two_ranks():
    lines = _run('--gpus', '2', '--batch', '3', '--steps', '6', '--warmup', '0')
    assert len(lines) == 2 and lines[0]['partial'] and not lines[-1]['partial']
    res = lines[-1]
    assert res['n_gpus'] == 2
    assert res['config']['global_batch'] == 6
    assert res['generations'] == 2 and res['steps'] == 8  # 6 requested steps -> 2 stub generations of 4
    assert res['value'] > 0 and res['scaling'] == 'weak'


def test_single_rank_default():
    res = _run('--batch', '2', '--steps', '1')[-1]
    assert res['n_gpus'] == 1 and res['generations'] == 1 and res['steps'] == 4
