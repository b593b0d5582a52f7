"""GPU: bench.py's real multi-rank path (NativeWorkload, dist.shard, gather_shards,
max_over_ranks) on one MI355X — two ranks over gloo sharing cuda:0 — against the
single-rank run of the same global batch: the gathered videos must be bitwise equal
(clips from one seed sliced per rank, noise keyed by global sample index)."""
import json
import os
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(tmp_path, gpus, batch, tag):
    dump = str(tmp_path / f'{tag}.pt')
    cmd = [sys.executable, os.path.join(REPO, 'bench.py'), '--gpus', str(gpus), '--batch', str(batch),
           '--sampling-steps', '4', '--warmup', '1', '--no-cpu-baseline', '--no-roofline', '--dump', dump]
    if gpus > 1:
        cmd += ['--dist-backend', 'gloo']
    env = {k: v for k, v in os.environ.items() if k not in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK')}
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=400)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [l for l in p.stdout.splitlines() if l.startswith('{')]
    return json.loads(lines[-1]), torch.load(dump, weights_only=True)


def test_two_gloo_ranks_equal_one_rank(tmp_path):
    r1, v1 = _run(tmp_path, 1, 4, 'one')
    r2, v2 = _run(tmp_path, 2, 2, 'two')
    assert r1['n_gpus'] == 1 and r2['n_gpus'] == 2
    assert r2['config']['global_batch'] == 4 and r2['config']['batch_per_gpu'] == 2
    assert v1.shape == v2.shape == (4, 3, 2 + 28, 64, 64)
    assert torch.isfinite(v2).all()
    assert torch.equal(v1, v2)
