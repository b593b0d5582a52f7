"""The N > 1 clip-shard path on CPU (gloo, world size 2 and 3): contiguous
slices keyed by the global sample index, gathered back to rank 0 in rank order, and the
max-over-ranks timing reduction. The per-sample "sampler" here is a CPU stand-in
whose output depends only on (seed, global sample index) — the property the
native Philox stream has (tests/test_gpu_parity.py checks that bitwise on GPU)."""
import importlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from tests.golden_inputs import PKG

D = importlib.import_module(PKG + '.dist')


def fake_sample(seed, sample_base, count):
    rows = []
    for i in range(count):
        g = torch.Generator().manual_seed(seed * 100003 + sample_base + i)
        rows.append(torch.randn(3, 4, 5, generator=g))
    return torch.stack(rows) if rows else torch.zeros(0, 3, 4, 5)


def _worker(rank, world, port, global_batch, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    try:
        start, count = D.shard(global_batch, world, rank)
        local = fake_sample(7, start, count)
        full = D.gather_shards(local, global_batch, world)
        slow = D.max_over_ranks(float(rank + 1))
        if rank == 0:
            q.put((full, slow))
        else:
            assert full is None  # only the destination rank materialises the batch
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


@pytest.mark.parametrize('world,global_batch', [(2, 8), (2, 5), (3, 7)])
def test_clip_shard_gather_matches_unsharded(world, global_batch):
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, global_batch, q)) for r in range(world)]
    for p in procs:
        p.start()
    full, slow = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert torch.equal(full, fake_sample(7, 0, global_batch))
    assert slow == float(world)


def test_shard_covers_batch():
    for world in (1, 2, 3, 8):
        for gb in (1, 7, 8, 33):
            spans = [D.shard(gb, world, r) for r in range(world)]
            assert sum(c for _, c in spans) == gb
            assert all(spans[r][0] + spans[r][1] == spans[r + 1][0] for r in range(world - 1))
