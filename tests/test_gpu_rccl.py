"""GPU: the RCCL code path bench.py's N > 1 run takes (dist backend "nccl" = RCCL on ROCm), at
world size 1 on the box's one MI355X: process-group initialisation bound to the device,
dist.gather_shards (device tensors straight into dist.gather, padded slices, rank-order
reassembly) and dist.max_over_ranks (a one-element device all-reduce). The multi-rank behaviour
of the same functions is covered on gloo (tests/test_dist_gloo.py) and, through bench.py's ranks,
by tests/test_gpu_bench_ranks.py."""
import importlib
import socket

import pytest
import torch
import torch.distributed as dist

from tests.golden_inputs import PKG

pytestmark = pytest.mark.gpu
D = importlib.import_module(PKG + '.dist')


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def test_rccl_world1_gather_and_max():
    dev = torch.device('cuda:0')
    torch.cuda.set_device(dev)
    dist.init_process_group('nccl', init_method=f'tcp://127.0.0.1:{_free_port()}', rank=0, world_size=1,
                            device_id=dev)
    try:
        assert dist.get_backend() == 'nccl'
        g = torch.Generator(device=dev).manual_seed(3)
        local = torch.randn(5, 3, 4, 8, 8, device=dev, generator=g)
        full = D.gather_shards(local, 5, 1)
        torch.cuda.synchronize()
        assert full.device == dev and torch.equal(full, local)
        assert D.max_over_ranks(1.25, device=dev) == 1.25
    finally:
        dist.destroy_process_group()
