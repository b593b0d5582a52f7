"""Clip-shard data parallelism for the sampling path.

Samples are independent (per-sample GroupNorm / LayerNorm / adaptor statistics,
eval BatchNorm, per-sample quantile, attention within a sample), so the global
'(b n)' batch is split into contiguous slices, one process per GPU, with no
collective on the data path; the noise stream is keyed by the global sample
index (`sample_base` = the slice start), so results do not depend on the rank
count. The one exchange step is the final gather of the generated videos to rank 0
(RCCL point-to-point over xGMI when the backend is "nccl").
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    """(world, rank, local_rank) from the torch.distributed.run environment."""
    return (int(os.environ.get('WORLD_SIZE', '1')), int(os.environ.get('RANK', '0')),
            int(os.environ.get('LOCAL_RANK', '0')))


def shard(global_batch, world, rank):
    """Contiguous slice [start, start + count) of the global batch for `rank`;
    the first global_batch % world ranks take one extra sample."""
    base, extra = divmod(global_batch, world)
    count = base + (1 if rank < extra else 0)
    start = rank * base + min(rank, extra)
    return start, count


def _host_staged():
    # gloo collectives take host tensors (the one-GPU rehearsal of the rank path)
    return dist.is_initialized() and dist.get_backend() == 'gloo'


def gather_shards(local, global_batch, world, dst=0):
    """Gather the ranks' slices (dim 0) into the global batch, in rank order, on rank `dst` only
    (the eval driver's consumer: the other ranks return None). Uneven slices are padded to the
    largest one for the collective. Over nccl (RCCL) the device tensors go straight into
    `dist.gather` (point-to-point xGMI transfers into dst: (world - 1) x cap x frame bytes arrive
    at dst, nothing at the others); over gloo they are staged through host memory. Without a
    process group (world 1) the local slice is the batch."""
    if not dist.is_initialized():
        assert world == 1, 'gather_shards: world > 1 without a process group'
        return local
    world = dist.get_world_size()
    rank = dist.get_rank()
    if _host_staged() and local.device.type != 'cpu':
        out = gather_shards(local.cpu(), global_batch, world, dst)
        return None if out is None else out.to(local.device)
    cap = -(-global_batch // world)
    pad = torch.zeros((cap,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
    dist.gather(pad, parts, dst=dst)
    if rank != dst:
        return None
    out = []
    for r in range(world):
        _, n = shard(global_batch, world, r)
        out.append(parts[r][:n])
    return torch.cat(out)


def max_over_ranks(value, device=None):
    """The slowest rank's wall time (bench.py's timing rule); over nccl the reduction runs on
    `device` (a one-element RCCL all-reduce)."""
    if not dist.is_initialized():
        return value
    t = torch.tensor([value], dtype=torch.float64, device=None if _host_staged() else device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())
