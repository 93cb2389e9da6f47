"""One process per GPU over torch.distributed (RCCL as backend "nccl" on ROCm; gloo for CPU tests).

Render (config 2): frames / 2048-ray chunks are independent, so ranks never exchange data on the
hot path; ``shard_chunks`` gives each rank a contiguous run of whole reference chunks (preserving
the per-chunk argmin / argmax semantics) when one frame is split.
Training (configs 3/4): the only exchange is one mean all-reduce of the flat gradient blob per step
(DDP semantics of trainer.py:13-18), plus scalar loss statistics.
"""
import os

import torch
import torch.distributed as dist


def env_rank():
    return int(os.environ.get('RANK', 0)), int(os.environ.get('WORLD_SIZE', 1)), int(os.environ.get('LOCAL_RANK', 0))


def init_from_env(backend='nccl', device=None):
    rank, world, _ = env_rank()
    if world > 1 and not dist.is_initialized():
        kw = {'device_id': device} if (backend == 'nccl' and device is not None) else {}
        dist.init_process_group(backend, **kw)
    return rank, world


def is_dist():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def allreduce_mean_(t, group=None):
    """In-place mean over ranks (one collective for the whole blob)."""
    if is_dist():
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
        t.div_(dist.get_world_size(group))
    return t


def max_over_ranks(x, device):
    t = torch.tensor([float(x)], device=device, dtype=torch.float64)
    if is_dist():
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def shard_chunks(n_rays, rank, world, chunk=2048):
    """[start, end) rays of this rank: a contiguous run of whole chunks (the last rank takes the
    partial chunk), so every rank sees exactly the reference's chunk boundaries."""
    n_chunks = (n_rays + chunk - 1) // chunk
    per = (n_chunks + world - 1) // world
    c0 = min(n_chunks, rank * per)
    c1 = min(n_chunks, c0 + per)
    return min(n_rays, c0 * chunk), min(n_rays, c1 * chunk)
