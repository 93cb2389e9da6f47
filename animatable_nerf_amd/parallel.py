"""One process per GPU over torch.distributed (RCCL as backend "nccl" on ROCm; gloo for CPU tests).

Render (config 2): frames / 2048-ray chunks are independent, so ranks never exchange data on the
hot path; ``shard_chunks`` gives each rank a contiguous run of whole reference chunks (preserving
the per-chunk argmin / argmax semantics) when one frame is split.
Training (configs 3/4): the only exchange is the mean all-reduce of the flat gradient blob per step
(DDP semantics of trainer.py:13-18), in two buckets overlapped with the backward (GradBuckets); the
loss scalars ride in the blob's tail, so the reported loss is the mean over ranks.
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


# ---- ray split of one training batch (north_star "rays-per-iteration shard"; anr_train_hooks) ----
def ray_split_range(n_rays, rank, world):
    """[start, end) of this rank's rays when one batch (a single reference chunk) is split over the ranks:
    contiguous, as even as possible."""
    return n_rays * rank // world, n_rays * (rank + 1) // world


_SIGN64 = -(1 << 63)
_MAX64 = (1 << 63) - 1


def reduce_keys_(t, op, group=None):
    """The exchange a ray-split training step makes through its reduce hook (in place, over ranks):
    op 0 = min of unsigned 64-bit keys whose all-ones value means "empty" (the per-chunk argmin of the
    prefilter, tpose_nerf_network.py:154), op 1 = max of unsigned 64-bit keys (the per-chunk argmax of
    sigma', :193-194), op 2 = float sum (the loss sums). ``t``: an int64 (ops 0, 1) or float32 (op 2)
    view of the device buffer. torch has no unsigned 64-bit reduction: the keys of op 0 stay below 2^63
    (non-negative float bits above the index), so only the empty marker is remapped; op 1 flips the top
    bit, which maps unsigned order onto signed order."""
    if not is_dist():
        return t
    if op == 0:
        t.masked_fill_(t == -1, _MAX64)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        t.masked_fill_(t == _MAX64, -1)
    elif op == 1:
        t.bitwise_xor_(_SIGN64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
        t.bitwise_xor_(_SIGN64)
    elif op == 2:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    else:
        raise ValueError(f'reduce op {op}')
    return t


class GradBuckets:
    """Mean all-reduce of a flat gradient blob in buckets, each issued as soon as the backward has
    finished it (DDP's reducer buckets parameters in reverse layer order and overlaps their all-reduce
    with the rest of the backward, trainer.py:13-18).

    ``bounds``: [(start, end), ...] in the order the backward finishes them. On a GPU blob the
    collectives run from a side stream: ``reduce(i, ready)`` makes it wait for the event ``ready``
    (recorded on the compute stream when bucket i is final; None: everything enqueued so far) and
    returns at once; ``wait()`` makes the current stream wait for every issued bucket. On a CPU blob
    (gloo) each ``reduce`` completes in place."""

    def __init__(self, blob, bounds, group=None, op='mean'):
        self.views = [blob[s:e] for s, e in bounds]
        self.group = group
        self.op = op  # 'mean' (DDP replicas) or 'sum' (a ray split: each rank holds a share of one gradient)
        self.comm = torch.cuda.Stream(device=blob.device) if blob.is_cuda else None

    def _reduce(self, v):
        if self.op == 'sum':
            dist.all_reduce(v, op=dist.ReduceOp.SUM, group=self.group)
        else:
            allreduce_mean_(v, self.group)

    def reduce(self, i, ready=None):
        if not is_dist():
            return
        if self.comm is None:
            self._reduce(self.views[i])
            return
        cur = torch.cuda.current_stream(self.views[i].device)
        with torch.cuda.stream(self.comm):
            if ready is not None:
                self.comm.wait_event(ready)
            else:
                self.comm.wait_stream(cur)
            self._reduce(self.views[i])

    def wait(self):
        if self.comm is not None and is_dist():
            torch.cuda.current_stream(self.views[0].device).wait_stream(self.comm)


def broadcast_(t, src=0, group=None):
    """In-place copy of rank ``src``'s tensor to every rank (what DistributedDataParallel does to
    the parameters and buffers when it is constructed, trainer.py:13-18)."""
    if is_dist():
        dist.broadcast(t, src=src, group=group)
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


# ---- one frame split over ranks (north_star "rays shard across the GPUs") ----
# Per-ray batch keys (tpose_dataset.py:236-277, batch dim 1): sliced per rank; everything else
# (A, volumes, bounds, R, Th, latent indices) is per frame and replicated.
RAY_KEYS = ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb')


def shard_batch(batch, rank, world, chunk=2048):
    """-> (this rank's batch, (start, end)): the rays of shard_chunks(R, rank, world, chunk)."""
    R = int(batch['ray_o'].shape[1])
    s, e = shard_chunks(R, rank, world, chunk)
    sub = dict(batch)
    for k in RAY_KEYS:
        v = batch.get(k)
        if torch.is_tensor(v) and v.dim() >= 2 and v.shape[1] == R:
            sub[k] = v[:, s:e]
    return sub, (s, e)


def gather_rays(t, n_rays, world, chunk=2048, group=None):
    """(1, r_local, ...) per rank -> (1, n_rays, ...) on every rank, in ray order: one all_gather of
    shards padded to the common size ceil(chunks / world) * chunk, then trimmed."""
    if world == 1 or not is_dist():
        return t
    n_chunks = (n_rays + chunk - 1) // chunk
    per = (n_chunks + world - 1) // world * chunk
    pad = torch.zeros((t.shape[0], per) + tuple(t.shape[2:]), dtype=t.dtype, device=t.device)
    pad[:, :t.shape[1]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad.contiguous(), group=group)
    out = []
    for r in range(world):
        s, e = shard_chunks(n_rays, r, world, chunk)
        out.append(parts[r][:, :e - s])
    return torch.cat(out, dim=1)


def gather_rows(t, group=None):
    """(1, m_r, ...) per rank, m_r varying -> (1, sum m_r, ...) on every rank in rank order (one all_gather
    of the counts, one of the rows padded to the largest count)."""
    if not is_dist():
        return t
    world = dist.get_world_size(group)
    n = torch.tensor([t.shape[1]], dtype=torch.int64, device=t.device)
    ns = [torch.empty_like(n) for _ in range(world)]
    dist.all_gather(ns, n, group=group)
    ns = [int(x.item()) for x in ns]
    mx = max(ns)
    pad = torch.zeros((t.shape[0], mx) + tuple(t.shape[2:]), dtype=t.dtype, device=t.device)
    pad[:, :t.shape[1]] = t
    parts = [torch.empty_like(pad) for _ in range(world)]
    dist.all_gather(parts, pad.contiguous(), group=group)
    return torch.cat([p[:, :k] for p, k in zip(parts, ns)], dim=1)


def render_sharded(renderer, batch, chunk=2048, group=None, rows=False):
    """Renderer.render_device over a whole frame with its rays split across the ranks by whole
    reference chunks (so every per-chunk argmin / argmax is the single-GPU one); the output keys of
    the reference's render dict are gathered to every rank in frame order: the per-ray maps and 'raw'
    by rays, and the per-chunk sdf_pdf 'msk_sdf' / 'msk_label' lists concatenated in rank order, which
    is chunk order. The large row outputs (aninerf 'pbw' / 'tbw' alpha_ind rows, sdf_pdf 'resd' /
    'gradients' kept rows: ~1.1 GB per 512x512 frame, padded to the largest rank's count by the
    all-gather) are gathered only when rows=True; otherwise each rank keeps its own shard's rows
    under 'pbw_local' etc. 'span' = this rank's rays [start, end)."""
    rank = dist.get_rank(group) if is_dist() else 0
    world = dist.get_world_size(group) if is_dist() else 1
    R = int(batch['ray_o'].shape[1])
    widens = getattr(renderer, 'widens_tbounds', False)
    tb0 = batch['tbounds'].detach().clone() if widens else None
    sub, (s, e) = shard_batch(batch, rank, world, chunk)
    dev = batch['ray_o'].device
    ns = int(getattr(renderer.cfg, 'N_samples', 64)) if hasattr(renderer, 'cfg') else 64
    if e > s:
        # the sdf_pdf renderer widens tbounds per chunk: this shard starts at reference chunk s / chunk
        out = renderer.render_device(sub, chunk_offset=s // chunk) if widens else renderer.render_device(sub)
    else:  # more ranks than chunks: an empty shard
        out = {'rgb_map': torch.zeros((1, 0, 3), device=dev), 'acc_map': torch.zeros((1, 0), device=dev),
               'depth_map': torch.zeros((1, 0), device=dev), 'raw': torch.zeros((1, 0, 4), device=dev)}
        if widens:
            out.update(sdf=torch.zeros((1, 0, 1), device=dev), resd=torch.zeros((1, 0, 3), device=dev),
                       gradients=torch.zeros((1, 0, 3), device=dev), msk_sdf=torch.zeros((1, 0), device=dev),
                       msk_label=torch.zeros((1, 0), device=dev))
        else:
            out.update(pbw=torch.zeros((1, 0, 24), device=dev), tbw=torch.zeros((1, 0, 24), device=dev))
    if widens:  # every rank leaves the frame's bounds as the whole single-GPU render does
        from .renderer_sdf import widen_tbounds
        with torch.no_grad():
            batch['tbounds'].copy_(widen_tbounds(tb0, (R + chunk - 1) // chunk))
    ret = {k: gather_rays(out[k], R, world, chunk, group) for k in ('rgb_map', 'acc_map', 'depth_map')}
    for k, w in (('raw', 4), ('sdf', 1)):  # per-sample outputs, gathered as per-ray rows
        if k in out:
            v = out[k].reshape(1, -1, ns * w)
            ret[k] = gather_rays(v, R, world, chunk, group).reshape(1, -1, w)
    for k in ('pbw', 'tbw', 'resd', 'gradients', 'msk_sdf', 'msk_label'):
        if k not in out:
            continue
        if rows or k in ('msk_sdf', 'msk_label'):
            ret[k] = gather_rows(out[k], group)
        else:
            ret[k + '_local'] = out[k]
    ret['span'] = (s, e)
    return ret


def psnr_sharded(rgb_pred, rgb_gt, group=None):
    """A18 PSNR (lib/evaluators/if_nerf.py:15-18: mse over the rendered in-box rays, -10 log10 mse)
    of a frame whose rays are split over the ranks: one all-reduce of [sum of squared errors,
    element count] (float64)."""
    d = (rgb_pred.double() - rgb_gt.double())
    t = torch.stack([(d * d).sum(), torch.tensor(float(d.numel()), dtype=torch.float64, device=d.device)])
    if is_dist():
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    return float(-10.0 * torch.log10(t[0] / t[1]))
