"""CPU, world_size 2 over gloo: the N>1 plumbing of animatable_nerf_amd.parallel — the mean
all-reduce of the flat gradient blob (training, DDP semantics of trainer.py:13-18) reproduces the
average of the per-rank oracle gradients, the max-over-ranks timing, and chunk-aligned ray shards."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from animatable_nerf_amd import parallel


def _free_port():
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        return s.getsockname()[1]


def _grads(seed):
    from oracle import restate
    from tests._common import batch_np, oracle_params, scene, to_torch
    torch.set_num_threads(1)
    sc = scene(0.05)
    ro, rd = sc.box_rays(48, seed=seed)
    rgb = np.random.default_rng(seed).random((48, 3)).astype(np.float32)
    b, _ = batch_np(sc, ro, rd, rgb=rgb)
    bt = to_torch(b)
    P = oracle_params(requires_grad=True)
    t_rand = torch.from_numpy(np.random.default_rng(seed + 1).random((bt['ray_o'].shape[1], 64)).astype(np.float32))
    ret = restate.render(P, bt, t_rand=t_rand)
    loss, _ = restate.loss_terms(ret, bt)
    loss.backward()
    return torch.cat([v.grad.reshape(-1) for v in P.values()])


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        r, w = parallel.init_from_env('gloo')
        assert (r, w) == (rank, world) and parallel.is_dist()
        g = _grads(100 + rank).clone()
        expect = (_grads(100) + _grads(101)) / 2
        parallel.allreduce_mean_(g)
        ok_grad = torch.allclose(g, expect, rtol=1e-6, atol=1e-12)
        tmax = parallel.max_over_ranks(1.0 + rank, 'cpu')
        q.put((rank, ok_grad, tmax))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gloo_world2_gradient_mean_and_timing():
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok_grad, tmax in res:
        assert ok_grad, rank
        assert tmax == 2.0


@pytest.mark.parametrize('n,world', [(262142, 8), (262142, 3), (1024, 2), (5000, 4), (2048, 8)])
def test_shard_chunks_cover_whole_chunks(n, world):
    spans = [parallel.shard_chunks(n, r, world) for r in range(world)]
    assert spans[0][0] == 0 and spans[-1][1] == n
    for (a0, a1), (b0, b1) in zip(spans, spans[1:]):
        assert a1 == b0
    for a0, a1 in spans:
        if a0 == a1:  # more ranks than chunks: trailing ranks are empty
            continue
        assert a0 % 2048 == 0 and (a1 % 2048 == 0 or a1 == n)


class _FakeRenderer:
    """Per-ray deterministic outputs (stand-in for the HIP renderer: the sharding, gather and PSNR
    plumbing is what this CPU test checks; tests/test_gpu_render.py checks the real shards)."""

    def render_device(self, b, bw_rows=True):
        o, d, near = b['ray_o'], b['ray_d'], b['near']
        rgb = torch.sigmoid(o * 3.0 + d * near[..., None])
        return {'rgb_map': rgb, 'acc_map': rgb.sum(-1) / 3.0, 'depth_map': near * 2.0,
                'raw': _per_sample(near, 4), 'pbw': _rows(o, 24, 0.0), 'tbw': _rows(o, 24, 1.0)}


def _per_sample(near, w):
    """(1, n*64, w) outputs that depend on each ray's own data only"""
    return (near[..., None, None] * torch.arange(64 * w, dtype=torch.float32).reshape(1, 1, 64, w)).reshape(1, -1, w)


def _rows(o, w, shift):
    """(1, m, w) row outputs: 0-2 rows per ray (by the ray's data), in ray order, like alpha_ind rows"""
    cnt = (o[0, :, 0] > 0).long() + (o[0, :, 1] > 0.5).long()
    r = torch.repeat_interleave(torch.arange(o.shape[1]), cnt)
    return (o[0, r, :1] + shift + torch.arange(w, dtype=torch.float32))[None]


def _frame(n):
    g = torch.Generator().manual_seed(5)
    return {'ray_o': torch.randn(1, n, 3, generator=g), 'ray_d': torch.randn(1, n, 3, generator=g),
            'near': torch.rand(1, n, generator=g), 'far': torch.rand(1, n, generator=g) + 1.0,
            'rgb': torch.rand(1, n, 3, generator=g), 'A': torch.eye(4).expand(1, 24, 4, 4)}


def _shard_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        parallel.init_from_env('gloo')
        b = _frame(n)
        ret = parallel.render_sharded(_FakeRenderer(), b, rows=True)
        full = _FakeRenderer().render_device(b)
        ok = all(torch.equal(ret[k], full[k]) for k in ('rgb_map', 'acc_map', 'depth_map', 'raw', 'pbw', 'tbw'))
        # default: the row outputs stay on their rank (no world-sized all-gather of the ~1 GB rows)
        lean = parallel.render_sharded(_FakeRenderer(), b)
        ok = ok and 'pbw' not in lean and 'tbw' not in lean and torch.equal(lean['rgb_map'], full['rgb_map'])
        mine = _FakeRenderer().render_device(parallel.shard_batch(b, rank, world, 2048)[0]) if ret['span'][1] > \
            ret['span'][0] else None
        ok = ok and (mine is None or torch.equal(lean['pbw_local'], mine['pbw']))
        s, e = ret['span']
        ok = ok and (s, e) == parallel.shard_chunks(n, rank, world)
        psnr = parallel.psnr_sharded(full['rgb_map'][:, s:e], b['rgb'][:, s:e])
        mse = float(((full['rgb_map'].double() - b['rgb'].double()) ** 2).mean())
        ok = ok and abs(psnr - (-10.0 * np.log10(mse))) < 1e-9
        q.put((rank, bool(ok)))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize('n,world', [(5000, 3), (5000, 4)])
def test_gloo_sharded_frame_render_gather_psnr(n, world):
    """One frame split over ranks by whole 2048-ray chunks (world 4 leaves one rank empty):
    all-gathered rgb/acc/depth equal the unsplit outputs in ray order on every rank, and the
    all-reduced PSNR equals the whole-frame formula."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, n, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in res:
        assert ok is True, (rank, ok)


def _fused_init_worker(rank, world, port, q):
    """FusedStep's constructor on CPU tensors (the C-ABI library loads without a GPU; nothing is
    launched): replicas that start from different weights, and an Adam state loaded on rank 0 only."""
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        from animatable_nerf_amd import config, network
        from animatable_nerf_amd.trainer import FusedStep
        parallel.init_from_env('gloo')
        torch.manual_seed(1000 + rank)  # a different init per rank (unseeded DDP-style start)
        net = network.Network()
        step = FusedStep(net, config.defaults())
        flat0 = step.flat.clone()
        got = [torch.empty_like(flat0) for _ in range(world)]
        dist.all_gather(got, flat0)
        same = all(torch.equal(got[0], x) for x in got)
        views_ok = torch.equal(torch.cat([p.detach().reshape(-1) for p in net.core_tensors()]), flat0)
        torch.manual_seed(7)
        ref_m = torch.rand(step.n)
        if rank == 0:  # a checkpoint read by rank 0 only
            sd = {'state': {}, 'param_groups': [{'lr': 3e-4}]}
            off = 0
            for i, p in enumerate(net.core_tensors()):
                k = p.numel()
                sd['state'][i] = {'exp_avg': ref_m[off:off + k].reshape(p.shape),
                                  'exp_avg_sq': 2 * ref_m[off:off + k].reshape(p.shape), 'step': torch.tensor(17.)}
                off += k
            step.load_adam_state_dict(sd)
        else:
            step.load_adam_state_dict({'state': {}, 'param_groups': [{'lr': 5e-4}]})
        adam_ok = torch.equal(step.m, ref_m) and torch.equal(step.v, 2 * ref_m) and step.t == 17 and \
            abs(step.lr - 3e-4) < 1e-12
        q.put((rank, bool(same and views_ok and adam_ok)))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gloo_fused_step_replicas_start_from_rank0():
    """DDP semantics of FusedStep (trainer.py:13-18): ranks built from different random weights all
    hold rank 0's blob after construction (and their parameter views alias it), and Adam moments /
    step count loaded on rank 0 only reach every rank."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_fused_init_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in res:
        assert ok is True, (rank, ok)


class _FakeSdfRenderer:
    """Stand-in for renderer_sdf.Renderer's chunk semantics: every chunk first widens tbounds in place
    (anisdf_pdf_network.py:204-206), and its rays' outputs depend on the widened bounds. A shard must
    therefore start from the bounds widened chunk_offset times (the real kernel: test_gpu_sdf.py)."""
    widens_tbounds = True

    def render_device(self, b, bw_rows=True, chunk_offset=0):
        from animatable_nerf_amd.renderer_sdf import widen_tbounds
        n = b['ray_o'].shape[1]
        tb = widen_tbounds(b['tbounds'], chunk_offset)
        rgb = torch.empty((1, n, 3))
        for c0 in range(0, n, 2048):
            tb = widen_tbounds(tb, 1)
            rgb[:, c0:c0 + 2048] = torch.sigmoid(b['ray_o'][:, c0:c0 + 2048] * tb[0, 1] + tb[0, 0])
        b['tbounds'].copy_(tb)
        o = b['ray_o']
        return {'rgb_map': rgb, 'acc_map': rgb.sum(-1), 'depth_map': b['near'] * 2.0, 'raw': _per_sample(b['near'], 4),
                'sdf': _per_sample(b['near'], 1), 'resd': _rows(o, 3, 0.0), 'gradients': _rows(o, 3, 2.0),
                'msk_sdf': _rows(o, 1, 3.0)[..., 0], 'msk_label': _rows(o, 1, 4.0)[..., 0]}


def _sdf_shard_worker(rank, world, port, n, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        parallel.init_from_env('gloo')
        b = _frame(n)
        b['tbounds'] = torch.tensor([[[-0.3, -0.9, -0.2], [0.3, 0.9, 0.2]]])
        full_b = {k: v.clone() for k, v in b.items()}
        full = _FakeSdfRenderer().render_device(full_b)
        ret = parallel.render_sharded(_FakeSdfRenderer(), b, rows=True)
        ok = all(torch.equal(ret[k], full[k]) for k in ('rgb_map', 'acc_map', 'depth_map', 'raw', 'sdf', 'resd',
                                                         'gradients', 'msk_sdf', 'msk_label'))
        ok = ok and torch.equal(b['tbounds'], full_b['tbounds'])
        q.put((rank, bool(ok)))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


@pytest.mark.parametrize('world', [3, 4])
def test_gloo_sharded_sdf_frame_keeps_tbounds_widening(world):
    """sdf_pdf frame split over ranks: each shard starts from tbounds widened once per preceding
    reference chunk, so the gathered outputs equal the single-GPU frame bit for bit, and every rank
    leaves batch['tbounds'] widened once per chunk of the whole frame."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_sdf_shard_worker, args=(r, world, port, 9000, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in res:
        assert ok is True, (rank, ok)


def _bucket_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        parallel.init_from_env('gloo')
        n = 1000
        blobs = [torch.arange(n + 4, dtype=torch.float32) * (r + 1) + r for r in range(world)]
        g = blobs[rank].clone()
        buckets = parallel.GradBuckets(g, [(0, 600), (600, n + 4)])
        buckets.reduce(0)
        buckets.reduce(1)
        buckets.wait()
        expect = sum(blobs) / world
        q.put((rank, bool(torch.allclose(g, expect, rtol=0, atol=1e-5))))
    except Exception as ex:  # pragma: no cover
        q.put((rank, repr(ex)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gloo_grad_buckets_mean_with_loss_tail():
    """FusedStep's reducer: the flat blob (gradients + the loss statistics in its last 4 floats) in two
    buckets, reduced one after the other, equals the mean over ranks everywhere."""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bucket_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, ok in res:
        assert ok is True, (rank, ok)


def _split_reduce_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    try:
        parallel.init_from_env('gloo')
        # argmin keys (pnorm bits << 32 | index): rank r has chunk 0's best on rank 1, chunk 1 empty everywhere
        # but rank 2, chunk 2 empty everywhere
        pn = [0.04, 0.01, 0.03]
        mins = torch.tensor([(int(np.float32(pn[rank]).view(np.uint32)) << 32) | (64 * rank + 5),
                             -1 if rank != 2 else (7 << 32) | 3, -1], dtype=torch.int64)
        parallel.reduce_keys_(mins, 0)
        # argmax keys: ordered(sigma) << 32 | ~index; the ordered bits of a positive sigma set the top bit
        def okey(sig, idx):
            u = int(np.float32(sig).view(np.uint32))
            o = (u ^ 0xffffffff) if u & 0x80000000 else (u | 0x80000000)
            v = (o << 32) | ((~idx) & 0xffffffff)
            return v - (1 << 64) if v >= (1 << 63) else v
        sig = [(2.5, 10), (3.0, 70), (3.0, 130)][rank]  # tie at 3.0: the lower index (rank 1's) wins
        maxs = torch.tensor([okey(*sig), okey(-1.0, rank)], dtype=torch.int64)
        parallel.reduce_keys_(maxs, 1)
        sums = torch.tensor([1.5 * (rank + 1), 1.0], dtype=torch.float32)
        parallel.reduce_keys_(sums, 2)
        # gradient shares are summed in a split, averaged across replicas otherwise
        blob = torch.full((6,), float(rank + 1))
        parallel.GradBuckets(blob, [(0, 3), (3, 6)], op='sum').reduce(0)
        q.put((rank, mins.tolist(), maxs.tolist(), sums.tolist(), blob.tolist(), okey(3.0, 70), okey(-1.0, 0)))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_gloo_world3_ray_split_reductions():
    """the three mid-step exchanges of a ray-split training step (trainer.FusedStep(ray_split=True),
    anr_train_hooks.reduce): min of argmin keys with empty markers, max of argmax keys (unsigned order,
    ties to the lower sample index), float sums; and the summed gradient buckets"""
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_split_reduce_worker, args=(r, 3, port, q)) for r in range(3)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in procs])
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    best = (int(np.float32(0.01).view(np.uint32)) << 32) | (64 + 5)
    for rank, mins, maxs, sums, blob, k_win, k_neg in res:
        assert mins == [best, (7 << 32) | 3, -1]
        assert maxs == [k_win, k_neg]
        assert sums == [9.0, 3.0]
        assert blob == [6.0, 6.0, 6.0] + [float(rank + 1)] * 3
    assert [parallel.ray_split_range(1024, r, 3) for r in range(3)] == [(0, 341), (341, 682), (682, 1024)]
