"""Strong split of one training iteration (north_star "rays-per-iteration shard across the GPUs";
SURVEY.md §8(d)(4) "1,024 split (strong)"): the same 1,024-ray batch on every rank, each rank training on
a contiguous share of its rays, the chunk-wide decisions of the reference's single 2048-ray chunk -- the
prefilter's forced argmin (tpose_nerf_network.py:154) and alpha_ind's forced argmax (:193-194) -- and the
loss sums exchanged mid-step (anr_train_hooks.reduce), the gradient shares summed over ranks.

Bar: the split step's losses equal the single-rank step's within 1e-5 relative and its summed gradient
within 1e-4 of each tensor's largest magnitude (fp32 sums in another order: split-K atomics, per-rank
partial sums); world 2 and 4 over gloo, the ranks sharing the box's one GPU."""
import numpy as np
import pytest
import torch

from ._common import batch_np, make_net, scene, to_torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    return torch.device('cuda:0')


def _batch(dev, n=1024, seed=51):
    sc = scene(0.05)
    ro, rd = sc.box_rays(n + 64, seed=seed)
    b, _ = batch_np(sc, ro, rd, rgb=np.random.default_rng(seed).random((n + 64, 3)).astype(np.float32))
    b = {k: (v[:, :n] if k in ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb') else v)
         for k, v in b.items()}
    b['mask_at_box'] = b['mask_at_box'].copy()
    b['mask_at_box'][0, ::7] = False  # rays outside the image mask: counted by the global ray total only
    t_rand = np.random.default_rng(seed + 1).random((n, 64)).astype(np.float32)
    return to_torch(b, dev), torch.from_numpy(t_rand).to(dev)


def _cfg(prec):
    from animatable_nerf_amd import config
    cfg = config.defaults()
    cfg.perturb = 1
    cfg.train_precision = prec
    return cfg


def _split_worker(rank, world, port, prec, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY='0')
    try:
        from animatable_nerf_amd import parallel
        from animatable_nerf_amd.trainer import FusedStep
        dev = torch.device('cuda:0')
        parallel.init_from_env('gloo')
        net = make_net(dev)
        net.train()
        step = FusedStep(net, _cfg(prec), lr=0.0, ray_split=True)
        assert step.ray_split
        bt, t_rand = _batch(dev)
        l3 = step.step(bt, t_rand=t_rand)
        torch.cuda.synchronize()
        if rank == 0:
            q.put((rank, l3[:3].cpu().numpy(), step.grad[:step.n].cpu().numpy(), step.renderer.last_counts))
        else:
            q.put((rank, l3[:3].cpu().numpy(), None, None))
    except Exception as ex:  # pragma: no cover
        import traceback
        q.put((rank, repr(ex) + traceback.format_exc(), None, None))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def _run_world(world, prec):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_split_worker, args=(r, world, port, prec, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=300) for _ in procs], key=lambda x: x[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert not isinstance(r[1], str), r[1]
    return res


@pytest.mark.parametrize('world,prec', [(2, 'fp32'), (4, 'fp32'), (2, 'bf16')])
def test_ray_split_step_equals_single_rank_step(dev, world, prec):
    from animatable_nerf_amd.trainer import FusedStep
    net = make_net(dev)
    net.train()
    step = FusedStep(net, _cfg(prec), lr=0.0)
    bt, t_rand = _batch(dev)
    l_ref = step.step(bt, t_rand=t_rand)[:3].cpu().numpy()
    g_ref = step.grad[:step.n].cpu().numpy()
    res = _run_world(world, prec)
    for rank, l3, _, _ in res:  # every rank reports the batch's losses
        np.testing.assert_allclose(l3, l_ref, rtol=1e-5, atol=0, err_msg=f'rank {rank}')
    g = res[0][2]
    off = 0
    for p in net.core_tensors():
        k = p.numel()
        a, b = g[off:off + k], g_ref[off:off + k]
        scale = np.abs(b).max()
        assert np.abs(a - b).max() <= 1e-4 * scale + 1e-12, (off, np.abs(a - b).max(), scale)
        off += k
