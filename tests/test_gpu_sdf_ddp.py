"""Config 5's multi-rank training step: trainer_sdf.SdfStep at world 2 over gloo, both
ranks on the one GPU of the box (gloo moves the blob; the bench's N-GPU runs use RCCL). DDP semantics
(lib/train/trainers/trainer.py:13-18): every replica starts from rank 0's weights, the gradient blob
is mean-all-reduced — in buckets, the colour net's issued from the library's mid-step hook
(anr_sdf_train_step_hooked) while the rest of the backward runs — and the replicas stay identical.

Checks per rank: the hook fired; after one step the ranks hold identical parameter blobs and loss
vectors; the reduced gradient equals the mean of the two ranks' own gradients of their batches,
computed separately with the same (broadcast) weights (relative 1e-4 of each tensor's largest
magnitude: split-K atomics reorder the sums between the two evaluations)."""
import socket

import numpy as np
import pytest
import torch

from ._common import make_net_sdf, pdf_batch_np, pdf_scene, sdf_cfg, to_torch

pytestmark = pytest.mark.gpu


def _sdf_ddp_worker(rank, world, port, q):
    import os
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), HSA_ENABLE_IPC_MODE_LEGACY='0')
    try:
        from animatable_nerf_amd import parallel, trainer_sdf
        dev = torch.device('cuda:0')
        parallel.init_from_env('gloo')
        net = make_net_sdf(dev)
        if rank == 1:  # a replica built from other weights: the broadcast must replace them
            with torch.no_grad():
                for prm in net.parameters():
                    prm.add_(0.01 * torch.randn_like(prm))
        net.train()
        cfg = sdf_cfg()
        cfg.perturb = 1
        step = trainer_sdf.SdfStep(net, cfg, lr=0.0)
        sc = pdf_scene()
        ro, rd = sc.box_rays(160, seed=500 + rank)  # a different batch per rank
        bnp, _ = pdf_batch_np(sc, ro, rd)
        R = bnp['ray_o'].shape[1]
        bnp['rgb'] = np.random.default_rng(rank).random((1, R, 3)).astype(np.float32)
        b = to_torch(bnp, dev)
        b['iter_step'] = 12000
        t_rand = torch.rand((R, 64), device=dev, generator=torch.Generator(device=dev).manual_seed(7 + rank))
        # this rank's own gradient with the broadcast weights (no collective)
        local = [torch.zeros_like(t) for t in net.tensors()]
        loss_local = torch.zeros(trainer_sdf.NLOSS, device=dev)
        trainer_sdf.sdf_train_step(step.renderer, dict(b, tbounds=b['tbounds'].clone()), local, loss_local, t_rand,
                                   iter_step=12000)
        step.step(dict(b, tbounds=b['tbounds'].clone()), t_rand=t_rand)
        torch.cuda.synchronize()
        flat_local = torch.cat([g.reshape(-1) for g in local])
        gl = [torch.empty_like(flat_local) for _ in range(world)]
        dist.all_gather(gl, flat_local)
        mean = torch.stack(gl).mean(0)
        reduced = step.grad[:step.n]
        worst, off = 0.0, 0
        for t in net.tensors():
            k = t.numel()
            sc_ = mean[off:off + k].abs().max().item()
            if sc_ > 0:
                worst = max(worst, (reduced[off:off + k] - mean[off:off + k]).abs().max().item() / sc_)
            off += k
        flats = [torch.empty_like(step.flat) for _ in range(world)]
        dist.all_gather(flats, step.flat)
        losses = [torch.empty_like(step.loss8) for _ in range(world)]
        dist.all_gather(losses, step.loss8.contiguous())
        q.put((rank, bool(step._issued), bool(torch.equal(flats[0], flats[1])), bool(torch.equal(losses[0], losses[1])),
               worst, bool(torch.isfinite(step.flat).all())))
    except Exception as ex:  # pragma: no cover
        import traceback
        traceback.print_exc()
        q.put((rank, repr(ex), False, False, 1.0, False))
    finally:
        if dist.is_initialized():
            dist.destroy_process_group()


def test_sdf_step_two_ranks_mean_gradient_and_identical_replicas():
    import torch.multiprocessing as mp
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    with socket.socket() as s:
        s.bind(('127.0.0.1', 0))
        port = s.getsockname()[1]
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    procs = [ctx.Process(target=_sdf_ddp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, issued, same_flat, same_loss, worst, finite in res:
        assert issued is True, (rank, issued)
        assert same_flat and same_loss and finite, (rank, same_flat, same_loss, finite)
        assert worst <= 1e-4, (rank, worst)
