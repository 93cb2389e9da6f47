"""GPU parity of the sdf_pdf training step (config 5; anr_sdf_train_step through trainer_sdf) against
the reference's own step (golden G13: tpose_trainer.NetworkWrapper + loss.backward() with the KNN
stub) and the oracle (oracle/restate_sdf.py render_train + loss_terms, autograd with create_graph).

Tolerances (the training tests' bars, tests/test_gpu_train.py): every loss term within 1e-4
relative (+1e-6); every parameter gradient within 5e-3 of its tensor's largest magnitude, checked
on all 62 differentiated tensors against the oracle and on the golden's kept tensors against G13.
The observed-gradient row count and the in-place tbounds widening are exact. Both training
precisions (cfg.sdf_train_precision: 'fp32' exact MFMA, 'bf16x3' split-bf16 products) are held to
these same bars."""
import numpy as np
import pytest
import torch

from oracle import restate_sdf

from ._common import golden, make_net_sdf, oracle_params_sdf, pdf_batch_np, pdf_scene, sdf_cfg, to_torch
from .test_oracle_sdf_train import g13_batch

pytestmark = pytest.mark.gpu
LOSS_RTOL = 1e-4
GRAD_TOL = 5e-3


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    return torch.device('cuda:0')


PRECS = ('fp32', 'bf16x3')


def _device_step(dev, b, t_rand, iter_step, prec='fp32'):
    from animatable_nerf_amd import trainer_sdf
    from animatable_nerf_amd.renderer_sdf import Renderer
    net = make_net_sdf(dev)
    net.train()
    cfg = sdf_cfg()
    cfg.perturb = 1
    cfg.sdf_train_precision = prec
    r = Renderer(net, cfg)
    grads = [torch.zeros_like(t) for t in net.tensors()]
    loss8 = torch.zeros(trainer_sdf.NLOSS, device=dev)
    bd = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in b.items()}
    ret = trainer_sdf.sdf_train_step(r, bd, grads, loss8, t_rand.to(dev), iter_step=iter_step)
    torch.cuda.synchronize()
    names = [k for k, _ in net.named_parameters()]
    return dict(zip(names, [g.cpu() for g in grads])), loss8.cpu(), ret, bd


def _oracle(b, t_rand):
    P = {k: v.requires_grad_() for k, v in oracle_params_sdf().items()}
    bc = {k: (v.clone() if torch.is_tensor(v) else v) for k, v in b.items()}
    ret = restate_sdf.render_train(P, bc, t_rand=t_rand)
    loss, stats = restate_sdf.loss_terms(ret, bc)
    loss.backward()
    return P, ret, loss, stats, bc


def _check(grads, loss8, P, ret, loss, stats, label):
    n_obs = int(ret['observed_gradients'].shape[1]) if 'observed_gradients' in ret else 0
    assert int(loss8[6]) == n_obs, (label, int(loss8[6]), n_obs)
    assert int(loss8[7]) == int(ret['msk_sdf'].shape[1])
    for i, k in enumerate(('loss', 'offset_loss', 'grad_loss', 'ograd_loss', 'mask_loss', 'img_loss')):
        ref = float(loss.detach()) if k == 'loss' else float(stats[k].detach()) if k in stats else 0.0
        assert abs(float(loss8[i]) - ref) <= LOSS_RTOL * abs(ref) + 1e-6, (label, k, float(loss8[i]), ref)
    checked = 0
    for name, prm in P.items():
        if prm.grad is None:
            assert grads[name].abs().max().item() == 0, name
            continue
        ref = prm.grad
        scale = ref.abs().max().item()
        err = (grads[name] - ref).abs().max().item()
        assert err <= GRAD_TOL * scale + 1e-9, (label, name, err, scale)
        checked += 1
    assert checked >= 60


@pytest.mark.parametrize('prec', PRECS)
def test_g13_sdf_train_step_matches_reference_and_oracle(dev, prec):
    g = golden('g13_sdf_train')
    b = g13_batch(g)
    t_rand = torch.from_numpy(g['t_rand'])
    grads, loss8, ret, bd = _device_step(dev, b, t_rand, int(g['iter_step']), prec)
    # the reference step itself (G13)
    assert int(loss8[6]) == int(g['n_observed'])
    assert np.array_equal(bd['tbounds'].cpu().numpy(), g['tbounds_after'])
    assert abs(float(loss8[0]) - float(g['loss'])) <= LOSS_RTOL * abs(float(g['loss']))
    for i, k in enumerate(('offset_loss', 'grad_loss', 'ograd_loss', 'mask_loss', 'img_loss')):
        ref = float(g['stat_' + k])
        assert abs(float(loss8[1 + i]) - ref) <= LOSS_RTOL * abs(ref) + 1e-6, (k, float(loss8[1 + i]), ref)
    for key in g.files:
        if key.startswith('grad_') and key != 'grad_keys':
            ref = torch.from_numpy(g[key])
            err = (grads[key[5:]] - ref).abs().max().item()
            assert err <= GRAD_TOL * ref.abs().max().item() + 1e-9, (key, err)
    # every tensor against the oracle (same inputs)
    P, oret, oloss, ostats, _ = _oracle(b, t_rand)
    _check(grads, loss8, P, oret, oloss, ostats, 'g13 ' + prec)


@pytest.mark.parametrize('prec', PRECS)
def test_sdf_train_step_larger_batch_matches_oracle(dev, prec):
    """~700 box rays (one 2048-ray chunk, the reference's training batch shape), a mask_at_box with
    holes, iter_step past two mask-alpha milestones (alpha 200)"""
    sc = pdf_scene()
    ro, rd = sc.box_rays(700, seed=41)
    bnp, _ = pdf_batch_np(sc, ro, rd)
    R = bnp['ray_o'].shape[1]
    rng = np.random.default_rng(5)
    bnp['rgb'] = rng.random((1, R, 3)).astype(np.float32)
    bnp['mask_at_box'] = rng.random((1, R)) < 0.8
    b = to_torch(bnp)
    b['iter_step'] = 25000
    t_rand = torch.from_numpy(rng.random((R, 64)).astype(np.float32))
    grads, loss8, _, bd = _device_step(dev, b, t_rand, 25000, prec)
    P, oret, oloss, ostats, bc = _oracle(b, t_rand)
    assert torch.equal(bd['tbounds'].cpu(), bc['tbounds'])
    _check(grads, loss8, P, oret, oloss, ostats, '%s R=%d' % (prec, R))


def test_network_wrapper_backward_and_native_step(dev):
    """the reference Trainer loop over trainer_sdf.NetworkWrapper: loss.backward() fills every
    parameter's .grad with the device gradients; SdfStep (flat blobs + Adam) keeps weights finite"""
    from animatable_nerf_amd import trainer_sdf
    g = golden('g13_sdf_train')
    b = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in g13_batch(g).items()}
    net = make_net_sdf(dev)
    net.train()
    cfg = sdf_cfg()
    cfg.perturb = 1
    w = trainer_sdf.NetworkWrapper(net, cfg)
    ret, loss, stats, _ = w(dict(b, tbounds=b['tbounds'].clone()), t_rand=torch.from_numpy(g['t_rand']).to(dev))
    assert set(stats) == {'offset_loss', 'grad_loss', 'ograd_loss', 'mask_loss', 'img_loss', 'loss'}
    assert ret['rgb_map'].shape == (1, b['ray_o'].shape[1], 3)
    loss.backward()
    assert abs(loss.item() - float(g['loss'])) <= LOSS_RTOL * float(g['loss'])
    ref = torch.from_numpy(g['grad_resd_fc.weight'])
    got = net.resd_fc.weight.grad.cpu()
    assert (got - ref).abs().max().item() <= GRAD_TOL * ref.abs().max().item()
    step = trainer_sdf.SdfStep(make_net_sdf(dev), cfg)
    for _ in range(2):
        l8 = step.step(dict(b, tbounds=b['tbounds'].clone()))
    torch.cuda.synchronize()
    assert torch.isfinite(step.flat).all() and torch.isfinite(l8[:6]).all()
