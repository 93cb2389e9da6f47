"""GPU parity of the sdf_pdf ``Network.forward(wpts, viewdir, dists, batch)`` call surface
(anisdf_pdf_network.py:156-224) -- the call a stock ``tpose_renderer`` makes per chunk
(tpose_renderer.py:95; configs/sdf_pdf/anisdf_pdf_s9p.yaml:9-12) -- driven by a restated
``tpose_renderer`` chunk loop (the oracle's sampling / compositing / msk lists around the device
network), against the reference goldens G6 (eval) and G13 (training: loss.backward() through the
call, second order) and the oracle.

Tolerances as tests/test_gpu_sdf.py and tests/test_gpu_sdf_train.py: keep mask, observed-row count
and the in-place tbounds widening exact; raw / sdf / resd / rgb within 1e-4, gradients 2e-4; losses
1e-4 relative; parameter gradients within 5e-3 of each tensor's largest magnitude."""
import numpy as np
import pytest
import torch

from oracle import restate, restate_sdf

from ._common import golden, make_net_sdf, oracle_params_sdf, pdf_batch_np, pdf_scene, sdf_cfg, to_torch
from .test_gpu_sdf_train import GRAD_TOL, LOSS_RTOL, _oracle
from .test_oracle_sdf_train import g13_batch

pytestmark = pytest.mark.gpu
TOL = 1e-4
TOL_GRAD = 2e-4


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    return torch.device('cuda:0')


def _close(a, b, tol, what):
    a = a.detach().cpu().numpy() if torch.is_tensor(a) else a
    b = b.detach().cpu().numpy() if torch.is_tensor(b) else b
    assert a.shape == b.shape, (what, a.shape, b.shape)
    err = np.abs(a - b).max() if a.size else 0.0
    assert err <= tol, (what, err)


def _net(dev, precision='fp32'):
    cfg = sdf_cfg()
    cfg.render_precision = precision
    from animatable_nerf_amd import network, network_sdf
    from ._common import state_dict_sdf_np
    net = network_sdf.Network(cfg)
    network.load_numpy_state(net, state_dict_sdf_np())
    net = net.to(dev)
    net.train()  # run.py evaluates in train() mode (perturb 0, no grad)
    return net


@pytest.mark.parametrize('precision', ['fp32', 'bf16x3', 'bf16x6'])
def test_g6_network_forward_in_chunk_loop(dev, precision):
    """eval (no grad): tpose_renderer.get_pixel_value's sampling around net(wpts, viewdir, dists, batch)"""
    g = golden('g6_sdf_tiny')
    sc = pdf_scene()
    ro, rd = sc.box_rays(64, seed=2)
    b, _ = pdf_batch_np(sc, ro, rd)
    bt = to_torch(b, dev)
    net = _net(dev, precision)
    with torch.no_grad():
        pts, z = restate.sample_points(bt['ray_o'], bt['ray_d'], bt['near'], bt['far'], 64)
        wpts = pts.reshape(-1, 3)
        vd = bt['ray_d'][:, :, None].repeat(1, 1, 64, 1).reshape(-1, 3)
        dists = z[..., 1:] - z[..., :-1]
        dists = torch.cat([dists, dists[..., -1:]], dim=2).reshape(-1)
        ret = net(wpts, vd, dists, bt)
        assert set(ret) == {'raw', 'sdf', 'resd', 'gradients'}
        rgb_map, acc, depth, _ = restate.raw2outputs(ret['raw'].reshape(-1, 64, 4), z.reshape(-1, 64))
    keep = ret['sdf'][0, :, 0].cpu().numpy() != 10
    assert np.array_equal(keep, g['out_sdf'][0, :, 0] != 10)
    for k in ('raw', 'sdf', 'resd'):
        _close(ret[k], g['out_' + k], TOL, k)
    _close(ret['gradients'], g['out_gradients'], TOL_GRAD, 'gradients')
    _close(rgb_map[None], g['out_rgb_map'], TOL, 'rgb_map')
    _close(acc[None], g['out_acc_map'], TOL, 'acc_map')
    _close(depth[None], g['out_depth_map'], TOL, 'depth_map')
    assert np.array_equal(bt['tbounds'].cpu().numpy(), g['tbounds_after'])  # widened once (one chunk)


@pytest.mark.parametrize('n,precision', [(30, 'fp32'), (700, 'fp32'), (700, 'bf16x6')])
def test_network_forward_free_points_match_oracle(dev, n, precision):
    """arbitrary free samples (a partial 64-group; n < 45 takes torch's small-matmul path for world ->
    pose and the view directions), forced argmin over the call, tbounds widened once per call"""
    sc = pdf_scene()
    ro, rd = sc.box_rays(256, seed=77)
    b, _ = pdf_batch_np(sc, ro, rd)
    rng = np.random.default_rng(n)
    lo, hi = b['pbounds'][0]
    wpts = torch.from_numpy(rng.uniform(lo - 0.05, hi + 0.05, size=(n, 3)).astype(np.float32))
    vd = torch.nn.functional.normalize(torch.from_numpy(rng.normal(size=(n, 3)).astype(np.float32)), dim=1)
    dists = torch.full((n,), 0.01)
    bt = to_torch(b, dev)  # before the oracle call: bc shares b's arrays and is widened in place
    bc = to_torch(b)
    with torch.no_grad():
        ref = restate_sdf.network_forward(oracle_params_sdf(), wpts, vd, dists, bc)
    net = _net(dev, precision)
    for call in range(2):  # a second call sees the bounds the first widened
        with torch.no_grad():
            ret = net(wpts.to(dev), vd.to(dev), dists.to(dev), bt)
        if call == 0:
            assert np.array_equal(ret['sdf'][0, :, 0].cpu().numpy() != 10, ref['sdf'][0, :, 0].numpy() != 10)
            for k in ('raw', 'sdf', 'resd'):
                _close(ret[k], ref[k], TOL, k)
            _close(ret['gradients'], ref['gradients'], TOL_GRAD, 'gradients')
            assert torch.equal(bt['tbounds'].cpu(), bc['tbounds'])
    tb2 = restate_sdf.network_forward(oracle_params_sdf(), wpts, vd, dists, bc)  # noqa: F841 (widens bc again)
    assert torch.equal(bt['tbounds'].cpu(), bc['tbounds'])


def test_g13_backward_through_network_forward(dev, monkeypatch):
    """training: the reference's tpose_renderer + tpose_trainer losses around the device Network.forward
    under autograd; loss.backward() reaches every parameter through the call's raw / sdf / resd /
    gradients / observed_gradients (second order where the reference's create_graph is)."""
    from ._common import state_dict_sdf_np  # noqa: F401
    g = golden('g13_sdf_train')
    b = g13_batch(g)
    t_rand = torch.from_numpy(g['t_rand'])
    net = _net(dev)
    bd = {k: (v.to(dev) if torch.is_tensor(v) else v) for k, v in b.items()}
    calls = []

    def device_network(P, wpts, vd, dists, batch, norm_th=0.1):
        ret = net(wpts, vd, dists, batch)
        calls.append(sorted(ret))
        return ret
    monkeypatch.setattr(restate_sdf, 'network_forward_train', device_network)
    ret = restate_sdf.render_train(None, bd, t_rand=t_rand.to(dev))
    loss, stats = restate_sdf.loss_terms(ret, bd)
    loss.backward()
    assert calls and 'observed_gradients' in calls[0]
    assert int(ret['observed_gradients'].shape[1]) == int(g['n_observed'])
    assert np.array_equal(bd['tbounds'].cpu().numpy(), g['tbounds_after'])
    assert abs(loss.item() - float(g['loss'])) <= LOSS_RTOL * abs(float(g['loss']))
    for k in ('offset_loss', 'grad_loss', 'ograd_loss', 'mask_loss', 'img_loss'):
        ref = float(g['stat_' + k])
        assert abs(float(stats[k]) - ref) <= LOSS_RTOL * abs(ref) + 1e-6, (k, float(stats[k]), ref)
    params = dict(net.named_parameters())
    for key in g.files:
        if key.startswith('grad_') and key != 'grad_keys':
            ref = torch.from_numpy(g[key])
            err = (params[key[5:]].grad.cpu() - ref).abs().max().item()
            assert err <= GRAD_TOL * ref.abs().max().item() + 1e-9, (key, err)
    monkeypatch.undo()
    P, _, _, _, _ = _oracle(b, t_rand)
    checked = 0
    for name, prm in P.items():
        got = params[name].grad
        if prm.grad is None:
            assert got is None or got.abs().max().item() == 0, name
            continue
        scale = prm.grad.abs().max().item()
        err = (got.cpu() - prm.grad).abs().max().item()
        assert err <= GRAD_TOL * scale + 1e-9, (name, err, scale)
        checked += 1
    assert checked >= 60
