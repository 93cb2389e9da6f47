"""GPU parity of config 5's novel-view / pose-sequence renderer (``tpose_renderer_mmsk`` over the sdf_pdf
network, configs/sdf_pdf/anisdf_pdf_s9p.yaml:108-139): renderer_sdf_mmsk.Renderer (the visibility filter in
the sdf front-end) against the oracle's mmsk loop (oracle/restate.py render_mmsk, pinned by golden G9) around
the sdf network restatement (oracle/restate_sdf.py network_forward, pinned by G6 / G7): rgb / acc / depth
within 1e-4 in every render precision, and batch['tbounds'] widened exactly as often as the reference
calls the network (only chunks with a visible sample)."""
import numpy as np
import pytest
import torch

from animatable_nerf_amd import synthetic
from oracle import restate, restate_sdf

from ._common import make_net_sdf, oracle_params_sdf, pdf_batch_np, pdf_scene, sdf_cfg, to_torch

pytestmark = pytest.mark.gpu
CHUNK = 512


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    return torch.device('cuda:0')


def _batch():
    """3 chunks of box rays, then a partial chunk of rays along the box's top-back edge (x direction,
    y within 0.01 of the top face, z within 0.01 of the back face: above the body, which ends 0.05 below
    the padded box) whose samples all project outside a training view's mask: a chunk without a network
    call, hence no tbounds widening"""
    sc = pdf_scene()
    ro, rd = sc.box_rays(3 * CHUNK, seed=41)
    rng = np.random.Generator(np.random.PCG64(3))
    b = sc.pbounds.astype(np.float64)
    o2 = np.stack([np.full(200, b[0, 0] - 0.5), b[1, 1] - rng.uniform(0.001, 0.01, 200),
                   b[0, 2] + rng.uniform(0.001, 0.01, 200)], 1)
    d2 = np.broadcast_to(np.array([1.0, 0.0, 0.0]), (200, 3))
    ro = np.concatenate([ro, o2.astype(np.float32)])
    rd = np.concatenate([rd, d2.astype(np.float32)])
    bb, mask = pdf_batch_np(sc, ro, rd)
    Ks, RTs, msks, H, W = synthetic.training_views(sc.pvertices, n_views=3, dilate=0)
    bb.update(Ks=Ks[None], RT=RTs[None], msks=msks[None], H=np.array([H]), W=np.array([W]))
    n_corner = int(mask[3 * CHUNK:].sum())
    return bb, n_corner


@pytest.mark.parametrize('precision', ['fp32', 'bf16x6', 'bf16x3'])
def test_sdf_mmsk_render_matches_oracle(dev, precision):
    from animatable_nerf_amd.renderer_sdf_mmsk import Renderer
    b, n_corner = _batch()
    R = b['ray_o'].shape[1]
    assert R > 3 * CHUNK and n_corner > 0
    bt = to_torch(b, dev)  # before the oracle call: bc shares b's arrays and is widened in place
    bc = to_torch(b)
    torch.set_num_threads(16)
    calls = []

    def net_fwd(P, wpts, viewdir, dists, batch):
        calls.append(len(wpts))
        return restate_sdf.network_forward(P, wpts, viewdir, dists, batch)
    with torch.no_grad():
        ref = restate.render_mmsk(oracle_params_sdf(), bc, chunk=CHUNK, net_forward=net_fwd)
    n_chunks = (R + CHUNK - 1) // CHUNK
    assert 0 < len(calls) < n_chunks  # the corner chunk has no visible sample: no call, no widening
    net = make_net_sdf(dev)
    net.train()
    cfg = sdf_cfg()
    cfg.render_precision = precision
    cfg.chunk = CHUNK
    out = Renderer(net, cfg).render(bt)
    assert set(out) == {'rgb_map', 'acc_map', 'depth_map'}
    for k in ('rgb_map', 'acc_map', 'depth_map'):
        assert out[k].shape == ref[k].shape, k
        err = float((out[k] - ref[k]).abs().max())
        assert err <= 1e-4, (k, err)
    assert torch.equal(bt['tbounds'].cpu(), bc['tbounds'])  # widened once per network call
