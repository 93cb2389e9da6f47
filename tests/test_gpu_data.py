"""GPU: the eval-split ray pipeline (get_rays_within_bounds, if_nerf_data_utils.py:310-339) through
anr_camera_rays, bit-exact against the reference run (golden G8) for float64 and float32 cameras."""
import numpy as np
import pytest
import torch

from ._common import golden

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('tag', ['f64', 'f32'])
def test_camera_rays_bit_exact(tag):
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    from animatable_nerf_amd import data
    g = golden('g8_rays')
    H, W = int(g[tag + '_H']), int(g[tag + '_W'])
    ro, rd, near, far, mask, coord = data.get_rays_within_bounds(H, W, g[tag + '_K'], g[tag + '_R'], g[tag + '_T'],
                                                                 g['bounds'])
    assert np.array_equal(mask.cpu().numpy(), g[tag + '_mask'])
    for k, v in (('ray_o', ro), ('ray_d', rd), ('near', near), ('far', far)):
        assert np.array_equal(v.cpu().numpy(), g[tag + '_' + k]), k
    assert np.array_equal(coord.cpu().numpy(), np.argwhere(g[tag + '_mask']))


def test_camera_rays_feed_render():
    """Full-resolution render straight from camera parameters: rays never leave the device."""
    from animatable_nerf_amd import config, data
    from animatable_nerf_amd.renderer import Renderer
    from ._common import make_net, scene
    dev = torch.device('cuda:0')
    sc = scene(0.05)
    K = np.array([[300.0, 0, 128.0], [0, 300.0, 128.0], [0, 0, 1]])
    R = np.array([[1.0, 0, 0], [0, -1.0, 0], [0, 0, -1.0]])
    T = np.array([[0.0], [0.0], [3.0]])
    ro, rd, near, far, mask, _ = data.get_rays_within_bounds(256, 256, K, R, T, sc.bounds, dev)
    b = sc.batch_arrays(np.zeros((1, 3), np.float32), np.zeros((1, 3), np.float32), np.zeros(1, np.float32),
                        np.zeros(1, np.float32))
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()}
    batch.update(ray_o=ro[None], ray_d=rd[None], near=near[None], far=far[None])
    net = make_net(dev)
    net.train()
    cfg = config.defaults()
    cfg.perturb = 0
    out = Renderer(net, cfg).render_device(batch, bw_rows=False)
    assert out['rgb_map'].shape == (1, int(mask.sum()), 3)
    assert torch.isfinite(out['rgb_map']).all() and out['acc_map'].max() > 0.1


class _CountingRNG:
    """np.random.RandomState that counts randint calls (the reference's call sequence)."""

    def __init__(self, seed):
        self.rs = np.random.RandomState(seed)
        self.calls = []

    def randint(self, lo, hi, n):
        r = self.rs.randint(lo, hi, n)
        self.calls.append(np.asarray(r, dtype=np.int64))
        return r


@pytest.mark.parametrize('case', [0, 1])
def test_train_ray_sampler_bit_exact(case):
    """(f) train-split sampler sample_ray_h36m(split='train') through anr_train_ray_lists/gather vs the
    reference run (golden G12): same draws, and rays, float64 box test, rgb and coords bit-exact."""
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    from animatable_nerf_amd import data
    g = golden('g12_train_rays')
    p = f'c{case}_'
    rng = _CountingRNG(int(g[p + 'seed']))
    rgb, ro, rd, near, far, coord, mab = data.sample_ray_h36m(
        g[p + 'img'], g[p + 'msk'], g[p + 'K'], g[p + 'R'], g[p + 'T'], g['bounds'], int(g['nrays']), 'train',
        mask_bkgd=True, body_sample_ratio=0.5, face_sample_ratio=float(g[p + 'face_ratio']),
        bound_mask=g[p + 'bound_mask'], rng=rng)
    assert len(rng.calls) == int(g[p + 'n_randint'])
    assert np.array_equal(np.concatenate(rng.calls), g[p + 'draws'])
    for k, v in (('rgb', rgb), ('ray_o', ro), ('ray_d', rd), ('near', near), ('far', far), ('coord', coord)):
        assert np.array_equal(v.cpu().numpy(), g[p + k].astype(v.cpu().numpy().dtype)), k
    assert bool(mab.all()) and mab.numel() == int(g['nrays'])


def test_train_ray_sampler_edge_cases():
    """Edge cases of the device sampler: an empty body list raises like np.random.randint(0, 0, n);
    the pixel lists equal np.argwhere order; the test split returns the eval pipeline's rays with
    rgb zeroed outside the bound mask."""
    from animatable_nerf_amd import data
    g = golden('g12_train_rays')
    img, msk, bm = g['c1_img'], g['c1_msk'], g['c1_bound_mask']
    with pytest.raises(ValueError):
        data.sample_ray_h36m(img, np.zeros_like(msk), g['c1_K'], g['c1_R'], g['c1_T'], g['bounds'], 64, 'train',
                             bound_mask=bm, rng=np.random.RandomState(0))
    rgb, ro, rd, near, far, coord, mab = data.sample_ray_h36m(img, msk, g['c1_K'], g['c1_R'], g['c1_T'], g['bounds'],
                                                              0, 'test', bound_mask=bm)
    m = mab.cpu().numpy().reshape(120, 100)
    c = coord.cpu().numpy()
    assert np.array_equal(c, np.argwhere(m))
    ref = np.where((bm == 1)[..., None], img, 0)[c[:, 0], c[:, 1]]
    assert np.array_equal(rgb.cpu().numpy(), ref)


def test_resident_frames_feed_render():
    """ResidentFrames batches render on the device; a second batch of the same frame moves no
    per-frame tensor host to device and renders the same rays identically."""
    from animatable_nerf_amd import config
    from animatable_nerf_amd.data import ResidentFrames
    from animatable_nerf_amd.renderer import Renderer
    from ._common import batch_np, make_net, scene
    sc = scene(0.05)
    ro, rd = sc.box_rays(4096, seed=6)
    b, _ = batch_np(sc, ro, rd)
    rf = ResidentFrames('cuda:0')
    cfg = config.defaults()
    cfg.perturb = 0
    net = make_net(torch.device('cuda:0'))
    net.train()
    r = Renderer(net, cfg)
    o1 = r.render_device(rf.to_device(b), bw_rows=False)
    n = rf.uploads
    o2 = r.render_device(rf.to_device(b), bw_rows=False)
    assert rf.uploads == n > 0
    for k in ('rgb_map', 'acc_map', 'depth_map'):
        assert torch.equal(o1[k], o2[k]), k
