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
