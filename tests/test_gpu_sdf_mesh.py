"""GPU parity of the sdf_pdf mesh path (sdf_mesh_renderer.py:16-110) and the network helper methods it
calls, against the reference run G14 (oracle/gen_goldens.py --sdf-mesh): tpose_human.sdf_network,
gradient_of_deformed_sdf, calculate_bigpose_smpl_bw on the device, the padded SDF cube, the device
marching cubes, the posed vertices, and renderer_sdf_mesh.Renderer.render end to end (the component
split is trimesh's, absent here: parity unpinned, the recorded mesh is a single piece)."""
import numpy as np
import pytest
import torch

from animatable_nerf_amd import synthetic
from animatable_nerf_amd.renderer_mesh import marching_cubes
from animatable_nerf_amd.renderer_sdf_mesh import Renderer, largest_component

from ._common import golden, make_net_sdf

pytestmark = pytest.mark.gpu
TOL = 1e-4


@pytest.fixture(scope='module')
def dev():
    if not torch.cuda.is_available():
        pytest.fail('GPU test run without a GPU')
    return torch.device('cuda:0')


def _batch(g, dev):
    b = synthetic.sdf_mesh_scene(voxel=0.02)
    assert tuple(b['pts'].shape[1:4]) == tuple(g['grid_shape'])
    for k in ('A', 'big_A', 'poses', 'weights', 'tvertices', 'tbounds', 'R', 'Th'):
        assert np.array_equal(b[k], g[k]), k
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(dev) for k, v in b.items()}


def _close(got, ref, tol, what):
    err = float((got.detach().cpu().double() - torch.from_numpy(np.asarray(ref)).double()).abs().max())
    assert err <= tol, (what, err)


def test_helper_methods_match_g14(dev):
    g = golden('g14_sdf_mesh')
    net = make_net_sdf(dev)
    net.train()
    batch = _batch(g, dev)
    with torch.no_grad():
        out = net.tpose_human.sdf_network(torch.from_numpy(g['sdfnet_x']).to(dev), batch)
    assert out.shape == (3000, 257)
    _close(out, g['sdfnet_out'], TOL, 'sdf_network')
    assert torch.equal(net.tpose_human.sdf_network.sdf(torch.from_numpy(g['sdfnet_x']).to(dev), batch)[:, 0],
                       out[:, 0])
    # the reference's batchify_normal_sdf: 32k-point chunks through gradient_of_deformed_sdf (:37-46)
    x = torch.from_numpy(g['godf_x']).to(dev)
    normals, sdfs = [], []
    for i in range(0, x.shape[1], 1024):
        nrm, s = net.gradient_of_deformed_sdf(x[:, i:i + 1024], batch)
        normals.append(nrm.detach().cpu().numpy())
        sdfs.append(s.detach().cpu().numpy())
    _close(torch.from_numpy(np.concatenate(normals, 1)), g['godf_g'], 2e-4, 'gradient_of_deformed_sdf')
    _close(torch.from_numpy(np.concatenate(sdfs, 1)), g['godf_y'], TOL, 'deformed sdf')
    ib = {'tbw': torch.from_numpy(g['bw_vol'][None]).to(dev), 'tbounds': torch.from_numpy(g['bw_bounds'][None]).to(dev)}
    bw = net.calculate_bigpose_smpl_bw(torch.from_numpy(g['bw_pts']).to(dev), ib)
    assert bw.shape == g['bigpose_bw'].shape
    _close(bw, g['bigpose_bw'], 1e-6, 'calculate_bigpose_smpl_bw')  # the exact grid_sample order


def test_cube_marching_cubes_and_posed_vertices_match_g14(dev):
    g = golden('g14_sdf_mesh')
    net = make_net_sdf(dev)
    net.train()
    batch = _batch(g, dev)
    r = Renderer(net)
    cube = r.sdf_volume(batch)
    ref = torch.from_numpy(g['cube'])
    assert cube.shape == ref.shape
    c = cube.cpu()
    assert torch.equal(c == -10, ref == -10)  # the KNN inside filter and the padding, exact
    _close(c[ref != -10], ref[ref != -10].numpy(), TOL, 'cube (-sdf)')
    # the device marching cubes over the recorded cube: the recorded triangulation (oracle/mcubes.py)
    v, t = marching_cubes(ref.to(dev), float(g['mc_th']), 0)
    assert torch.equal(t.cpu(), torch.from_numpy(g['mc_triangles']))
    assert torch.equal(v.cpu(), torch.from_numpy(g['mc_vertices']))
    with torch.no_grad():
        posed = r.posed_vertices(g['vertex'], batch)
    _close(posed, g['posed_vertex'], TOL, 'posed_vertex')


def test_render_end_to_end(dev):
    """renderer_sdf_mesh.Renderer.render vs the reference's outputs, restricted to the largest watertight
    component of the recorded mesh (the reference run's trimesh stub kept it whole)"""
    g = golden('g14_sdf_mesh')
    net = make_net_sdf(dev)
    net.train()
    from animatable_nerf_amd import config
    cfg = config.subject('anisdf_pdf_s9p', perturb=0)
    cfg.voxel_size = [0.02, 0.02, 0.02]
    ret = Renderer(net, cfg).render(_batch(g, dev))
    kv, kt = largest_component(g['mc_vertices'], g['mc_triangles'])
    assert len(kv) == len(g['mc_vertices']) and np.array_equal(kt, g['mc_triangles'])  # one watertight piece
    assert np.array_equal(ret['triangle'], g['triangle'])
    assert ret['vertex'].shape == g['vertex'].shape and ret['posed_vertex'].shape == g['posed_vertex'].shape
    # Marching cubes places a vertex at (iso - f0) / (f1 - f0) along its edge: where the cube's two values
    # nearly agree, the cube's own <= 1e-4 difference moves the vertex by much more (measured: 5 of 6,348
    # coordinates by up to 2.3e-4). So the vertices are checked exactly against the oracle's marching
    # cubes of the cube this render produced. The posed vertices are held to 1e-4 on >= 99.5 % of the
    # vertices and 1e-3 everywhere: a vertex displaced by even 1e-5 can change its 5 nearest SMPL vertices
    # and so its blend weights (measured: one of 2,116 vertices moved 2.3e-4 for a 1e-5 displacement);
    # test_cube_marching_cubes_and_posed_vertices_match_g14 checks the posed vertices of the reference's
    # own vertices at 1e-4 everywhere.
    cube = Renderer(net, cfg).sdf_volume(_batch(g, dev)).cpu().numpy().astype(np.float64)
    from oracle import mcubes
    mv, mt = mcubes.marching_cubes(cube, 0.0)
    kv2, kt2 = largest_component(mv, mt)
    assert np.array_equal(ret['triangle'], kt2)
    np.testing.assert_array_equal(ret['vertex'], (kv2 - 10) * 0.02 + g['tbounds'][0, 0].astype(np.float64))
    dv = np.abs(ret['vertex'] - g['vertex']).max(1, keepdims=True)
    assert float(dv.max()) < 1e-3
    perr = np.abs(ret['posed_vertex'] - g['posed_vertex']).max(1)
    assert float(np.mean(perr <= TOL)) >= 0.995 and float(perr.max()) <= 1e-3, (float(np.mean(perr <= TOL)), perr.max())
