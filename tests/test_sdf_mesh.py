"""sdf_pdf mesh path (sdf_mesh_renderer.py:16-110), CPU side: the oracle's SDF network and deformed-SDF
gradient against the reference run (golden G14, oracle/gen_goldens.py --sdf-mesh), the oracle's
marching cubes against the triangulation recorded there, and the host component pass that stands in
for trimesh's split (trimesh is not installed: parity unpinned, checked by its properties)."""
import numpy as np
import torch

from animatable_nerf_amd.renderer_sdf_mesh import largest_component
from oracle import mcubes, restate_sdf

from ._common import assert_golden_equal, golden, oracle_params_sdf


def test_oracle_sdf_network_and_deformed_gradient_match_g14():
    g = golden('g14_sdf_mesh')
    P = oracle_params_sdf()
    torch.set_num_threads(1)
    with torch.no_grad():
        out = restate_sdf.sdf_network(P, torch.from_numpy(g['sdfnet_x']))
    assert_golden_equal(out, g['sdfnet_out'], 'sdf_network')
    batch = {'poses': torch.from_numpy(g['poses'])}
    n = 400  # a slice of the vertices (the gradient pass is autograd on the CPU)
    gr, y = restate_sdf.gradient_of_deformed_sdf(P, torch.from_numpy(g['godf_x'][:, :n].copy()), batch)
    assert_golden_equal(gr.detach(), g['godf_g'][:, :n], 'gradient_of_deformed_sdf')
    assert_golden_equal(y.detach(), g['godf_y'][:, :n], 'sdf at the vertices')


def test_oracle_marching_cubes_is_the_recorded_triangulation():
    g = golden('g14_sdf_mesh')
    v, t = mcubes.marching_cubes(g['cube'].astype(np.float64), float(g['mc_th']))
    assert np.array_equal(t, g['mc_triangles'])
    assert np.array_equal(v, g['mc_vertices'])
    # the reference's vertex transform (:78-79) of the (single-component) mesh
    np.testing.assert_array_equal(g['vertex'], (g['mc_vertices'] - 10) * 0.02 + g['tbounds'][0, 0].astype(np.float64))


def _box(offset, scale=1.0):
    v = (np.array([[x, y, z] for x in (0, 1) for y in (0, 1) for z in (0, 1)], np.float64) * scale) + offset
    q = [(0, 1, 3, 2), (4, 6, 7, 5), (0, 4, 5, 1), (2, 3, 7, 6), (0, 2, 6, 4), (1, 5, 7, 3)]
    t = [(a, b, c) for a, b, c, d in q] + [(a, c, d) for a, b, c, d in q]
    return v, np.array(t, np.int64)


def test_largest_component_keeps_the_biggest_watertight_piece():
    v1, t1 = _box(0.0)
    v2, t2 = _box(5.0, 2.0)
    # a third, larger but open piece (one face missing): not watertight, so never kept
    v3 = np.concatenate([_box(-9.0)[0], _box(-9.0)[0][:4] + 0.5])
    t3 = _box(-9.0)[1][:-1]
    # interleave the pieces' vertices so that the kept piece's vertex order must be preserved
    v = np.concatenate([v1, v2, v3])
    t = np.concatenate([t1, t2 + 8, t3 + 16])
    perm = np.random.default_rng(0).permutation(len(v))
    inv = np.argsort(perm)
    vp, tp = v[perm], inv[t]
    kv, kt = largest_component(vp, tp)
    assert len(kv) == 8 and len(kt) == 12  # the two boxes tie on vertices: the first root (lowest face) wins
    # the kept faces are one closed box with its vertices in their original relative order
    e = np.sort(np.concatenate([kt[:, [0, 1]], kt[:, [1, 2]], kt[:, [2, 0]]]), axis=1)
    _, cnt = np.unique(e, axis=0, return_counts=True)
    assert np.all(cnt == 2)
    src = np.nonzero(np.isin(np.arange(len(vp)), np.unique(tp[:12])))[0]
    np.testing.assert_array_equal(kv, vp[src])
    # bigger watertight piece wins
    v4, t4 = _box(20.0)
    big_v = np.concatenate([v1, v4, v4 + 100.0])
    big_t = np.concatenate([t1, t4 + 8, t4 + 16, np.array([[8, 9, 16]])])  # pieces 2 and 3 glued by a face:
    kv, kt = largest_component(big_v, big_t)                                 # not watertight -> box 1
    assert len(kv) == 8 and np.allclose(kv, v1)


def test_largest_component_no_watertight_piece_returns_input():
    v, t = _box(0.0)
    kv, kt = largest_component(v, t[:-1])
    assert kv is v and np.array_equal(kt, t[:-1])
