"""CPU: the mesh path's oracle.

* get_alpha restatement (oracle/restate.py) bit-exact vs the reference run (golden G10: the cube the
  reference renderer hands to mcubes, and 4096-point batchify chunks incl. a forced-argmin-only
  chunk and a 30-point chunk on torch's small-matmul path);
* the marching-cubes case table (tools/gen_mc_table.py) and its numpy restatement
  (oracle/mcubes.py): closed, consistently oriented, outward-wound surfaces; one vertex per
  crossing edge; Euler characteristic 2 for a sphere. PyMCubes itself is absent: parity of the
  triangulation against it is unpinned.
"""
import numpy as np
import pytest
import torch

from ._common import assert_golden_equal, golden, oracle_params


def _g10_batch():
    g = golden('g10_mesh')
    keys = ('A', 'pbw', 'tbw', 'pbounds', 'wbounds', 'tbounds', 'R', 'Th', 'latent_index')
    return g, {k: torch.from_numpy(np.ascontiguousarray(g[k])) for k in keys}


@pytest.fixture(scope='module')
def g10_pts():
    from animatable_nerf_amd import synthetic
    g, _ = _g10_batch()
    b = synthetic.mesh_scene(voxel=0.02)
    assert np.array_equal(b['inside'], g['inside']) and np.array_equal(b['wbounds'], g['wbounds'])
    return b['pts'][0][b['inside'][0].astype(bool)]


def test_get_alpha_oracle_matches_reference_cube(g10_pts):
    from oracle import restate
    torch.set_num_threads(1)
    g, batch = _g10_batch()
    with torch.no_grad():
        a = restate.mesh_alpha(oracle_params(), torch.from_numpy(g10_pts), batch).numpy()
    assert float(g['mesh_th']) == 5.0
    assert_golden_equal(a, g['alpha_inside'], 'alpha_inside')
    assert np.array_equal(a != 0, g['alpha_inside'] != 0)  # the kept pattern is exact


def test_get_alpha_oracle_matches_reference_small_chunks():
    from oracle import restate
    torch.set_num_threads(1)
    g, batch = _g10_batch()
    with torch.no_grad():
        a = restate.mesh_alpha(oracle_params(), torch.from_numpy(g['pts_b']), batch, chunk=int(g['chunk_b'])).numpy()
    assert_golden_equal(a, g['alpha_b'], 'alpha_b')
    assert np.array_equal(a != 0, g['alpha_b'] != 0)
    # the far chunk keeps exactly its argmin point; the 30-point tail chunk ran
    assert len(a) == 17 * 4096 + 30
    far = a[16 * 4096:17 * 4096]
    assert (far != 0).sum() == 1


def _closed_oriented(tris):
    """every directed edge once and its reverse once: closed 2-manifold, consistent winding"""
    e = np.concatenate([tris[:, [0, 1]], tris[:, [1, 2]], tris[:, [2, 0]]])
    d = set(map(tuple, e))
    return len(d) == len(e) and all((b, a) in d for a, b in d)


def _signed_volume(v, t):
    a, b, c = v[t[:, 0]], v[t[:, 1]], v[t[:, 2]]
    return np.einsum('ij,ij->i', a, np.cross(b, c)).sum() / 6.0


@pytest.mark.parametrize('seed', [0, 1, 2, 3])
def test_mc_random_volume_closed_and_outward(seed):
    from oracle import mcubes
    rng = np.random.Generator(np.random.PCG64(seed))
    vol = rng.uniform(0.0, 10.0, size=(9, 8, 7))
    v, t = mcubes.marching_cubes(vol, 5.0, pad=2)
    assert len(t) > 0 and _closed_oriented(t)
    assert _signed_volume(v, t) > 0  # normals point from the high (inside) to the low region
    # one vertex per crossing grid edge, on the edge at the linear iso crossing
    p = np.pad(vol, 2)
    n_cross = sum(((p <= 5.0) != (np.roll(p, -1, a) <= 5.0))[tuple(slice(0, -1) if k == a else slice(None)
                                                                     for k in range(3))].sum() for a in range(3))
    assert len(v) == n_cross
    assert len(np.unique(t)) == len(v)


def test_mc_every_case_is_closed():
    from tools.gen_mc_table import case_triangles
    # each single cube case embedded in a zero border: a closed surface for every case
    from oracle import mcubes
    corners = [(0, 0, 0), (1, 0, 0), (1, 1, 0), (0, 1, 0), (0, 0, 1), (1, 0, 1), (1, 1, 1), (0, 1, 1)]
    for case in range(256):
        vol = np.zeros((2, 2, 2))
        for m, c in enumerate(corners):
            vol[c] = 0.0 if (case >> m) & 1 else 10.0
        v, t = mcubes.marching_cubes(vol, 5.0, pad=1)
        if case == 255:
            assert len(t) == 0
            continue
        assert _closed_oriented(t), case
        assert _signed_volume(v, t) > 0, case
        assert len(case_triangles(case)) <= 5


def test_mc_sphere_topology_and_area():
    from oracle import mcubes
    n = 40
    x = np.arange(n) - (n - 1) / 2
    r = np.sqrt(x[:, None, None] ** 2 + x[None, :, None] ** 2 + x[None, None, :] ** 2)
    vol = 10.0 * (12.0 - r)  # > 5 inside radius 11.5
    v, t = mcubes.marching_cubes(vol, 5.0, pad=10)
    assert _closed_oriented(t)
    edges = set()
    for a, b in ((0, 1), (1, 2), (2, 0)):
        edges |= set(map(tuple, np.sort(t[:, [a, b]], axis=1)))
    assert len(v) - len(edges) + len(t) == 2  # Euler characteristic of a sphere
    a, b, c = v[t[:, 0]], v[t[:, 1]], v[t[:, 2]]
    area = 0.5 * np.linalg.norm(np.cross(b - a, c - a), axis=1).sum()
    assert abs(area / (4 * np.pi * 11.5 ** 2) - 1) < 0.03
    vol_est = _signed_volume(v, t)
    assert abs(vol_est / (4 / 3 * np.pi * 11.5 ** 3) - 1) < 0.03


def test_generated_header_matches_generator():
    import os
    from tools.gen_mc_table import mc_tables
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = open(os.path.join(root, 'animatable_nerf_amd', 'csrc', 'anr_mc_table.h')).read()
    count, table = mc_tables()
    body = src[src.index('kMcCount[256] = {') + 17:]
    got = [int(x) for x in body[:body.index('}')].replace('\n', ' ').split(',') if x.strip()]
    assert got == list(count)
    body = src[src.index('kMcTris[256]'):]
    body = body[body.index('= {') + 3:body.index('};')]
    rows = [[int(x) for x in r.replace('}', '').split(',') if x.strip()]
            for r in body.replace('\n', '').split('{') if r.strip()]
    rows = [r for r in rows if r]
    assert np.array_equal(np.array(rows), table)
