"""CPU: pin the sdf_pdf oracle (oracle/restate_sdf.py, config 5) to the reference run
(tests/golden/g6_sdf_tiny.npz, g7_sdf_chunks.npz from oracle/gen_goldens.py --sdf).

KNN boundary unpinned: pytorch3d is absent, so the reference ran with the oracle's own
``knn_points`` restatement as its stub (oracle/restate_sdf.py header); those tests check the
restatement's stated properties instead (exact squared distances, lexicographic ties)."""
import numpy as np
import pytest
import torch

from animatable_nerf_amd import synthetic
from oracle import restate_sdf

from ._common import assert_golden_equal, golden, oracle_params_sdf, pdf_batch_np, pdf_g7_rays, pdf_scene, to_torch

torch.set_num_threads(1)


def test_pdf_scene_matches_generator():
    g = golden('g6_sdf_tiny')
    sc = pdf_scene()
    assert_golden_equal(g['tbounds_before'][0], sc.tbounds)
    ro, rd = sc.box_rays(64, seed=2)
    b, mask = pdf_batch_np(sc, ro, rd)
    assert np.array_equal(mask, g['mask'])
    assert np.array_equal(b['near'], g['near']) and np.array_equal(b['far'], g['far'])
    assert np.array_equal(b['occupancy'], g['occupancy'])


def test_knn_restatement_properties():
    rng = np.random.Generator(np.random.PCG64(3))
    ref = rng.uniform(-1, 1, (500, 3)).astype(np.float32)
    ref[10] = ref[3]  # exact duplicate -> tie on distance, the lower index first
    src = np.concatenate([rng.uniform(-1, 1, (300, 3)), ref[3:4] + 1e-3]).astype(np.float32)
    d2, idx = restate_sdf.knn_points(torch.from_numpy(src)[None], torch.from_numpy(ref)[None], K=5)
    d2, idx = d2[0].numpy(), idx[0].numpy()
    diff = src[:, None, :] - ref[None]
    full = (diff[..., 0] * diff[..., 0] + diff[..., 1] * diff[..., 1]) + diff[..., 2] * diff[..., 2]
    order = np.lexsort((np.broadcast_to(np.arange(500), full.shape), full), axis=1)[:, :5]
    np.testing.assert_array_equal(idx, order)
    np.testing.assert_array_equal(d2, np.take_along_axis(full, order, 1))
    assert idx[-1, 0] == 3 and idx[-1, 1] == 10


def test_g6_sdf_render_and_intermediates():
    g = golden('g6_sdf_tiny')
    sc = pdf_scene()
    ro, rd = sc.box_rays(64, seed=2)
    b, _ = pdf_batch_np(sc, ro, rd)
    bt = to_torch(b)
    trace = {}
    with torch.no_grad():
        ret = restate_sdf.render(oracle_params_sdf(), bt, trace=trace)
    assert_golden_equal(trace['pnorm'].numpy(), g['pnorm'][..., 0])
    for k, gk, tol in (('pbw', 'kept_bw', 0), ('init_bigpose', 'init_bigpose', 0), ('resd', 'resd', 0),
                       ('tpose', 'tpose', 0), ('tpose_dirs', 'tpose_dirs', 0), ('sdf_c', 'th_sdf', 0)):
        v = trace[k].numpy()
        if k == 'pbw':
            v = v.transpose(0, 2, 1)
        assert_golden_equal(v, g[gk], err_msg=k)
    for k in ('raw', 'sdf', 'resd', 'gradients', 'rgb_map', 'acc_map', 'depth_map', 'msk_sdf', 'msk_label'):
        assert_golden_equal(ret[k].numpy(), g['out_' + k], err_msg=k)
    assert_golden_equal(bt['tbounds'].numpy(), g['tbounds_after'])


@pytest.mark.slow
def test_g7_sdf_chunks():
    """3 chunks: cumulative in-place tbounds widening, forced argmin, msk_sdf ordering."""
    torch.set_num_threads(8)
    try:
        g = golden('g7_sdf_chunks')
        sc = pdf_scene()
        ro, rd = pdf_g7_rays()
        b, mask = pdf_batch_np(sc, ro, rd)
        assert np.array_equal(mask, g['mask'])
        bt = to_torch(b)
        trace = {}
        with torch.no_grad():
            ret = restate_sdf.render(oracle_params_sdf(), bt)
        keep = ret['sdf'][0, :, 0].numpy() != 10
        assert np.array_equal(np.packbits(keep), g['keep_bits'])
        for k in ('rgb_map', 'acc_map', 'depth_map', 'msk_sdf', 'msk_label'):
            np.testing.assert_allclose(ret[k].numpy(), g['out_' + k], rtol=0, atol=1e-5, err_msg=k)
        np.testing.assert_allclose(ret['raw'][0, keep].numpy(), g['kept_raw'], rtol=0, atol=1e-5)
        rows = g['row_idx']
        np.testing.assert_allclose(ret['resd'][0, rows].numpy(), g['resd_rows'], rtol=0, atol=1e-6)
        np.testing.assert_allclose(ret['gradients'][0, rows].numpy(), g['grad_rows'], rtol=0, atol=1e-4)
        assert_golden_equal(bt['tbounds'].numpy(), g['tbounds_after'])
    finally:
        torch.set_num_threads(1)
