"""Shared fixtures: synthetic scene, deterministic weights, batches (tests only)."""
import functools
import os

import numpy as np
import torch

from animatable_nerf_amd import network, synthetic

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def golden(name):
    return np.load(os.path.join(GOLDEN, name + '.npz'))


def golden_strict():
    """Bit-exact oracle-vs-golden checks are opt-in (ANR_GOLDEN_STRICT=1): the oracle reproduces the
    reference's fp32 bits only on a CPU whose PyTorch kernels (MKL GEMM, vectorised reductions,
    transcendentals) dispatch exactly as on the host that generated the goldens, and vendor / ISA do
    not identify that dispatch (an MKL or torch version, an AMX part can change it). Run strict on the
    generating host to re-pin the oracle bit for bit."""
    return os.environ.get('ANR_GOLDEN_STRICT') == '1'


def assert_golden_equal(got, ref, err_msg='', rtol=3e-5, atol=1e-6):
    """Oracle-vs-golden check.

    * Bool / integer arrays (masks, indices, labels): bit-exact everywhere.
    * Float arrays: bit-exact under ANR_GOLDEN_STRICT=1 (``golden_strict``); otherwise within fp32
      roundoff of a reordered sum: |got - ref| <= max(atol, rtol * max|ref|) + rtol * |ref| (rtol 3e-5,
      three times tighter than the GPU north_star tolerance; the scale term keeps small elements of a
      wide-range array from failing on cancellation noise of its large ones)."""
    got = np.asarray(got.detach().numpy() if hasattr(got, 'detach') else got)
    ref = np.asarray(ref)
    assert got.shape == ref.shape, (err_msg, got.shape, ref.shape)
    if np.array_equal(got, ref):
        return
    assert np.issubdtype(ref.dtype, np.floating), f'{err_msg}: integer/bool golden differs'
    if golden_strict():
        n = int(np.sum(got != ref))
        raise AssertionError(f'{err_msg}: {n} of {ref.size} elements differ from the golden bits '
                             '(ANR_GOLDEN_STRICT=1)')
    scale = float(np.max(np.abs(ref))) if ref.size else 0.0
    np.testing.assert_allclose(got, ref, rtol=rtol, atol=max(atol, rtol * scale), err_msg=err_msg)


@functools.lru_cache(maxsize=4)
def scene(vsize=0.05):
    return synthetic.Scene(vsize=vsize)


@functools.lru_cache(maxsize=1)
def state_dict_np():
    net = network.Network()
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    return synthetic.init_state_dict(shapes)


def oracle_params(requires_grad=False):
    return {k: torch.from_numpy(v.copy()).requires_grad_(requires_grad) for k, v in state_dict_np().items()}


def make_net(device='cpu'):
    net = network.Network()
    network.load_numpy_state(net, state_dict_np())
    return net.to(device)


def batch_np(sc, ray_o, ray_d, rgb=None):
    """near/far + hit filtering by the oracle's float64 slab test, then the collated batch."""
    from oracle import restate
    near, far, mask = restate.near_far(sc.bounds, ray_o, ray_d)
    b = sc.batch_arrays(ray_o[mask], ray_d[mask], near.astype(np.float32), far.astype(np.float32),
                        rgb=None if rgb is None else rgb[mask])
    return b, mask


def to_torch(b, device='cpu'):
    return {k: torch.from_numpy(np.ascontiguousarray(v)).to(device) for k, v in b.items()}


def novel_cfg():
    from animatable_nerf_amd import config
    cfg = config.defaults()
    cfg.aninerf_animation = True
    cfg.test_novel_pose = True
    cfg.num_eval_frame = 133
    cfg.perturb = 0
    return cfg


@functools.lru_cache(maxsize=1)
def state_dict_novel_np():
    net = network.Network(novel_cfg())
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    return synthetic.init_state_dict(shapes)


def make_net_novel(device='cpu'):
    net = network.Network(novel_cfg())
    network.load_numpy_state(net, state_dict_novel_np())
    return net.to(device)


def novel_batch_np():
    sc = scene(0.05)
    ro, rd = sc.box_rays(64, seed=2)
    b, mask = batch_np(sc, ro, rd)
    b['latent_index'] = np.array([3])
    b['bw_latent_index'] = np.array([5])
    return b


# ---- sdf_pdf (config 5)
@functools.lru_cache(maxsize=2)
def pdf_scene(vsize=0.05):
    return synthetic.PdfScene(vsize=vsize)


@functools.lru_cache(maxsize=1)
def state_dict_sdf_np():
    from animatable_nerf_amd import network_sdf
    net = network_sdf.Network(sdf_cfg())
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    return synthetic.init_state_dict_sdf(shapes)


def oracle_params_sdf():
    return {k: torch.from_numpy(v.copy()) for k, v in state_dict_sdf_np().items()}


def sdf_cfg():
    from animatable_nerf_amd import config
    return config.subject('anisdf_pdf_s9p', perturb=0)


def make_net_sdf(device='cpu'):
    from animatable_nerf_amd import network_sdf
    net = network_sdf.Network(sdf_cfg())
    network.load_numpy_state(net, state_dict_sdf_np())
    return net.to(device)


def pdf_batch_np(sc, ray_o, ray_d, latent_index=7):
    from oracle import restate
    near, far, mask = restate.near_far(sc.pbounds, ray_o, ray_d)
    b = sc.batch_arrays(ray_o[mask], ray_d[mask], near.astype(np.float32), far.astype(np.float32),
                        latent_index=latent_index)
    return b, mask


def pdf_g7_rays():
    """The 4,608 G7 rays (oracle/gen_goldens.py main_sdf)."""
    g = golden('g7_sdf_chunks')
    return g['ray_o'], g['ray_d']


def rotated_batch_np(n_rays=3000, seed=23, vsize=0.05):
    """A frame with a non-trivial smpl->world transform (R = Rodrigues(0.3, -0.2, 0.5),
    Th = (0.1, -0.05, 0.2)): world rays towards the world-space box, pbw/tbw in the pose frame."""
    from oracle import restate
    sc = scene(vsize)
    R = synthetic.batch_rodrigues(np.array([[0.3, -0.2, 0.5]]))[0].astype(np.float32)
    Th = np.array([0.1, -0.05, 0.2], np.float32)
    wverts = (sc.verts.astype(np.float64) @ R.T.astype(np.float64) + Th).astype(np.float32)
    wb = synthetic.get_bounds(wverts)
    rng = np.random.Generator(np.random.PCG64(seed))
    tgt = rng.uniform(wb[0].astype(np.float64), wb[1].astype(np.float64), size=(n_rays, 3))
    o = np.broadcast_to(np.array([0.0, 0.0, 3.0]), (n_rays, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    ro, rd = o.astype(np.float32).copy(), d.astype(np.float32)
    near, far, mask = restate.near_far(wb, ro, rd)
    b = sc.batch_arrays(ro[mask], rd[mask], near.astype(np.float32), far.astype(np.float32))
    b['R'] = R[None]
    b['Th'] = Th[None]
    b['wbounds'] = wb[None]
    return b


def mmsk_batch_np(ro, rd):
    """Batch with the training-view keys of tpose_novel_view_dataset.py:191 (synthetic views)."""
    sc = scene(0.05)
    b, mask = batch_np(sc, ro, rd)
    Ks, RTs, msks, H, W = synthetic.training_views(sc.verts)
    b.update(Ks=Ks[None], RT=RTs[None], msks=msks[None], H=np.array([H]), W=np.array([W]))
    return b, mask
