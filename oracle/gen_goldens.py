"""ORACLE — test infrastructure only. Generates tests/golden/*.npz by running the REAL reference
(/root/reference, read-only) on CPU in THIS container. It never travels to the GPU box: only its
outputs (small .npz fixtures) are committed.

Recipe:
  1. no bytecode writes (the tree is read-only);
  2. dummy modules for third-party packages the hot path imports but never calls
     (pytorch3d, cv2, trimesh, termcolor, imageio, tensorboardX, plyfile);
  3. ``sys.argv`` set BEFORE ``import lib.config`` (it parses argv at import, config.py:183-194);
  4. cwd = /root/reference (relative parent_cfg / network_path).
Goldens use ``torch.set_num_threads(1)``.

Run:  python oracle/gen_goldens.py            (writes tests/golden/; --novel, --sdf, --rays, --train-rays,
      --mmsk, --mesh, --sdf-mesh, --anim, --state-dicts for the other fixtures)
"""
import os
import sys
import types
import zlib

import numpy as np

REF = '/root/reference'
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, 'tests', 'golden')


class _Stub(types.ModuleType):
    def __getattr__(self, name):
        if name.startswith('__'):
            raise AttributeError(name)
        return _StubObj()


class _StubObj:
    def __call__(self, *a, **k):
        return _StubObj()

    def __getattr__(self, name):
        if name.startswith('__'):
            raise AttributeError(name)
        return _StubObj()


def _install_stubs():
    for name in ['pytorch3d', 'pytorch3d._C', 'pytorch3d.structures', 'pytorch3d.ops',
                 'pytorch3d.ops.knn', 'pytorch3d.ops.packed_to_padded',
                 'pytorch3d.ops.mesh_face_areas_normals', 'pytorch3d.ops.sample_points_from_meshes',
                 'cv2', 'trimesh', 'termcolor', 'imageio', 'tensorboardX', 'plyfile', 'mcubes']:
        sys.modules[name] = _Stub(name)


def import_reference(cfg_file='configs/aninerf_s9p.yaml', opts=(), knn=None):
    sys.dont_write_bytecode = True
    os.environ['PYTHONDONTWRITEBYTECODE'] = '1'
    _install_stubs()
    if knn is not None:  # the KNN restatement stands in for pytorch3d (unpinned boundary)
        sys.modules['pytorch3d.ops.knn'].knn_points = knn
    os.chdir(REF)
    sys.path.insert(0, REF)
    sys.argv = ['gen_goldens', '--cfg_file', cfg_file, 'gpus', '[]'] + list(opts)
    import lib.config  # noqa: F401  (parses argv)
    from lib.config import cfg
    from lib.networks import make_network
    from lib.networks.renderer import make_renderer
    return cfg, make_network, make_renderer


def main():
    import torch
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from animatable_nerf_amd.synthetic import Scene, init_state_dict, rigid_transformation, PARENTS
    cfg, make_network, make_renderer = import_reference()
    import lib.networks.bw_deform.tpose_nerf_network as tnn
    from lib.utils.if_nerf import if_nerf_data_utils as dutils

    os.makedirs(OUT, exist_ok=True)
    net = make_network(cfg)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    sd = init_state_dict(shapes)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    cfg.perturb = 0
    net.train()  # run.py evaluates in train() mode with perturb=0 (run.py:53-58)
    renderer = make_renderer(cfg, net)

    scene = Scene(vsize=0.05)
    meta = dict(vol_crc=zlib.crc32(scene.volume.tobytes()), A_crc=zlib.crc32(scene.A.tobytes()),
                vol_shape=np.array(scene.volume.shape))

    # ---- A15: rigid transformation + A14 near/far on the scene's own rays
    A_ref = dutils.get_rigid_transformation(scene.poses, scene.joints, PARENTS)
    assert np.array_equal(A_ref, rigid_transformation(scene.poses, scene.joints, PARENTS))

    def batch_for(ray_o, ray_d):
        near, far, mask = dutils.get_near_far(scene.bounds, ray_o, ray_d)
        b = scene.batch_arrays(ray_o[mask], ray_d[mask], near.astype(np.float32), far.astype(np.float32))
        return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in b.items()}, mask

    # ---- G1 tiny: 64 rays, intermediates captured by wrapping the module-level helpers
    rec = {}
    orig_psbw = tnn.pts_sample_blend_weights
    orig_p2t = tnn.pose_points_to_tpose_points
    calls = []

    def psbw(pts, bw, bounds):
        out = orig_psbw(pts, bw, bounds)
        calls.append(out.detach().clone())
        return out

    def p2t(ppts, bw, A):
        out = orig_p2t(ppts, bw, A)
        rec['tpose'] = out.detach().clone()
        rec['pbw_full'] = bw.detach().clone()
        return out

    orig_nbw = tnn.Network.calculate_neural_blend_weights
    bws = []

    def nbw(self, pts, smpl_bw, idx):
        out = orig_nbw(self, pts, smpl_bw, idx)
        bws.append(out.detach().clone())
        return out

    orig_ar = tnn.TPoseHuman.calculate_alpha_rgb

    def ar(self, pts, vd, ind):
        a, c = orig_ar(self, pts, vd, ind)
        rec['sigma_raw'] = a.detach().clone()
        rec['rgb_raw'] = c.detach().clone()
        return a, c

    tnn.pts_sample_blend_weights = psbw
    tnn.pose_points_to_tpose_points = p2t
    tnn.Network.calculate_neural_blend_weights = nbw
    tnn.TPoseHuman.calculate_alpha_rgb = ar
    ro, rd = scene.box_rays(64, seed=2)
    batch, mask = batch_for(ro, rd)
    with torch.no_grad():
        ret = renderer.render(batch)
    tnn.pts_sample_blend_weights = orig_psbw
    tnn.pose_points_to_tpose_points = orig_p2t
    tnn.Network.calculate_neural_blend_weights = orig_nbw
    tnn.TPoseHuman.calculate_alpha_rgb = orig_ar
    g1 = dict(ray_seed=2, n_rays=64, mask=mask, near=batch['near'].numpy(), far=batch['far'].numpy(),
              pre_bw=calls[0].numpy(), init_pbw=calls[1].numpy(), init_tbw=calls[2].numpy(),
              pbw=bws[0].numpy(), tbw=bws[1].numpy(), tpose=rec['tpose'].numpy(),
              sigma_raw=rec['sigma_raw'].numpy(), rgb_raw=rec['rgb_raw'].numpy(),
              **{'out_' + k: v.numpy() for k, v in ret.items()}, **meta)
    np.savez_compressed(os.path.join(OUT, 'g1_tiny.npz'), **g1)

    # ---- G2 chunks: 4096 box rays + 512 corner-grazing rays (a chunk with pnorm >= th everywhere)
    ro, rd = scene.box_rays(4096, seed=5)
    rng = np.random.Generator(np.random.PCG64(7))
    corners = np.array([[sx, sy, sz] for sx in (0, 1) for sy in (0, 1) for sz in (0, 1)])
    b = scene.bounds.astype(np.float64)
    tgt = b[corners[rng.integers(0, 8, 512)], [0, 1, 2]]
    tgt = tgt - np.sign(tgt) * rng.uniform(0.0, 0.01, size=(512, 3))
    o2 = np.broadcast_to(np.array([0.0, 0.0, 3.0]), (512, 3))
    d2 = tgt - o2
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    ro = np.concatenate([ro, o2.astype(np.float32)])
    rd = np.concatenate([rd, d2.astype(np.float32)])
    batch, mask = batch_for(ro, rd)
    with torch.no_grad():
        ret = renderer.render(batch)
    keep = (ret['raw'][0, :, :3].abs().sum(-1) != 0).numpy()
    rows = np.arange(0, ret['pbw'].shape[1], 37)
    g2 = dict(ray_o=ro, ray_d=rd, mask=mask, **{'out_' + k: ret[k].numpy() for k in
                                                ('rgb_map', 'acc_map', 'depth_map')},
              keep_bits=np.packbits(keep), kept_alpha=ret['raw'][0, keep, 3].numpy(),
              bw_rows=np.int64(ret['pbw'].shape[1]), bw_sample_idx=rows,
              pbw_sample=ret['pbw'][0, rows].numpy(), tbw_sample=ret['tbw'][0, rows].numpy(),
              pbw_sum=ret['pbw'].double().sum(1).numpy(), tbw_sum=ret['tbw'].double().sum(1).numpy(), **meta)
    np.savez_compressed(os.path.join(OUT, 'g2_chunks.npz'), **g2)

    # ---- G3 hits: camera rays (64x64) + adversarial rays through get_near_far
    K = np.array([[75.0, 0, 32.0], [0, 75.0, 32.0], [0, 0, 1]], np.float32)
    Rc = np.array([[1, 0, 0], [0, -1, 0], [0, 0, -1]], np.float32)
    Tc = np.array([[0.0], [0.0], [3.0]], np.float32)
    cam_o, cam_d = dutils.get_rays(64, 64, K, Rc, Tc)
    cam_o = cam_o.reshape(-1, 3).astype(np.float32)
    cam_d = cam_d.reshape(-1, 3).astype(np.float32)
    adv_o, adv_d = adversarial_rays(scene.bounds, 1024)
    ray_o = np.concatenate([cam_o, adv_o])
    ray_d = np.concatenate([cam_d, adv_d])
    with np.errstate(all='ignore'):
        near, far, mask = dutils.get_near_far(scene.bounds, ray_o, ray_d)
    g3 = dict(K=K, Rc=Rc, Tc=Tc, cam_o=cam_o, cam_d=cam_d, ray_o=ray_o, ray_d=ray_d,
              bounds=scene.bounds, mask=mask, near=near.astype(np.float32), far=far.astype(np.float32),
              near64=near, far64=far, A_ref=A_ref, poses=scene.poses, joints=scene.joints)
    np.savez_compressed(os.path.join(OUT, 'g3_hits.npz'), **g3)

    # ---- G4 train step: 256 rays, perturb=1, recorded t_rand, grads, Adam update
    from lib.train import make_optimizer
    from lib.train.trainers.tpose_trainer import NetworkWrapper
    cfg.perturb = 1
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    net.train()
    wrapper = NetworkWrapper(net)
    ro, rd = scene.box_rays(256, seed=11)
    batch, mask = batch_for(ro, rd)
    trng = np.random.Generator(np.random.PCG64(3))
    R = batch['ray_o'].shape[1]
    t_rand = torch.from_numpy(trng.random((R, 64)).astype(np.float32))
    batch['rgb'] = torch.from_numpy(trng.random((1, R, 3)).astype(np.float32))
    batch['mask_at_box'] = torch.ones((1, R), dtype=torch.bool)
    orig_rand = torch.rand
    pos = [0]

    def fake_rand(shape, *a, **k):
        n = shape[1]
        out = t_rand[pos[0]:pos[0] + n][None].clone()
        pos[0] += n
        return out

    torch.rand = fake_rand
    optimizer = make_optimizer(cfg, net)
    _, loss, stats, _ = wrapper(batch)
    optimizer.zero_grad()
    loss.backward()
    torch.nn.utils.clip_grad_value_(net.parameters(), 40)
    grads = {k: v.grad.detach().clone().numpy() for k, v in net.named_parameters() if v.grad is not None}
    before = {k: v.detach().clone() for k, v in net.named_parameters()}
    optimizer.step()
    torch.rand = orig_rand
    delta = {k: (v.detach() - before[k]).numpy() for k, v in net.named_parameters()}
    keep = ['bw_linears.0.weight', 'bw_linears.7.bias', 'bw_fc.weight', 'tpose_human.pts_linears.0.weight',
            'tpose_human.pts_linears.5.weight', 'tpose_human.rgb_fc.weight', 'tpose_human.alpha_fc.bias',
            'bw_latent.weight', 'tpose_human.nf_latent.weight']
    g4 = dict(ray_o=ro, ray_d=rd, mask=mask, t_rand=t_rand.numpy(), rgb=batch['rgb'].numpy(),
              loss=loss.detach().numpy(), **{'stat_' + k: v.detach().numpy() for k, v in stats.items()},
              **{'grad_' + k: grads[k] for k in keep if k in grads},
              **{'delta_' + k: delta[k] for k in keep}, lr=np.float32(cfg.train.lr))
    np.savez_compressed(os.path.join(OUT, 'g4_train.npz'), **g4)
    cfg.perturb = 0
    print('goldens written to', OUT)


def adversarial_rays(bounds, n):
    """Edge/corner-grazing, axis-parallel (zero components) and face-tangent rays."""
    rng = np.random.Generator(np.random.PCG64(17))
    b = bounds.astype(np.float64) + np.array([-0.01, 0.01])[:, None]   # the padded box the test uses
    lo, hi = b[0], b[1]
    o_list, d_list = [], []
    q = n // 4
    # 1) axis-parallel rays (two zero direction components) through / beside / on the box
    for i in range(q):
        ax = i % 3
        o = rng.uniform(lo - 0.05, hi + 0.05)
        o[ax] = (lo[ax] - 1.0) if (i // 3) % 2 == 0 else (hi[ax] + 1.0)
        if i % 5 == 0:                            # exactly on a face plane
            o[(ax + 1) % 3] = lo[(ax + 1) % 3]
        d = np.zeros(3)
        d[ax] = 1.0 if o[ax] < lo[ax] else -1.0
        o_list.append(o)
        d_list.append(d)
    # 2) rays through box corners
    for i in range(q):
        c = np.where(rng.integers(0, 2, 3) == 1, hi, lo)
        o = rng.uniform(-2.0, 2.0, 3) + np.array([0, 0, 3.0])
        d = c - o
        o_list.append(o)
        d_list.append(d / np.linalg.norm(d))
    # 3) rays through edge midpoints
    for i in range(q):
        c = np.where(rng.integers(0, 2, 3) == 1, hi, lo)
        k = rng.integers(0, 3)
        c[k] = rng.uniform(lo[k], hi[k])
        o = rng.uniform(-2.0, 2.0, 3) + np.array([0, 0, 3.0])
        d = c - o
        o_list.append(o)
        d_list.append(d / np.linalg.norm(d))
    # 4) face-tangent rays (one zero component, lying in a face plane)
    for i in range(n - 3 * q):
        ax = i % 3
        o = rng.uniform(lo - 0.5, hi + 0.5)
        o[ax] = lo[ax] if i % 2 == 0 else hi[ax]
        d = rng.standard_normal(3)
        d[ax] = 0.0
        o_list.append(o)
        d_list.append(d / np.linalg.norm(d))
    return np.array(o_list, np.float32), np.array(d_list, np.float32)


def main_novel():
    """G5: novel-pose render (cfg.test_novel_pose: pose-space blend weights from novel_pose_bw with
    bw_latent_index, tpose_nerf_network.py:93-94), 64 rays, latent_index 3, bw_latent_index 5."""
    import torch
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from animatable_nerf_amd.synthetic import Scene, init_state_dict
    cfg, make_network, make_renderer = import_reference(opts=('aninerf_animation', 'True', 'test_novel_pose', 'True'))
    from lib.utils.if_nerf import if_nerf_data_utils as dutils
    net = make_network(cfg)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    sd = init_state_dict(shapes)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    cfg.perturb = 0
    net.train()
    renderer = make_renderer(cfg, net)
    scene = Scene(vsize=0.05)
    ro, rd = scene.box_rays(64, seed=2)
    near, far, mask = dutils.get_near_far(scene.bounds, ro, rd)
    b = scene.batch_arrays(ro[mask], rd[mask], near.astype(np.float32), far.astype(np.float32), latent_index=3)
    b['bw_latent_index'] = np.array([5])
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in b.items()}
    with torch.no_grad():
        ret = renderer.render(batch)
    np.savez_compressed(os.path.join(OUT, 'g5_novel_pose.npz'), latent_index=3, bw_latent_index=5,
                        num_eval_frame=cfg.num_eval_frame, **{'out_' + k: v.numpy() for k, v in ret.items()})
    print('novel-pose golden written')


def main_sdf():
    """G6 / G7: the sdf_pdf variant (configs/sdf_pdf/anisdf_pdf_s9p.yaml, config 5), eval render.

    pytorch3d.ops.knn.knn_points is replaced by ``oracle.restate_sdf.knn_points`` (pytorch3d is not
    installed, so parity at the KNN boundary is unpinned); everything after it is the reference.
    G6: 64 rays with intermediates. G7: 4,608 rays = 3 chunks (the in-place tbounds widening per
    chunk, anisdf_pdf_network.py:203-205; forced argmin in the corner-grazing chunk; msk_sdf lists).
    """
    import torch
    from collections import namedtuple
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from oracle.restate_sdf import knn_points as knn_restated
    from animatable_nerf_amd.synthetic import PdfScene, init_state_dict_sdf, PARENTS
    KNN = namedtuple('KNN', ['dists', 'idx', 'knn'])

    def knn_stub(src, ref, K=1, **kw):
        d, i = knn_restated(src, ref, K)
        return KNN(d, i, None)

    cfg, make_network, make_renderer = import_reference('configs/sdf_pdf/anisdf_pdf_s9p.yaml',
                                                        opts=('init_sdf', "''"), knn=knn_stub)
    import lib.networks.bw_deform.anisdf_pdf_network as sdfn
    from lib.utils import sample_utils
    from lib.utils.if_nerf import if_nerf_data_utils as dutils
    net = make_network(cfg)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    sd = init_state_dict_sdf(shapes)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    cfg.perturb = 0
    net.train()
    renderer = make_renderer(cfg, net)
    scene = PdfScene(vsize=0.05)
    big_ref = dutils.get_rigid_transformation(scene.big_poses.reshape(-1, 3), scene.joints, PARENTS)
    assert np.array_equal(big_ref.astype(np.float32), scene.big_A)

    def batch_for(ray_o, ray_d):
        near, far, mask = dutils.get_near_far(scene.pbounds, ray_o, ray_d)
        b = scene.batch_arrays(ray_o[mask], ray_d[mask], near.astype(np.float32), far.astype(np.float32),
                               latent_index=7)
        return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in b.items()}, mask

    rec = {'sbc': [], 'resd': [], 'th': []}
    orig_sbc = sample_utils.sample_blend_closest_points
    orig_resd = sdfn.Network.calculate_residual_deformation
    orig_th = sdfn.TPoseHuman.forward

    def sbc(src, ref, values, K=5, exp=1e-8):
        out = orig_sbc(src, ref, values, K, exp)
        rec['sbc'].append(tuple(o.detach().clone() for o in out))
        return out

    def resd_fn(self, tpose, batch):
        out = orig_resd(self, tpose, batch)
        rec['resd'].append((tpose.detach().clone(), out.detach().clone()))
        return out

    def th_fn(self, wpts, viewdir, dists, batch):
        x, v = wpts.detach().clone(), viewdir.detach().clone()
        out = orig_th(self, wpts, viewdir, dists, batch)
        rec['th'].append((x, v, {k: t.detach().clone() for k, t in out.items()}))
        return out

    sample_utils.sample_blend_closest_points = sbc
    sdfn.Network.calculate_residual_deformation = resd_fn
    sdfn.TPoseHuman.forward = th_fn

    # ---- G6 tiny
    ro, rd = scene.box_rays(64, seed=2)
    batch, mask = batch_for(ro, rd)
    tb0 = batch['tbounds'].clone()
    with torch.no_grad():
        ret = renderer.render(batch)
    pre_bw, pnorm = rec['sbc'][0]
    kbw, _ = rec['sbc'][1]
    bigpose, resd = rec['resd'][0]
    tpose, tdirs, th = rec['th'][0]
    g6 = dict(mask=mask, near=batch['near'].numpy(), far=batch['far'].numpy(), tbounds_before=tb0.numpy(),
              tbounds_after=batch['tbounds'].numpy(), occupancy=batch['occupancy'].numpy(),
              pre_bw=pre_bw.numpy(), pnorm=pnorm.numpy(), kept_bw=kbw.numpy(), init_bigpose=bigpose.numpy(),
              resd=resd.numpy(), tpose=tpose.numpy(), tpose_dirs=tdirs.numpy(),
              th_sdf=th['sdf'].numpy(), th_gradients=th['gradients'].numpy(), th_raw=th['raw'].numpy(),
              **{'out_' + k: v.numpy() for k, v in ret.items()})
    np.savez_compressed(os.path.join(OUT, 'g6_sdf_tiny.npz'), **g6)

    # ---- G7 chunks: 4096 box rays + 512 corner-grazing rays
    for v in rec.values():
        v.clear()
    ro, rd = scene.box_rays(4096, seed=5)
    rng = np.random.Generator(np.random.PCG64(7))
    corners = np.array([[sx, sy, sz] for sx in (0, 1) for sy in (0, 1) for sz in (0, 1)])
    b = scene.pbounds.astype(np.float64)
    tgt = b[corners[rng.integers(0, 8, 512)], [0, 1, 2]]
    tgt = tgt - np.sign(tgt) * rng.uniform(0.0, 0.01, size=(512, 3))
    o2 = np.broadcast_to(np.array([0.0, 0.0, 3.0]), (512, 3))
    d2 = tgt - o2
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    ro = np.concatenate([ro, o2.astype(np.float32)])
    rd = np.concatenate([rd, d2.astype(np.float32)])
    batch, mask = batch_for(ro, rd)
    with torch.no_grad():
        ret = renderer.render(batch)
    keep = []
    for c in range(0, len(rec['sbc']), 2):
        pn = rec['sbc'][c][1][..., 0]
        k = pn < 0.1
        k[torch.arange(len(pn)), pn.argmin(dim=1)] = True
        keep.append(k[0])
    keep = torch.cat(keep).numpy()
    n_kept = int(keep.sum())
    rows = np.arange(0, n_kept, 29)
    g7 = dict(ray_o=ro, ray_d=rd, mask=mask, keep_bits=np.packbits(keep), n_kept=np.int64(n_kept),
              tbounds_after=batch['tbounds'].numpy(),
              **{'out_' + k: ret[k].numpy() for k in ('rgb_map', 'acc_map', 'depth_map', 'msk_sdf', 'msk_label')},
              kept_raw=ret['raw'][0, keep].numpy(), kept_sdf=ret['sdf'][0, keep, 0].numpy(),
              row_idx=rows, resd_rows=ret['resd'][0, rows].numpy(), grad_rows=ret['gradients'][0, rows].numpy(),
              resd_sum=ret['resd'].double().sum(1).numpy(), grad_sum=ret['gradients'].double().sum(1).numpy())
    np.savez_compressed(os.path.join(OUT, 'g7_sdf_chunks.npz'), **g7)
    sample_utils.sample_blend_closest_points = orig_sbc
    sdfn.Network.calculate_residual_deformation = orig_resd
    sdfn.TPoseHuman.forward = orig_th
    print('sdf_pdf goldens written')


def main_rays():
    """G8: the eval-split ray pipeline (get_rays + get_near_far + filtering =
    get_rays_within_bounds, if_nerf_data_utils.py:64-89, 310-339) for a float64 camera (the dtype of
    the datasets' annots) and a float32 one, on the synthetic subject's bounds."""
    sys.path.insert(0, REPO)
    from animatable_nerf_amd.synthetic import Scene
    import_reference()
    from lib.utils.if_nerf import if_nerf_data_utils as dutils
    scene = Scene(vsize=0.05)
    out = {}
    for tag, dt in (('f64', np.float64), ('f32', np.float32)):
        H, W = 120, 100
        a = np.deg2rad(20.0)
        K = np.array([[140.5, 0.0, 49.3], [0.0, 141.25, 61.7], [0.0, 0.0, 1.0]], dtype=dt)
        R = np.array([[np.cos(a), 0.0, -np.sin(a)], [0.0, -1.0, 0.0], [-np.sin(a), 0.0, -np.cos(a)]], dtype=dt)
        T = np.array([[0.05], [-0.02], [2.9]], dtype=dt)
        ray_o, ray_d = dutils.get_rays(H, W, K, R, T)
        ro, rd, near, far, mask = dutils.get_rays_within_bounds(H, W, K, R, T, scene.bounds)
        out.update({f'{tag}_K': K, f'{tag}_R': R, f'{tag}_T': T, f'{tag}_H': H, f'{tag}_W': W,
                    f'{tag}_all_o': ray_o, f'{tag}_all_d': ray_d, f'{tag}_Kinv': np.linalg.inv(K),
                    f'{tag}_ray_o': ro, f'{tag}_ray_d': rd, f'{tag}_near': near, f'{tag}_far': far,
                    f'{tag}_mask': mask})
    out['bounds'] = scene.bounds
    np.savez_compressed(os.path.join(OUT, 'g8_rays.npz'), **out)
    print('ray goldens written')


def main_train_rays():
    """G12: the train-split sampler sample_ray_h36m(split='train') (if_nerf_data_utils.py:198-283)
    of the real reference, for a float64 and a float32 camera, the second with face pixels
    (msk == 13) and cfg.face_sample_ratio = 0.2. get_bound_2d_mask uses cv2.fillPoly (cv2 absent):
    the reference is run with it replaced by animatable_nerf_amd.data.get_bound_2d_mask (case 1: that
    mask dilated by 8 px, so some drawn rays miss the box and the sampling loop runs again) and the
    mask is recorded as an input; every np.random.randint call is recorded too."""
    sys.path.insert(0, REPO)
    from animatable_nerf_amd.synthetic import Scene
    from animatable_nerf_amd.data import get_bound_2d_mask
    cfg, _, _ = import_reference()
    from lib.utils.if_nerf import if_nerf_data_utils as dutils
    scene = Scene(vsize=0.05)
    real_randint = np.random.randint
    draws = []

    def rec_randint(lo, hi, n):
        r = real_randint(lo, hi, n)
        draws.append(np.asarray(r, dtype=np.int64))
        return r
    np.random.randint = rec_randint
    out = {'bounds': scene.bounds}
    for case, dt, face_ratio in ((0, np.float64, 0.0), (1, np.float32, 0.2)):
        H, W = 120, 100
        a = np.deg2rad(20.0 + 15.0 * case)
        K = np.array([[140.5, 0.0, 49.3], [0.0, 141.25, 61.7], [0.0, 0.0, 1.0]], dtype=dt)
        R = np.array([[np.cos(a), 0.0, -np.sin(a)], [0.0, -1.0, 0.0], [-np.sin(a), 0.0, -np.cos(a)]], dtype=dt)
        T = np.array([[0.05], [-0.02], [2.9]], dtype=dt)
        g = np.random.default_rng(40 + case)
        img = g.random((H, W, 3), dtype=np.float32)
        yy, xx = np.mgrid[0:H, 0:W]
        e = ((xx - 50.0) / 16.0) ** 2 + ((yy - 58.0) / 40.0) ** 2
        msk = np.zeros((H, W), dtype=np.uint8)
        msk[e < 1.0] = 1
        msk[(e >= 1.0) & (e < 1.3)] = 100  # the dataset's eroded/dilated border band
        if case == 1:
            msk[(np.abs(xx - 50) < 4) & (np.abs(yy - 26) < 4)] = 13
        cfg.face_sample_ratio = face_ratio
        cfg.body_sample_ratio = 0.5
        cfg.mask_bkgd = True
        pose = np.concatenate([R, T], axis=1)
        bm = get_bound_2d_mask(scene.bounds, K, pose, H, W)
        if case == 1:  # a mask wider than the box (8 px) so that rays miss and the loop runs again
            d = np.zeros_like(bm)
            for dy in range(-8, 9):
                for dx in range(-8, 9):
                    d |= np.roll(np.roll(bm, dy, 0), dx, 1)
            bm = d
        dutils.get_bound_2d_mask = lambda *a, _bm=bm: _bm.copy()
        np.random.seed(100 + case)
        draws.clear()
        rgb, ro, rd, near, far, coord, mab = dutils.sample_ray_h36m(img.copy(), msk.copy(), K, R, T, scene.bounds,
                                                                  512, 'train')
        pre = f'c{case}_'
        out.update({pre + 'K': K, pre + 'R': R, pre + 'T': T, pre + 'img': img, pre + 'msk': msk, pre + 'bound_mask': bm,
                    pre + 'seed': 100 + case, pre + 'face_ratio': face_ratio, pre + 'rgb': rgb, pre + 'ray_o': ro,
                    pre + 'ray_d': rd, pre + 'near': near, pre + 'far': far, pre + 'coord': coord,
                    pre + 'n_randint': len(draws), pre + 'draws': np.concatenate(draws)})
        print('case', case, 'rounds', len(draws), 'rays', len(near))
    np.random.randint = real_randint
    out['nrays'] = 512
    np.savez_compressed(os.path.join(OUT, 'g12_train_rays.npz'), **out)
    print('train-ray goldens written')


def main_mmsk():
    """G9: the novel-view renderer with the training-view visibility filter
    (lib/networks/renderer/tpose_renderer_mmsk.py) over the aninerf network: 3 training views
    (synthetic.training_views), 64 box rays + a 2-chunk case whose second chunk (corner-grazing rays)
    has no visible sample."""
    import torch
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from animatable_nerf_amd.synthetic import Scene, init_state_dict, training_views
    cfg, make_network, _ = import_reference()
    import importlib
    mmsk = importlib.import_module('lib.networks.renderer.tpose_renderer_mmsk')
    from lib.utils.if_nerf import if_nerf_data_utils as dutils
    net = make_network(cfg)
    sd = init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    cfg.perturb = 0
    net.train()
    renderer = mmsk.Renderer(net)
    scene = Scene(vsize=0.05)
    Ks, RTs, msks, H, W = training_views(scene.verts)

    def batch_for(ro, rd):
        near, far, mask = dutils.get_near_far(scene.bounds, ro, rd)
        b = scene.batch_arrays(ro[mask], rd[mask], near.astype(np.float32), far.astype(np.float32))
        b.update(Ks=Ks[None], RT=RTs[None], msks=msks[None], H=np.array([H]), W=np.array([W]))
        return {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in b.items()}, mask

    out = {}
    ro, rd = scene.box_rays(64, seed=2)
    batch, mask = batch_for(ro, rd)
    insides = []
    orig = mmsk.Renderer.prepare_inside_pts

    def rec(self, pts, b):
        r = orig(self, pts, b)
        insides.append(r.clone())
        return r

    mmsk.Renderer.prepare_inside_pts = rec
    with torch.no_grad():
        ret = renderer.render(batch)
    out.update({'tiny_' + k: v.numpy() for k, v in ret.items()})
    out['tiny_inside'] = insides[0].numpy()
    # 2 chunks: 2048 box rays, then 256 corner-grazing rays
    ro, rd = scene.box_rays(2048, seed=13)
    rng = np.random.Generator(np.random.PCG64(19))
    corners = np.array([[sx, sy, sz] for sx in (0, 1) for sy in (0, 1) for sz in (0, 1)])
    b = scene.bounds.astype(np.float64)
    tgt = b[corners[rng.integers(0, 8, 256)], [0, 1, 2]]
    tgt = tgt - np.sign(tgt) * rng.uniform(0.0, 0.005, size=(256, 3))
    o2 = np.broadcast_to(np.array([0.0, 0.0, 3.0]), (256, 3))
    d2 = tgt - o2
    d2 /= np.linalg.norm(d2, axis=1, keepdims=True)
    ro = np.concatenate([ro, o2.astype(np.float32)])
    rd = np.concatenate([rd, d2.astype(np.float32)])
    batch, mask = batch_for(ro, rd)
    insides.clear()
    with torch.no_grad():
        ret = renderer.render(batch)
    mmsk.Renderer.prepare_inside_pts = orig
    out.update({'chunks_' + k: v.numpy() for k, v in ret.items()})
    out['chunks_ray_o'], out['chunks_ray_d'] = ro, rd
    out['chunks_inside_bits'] = np.packbits(torch.cat([x[0] for x in insides]).numpy())
    out['chunks_visible_per_chunk'] = np.array([int(x.sum()) for x in insides])
    np.savez_compressed(os.path.join(OUT, 'g9_mmsk.npz'), **out)
    print('mmsk golden written; visible samples per chunk:', out['chunks_visible_per_chunk'])


def main_mesh():
    """G10: the mesh renderer's density volume (lib/networks/renderer/aninerf_mesh_renderer.py:26-41
    over Network.get_alpha, tpose_nerf_network.py:105-137) in a rotated / translated world frame:
    (a) the reference render() on a 0.02 m voxel grid with a seeded `inside` mask — the cube it hands
    to mcubes.marching_cubes is recorded (mcubes itself is not installed: stubbed); (b) its
    batchify_rays with 4096-point chunks over the inside points plus a trailing chunk of far points
    (all pnorm >= 0.1: the forced argmin alone) and a 30-point chunk (torch's small-matmul path)."""
    import torch
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from animatable_nerf_amd.synthetic import init_state_dict, mesh_scene
    cfg, make_network, make_renderer = import_reference(opts=('vis_posed_mesh', 'True'))
    import mcubes
    net = make_network(cfg)
    sd = init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    net.train()
    renderer = make_renderer(cfg, net)
    b = mesh_scene(voxel=0.02)
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in b.items()}
    seen = {}

    def mc(cube, th):
        seen['cube'], seen['th'] = np.array(cube), th
        return np.zeros((0, 3)), np.zeros((0, 3), np.int64)

    mcubes.marching_cubes = mc
    with torch.no_grad():
        renderer.render(batch)
    cube = seen['cube'][10:-10, 10:-10, 10:-10]
    inside = b['inside'][0].astype(bool)
    assert np.all(cube[~inside] == 0)
    pts_in = b['pts'][0][inside]
    far = pts_in[:4096] + np.float32(5.0)  # far outside the pbw volume: pnorm = border value
    tail = pts_in[:30] + np.float32(0.001)
    pts_b = np.concatenate([pts_in[:16 * 4096], far, tail]).astype(np.float32)  # far = chunk 16, tail = 17
    with torch.no_grad():
        alpha_b = renderer.batchify_rays(torch.from_numpy(pts_b), lambda x: net.get_alpha(x, batch), net, 4096, batch)
    out = {k: v for k, v in b.items() if k not in ('pts',)}
    out.update(mesh_th=seen['th'], alpha_inside=cube[inside].astype(np.float32), pts_b=pts_b,
               alpha_b=np.asarray(alpha_b, np.float32), chunk_b=4096)
    np.savez_compressed(os.path.join(OUT, 'g10_mesh.npz'), **out)
    print('mesh golden written: grid', b['pts'].shape, 'inside', int(inside.sum()), 'nonzero alpha',
          int((cube != 0).sum()), 'batchify points', len(pts_b))


def main_sdf_mesh():
    """G14: the sdf_pdf mesh renderer (lib/networks/renderer/sdf_mesh_renderer.py:16-110 over
    anisdf_pdf_network.Network) on synthetic.sdf_mesh_scene (0.02 m grid over tbounds, rotated world
    frame). KNN = oracle.restate_sdf.knn_points (pytorch3d absent, unpinned). mcubes is stubbed to record
    the padded cube it is handed and to return oracle/mcubes.py's triangulation of it (PyMCubes absent);
    trimesh is stubbed with a single-component Trimesh (split() -> [itself]), so the recorded mesh is the
    whole triangulation. Recorded: the cube, the mesh handed back, the vertex / posed_vertex / triangle
    outputs, and gradient_of_deformed_sdf's normals and sdf at the vertices; plus sdf_network and
    calculate_bigpose_smpl_bw on a point sample."""
    import torch
    from collections import namedtuple
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from oracle.restate_sdf import knn_points as knn_restated
    from oracle import mcubes as mc_restated
    from animatable_nerf_amd.synthetic import init_state_dict_sdf, sdf_mesh_scene, Scene
    KNN = namedtuple('KNN', ['dists', 'idx', 'knn'])

    def knn_stub(src, ref, K=1, **kw):
        d, i = knn_restated(src, ref, K)
        return KNN(d, i, None)

    cfg, make_network, make_renderer = import_reference(
        'configs/sdf_pdf/anisdf_pdf_s9p.yaml', opts=('init_sdf', "''", 'vis_posed_mesh', 'True',
                                                     'voxel_size', '[0.02, 0.02, 0.02]'), knn=knn_stub)
    import mcubes
    import trimesh
    net = make_network(cfg)
    sd = init_state_dict_sdf({k: tuple(v.shape) for k, v in net.state_dict().items()})
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    net.train()
    renderer = make_renderer(cfg, net)
    assert type(renderer).__module__.endswith('sdf_mesh_renderer'), type(renderer).__module__
    b = sdf_mesh_scene(voxel=0.02)
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in b.items()}
    seen = {}

    def mc(cube, th):
        seen['cube'], seen['th'] = np.array(cube), th
        v, t = mc_restated.marching_cubes(np.asarray(cube, np.float64), th)
        seen['mc_vertices'], seen['mc_triangles'] = v, t
        return v, t

    class Mesh:
        def __init__(self, v, t):
            self.vertices, self.faces = np.asarray(v), np.asarray(t)

        def split(self):
            return [self]

    mcubes.marching_cubes = mc
    trimesh.Trimesh = Mesh
    rec = {}
    orig = type(net).gradient_of_deformed_sdf

    def godf(self, x, bt):
        g, y = orig(self, x, bt)
        rec.setdefault('x', []).append(x.detach().clone())
        rec.setdefault('g', []).append(g.detach().clone())
        rec.setdefault('y', []).append(y.detach().clone())
        return g, y
    type(net).gradient_of_deformed_sdf = godf
    ret = renderer.render(batch)
    type(net).gradient_of_deformed_sdf = orig
    # point-sample helpers: sdf_network on a seeded sample of the grid, calculate_bigpose_smpl_bw with the
    # aninerf scene's (X,Y,Z,25) volume standing in for input_bw['tbw'] (the renderer itself never calls it)
    rng = np.random.Generator(np.random.PCG64(14))
    flat = b['pts'].reshape(-1, 3)
    sel = rng.choice(len(flat), 3000, replace=False)
    xs = torch.from_numpy(flat[sel])
    with torch.no_grad():
        sdfnet = net.tpose_human.sdf_network(xs, batch)
    sc = Scene(vsize=0.05)
    ib = {'tbw': torch.from_numpy(sc.volume[None]), 'tbounds': torch.from_numpy(sc.bounds[None])}
    bwp = torch.from_numpy(rng.uniform(sc.bounds[0] - 0.05, sc.bounds[1] + 0.05, size=(1, 2000, 3)).astype(np.float32))
    bigbw = net.calculate_bigpose_smpl_bw(bwp, ib)
    out = {k: v for k, v in b.items() if k not in ('pts',)}
    out.update(grid_shape=np.array(b['pts'].shape[1:4]), cube=seen['cube'].astype(np.float32), mc_th=seen['th'],
               mc_vertices=seen['mc_vertices'], mc_triangles=seen['mc_triangles'],
               vertex=np.asarray(ret['vertex']), posed_vertex=np.asarray(ret['posed_vertex']),
               triangle=np.asarray(ret['triangle']),
               godf_x=torch.cat(rec['x'], 1).numpy(), godf_g=torch.cat(rec['g'], 1).numpy(),
               godf_y=torch.cat(rec['y'], 1).numpy(), sdfnet_x=xs.numpy(), sdfnet_out=sdfnet.numpy(),
               bw_pts=bwp.numpy(), bw_vol=sc.volume, bw_bounds=sc.bounds, bigpose_bw=bigbw.numpy())
    np.savez_compressed(os.path.join(OUT, 'g14_sdf_mesh.npz'), **out)
    print('sdf mesh golden written: grid', b['pts'].shape, 'vertices', len(ret['vertex']), 'triangles',
          len(ret['triangle']))


ANIM_N = 4096  # points per path (the reference's get_sampling_points hardcodes 1024 * 64)
ANIM_GRADS = ('bw_latent.weight', 'bw_linears.0.weight', 'bw_linears.0.bias', 'bw_linears.4.bias',
              'bw_linears.5.bias', 'bw_linears.7.weight', 'bw_linears.7.bias', 'bw_fc.weight', 'bw_fc.bias')


def main_anim():
    """G11: one forward + backward of the animation stage (lib/train/trainers/
    aninerf_animation_trainer.py NetworkWrapper, configs aninerf_animation True) in a rotated world
    frame. The module's get_sampling_points is replaced by the same formula (:143-160) at
    ANIM_N points per path with the torch.rand draws recorded; loss, the two bw losses and the
    gradients of novel_pose_bw tensors (bw_latent row bw_latent_index) are stored."""
    import torch
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from animatable_nerf_amd.synthetic import init_state_dict, mesh_scene
    cfg, make_network, _ = import_reference(opts=('aninerf_animation', 'True'))
    import importlib
    at = importlib.import_module('lib.train.trainers.aninerf_animation_trainer')
    net = make_network(cfg)
    sd = init_state_dict({k: tuple(v.shape) for k, v in net.state_dict().items()})
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    net.train()
    wrapper = at.NetworkWrapper(net)
    b = mesh_scene(voxel=0.1)
    b.pop('pts')
    b.pop('inside')
    b['bw_latent_index'] = np.array([7])
    batch = {k: torch.from_numpy(np.ascontiguousarray(v)) for k, v in b.items()}
    draws = []

    def sampling(bounds):
        sh = bounds.shape
        min_xyz, max_xyz = bounds[:, 0], bounds[:, 1]
        vals = [torch.rand([sh[0], ANIM_N]) for _ in range(3)]
        draws.append(torch.stack(vals, dim=2).numpy().copy())
        vals = torch.stack(vals, dim=2).to(bounds.device)
        return (max_xyz - min_xyz)[:, None] * vals + min_xyz[:, None]

    at.get_sampling_points = sampling
    torch.manual_seed(5)
    ret, loss, stats, _ = wrapper(batch)
    loss.backward()
    grads = {'grad_' + k: net.novel_pose_bw.state_dict(keep_vars=True)[k].grad.numpy().copy() for k in ANIM_GRADS}
    grads['grad_bw_latent.weight'] = grads['grad_bw_latent.weight'][7]
    out = dict(b, wvals=draws[0], tvals=draws[1], loss=loss.item(), bw_loss0=stats['bw_loss0'].item(),
               bw_loss1=stats['bw_loss1'].item(), norm_th=cfg.norm_th, train_th=cfg.train_th,
               m0=len(ret['pbw0']), **grads)
    assert all(np.all(np.isfinite(v)) for v in grads.values())
    np.savez_compressed(os.path.join(OUT, 'g11_anim.npz'), **out)
    print('anim golden written: loss', out['loss'], 'rows path 1', out['m0'])


SDF_TRAIN_KEEP = ['tpose_human.sdf_network.lin0.weight_v', 'tpose_human.sdf_network.lin3.weight_v',
                  'tpose_human.sdf_network.lin8.weight_v', 'tpose_human.beta_network.beta',
                  'tpose_human.color_network.color_latent.weight', 'tpose_human.color_network.lin0.weight_v',
                  'tpose_human.color_network.lin4.weight_v', 'resd_linears.0.weight', 'resd_linears.5.weight',
                  'resd_fc.weight', 'resd_fc.bias']


def main_sdf_train():
    """G13s: one training step of the sdf_pdf variant (config 5) through the reference's own wrapper
    (tpose_trainer.NetworkWrapper over anisdf_pdf_network.Network + tpose_renderer, perturb 1, the
    torch.rand draws recorded, iter_step past the first mask-alpha milestone) with the KNN stub:
    loss and every scalar stat, the gradients of every bias / weight_g / small tensor and of the
    SDF_TRAIN_KEEP weights, the observed-gradient row count."""
    import torch
    from collections import namedtuple
    torch.set_num_threads(1)
    sys.path.insert(0, REPO)
    from oracle.restate_sdf import knn_points as knn_restated
    from animatable_nerf_amd.synthetic import PdfScene, init_state_dict_sdf
    KNN = namedtuple('KNN', ['dists', 'idx', 'knn'])

    def knn_stub(src, ref, K=1, **kw):
        d, i = knn_restated(src, ref, K)
        return KNN(d, i, None)

    cfg, make_network, make_renderer = import_reference('configs/sdf_pdf/anisdf_pdf_s9p.yaml',
                                                        opts=('init_sdf', "''"), knn=knn_stub)
    from lib.utils.if_nerf import if_nerf_data_utils as dutils
    from lib.train.trainers.tpose_trainer import NetworkWrapper
    net = make_network(cfg)
    shapes = {k: tuple(v.shape) for k, v in net.state_dict().items()}
    sd = init_state_dict_sdf(shapes)
    net.load_state_dict({k: torch.from_numpy(v) for k, v in sd.items()}, strict=True)
    cfg.perturb = 1
    net.train()
    wrapper = NetworkWrapper(net)
    scene = PdfScene(vsize=0.05)
    ro, rd = scene.box_rays(SDF_TRAIN_RAYS, seed=21)
    near, far, mask = dutils.get_near_far(scene.pbounds, ro, rd)
    trng = np.random.Generator(np.random.PCG64(13))
    R = int(mask.sum())
    rgb = trng.random((R, 3)).astype(np.float32)
    b = scene.batch_arrays(ro[mask], rd[mask], near.astype(np.float32), far.astype(np.float32), latent_index=7,
                           rgb=rgb)
    b['mask_at_box'] = (trng.random((1, R)) < 0.9)
    batch = {k: torch.from_numpy(np.array(v, copy=True)) for k, v in b.items()}  # the golden keeps the inputs
    batch['iter_step'] = SDF_TRAIN_ITER
    t_rand = torch.from_numpy(trng.random((R, 64)).astype(np.float32))
    orig_rand = torch.rand
    pos = [0]

    def fake_rand(shape, *a, **k):
        n = shape[1]
        out = t_rand[pos[0]:pos[0] + n][None].clone()
        pos[0] += n
        return out

    torch.rand = fake_rand
    ret, loss, stats, _ = wrapper(batch)
    net.zero_grad()
    loss.backward()
    torch.rand = orig_rand
    grads = {k: v.grad.detach().clone().numpy() for k, v in net.named_parameters() if v.grad is not None}
    keep = {k: g for k, g in grads.items() if g.size <= 4096 or k in SDF_TRAIN_KEEP}
    n_obs = int(ret['observed_gradients'].shape[1]) if 'observed_gradients' in ret else 0
    out = dict(b, t_rand=t_rand.numpy(), iter_step=SDF_TRAIN_ITER, loss=loss.detach().numpy(),
               n_observed=n_obs, n_kept=int(ret['resd'].shape[1]), msk_len=int(ret['msk_sdf'].shape[1]),
               grad_keys=np.array(sorted(grads)), tbounds_after=batch['tbounds'].numpy(),
               **{'stat_' + k: v.detach().numpy() for k, v in stats.items()},
               **{'grad_' + k: v for k, v in keep.items()})
    np.savez_compressed(os.path.join(OUT, 'g13_sdf_train.npz'), **out)
    print('sdf train golden written: loss', float(loss), {k: float(v) for k, v in stats.items()}, 'kept',
          out['n_kept'], 'observed', n_obs, 'grads kept', len(keep), 'of', len(grads))


SDF_TRAIN_RAYS = 96
SDF_TRAIN_ITER = 12000


STATE_DICT_CONFIGS = {
    # name: (cfg_file, opts) -- the configs BASELINE.json names (s9p, 313, sdf_pdf) + the animation stage
    's9p': ('configs/aninerf_s9p.yaml', ()),
    '313': ('configs/aninerf_313.yaml', ()),
    's9p_animation': ('configs/aninerf_s9p.yaml', ('aninerf_animation', 'True')),
    'sdf_pdf_s9p': ('configs/sdf_pdf/anisdf_pdf_s9p.yaml', ('init_sdf', "''")),
}


def state_dict_one(name):
    """the reference Network's state_dict names / shapes (make_network(cfg)) for one config, and the
    cfg values the plugins size themselves from -> one JSON line on stdout"""
    import json
    cfg_file, opts = STATE_DICT_CONFIGS[name]
    cfg, make_network, _ = import_reference(cfg_file, opts=opts)
    net = make_network(cfg)
    print(json.dumps({'config': name, 'cfg_file': cfg_file, 'opts': list(opts),
                      'num_train_frame': int(cfg.num_train_frame), 'num_eval_frame': int(cfg.num_eval_frame),
                      'num_latent_code': int(cfg.num_latent_code), 'perturb': cfg.perturb,
                      'network_module': cfg.network_module,
                      'state_dict': [[k, list(v.shape)] for k, v in net.state_dict().items()]}))


def main_state_dicts():
    """G13: tests/golden/g13_state_dicts.json (one subprocess per config: lib.config parses argv
    once, at import)."""
    import json
    import subprocess
    out = {}
    for name in STATE_DICT_CONFIGS:
        r = subprocess.run([sys.executable, os.path.abspath(__file__), '--state-dict-one', name],
                           capture_output=True, text=True, check=True)
        line = [l for l in r.stdout.splitlines() if l.startswith('{')][-1]
        out[name] = json.loads(line)
    with open(os.path.join(OUT, 'g13_state_dicts.json'), 'w') as f:
        json.dump(out, f, indent=0)
    print('state_dict golden written:', {k: len(v['state_dict']) for k, v in out.items()})


if __name__ == '__main__':
    if len(sys.argv) > 2 and sys.argv[1] == '--state-dict-one':
        state_dict_one(sys.argv[2])
    elif len(sys.argv) > 1 and sys.argv[1] == '--state-dicts':
        main_state_dicts()
    elif len(sys.argv) > 1 and sys.argv[1] == '--sdf-train':
        main_sdf_train()
    elif len(sys.argv) > 1 and sys.argv[1] == '--anim':
        main_anim()
    elif len(sys.argv) > 1 and sys.argv[1] == '--mesh':
        main_mesh()
    elif len(sys.argv) > 1 and sys.argv[1] == '--sdf-mesh':
        main_sdf_mesh()
    elif len(sys.argv) > 1 and sys.argv[1] == '--mmsk':
        main_mmsk()
    elif len(sys.argv) > 1 and sys.argv[1] == '--train-rays':
        main_train_rays()
    elif len(sys.argv) > 1 and sys.argv[1] == '--rays':
        main_rays()
    elif len(sys.argv) > 1 and sys.argv[1] == '--novel':
        main_novel()
    elif len(sys.argv) > 1 and sys.argv[1] == '--sdf':
        main_sdf()
    else:
        main()
