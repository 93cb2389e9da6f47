"""Seeded synthetic Animatable-NeRF scene and deterministic weight recipe.

The licensed H36M / ZJU-MoCap data and the pretrained checkpoints are not available offline,
so every test, the golden generator and ``bench.py`` use this scene. Both the reference run
(``oracle/gen_goldens.py``, this container only) and the HIP path draw it from here, so the
same seed gives the same bytes on both sides.

Scene (all numpy, PCG64):
  * 6,890 "vertices" = Gaussian directions normalised to unit length (seed 0), scaled to an
    ellipsoid with semi-axes (0.25, 0.85, 0.15) m;
  * 24 joints ~ U(+-(0.2, 0.7, 0.1)) from the same generator; SMPL kinematic tree ``PARENTS``;
  * skin weights exp(-d/0.05) over the vertex->joint distance, normalised per vertex;
  * blend-weight volume laid out like ``tools/custom_dataset/prepare_blend_weights.py:156-209``:
    an ``ij`` meshgrid with ``vsize`` spacing over the vertex bounds +-0.05, channels 0-23 = skin
    weights of the nearest vertex, channel 24 = distance to that vertex, shape (X, Y, Z, 25) f32;
  * pose = axis-angles N(0, 0.1^2) (seed 1, root zero) -> A (24,4,4) by the kinematic chain of
    ``lib/utils/if_nerf/if_nerf_data_utils.py:414-458``; R = I, Th = 0, so world = pose space;
  * bounds via ``get_bounds`` (``if_nerf_data_utils.py:566-579``): vertex min/max +- box_padding.

Rays ("box" generator, seed 2): origin (0, 0, 3), targets U(pbounds), unit directions, then the
float64 near/far slab test of A14 (``if_nerf_data_utils.py:156-196``).
"""
import numpy as np

PARENTS = np.array([-1, 0, 0, 0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 9, 9, 12, 13, 14, 16, 17, 18, 19, 20, 21],
                   dtype=np.int64)
SEMI_AXES = np.array([0.25, 0.85, 0.15])
JOINT_RANGE = np.array([0.2, 0.7, 0.1])
BOX_PADDING = 0.05


def batch_rodrigues(poses):
    """Axis-angle (N,3) -> rotation matrices (N,3,3); same formula as
    ``if_nerf_data_utils.py:392-411`` (angle = |poses + 1e-8|)."""
    n = poses.shape[0]
    angle = np.linalg.norm(poses + 1e-8, axis=1, keepdims=True)
    axis = poses / angle
    c = np.cos(angle)[:, None]
    s = np.sin(angle)[:, None]
    rx, ry, rz = axis[:, 0:1], axis[:, 1:2], axis[:, 2:3]
    z = np.zeros((n, 1))
    K = np.concatenate([z, -rz, ry, rz, z, -rx, -ry, rx, z], axis=1).reshape(n, 3, 3)
    return np.eye(3)[None] + s * K + (1 - c) * np.matmul(K, K)


def rigid_transformation(poses, joints, parents):
    """24-joint chain -> A = G(pose, j_rel) G(0, j)^-1 as (24,4,4) f32.

    Restates ``get_rigid_transformation`` (``if_nerf_data_utils.py:414-458``) in float64 and
    casts once at the end, as the reference does.
    """
    rot = batch_rodrigues(poses)
    rel = joints.copy()
    rel[1:] -= joints[parents[1:]]
    local = np.zeros((24, 4, 4))
    local[:, :3, :3] = rot
    local[:, :3, 3] = rel
    local[:, 3, 3] = 1.0
    chain = [local[0]]
    for i in range(1, 24):
        chain.append(np.dot(chain[parents[i]], local[i]))
    G = np.stack(chain, axis=0)
    jh = np.concatenate([joints, np.zeros((24, 1))], axis=1)
    G[..., 3] = G[..., 3] - np.sum(G * jh[:, None], axis=2)
    return G.astype(np.float32)


def get_bounds(xyz, box_padding=BOX_PADDING):
    lo = np.min(xyz, axis=0) - box_padding
    hi = np.max(xyz, axis=0) + box_padding
    return np.stack([lo, hi], axis=0).astype(np.float32)


def _nearest_vertex(pts, verts, block=4096):
    idx = np.empty(len(pts), dtype=np.int64)
    dist = np.empty(len(pts), dtype=np.float64)
    v2 = np.sum(verts * verts, axis=1)
    for s in range(0, len(pts), block):
        p = pts[s:s + block]
        d2 = np.sum(p * p, axis=1)[:, None] - 2.0 * p @ verts.T + v2[None]
        j = np.argmin(d2, axis=1)
        idx[s:s + block] = j
        dist[s:s + block] = np.linalg.norm(p - verts[j], axis=1)
    return idx, dist


def blend_weight_volume(verts, skin, vsize):
    """(X,Y,Z,25) f32 volume over verts bounds +-0.05 (``prepare_blend_weights.py:156-209``)."""
    lo = verts.min(axis=0) - 0.05
    hi = verts.max(axis=0) + 0.05
    axes = [np.arange(lo[i], hi[i] + vsize, vsize) for i in range(3)]
    grid = np.stack(np.meshgrid(*axes, indexing='ij'), axis=-1)
    sh = grid.shape[:3]
    idx, dist = _nearest_vertex(grid.reshape(-1, 3), verts)
    vol = np.concatenate([skin[idx], dist[:, None]], axis=1)
    return vol.reshape(*sh, 25).astype(np.float32)


class Scene:
    """One frame of the synthetic subject; ``batch_arrays`` gives the collated batch keys."""

    def __init__(self, vsize=0.025, pose_scale=0.1, seed=0):
        rng = np.random.Generator(np.random.PCG64(seed))
        d = rng.standard_normal((6890, 3))
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        self.verts = (d * SEMI_AXES).astype(np.float32)
        self.joints = rng.uniform(-JOINT_RANGE, JOINT_RANGE, size=(24, 3)).astype(np.float32)
        dj = np.linalg.norm(self.verts[:, None].astype(np.float64) - self.joints[None], axis=2)
        w = np.exp(-dj / 0.05)
        self.skin = (w / w.sum(axis=1, keepdims=True)).astype(np.float32)
        self.volume = blend_weight_volume(self.verts.astype(np.float64), self.skin, vsize)
        prng = np.random.Generator(np.random.PCG64(seed + 1))
        poses = prng.normal(0.0, pose_scale, size=(24, 3))
        poses[0] = 0.0
        self.poses = poses
        self.A = rigid_transformation(poses, self.joints, PARENTS)
        self.bounds = get_bounds(self.verts)
        self.R = np.eye(3, dtype=np.float32)
        self.Th = np.zeros(3, dtype=np.float32)

    def box_rays(self, n, seed=2, origin=(0.0, 0.0, 3.0)):
        """n rays from ``origin`` towards U(bounds) targets; unit f32 directions."""
        rng = np.random.Generator(np.random.PCG64(seed))
        tgt = rng.uniform(self.bounds[0].astype(np.float64), self.bounds[1].astype(np.float64), size=(n, 3))
        o = np.broadcast_to(np.asarray(origin, dtype=np.float64), (n, 3))
        d = tgt - o
        d /= np.linalg.norm(d, axis=1, keepdims=True)
        return o.astype(np.float32).copy(), d.astype(np.float32)

    def batch_arrays(self, ray_o, ray_d, near, far, latent_index=0, rgb=None):
        """Collated (batch-dim 1) numpy batch with the keys of ``tpose_dataset.py:236-277``."""
        R = ray_o.shape[0]
        if rgb is None:
            rgb = np.zeros((R, 3), np.float32)
        return {
            'ray_o': ray_o[None].astype(np.float32), 'ray_d': ray_d[None].astype(np.float32),
            'near': near[None].astype(np.float32), 'far': far[None].astype(np.float32),
            'occupancy': np.ones((1, R), np.uint8), 'mask_at_box': np.ones((1, R), np.bool_),
            'rgb': rgb[None].astype(np.float32),
            'A': self.A[None], 'big_A': self.A[None],
            'pbw': self.volume[None], 'tbw': self.volume[None],
            'pbounds': self.bounds[None], 'wbounds': self.bounds[None], 'tbounds': self.bounds[None],
            'R': self.R[None], 'Th': self.Th[None],
            'H': np.array([0]), 'W': np.array([0]),
            'latent_index': np.array([latent_index]), 'bw_latent_index': np.array([latent_index]),
            'frame_index': np.array([0]), 'cam_ind': np.array([0]),
        }


def mesh_scene(voxel=0.02, vsize=0.05, inside_frac=0.8, seed=11):
    """The mesh path's batch (aninerf_mesh_dataset.py:126-174) for the synthetic subject in a rotated
    and translated world frame: world vertices w = p R^T + Th so that (w - Th) R = p; pbounds /
    wbounds from the pose / world vertices; the voxel grid over wbounds; a seeded `inside` mask
    standing in for the training-view mask test (prepare_inside_pts :93-117)."""
    sc = Scene(vsize=vsize)
    R = batch_rodrigues(np.array([[0.2, -0.3, 0.1]]))[0].astype(np.float32)
    Th = np.array([0.1, -0.05, 0.2], np.float32)
    wverts = (sc.verts.astype(np.float64) @ R.T.astype(np.float64) + Th).astype(np.float32)
    wbounds = get_bounds(wverts)
    axes = [np.arange(wbounds[0, c], wbounds[1, c] + voxel, voxel) for c in range(3)]
    pts = np.stack(np.meshgrid(*axes, indexing='ij'), axis=-1).astype(np.float32)
    rng = np.random.Generator(np.random.PCG64(seed))
    inside = (rng.random(pts.shape[:-1]) < inside_frac).astype(np.uint8)
    return {'pts': pts[None], 'inside': inside[None], 'A': sc.A[None], 'pbw': sc.volume[None],
            'tbw': sc.volume[None], 'pbounds': sc.bounds[None], 'wbounds': wbounds[None],
            'tbounds': sc.bounds[None], 'R': R[None], 'Th': Th[None, None],
            'latent_index': np.array([2]), 'frame_index': np.array([0])}


def sdf_mesh_scene(voxel=0.02, vsize=0.05):
    """The sdf_pdf mesh path's batch (anisdf_mesh_dataset.py:145-206) for the synthetic subject: the voxel
    grid (float64 np.arange per axis, ij meshgrid, float32) over the big-pose bounds tbounds, the big-pose
    vertices, skin weights, big_A / A / poses, and a rotated / translated world frame (R, Th) for the
    posed vertices."""
    sc = PdfScene(vsize=vsize)
    tb = sc.tbounds
    axes = [np.arange(tb[0, c], tb[1, c] + voxel, voxel) for c in range(3)]
    pts = np.stack(np.meshgrid(*axes, indexing='ij'), axis=-1).astype(np.float32)
    R = batch_rodrigues(np.array([[0.2, -0.3, 0.1]]))[0].astype(np.float32)
    Th = np.array([0.1, -0.05, 0.2], np.float32)
    return {'pts': pts[None], 'A': sc.A[None], 'big_A': sc.big_A[None], 'poses': sc.pose_vec[None],
            'weights': sc.skin[None], 'tvertices': sc.tvertices[None], 'pvertices': sc.pvertices[None],
            'tbounds': tb[None], 'pbounds': sc.pbounds[None], 'wbounds': sc.pbounds[None],
            'inside': np.ones(pts.shape[:-1], np.uint8)[None], 'R': R[None], 'Th': Th[None, None],
            'latent_index': np.array([3]), 'frame_index': np.array([0])}


def training_views(verts, n_views=3, H=100, W=100, focal=80.0, dist=3.0, dilate=1):
    """Training cameras + silhouettes for the novel-view visibility filter
    (``tpose_renderer_mmsk.py:14-57``; keys of ``tpose_novel_view_dataset.py:191``): cameras on a
    circle around the y axis (0, 90, 200 degrees, ...) looking at the origin, K with the principal
    point at the image centre, RT = [R | T] world->camera (float32); msks = the vertices splatted into
    each image and dilated by ``dilate`` pixels (uint8 0/1), i.e. the subject's silhouette."""
    angles = np.deg2rad(np.array([0.0, 90.0, 200.0, 300.0, 45.0, 135.0])[:n_views])
    K = np.array([[focal, 0.0, (W - 1) / 2.0], [0.0, focal, (H - 1) / 2.0], [0.0, 0.0, 1.0]], np.float32)
    Ks, RTs, msks = [], [], []
    for a in angles:
        c = np.array([dist * np.sin(a), 0.0, dist * np.cos(a)])   # camera centre, looking at 0
        fwd = -c / np.linalg.norm(c)
        up = np.array([0.0, 1.0, 0.0])
        right = np.cross(up, fwd)
        right /= np.linalg.norm(right)
        down = np.cross(fwd, right)
        R = np.stack([right, down, fwd], 0)                       # rows: camera x, y, z in world
        T = -R @ c
        RT = np.concatenate([R, T[:, None]], 1).astype(np.float32)
        cam = verts.astype(np.float64) @ R.T + T
        uv = cam @ K.astype(np.float64).T
        uv = uv[:, :2] / uv[:, 2:]
        m = np.zeros((H, W), np.uint8)
        ij = np.round(uv).astype(int)
        ok = (ij[:, 0] >= 0) & (ij[:, 0] < W) & (ij[:, 1] >= 0) & (ij[:, 1] < H)
        m[ij[ok, 1], ij[ok, 0]] = 1
        for _ in range(dilate):
            m2 = m.copy()
            m2[1:] |= m[:-1]; m2[:-1] |= m[1:]; m2[:, 1:] |= m[:, :-1]; m2[:, :-1] |= m[:, 1:]
            m = m2
        Ks.append(K)
        RTs.append(RT)
        msks.append(m)
    return np.stack(Ks), np.stack(RTs), np.stack(msks), H, W


def lbs_vertices(verts, skin, A):
    """Forward LBS of (V,3) vertices with per-vertex weights (V,24) and A (24,4,4), float64 -> f32."""
    T = np.einsum('vj,jab->vab', skin.astype(np.float64), A.astype(np.float64))
    v = np.einsum('vab,vb->va', T[:, :3, :3], verts.astype(np.float64)) + T[:, :3, 3]
    return v.astype(np.float32)


def big_pose_A(joints):
    """``tpose_pdf_dataset.py:91-100`` load_bigpose: float32 axis-angles, joints 1/2 z = +-30 deg."""
    big = np.zeros([24, 3]).astype(np.float32).ravel()
    big[5] = np.deg2rad(30)
    big[8] = np.deg2rad(-30)
    return rigid_transformation(big.reshape(-1, 3), joints, PARENTS), big


class PdfScene(Scene):
    """Config 5 (sdf_pdf) frame: the same subject as ``Scene`` with the keys of
    ``tpose_pdf_dataset.py:270-291``. The ellipsoid vertices are the T pose; ``pvertices`` = LBS with
    the frame's A, ``tvertices`` = LBS with ``big_A``; ``weights`` = the per-vertex skin weights;
    pbounds = wbounds = bounds of pvertices (R = I, Th = 0), tbounds = bounds of tvertices.
    ``occupancy`` is a seeded random pixel mask (PCG64 seed 9) so both ``msk_sdf`` branches are hit.
    """

    def __init__(self, vsize=0.05, pose_scale=0.1, seed=0):
        super().__init__(vsize=vsize, pose_scale=pose_scale, seed=seed)
        self.big_A, self.big_poses = big_pose_A(self.joints)
        self.pvertices = lbs_vertices(self.verts, self.skin, self.A)
        self.tvertices = lbs_vertices(self.verts, self.skin, self.big_A)
        self.pbounds = get_bounds(self.pvertices)
        self.tbounds = get_bounds(self.tvertices)
        self.bounds = self.pbounds  # box rays and near/far use the posed body
        self.pose_vec = self.poses.ravel().astype(np.float32)

    def batch_arrays(self, ray_o, ray_d, near, far, latent_index=0, rgb=None, occ_seed=9):
        R = ray_o.shape[0]
        if rgb is None:
            rgb = np.zeros((R, 3), np.float32)
        occ = np.random.Generator(np.random.PCG64(occ_seed)).integers(0, 2, R).astype(np.uint8)
        return {
            'ray_o': ray_o[None].astype(np.float32), 'ray_d': ray_d[None].astype(np.float32),
            'near': near[None].astype(np.float32), 'far': far[None].astype(np.float32),
            'occupancy': occ[None], 'mask_at_box': np.ones((1, R), np.bool_),
            'rgb': rgb[None].astype(np.float32),
            'A': self.A[None], 'big_A': self.big_A[None], 'poses': self.pose_vec[None],
            'weights': self.skin[None], 'tvertices': self.tvertices[None], 'pvertices': self.pvertices[None],
            'pbounds': self.pbounds[None], 'wbounds': self.pbounds[None],
            'tbounds': self.tbounds[None].copy(),  # the network widens it in place (own copy per batch)
            'R': self.R[None], 'Th': self.Th[None],
            'H': np.array([0]), 'W': np.array([0]),
            'latent_index': np.array([latent_index]), 'bw_latent_index': np.array([latent_index]),
            'frame_index': np.array([0]), 'cam_ind': np.array([0]),
        }


def init_state_dict_sdf(shapes, seed=4321):
    """Deterministic weights for the sdf_pdf network (``anisdf_pdf_network.py``), per tensor a PCG64
    stream seeded with (seed, index):

      * ``sdf_network.lin*``: the geometric init of ``anisdf_pdf_network.py:388-410`` (last layer
        N(sqrt(pi)/sqrt(256), 1e-4) with bias -0.5; lin0 only on xyz; lin4 zero on the gamma part),
        hidden biases U(+-0.01) instead of 0 so the bias path is exercised;
      * ``weight_v`` of the colour net U(+-1/sqrt(in)), its biases likewise;
      * every ``weight_g`` = row norm of its ``weight_v`` times U(0.8, 1.2) (so weight-norm is not
        the identity);
      * Conv1d (``resd_linears``/``resd_fc``) U(+-1/sqrt(fan_in)), ``resd_fc.weight`` x16 (so the
        displacement reaches a few cm), ``resd_fc.bias`` = 0 (``anisdf_pdf_network.py:31``);
        embeddings N(0,1); ``beta`` = 0.1.
    """
    out = {}
    names = list(shapes)
    rngs = {n: np.random.Generator(np.random.PCG64([seed, i])) for i, n in enumerate(names)}
    d0 = 39
    for name in names:
        shape = shapes[name]
        rng = rngs[name]
        if name.endswith('beta'):
            out[name] = np.array(0.1, np.float32)
            continue
        if len(shape) == 2 and name.endswith('.weight') and 'latent' in name:
            out[name] = rng.standard_normal(shape).astype(np.float32)
            continue
        mod, leaf = name.rsplit('.', 1)
        if 'sdf_network' in mod:
            l = int(mod[-1])
            if leaf == 'weight_v':
                o, i = shape
                if l == 8:
                    v = rng.normal(np.sqrt(np.pi) / np.sqrt(i), 1e-4, size=shape)
                elif l == 0:
                    v = np.zeros(shape)
                    v[:, :3] = rng.normal(0.0, np.sqrt(2) / np.sqrt(o), size=(o, 3))
                else:
                    v = rng.normal(0.0, np.sqrt(2) / np.sqrt(o), size=shape)
                    if l == 4:
                        v[:, -(d0 - 3):] = 0.0
                out[name] = v.astype(np.float32)
            elif leaf == 'bias':
                out[name] = (np.full(shape, -0.5) if l == 8 else rng.uniform(-0.01, 0.01, size=shape)).astype(np.float32)
            continue
        if 'color_network' in mod:
            if leaf == 'weight_v':
                out[name] = rng.uniform(-1, 1, size=shape).astype(np.float32) / np.float32(np.sqrt(shape[1]))
            elif leaf == 'bias':
                fan = shapes[mod + '.weight_v'][1]
                out[name] = rng.uniform(-1, 1, size=shape).astype(np.float32) / np.float32(np.sqrt(fan))
            continue
        if leaf in ('weight', 'bias') and len(shapes[mod + '.weight']) == 3:
            fan = shapes[mod + '.weight'][1]
            arr = rng.uniform(-1, 1, size=shape) / np.sqrt(fan)
            if name == 'resd_fc.bias':
                arr = np.zeros(shape)
            elif name == 'resd_fc.weight':
                arr = arr * 16.0  # displacements of a few cm, so 0.05*tanh is not ~linear
            out[name] = arr.astype(np.float32)
    for name in names:  # weight_g after every weight_v exists
        if name.endswith('weight_g'):
            v = out[name[:-1] + 'v'].astype(np.float64)
            s = rngs[name].uniform(0.8, 1.2, size=(v.shape[0], 1))
            out[name] = (np.linalg.norm(v, axis=1, keepdims=True) * s).astype(np.float32)
    return {n: out[n] for n in names}


def init_state_dict(shapes, seed=1234, alpha_bias=3.0):
    """Deterministic weights for a state_dict given {name: shape} (insertion order matters).

    Per tensor a PCG64 stream seeded with (seed, index): Conv1d weights and biases U(+-1/sqrt(fan_in))
    (PyTorch's default Conv1d init bound), embeddings N(0,1); ``tpose_human.alpha_fc.bias`` = +3 so
    densities are non-trivial.
    """
    out = {}
    fan_in = {}
    for name, shape in shapes.items():
        if name.endswith('.weight') and len(shape) == 3:
            fan_in[name[:-len('.weight')]] = shape[1] * shape[2]
    for i, (name, shape) in enumerate(shapes.items()):
        rng = np.random.Generator(np.random.PCG64([seed, i]))
        if len(shape) == 2:  # nn.Embedding
            arr = rng.standard_normal(shape)
        else:
            mod = name.rsplit('.', 1)[0]
            bound = 1.0 / np.sqrt(fan_in[mod])
            arr = rng.uniform(-bound, bound, size=shape)
        out[name] = arr.astype(np.float32)
    if 'tpose_human.alpha_fc.bias' in out:
        out['tpose_human.alpha_fc.bias'][:] = alpha_bias
    return out
