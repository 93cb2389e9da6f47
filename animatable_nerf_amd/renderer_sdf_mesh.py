"""sdf_pdf mesh renderer plugin (``lib/networks/renderer/sdf_mesh_renderer.py:10-110``; the config-5
``mesh_cfg``, ``configs/sdf_pdf/anisdf_pdf_s9p.yaml:141-149``).

``Renderer(net).render(batch)`` takes the batch of ``lib/datasets/anisdf_mesh_dataset.py:145-206``
(``pts (1,X,Y,Z,3)`` voxel grid over ``tbounds``, ``tvertices``, ``weights``, ``big_A``, ``A``, ``R``,
``Th``, ``poses``, ``latent_index``) and returns ``{'vertex', 'posed_vertex', 'triangle'}`` as numpy arrays:

* the ``inside`` filter ``tnorm < 0.1`` of sample_blend_closest_points against ``tvertices`` (:56-62):
  ``anr_knn_blend`` (the render front-end's exact 5-NN);
* ``tpose_human.sdf_network`` over the inside points (:64-68): ``anr_sdf_points`` (exact fp32);
* ``cube = -sdf`` (10 outside), padded by 10 with -10 (:70-75), marching cubes at 0: the device marching
  cubes of the aninerf mesh path (``renderer_mesh.marching_cubes``) over the padded cube;
* ``trimesh.Trimesh(...).split()`` and the largest component (:76-77): ``largest_component`` (host graph
  pass over the triangle list: faces joined through shared edges, watertight components only, the
  vertices of the kept component in their original order) — trimesh is not installed here, so this
  step is parity unpinned;
* vertices to the big-pose frame (:78-79); their blend weights (:82-84, ``anr_knn_blend``); the
  deformation ``-normal * sdf`` of ``gradient_of_deformed_sdf`` (:88-92, ``anr_sdf_points``); big pose ->
  T pose -> pose -> world (:96-101, ``anr_sdf_mesh_pose``).
"""
import numpy as np
import torch

from . import _lib
from . import config as _config
from .renderer_mesh import marching_cubes

MC_PAD = 10      # sdf_mesh_renderer.py:73
NORM_TH = 0.1    # :59


def largest_component(vertices, triangles):
    """``max(trimesh.Trimesh(v, t).split(), key=lambda m: len(m.vertices))`` (sdf_mesh_renderer.py:76-77):
    faces are connected through shared edges; only watertight components (every edge in exactly two of
    the component's faces) count, as ``split(only_watertight=True)``; the kept component's vertices keep
    their relative order (the sorted unique vertex ids of its faces) and its faces are renumbered.
    -> (vertices (V',3), triangles (T',3)); the inputs unchanged when no component is watertight."""
    v = np.asarray(vertices)
    t = np.asarray(triangles, dtype=np.int64)
    if len(t) == 0:
        return v, t
    e = np.sort(np.concatenate([t[:, [0, 1]], t[:, [1, 2]], t[:, [2, 0]]]), axis=1)
    face = np.tile(np.arange(len(t)), 3)
    key = e[:, 0] * (int(e.max()) + 1) + e[:, 1]
    order = np.argsort(key, kind='stable')
    ks, fs = key[order], face[order]
    # union-find over faces through each edge's faces
    parent = np.arange(len(t))

    def find(a):
        while parent[a] != a:
            parent[a] = parent[parent[a]]
            a = parent[a]
        return a
    same = np.nonzero(ks[1:] == ks[:-1])[0]
    for i in same:
        ra, rb = find(fs[i]), find(fs[i + 1])
        if ra != rb:
            parent[max(ra, rb)] = min(ra, rb)
    root = np.array([find(f) for f in range(len(t))])
    # watertight: every edge of the component appears exactly twice
    _, first, counts = np.unique(ks, return_index=True, return_counts=True)
    bad_edge_face = fs[first[counts != 2]]
    bad_roots = set(root[bad_edge_face].tolist())
    best, best_nv = None, -1
    for r in np.unique(root):
        if int(r) in bad_roots:
            continue
        nv = len(np.unique(t[root == r]))
        if nv > best_nv:
            best, best_nv = r, nv
    if best is None:
        return v, t
    ft = t[root == best]
    uv, inv = np.unique(ft, return_inverse=True)
    return v[uv], inv.reshape(-1, 3).astype(np.int64)


class Renderer:
    def __init__(self, net, cfg=None):
        self.net = net
        self.cfg = cfg if cfg is not None else _config.active()

    def sdf_volume(self, batch):
        """-> the padded cube (X+20, Y+20, Z+20) the reference hands to mcubes (:56-75), on the device"""
        dev = next(self.net.parameters()).device
        r = self.net._device()
        pts = batch['pts'].to(device=dev, dtype=torch.float32)
        sh = pts.shape
        flat = pts.reshape(-1, 3)
        inside = r.knn_blend(flat, batch['tvertices'][0], batch['weights'][0], NORM_TH, bw=False, inside=True)
        sdf = self.net.tpose_human.sdf_network(flat[inside], batch)[:, :1]
        full = torch.full((flat.shape[0],), 10.0, device=dev)
        full[inside] = sdf[:, 0]
        cube = torch.full(tuple(s + 2 * MC_PAD for s in sh[1:-1]), -10.0, device=dev)
        cube[MC_PAD:-MC_PAD, MC_PAD:-MC_PAD, MC_PAD:-MC_PAD] = (-full).reshape(sh[1:-1])
        return cube

    def posed_vertices(self, vertices, batch):
        """big-pose vertices (V,3) -> world-space posed vertices (V,3) (:81-102), on the device"""
        dev = next(self.net.parameters()).device
        r = self.net._device()
        pts = torch.as_tensor(vertices, device=dev).to(torch.float32).reshape(1, -1, 3)
        n = pts.shape[1]
        if n == 0:
            return pts[0]
        tbw = r.knn_blend(pts[0], batch['tvertices'][0], batch['weights'][0], NORM_TH, bw=True)
        normal, sdf = self.net.gradient_of_deformed_sdf(pts, batch)
        deformed = (pts + (-normal * sdf))[0].contiguous()
        keep = {k: batch[k].to(device=dev, dtype=torch.float32).contiguous() for k in ('big_A', 'A', 'R', 'Th')}
        out = torch.empty((n, 3), device=dev)
        _lib.check(r.lib.anr_sdf_mesh_pose(_lib.ptr(deformed), _lib.ptr(tbw.contiguous()), n, _lib.ptr(keep['big_A']),
                                           _lib.ptr(keep['A']), _lib.ptr(keep['R']), _lib.ptr(keep['Th']),
                                           _lib.ptr(out), _lib.stream_ptr(dev)), 'anr_sdf_mesh_pose')
        return out

    def render(self, batch):
        with torch.no_grad():
            cube = self.sdf_volume(batch)
            verts, tris = marching_cubes(cube, 0.0, 0)
            vertices, triangles = largest_component(verts.cpu().numpy(), tris.cpu().numpy())
            voxel = self.cfg.get('voxel_size', [0.005, 0.005, 0.005])
            vertices = (vertices - MC_PAD) * voxel[0]
            vertices = vertices + batch['tbounds'][0, 0].detach().cpu().numpy()
            posed = self.posed_vertices(vertices, batch).cpu().numpy()
        return {'vertex': vertices, 'posed_vertex': posed, 'triangle': triangles}
