"""Mesh renderer plugin (``lib/networks/renderer/aninerf_mesh_renderer.py``).

``Renderer(net).render(batch)`` takes the batch of ``lib/datasets/aninerf_mesh_dataset.py:126-174``
(``pts (1,X,Y,Z,3)`` voxel grid in world space, ``inside (1,X,Y,Z)``, frame keys) and returns
``{'vertex', 'posed_vertex', 'triangle'}`` as numpy arrays like the reference (:55-61):

* ``alpha_points``: ``Network.get_alpha`` (tpose_nerf_network.py:105-137) over the inside points,
  with the reference's batchify chunks of 2048 x 64 points (:14-23) — per-chunk forced argmin
  included — on the device (``anr_alpha_points``: prefilter, compaction and the density program
  of the fused network kernel);
* the volume ``cube[inside] = alpha`` (:38-41) is assembled on the device;
* ``marching_cubes``: ``mcubes.marching_cubes(np.pad(cube, 10), cfg.mesh_th)`` (:43-45) through
  ``anr_mc_count`` / ``anr_mc_emit`` (padding virtual), then ``(v - 10) * voxel_size[0] +
  wbounds[0]`` (:46-47).

PyMCubes is not installed here, so its triangulation cannot be pinned: the vertex set (one vertex
per crossing grid edge, linear interpolation) is table-independent; the triangles follow the case
table of ``tools/gen_mc_table.py`` (closed, consistently oriented surface). See DESIGN.md.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from . import renderer as _renderer

MESH_CHUNK = 2048 * 64   # aninerf_mesh_renderer.py:36
MESH_NORM_TH = 0.1       # tpose_nerf_network.py:113
MC_PAD = 10              # aninerf_mesh_renderer.py:43


def grid_points(wbounds, voxel_size):
    """The voxel grid of aninerf_mesh_dataset.py:143-153: float64 ``np.arange`` per axis over the
    world bounds, ``ij`` meshgrid, cast to float32 -> (X, Y, Z, 3)."""
    wb = np.asarray(wbounds)
    axes = [np.arange(wb[0, c], wb[1, c] + voxel_size[c], voxel_size[c]) for c in range(3)]
    return np.stack(np.meshgrid(*axes, indexing='ij'), axis=-1).astype(np.float32)


def marching_cubes(cube, iso, pad=MC_PAD):
    """Device marching cubes over ``cube`` (X,Y,Z) float32 padded by ``pad`` zeros per side:
    -> vertices (V,3) float64 in padded index coordinates, triangles (T,3) int64 (both on the
    cube's device). One host read of the two counts sizes the outputs."""
    lib = _lib.load()
    dev = cube.device
    vol = cube.to(torch.float32).contiguous()
    X, Y, Z = (int(s) for s in vol.shape)
    nbytes = lib.anr_mc_workspace_bytes(X, Y, Z, pad)
    ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
    counts = torch.zeros(2, dtype=torch.int32, device=dev)
    st = _lib.stream_ptr(dev)
    _lib.check(lib.anr_mc_count(_lib.ptr(vol), X, Y, Z, pad, float(iso), _lib.ptr(counts), _lib.ptr(ws), nbytes, st),
               'anr_mc_count')
    nv, nt = (int(v) for v in counts.cpu())
    verts = torch.empty((nv, 3), dtype=torch.float64, device=dev)
    tris = torch.empty((nt, 3), dtype=torch.int64, device=dev)
    if nv > 0 or nt > 0:
        _lib.check(lib.anr_mc_emit(_lib.ptr(vol), X, Y, Z, pad, float(iso), _lib.ptr(verts), _lib.ptr(tris),
                                   _lib.ptr(ws), nbytes, st), 'anr_mc_emit')
    return verts, tris


class Renderer(_renderer.Renderer):
    def _frame(self, batch, dev):
        keep = {}
        f = _lib.Frame()
        for k in ('A', 'R', 'Th', 'pbw', 'pbounds'):
            keep[k] = _renderer._f32(batch[k], dev)
        f.A, f.R, f.Th = keep['A'].data_ptr(), keep['R'].data_ptr(), keep['Th'].data_ptr()
        f.pbw, f.pbounds = keep['pbw'].data_ptr(), keep['pbounds'].data_ptr()
        for i in range(3):
            f.pbw_dims[i] = keep['pbw'].shape[1 + i]
        keep['li'] = batch['latent_index'].to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        keep['bli'] = batch.get('bw_latent_index', batch['latent_index']).to(
            device=dev, dtype=torch.int64).reshape(-1).contiguous()
        f.latent_index, f.bw_latent_index = keep['li'].data_ptr(), keep['bli'].data_ptr()
        return f, keep

    def alpha_points(self, wpts, batch, chunk_pts=MESH_CHUNK):
        """get_alpha of (n,3) world points -> (n,) raw alpha on the device (0 where dropped)."""
        p = self.params()
        dev = self._packed.device
        pts = _renderer._f32(wpts, dev).reshape(-1, 3)
        n = pts.shape[0]
        alpha = torch.zeros(n, device=dev)
        if n == 0:
            return alpha
        f, keep = self._frame(batch, dev)
        o = _lib.AlphaOpts()
        o.chunk_pts = int(chunk_pts)
        o.norm_th = MESH_NORM_TH
        o.novel_pose = 1 if self.cfg.get('test_novel_pose', False) else 0
        rprec = self.cfg.get('render_precision', 'fp32')
        rprecs = {'fp32': _lib.FP32, 'bf16x3': _lib.BF16X3, 'bf16x6': _lib.BF16X6}
        if rprec not in rprecs:
            raise ValueError(f"render_precision must be one of {sorted(rprecs)}, got {rprec!r}")
        o.precision = rprecs[rprec]
        nbytes = self.lib.anr_alpha_workspace_bytes(n, ctypes.byref(o), ctypes.byref(f))
        if nbytes == 0:
            raise ValueError('anr_alpha_workspace_bytes: bad arguments (chunk_pts must be a multiple of 64)')
        ws = self._workspace('_aws', nbytes, dev)
        _lib.check(self.lib.anr_alpha_points(ctypes.byref(p), ctypes.byref(f), _lib.ptr(pts), n, ctypes.byref(o),
                                             _lib.ptr(alpha), _lib.ptr(ws), nbytes, _lib.stream_ptr(dev)),
                   'anr_alpha_points')
        self._keep = keep
        return alpha

    _aws = None

    def alpha_volume(self, batch):
        """cube (X,Y,Z) float32 on the device: alpha at the inside voxels, 0 elsewhere (:30-41)."""
        dev = self.device()
        pts = batch['pts']
        sh = pts.shape
        inside = batch['inside'][0].to(dev).bool()
        wpts = _renderer._f32(pts[0], dev)[inside]
        alpha = self.alpha_points(wpts, batch)
        cube = torch.zeros(tuple(sh[1:-1]), device=dev)
        cube[inside] = alpha
        return cube

    def render(self, batch):
        with torch.no_grad():
            cube = self.alpha_volume(batch)
            verts, tris = marching_cubes(cube, float(self.cfg.get('mesh_th', 5.0)), MC_PAD)
        voxel = self.cfg.get('voxel_size', [0.005, 0.005, 0.005])
        wmin = batch['wbounds'][0, 0].detach().cpu().numpy()
        vertices = (verts.cpu().numpy() - MC_PAD) * voxel[0]
        vertices = vertices + wmin
        triangles = tris.cpu().numpy()
        return {'vertex': vertices, 'posed_vertex': vertices, 'triangle': triangles}
