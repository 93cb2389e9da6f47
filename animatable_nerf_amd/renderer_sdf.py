"""Renderer plugin for the sdf_pdf network (config 5): ``Renderer(net).render(batch)`` as
``tpose_renderer.py:159-186`` runs it over ``anisdf_pdf_network.Network`` (``:156-223``).

One call renders every ray through ``anr_sdf_render_fwd`` (include/aninerf.h): KNN-blend prefilter,
LBS to the big pose, residual deformation, SDF network + its input gradient, Laplace density,
colour network, compositing and the ``msk_sdf`` lists, with the reference's 2048-ray chunk
semantics (forced argmin keep, the per-chunk in-place ``tbounds`` widening) kept on the device.
Output keys and shapes are the reference's eval outputs: ``raw (1,R*64,4)``, ``sdf (1,R*64,1)``,
``resd (1,n',3)``, ``gradients (1,n',3)``, ``rgb_map (1,R,3)``, ``acc_map``/``depth_map (1,R)``,
``msk_sdf``/``msk_label (1,L)``; ``render`` moves them to the CPU (``:154-155``) and, like the
reference, widens ``batch['tbounds']`` in place by 0.05 per chunk.

Training of this variant (``observed_gradients``, second-order grad loss) runs through
``trainer_sdf`` (``anr_sdf_train_step``); ``render`` with grad enabled points there.
"""
import ctypes

import torch

from . import _lib
from . import config as _config

CHUNK = 2048
RAY_KEYS = ('ray_o', 'ray_d', 'near', 'far')
FRAME_KEYS = ('A', 'big_A', 'R', 'Th', 'poses', 'pvertices', 'weights', 'tbounds')
NORM_TH = 0.1  # anisdf_pdf_network.py:172 (hard-coded, not cfg.norm_th)


def _f32(t, device):
    return t.to(device=device, dtype=torch.float32).contiguous()


def widen_tbounds(tbounds, k):
    """tbounds after the reference's in-place widening ran k times (anisdf_pdf_network.py:204-206):
    the same fp32 subtract / add per chunk as the device's k_sdf_tbtab, so the bits agree."""
    tb = tbounds.detach().clone().reshape(2, 3)
    for _ in range(int(k)):
        tb[0] -= 0.05
        tb[1] += 0.05
    return tb.reshape(tbounds.shape).contiguous()


class Renderer:
    widens_tbounds = True  # per chunk, in place (anisdf_pdf_network.py:204-206)

    def __init__(self, net, cfg=None):
        self.net = net
        self.cfg = cfg if cfg is not None else _config.active()
        self.lib = _lib.load()
        self._ws = None
        self.last_counts = None

    def device(self):
        return next(self.net.parameters()).device

    def params(self):
        ts = [t.detach() for t in self.net.tensors()]
        if ts[0].device.type != 'cuda':
            raise RuntimeError('Renderer: the network must be on a GPU (net.cuda()); there is no CPU path')
        p = _lib.SdfParams()
        for i, t in enumerate(ts):
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError('Renderer: parameters must be contiguous float32')
            p.t[i] = t.data_ptr()
        return p

    def prepare(self, batch, t_rand=None, chunk_offset=0):
        """Device tensors and C structs of one call over ``batch`` (kept alive in the returned dict):
        params, frame, rays, opts (render precision, stratification draws when perturbing)."""
        p = self.params()
        dev = self.device()
        R = batch['ray_o'].shape[1]
        ns = int(self.cfg.N_samples)
        if t_rand is None and self.cfg.perturb > 0 and self.net.training:
            t_rand = torch.rand((R, ns), device=dev)
        rays = {k: _f32(batch[k], dev) for k in RAY_KEYS}
        fr = {k: _f32(batch[k], dev) for k in FRAME_KEYS}
        if chunk_offset > 0:
            fr['tbounds'] = widen_tbounds(fr['tbounds'], chunk_offset)
        tr = None if t_rand is None else _f32(t_rand, dev).reshape(R, ns)
        li = batch['latent_index'].to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        occ = batch['occupancy'].to(device=dev, dtype=torch.uint8).reshape(-1).contiguous()
        f = _lib.SdfFrame()
        for k in FRAME_KEYS:
            setattr(f, k, fr[k].data_ptr())
        f.n_verts = fr['pvertices'].shape[-2]
        f.latent_index, f.occupancy = li.data_ptr(), occ.data_ptr()
        o = _lib.RenderOpts()
        o.n_samples, o.chunk, o.norm_th, o.train_th = ns, int(self.cfg.get('chunk', CHUNK)), NORM_TH, 0.0
        o.t_rand = tr.data_ptr() if tr is not None else None
        o.novel_pose = 0
        # cfg.render_precision 'fp32' (exact fp32 MFMA GEMMs) or 'bf16x3' (split-bf16 MFMA GEMMs for the
        # forward and input-gradient layers, fp32-level; include/aninerf.h anr_render_opts.precision)
        rprec = self.cfg.get('render_precision', 'fp32')
        if rprec not in ('fp32', 'bf16x3'):
            raise ValueError(f"render_precision must be 'fp32' or 'bf16x3', got {rprec!r}")
        o.precision = _lib.BF16X3 if rprec == 'bf16x3' else _lib.FP32
        return {'p': p, 'dev': dev, 'R': R, 'ns': ns, 'rays': rays, 'fr': fr, 't_rand': tr, 'li': li, 'occ': occ,
                'frame': f, 'opts': o}

    def render_device(self, batch, t_rand=None, chunk_offset=0, bw_rows=True):
        """All outputs stay in HBM; ``batch['tbounds']`` is widened in place (reference quirk).
        ``chunk_offset`` c0 > 0: these rays are the reference's chunks c0, c0+1, ... of a larger frame
        (a rank's shard, parallel.render_sharded): the reference has widened tbounds c0 times before
        them (anisdf_pdf_network.py:204-206), so the device starts from those bounds. ``bw_rows`` is
        accepted for the aninerf renderer's signature (this network has no pbw / tbw rows)."""
        c = self.prepare(batch, t_rand, chunk_offset)
        p, dev, R, ns, rays, f, o = c['p'], c['dev'], c['R'], c['ns'], c['rays'], c['frame'], c['opts']
        rgb = torch.empty((1, R, 3), device=dev)
        acc = torch.empty((1, R), device=dev)
        depth = torch.empty((1, R), device=dev)
        raw = torch.empty((1, R * ns, 4), device=dev)
        sdf = torch.empty((1, R * ns, 1), device=dev)
        tb_out = torch.empty((2, 3), device=dev)
        out = _lib.SdfRenderOut(rgb.data_ptr(), acc.data_ptr(), depth.data_ptr(), raw.data_ptr(), sdf.data_ptr(),
                                tb_out.data_ptr())
        ws_bytes = self.lib.anr_sdf_render_workspace_bytes(R, ctypes.byref(o))
        if self._ws is None or self._ws.numel() < ws_bytes or self._ws.device != dev:
            self._ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        ws = self._ws
        st = _lib.stream_ptr(dev)
        _lib.check(self.lib.anr_sdf_render_fwd(ctypes.byref(p), ctypes.byref(f), *[_lib.ptr(rays[k]) for k in RAY_KEYS],
                                               R, ctypes.byref(o), ctypes.byref(out), _lib.ptr(ws), ws_bytes, st),
                   'anr_sdf_render_fwd')
        addr = self.lib.anr_sdf_render_counts(_lib.ptr(ws), R, ctypes.byref(o))
        cnt = ws[addr - ws.data_ptr():addr - ws.data_ptr() + 8].view(torch.int32).cpu()  # host sync
        n_kept, n_msk = int(cnt[0]), int(cnt[1])
        self.last_counts = (n_kept, n_msk)
        resd = torch.empty((1, n_kept, 3), device=dev)
        grad = torch.empty((1, n_kept, 3), device=dev)
        msk_sdf = torch.empty((1, n_msk), device=dev)
        msk_label = torch.empty((1, n_msk), device=dev)
        _lib.check(self.lib.anr_sdf_render_rows(_lib.ptr(ws), R, ctypes.byref(o), _lib.ptr(resd), _lib.ptr(grad),
                                                _lib.ptr(msk_sdf), _lib.ptr(msk_label), st), 'anr_sdf_render_rows')
        with torch.no_grad():
            batch['tbounds'].copy_(tb_out.view_as(batch['tbounds']))
        self._last_R, self._last_opts = R, o
        return {'raw': raw, 'sdf': sdf, 'resd': resd, 'gradients': grad, 'rgb_map': rgb, 'acc_map': acc,
                'depth_map': depth, 'msk_sdf': msk_sdf, 'msk_label': msk_label}

    def knn_records(self):
        """(R*64, 8) uint32 view of the last render's KNN records (anr_sdf_render_knn): w0..w4 float
        bits, then the five vertex indices packed as i0 | i1 << 16, i2 | i3 << 16, i4 (tests, debugging)."""
        R = self._last_R
        addr = self.lib.anr_sdf_render_knn(_lib.ptr(self._ws), R, ctypes.byref(self._last_opts))
        if not addr:
            raise RuntimeError('anr_sdf_render_knn: no records')
        off = addr - self._ws.data_ptr()
        return self._ws[off:off + R * 64 * 32].view(torch.int32).view(R * 64, 8)

    def render(self, batch):
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.net.parameters()) and self.net.training:
            raise RuntimeError('sdf_pdf training runs as one fused step: use trainer_sdf.NetworkWrapper(net) '
                               '(tpose_trainer.py:21-73) or trainer_sdf.SdfStep; render under torch.no_grad() '
                               'for evaluation')
        with torch.no_grad():
            ret = self.render_device(batch)
        from .renderer import to_host
        return to_host(ret)
