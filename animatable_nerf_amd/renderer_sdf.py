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


def _sdf_precision(cfg):
    """cfg.render_precision (include/aninerf.h anr_render_opts.precision): 'fp32' exact fp32 MFMA layer
    GEMMs; 'bf16x3' the four fused launches in split bf16 (hi/lo, 3 products per multiply-add); 'bf16x6'
    the fused launches with hi/mid/lo bf16 (6 products, fp32-level, libm-grade softplus)."""
    rprec = cfg.get('render_precision', 'fp32')
    precs = {'fp32': _lib.FP32, 'bf16x3': _lib.BF16X3, 'bf16x6': _lib.BF16X6}
    if rprec not in precs:
        raise ValueError(f"render_precision must be one of {sorted(precs)}, got {rprec!r}")
    return precs[rprec]


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
    visibility_filter = False  # renderer_sdf_mmsk.Renderer turns it on

    def __init__(self, net, cfg=None):
        self.net = net
        self.cfg = cfg if cfg is not None else _config.active()
        self.lib = _lib.load()
        self._ws = None
        self._pcache = None  # (parameter pointers, SdfParams) of the last call
        self.last_counts = None

    def device(self):
        return next(self.net.parameters()).device

    def params(self):
        # per-call host work: the struct is rebuilt (detach + checks of 63 tensors, ~0.1 ms of Python that
        # the GPU waits out at every training step's host sync) only when a parameter moved
        key = tuple(t.data_ptr() for t in self.net.tensors())
        if self._pcache is not None and self._pcache[0] == key:
            return self._pcache[1]
        ts = [t.detach() for t in self.net.tensors()]
        if ts[0].device.type != 'cuda':
            raise RuntimeError('Renderer: the network must be on a GPU (net.cuda()); there is no CPU path')
        p = _lib.SdfParams()
        for i, t in enumerate(ts):
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError('Renderer: parameters must be contiguous float32')
            p.t[i] = t.data_ptr()
        self._pcache = (key, p)
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
        views = {}
        if self.visibility_filter:  # renderer_sdf_mmsk: tpose_renderer_mmsk.py:14-57 on the device
            views = {k: _f32(batch[k], dev) for k in ('Ks', 'RT')}
            views['msks'] = batch['msks'].to(device=dev, dtype=torch.uint8).contiguous()
            f.n_views = int(views['Ks'].shape[1])
            f.Ks, f.RT, f.msks = views['Ks'].data_ptr(), views['RT'].data_ptr(), views['msks'].data_ptr()
            f.img_h, f.img_w = int(batch['H']), int(batch['W'])
        o = _lib.RenderOpts()
        o.n_samples, o.chunk, o.norm_th, o.train_th = ns, int(self.cfg.get('chunk', CHUNK)), NORM_TH, 0.0
        o.t_rand = tr.data_ptr() if tr is not None else None
        o.novel_pose = 0
        o.precision = _sdf_precision(self.cfg)
        return {'p': p, 'dev': dev, 'R': R, 'ns': ns, 'rays': rays, 'fr': fr, 't_rand': tr, 'li': li, 'occ': occ,
                'frame': f, 'opts': o, 'views': views}

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

    # ---- Network.forward over free samples (anisdf_pdf_network.py:156-224) ------------------------
    def _net_frame(self, batch):
        """SdfFrame of one Network.forward call (no rays): the frame tensors, tbounds as a private copy
        (the call widens batch['tbounds'] in place; a backward re-run needs the bounds it started from)."""
        dev = self.device()
        fr = {k: _f32(batch[k], dev) for k in FRAME_KEYS}
        fr['tbounds'] = fr['tbounds'].clone()
        li = batch['latent_index'].to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        f = _lib.SdfFrame()
        for k in FRAME_KEYS:
            setattr(f, k, fr[k].data_ptr())
        f.n_verts = fr['pvertices'].shape[-2]
        f.latent_index, f.occupancy = li.data_ptr(), None
        o = _lib.RenderOpts()
        o.n_samples, o.chunk, o.norm_th, o.train_th = int(self.cfg.N_samples), 1, NORM_TH, 0.0
        o.t_rand, o.novel_pose = None, 0
        o.precision = _sdf_precision(self.cfg)
        return {'fr': fr, 'li': li, 'frame': f, 'opts': o}

    @staticmethod
    def _samples(wpts, viewdir, dists, dev):
        wp = _f32(wpts, dev).reshape(-1, 3)
        vd = _f32(viewdir, dev).reshape(-1, 3)
        n = wp.shape[0]
        if vd.shape[0] != n or dists.numel() != n:
            raise ValueError(f'Network.forward: wpts {tuple(wpts.shape)}, viewdir {tuple(viewdir.shape)}, '
                             f'dists {tuple(dists.shape)} disagree on the sample count')
        if n == 0:
            raise ValueError('Network.forward: no samples')
        return wp, vd, _lib.Samples(wp.data_ptr(), vd.data_ptr(), None, n)

    def network_forward(self, wpts, viewdir, dists, batch):
        """``Network.forward(wpts (n,3), viewdir (n,3), dists (n), batch)`` of anisdf_pdf_network (:156-224)
        -> {'raw' (1,n,4), 'sdf' (1,n,1), 'resd' (1,n',3), 'gradients' (1,n',3)} (+ 'observed_gradients'
        (1,n_o,3) under autograd when a kept sample has |sdf| < 0.02, :194-199); ``batch['tbounds']`` is
        widened by 0.05 in place, once per call (:204-206). One call = one reference chunk (the forced
        argmin spans the call). Under autograd with a training network: the layer-wise exact-fp32 executor
        (anr_sdf_network_train_fwd / _bwd), differentiable w.r.t. every parameter with the second-order
        terms of the reference's create_graph input gradients; else anr_sdf_network_fwd (render
        precision). ``dists`` is not read (the density uses the constant 0.005, :330)."""
        if torch.is_grad_enabled() and self.net.training and any(p.requires_grad for p in self.net.parameters()):
            outs = _SdfTrainNetwork.apply(self, batch, (wpts, viewdir, dists), *self.net.tensors())
            raw, sdf, resd, grad, og = outs
            ret = {'raw': raw, 'sdf': sdf, 'resd': resd, 'gradients': grad}
            if og.shape[1] > 0:
                ret['observed_gradients'] = og
            return ret
        with torch.no_grad():
            p = self.params()
            dev = self.device()
            c = self._net_frame(batch)
            wp, vd, x = self._samples(wpts, viewdir, dists, dev)
            n = x.n_pts
            raw = torch.empty((1, n, 4), device=dev)
            sdf = torch.empty((1, n, 1), device=dev)
            tb_out = torch.empty((2, 3), device=dev)
            ws_bytes = self.lib.anr_sdf_network_workspace_bytes(n, ctypes.byref(c['opts']))
            if self._ws is None or self._ws.numel() < ws_bytes or self._ws.device != dev:
                self._ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
            ws = self._ws
            st = _lib.stream_ptr(dev)
            _lib.check(self.lib.anr_sdf_network_fwd(ctypes.byref(p), ctypes.byref(c['frame']), ctypes.byref(x),
                                                    ctypes.byref(c['opts']), _lib.ptr(raw), _lib.ptr(sdf), _lib.ptr(tb_out),
                                                    _lib.ptr(ws), ws_bytes, st), 'anr_sdf_network_fwd')
            addr = self.lib.anr_sdf_network_counts(_lib.ptr(ws), n)
            n_kept = int(ws[addr - ws.data_ptr():addr - ws.data_ptr() + 4].view(torch.int32).item())  # host sync
            self.last_counts = (n_kept, 0)
            resd = torch.empty((1, n_kept, 3), device=dev)
            grad = torch.empty((1, n_kept, 3), device=dev)
            _lib.check(self.lib.anr_sdf_network_rows(_lib.ptr(ws), n, _lib.ptr(resd), _lib.ptr(grad), st),
                       'anr_sdf_network_rows')
            batch['tbounds'].copy_(tb_out.view_as(batch['tbounds']))
        return {'raw': raw, 'sdf': sdf, 'resd': resd, 'gradients': grad}

    # ---- the network's point helpers (anr_sdf_points; the sdf mesh path) ------------------------------
    def points(self, x, batch, mode):
        """anr_sdf_points over x (n,3) big-pose points: mode _lib.SDFP_NETWORK -> (n,257) [sdf || feature]
        (tpose_human.sdf_network, anisdf_pdf_network.py:421-437); SDFP_GRADIENT -> (d sdf/dx (n,3), sdf (n,1))
        (SDFNetwork.gradient, :441-451); SDFP_DEFORMED_GRADIENT -> (gradient of sdf(x + resd(x)) (n,3), that
        sdf (n,1)) (Network.gradient_of_deformed_sdf, :140-154). Exact fp32 products; no host sync."""
        dev = self.device()
        p = self.params()
        xs = _f32(x, dev).reshape(-1, 3)
        n = xs.shape[0]
        out = torch.empty((n, 257) if mode == _lib.SDFP_NETWORK else (n, 3), device=dev)
        out2 = None if mode == _lib.SDFP_NETWORK else torch.empty((n, 1), device=dev)
        if n == 0:
            return out if out2 is None else (out, out2)
        poses = _f32(batch['poses'], dev)
        li = batch['latent_index'].to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        f = _lib.SdfFrame()
        f.poses, f.latent_index = poses.data_ptr(), li.data_ptr()
        ws_bytes = self.lib.anr_sdf_points_workspace_bytes(n)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        _lib.check(self.lib.anr_sdf_points(ctypes.byref(p), ctypes.byref(f), _lib.ptr(xs), n, int(mode), _lib.ptr(out),
                                           _lib.ptr(out2) if out2 is not None else None, _lib.ptr(ws), ws_bytes,
                                           _lib.stream_ptr(dev)), 'anr_sdf_points')
        return out if out2 is None else (out, out2)

    def knn_blend(self, pts, verts, weights, norm_th=NORM_TH, bw=True, inside=False):
        """sample_blend_closest_points (sample_utils.py:323-348) of pts (n,3) against verts (nv,3) / weights
        (nv,24): -> blended weights (n,24) and / or the mask weighted-distance < norm_th (n,) bool."""
        dev = self.device()
        ps = _f32(pts, dev).reshape(-1, 3)
        vs = _f32(verts, dev).reshape(-1, 3)
        ws_ = _f32(weights, dev).reshape(-1, 24)
        n = ps.shape[0]
        out_bw = torch.empty((n, 24), device=dev) if bw else None
        out_in = torch.empty((n,), dtype=torch.uint8, device=dev) if inside else None
        if n > 0:
            nbytes = self.lib.anr_knn_blend_workspace_bytes(n)
            wk = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            _lib.check(self.lib.anr_knn_blend(_lib.ptr(vs), _lib.ptr(ws_), vs.shape[0], _lib.ptr(ps), n, float(norm_th),
                                              _lib.ptr(out_bw) if bw else None, _lib.ptr(out_in) if inside else None,
                                              _lib.ptr(wk), nbytes, _lib.stream_ptr(dev)), 'anr_knn_blend')
        res = tuple(v for v in (out_bw, None if out_in is None else out_in.bool()) if v is not None)
        return res[0] if len(res) == 1 else res

    def render(self, batch):
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.net.parameters()) and self.net.training:
            raise RuntimeError('sdf_pdf training runs as one fused step: use trainer_sdf.NetworkWrapper(net) '
                               '(tpose_trainer.py:21-73) or trainer_sdf.SdfStep; render under torch.no_grad() '
                               'for evaluation')
        with torch.no_grad():
            ret = self.render_device(batch)
        from .renderer import to_host
        return to_host(ret)


class _SdfTrainNetwork(torch.autograd.Function):
    """sdf_pdf Network.forward under autograd: forward = anr_sdf_network_train_fwd (raw, sdf, resd,
    gradients, observed_gradients), backward = anr_sdf_network_train_bwd from the upstream adjoints of
    all five (parameter gradients; the inputs wpts / viewdir / dists get none: the reference's renderer
    builds them without grad)."""

    @staticmethod
    def forward(ctx, renderer, batch, samples, *params):
        lib = renderer.lib
        p = renderer.params()
        dev = params[0].device
        c = renderer._net_frame(batch)
        wp, vd, x = renderer._samples(*samples, dev)
        n = x.n_pts
        ws_bytes = lib.anr_sdf_network_train_workspace_bytes(n)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)  # owned by this forward until its backward
        raw = torch.empty((1, n, 4), device=dev)
        sdf = torch.empty((1, n, 1), device=dev)
        tb_out = torch.empty((2, 3), device=dev)
        st = _lib.stream_ptr(dev)
        _lib.check(lib.anr_sdf_network_train_fwd(ctypes.byref(p), ctypes.byref(c['frame']), ctypes.byref(x),
                                                 ctypes.byref(c['opts']), _lib.ptr(raw), _lib.ptr(sdf), _lib.ptr(tb_out),
                                                 _lib.ptr(ws), ws_bytes, st), 'anr_sdf_network_train_fwd')
        addr = lib.anr_sdf_network_train_counts(_lib.ptr(ws), n)
        cnt = ws[addr - ws.data_ptr():addr - ws.data_ptr() + 16].view(torch.int32).cpu()  # host sync
        n_kept, n_obs = int(cnt[0]), int(cnt[2])
        renderer.last_counts = (n_kept, n_obs)
        resd = torch.empty((1, n_kept, 3), device=dev)
        grad = torch.empty((1, n_kept, 3), device=dev)
        og = torch.empty((1, n_obs, 3), device=dev)
        _lib.check(lib.anr_sdf_network_train_rows(_lib.ptr(ws), n, _lib.ptr(resd), _lib.ptr(grad), _lib.ptr(og), st),
                   'anr_sdf_network_train_rows')
        with torch.no_grad():
            batch['tbounds'].copy_(tb_out.view_as(batch['tbounds']))
        ctx.renderer, ctx.c, ctx.samples, ctx.ws, ctx.ws_bytes = renderer, c, (wp, vd, x), ws, ws_bytes
        return raw, sdf, resd, grad, og

    @staticmethod
    def backward(ctx, d_raw, d_sdf, d_resd, d_grad, d_og):
        r, c = ctx.renderer, ctx.c
        params = r.net.tensors()
        dev = params[0].device
        p = r.params()
        grads = [torch.zeros_like(t) for t in params]
        gp = (ctypes.c_void_p * _lib.NUM_SDF_TENSORS)(*[g.data_ptr() for g in grads])
        keep = [t.contiguous() if t is not None else None for t in (d_raw, d_sdf, d_resd, d_grad, d_og)]
        _lib.check(r.lib.anr_sdf_network_train_bwd(ctypes.byref(p), gp, ctypes.byref(c['frame']),
                                                   ctypes.byref(ctx.samples[2]), ctypes.byref(c['opts']),
                                                   *[_lib.ptr(t) for t in keep], _lib.ptr(ctx.ws), ctx.ws_bytes,
                                                   _lib.stream_ptr(dev)), 'anr_sdf_network_train_bwd')
        return (None, None, None, *grads)
