"""Renderer plugin: ``Renderer(net).render(batch)`` (tpose_renderer.py:159-186) on the HIP library.

One call renders every ray of the batch through the C-ABI (``anr_render_fwd``): sampling,
prefilter, deformation, canonical NeRF and compositing run as device kernels, with the reference's
2048-ray chunk semantics (forced argmin keep, forced argmax loss row) preserved without a chunk
loop on the host. Output keys and shapes are the reference's:
``rgb_map (1,R,3)``, ``acc_map (1,R)``, ``depth_map (1,R)``, ``raw (1,R*64,4)``, ``pbw/tbw (1,m,24)``.
As in the reference (tpose_renderer.py:154-155), outputs that do not require grad are returned on
the CPU by ``render``; ``render_device`` keeps them in HBM.
"""
import ctypes

import torch

from . import _lib
from . import config as _config

CHUNK = 2048  # tpose_renderer.py:170


def _f32(t, device):
    return t.to(device=device, dtype=torch.float32).contiguous()


class Renderer:
    def __init__(self, net, cfg=None):
        self.net = net
        self.cfg = cfg if cfg is not None else _config.cfg
        self.lib = _lib.load()
        self._packed = None
        self._pack_key = None
        self._ws = None
        self.last_counts = None

    # ---- weights --------------------------------------------------------------------------
    def params(self):
        ts = [t.detach() for t in self.net.core_tensors()]
        dev = ts[0].device
        if dev.type != 'cuda':
            raise RuntimeError('Renderer: the network must be on a GPU (net.cuda()); there is no CPU path')
        for t in ts:
            if t.dtype != torch.float32 or not t.is_contiguous():
                raise RuntimeError('Renderer: parameters must be contiguous float32')
        p = _lib.Params()
        for i, t in enumerate(ts):
            p.t[i] = t.data_ptr()
        p.num_train_frame = self.net.num_train_frame
        key = tuple((t.data_ptr(), t._version) for t in ts)
        if self._packed is None or self._packed.device != dev:
            self._packed = torch.empty(self.lib.anr_params_packed_bytes(), dtype=torch.uint8, device=dev)
            self._pack_key = None
        p.packed = self._packed.data_ptr()
        if key != self._pack_key:
            _lib.check(self.lib.anr_params_pack(ctypes.byref(p), _lib.ptr(self._packed), _lib.stream_ptr(dev)),
                       'anr_params_pack')
            self._pack_key = key
        return p

    # ---- render -----------------------------------------------------------------------------
    def render_device(self, batch, t_rand=None, bw_rows=True):
        """Render on the GPU; all returned tensors stay in HBM. ``t_rand`` (R, N_samples) overrides
        the stratification draws (tests); by default they are drawn when perturb > 0 and the
        network is in training mode (tpose_renderer.py:29-36)."""
        p = self.params()
        dev = self._packed.device
        ray_o = _f32(batch['ray_o'], dev)
        ray_d = _f32(batch['ray_d'], dev)
        near = _f32(batch['near'], dev)
        far = _f32(batch['far'], dev)
        R = ray_o.shape[1]
        ns = int(self.cfg.N_samples)
        if t_rand is None and self.cfg.perturb > 0 and self.net.training:
            t_rand = torch.rand((R, ns), device=dev)
        if t_rand is not None:
            t_rand = _f32(t_rand, dev).reshape(R, ns)
        keep_alive = [ray_o, ray_d, near, far, t_rand]

        f = _lib.Frame()
        fr = {k: _f32(batch[k], dev) for k in ('A', 'R', 'Th', 'pbw', 'pbounds', 'tbw', 'tbounds')}
        li = batch['latent_index'].to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        keep_alive += list(fr.values()) + [li]
        f.A, f.R, f.Th = fr['A'].data_ptr(), fr['R'].data_ptr(), fr['Th'].data_ptr()
        f.pbw, f.pbounds = fr['pbw'].data_ptr(), fr['pbounds'].data_ptr()
        f.tbw, f.tbounds = fr['tbw'].data_ptr(), fr['tbounds'].data_ptr()
        for i in range(3):
            f.pbw_dims[i] = fr['pbw'].shape[1 + i]
            f.tbw_dims[i] = fr['tbw'].shape[1 + i]
        f.latent_index = li.data_ptr()

        o = _lib.RenderOpts()
        o.n_samples = ns
        o.chunk = int(self.cfg.get('chunk', CHUNK))
        o.norm_th = float(self.cfg.norm_th)
        o.train_th = float(self.cfg.train_th)
        o.t_rand = t_rand.data_ptr() if t_rand is not None else None

        rgb = torch.empty((1, R, 3), device=dev)
        acc = torch.empty((1, R), device=dev)
        depth = torch.empty((1, R), device=dev)
        raw = torch.empty((1, R * ns, 4), device=dev)
        out = _lib.RenderOut(rgb.data_ptr(), acc.data_ptr(), depth.data_ptr(), raw.data_ptr())

        ws_bytes = self.lib.anr_render_workspace_bytes(R, ctypes.byref(o), ctypes.byref(f))
        if self._ws is None or self._ws.numel() < ws_bytes or self._ws.device != dev:
            self._ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        stream = _lib.stream_ptr(dev)
        _lib.check(self.lib.anr_render_fwd(ctypes.byref(p), ctypes.byref(f), _lib.ptr(ray_o), _lib.ptr(ray_d),
                                           _lib.ptr(near), _lib.ptr(far), R, ctypes.byref(o), ctypes.byref(out),
                                           _lib.ptr(self._ws), ws_bytes, stream), 'anr_render_fwd')
        ret = {'rgb_map': rgb, 'acc_map': acc, 'depth_map': depth, 'raw': raw}
        if bw_rows:
            counts_addr = self.lib.anr_render_counts(_lib.ptr(self._ws), R)
            base = self._ws.data_ptr()
            counts = self._ws[counts_addr - base:counts_addr - base + 8].view(torch.int32).cpu()  # host sync
            n_kept, m = int(counts[0]), int(counts[1])
            self.last_counts = (n_kept, m)
            pbw = torch.empty((1, m, 24), device=dev)
            tbw = torch.empty((1, m, 24), device=dev)
            if m > 0:
                _lib.check(self.lib.anr_render_bw_rows(_lib.ptr(self._ws), R, _lib.ptr(pbw), _lib.ptr(tbw), stream),
                           'anr_render_bw_rows')
            ret['pbw'] = pbw
            ret['tbw'] = tbw
        del keep_alive
        return ret

    def render(self, batch):
        ret = self.render_device(batch)
        if not ret['rgb_map'].requires_grad:
            ret = {k: v.detach().cpu() for k, v in ret.items()}
        return ret

    def counts(self, n_rays):
        """(kept samples, alpha_ind rows) of the last render (device read, syncs)."""
        addr = self.lib.anr_render_counts(_lib.ptr(self._ws), n_rays)
        base = self._ws.data_ptr()
        c = self._ws[addr - base:addr - base + 8].view(torch.int32).cpu()
        return int(c[0]), int(c[1])


def near_far(bounds, ray_o, ray_d):
    """A14 on the GPU: (near (n',), far (n',), mask (n,) bool) like get_near_far
    (if_nerf_data_utils.py:156-196); bit-exact float64 plane tests."""
    lib = _lib.load()
    dev = ray_o.device
    ro = _f32(ray_o, dev).reshape(-1, 3)
    rd = _f32(ray_d, dev).reshape(-1, 3)
    b = _f32(bounds, dev).reshape(2, 3)
    n = ro.shape[0]
    mask = torch.empty(n, dtype=torch.uint8, device=dev)
    nr = torch.empty(n, device=dev)
    fr = torch.empty(n, device=dev)
    _lib.check(lib.anr_near_far(_lib.ptr(ro), _lib.ptr(rd), n, _lib.ptr(b), _lib.ptr(mask), _lib.ptr(nr),
                                _lib.ptr(fr), _lib.stream_ptr(dev)), 'anr_near_far')
    m = mask.bool()
    return nr[m], fr[m], m
