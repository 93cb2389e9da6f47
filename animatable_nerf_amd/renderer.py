"""Renderer plugin: ``Renderer(net).render(batch)`` (tpose_renderer.py:159-186) on the HIP library.

One call renders every ray of the batch through the C-ABI: sampling, prefilter, deformation,
canonical NeRF and compositing run as device kernels, with the reference's 2048-ray chunk semantics
(forced argmin keep, forced argmax loss row) preserved without a chunk loop on the host. Output keys
and shapes are the reference's: ``rgb_map (1,R,3)``, ``acc_map (1,R)``, ``depth_map (1,R)``,
``raw (1,R*64,4)``, ``pbw/tbw (1,m,24)``.

* no grad (evaluation, run.py:63-69): the fused single-kernel network (``anr_render_fwd``); outputs
  are moved to the CPU by ``render`` as the reference does (tpose_renderer.py:154-155),
  ``render_device`` keeps them in HBM;
* grad enabled (training, tpose_trainer.py:22): the layer-wise training executor
  (``anr_train_fwd``) behind a ``torch.autograd.Function`` whose backward is ``anr_train_bwd``, so
  the reference's ``loss.backward()`` / optimizer loop drives it unchanged.
"""
import ctypes
import os

import torch

from . import _lib
from . import config as _config

CHUNK = 2048  # tpose_renderer.py:170
RAY_KEYS = ('ray_o', 'ray_d', 'near', 'far')
FRAME_KEYS = ('A', 'R', 'Th', 'pbw', 'pbounds', 'tbw', 'tbounds')


def _f32(t, device):
    return t.to(device=device, dtype=torch.float32).contiguous()


class _Call:
    """Device tensors + C structs of one render/train call (keeps the tensors alive)."""

    def __init__(self, renderer, batch, t_rand, samples=None):
        cfg = renderer.cfg
        self.dev = dev = renderer.device()
        ns = int(cfg.N_samples)
        if samples is None:
            self.rays = {k: _f32(batch[k], dev) for k in RAY_KEYS}
            self.R = R = self.rays['ray_o'].shape[1]
            self.t_rand = None if t_rand is None else _f32(t_rand, dev).reshape(R, ns)
        else:  # Network.forward(wpts, viewdir, dists, batch): free samples instead of rays
            wpts, viewdir, dists = samples
            self.wpts = _f32(wpts, dev).reshape(-1, 3)
            self.vdir = _f32(viewdir, dev).reshape(-1, 3)
            self.dists = _f32(dists, dev).reshape(-1)
            n = self.wpts.shape[0]
            if self.vdir.shape[0] != n or self.dists.shape[0] != n:
                raise ValueError(f'Network.forward: wpts {tuple(wpts.shape)}, viewdir {tuple(viewdir.shape)}, '
                                 f'dists {tuple(dists.shape)} disagree on the sample count')
            self.samples = _lib.Samples(self.wpts.data_ptr(), self.vdir.data_ptr(), self.dists.data_ptr(), n)
            self.n = n
            self.t_rand = None
        fr = {k: _f32(batch[k], dev) for k in FRAME_KEYS}
        self.fr = fr
        self.li = batch['latent_index'].to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        bli = batch.get('bw_latent_index', batch['latent_index'])
        self.bli = bli.to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        f = _lib.Frame()
        f.A, f.R, f.Th = fr['A'].data_ptr(), fr['R'].data_ptr(), fr['Th'].data_ptr()
        f.pbw, f.pbounds = fr['pbw'].data_ptr(), fr['pbounds'].data_ptr()
        f.tbw, f.tbounds = fr['tbw'].data_ptr(), fr['tbounds'].data_ptr()
        for i in range(3):
            f.pbw_dims[i] = fr['pbw'].shape[1 + i]
            f.tbw_dims[i] = fr['tbw'].shape[1 + i]
        f.latent_index = self.li.data_ptr()
        f.bw_latent_index = self.bli.data_ptr()
        f.n_views = 0
        if renderer.visibility_filter and 'msks' in batch:
            # tpose_renderer_mmsk.py:14-57 keys (tpose_novel_view_dataset.py:191)
            self.Ks = _f32(batch['Ks'], dev).reshape(-1, 3, 3)
            self.RT = _f32(batch['RT'], dev).reshape(-1, 3, 4)
            self.msks = batch['msks'].to(device=dev, dtype=torch.uint8).contiguous()
            f.n_views = self.Ks.shape[0]
            f.Ks, f.RT, f.msks = self.Ks.data_ptr(), self.RT.data_ptr(), self.msks.data_ptr()
            f.img_h, f.img_w = int(batch['H'].reshape(-1)[0]), int(batch['W'].reshape(-1)[0])
            if tuple(self.msks.shape[-2:]) != (f.img_h, f.img_w):
                raise ValueError(f"msks {tuple(self.msks.shape)} do not match H, W = {f.img_h}, {f.img_w}")
        self.frame = f
        o = _lib.RenderOpts()
        o.n_samples = ns
        o.chunk = int(cfg.get('chunk', CHUNK))
        o.norm_th = float(cfg.norm_th)
        o.train_th = float(cfg.train_th)
        o.t_rand = self.t_rand.data_ptr() if self.t_rand is not None else None
        o.novel_pose = 1 if cfg.get('test_novel_pose', False) else 0
        prec = cfg.get('train_precision', 'fp32')
        precs = {'fp32': _lib.FP32, 'bf16': _lib.BF16, 'bf16_all': _lib.BF16_ALL}
        if prec not in precs:
            raise ValueError(f"train_precision must be one of {sorted(precs)}, got {prec!r}")
        o.precision = precs[prec]
        self.render_precision = _lib.FP32
        rprec = cfg.get('render_precision', 'fp32')
        rprecs = {'fp32': _lib.FP32, 'bf16x3': _lib.BF16X3, 'bf16x6': _lib.BF16X6}
        if rprec not in rprecs:
            raise ValueError(f"render_precision must be one of {sorted(rprecs)}, got {rprec!r}")
        self.render_precision = rprecs[rprec]
        self.opts = o
        if samples is not None:
            return
        self.rgb = torch.empty((1, R, 3), device=dev)
        self.acc = torch.empty((1, R), device=dev)
        self.depth = torch.empty((1, R), device=dev)
        self.raw = torch.empty((1, R * ns, 4), device=dev)
        self.out = _lib.RenderOut(self.rgb.data_ptr(), self.acc.data_ptr(), self.depth.data_ptr(), self.raw.data_ptr())

    def ray_ptrs(self):
        return [_lib.ptr(self.rays[k]) for k in RAY_KEYS]


class Renderer:
    visibility_filter = False  # renderer_mmsk.Renderer turns it on

    def __init__(self, net, cfg=None):
        self.net = net
        self.cfg = cfg if cfg is not None else _config.active()
        self.lib = _lib.load()
        self._packed = None
        self._pack_key = None
        self._ws = None
        self._tws = None
        self.last_counts = None

    def device(self):
        return next(self.net.parameters()).device

    # ---- weights --------------------------------------------------------------------------
    def params(self, pack=True):
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
        novel = self.net.novel_tensors()
        for i, t in enumerate(novel):
            p.novel[i] = t.detach().data_ptr()
        ts = ts + [t.detach() for t in novel]
        if not pack:
            return p
        key = (getattr(self.net, '_anr_weights_epoch', 0),) + tuple((t.data_ptr(), t._version) for t in ts)
        if self._packed is None or self._packed.device != dev:
            self._packed = torch.empty(self.lib.anr_params_packed_bytes(), dtype=torch.uint8, device=dev)
            self._pack_key = None
        p.packed = self._packed.data_ptr()
        if key != self._pack_key:
            _lib.check(self.lib.anr_params_pack(ctypes.byref(p), _lib.ptr(self._packed), _lib.stream_ptr(dev)),
                       'anr_params_pack')
            self._pack_key = key
        return p

    def _workspace(self, attr, nbytes, dev):
        ws = getattr(self, attr, None)
        if ws is None or ws.numel() < nbytes or ws.device != dev:
            ws = torch.empty(nbytes, dtype=torch.uint8, device=dev)
            setattr(self, attr, ws)
        return ws

    def _counts(self, ws, R):
        addr = self.lib.anr_render_counts(_lib.ptr(ws), R)
        base = ws.data_ptr()
        c = ws[addr - base:addr - base + 8].view(torch.int32).cpu()  # host sync
        self.last_counts = (int(c[0]), int(c[1]))
        return self.last_counts

    def _bw_rows(self, ws, R, dev):
        _, m = self._counts(ws, R)
        pbw = torch.empty((1, m, 24), device=dev)
        tbw = torch.empty((1, m, 24), device=dev)
        if m > 0:
            _lib.check(self.lib.anr_render_bw_rows(_lib.ptr(ws), R, _lib.ptr(pbw), _lib.ptr(tbw), _lib.stream_ptr(dev)),
                       'anr_render_bw_rows')
        return pbw, tbw

    def _last_device_ws(self, what):
        """The workspace of the last render_device() call. render() renders a frame in parts on two
        workspaces, so after it no single workspace describes the frame: use last_counts there."""
        ws = getattr(self, '_last_ws', None)
        if ws is None:
            raise RuntimeError(f'Renderer.{what} describes the last render_device() call; the last render was '
                               'render() (the frame in parts): use Renderer.last_counts')
        return ws

    def row_ids(self, n_rays):
        """Sample ids (ray * N_samples + sample) of the alpha_ind rows of the last render_device(), (m,)
        int64 on the device, in row order (anr_render_row_ids)."""
        ws = self._last_device_ws('row_ids()')
        _, m = self._counts(ws, n_rays)
        ids = torch.empty((m,), dtype=torch.int32, device=ws.device)
        if m > 0:
            _lib.check(self.lib.anr_render_row_ids(_lib.ptr(ws), n_rays, _lib.ptr(ids),
                                                   _lib.stream_ptr(ws.device)), 'anr_render_row_ids')
        return ids.long()

    def _t_rand(self, R, dev, t_rand):
        if t_rand is None and self.cfg.perturb > 0 and self.net.training:
            t_rand = torch.rand((R, int(self.cfg.N_samples)), device=dev)
        return t_rand

    # ---- render -----------------------------------------------------------------------------
    def render_device(self, batch, t_rand=None, bw_rows=True):
        """Evaluation render on the GPU (fused network kernel); all returned tensors stay in HBM.
        ``t_rand`` (R, N_samples) overrides the stratification draws (tests); by default they are
        drawn when perturb > 0 and the network is in training mode (tpose_renderer.py:29-36)."""
        p = self.params()
        dev = self._packed.device
        R = batch['ray_o'].shape[1]
        c = _Call(self, batch, self._t_rand(R, dev, t_rand))
        ws_bytes = self.lib.anr_render_workspace_bytes(R, ctypes.byref(c.opts), ctypes.byref(c.frame))
        ws = self._workspace('_ws', ws_bytes, dev)
        c.opts.precision = c.render_precision
        _lib.check(self.lib.anr_render_fwd(ctypes.byref(p), ctypes.byref(c.frame), *c.ray_ptrs(), R,
                                           ctypes.byref(c.opts), ctypes.byref(c.out), _lib.ptr(ws), ws_bytes,
                                           _lib.stream_ptr(dev)), 'anr_render_fwd')
        self._last_ws = ws
        ret = {'rgb_map': c.rgb, 'acc_map': c.acc, 'depth_map': c.depth, 'raw': c.raw}
        if bw_rows:
            ret['pbw'], ret['tbw'] = self._bw_rows(ws, R, dev)
        return ret

    def render_train(self, batch, t_rand=None):
        """Training forward (autograd-enabled): returns the render dict; ``rgb_map``, ``pbw`` and
        ``tbw`` carry gradients to every network parameter through ``anr_train_bwd``."""
        dev = self.device()
        R = batch['ray_o'].shape[1]
        t_rand = self._t_rand(R, dev, t_rand)
        params = self.net.core_tensors()
        rgb, acc, depth, raw, pbw, tbw = _TrainRender.apply(self, batch, t_rand, *params)
        return {'rgb_map': rgb, 'acc_map': acc, 'depth_map': depth, 'raw': raw, 'pbw': pbw, 'tbw': tbw}

    # render(): the frame in this many parts (whole reference chunks) so part k's outputs cross the
    # host link while part k + 1 renders (a 512x512 frame moves ~1.4 GB to the host); 8 parts measured
    # 146.0 ms against 149.3 for 4 (profiles/r6c_*); ANR_HOST_PARTS overrides (read per call)
    HOST_PARTS = 8
    # headroom of the alpha_ind row buffers over the previous frame's row count
    ROWS_HEADROOM = 1.125

    def render(self, batch):
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.net.parameters()) and self.net.training:
            return self.render_train(batch)
        R = batch['ray_o'].shape[1]
        chunk = int(self.cfg.get('chunk', CHUNK))
        n_chunks = (R + chunk - 1) // chunk
        # at least two chunks per part; fewer than two parts: one device render and one copy
        parts = min(int(os.environ.get('ANR_HOST_PARTS', self.HOST_PARTS)), n_chunks // 2)
        with torch.no_grad():
            if parts < 2 or not self.device().type == 'cuda':
                return to_host(self.render_device(batch))
            return self._render_overlapped(batch, R, chunk, parts)

    def _render_launch(self, batch, attr):
        """anr_render_fwd of one part on the current stream into workspace `attr`, no host read."""
        p = self.params()
        dev = self._packed.device
        R = batch['ray_o'].shape[1]
        c = _Call(self, batch, self._t_rand(R, dev, None))
        ws_bytes = self.lib.anr_render_workspace_bytes(R, ctypes.byref(c.opts), ctypes.byref(c.frame))
        ws = self._workspace(attr, ws_bytes, dev)
        c.opts.precision = c.render_precision
        _lib.check(self.lib.anr_render_fwd(ctypes.byref(p), ctypes.byref(c.frame), *c.ray_ptrs(), R,
                                           ctypes.byref(c.opts), ctypes.byref(c.out), _lib.ptr(ws), ws_bytes,
                                           _lib.stream_ptr(dev)), 'anr_render_fwd')
        return c, ws, R

    def _render_overlapped(self, batch, R, chunk, parts):
        """The frame in parts of whole chunks (per-chunk semantics unchanged: the rows of the parts,
        concatenated in order, are the whole frame's, as parallel.render_sharded relies on), pipelined:
        part k + 1 is issued (on the other of two workspaces) before part k's row count is read, so the
        GPU renders back to back while the host reads counts; part k's alpha_ind rows are extracted and
        every output of it copied into page-locked host buffers on a side stream. The alpha_ind rows go
        to their final offset in one (1, cap, 24) page-locked buffer sized from the previous frame's row
        count with ROWS_HEADROOM (the first frame: from the rows seen so far), and the returned (1, m, 24)
        tensors are its first m rows (contiguous; no capacity-sized host buffer, no host concatenation).
        A frame whose rows outgrow the buffer moves the placed rows into an exact-size one (one host
        copy) and the rest from the device."""
        from .parallel import RAY_KEYS as SLICED, shard_chunks
        dev = self.device()
        ns = int(self.cfg.N_samples)
        with torch.cuda.device(dev):
            if getattr(self, '_copy_stream', None) is None:
                self._copy_stream = torch.cuda.Stream(dev)
            cs = self._copy_stream
            cur = torch.cuda.current_stream(dev)
            pin = dict(dtype=torch.float32, pin_memory=True)
            h = {'rgb_map': torch.empty((1, R, 3), **pin), 'acc_map': torch.empty((1, R), **pin),
                 'depth_map': torch.empty((1, R), **pin), 'raw': torch.empty((1, R * ns, 4), **pin)}
            st = dict(late=[], kept=0, off=0, hp=None, ht=None, keep=[], k=0)
            self._last_ws = None  # the parts alternate between two workspaces (row_ids / counts refuse)
            # the previous frame's row count, when it had the same rays (another frame size: extrapolated)
            est_R, est_m = getattr(self, '_rows_est', (0, 0))
            est = int(est_m) if est_R == R else 0
            ws_free = [None, None]  # per workspace: an event on cs after its last part's rows were extracted

            def finish(part):
                a, b, c, ws, Rp, launched, slot = part
                with torch.cuda.stream(cs):
                    cs.wait_event(launched)  # this part only (the next one is queued behind it on cur)
                    addr = self.lib.anr_render_counts(_lib.ptr(ws), Rp)
                    cnt = ws[addr - ws.data_ptr():addr - ws.data_ptr() + 8].view(torch.int32).cpu()  # host read
                    kept_k, n = int(cnt[0]), int(cnt[1])
                    pr = torch.empty((1, n, 24), device=dev)
                    tr = torch.empty((1, n, 24), device=dev)
                    if n:
                        _lib.check(self.lib.anr_render_bw_rows(_lib.ptr(ws), Rp, _lib.ptr(pr), _lib.ptr(tr),
                                                               _lib.stream_ptr(dev)), 'anr_render_bw_rows')
                    ev = torch.cuda.Event()
                    ev.record(cs)
                    ws_free[slot] = ev
                    if st['hp'] is None and (est > 0 or n > 0):
                        # the previous frame's rows, or (first frame) the rows per part so far, extrapolated
                        guess = est if est > 0 else (st['off'] + n) * parts // (st['k'] + 1)
                        cap = int(guess * self.ROWS_HEADROOM) + 64
                        st['hp'] = torch.empty((1, cap, 24), **pin)
                        st['ht'] = torch.empty((1, cap, 24), **pin)
                    h['rgb_map'][:, a:b].copy_(c.rgb, non_blocking=True)
                    h['acc_map'][:, a:b].copy_(c.acc, non_blocking=True)
                    h['depth_map'][:, a:b].copy_(c.depth, non_blocking=True)
                    h['raw'][:, a * ns:b * ns].copy_(c.raw, non_blocking=True)
                    off, hp, ht = st['off'], st['hp'], st['ht']
                    if n and hp is not None and off + n <= hp.shape[1] and not st['late']:
                        hp[:, off:off + n].copy_(pr, non_blocking=True)
                        ht[:, off:off + n].copy_(tr, non_blocking=True)
                    elif n:
                        st['late'].append((off, pr, tr))
                st['keep'].append((c, pr, tr))  # device tensors alive until the copies are done
                st['off'] += n
                st['kept'] += kept_k
                st['k'] += 1

            pending = None
            for k in range(parts):
                a, b = shard_chunks(R, k, parts, chunk)
                if a >= b:
                    continue
                slot = k % 2
                if ws_free[slot] is not None:
                    cur.wait_event(ws_free[slot])  # the workspace's previous part has its rows out
                sub = {key_: (v[:, a:b] if key_ in SLICED and torch.is_tensor(v) else v) for key_, v in batch.items()}
                c, ws, Rp = self._render_launch(sub, '_ws' if slot == 0 else '_ws_b')
                launched = torch.cuda.Event()
                launched.record(cur)
                if pending is not None:
                    finish(pending)
                pending = (a, b, c, ws, Rp, launched, slot)
            if pending is not None:
                finish(pending)
            m = st['off']
            late, hp, ht = st['late'], st['hp'], st['ht']
            if late or hp is None:
                # outgrew the estimate: the placed rows into exact-size buffers, the rest from the device
                cs.synchronize()
                placed = late[0][0] if late else 0
                ep = torch.empty((1, m, 24), **pin)
                et = torch.empty((1, m, 24), **pin)
                if placed:
                    ep[:, :placed].copy_(hp[:, :placed])
                    et[:, :placed].copy_(ht[:, :placed])
                with torch.cuda.stream(cs):
                    for o, p, t in late:
                        ep[:, o:o + p.shape[1]].copy_(p, non_blocking=True)
                        et[:, o:o + t.shape[1]].copy_(t, non_blocking=True)
                hp, ht = ep, et
            cs.synchronize()
            cur.wait_stream(cs)  # later work on the caller's stream may reuse the workspaces
            if hp.shape[1] > 2 * m + 4096:
                # the estimate overshot (another frame's rows): exact-size buffers, so the returned tensors
                # hold no capacity-sized host allocation
                hp = torch.empty((1, m, 24), **pin).copy_(hp[:, :m])
                ht = torch.empty((1, m, 24), **pin).copy_(ht[:, :m])
            h['pbw'] = hp[:, :m]
            h['tbw'] = ht[:, :m]
        self._rows_est = (R, m)
        self.last_counts = (st['kept'], m)
        return h

    def counts(self, n_rays):
        """(kept samples, alpha_ind rows) of the last render_device() (device read, syncs); after render()
        (the frame in parts) see last_counts."""
        return self._counts(self._last_device_ws('counts()'), n_rays)

    # ---- Network.forward over free samples (tpose_nerf_network.py:139-215) -----------------
    def network_forward(self, wpts, viewdir, dists, batch):
        """``Network.forward(wpts (n,3), viewdir (n,3), dists (n), batch)`` -> {'raw' (1,n,4), 'pbw' (1,m,24),
        'tbw' (1,m,24)}: one reference network call (its forced argmin / argmax span the call). Under autograd
        with a training network: the layer-wise executor (anr_network_train_fwd/bwd); else the fused kernel."""
        if torch.is_grad_enabled() and self.net.training and any(p.requires_grad for p in self.net.parameters()):
            raw, pbw, tbw = _TrainNetwork.apply(self, batch, (wpts, viewdir, dists), *self.net.core_tensors())
            return {'pbw': pbw, 'tbw': tbw, 'raw': raw}
        with torch.no_grad():
            p = self.params()
            dev = self._packed.device
            c = _Call(self, batch, None, samples=(wpts, viewdir, dists))
            c.opts.precision = c.render_precision
            ws_bytes = self.lib.anr_network_workspace_bytes(c.n, ctypes.byref(c.opts), ctypes.byref(c.frame))
            ws = self._workspace('_nws', ws_bytes, dev)
            raw = torch.empty((1, c.n, 4), device=dev)
            _lib.check(self.lib.anr_network_fwd(ctypes.byref(p), ctypes.byref(c.frame), ctypes.byref(c.samples),
                                                ctypes.byref(c.opts), _lib.ptr(raw), _lib.ptr(ws), ws_bytes,
                                                _lib.stream_ptr(dev)), 'anr_network_fwd')
            pbw, tbw = self._net_rows(ws, c.n, dev)
        return {'pbw': pbw, 'tbw': tbw, 'raw': raw}

    def _net_rows(self, ws, n, dev):
        addr = self.lib.anr_network_counts(_lib.ptr(ws), n)
        base = ws.data_ptr()
        cnt = ws[addr - base:addr - base + 8].view(torch.int32).cpu()  # host sync (the reference's alpha_ind)
        self.last_counts = (int(cnt[0]), int(cnt[1]))
        m = self.last_counts[1]
        pbw = torch.empty((1, m, 24), device=dev)
        tbw = torch.empty((1, m, 24), device=dev)
        if m > 0:
            _lib.check(self.lib.anr_network_bw_rows(_lib.ptr(ws), n, _lib.ptr(pbw), _lib.ptr(tbw), _lib.stream_ptr(dev)),
                       'anr_network_bw_rows')
        return pbw, tbw

    def blend_weights(self, pts, smpl_bw, latent_index, field=0, row_add=0):
        """calculate_neural_blend_weights (field 0, tpose_nerf_network.py:55-77) / novel_pose_bw (field 1,
        :304-315): pts (1,n,3), smpl_bw (1,24,n), latent_index (int64 tensor) -> bw (1,24,n). Forward only."""
        p = self.params(pack=False)
        dev = self.device()
        pts = _f32(pts, dev).reshape(-1, 3)
        n = pts.shape[0]
        sbw = _f32(smpl_bw, dev).reshape(24, n)
        li = latent_index.to(device=dev, dtype=torch.int64).reshape(-1).contiguous()
        if field == 1 and not self.net.novel_tensors():
            raise RuntimeError('novel_pose_bw is absent (cfg.aninerf_animation is False)')
        bw = torch.empty((1, 24, n), device=dev)
        if n == 0:
            return bw
        ws_bytes = self.lib.anr_points_workspace_bytes(n)
        ws = self._workspace('_pws', ws_bytes, dev)
        _lib.check(self.lib.anr_blend_weights(ctypes.byref(p), field, _lib.ptr(pts), _lib.ptr(sbw), n, _lib.ptr(li),
                                              row_add, _lib.ptr(bw), _lib.ptr(ws), ws_bytes, _lib.stream_ptr(dev)),
                   'anr_blend_weights')
        return bw

    def canonical_alpha(self, nf_pts):
        """TPoseHuman.calculate_alpha (tpose_nerf_network.py:241-250): nf_pts (1,n,3) -> alpha (1,1,n)."""
        p = self.params(pack=False)
        dev = self.device()
        pts = _f32(nf_pts, dev).reshape(-1, 3)
        n = pts.shape[0]
        alpha = torch.empty((1, 1, n), device=dev)
        if n == 0:
            return alpha
        ws_bytes = self.lib.anr_points_workspace_bytes(n)
        ws = self._workspace('_pws', ws_bytes, dev)
        _lib.check(self.lib.anr_canonical_alpha(ctypes.byref(p), _lib.ptr(pts), n, _lib.ptr(alpha), _lib.ptr(ws),
                                                ws_bytes, _lib.stream_ptr(dev)), 'anr_canonical_alpha')
        return alpha


def to_host(ret):
    """the eval outputs on the CPU, as tpose_renderer.py:154-155 leaves them: copied into page-locked
    buffers (torch's caching host allocator reuses them call after call) with one stream sync, so the
    ~1.4 GB of a 512x512 frame (raw + pbw / tbw rows) moves at the link's DMA rate."""
    out, devs = {}, set()
    for k, v in ret.items():
        if v.is_cuda:
            h = torch.empty(v.shape, dtype=v.dtype, pin_memory=True)
            with torch.cuda.device(v.device):  # the copy runs on (and is awaited on) v's device's stream
                h.copy_(v, non_blocking=True)
            devs.add(v.device)
            out[k] = h
        else:
            out[k] = v
    for d in devs:
        torch.cuda.current_stream(d).synchronize()
    return out


class _TrainRender(torch.autograd.Function):
    """forward = anr_train_fwd, backward = anr_train_bwd (parameter gradients accumulate)."""

    @staticmethod
    def forward(ctx, renderer, batch, t_rand, *params):
        lib = renderer.lib
        p = renderer.params(pack=False)
        dev = params[0].device
        R = batch['ray_o'].shape[1]
        c = _Call(renderer, batch, t_rand)
        ws_bytes = lib.anr_train_workspace_bytes(R, ctypes.byref(c.opts), ctypes.byref(c.frame))
        # each forward owns its activations until its backward: a second render_train before the
        # first backward (gradient accumulation, two forwards and one loss) must not overwrite them
        # (torch's caching allocator makes the per-call allocation cheap)
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        _lib.check(lib.anr_train_fwd(ctypes.byref(p), ctypes.byref(c.frame), *c.ray_ptrs(), R, ctypes.byref(c.opts),
                                     ctypes.byref(c.out), _lib.ptr(ws), ws_bytes, _lib.stream_ptr(dev)),
                   'anr_train_fwd')
        pbw, tbw = renderer._bw_rows(ws, R, dev)
        ctx.renderer, ctx.call, ctx.ws, ctx.ws_bytes, ctx.m = renderer, c, ws, ws_bytes, pbw.shape[1]
        ctx.mark_non_differentiable(c.acc, c.depth, c.raw)
        return c.rgb, c.acc, c.depth, c.raw, pbw, tbw

    @staticmethod
    def backward(ctx, d_rgb, d_acc, d_depth, d_raw, d_pbw, d_tbw):
        r, c = ctx.renderer, ctx.call
        lib = r.lib
        params = r.net.core_tensors()
        dev = params[0].device
        p = r.params(pack=False)
        grads = [torch.zeros_like(t) for t in params]
        gp = (ctypes.c_void_p * _lib.NUM_TENSORS)(*[g.data_ptr() for g in grads])
        keep = [t.contiguous() if t is not None else None for t in (d_rgb, d_pbw, d_tbw)]
        _lib.check(lib.anr_train_bwd(ctypes.byref(p), gp, ctypes.byref(c.frame), *c.ray_ptrs(), c.R,
                                     ctypes.byref(c.opts), *[_lib.ptr(t) for t in keep], _lib.ptr(ctx.ws),
                                     ctx.ws_bytes, _lib.stream_ptr(dev)), 'anr_train_bwd')
        return (None, None, None, *grads)


class _TrainNetwork(torch.autograd.Function):
    """Network.forward under autograd: forward = anr_network_train_fwd, backward = anr_network_train_bwd
    from the upstream d raw and d pbw / d tbw rows (parameter gradients)."""

    @staticmethod
    def forward(ctx, renderer, batch, samples, *params):
        lib = renderer.lib
        p = renderer.params(pack=False)
        dev = params[0].device
        c = _Call(renderer, batch, None, samples=samples)
        ws_bytes = lib.anr_network_train_workspace_bytes(c.n, ctypes.byref(c.opts), ctypes.byref(c.frame))
        ws = torch.empty(ws_bytes, dtype=torch.uint8, device=dev)
        raw = torch.empty((1, c.n, 4), device=dev)
        _lib.check(lib.anr_network_train_fwd(ctypes.byref(p), ctypes.byref(c.frame), ctypes.byref(c.samples),
                                             ctypes.byref(c.opts), _lib.ptr(raw), _lib.ptr(ws), ws_bytes,
                                             _lib.stream_ptr(dev)), 'anr_network_train_fwd')
        pbw, tbw = renderer._net_rows(ws, c.n, dev)
        ctx.renderer, ctx.call, ctx.ws, ctx.ws_bytes = renderer, c, ws, ws_bytes
        return raw, pbw, tbw

    @staticmethod
    def backward(ctx, d_raw, d_pbw, d_tbw):
        r, c = ctx.renderer, ctx.call
        params = r.net.core_tensors()
        dev = params[0].device
        p = r.params(pack=False)
        grads = [torch.zeros_like(t) for t in params]
        gp = (ctypes.c_void_p * _lib.NUM_TENSORS)(*[g.data_ptr() for g in grads])
        keep = [t.contiguous() if t is not None else None for t in (d_raw, d_pbw, d_tbw)]
        _lib.check(r.lib.anr_network_train_bwd(ctypes.byref(p), gp, ctypes.byref(c.frame), ctypes.byref(c.samples),
                                               ctypes.byref(c.opts), *[_lib.ptr(t) for t in keep], _lib.ptr(ctx.ws),
                                               ctx.ws_bytes, _lib.stream_ptr(dev)), 'anr_network_train_bwd')
        return (None, None, None, *grads)


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
