"""Trainer plugin (lib/train/trainers/tpose_trainer.py:11-73, trainer.py:9-102, optimizer.py:12-27,
lib/utils/optimizer/lr_scheduler.py:66-75).

Two ways to train, same kernels:

* ``NetworkWrapper(net)`` — the reference's wrapper: ``forward(batch) -> (ret, loss, scalar_stats,
  image_stats)``; the render goes through ``Renderer.render_train`` (an autograd Function over
  ``anr_train_fwd`` / ``anr_train_bwd``), so the reference ``Trainer.train`` loop
  (``loss.backward(); clip_grad_value_(40); optimizer.step()``) runs unchanged.
* ``FusedStep(net)`` — the native path: parameters and gradients live in one flat HBM blob, one
  ``anr_train_step_hooked`` call runs forward + losses + backward, one ``anr_adam`` call clips and
  updates; for N GPUs the blob (with the loss statistics in its tail) is mean-all-reduced over RCCL
  in two buckets, the canonical NeRF's while the blend-weight backward still runs (DDP semantics).
"""
import ctypes
import math
import os

import torch
import torch.nn.functional as F

from . import _lib
from . import config as _config
import torch.distributed as dist

from .parallel import GradBuckets, broadcast_, is_dist, ray_split_range, reduce_keys_
from .renderer import FRAME_KEYS, RAY_KEYS, Renderer, _Call


class NetworkWrapper(torch.nn.Module):
    """tpose_trainer.NetworkWrapper: loss = smooth_l1(pbw, tbw) + mse(rgb_map[mask], rgb[mask])."""

    def __init__(self, net, cfg=None):
        super().__init__()
        self.net = net
        self.renderer = Renderer(net, cfg)
        self.bw_crit = F.smooth_l1_loss
        self.img2mse = lambda x, y: torch.mean((x - y) ** 2)

    def forward(self, batch, t_rand=None):
        ret = self.renderer.render_train(batch, t_rand=t_rand)
        scalar_stats = {}
        loss = 0
        bw_loss = self.bw_crit(ret['pbw'], ret['tbw'])
        scalar_stats.update({'bw_loss': bw_loss})
        loss += bw_loss
        mask = batch['mask_at_box'].to(ret['rgb_map'].device).bool()
        rgb = batch['rgb'].to(ret['rgb_map'].device)
        img_loss = self.img2mse(ret['rgb_map'][mask], rgb[mask])
        scalar_stats.update({'img_loss': img_loss})
        loss += img_loss
        scalar_stats.update({'loss': loss})
        return ret, loss, scalar_stats, {}


def make_optimizer(cfg, net, lr=None, weight_decay=None):
    """optimizer.py:12-27: Adam with one parameter group per tensor."""
    lr = cfg.train.lr if lr is None else lr
    wd = cfg.train.weight_decay if weight_decay is None else weight_decay
    groups = [{'params': [v], 'lr': lr, 'weight_decay': wd} for _, v in net.named_parameters() if v.requires_grad]
    return torch.optim.Adam(groups, lr, weight_decay=wd)


def exponential_lr(base_lr, epoch, gamma=0.1, decay_epochs=1000):
    """lr_scheduler.ExponentialLR (lr_scheduler.py:66-75): base_lr * gamma ** (epoch / decay_epochs)."""
    return base_lr * gamma ** (epoch / decay_epochs)


class FusedStep:
    """Native training step on a flat parameter blob (configs 3 / 4).

    ``step(batch)`` = forward + losses + backward (``anr_train_step``) + [RCCL all-reduce of the
    gradient blob] + clip_grad_value_(40) + Adam (``anr_adam``). Returns the device loss triple
    (loss, img_loss, bw_loss) without synchronising.
    """

    def __init__(self, net, cfg=None, lr=None, clip=40.0, betas=(0.9, 0.999), eps=1e-8, group=None, ray_split=False):
        self.cfg = cfg if cfg is not None else _config.active()
        self.net = net
        self.renderer = Renderer(net, self.cfg)
        self.lib = self.renderer.lib
        self.lr = float(self.cfg.train.lr if lr is None else lr)
        self.wd = float(self.cfg.train.weight_decay)
        self.clip, self.betas, self.eps = clip, betas, eps
        self.group = group
        ps = net.core_tensors()
        dev = ps[0].device
        n = sum(p.numel() for p in ps)
        self.flat = torch.empty(n, device=dev)
        # gradient blob + 4 floats of loss statistics in its tail: one all-reduce carries both (the
        # north_star's "all-reduce of the image/PSNR loss" next to DDP's gradient mean)
        self.grad = torch.zeros(n + 4, device=dev)
        self.m = torch.zeros(n, device=dev)
        self.v = torch.zeros(n, device=dev)
        off = 0
        self.grad_views = []
        for p in ps:
            k = p.numel()
            self.flat[off:off + k].copy_(p.detach().reshape(-1))
            p.data = self.flat[off:off + k].view_as(p)
            g = self.grad[off:off + k].view_as(p)
            p.grad = g
            self.grad_views.append(g)
            off += k
        self.n = n
        self.t = 0
        self.loss3 = self.grad[n:n + 4]
        # buckets in the order anr_train_step_hooked finishes them: the canonical NeRF (tensors 0..26,
        # final before the blend-weight backward runs), then the blend-weight MLP (27..45) + losses
        n_nerf = sum(p.numel() for p in ps[:27])
        # ray_split: every rank gets the SAME batch and trains on its own contiguous share of its rays
        # (one reference chunk split over the ranks: strong scaling of one iteration). The chunk-wide
        # argmin / argmax and the loss sums are exchanged mid-step through the library's reduce hook,
        # so the losses are the batch's on every rank and the gradients are shares of its gradient:
        # summed (not averaged), the loss tail left as it is
        self.ray_split = bool(ray_split) and is_dist()
        if self.ray_split:
            self.buckets = GradBuckets(self.grad, [(0, n_nerf), (n_nerf, n)], group, op='sum')
            self._reduce_cb = _lib.REDUCE_FN(self._reduce_hook)  # kept alive with the step
        else:
            self.buckets = GradBuckets(self.grad, [(0, n_nerf), (n_nerf, n + 4)], group)
            self._reduce_cb = _lib.REDUCE_FN()
        self._st = None  # fixed input / output buffers of the step (see _static_call)
        self._calls = {}  # direct calls per distinct batch (see _direct_call)
        self._p = self._gp = None  # parameter / gradient pointer tables (views of flat / grad: fixed)
        self._ws_bytes, self._hooks = {}, {}
        self._trand = None
        self.nerf_ready = None
        if dev.type == 'cuda':
            self.nerf_ready = torch.cuda.Event()
            self.nerf_ready.record()  # creates the underlying hipEvent (re-recorded by the library)
        # DDP semantics (trainer.py:13-18): every replica starts from rank 0's weights, so the
        # averaged gradient describes one model and the replicas stay identical
        broadcast_(self.flat, 0, group)

    def adam_state_dict(self):
        """torch.optim.Adam-format state (one group per tensor, optimizer.py:12-27)."""
        from .checkpoint import adam_state_dict
        return adam_state_dict(self.net.core_tensors(), self.m, self.v, self.t, self.lr, self.betas, self.eps, self.wd)

    def load_adam_state_dict(self, sd):
        from .checkpoint import load_adam_state_dict
        self.t, self.lr = load_adam_state_dict(sd, self.net.core_tensors(), self.m, self.v)
        # every rank must call this (a collective): the replicas then continue from rank 0's weights
        # (the views of self.flat that load_model filled), moments and step count (which sets Adam's
        # bias corrections), whatever each rank's checkpoint read produced
        broadcast_(self.flat, 0, self.group)
        broadcast_(self.m, 0, self.group)
        broadcast_(self.v, 0, self.group)
        tl = broadcast_(torch.tensor([float(self.t), float(self.lr)], dtype=torch.float64, device=self.m.device),
                        0, self.group)
        self.t, self.lr = int(tl[0]), float(tl[1])

    _STATIC_KEYS = RAY_KEYS + FRAME_KEYS + ('latent_index', 'rgb', 'mask_at_box')
    _OPT_KEYS = ('bw_latent_index',)  # read by _Call when present

    _DIRECT_CACHE = 8  # distinct batches whose direct calls are kept

    def _direct_call(self, batch, t_rand):
        """Without graph replay (the default; ANR_TRAIN_GRAPH=1 takes _static_call) the step reads the
        batch's own device tensors: one _Call per distinct batch, kept for the next steps that see it,
        so no step spends device copies on its inputs (the fixed-buffer copies cost ~0.17 ms of a 2 ms
        step, measured).

        Only a batch whose inputs all live on the step's device is cached: then the key (address,
        version counter, dtype and shape of every input) names live memory, because the entry holds
        the input tensors themselves (no other tensor can take their addresses while it lives), and
        any conversion _Call made (bool mask -> uint8, int64 indices) is of a device tensor whose
        in-place writes bump its version. A batch with host tensors is converted afresh every step
        (writes through numpy views of host tensors do not bump versions)."""
        dev = self.flat.device
        R = batch['ray_o'].shape[1]
        ns = int(self.cfg.N_samples)
        tr = self._trand
        if tr is None or tuple(tr.shape) != (R, ns):
            tr = self._trand = torch.empty((R, ns), device=dev)
        if t_rand is not None:
            tr.copy_(t_rand.reshape(R, ns))
        elif self.cfg.perturb > 0:
            tr.uniform_()
        srcs = tuple(batch[k] for k in self._STATIC_KEYS) + tuple(batch[k] for k in self._OPT_KEYS if k in batch)
        cfg_key = tuple(self.cfg.get(k, None) for k in ('train_precision', 'chunk', 'N_samples', 'norm_th', 'train_th',
                                                        'test_novel_pose'))
        cacheable = all(torch.is_tensor(v) and v.device == dev for v in srcs)
        key = None
        if cacheable:
            key = (tuple((v.data_ptr(), v._version, v.dtype, tuple(v.shape)) for v in srcs),
                   tuple(k for k in self._OPT_KEYS if k in batch), cfg_key)
        ent = self._calls.pop(key, None) if cacheable else None
        if ent is None:
            c = _Call(self.renderer, batch, tr)
            rgb = batch['rgb'].to(device=dev, dtype=torch.float32).contiguous()
            mask = batch['mask_at_box'].to(device=dev, dtype=torch.uint8).reshape(-1).contiguous()
            ent = (c, rgb, mask, srcs)  # the source tensors stay referenced: their addresses are not reused
        if cacheable:
            self._calls[key] = ent  # most recent last
            while len(self._calls) > self._DIRECT_CACHE:
                self._calls.pop(next(iter(self._calls)))
        c, rgb, mask, _ = ent
        c.opts.t_rand = tr.data_ptr() if (t_rand is not None or self.cfg.perturb > 0) else None
        return c, rgb, mask

    def _static_call(self, batch, t_rand):
        """The step's inputs copied into fixed device buffers (and one fixed set of outputs), so that
        consecutive steps call anr_train_step_hooked with identical arguments: from the second such
        call on, the library replays the step as one captured graph. A buffer is rebuilt when a
        shape changes; a source tensor unchanged since the last copy (same storage and version
        counter, e.g. a frame's resident volumes) is not copied again."""
        dev = self.flat.device
        R = batch['ray_o'].shape[1]
        ns = int(self.cfg.N_samples)
        cfg = self.cfg
        shapes = (tuple(tuple(batch[k].shape) for k in self._STATIC_KEYS),
                  tuple(cfg.get(k, None) for k in ('train_precision', 'chunk', 'N_samples', 'norm_th', 'train_th')))
        st = self._st
        if st is None or st['shapes'] != shapes:
            sb = {}
            for k in self._STATIC_KEYS:
                v = batch[k]
                dt = torch.int64 if k == 'latent_index' else (torch.uint8 if k == 'mask_at_box' else torch.float32)
                sb[k] = torch.empty(tuple(v.shape), dtype=dt, device=dev)
            st = self._st = {'shapes': shapes, 'batch': sb, 'src': {}, 't_rand': torch.empty((R, ns), device=dev)}
            st['call'] = _Call(self.renderer, sb, st['t_rand'])
        sb, src = st['batch'], st['src']
        for k in self._STATIC_KEYS:
            v = batch[k]
            tag = (v.data_ptr(), v._version, v.device)
            if src.get(k) != tag:
                sb[k].copy_(v)
                src[k] = tag
        if t_rand is not None:
            st['t_rand'].copy_(t_rand.reshape(R, ns))
        elif self.cfg.perturb > 0:
            st['t_rand'].uniform_()
        st['call'].opts.t_rand = st['t_rand'].data_ptr() if (t_rand is not None or self.cfg.perturb > 0) else None
        return st['call'], sb['rgb'], sb['mask_at_box'].reshape(-1)

    def _reduce_hook(self, user, buf, count, op, stream):
        """anr_train_hooks.reduce: the step's mid-step exchange over the ranks (parallel.reduce_keys_) on a
        view of the workspace buffer the library hands over, issued on the stream the library hands over
        (its own main stream, not the caller's)."""
        try:
            ws = self._ws_now
            off = buf - ws.data_ptr()
            isz = 4 if op == _lib.REDUCE_SUM_F32 else 8
            view = ws[off:off + count * isz].view(torch.float32 if isz == 4 else torch.int64)
            if stream and ws.is_cuda:
                with torch.cuda.stream(torch.cuda.ExternalStream(stream, device=ws.device)):
                    reduce_keys_(view, op, self.group)
            else:
                reduce_keys_(view, op, self.group)
            return 0
        except BaseException:  # pragma: no cover - fatal to the job
            # The peer ranks are already waiting in the matching collective, so returning an error to the
            # library (which would abort only this rank's step) would leave them hung. A failed exchange is
            # fatal: report it and end this process non-zero, so the launcher (torchrun) tears the job down.
            import os
            import sys
            import traceback
            traceback.print_exc()
            sys.stderr.write('anr_train_hooks.reduce failed on this rank: exiting so the peer ranks do not hang\n')
            sys.stderr.flush()
            os._exit(70)

    def _split_share(self, batch, t_rand):
        """this rank's rays of the (replicated) batch and their offset within it"""
        from .parallel import RAY_KEYS as SPLIT_KEYS
        R = int(batch['ray_o'].shape[1])
        world = dist.get_world_size(self.group)
        rank = dist.get_rank(self.group)
        chunk = int(self.cfg.get('chunk', 2048))
        if R > chunk or R < world:
            raise ValueError(f'ray_split: the batch ({R} rays) must fit one reference chunk ({chunk}) and give '
                             f'every one of the {world} ranks a ray')
        a, b = ray_split_range(R, rank, world)
        sub = {k: (v[:, a:b] if k in SPLIT_KEYS and torch.is_tensor(v) and v.dim() >= 2 and v.shape[1] == R else v)
               for k, v in batch.items()}
        if t_rand is not None:
            t_rand = t_rand.reshape(R, -1)[a:b]
        return sub, t_rand, a

    def step(self, batch, t_rand=None, lr=None):
        r = self.renderer
        dev = self.flat.device
        ray_offset = 0
        if self.ray_split:
            batch, t_rand, ray_offset = self._split_share(batch, t_rand)
        R = batch['ray_o'].shape[1]
        if os.environ.get('ANR_TRAIN_GRAPH') == '1':
            c, rgb, mask = self._static_call(batch, t_rand)
        else:
            c, rgb, mask = self._direct_call(batch, t_rand)
        # per-step host work kept small (the step issues ~175 launches; its Python side ran ~0.2 ms):
        # the parameter and gradient pointer tables are views into this step's flat blobs, built once
        if self._p is None:
            self._p = r.params(pack=False)
            self._gp = (ctypes.c_void_p * _lib.NUM_TENSORS)(*[g.data_ptr() for g in self.grad_views])
        p, gp = self._p, self._gp
        fr = c.frame  # the workspace depends on the ray count, the chunk and the volume dims only
        wkey = (R, int(c.opts.chunk), tuple(fr.pbw_dims), tuple(fr.tbw_dims))
        ws_bytes = self._ws_bytes.get(wkey)
        if ws_bytes is None:
            ws_bytes = self.lib.anr_train_workspace_bytes(R, ctypes.byref(c.opts), ctypes.byref(c.frame))
            if len(self._ws_bytes) > 64:
                self._ws_bytes.clear()
            self._ws_bytes[wkey] = ws_bytes
        ws = r._workspace('_tws', ws_bytes, dev)
        self.grad.zero_()
        stream = _lib.stream_ptr(dev)
        overlap = is_dist() and self.nerf_ready is not None
        hkey = (overlap, ray_offset)
        hooks = self._hooks.get(hkey)
        if hooks is None:
            hooks = self._hooks[hkey] = _lib.TrainHooks(self.nerf_ready.cuda_event if overlap else None, ray_offset,
                                                        self._reduce_cb, None)
        self._ws_now = ws
        _lib.check(self.lib.anr_train_step_hooked(ctypes.byref(p), gp, ctypes.byref(c.frame), *c.ray_ptrs(), R,
                                                  ctypes.byref(c.opts), _lib.ptr(rgb), _lib.ptr(mask),
                                                  ctypes.byref(c.out), _lib.ptr(self.loss3), ctypes.byref(hooks),
                                                  _lib.ptr(ws), ws_bytes, stream), 'anr_train_step_hooked')
        # N > 1: the NeRF bucket's all-reduce runs beside the blend-weight backward, then the rest
        self.buckets.reduce(0, self.nerf_ready if overlap else None)
        self.buckets.reduce(1)
        self.buckets.wait()
        self.t += 1
        _lib.check(self.lib.anr_adam(_lib.ptr(self.flat), _lib.ptr(self.grad), _lib.ptr(self.m), _lib.ptr(self.v),
                                     self.n, float(self.lr if lr is None else lr), self.betas[0], self.betas[1],
                                     self.eps, self.wd, self.t, self.clip, stream), 'anr_adam')
        # the update bypassed torch's version counters: invalidate the renderer's packed weights
        self.net._anr_weights_epoch = getattr(self.net, '_anr_weights_epoch', 0) + 1
        self.last = c
        return self.loss3


def psnr_from_mse(mse):
    return -10.0 * math.log10(mse)
